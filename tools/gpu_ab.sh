# A/B: full GPU parity suite on the in-tree library, then each var/ library's bench lines
# for CFGS (default C1 C3), REPS repetitions interleaved (variants alternate per rep).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_tests.log | tail -2; [ $rc -ne 0 ] && exit $rc
fi
for rep in $(seq 1 ${REPS:-2}); do
  for L in var/lib_*.so; do
    n=$(basename $L .so)
    for c in ${CFGS:-C1 C3}; do
      VPX_LIB=$L timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu --no-extra > gpurun_out/ab_${n}_$c.log 2>&1; rc=$?
      echo "$rep $n $c rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"stages_ms": {[^}]*}' gpurun_out/ab_${n}_$c.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 gpurun_out/ab_${n}_$c.log; exit $rc; }
    done
  done
done
exit 0
