# A/B: bench each prebuilt variant library in var/ (parity spot-check on each); BENCH_ARGS
# and CFGS (space-separated configs, default C1) select the workload(s).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for L in var/lib_*.so; do
  n=$(basename $L .so)
  VPX_LIB=$L timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "render or trace" > gpurun_out/t_$n.log 2>&1; rc=$?
  echo "$n tests rc=$rc $(tail -1 gpurun_out/t_$n.log)"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  for c in ${CFGS:-C1}; do
    VPX_LIB=$L timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu ${BENCH_ARGS:-} > gpurun_out/b_${n}_$c.log 2>&1; rc=$?
    echo "$n $c bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"stages_ms": {[^}]*}' gpurun_out/b_${n}_$c.log | tr '\n' ' ')"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/b_${n}_$c.log; exit $rc; fi
  done
done
if [ -f var/ph.so ]; then VPX_LIB=var/ph.so timeout -k 10 300 python tools/phase_prof.py > gpurun_out/phase.log 2>&1; echo "phase rc=$?"; grep -v amdgpu.ids gpurun_out/phase.log | tail -2; fi
