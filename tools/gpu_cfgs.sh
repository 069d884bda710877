# GPU parity suite (optional, TESTS=0 skips) then one bench line per config in CFGS.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
  echo "gpu tests rc=$rc"; grep -v amdgpu.ids gpurun_out/gputests.log | tail -4
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for c in ${CFGS:-C1}; do
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench_$c.log 2>&1; rc=$?
  echo "$c rc=$rc"; grep '^{' gpurun_out/bench_$c.log | cut -c1-600
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_$c.log; exit $rc; fi
done
