# parity tests, then bench under each VPX_PERSIST setting
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gputests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/gputests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for p in 1 0; do
  VPX_PERSIST=$p timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench_p$p.log 2>&1; rc=$?
  echo "persist=$p rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"dda_cells": [0-9.]*' gpurun_out/bench_p$p.log | tr '\n' ' '; echo
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_p$p.log; exit $rc; fi
done
