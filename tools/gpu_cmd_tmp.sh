set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/gt.log 2>&1; rc=$?; tail -3 gpurun_out/gt.log; [ $rc -ne 0 ] && exit $rc
CFGS="${CFGS:-C1 C3}" bash tools/gpu_var.sh
