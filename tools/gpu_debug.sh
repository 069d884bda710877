set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_dump.py > gpurun_out/debug.log 2>&1; echo rc=$?; tail -3 gpurun_out/debug.log
