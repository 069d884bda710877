set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
CFGS="${CFGS:-C1 C3}" bash tools/gpu_var.sh
