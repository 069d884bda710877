# full GPU parity suite on the in-tree library, then the var/ A/B (tools/gpu_var.sh)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputests_full.log 2>&1; rc=$?
echo "full gpu tests rc=$rc"; grep -v amdgpu.ids gpurun_out/gputests_full.log | tail -4
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_var.sh
