# iteration: parity tests, then a rocprofv3 kernel-trace of a short bench run
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gputests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -v amdgpu.ids gpurun_out/gputests.log | tail -3
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_prof.sh
