# Round-1 GPU session: smoke, parity tests, bench, rocprofv3 kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids gpurun_out/$name.log | tail -4; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run smoke 400 python __graft_entry__.py smoke
run gputests 900 python -m pytest tests/test_gpu_parity.py -q -m gpu
run bench 400 python bench.py --steps 10 --warmup 2 --cpu-budget 8
export TMPDIR=/tmp
run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python bench.py --steps 10 --warmup 2 --no-cpu
find gpurun_out/prof -name '*stats*' | head
