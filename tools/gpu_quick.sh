# quick GPU iteration: parity tests + bench (no cpu baseline)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-4}; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run gputests 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x
run bench 400 python bench.py --steps 10 --warmup 2 --no-cpu
