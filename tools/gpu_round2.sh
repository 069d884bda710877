# Round-2 evidence run: GPU parity suite, smoke, full bench (N=1, extras + CPU baseline),
# 2- and 4-rank rehearsals of the strong-scaling flow on the one GPU (gloo via host).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r2
export TMPDIR=/tmp
O=gpurun_out/r2
step() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-2} | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
if [ "${TESTS:-1}" = 1 ]; then
  step gputests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python bench.py
for n in ${REHEARSE:-2 4}; do
  step rehearse$n 600 env VPX_BENCH_SHARED_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 2
done
