# GPU tests + N-rank rehearsal of bench.py on one GPU (both gather flows).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gt.log 2>&1; rc=$?
tail -3 gpurun_out/gt.log; [ $rc -ne 0 ] && exit $rc
for g in rgb8 samples; do
  VPX_BENCH_SHARED_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --gather $g > gpurun_out/reh_$g.log 2>&1; rc=$?
  echo "rehearsal $g rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"parallelism": "[^"]*"' gpurun_out/reh_$g.log | tr '\n' ' '; echo
  [ $rc -ne 0 ] && { tail -20 gpurun_out/reh_$g.log; exit $rc; }
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b1.log 2>&1; rc=$?
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/b1.log | tr '\n' ' '; echo; exit $rc
