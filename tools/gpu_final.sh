# Round evidence in two calls (each within gpurun's 1200 s):
#   PART=1: GPU parity suite, smoke(), rocprofv3 kernel-trace stats of the C1 bench line, PMC
#           passes for PMC_CFGS, and their per-launch traffic into profiles/ (sha256-tagged);
#   PART=2: the full bench line (N=1, extras, CPU baseline; roofline.traffic from PART 1's
#           summaries when the library is unchanged) and the 2-/4-rank one-GPU rehearsals.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/fin
export TMPDIR=/tmp
TAG=${TAG:-r02}
O=gpurun_out/fin
step() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-2} | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
if [ "${PART:-1}" = 1 ]; then
  step gputests 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o run -- python bench.py --no-cpu --no-extra
  declare -A WH=([C1]="1920 1080" [C2]="1920 1080" [C3]="3840 2160" [C4]="3840 2160")
  for c in ${PMC_CFGS:-C1 C2 C3 C4}; do
    TAG=fin/pmc_$c BENCH_ARGS="--config $c" bash tools/gpu_pmc.sh > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
    python tools/pmc_traffic.py $O/pmc_$c profiles/${TAG}_pmc_traffic_$c.json $c ${WH[$c]} > /dev/null && cp profiles/${TAG}_pmc_traffic_$c.json $O/ && echo "pmc $c ok"
  done
else
  step bench 600 python bench.py
  for n in ${REHEARSE:-2 4}; do
    step rehearse$n 300 env VPX_BENCH_SHARED_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 2
  done
fi
