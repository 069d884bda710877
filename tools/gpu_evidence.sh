# Round evidence for the current library build, in two gpurun calls (each within 1200 s):
#   PART=1: GPU parity suite, smoke(), rocprofv3 kernel-trace stats of each config's bench
#           line (C1-C4), and rank 0's share of the strong-scaling frame (tools/rank_share.py,
#           C1 and C3 with frames in flight);
#   PART=2: PMC passes per config and their per-launch traffic (sha256-tagged; written to
#           profiles/ on the box too, where bench.py reads roofline.traffic), the full bench
#           line (N=1, extras, CPU baseline), and the 2-/4-rank rehearsals.
# Only gpurun_out/ comes back: tools/collect_evidence.sh then files the results under
# profiles/${TAG}_* here.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ev
export TMPDIR=/tmp
TAG=${TAG:-r06}
O=gpurun_out/ev
step() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-2} | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so | tee $O/lib.sha256
if [ "${PART:-1}" = 1 ]; then
  step gputests 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  for c in ${CFGS:-C1 C2 C3 C4 Z1}; do
    steps=10; [ $c = C4 ] && steps=3
    step prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_$c" -o run -- python bench.py --config $c --steps $steps --warmup 2 --no-cpu --no-extra
  done
  step share_C1 300 env CFG=C1 PIPE=3 python tools/rank_share.py
  step share_C3 300 env CFG=C3 PIPE=3 python tools/rank_share.py
  step share_C3p4 300 env CFG=C3 PIPE=4 python tools/rank_share.py
  step share_C4p4 600 env CFG=C4 PIPE=4 K=5 python tools/rank_share.py
  step share_C4p3 600 env CFG=C4 PIPE=3 K=5 python tools/rank_share.py
  step share_C4p4w0 600 env CFG=C4 PIPE=4 K=5 WINDOW=0 python tools/rank_share.py
else
  declare -A WH=([C1]="1920 1080" [C2]="1920 1080" [C3]="3840 2160" [C4]="3840 2160" [Z1]="1920 1080")
  for c in ${PMC_CFGS:-C1 C2 C3 C4 Z1}; do
    TAG=ev/pmc_$c BENCH_ARGS="--config $c" bash tools/gpu_pmc.sh > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
    python tools/pmc_traffic.py $O/pmc_$c profiles/${TAG}_pmc_traffic_$c.json $c ${WH[$c]} > /dev/null
    cp profiles/${TAG}_pmc_traffic_$c.json $O/
    echo "pmc $c ok"
  done
  for c in ${PROF_CFGS:-}; do  # kernel-trace stats again for configs whose bench settings changed
    steps=10; [ $c = C4 ] && steps=3
    step prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_$c" -o run -- python bench.py --config $c --steps $steps --warmup 2 --no-cpu --no-extra
  done
  step bench 600 python bench.py
  for n in ${REHEARSE:-2 4}; do
    step rehearse$n 300 env VPX_BENCH_SHARED_DEVICE=1 python bench.py --gpus $n --steps 10 --warmup 2
  done
fi
