# Round evidence for the current library build, in two gpurun calls (each within 1200 s):
#   PART=1: GPU parity suite, smoke(), rocprofv3 kernel-trace stats of each config's bench
#           line (C1-C4) with the busy-time view of the trace (tools/trace_busy.py), and rank
#           0's share of the strong-scaling frame (tools/rank_share.py, C1 and C3);
#   PART=2: PMC passes per config and their per-launch traffic (sha256-tagged, read by
#           bench.py), the full bench line (N=1, extras, CPU baseline), 2-/4-rank rehearsals.
# Everything judged lands in profiles/${TAG}_*.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ev
export TMPDIR=/tmp
TAG=${TAG:-r03}
O=gpurun_out/ev
step() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-2} | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so | tee $O/lib.sha256
if [ "${PART:-1}" = 1 ]; then
  step gputests 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
  tail -3 $O/gputests.log > profiles/${TAG}_gputests_tail.txt
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  for c in ${CFGS:-C1 C2 C3 C4}; do
    steps=10; [ $c = C4 ] && steps=3
    step prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_$c" -o run -- python bench.py --config $c --steps $steps --warmup 2 --no-cpu --no-extra
    cp $(find $O/prof_$c -name 'run_kernel_stats.csv' | head -1) profiles/${TAG}_kernel_stats_$c.csv
    python tools/trace_busy.py $(find $O/prof_$c -name 'run_kernel_trace.csv' | head -1) k_ composite blend --json profiles/${TAG}_trace_busy_$c.json > /dev/null
    grep '^{' $O/prof_$c.log | tail -1 > profiles/${TAG}_prof_bench_$c.json
  done
  for c in C1 C3; do
    step share_$c 300 env CFG=$c PIPE=3 python tools/rank_share.py
    grep -h 'R=1' $O/share_$c.log >> $O/rank_share.txt
  done
  cp $O/rank_share.txt profiles/${TAG}_rank_share.txt
else
  declare -A WH=([C1]="1920 1080" [C2]="1920 1080" [C3]="3840 2160" [C4]="3840 2160")
  for c in ${PMC_CFGS:-C1 C2 C3 C4}; do
    TAG=ev/pmc_$c BENCH_ARGS="--config $c" bash tools/gpu_pmc.sh > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
    python tools/pmc_traffic.py $O/pmc_$c profiles/${TAG}_pmc_traffic_$c.json $c ${WH[$c]} > /dev/null
    python tools/pmc_summary.py $O/pmc_$c > profiles/${TAG}_pmc_counters_$c.txt
    echo "pmc $c ok"
  done
  step bench 600 python bench.py
  grep '^{' $O/bench.log | tail -1 > profiles/${TAG}_bench.json
  for n in ${REHEARSE:-2 4}; do
    step rehearse$n 300 env VPX_BENCH_SHARED_DEVICE=1 python bench.py --gpus $n --steps 10 --warmup 2
    grep '^{' $O/rehearse$n.log | tail -1 > profiles/${TAG}_rehearse$n.json
  done
fi
