# File the results of tools/gpu_evidence.sh (merged back under gpurun_out/ev) as
# profiles/${TAG}_*: kernel-trace stats and busy times per config, the bench lines, the
# GPU-suite tail, rank shares, PMC traffic and counters.  Runs here, not on the GPU box.
set -eu
cd "$(dirname "$0")/.."
TAG=${TAG:-r06}
E=gpurun_out/ev
if [ -f $E/gputests.log ]; then tail -3 $E/gputests.log > profiles/${TAG}_gputests_tail.txt; fi
for c in C1 C2 C3 C4 Z1; do
  if [ -d $E/prof_$c ]; then
    cp "$(find $E/prof_$c -name run_kernel_stats.csv | head -1)" profiles/${TAG}_kernel_stats_$c.csv
    python tools/trace_busy.py "$(find $E/prof_$c -name run_kernel_trace.csv | head -1)" k_ composite blend \
      --json profiles/${TAG}_trace_busy_$c.json > /dev/null
    grep '^{' $E/prof_$c.log | tail -1 > profiles/${TAG}_prof_bench_$c.json
  fi
  if [ -f $E/${TAG}_pmc_traffic_$c.json ]; then
    cp $E/${TAG}_pmc_traffic_$c.json profiles/
    python tools/pmc_summary.py $E/pmc_$c k_ composite blend > profiles/${TAG}_pmc_counters_$c.txt
  fi
done
if [ -f $E/share_C1.log ]; then grep -h 'R=1' $E/share_C*.log > profiles/${TAG}_rank_share.txt; fi
if [ -f $E/bench.log ]; then grep '^{' $E/bench.log | tail -1 > profiles/${TAG}_bench.json; fi
for n in 2 4; do
  if [ -f $E/rehearse$n.log ]; then grep '^{' $E/rehearse$n.log | tail -1 > profiles/${TAG}_rehearse$n.json; fi
done
echo "collected into profiles/${TAG}_*"
