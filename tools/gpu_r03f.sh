# Round-3 PMC evidence for the current library: per config, rocprofv3 --pmc passes
# (tools/gpu_pmc.sh: FETCH_SIZE / WRITE_SIZE / SQ_* / TCC_*), per-launch HBM traffic into
# profiles/r03_pmc_traffic_<C>.json (sha256-tagged, read by bench.py) and the counter summary.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/f
export TMPDIR=/tmp
declare -A WH=([C1]="1920 1080" [C2]="1920 1080" [C3]="3840 2160" [C4]="3840 2160")
for c in ${PMC_CFGS:-C1 C2 C3 C4}; do
  TAG=f/pmc_$c BENCH_ARGS="--config $c" bash tools/gpu_pmc.sh > gpurun_out/f/pmc_$c.log 2>&1 || { tail -5 gpurun_out/f/pmc_$c.log; exit 1; }
  python tools/pmc_traffic.py gpurun_out/f/pmc_$c profiles/r03_pmc_traffic_$c.json $c ${WH[$c]} > /dev/null && cp profiles/r03_pmc_traffic_$c.json gpurun_out/f/ && echo "pmc $c ok"
  python tools/pmc_summary.py gpurun_out/f/pmc_$c k_frame0 k_nearest k_shadow k_primary k_shade composite > gpurun_out/f/pmc_counters_$c.txt
done
