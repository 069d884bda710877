# rocprofv3 evidence for the current library: kernel-trace stats of the C1 bench line, then
# PMC passes (separate runs, no tracing domains) for each config in PMC_CFGS.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run -- python bench.py --no-cpu --no-extra > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "kernel-trace rc=$rc"; grep '^{' gpurun_out/${TAG}_prof.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
for c in ${PMC_CFGS:-C1}; do
  TAG=${TAG}_pmc_$c BENCH_ARGS="--config $c" bash tools/gpu_pmc.sh || exit $?
done
