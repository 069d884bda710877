# rocprofv3 kernel-trace summary of a short bench run (round-1 profile).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-prof}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG" -o run -- python bench.py --steps 10 --warmup 2 --no-cpu ${BENCH_ARGS:-} > gpurun_out/$TAG.log 2>&1
rc=$?; echo rc=$rc; grep '^{' gpurun_out/$TAG.log | cut -c1-400
cut -d, -f1-5 gpurun_out/$TAG/run_kernel_stats.csv | head -12
