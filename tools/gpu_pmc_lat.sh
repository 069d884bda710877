# Vector-L1 (TCP) behaviour of the walkers: hit rate and L1->L2 read latency, two
# rocprofv3 --pmc passes (kernel-trace only) over a short bench run of BENCH_ARGS.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmclat}
B="python bench.py --steps 3 --warmup 1 --no-cpu --no-extra ${BENCH_ARGS:-}"
i=0
for set in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_READ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/p$i" -o run -- $B > gpurun_out/$TAG.p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/$TAG.p$i.log; exit $rc; fi
done
