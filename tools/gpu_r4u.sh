# Round 4: vector-L1 behaviour of the pool walkers (C2 bounce pool, C3 shadow pool) and the
# multi-volume tile walker (Z1) on the shipped build: tools/gpu_pmc_lat.sh per config.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4u
export TMPDIR=/tmp
for c in C2 C3 Z1; do
  TAG=r4u/lat_$c BENCH_ARGS="--config $c" timeout -k 10 400 bash tools/gpu_pmc_lat.sh > gpurun_out/r4u/lat_$c.log 2>&1; rc=$?
  echo "lat $c rc=$rc"; [ $rc -ne 0 ] && { tail -3 gpurun_out/r4u/lat_$c.log; exit $rc; }
done
