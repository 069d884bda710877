# Rank-0 share of the strong-scaling frame per var/lib_*.so (tools/rank_share.py).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for L in var/lib_*.so; do
  n=$(basename $L .so)
  for c in ${CFGS:-C1}; do
    CFG=$c VPX_LIB=$L timeout -k 10 300 python tools/rank_share.py > gpurun_out/share_${n}_$c.log 2>&1 || { tail -3 gpurun_out/share_${n}_$c.log; exit 1; }
    echo "$n $(grep -h 'R=1' gpurun_out/share_${n}_$c.log)"
  done
done
