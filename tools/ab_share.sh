# Rank-0 share A/B (tools/rank_share.py) of var/lib_*.so, CFGS, PIPE lanes, REPS rounds.
set -u
cd "$GRAFT_REPO_ROOT"
for rep in $(seq 1 ${REPS:-2}); do for L in var/lib_*.so; do n=$(basename $L .so)
  for c in ${CFGS:-C1}; do
    VPX_LIB=$L CFG=$c PIPE=${PIPE:-3} timeout -k 10 300 python tools/rank_share.py > gpurun_out/share_${n}_$c.log 2>&1 || exit 1
    echo "$rep $n $(grep 'R=1' gpurun_out/share_${n}_$c.log)"
  done
done; done
