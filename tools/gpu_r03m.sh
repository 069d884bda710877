# Frames-in-flight steady state: ms/step against the number of timed steps (5 / 20 / 60) for
# serial frames (0) and the per-config default, C1-C3.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/m
O=gpurun_out/m
for c in C1 C2 C3; do for p in 0 d; do for k in 5 20 60; do
  a="--pipeline $p"; [ $p = d ] && a=""
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-extra --steps $k --warmup 3 $a > $O/${c}_p${p}_k$k.log 2>&1 || exit 1
  echo "$c p$p k$k $(grep -o '"ms_per_step": [0-9.]*' $O/${c}_p${p}_k$k.log) $(grep -o '"frames_in_flight": [0-9]*' $O/${c}_p${p}_k$k.log)"
done; done; done
