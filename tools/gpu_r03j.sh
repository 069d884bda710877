# C3 (3840x2160, 32400 tiles, area lights: 3 slots per path) through k_frame0 (the whole
# depth-0 frame in one launch, shade records in LDS) vs k_primary + k_shadow_finish, with
# 3 lanes; three interleaved rounds.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/j
O=gpurun_out/j
for r in 1 2 3; do for L in var/lib_base.so var/lib_ft40k.so; do n=$(basename $L .so)
  VPX_LIB=$L timeout -k 10 300 python bench.py --config C3 --no-cpu --no-extra --steps 10 > $O/${n}_$r.log 2>&1 || exit 1
  echo "$r $n $(grep -o '"ms_per_step": [0-9.]*' $O/${n}_$r.log)"
done; done
