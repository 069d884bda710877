# k_frame0 occupancy A/B with frames in flight: var/lib_base.so (5 waves/SIMD, no spills)
# vs var/lib_fr6.so (6 waves/SIMD, 22 spilled VGPRs), C1 only, three interleaved rounds.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/h
export TMPDIR=/tmp
O=gpurun_out/h
for r in 1 2 3; do for L in var/lib_base.so var/lib_fr6.so; do n=$(basename $L .so)
  VPX_LIB=$L timeout -k 10 300 python bench.py --no-cpu --no-extra --steps 30 > $O/${n}_$r.log 2>&1 || exit 1
  echo "$r $n $(grep -o '"ms_per_step": [0-9.]*' $O/${n}_$r.log)"
done; done
