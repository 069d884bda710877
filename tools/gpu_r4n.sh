# Round 4: occupancy caps of the multi-volume tile walkers — k_nearest_tile at 5 waves/SIMD
# (var/lib_nt5.so, 49 spilled VGPRs) and the multi-volume shadow kernels at 6 (var/lib_st6.so)
# against the shipped caps (4 / 5) on Z1 and C4; Z1 at 2 / 4 frames in flight.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4n
export TMPDIR=/tmp
O=gpurun_out/r4n
sha256sum var/*.so | tee $O/lib.sha256
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra $PIPE > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2 3; do
  PIPE="" b Z1_base.$rep Z1 10 VPX_LIB=var/lib_base.so
  PIPE="" b Z1_nt5.$rep Z1 10 VPX_LIB=var/lib_nt5.so
  PIPE="" b Z1_st6.$rep Z1 10 VPX_LIB=var/lib_st6.so
  PIPE="--pipeline 2" b Z1_p2.$rep Z1 10 VPX_LIB=var/lib_base.so
  PIPE="--pipeline 4" b Z1_p4.$rep Z1 10 VPX_LIB=var/lib_base.so
  PIPE="" b C4_base.$rep C4 3 VPX_LIB=var/lib_base.so
  PIPE="" b C4_st6.$rep C4 3 VPX_LIB=var/lib_st6.so
done
