# Round 4: occupancy caps again — single-volume shadow tile kernels at 6 / 8 waves/SIMD
# (var/lib_sh6.so, var/lib_sh8.so; shipped 7) on C2, multi-volume FindNearest kernels at 5
# (var/lib_mn5.so; shipped 4) on C4 and Z1.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4o
export TMPDIR=/tmp
O=gpurun_out/r4o
sha256sum var/*.so | tee $O/lib.sha256
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2 3; do
  for L in base sh6 sh8; do b C2_$L.$rep C2 10 VPX_LIB=var/lib_$L.so; done
  for L in base mn5; do b C4_$L.$rep C4 3 VPX_LIB=var/lib_$L.so; b Z1_$L.$rep Z1 10 VPX_LIB=var/lib_$L.so; done
done
