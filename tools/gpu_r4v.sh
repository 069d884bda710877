# Round 4: the bounce pool's occupancy cap with the level fork at 2 lanes (C2): 4 / 6 waves/SIMD
# (var/lib_b4.so, var/lib_b6.so) vs the shipped 5.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4v
export TMPDIR=/tmp
O=gpurun_out/r4v
sha256sum var/*.so | tee $O/lib.sha256
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; if [ $rc -ne 0 ]; then tail -3 $O/$tag.log; exit $rc; fi; }
for rep in 1 2 3; do
  for L in base b4 b6; do b C2_$L.$rep C2 20 VPX_LIB=var/lib_$L.so; done
done
