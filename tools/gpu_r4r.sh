# Round 4: k_frame0's occupancy cap again on the round-4 build: 6 waves/SIMD (shipped: 80 VGPRs,
# 3 spilled VGPRs, 38 spilled SGPRs) vs 5 (var/lib_fr5.so), C1 interleaved.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4r
export TMPDIR=/tmp
O=gpurun_out/r4r
sha256sum var/*.so | tee $O/lib.sha256
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 3 --no-cpu --no-extra > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2 3 4; do
  for L in base fr5; do b C1_$L.$rep C1 40 VPX_LIB=var/lib_$L.so; done
done
