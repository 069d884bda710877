# Round 4: the shadow pool's occupancy cap at 4 waves/SIMD (var/lib_sp4.so) vs the shipped 5,
# C3 and C4.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4w
export TMPDIR=/tmp
O=gpurun_out/r4w
sha256sum var/*.so | tee $O/lib.sha256
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; if [ $rc -ne 0 ]; then tail -3 $O/$tag.log; exit $rc; fi; }
for rep in 1 2 3; do
  for L in base sp4; do b C3_$L.$rep C3 10 VPX_LIB=var/lib_$L.so; b C4_$L.$rep C4 5 VPX_LIB=var/lib_$L.so; done
done
