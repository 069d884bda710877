# Round 4: the bounce pool's refill threshold and grab size again with the level fork at 2 lanes
# (C2): leave at 32 / 8 finished lanes (shipped 16), grabs of 2 mask words (shipped 4).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4t
export TMPDIR=/tmp
O=gpurun_out/r4t
sha256sum var/*.so | tee $O/lib.sha256
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2 3; do
  for L in base leave32 leave8 grab2; do b C2_$L.$rep C2 20 VPX_LIB=var/lib_$L.so; done
done
