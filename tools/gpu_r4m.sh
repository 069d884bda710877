# Round 4: frames-in-flight depth again for C1 and C4 with the round-4 build (lane tails, level
# fork policy): 2 / 3 / 4 lanes, interleaved.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4m
export TMPDIR=/tmp
O=gpurun_out/r4m
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so | tee $O/lib.sha256
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra "$@" > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2; do
  for p in 2 3 4; do
    b C1_p$p.$rep C1 20 --pipeline $p
    b C4_p$p.$rep C4 3 --pipeline $p
  done
done
