# Round 4: frames in flight x level fork — C2 / Z1 at 2 / 3 / 4 lanes with the fork on the lanes
# too (var/lib_forklanes.so) vs the shipped build (fork only on the context's stream).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4j
export TMPDIR=/tmp
O=gpurun_out/r4j
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so var/*.so | tee $O/lib.sha256
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra $PIPE > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2; do
  for p in 2 3 4; do
    for L in base forklanes; do
      PIPE="--pipeline $p" b C2_${L}_p$p.$rep C2 10 VPX_LIB=var/lib_$L.so
      PIPE="--pipeline $p" b Z1_${L}_p$p.$rep Z1 10 VPX_LIB=var/lib_$L.so
    done
  done
done
