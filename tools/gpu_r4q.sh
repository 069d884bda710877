# Round 4: XCD-banded pool grabs (VPX_POOL_XCD: each XCD's waves take their band of the frame's
# tiles first) — GPU suite on the in-tree library, then interleaved A/B against
# var/lib_noxcd.so (one frame-wide grab counter) on C2 / C3 / C4 at K = 10 / 6 / 3 steps.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4q
export TMPDIR=/tmp
O=gpurun_out/r4q
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so var/*.so | tee $O/lib.sha256
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -v amdgpu.ids $O/tests.log | tail -3 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2 3; do
  for L in base noxcd; do
    b C2_$L.$rep C2 10 VPX_LIB=var/lib_$L.so
    b C3_$L.$rep C3 6 VPX_LIB=var/lib_$L.so
    b C4_$L.$rep C4 3 VPX_LIB=var/lib_$L.so
  done
done
