# Round 4: persistent waves for the multi-volume / shape bounce levels (k_nearest_mpool, grabs of
# 4 or 16 mask words, var/lib_mpool{4,16}.so) against k_nearest_tile (var/lib_base.so) on Z1 —
# the multi-volume / zone parity tests through the pool build first.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4i
export TMPDIR=/tmp
O=gpurun_out/r4i
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so var/*.so | tee $O/lib.sha256
timeout -k 10 600 env VPX_LIB=var/lib_mpool4.so python -u -m pytest tests -x -q -m gpu -k "zone or multi or shape or instance or tlas or triangle or sphere" --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -v amdgpu.ids $O/tests.log | tail -3 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2 3; do
  for L in base mpool4 mpool16; do
    b Z1_$L.$rep Z1 10 VPX_LIB=var/lib_$L.so
  done
done
