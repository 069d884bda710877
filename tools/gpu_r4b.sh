# Round 4: the path pool (k_path_pool) — GPU parity suite on the in-tree library, then C2 with
# the pool vs the per-level kernels (VPX_PATH_POOL=0), and the -fno-slp-vectorize variant.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4b
export TMPDIR=/tmp
O=gpurun_out/r4b
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so var/*.so | tee $O/lib.sha256
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -v amdgpu.ids $O/tests.log | tail -4 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
fi
b() { tag=$1; cfg=$2; shift 2; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps ${STEPS:-10} --warmup 2 --no-cpu --no-extra > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"stages_ms": {[^}]*}\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2; do
  for c in ${CFGS:-C2}; do
    b base_pool_$c.$rep $c VPX_LIB=var/lib_base.so VPX_PATH_POOL=1
    b base_levels_$c.$rep $c VPX_LIB=var/lib_base.so VPX_PATH_POOL=0
    b noslp_pool_$c.$rep $c VPX_LIB=var/lib_noslp.so VPX_PATH_POOL=1
  done
done
