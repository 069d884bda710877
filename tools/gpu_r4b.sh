# Round 4: the path pool (k_path_pool) and the instance candidate mask (k_shadow_inst) —
# GPU parity suite on the in-tree library, then interleaved A/Bs:
#   C2: path pool vs per-level kernels (VPX_PATH_POOL=0), and the -fno-slp-vectorize build;
#   C4: candidate-mask instance occlusion vs the linear loop (var/lib_linear.so).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4b
export TMPDIR=/tmp
O=gpurun_out/r4b
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so var/*.so | tee $O/lib.sha256
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/test_path_pool.py tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -v amdgpu.ids $O/tests.log | tail -4 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
fi
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"stages_ms": {[^}]*}\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2; do
  b C2_pool.$rep C2 10 VPX_LIB=var/lib_base.so VPX_PATH_POOL=1
  b C2_levels.$rep C2 10 VPX_LIB=var/lib_base.so VPX_PATH_POOL=0
  b C2_noslp_pool.$rep C2 10 VPX_LIB=var/lib_noslp.so VPX_PATH_POOL=1
done
for rep in 1 2; do
  b C4_base.$rep C4 3 VPX_LIB=var/lib_base.so
  b C4_linear.$rep C4 3 VPX_LIB=var/lib_linear.so
  b C4_notail.$rep C4 3 VPX_LIB=var/lib_notail.so
  b C3_base.$rep C3 6 VPX_LIB=var/lib_base.so
  b C3_notail.$rep C3 6 VPX_LIB=var/lib_notail.so
done
