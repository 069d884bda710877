# Round 4: the level fork (bounce walks beside the shadow walks, VPX_LEVEL_FORK) and the skip
# box continuation (VPX_SKIP_CONT) — GPU suite on the in-tree library (both on), then
# interleaved A/Bs against var/lib_nofork.so and var/lib_nocont.so; then the walkers' vector-L1
# counters and TA busy on C1.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4h
export TMPDIR=/tmp
O=gpurun_out/r4h
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so var/*.so | tee $O/lib.sha256
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -v amdgpu.ids $O/tests.log | tail -3 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
fi
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2; do
  for L in base nocont; do
    b C1_$L.$rep C1 20 VPX_LIB=var/lib_$L.so
    b C3_$L.$rep C3 6 VPX_LIB=var/lib_$L.so
  done
  for L in base nofork nocont; do
    b C2_$L.$rep C2 10 VPX_LIB=var/lib_$L.so
  done
  for L in base nofork; do
    b Z1_$L.$rep Z1 10 VPX_LIB=var/lib_$L.so
    b C4_$L.$rep C4 3 VPX_LIB=var/lib_$L.so
  done
done
TAG=r4h/lat_C1 BENCH_ARGS="--config C1" timeout -k 10 400 bash tools/gpu_pmc_lat.sh > $O/lat_C1.log 2>&1; echo "lat rc=$?"
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE --output-format csv -d "$GRAFT_REPO_ROOT/$O/ta" -o run -- python bench.py --steps 3 --warmup 1 --no-cpu --no-extra > $O/ta.log 2>&1; echo "ta rc=$?"
