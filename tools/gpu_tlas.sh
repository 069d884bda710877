# TLAS A/B: multi-volume parity tests on each var/ library, then C4 bench lines.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "tlas or multi_volume or cull or smoke_material or trace_rays" > gpurun_out/tlas_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -v amdgpu.ids gpurun_out/tlas_tests.log | tail -3; [ $rc -ne 0 ] && exit $rc
for L in var/lib_*.so; do
  n=$(basename $L .so)
  VPX_LIB=$L timeout -k 10 300 python bench.py --config C4 --steps 4 --warmup 1 --no-cpu --no-extra > gpurun_out/b_$n.log 2>&1; rc=$?
  echo "$n C4 rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"stages_ms": {[^}]*}' gpurun_out/b_$n.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 gpurun_out/b_$n.log; exit $rc; }
done
exit 0
