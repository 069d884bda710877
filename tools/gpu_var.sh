# A/B: bench each prebuilt variant library in var/ (parity spot-check on each)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for L in var/lib_*.so; do
  n=$(basename $L .so)
  VPX_LIB=$L timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "render or trace" > gpurun_out/t_$n.log 2>&1; rc=$?
  echo "$n tests rc=$rc $(tail -1 gpurun_out/t_$n.log)"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  VPX_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu ${BENCH_ARGS:-} > gpurun_out/b_$n.log 2>&1; rc=$?
  echo "$n bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_$n.log)"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/b_$n.log; exit $rc; fi
done
if [ -f var/ph.so ]; then VPX_LIB=var/ph.so timeout -k 10 300 python tools/phase_prof.py > gpurun_out/phase.log 2>&1; echo "phase rc=$?"; grep -v amdgpu.ids gpurun_out/phase.log | tail -2; fi
