set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for L in var/lib_*.so; do
  n=$(basename $L .so)
  VPX_LIB=$L timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "render or trace or full or sharded or tiles" > gpurun_out/t_$n.log 2>&1; rc=$?
  echo "$n tests rc=$rc $(tail -1 gpurun_out/t_$n.log)"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  VPX_LIB=$L timeout -k 10 120 python tools/tiny_frame.py > gpurun_out/tiny_$n.log 2>&1 || exit 1
  echo "$n $(grep -h 'us' gpurun_out/tiny_$n.log | tr '\n' ' ')"
  for c in C1 C3 C4; do
    VPX_LIB=$L timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-extra > gpurun_out/b_${n}_$c.log 2>&1 || exit 1
    echo "$n $c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_${n}_$c.log)"
  done
done
