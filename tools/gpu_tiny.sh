# Latency floor A/B: tiny C1 frames (per-stage µs) for each var/lib_*.so, then the C1 bench.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for L in var/lib_*.so; do
  n=$(basename $L .so)
  VPX_LIB=$L timeout -k 10 120 python tools/tiny_frame.py > gpurun_out/tiny_$n.log 2>&1 || { tail -3 gpurun_out/tiny_$n.log; exit 1; }
  VPX_LIB=$L TW=256 TH=144 timeout -k 10 120 python tools/tiny_frame.py >> gpurun_out/tiny_$n.log 2>&1 || exit 1
  echo "$n $(grep -h 'us$\|us ' gpurun_out/tiny_$n.log | tr '\n' ' ')"
  VPX_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-extra > gpurun_out/bt_$n.log 2>&1 || exit 1
  echo "$n C1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bt_$n.log)"
done
