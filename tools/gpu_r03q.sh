# A/B: 8x8-pixel waves (var/lib_w8.so, -DVPX_WAVE_8X8=1) vs 16x4 strips (in-tree), configs
# twice each in one process, 20 steps, three rounds; then a frame-level check of the variant.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/q
O=gpurun_out/q
export STEPS=20
for r in 1 2 3; do for L in raytracer-voxpopuli_amd/libvpx_hip.so var/lib_w8.so; do n=$(basename $L .so)
  VPX_LIB=$L timeout -k 10 300 python tools/order_probe.py C1 C1 C2 C2 C3 C3 > $O/${n}_$r.log 2>&1 || { tail $O/${n}_$r.log; exit 1; }
  echo "$r $n $(grep -E '^C[0-9] ' $O/${n}_$r.log | tr '\n' ' ')"
done; done
VPX_LIB=var/lib_w8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "frame or trace" > $O/w8tests.log 2>&1; tail -3 $O/w8tests.log
