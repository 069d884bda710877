# (1) GPU suite on the in-tree library (32-bit plane parent + unshifted cube byte in the
# walkers); (2) in-tree vs var/lib_prev.so, configs twice each in one process (20 steps; the
# second run of a config is past the first-in-process effect), three rounds; (3) the in-tree
# library with GPU_MAX_HW_QUEUES 8 and 16 (HIP's default is 4).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/p
O=gpurun_out/p
export STEPS=20
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
for r in 1 2 3; do for L in raytracer-voxpopuli_amd/libvpx_hip.so var/lib_prev.so; do n=$(basename $L .so)
  VPX_LIB=$L timeout -k 10 300 python tools/order_probe.py C1 C1 C2 C2 C3 C3 > $O/${n}_$r.log 2>&1 || { tail $O/${n}_$r.log; exit 1; }
  echo "$r $n $(grep -E '^C[0-9] ' $O/${n}_$r.log | tr '\n' ' ')"
done; done
for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/order_probe.py C1 C1 C2 C2 C3 C3 > $O/q$q.log 2>&1 || { tail $O/q$q.log; exit 1; }
  echo "queues $q $(grep -E '^C[0-9] ' $O/q$q.log | tr '\n' ' ')"
done
