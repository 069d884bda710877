# A/B: frame lanes on high-priority streams (var/lib_prio.so) vs normal priority (in-tree):
# each config first-in-process and second, 20 steps, two rounds.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/s
O=gpurun_out/s
export STEPS=20
for r in 1 2; do for L in raytracer-voxpopuli_amd/libvpx_hip.so var/lib_prio.so; do n=$(basename $L .so)
  for c in C1 C2 C3; do
    VPX_LIB=$L timeout -k 10 300 python tools/order_probe.py $c $c > $O/${n}_${c}_$r.log 2>&1 || { tail $O/${n}_${c}_$r.log; exit 1; }
    echo "$r $n $(grep -E '^C[0-9] ' $O/${n}_${c}_$r.log | tr '\n' ' ')"
  done
done; done
