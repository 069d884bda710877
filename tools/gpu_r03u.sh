# Lanes x stream priority on another box: C1 at 2 / 3 / 4 lanes, C2 / C3 at 2 / 3 / 4, normal
# (in-tree) vs high-priority lanes (var/lib_prio.so); two contexts per process, 20 steps.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/u
O=gpurun_out/u
export STEPS=20
for c in C1 C2 C3; do for L in raytracer-voxpopuli_amd/libvpx_hip.so var/lib_prio.so; do n=$(basename $L .so)
  for p in 2 3 4; do
    PIPE=$p VPX_LIB=$L timeout -k 10 300 python tools/order_probe.py $c $c > $O/${c}_${n}_p${p}.log 2>&1 || { tail $O/${c}_${n}_p${p}.log; exit 1; }
    echo "$n lanes=$p $(grep -E '^C[0-9] ' $O/${c}_${n}_p${p}.log | tr '\n' ' ')"
  done
done; done
