# C1 lanes x stream priority: in-tree (normal-priority lanes) vs var/lib_prio.so (high), 2 / 3 / 4
# lanes, three C1 contexts per process, 20 steps; two rounds.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/t
O=gpurun_out/t
export STEPS=20
for r in 1 2; do for L in raytracer-voxpopuli_amd/libvpx_hip.so var/lib_prio.so; do n=$(basename $L .so)
  for p in 2 3 4; do
    PIPE=$p VPX_LIB=$L timeout -k 10 300 python tools/order_probe.py C1 C1 C1 > $O/${n}_p${p}_$r.log 2>&1 || { tail $O/${n}_p${p}_$r.log; exit 1; }
    echo "$r $n lanes=$p $(grep -E '^C[0-9] ' $O/${n}_p${p}_$r.log | tr '\n' ' ')"
  done
done; done
