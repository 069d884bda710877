# Lane streams and hardware queues: C1 at 3 / 4 lanes, normal lanes (in-tree) vs lanes on
# full-CU-mask streams (var/lib_cum.so), timed (two contexts per process, 20 steps) and traced
# (queue ids per stream).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/w
O=gpurun_out/w
export TMPDIR=/tmp
for r in 1 2; do for L in raytracer-voxpopuli_amd/libvpx_hip.so var/lib_cum.so; do n=$(basename $L .so)
  for p in 3 4; do
    PIPE=$p STEPS=20 VPX_LIB=$L timeout -k 10 300 python tools/order_probe.py C1 C1 > $O/${n}_p${p}_$r.log 2>&1 || { tail $O/${n}_p${p}_$r.log; exit 1; }
    echo "$r $n lanes=$p $(grep -E '^C[0-9] ' $O/${n}_p${p}_$r.log | tr '\n' ' ')"
  done
done; done
for L in raytracer-voxpopuli_amd/libvpx_hip.so var/lib_cum.so; do n=$(basename $L .so)
  for p in 3 4; do
    PIPE=$p STEPS=10 VPX_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tr_${n}_$p -o run -- python tools/order_probe.py C1 > $O/tr_${n}_$p.log 2>&1 || { tail $O/tr_${n}_$p.log; exit 1; }
    echo "== $n lanes=$p"; python tools/queue_map.py $(find $O/tr_${n}_$p -name '*kernel_trace.csv' | head -1) k_frame0 composite
  done
done
