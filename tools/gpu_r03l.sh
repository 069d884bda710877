# DPP wave reductions / scans (fewer spilled VGPRs) and the fused level variant: GPU suite on
# the in-tree library, then C1 / C2 A/B of in-tree vs var/lib_oldwave.so (shuffle-based wave
# ops) vs var/lib_fl.so (+ fused bounce-shade and shadow-resolve), three rounds.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/l
O=gpurun_out/l
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
for r in 1 2 3; do for L in raytracer-voxpopuli_amd/libvpx_hip.so var/lib_oldwave.so var/lib_fl.so; do n=$(basename $L .so)
  for c in C1 C2; do
    VPX_LIB=$L timeout -k 10 300 python bench.py --config $c --no-cpu --no-extra --steps 20 > $O/${n}_${c}_$r.log 2>&1 || exit 1
    echo "$r $n $c $(grep -o '"ms_per_step": [0-9.]*' $O/${n}_${c}_$r.log)"
  done
done; done
