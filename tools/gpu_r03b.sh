# Frames in flight: parity of the lanes on the GPU, then an A/B of the bench line with
# 0 / 2 / 3 lanes (C1, C2, C3, C4), and the one-GPU 2- / 8-rank share.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/b
export TMPDIR=/tmp
O=gpurun_out/b
step() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-2} | cut -c1-700; if [ $rc -ne 0 ]; then exit $rc; fi; }
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so > $O/lib.sha256
step gputests 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for pl in 0 2 3 0 2 3; do
  step bench_p$pl 300 python bench.py --no-cpu --pipeline $pl --steps 20
done
step launch2 300 env VPX_BENCH_SHARED_DEVICE=1 python bench.py --gpus 2 --steps 10 --warmup 2 --no-extra
for c in C1 C2 C3 C4; do
  step prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_$c" -o run -- python bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-extra
done
for pl in 0 2 3; do
  step share_C1_p$pl 300 env PIPE=$pl CFG=C1 python tools/rank_share.py
done
