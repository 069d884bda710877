# Round-3 check after the variant prune + host fixes: GPU parity suite, smoke, the bench's
# self-launch of 2 ranks on one GPU (VPX_BENCH_SHARED_DEVICE=1, no torchrun), and
# rocprofv3 kernel-trace stats of the C1..C4 bench lines.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/a
export TMPDIR=/tmp
O=gpurun_out/a
step() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-2} | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; }
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so > $O/lib.sha256
step gputests 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step launch2 300 env VPX_BENCH_SHARED_DEVICE=1 python bench.py --gpus 2 --steps 10 --warmup 2 --no-extra
for c in C1 C2 C3 C4; do
  step prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_$c" -o run -- python bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-extra
done
