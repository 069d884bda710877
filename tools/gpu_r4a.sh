# Round 4, first box call: GPU suite (incl. the box-host x86-approximation rates), smoke, the
# full bench line, a 2-rank one-GPU rehearsal (the N > 1 line's new keys).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4a
export TMPDIR=/tmp
O=gpurun_out/r4a
step() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-2} | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so | tee $O/lib.sha256
step gputests 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
cp gpurun_out/x86_approx_rates.json $O/ 2>/dev/null
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
step rehearse2 300 env VPX_BENCH_SHARED_DEVICE=1 python bench.py --gpus 2 --steps 10 --warmup 2
