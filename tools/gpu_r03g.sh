# Round-3 evidence for the current library, two calls (each within gpurun's limit):
#   PART=1: GPU parity suite + smoke, then the PMC passes per config (tools/gpu_r03f.sh);
#   PART=2: kernel-trace stats per config (bench defaults), busy time of the headline kernel,
#           the full bench line (CPU baseline included), and 2- / 4-rank rehearsals started
#           by bench.py itself (no torchrun; every rank on the one GPU).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/g
export TMPDIR=/tmp
O=gpurun_out/g
step() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so > $O/lib.sha256
if [ "${PART:-1}" = 1 ]; then
  step gputests 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step pmc 900 bash tools/gpu_r03f.sh
else
  for c in C1 C2 C3 C4; do
    step prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_$c" -o run -- python bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-extra
  done
  python tools/trace_busy.py $O/prof_C1/run_kernel_trace.csv k_frame0 composite --json $O/busy_C1.json
  step bench 600 python bench.py
  for n in 2 4; do
    step rehearse$n 300 env VPX_BENCH_SHARED_DEVICE=1 python bench.py --gpus $n --steps 10 --warmup 2
  done
fi
