# Kernel trace of one config's bench run (rocprofv3 --kernel-trace --stats), then the per-kernel
# busy time per dispatch (tools/trace_busy.py).  Usage (on the GPU box, from the repo root):
#   bash tools/gpu_trace.sh OUTDIR CFG [extra bench args]
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/$1; CFG=$2; shift 2
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof_$CFG" -o run -- \
  python bench.py --config "$CFG" --steps 10 --warmup 2 --no-cpu --no-extra "$@" > "$OUT/prof_$CFG.log" 2>&1
rc=$?; echo "trace $CFG rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/prof_$CFG.log"; exit $rc; }
f=$(ls "$OUT"/prof_$CFG/*/run_kernel_trace.csv "$OUT"/prof_$CFG/run_kernel_trace.csv 2>/dev/null | head -1)
python tools/trace_busy.py "$f" --json "$OUT/busy_$CFG.json" | head -20
