# tools/gpu_run.sh — the one parametrised GPU-box runner (replaces round 4's one-off gpu_r4*.sh).
#
#   gpurun -- bash tools/gpu_run.sh OUT 'name|seconds|command' ['name|seconds|command' ...]
#
# Runs each step under its own `timeout -k 10 seconds`, logging to gpurun_out/OUT/name.log, and
# stops at the first step that fails (a GPU fault, abort or time limit ends the call there).
# Prints the last lines of each log.  TAILN (default 3) lines per step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
(sha256sum raytracer-voxpopuli_amd/libvpx_hip.so | cut -c1-64) > "$OUT/lib.sha256"
for spec in "$@"; do
  name=${spec%%|*}
  rest=${spec#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc"
  grep -v amdgpu.ids "$OUT/$name.log" | tail -"${TAILN:-3}" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
done
