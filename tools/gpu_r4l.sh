# Round 4: the level-fork policy build (context stream, or single-volume frames with <= 2
# lanes; C2 at 2 lanes) — GPU suite, then two full bench lines (C1 + extras, as the driver runs).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4l
export TMPDIR=/tmp
O=gpurun_out/r4l
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so | tee $O/lib.sha256
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -v amdgpu.ids $O/tests.log | tail -3 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 600 python bench.py --no-cpu > $O/bench.$rep.log 2>&1; rc=$?; echo "bench $rep rc=$rc"; [ $rc -ne 0 ] && { tail -3 $O/bench.$rep.log; exit $rc; }
  python - $O/bench.$rep.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print("C1", d["ms_per_step"], d.get("serial_ms_per_frame"))
for k, v in d.get("extra_configs", {}).items(): print(k, v.get("ms_per_step"), v.get("serial_ms_per_frame"), v.get("pipeline"))
PY
done
