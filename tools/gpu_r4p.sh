# Round 4: the full bench line with the extras timed over as many steps as the headline (was
# K / 4 = 5), twice, with the wall time of each run.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4p
export TMPDIR=/tmp
O=gpurun_out/r4p
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so | tee $O/lib.sha256
for rep in 1 2; do
  t0=$(date +%s); timeout -k 10 900 python bench.py > $O/bench.$rep.log 2>&1; rc=$?; t1=$(date +%s)
  echo "bench $rep rc=$rc wall=$((t1 - t0)) s"; [ $rc -ne 0 ] && { tail -3 $O/bench.$rep.log; exit $rc; }
  python - $O/bench.$rep.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print("C1", d["ms_per_step"], d.get("serial_ms_per_frame"), d["roofline"].get("traffic_source", "")[:40])
for k, v in d.get("extra_configs", {}).items(): print(k, v.get("ms_per_step"), v.get("serial_ms_per_frame"), v.get("pipeline"), v["roofline"].get("bound_by", "")[:50])
PY
done
