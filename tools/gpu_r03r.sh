# GPU suite on the in-tree library (8x8-quadrant waves, packed lane order), then the default bench.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r
O=gpurun_out/r
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --no-cpu > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print('C1', d['ms_per_step'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d['extra_configs'].items()})"
