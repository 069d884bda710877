# Order effect: C2 / C3 inside the full bench (after C1, same process) against C2 / C3 alone.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/n
O=gpurun_out/n
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu > $O/full_$r.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('$O/full_$r.log').read().strip().splitlines()[-1]); print('full C1', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['extra_configs'].items()})"
  for c in C2 C3; do
    timeout -k 10 300 python bench.py --config $c --no-cpu --no-extra --steps 5 --warmup 2 > $O/${c}_$r.log 2>&1 || exit 1
    echo "alone $c $(grep -o '"ms_per_step": [0-9.]*' $O/${c}_$r.log)"
  done
done
