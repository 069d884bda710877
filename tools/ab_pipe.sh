# A/B of var/ libraries on one config at several lane counts: CFG, PIPES (e.g. "2 3"), REPS, STEPS.
cd "$GRAFT_REPO_ROOT"
for rep in $(seq 1 ${REPS:-2}); do for L in var/lib_*.so; do for p in ${PIPES:-3}; do
  echo "$rep $(basename $L .so) pipe=$p $(VPX_LIB=$L timeout -k 10 200 python bench.py --config ${CFG:-C2} --steps ${STEPS:-20} --warmup 2 --no-cpu --no-extra --pipeline $p 2>&1 | grep -o '"ms_per_step": [0-9.]*')"
done; done; done
