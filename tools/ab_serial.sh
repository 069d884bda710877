# Serial-frame A/B (--pipeline 0: a host synchronize after every frame) of var/lib_*.so on CFGS.
set -u
cd "$GRAFT_REPO_ROOT"
for rep in $(seq 1 ${REPS:-2}); do for L in var/lib_*.so; do n=$(basename $L .so)
  for c in ${CFGS:-Z1}; do
    VPX_LIB=$L timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-20} --warmup 2 --no-cpu --no-extra --pipeline 0 > gpurun_out/ser_${n}_$c.log 2>&1 || exit 1
    echo "$rep $n $c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ser_${n}_$c.log)"
  done
done; done
