# A/B of var/ libraries on chosen configs: optional parity spot check per variant (CHECK="name ..."),
# then REPS interleaved bench runs; PAIRS="lib:cfg[:pipeline] ..." lists which library runs which
# config (and, optionally, with how many frames in flight).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab2
O=gpurun_out/ab2
for n in ${CHECK:-}; do
  VPX_LIB=var/lib_$n.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "${K:-render or trace or frame}" --timeout 120 --timeout-method thread > $O/t_$n.log 2>&1; rc=$?
  echo "$n tests rc=$rc $(tail -1 $O/t_$n.log)"; [ $rc -ne 0 ] && exit $rc
done
for rep in $(seq 1 ${REPS:-3}); do
  for pc in $PAIRS; do
    IFS=: read -r n c pl <<< "$pc"
    VPX_LIB=var/lib_$n.so timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu --no-extra ${pl:+--pipeline $pl} > $O/b_${n}_$c.log 2>&1; rc=$?
    echo "$rep $n $c ${pl:-} rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"stages_ms": {[^}]*}' $O/b_${n}_$c.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/b_${n}_$c.log; exit $rc; }
  done
done
exit 0
