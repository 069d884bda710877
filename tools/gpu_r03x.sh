# Lanes on dedicated hardware queues (CU-mask streams): GPU suite, then 2 / 3 / 4 lanes for
# C2, C3 (two contexts per process, 20 steps) and C4 (one context, 4 steps).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/x
O=gpurun_out/x
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
for c in C2 C3; do for p in 2 3 4; do
  PIPE=$p STEPS=20 timeout -k 10 300 python tools/order_probe.py $c $c > $O/${c}_p$p.log 2>&1 || { tail $O/${c}_p$p.log; exit 1; }
  echo "lanes=$p $(grep -E '^C[0-9] ' $O/${c}_p$p.log | tr '\n' ' ')"
done; done
for p in 2 3 4; do
  PIPE=$p STEPS=4 timeout -k 10 300 python tools/order_probe.py C4 > $O/C4_p$p.log 2>&1 || { tail $O/C4_p$p.log; exit 1; }
  echo "lanes=$p $(grep -E '^C[0-9] ' $O/C4_p$p.log | tr '\n' ' ')"
done
