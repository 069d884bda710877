# Lanes for C4 (2 / 3 / 4, one context per process, 4 steps of 16 frames) and C1 (3 / 4, two
# contexts per process, 20 steps) on the current library.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/v
O=gpurun_out/v
for p in 3 4 2; do
  PIPE=$p STEPS=4 timeout -k 10 300 python tools/order_probe.py C4 > $O/C4_p$p.log 2>&1 || { tail $O/C4_p$p.log; exit 1; }
  echo "lanes=$p $(grep -E '^C[0-9] ' $O/C4_p$p.log | tr '\n' ' ')"
done
for p in 3 4 3 4; do
  PIPE=$p STEPS=20 timeout -k 10 300 python tools/order_probe.py C1 C1 > $O/C1_p$p.log 2>&1 || { tail $O/C1_p$p.log; exit 1; }
  echo "lanes=$p $(grep -E '^C[0-9] ' $O/C1_p$p.log | tr '\n' ' ')"
done
