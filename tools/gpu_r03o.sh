# Order probe (tools/order_probe.py): C2 repeated in one process, after C1, after C3; C3 repeated.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/o
O=gpurun_out/o
i=0
for seq in "C2 C2 C2 C2" "C1 C2 C2" "C3 C2 C2" "C3 C3 C3" "C1 C3 C3"; do i=$((i+1))
  timeout -k 10 300 python tools/order_probe.py $seq > $O/p$i.log 2>&1 || { tail $O/p$i.log; exit 1; }
  echo "[$seq] -> $(grep -E '^C[0-9] ' $O/p$i.log | tr '\n' ' ')"
done
