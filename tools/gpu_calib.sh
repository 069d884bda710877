# FETCH_SIZE / WRITE_SIZE calibration for narrow gathers (tools/native/fetch_calib.hip):
# one plain run (known bytes and times), then one PMC pass per counter group.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/calib
export TMPDIR=/tmp
O=gpurun_out/calib
timeout -k 10 60 tools/native/fetch_calib > $O/plain.log 2>&1; rc=$?; echo "plain rc=$rc"; cat $O/plain.log; [ $rc -ne 0 ] && exit $rc
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d "$GRAFT_REPO_ROOT/$O/p$i" -o run -- tools/native/fetch_calib > $O/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/p$i.log; exit $rc; fi
done
exit 0
