# Round evidence: parity tests, smoke, bench (with CPU baseline), rocprofv3 kernel-trace
# stats of the same bench command, PMC traffic passes.  Outputs under gpurun_out/round/.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/round
export TMPDIR=/tmp
O=gpurun_out/round
step() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-3}; if [ $rc -ne 0 ]; then exit $rc; fi; }
step gputests 900 python -m pytest tests -q -m gpu
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o run -- python bench.py --no-cpu
i=0
for set in "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  step pmc$i 600 rocprofv3 --pmc $set --output-format csv -d "$GRAFT_REPO_ROOT/$O/pmc/p$i" -o run -- python bench.py --steps 5 --warmup 1 --no-cpu
done
ls $O/prof
