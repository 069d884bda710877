# rocprofv3 PMC passes (kernel-trace only, no sys/runtime tracing) on a short bench run.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc}
B="python bench.py --steps 3 --warmup 1 --no-cpu --no-extra ${BENCH_ARGS:-}"
mkdir -p gpurun_out/$TAG && sha256sum raytracer-voxpopuli_amd/libvpx_hip.so > gpurun_out/$TAG/lib.sha256
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/p$i" -o run -- $B > gpurun_out/$TAG.p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/$TAG.p$i.log; exit $rc; fi
done
ls gpurun_out/$TAG/*/
