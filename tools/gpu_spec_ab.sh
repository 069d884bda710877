# Parity spot checks of the candidate variants (render/trace tests through VPX_LIB), then the
# interleaved A/B of every var/ library (tools/gpu_ab.sh, no full suite).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for n in ${CHECK:-spec specxor}; do
  VPX_LIB=var/lib_$n.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "render or trace or full" --timeout 120 --timeout-method thread > gpurun_out/t_$n.log 2>&1; rc=$?
  echo "$n parity rc=$rc $(tail -1 gpurun_out/t_$n.log)"; [ $rc -ne 0 ] && exit $rc
done
TESTS=0 bash tools/gpu_ab.sh
