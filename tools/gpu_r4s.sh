# Round 4: a third closed-form segment per lean skip (VPX_SEG3: fewer skips per shadow walk,
# more registers) — the GPU suite with it, then interleaved A/B against var/lib_noseg3.so on
# C1 / C2 / C3.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4s
export TMPDIR=/tmp
O=gpurun_out/r4s
sha256sum var/*.so | tee $O/lib.sha256
timeout -k 10 900 env VPX_LIB=var/lib_seg3.so python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -v amdgpu.ids $O/tests.log | tail -3 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2 3; do
  for L in seg3 noseg3; do
    b C1_$L.$rep C1 20 VPX_LIB=var/lib_$L.so
    b C2_$L.$rep C2 10 VPX_LIB=var/lib_$L.so
    b C3_$L.$rep C3 6 VPX_LIB=var/lib_$L.so
  done
done
