# Round 4: the split multi-volume primary (world walk + k_instances) — GPU suite, then
# interleaved A/Bs on C4 and Z1 against the one-launch primary (var/lib_nosplit.so), and the
# C4 stage split (tools/c4_split.py).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4d
export TMPDIR=/tmp
O=gpurun_out/r4d
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so var/*.so | tee $O/lib.sha256
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -v amdgpu.ids $O/tests.log | tail -4 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
fi
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"stages_ms": {[^}]*}\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2; do
  b C4_split.$rep C4 3 VPX_LIB=var/lib_base.so
  b C4_nosplit.$rep C4 3 VPX_LIB=var/lib_nosplit.so
  b C4_nocull.$rep C4 3 VPX_LIB=var/lib_nocull.so
  b Z1_split.$rep Z1 10 VPX_LIB=var/lib_base.so
  b Z1_nosplit.$rep Z1 10 VPX_LIB=var/lib_nosplit.so
done
timeout -k 10 300 python tools/c4_split.py > $O/c4_split.json 2> $O/c4_split.err; echo "c4_split rc=$?"; python -c "
import json; d=json.load(open('$O/c4_split.json'))
for k,v in d.items(): print(k, v['ms_per_frame'], v['stages_ms'])"
