# Round 4: C4 instance-pass A/Bs (per-lane instance walks with bound culling vs the
# wave-uniform union loop) and the diagnostic no-walk build's stage split.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4e
export TMPDIR=/tmp
O=gpurun_out/r4e
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so var/*.so | tee $O/lib.sha256
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -v amdgpu.ids $O/tests.log | tail -3 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
fi
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"stages_ms": {[^}]*}\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2; do
  b C4_base.$rep C4 3 VPX_LIB=var/lib_base.so
  b C4_nolanes.$rep C4 3 VPX_LIB=var/lib_nolanes.so
done
for L in base nolanes diagnowalk; do
  VPX_LIB=var/lib_$L.so timeout -k 10 300 python tools/c4_split.py > $O/split_$L.json 2> $O/split_$L.err; echo "split $L rc=$?"
  python -c "
import json; d=json.load(open('$O/split_$L.json'))
for k,v in d.items(): print('  ', k, v['ms_per_frame'], v['stages_ms'], int(v['rays_per_frame']['cells']))"
done
