# Lanes after releasing the context's own stream (3 / 4 lanes, two rounds), then the walker
# spill A/B (var/lib_*.so: base, shadow walkers at 5 / 6 waves/SIMD, bounce walkers at 5)
# on C1-C4 with 3 lanes.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/d
export TMPDIR=/tmp
O=gpurun_out/d
step() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so var/*.so > $O/lib.sha256
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for r in 1 2; do for pl in 3 4; do
  step bench_p${pl}_$r 300 python bench.py --no-cpu --pipeline $pl --steps 20
done; done
step share_C1_p4 300 env PIPE=4 CFG=C1 python tools/rank_share.py
for r in 1 2; do for L in var/lib_*.so; do n=$(basename $L .so)
  step ab_${n}_$r 300 env VPX_LIB=$L python bench.py --no-cpu --pipeline 3 --steps 20
done; done
