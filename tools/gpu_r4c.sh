# Round 4: where C4's frame goes (tools/c4_split.py) and the zone scene's stages; the bench
# line with Z1 among the extras.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c
export TMPDIR=/tmp
O=gpurun_out/r4c
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so | tee $O/lib.sha256
timeout -k 10 300 python tools/c4_split.py > $O/c4_split.json 2> $O/c4_split.err; rc=$?; echo "c4_split rc=$rc"; cat $O/c4_split.json | head -80; [ $rc -ne 0 ] && { tail -5 $O/c4_split.err; exit $rc; }
timeout -k 10 600 python bench.py --no-cpu > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 3000 $O/bench.log | cut -c1-3000
