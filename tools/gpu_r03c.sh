# LDS-resident depth-0 frame + frames-in-flight A/B (0 / 3 / 4 lanes, two rounds), the
# one-GPU rank shares, and a kernel trace of the pipelined C1 bench (busy time per dispatch).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c
export TMPDIR=/tmp
O=gpurun_out/c
step() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-2} | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so > $O/lib.sha256
step gputests 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
for r in 1 2; do for pl in 0 3 4; do
  step bench_p${pl}_$r 300 python bench.py --no-cpu --pipeline $pl --steps 20
done; done
for pl in 0 3 4; do step share_C1_p$pl 300 env PIPE=$pl CFG=C1 python tools/rank_share.py; done
step share_C3_p3 300 env PIPE=3 CFG=C3 K=10 python tools/rank_share.py
step prof_C1_p3 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_C1_p3" -o run -- python bench.py --steps 20 --warmup 3 --no-cpu --no-extra --pipeline 3
python tools/trace_busy.py $O/prof_C1_p3/run_kernel_trace.csv k_frame0 composite
