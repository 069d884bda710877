# Default bench line (per-config frames in flight) twice, GPU suite + smoke, kernel-trace
# stats per config with the defaults, and the bounce-sort variant's kernel trace on C2 (serial
# frames) beside the in-tree library's.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/e
export TMPDIR=/tmp
O=gpurun_out/e
step() { name=$1; shift; echo "== $name"; timeout -k 10 "$@" > $O/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAILN:-1} | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
sha256sum raytracer-voxpopuli_amd/libvpx_hip.so var/*.so > $O/lib.sha256
step gputests 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_1 300 python bench.py --no-cpu --steps 20
step bench_2 300 python bench.py --no-cpu --steps 20
for c in C1 C2 C3 C4; do
  step prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_$c" -o run -- python bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-extra
done
step sortprof_base 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/sortprof_base" -o run -- python bench.py --config C2 --steps 5 --warmup 2 --no-cpu --no-extra --pipeline 0
step sortprof_sort 300 env VPX_LIB=var/lib_sort.so rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/sortprof_sort" -o run -- python bench.py --config C2 --steps 5 --warmup 2 --no-cpu --no-extra --pipeline 0
