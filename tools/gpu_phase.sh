set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in C1 C3; do
  CFG=$c VPX_LIB=var/ph.so timeout -k 10 300 python tools/phase_prof.py > gpurun_out/phase_$c.log 2>&1 || exit $?
  echo "== $c"; grep -v amdgpu.ids gpurun_out/phase_$c.log | tail -2
done
