# Round 4: walk phase split (step / skip cycles and lanes) of the current walkers, C1 / C2 / C3.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4f
export TMPDIR=/tmp
O=gpurun_out/r4f
for c in C1 C2 C3; do
  VPX_LIB=var/ph.so CFG=$c timeout -k 10 300 python tools/phase_prof.py > $O/ph_$c.log 2>&1; echo "$c rc=$?"; grep "^\[" $O/ph_$c.log
done
