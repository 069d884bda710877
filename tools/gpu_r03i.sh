# Walk phase split (step / skip phases, VPX_PHASE_PROF build var/ph.so) for C1 / C2 / C3 with
# the round-3 kernels, and C1 / C4 at 3 vs 4 lanes with k_frame0 at 6 waves/SIMD.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/i
export TMPDIR=/tmp
O=gpurun_out/i
for c in C1 C2 C3; do
  CFG=$c VPX_LIB=var/ph.so timeout -k 10 300 python tools/phase_prof.py > $O/phase_$c.log 2>&1 || exit 1
  echo "== $c"; grep -v amdgpu.ids $O/phase_$c.log | tail -2
done
for r in 1 2; do for pl in 3 4; do
  timeout -k 10 300 python bench.py --no-cpu --no-extra --steps 30 --pipeline $pl > $O/c1_p${pl}_$r.log 2>&1 || exit 1
  echo "$r C1 p$pl $(grep -o '"ms_per_step": [0-9.]*' $O/c1_p${pl}_$r.log)"
  timeout -k 10 300 python bench.py --config C4 --no-cpu --no-extra --steps 5 --warmup 1 --pipeline $pl > $O/c4_p${pl}_$r.log 2>&1 || exit 1
  echo "$r C4 p$pl $(grep -o '"ms_per_step": [0-9.]*' $O/c4_p${pl}_$r.log)"
done; done
