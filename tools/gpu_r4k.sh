# Round 4: the level fork on frames in flight with the fork streams on dedicated hardware
# queues (var/lib_forklanes.so) or from the shared queue pool (var/lib_forklanes_pooled.so),
# against the shipped build (var/lib_base.so: fork only on the context's stream), C2 / Z1.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4k
export TMPDIR=/tmp
O=gpurun_out/r4k
sha256sum var/*.so | tee $O/lib.sha256
b() { tag=$1; cfg=$2; st=$3; shift 3; timeout -k 10 300 env "$@" python bench.py --config $cfg --steps $st --warmup 2 --no-cpu --no-extra $PIPE > $O/$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"serial_ms_per_frame": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; [ $rc -ne 0 ] && { tail -3 $O/$tag.log; exit $rc; }; return 0; }
for rep in 1 2 3; do
  PIPE="--pipeline 3" b C2_base_p3.$rep C2 10 VPX_LIB=var/lib_base.so
  PIPE="--pipeline 2" b C2_forklanes_p2.$rep C2 10 VPX_LIB=var/lib_forklanes.so
  PIPE="--pipeline 2" b C2_pooled_p2.$rep C2 10 VPX_LIB=var/lib_forklanes_pooled.so
  PIPE="--pipeline 3" b C2_pooled_p3.$rep C2 10 VPX_LIB=var/lib_forklanes_pooled.so
  PIPE="--pipeline 3" b Z1_base_p3.$rep Z1 10 VPX_LIB=var/lib_base.so
  PIPE="--pipeline 2" b Z1_pooled_p2.$rep Z1 10 VPX_LIB=var/lib_forklanes_pooled.so
  PIPE="--pipeline 3" b Z1_pooled_p3.$rep Z1 10 VPX_LIB=var/lib_forklanes_pooled.so
done
