# Build a variant of libvpx_hip.so into var/lib_<name>.so with extra -D flags, for
# tools/gpu_var.sh A/B runs.  Usage: tools/build_var.sh <name> [-DFLAG=...]...
# (name "ph" builds var/ph.so, the phase-profiling library used by tools/phase_prof.py.)
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
out=var/lib_$name.so; [ "$name" = ph ] && out=var/ph.so
mkdir -p var
C=raytracer-voxpopuli_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fgpu-flush-denormals-to-zero -Wall "$@" \
  -shared -o $out $C/vpx_kernels.hip $C/vpx_host.cpp $C/vpx_x86_host.cpp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built $out"
