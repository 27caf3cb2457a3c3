# Build a library variant with extra flags for ipm_riccati.hip only (other objects from build/obj),
# for A/B runs through tools/gpu/sched_sweep.sh (CARMPC_LIB=build/exp_<name>/libcarmpc.so).
# usage: bash tools/gpu/mkvar.sh NAME [hipcc flags...]   e.g. NAME=u2 -DCARMPC_RIC_UNROLL=2
# SCHED overrides the scheduler flag (default: the iterative-ILP strategy of carmpc_amd/build.py).
set -e
cd "$(dirname "$0")/../.."
v=$1; shift
mkdir -p build/exp_$v
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Iinclude \
    -Xclang -target-feature -Xclang -packed-fp32-ops \
    ${SCHED--mllvm --amdgpu-sched-strategy=iterative-ilp -mllvm --amdgpu-mfma-vgpr-form} "$@" -c carmpc_amd/csrc/ipm_riccati.hip -o build/exp_$v/ipm_riccati.o
objs=$(ls build/obj/*.o | grep -v ipm_riccati)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build/exp_$v/ipm_riccati.o -o build/exp_$v/libcarmpc.so
echo "built build/exp_$v/libcarmpc.so"
