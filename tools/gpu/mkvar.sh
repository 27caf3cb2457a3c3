# Build a library variant with extra flags for the Riccati kernel's translation units only (other objects from
# build/obj), for A/B runs through tools/gpu/*.sh (CARMPC_LIB=build/exp_<name>/libcarmpc.so).
# usage: bash tools/gpu/mkvar.sh NAME [hipcc flags...]   e.g. NAME=u2 -DCARMPC_RIC_UNROLL=2
# SCHED overrides the scheduler flags (default: those of carmpc_amd/build.py); SCHED_M2 those of the polish
# launch's unit alone.
set -e
cd "$(dirname "$0")/../.."
v=$1; shift
mkdir -p build/exp_$v
DEF="-mllvm --amdgpu-sched-strategy=iterative-ilp -mllvm --amdgpu-mfma-vgpr-form"
S=${SCHED-$DEF}
pids=""
for u in ipm_riccati ipm_riccati_m0 ipm_riccati_m1 ipm_riccati_m2 ipm_riccati_het; do
  F=$S
  [ $u = ipm_riccati_m2 ] && F=${SCHED_M2--mllvm --amdgpu-mfma-vgpr-form}
  [ $u = ipm_riccati ] && F=""
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Iinclude \
      -Xclang -target-feature -Xclang -packed-fp32-ops $F "$@" -c carmpc_amd/csrc/$u.hip -o build/exp_$v/$u.o &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
objs=$(ls build/obj/*.o | grep -v ipm_riccati)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build/exp_$v/ipm_riccati*.o -o build/exp_$v/libcarmpc.so
echo "built build/exp_$v/libcarmpc.so"
