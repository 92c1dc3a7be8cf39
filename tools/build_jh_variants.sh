# Build libbos.so variants that differ only in the compile flags of the HIP sources (kernels.hip,
# multifrontal.hip, solver_capi.hip: J+H and solver experiments), into gpurun_exp/: the host objects
# from the in-tree build (make first). Usage: tools/build_jh_variants.sh name1 "flags1" [name2 "flags2" ...]
set -e
cd "$(dirname "$0")/../prb-project-bearing-only-slam_amd"
HIPFLAGS="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-parameter -Wno-unused-result -mllvm -pragma-unroll-threshold=1000000 -mllvm -amdgpu-mfma-vgpr-form=1"
LD="-pthread -L/opt/rocm/lib -lrocsolver -lrocblas -lrccl -Wl,--no-as-needed -lrocsparse -Wl,--as-needed -lamdhip64 -Wl,-rpath,/opt/rocm/lib"
mkdir -p ../gpurun_exp /tmp/jhv
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc $HIPFLAGS $flags -x hip -c csrc/hip/kernels.hip -o /tmp/jhv/k_$name.o &
  /opt/rocm/bin/hipcc $HIPFLAGS $flags -x hip -c csrc/hip/solver_capi.hip -o /tmp/jhv/c_$name.o &
  /opt/rocm/bin/hipcc $HIPFLAGS $flags -x hip -c csrc/hip/multifrontal.hip -o /tmp/jhv/m_$name.o &
  wait
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../gpurun_exp/libbos_$name.so build/host/*.o /tmp/jhv/k_$name.o /tmp/jhv/m_$name.o /tmp/jhv/c_$name.o $LD
  echo built gpurun_exp/libbos_$name.so
done
