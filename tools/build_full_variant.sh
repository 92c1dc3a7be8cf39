# Build a libbos.so variant with every source (host and HIP) compiled with extra flags, into
# gpurun_exp/libbos_<name>.so (experiments that change host-side layout constants too).
# Usage: tools/build_full_variant.sh name "flags"
set -e
cd "$(dirname "$0")/../prb-project-bearing-only-slam_amd"
name=$1; flags=$2
HIPFLAGS="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-parameter -Wno-unused-result -mllvm -pragma-unroll-threshold=1000000 -mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize"
CXXFLAGS="-O2 -pthread -fPIC -std=c++17 -Wno-unused-parameter -I/opt/rocm/include"
LD="-pthread -L/opt/rocm/lib -lrocsolver -lrocblas -lrccl -Wl,--no-as-needed -lrocsparse -Wl,--as-needed -lamdhip64 -Wl,-rpath,/opt/rocm/lib"
D=/tmp/fv_$name
mkdir -p $D ../gpurun_exp
objs=""
for f in csrc/host/*.cpp; do b=$(basename $f .cpp); g++ $CXXFLAGS $flags -c $f -o $D/h_$b.o & objs="$objs $D/h_$b.o"; done
for f in csrc/hip/*.hip; do b=$(basename $f .hip); /opt/rocm/bin/hipcc $HIPFLAGS $flags -x hip -c $f -o $D/d_$b.o & objs="$objs $D/d_$b.o"; done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../gpurun_exp/libbos_$name.so $objs $LD
echo built gpurun_exp/libbos_$name.so
