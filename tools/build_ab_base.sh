#!/bin/bash
# Builds the A/B baseline libraries for tools/gpu_wave_ab.sh: the engine with
# ONE kernel translation unit taken from git revision REV (default HEAD),
# everything else as in the working tree.
#   tools/build_ab_base.sh [REV] [KERNEL]   (KERNEL default spf_route_wave)
# -> openr_amd/lib/libopenr_gpu_base.so, openr_amd/lib/libopenr_gpu_stamps_base.so
set -e
REV=${1:-HEAD}
K=${2:-spf_route_wave}
H=/opt/rocm/bin/hipcc
T=$(mktemp -d)
git show "$REV:openr_amd/csrc/kernels/$K.hip" > "$T/$K.hip"
cp openr_amd/csrc/kernels/*.h "$T/"
make -s all stamps
$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I"$T" -c "$T/$K.hip" -o "$T/base.o"
$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DOGS_STAMPS -Iinclude -I"$T" -c "$T/$K.hip" -o "$T/base_st.o"
objs=$(ls build/kernels/*.o | grep -v "/$K.o" | grep -v "/diag_")
sobjs=$(ls build/stamps/*.o | grep -v "/$K.o" | grep -v "/diag_")
$H --offload-arch=gfx950 -shared $objs "$T/base.o" -o openr_amd/lib/libopenr_gpu_base.so
$H --offload-arch=gfx950 -shared $sobjs "$T/base_st.o" -o openr_amd/lib/libopenr_gpu_stamps_base.so
rm -rf "$T"
echo "built A/B base ($K.hip @ $REV)"
