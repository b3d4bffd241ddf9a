#!/bin/bash
# Builds the A/B baseline library: the engine with the kernel translation
# units KERNELS taken from git revision REV (default HEAD), everything else
# (and every header) as in the working tree.
#   tools/build_ab_base.sh [REV] [KERNEL ...]   (KERNEL default spf_route_wave)
# -> openr_amd/lib/libopenr_gpu_base.so (tools/c3_opt_ab.py variant lib=base)
set -e
REV=${1:-HEAD}
shift || true
KS=${*:-spf_route_wave}
H=/opt/rocm/bin/hipcc
T=$(mktemp -d)
cp openr_amd/csrc/kernels/*.h "$T/"
make -s all
objs=$(ls build/kernels/*.o)
for K in $KS; do
  git show "$REV:openr_amd/csrc/kernels/$K.hip" > "$T/$K.hip"
  $H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I"$T" -c "$T/$K.hip" -o "$T/$K.o" &
  objs=$(echo "$objs" | grep -v "/$K.o")
done
wait
$H --offload-arch=gfx950 -shared $objs $(for K in $KS; do echo "$T/$K.o"; done) -o openr_amd/lib/libopenr_gpu_base.so
rm -rf "$T"
echo "built A/B base ($KS @ $REV)"
