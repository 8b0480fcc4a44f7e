# tools/bin/libcyclone_<NAME>.so: the in-tree objects with SRC (one .hip of
# cycloneml_amd/csrc) rebuilt under extra DEFINES, for tools/ab_lib.sh.
# usage: bash tools/build_variant.sh NAME SRC "-DFOO=1 ..."
set -e
NAME=$1; SRC=$2; DEFS=$3
cd "$(dirname "$0")/../cycloneml_amd/csrc"
make -s -j8
base=$(basename "$SRC" .hip)
extra=""; [ "$base" = kmeans_i8 ] && extra="-fno-slp-vectorize"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $extra $DEFS -c -o /tmp/variant_$NAME.o "$base.hip"
objs=$(ls build/*.o | grep -v -e "build/$base.o" -e "build/blas.o")
mkdir -p ../../tools/bin
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../tools/bin/libcyclone_$NAME.so $objs /tmp/variant_$NAME.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
