# tools/bin/libcyclone_<NAME>.so: the in-tree objects with one source of
# cycloneml_amd/csrc rebuilt -- under extra DEFINES, or as it was at a git
# revision (SRC = REV:name.hip) -- for tools/ab_lib.sh.
# An A/B baseline is built from the committed kernel (REV:), not from a
# define of the rewritten one: a rewrite can change more than its switch.
# usage: bash tools/build_variant.sh NAME SRC "-DFOO=1 ..."
#        bash tools/build_variant.sh orig HEAD~1:logistic.hip
set -e
NAME=$1; SRC=$2; DEFS=${3:-}
cd "$(dirname "$0")/../cycloneml_amd/csrc"
make -s -j8
if [[ "$SRC" == *:* ]]; then
  rev=${SRC%%:*}; file=${SRC#*:}
  base=$(basename "$file" .hip)
  git show "$rev:cycloneml_amd/csrc/$base.hip" > /tmp/variant_src_$NAME.hip
  in=/tmp/variant_src_$NAME.hip
else
  base=$(basename "$SRC" .hip)
  in=$base.hip
fi
extra=""; [ "$base" = kmeans_i8 ] && extra="-fno-slp-vectorize"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I. $extra $DEFS -c -o /tmp/variant_$NAME.o "$in"
objs=$(ls build/*.o | grep -v -e "build/$base.o" -e "build/blas.o")
mkdir -p ../../tools/bin
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../tools/bin/libcyclone_$NAME.so $objs /tmp/variant_$NAME.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
