#!/bin/bash
# Build an experiment variant of the library with extra -D flags into
# cmsis-dsp_amd/lib/variants/lib_<name>.so (load it with CMSISDSP_MI355X_LIB=...).
# Usage: tools/build_variant.sh <name> "-DFOO=1 -DBAR=2"
set -e
NAME=$1; DEFS=$2
cd "$(dirname "$0")/../cmsis-dsp_amd"
make -s -j8 >/dev/null
OUT=build/v_$NAME; mkdir -p $OUT lib/variants
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wno-unused-result $DEFS"
OBJS=""
for src in csrc/*.hip; do
  f=$(basename $src .hip)
  EXTRA=""; { [ $f = fir ] || [ $f = conv ] || [ $f = fir_lattice ]; } && EXTRA="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc $FLAGS $EXTRA -c $src -o $OUT/$f.o &
  OBJS="$OBJS $OUT/$f.o"
done
SRC_ID=$(cat build/srcid.stamp 2>/dev/null || echo unknown)
/opt/rocm/bin/hipcc $FLAGS -DMI355X_BUILD_DEFS="\"$DEFS\"" -DMI355X_SRC_ID="\"$SRC_ID\"" -c csrc/api.cpp -o $OUT/api.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o lib/variants/lib_$NAME.so \
  $OBJS $OUT/api.o build/runtime.o build/init.o build/buffer_sizes.o build/tables_data.o
echo "lib/variants/lib_$NAME.so"
