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
for f in cfft_f32 cfft_fixed rfft_f32 mat_mult_f32 mfcc_f32; do /opt/rocm/bin/hipcc $FLAGS -c csrc/$f.hip -o $OUT/$f.o & done
/opt/rocm/bin/hipcc $FLAGS -fno-slp-vectorize -c csrc/fir.hip -o $OUT/fir.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o lib/variants/lib_$NAME.so \
  $OUT/cfft_f32.o $OUT/cfft_fixed.o $OUT/rfft_f32.o $OUT/fir.o $OUT/mat_mult_f32.o $OUT/mfcc_f32.o \
  build/runtime.o build/api.o build/init.o build/tables_data.o
echo "lib/variants/lib_$NAME.so"
