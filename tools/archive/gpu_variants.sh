#!/bin/bash
# conv_bench over variant libraries (build_native.py -D ... --lib lib/libplastic_unet_<name>.so)
#   bash tools/gpu_variants.sh name1 name2 ...     (product library first, as "base")
set -u
OUT=gpurun_out/variants
mkdir -p $OUT
timeout -k 10 300 python tools/conv_bench.py > $OUT/base.log 2>&1 || exit $?
for v in "$@"; do
  PLASTIC_UNET_LIB=$PWD/plastic-unet_amd/lib/libplastic_unet_$v.so timeout -k 10 300 python tools/conv_bench.py > $OUT/$v.log 2>&1 || exit $?
done
