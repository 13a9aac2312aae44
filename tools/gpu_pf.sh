#!/bin/bash
# variant check: GPU tests on the product library and each variant library, then conv_bench
# base vs variants:   bash tools/gpu_pf.sh name1 name2 ...   (lib/libplastic_unet_<name>.so)
set -u
OUT=gpurun_out/variants; mkdir -p $OUT
TESTS="tests/test_kernels_gpu.py tests/test_precision_gpu.py tests/test_model_gpu.py"
timeout -k 10 300 python -m pytest $TESTS -q -x -p no:cacheprovider > $OUT/tests_base.log 2>&1 || { echo "tests base failed"; tail -20 $OUT/tests_base.log; exit 1; }
for v in "$@"; do
  PLASTIC_UNET_LIB=$PWD/plastic-unet_amd/lib/libplastic_unet_$v.so timeout -k 10 300 python -m pytest $TESTS -q -x -p no:cacheprovider > $OUT/tests_$v.log 2>&1 || { echo "tests $v failed rc=$?"; tail -20 $OUT/tests_$v.log; exit 1; }
done
bash tools/gpu_variants.sh "$@"
