#!/bin/bash
set -u
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_coord_gpu.py tests/test_res_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ss_pytest.log 2>&1 || { tail -30 gpurun_out/ss_pytest.log; exit 1; }
tail -1 gpurun_out/ss_pytest.log
PAT=stem CONFIG=c2 bash tools/ab_lib_tags.sh libplastic_unet_igemmold.so || exit 1
PAT=x6s CONFIG=c5 bash tools/ab_lib_tags.sh libplastic_unet_smallconvold.so || exit 1
