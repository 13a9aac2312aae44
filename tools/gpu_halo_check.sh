#!/bin/bash
# Halo conv kernel iteration: its parity tests, conv_bench A/B (halo vs per-tap) on the halo-eligible
# C2 layers, then the C2 bench line.   bash tools/gpu_halo_check.sh [tag] [--bench]
set -u
O=gpurun_out/${1:-h1}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_halo_conv_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/conv_bench.py --layers top,top_cat,l2,l2_cat,l3 --ops fwd,dgrad > $O/cb_halo.txt 2>&1 || { tail -20 $O/cb_halo.txt; exit 1; }
PU_CONV_HALO=0 timeout -k 10 200 python tools/conv_bench.py --layers top,top_cat,l2,l2_cat,l3 --ops fwd,dgrad > $O/cb_lean.txt 2>&1 || { tail -20 $O/cb_lean.txt; exit 1; }
grep -v amdgpu.ids $O/cb_halo.txt; grep -v amdgpu.ids $O/cb_lean.txt
if [ "${2:-}" = "--bench" ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | cut -c1-300
fi
