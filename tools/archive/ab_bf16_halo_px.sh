# bf16 halo conv: 256- vs 512-pixel blocks (PU_BF16_HALO_PX), parity tests under 512, conv A/B, C3 bench
set -u
O=gpurun_out/abpx; mkdir -p $O
PU_BF16_HALO_PX=512 timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -x -q --timeout 150 --timeout-method thread > $O/pytest512.log 2>&1 || { tail -30 $O/pytest512.log; exit 1; }
tail -1 $O/pytest512.log
for rep in 1 2; do for px in 256 512; do
  PU_BF16_HALO_PX=$px timeout -k 10 200 python tools/conv_bench.py --bf16 --layers top,top_cat,l2,l2_cat,l3 --ops fwd,dgrad > $O/cb_$px.$rep.txt 2>&1 || exit 1
  echo "== px $px ($rep)"; grep -v "amdgpu.ids\|peak" $O/cb_$px.$rep.txt
done; done
for px in 256 512; do
  PU_BF16_HALO_PX=$px timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $O/c3_$px.log 2>&1 || exit 1
  echo "c3 px $px: $(tail -1 $O/c3_$px.log | cut -c1-120)"
done
