#!/bin/bash
# End-to-end A/B of the default library against a variant .so: bench lines alternating on one box.
#   bash tools/ab_bench_libs.sh tag variant.so "c2 c3"
set -u
O=gpurun_out/$1; mkdir -p $O
VAR=plastic-unet_amd/lib/$2
for c in ${3:-c2}; do
  for lib in default $2 default $2; do
    if [ $lib = default ]; then E=""; else E="PLASTIC_UNET_LIB=$VAR"; fi
    env $E timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/${c}_$lib.log 2>&1 || { tail -20 $O/${c}_$lib.log; exit 1; }
    echo "$c $lib: $(tail -1 $O/${c}_$lib.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], (d.get("oja_update") or {}).get("fused_head_bs32", {}).get("us_per_launch"))')"
  done
done
