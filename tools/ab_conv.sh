# A/B timing of two library builds on tools/conv_bench.py (alternating, 2 rounds each):
#   LIBS="lib/a.so lib/b.so" LAYERS=top,l3 OPS=fwd,dgrad,wgrad bash tools/ab_conv.sh
set -u
mkdir -p gpurun_out/ab
i=0
for round in 1 2; do
  for L in $LIBS; do
    i=$((i+1))
    PLASTIC_UNET_LIB=$L timeout -k 10 180 python tools/conv_bench.py --layers ${LAYERS:-top,l2,l3,l4} --ops ${OPS:-fwd,dgrad,wgrad} --reps 20 > gpurun_out/ab/r$i.log 2>&1 || exit 1
    echo "== $L (round $round)"; grep -E "TF" gpurun_out/ab/r$i.log
  done
done
