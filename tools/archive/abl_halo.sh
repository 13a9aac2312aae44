# halo weight-gradient timing ablations (wrong results; libraries built with -D PU_ABL=<bits>)
set -u
mkdir -p gpurun_out/abl
for a in ${ABL:-0 1 2 4 6 7}; do
  if [ $a = 0 ]; then L=plastic-unet_amd/lib/libplastic_unet.so; else L=plastic-unet_amd/lib/abl$a.so; fi
  PLASTIC_UNET_LIB=$L timeout -k 10 120 python tools/conv_bench.py --layers top,l2,l3,l4 --ops wgrad --reps 20 > gpurun_out/abl/a$a.log 2>&1 || exit 1
  echo "== abl $a"; grep -i "wgrad" gpurun_out/abl/a$a.log | head -8
done
