set -u
# Winograd wide items for the short-reduction (concat) data gradients: PU_WINO4_WIDE=2 vs 0
mkdir -p gpurun_out/r06h
for rep in 1 2; do for v in 0 2; do
  echo "== PU_WINO4_WIDE=$v"
  PU_WINO4_WIDE=$v timeout -k 10 150 python tools/conv_bench.py --layers top_cat,l2_cat --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids | grep -v peak || exit 1
done; done
for rep in 1 2; do for v in 0 2; do
  PU_WINO4_WIDE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-oja --no-kernel-profile > gpurun_out/r06h/c2_$v.json 2> gpurun_out/r06h/c2_$v.err || { tail -5 gpurun_out/r06h/c2_$v.err; exit 1; }
  echo -n "C2 PU_WINO4_WIDE=$v "; tail -1 gpurun_out/r06h/c2_$v.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done; done
