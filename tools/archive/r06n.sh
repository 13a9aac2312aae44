set -u
# C3: bf16 halo weight-gradient splits divided by PU_BF16_WG_DIV (1 = default)
mkdir -p gpurun_out/r06n
for rep in 1 2; do for v in 1 2 4; do
  PU_BF16_WG_DIV=$v timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --no-oja --no-kernel-profile > gpurun_out/r06n/c3_$v.json 2> gpurun_out/r06n/c3_$v.err || { tail -5 gpurun_out/r06n/c3_$v.err; exit 1; }
  echo -n "C3 div=$v "; tail -1 gpurun_out/r06n/c3_$v.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done; done
