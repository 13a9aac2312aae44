# A/B of an environment switch on a bench config (alternating, 2 rounds):
#   VAR=PU_BF16_KG VALUES="1 2 3" CONFIG=c3 bash tools/ab_env_bench.sh
set -u
mkdir -p gpurun_out/abe
for r in 1 2; do
  for v in $VALUES; do
    env $VAR=$v timeout -k 10 200 python bench.py --config ${CONFIG:-c2} --no-cpu-baseline --no-oja > gpurun_out/abe/$v.$r.log 2>&1 || exit 1
    tail -1 gpurun_out/abe/$v.$r.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
ks=d['kernels']; top=sorted(ks.items(), key=lambda kv:-kv[1]['ms_per_step'])[:5]
print('$VAR=$v r$r', d['value'], d['ms_per_step'], ' | '.join('%s %.3f' % (k, v['ms_per_step']) for k, v in top))"
  done
done
