# A/B of an environment switch, printing the kernel-table rows whose tag contains PAT:
#   VAR=PU_X VALUES="1 0" CONFIG=c3 PAT=lean bash tools/ab_env_tags.sh
set -u
mkdir -p gpurun_out/abt
for r in 1 2 3; do
  for v in $VALUES; do
    env $VAR=$v timeout -k 10 200 python bench.py --config ${CONFIG:-c2} --no-cpu-baseline --no-oja > gpurun_out/abt/$v.$r.log 2>&1 || exit 1
    tail -1 gpurun_out/abt/$v.$r.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
ks=d['kernels']; sel=[(k, v) for k, v in ks.items() if '${PAT:-}' in k]
print('$VAR=$v r$r', d['value'], d['ms_per_step'], ' | '.join('%s %.0fx%.3f' % (k, v['launches_per_step'], v['ms_per_step']) for k, v in sel))"
  done
done
