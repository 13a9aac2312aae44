set -u
# C3 eager vs HIP-graph step; the graph's replay queues (DEBUG_HIP_FORCE_GRAPH_QUEUES)
run() {
  local tag=$1; shift
  echo -n "$tag "
  timeout -k 10 240 env "$@" > gpurun_out/r06f/$tag.json 2> gpurun_out/r06f/$tag.err || { echo FAIL; tail -5 gpurun_out/r06f/$tag.err; return 1; }
  tail -1 gpurun_out/r06f/$tag.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
}
mkdir -p gpurun_out/r06f
B="python bench.py --config c3 --steps 40 --warmup 6 --no-cpu-baseline --no-kernel-profile --no-oja"
for rep in 1 2; do
  run eager$rep PU_X=0 $B --graph off || exit 1
  run graph$rep PU_X=0 $B --graph on || exit 1
  run graphq2_$rep DEBUG_HIP_FORCE_GRAPH_QUEUES=2 $B --graph on || exit 1
  run graphq4_$rep DEBUG_HIP_FORCE_GRAPH_QUEUES=4 $B --graph on || exit 1
done
