#!/bin/bash
# Round-end check of the final build in one GPU call: the -m gpu suite, smoke(), then the profile
# round (tools/profile_round.sh) whose summaries go to profiles/.   bash tools/round_final.sh [tag]
set -u
TAG=${1:-r02final}
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
bash tools/profile_round.sh $TAG
