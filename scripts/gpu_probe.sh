#!/bin/bash
# One-call probe of the resident path: kernel trace phases (tools/res_trace.py) per config
# and the SQ counters of the C2 bench (scripts/gpu_sq.sh).
# usage: scripts/gpu_probe.sh TAG [CONFIG ...]   (outputs under gpurun_out/probe_TAG/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
CFGS=${@:-nyu}
O=$R/gpurun_out/probe_$TAG
mkdir -p $O
cd $R
for CFG in $CFGS; do
  BG=""; [ "$CFG" = kitti ] && BG="--bg 2"
  timeout -k 10 120 python tools/res_trace.py --config $CFG $BG --out $O/res_trace_$CFG.json > $O/res_trace_$CFG.log 2>&1 || exit 1
done
bash $R/scripts/gpu_sq.sh $TAG nyu || exit 1
cp -r $R/gpurun_out/sq_${TAG}_nyu $O/
