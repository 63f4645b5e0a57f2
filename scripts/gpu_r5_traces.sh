#!/bin/bash
# Resident traces (tools/res_trace.py, experiments build) under environment settings.
# usage: TAG=x scripts/gpu_r5_traces.sh CFG[:NAME=VAL[,NAME=VAL]] ...   (outputs under gpurun_out/TAG/)
set -o pipefail
O=gpurun_out/${TAG:-r5}; mkdir -p $O
for spec in "$@"; do
  CFG=${spec%%:*}; envs=""; [ "$spec" != "$CFG" ] && envs=${spec#*:}
  name=$(echo "$spec" | tr ':,=' '___')
  BG=""; [ "$CFG" = kitti ] && BG="--bg 2"
  ( for e in ${envs//,/ }; do export "$e"; done
    timeout -k 10 120 python tools/res_trace.py --config $CFG $BG --out $O/trace_$name.json > $O/trace_$name.log 2>&1 ) || { tail $O/trace_$name.log; exit 1; }
  python -c "import json;d=json.load(open('$O/trace_$name.json'));g=d['group0'];print('$spec', {k:(v['median'] if isinstance(v,dict) and 'median' in v else v) for k,v in g.items()})"
done
