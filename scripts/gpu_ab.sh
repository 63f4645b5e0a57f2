#!/bin/bash
# Same-box A/B of library builds / env toggles: C2 bench value, alternated rounds.
# usage: scripts/gpu_ab.sh NAME=LIBPATH_OR_-[:ENV=VAL] ...   ("-" = the in-tree build)
# e.g.   scripts/gpu_ab.sh cur=- r01=nlspn_eccv20_amd/lib/ab/libnlspn_r01.so noguard=nlspn_eccv20_amd/lib/exp/libnlspn_hip_exp.so:NLSPN_RES_GUARD=0
set -o pipefail
O=gpurun_out/ab; mkdir -p $O
CFG=${AB_CONFIG:-nyu}
for r in 1 2 3; do
  for spec in "$@"; do
    name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; envs=""
    [ "$rest" != "$lib" ] && envs=${rest#*:}
    ( if [ "$lib" != "-" ]; then export NLSPN_LIB_PATH=$lib; else unset NLSPN_LIB_PATH; fi
      for e in ${envs//,/ }; do export "$e"; done
      timeout -k 10 120 python bench.py --config $CFG --no-cpu-baseline --no-backward --no-gru --no-extra-configs --no-heads \
          --steps 200 --warmup 20 > $O/$name$r.json 2> $O/$name$r.err ) || exit 1
    python -c "import json;d=json.load(open('$O/$name$r.json'));print('$name', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'])"
  done
done
