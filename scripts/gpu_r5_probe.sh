#!/bin/bash
# Round-5 probes: setup-load microbenchmark (tools/setup_load_bench) and an env A/B (tools/ab_env.py).
# usage: AB_ENV="NAME=VAL" AB_CFGS=nyu,kitti,nyu_b1 scripts/gpu_r5_probe.sh TAG
set -o pipefail
O=gpurun_out/probe_$1; mkdir -p $O
if [ -x tools/setup_load_bench ]; then
  timeout -k 10 60 tools/setup_load_bench 27 > $O/setup_load_27.txt 2>&1 || exit 1
  timeout -k 10 60 tools/setup_load_bench 9 > $O/setup_load_9.txt 2>&1 || exit 1
  cat $O/setup_load_*.txt
fi
if [ -n "$AB_ENV" ]; then
  timeout -k 10 300 python tools/ab_env.py --env $AB_ENV --configs ${AB_CFGS:-nyu,kitti,nyu_b1} > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  cat $O/ab.json
fi
