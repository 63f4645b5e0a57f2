#!/bin/bash
# Same-box A/B of two library builds (NLSPN_LIB_PATH): C2 bench value, alternated.
set -o pipefail
O=gpurun_out/ab; mkdir -p $O
B=nlspn_eccv20_amd/lib/ab/libnlspn_hip_head.so
for r in 1 2 3; do
  for v in new head; do
    if [ $v = head ]; then export NLSPN_LIB_PATH=$B; else unset NLSPN_LIB_PATH; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-backward --no-gru --steps 200 --warmup 20 > $O/$v$r.json 2> $O/$v$r.err || exit 1
    python -c "import json;d=json.load(open('$O/$v$r.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_mean'])"
  done
done
