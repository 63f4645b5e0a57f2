#!/bin/bash
# Round 6: pass 2 with fused multiply-adds (A/B library built with -DNLSPN_BWD_FC=1) against the
# experiments build: tools/ab_bwd.py in two processes back to back, twice each (alternated).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_fc_${1:-a}; mkdir -p $O
cd $R
for r in 1 2; do
  for v in exp fc; do
    lib=$R/nlspn_eccv20_amd/lib/exp/libnlspn_hip_exp.so; [ $v = fc ] && lib=$R/nlspn_eccv20_amd/lib/exp/libnlspn_fc.so
    NLSPN_LIB_PATH=$lib timeout -k 10 200 python tools/ab_bwd.py --config nyu res= steps=NLSPN_BWD_RESIDENT=0 \
        > $O/ab_${v}_$r.json 2> $O/ab_${v}_$r.err || { tail -5 $O/ab_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/ab_${v}_$r.json'));print('$v', d['res'], d['steps'])"
  done
done
