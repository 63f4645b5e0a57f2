#!/bin/bash
# round-4 final evidence, part a (one call): same-box A/B of this tree vs the poison commit,
# then the round script's part a (full GPU suite, default bench line, kernel stats)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
L=nlspn_eccv20_amd/lib/ab
O=gpurun_out/exp_r4o; mkdir -p $O
for CFG in nyu kitti nyu_b1; do
  AB_CONFIG=$CFG bash scripts/gpu_ab.sh poison=$L/libnlspn_r4poison.so cur=- > $O/ab_$CFG.txt 2>&1 || { cat $O/ab_$CFG.txt; exit 1; }
  echo "== $CFG"; cat $O/ab_$CFG.txt
done
PART=a bash scripts/gpu_round.sh r04 || exit 1
tail -3 gpurun_out/round_r04/pytest_gpu.log
python -c "import json;d=json.load(open('gpurun_out/round_r04/bench.json'));print(d['value'], {k:v['value'] for k,v in d['configs'].items()})"
