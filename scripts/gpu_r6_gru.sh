#!/bin/bash
# Round 6: the GRU-mode section with the native convolutions — the bench's gru_section leg
# (native vs MIOpen modules) and a kernel breakdown of the native section (rocprofv3).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_gru_${1:-a}; mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-backward --no-heads --no-extra-configs --no-cpu-baseline \
    > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(json.dumps(d['gru_section']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/tools/gru_prof.py --steps 5 > $O/prof.log 2>&1 || exit 1
cat $O/prof.log
