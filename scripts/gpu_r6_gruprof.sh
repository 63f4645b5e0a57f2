#!/bin/bash
# Round 6: kernel breakdown of the GRU-mode section (tools/gru_prof.py) under rocprofv3,
# MIOpen default and tuned channels_last.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_gruprof_${1:-a}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/def -o run --output-format csv -- \
    python3 $R/tools/gru_prof.py --steps 5 > $O/def.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/cl -o run --output-format csv -- \
    python3 $R/tools/gru_prof.py --steps 5 --bench 1 --cl 1 > $O/cl.log 2>&1 || exit 1
tail -2 $O/def.log $O/cl.log
