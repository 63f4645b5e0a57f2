#!/bin/bash
# Round 6: kernel breakdown of the native GRU-mode section (tools/gru_prof.py) under rocprofv3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_gruprof_${1:-a}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/nat -o run --output-format csv -- \
    python3 $R/tools/gru_prof.py --steps 10 > $O/nat.log 2>&1 || exit 1
tail -2 $O/nat.log
