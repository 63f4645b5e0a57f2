#!/bin/bash
# Round 6: GRU-mode tests + the GRU section's kernel breakdown after a gconv change.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_gsmall_${1:-a}; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_gru.py tests/test_backward_golden.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/nat -o run --output-format csv -- \
    python3 $R/tools/gru_prof.py --steps 10 > $O/nat.log 2>&1 || exit 1
tail -1 $O/nat.log
