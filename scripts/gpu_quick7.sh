#!/bin/bash
# Resident kernel: its GPU tests, a timing probe with the decomposition switches, bench line.
set -o pipefail
O=gpurun_out/q9; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_resident.py > $O/pytest_res.log 2>&1 || { echo "pytest resident failed"; tail -40 $O/pytest_res.log; exit 1; }
tail -2 $O/pytest_res.log
timeout -k 10 120 python tools/res_probe.py resident=1 dbgs=0,2,6 > $O/probe.txt 2>&1 && cat $O/probe.txt || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-backward --no-gru > $O/bench.json 2> $O/bench.err && cut -c1-400 $O/bench.json
