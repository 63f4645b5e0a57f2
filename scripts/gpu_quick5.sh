#!/bin/bash
set -o pipefail
O=gpurun_out/q5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python tools/res_probe.py resident=1 dbgs=0,1,2,4,3,6,7 > $O/probe.txt 2>&1 && cat $O/probe.txt &&
timeout -k 10 120 python tools/launch_probe.py > $O/launch.txt 2>&1 && cat $O/launch.txt &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-backward --no-gru > $O/bench.json 2> $O/bench.err && cat $O/bench.json
