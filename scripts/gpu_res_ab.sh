#!/bin/bash
# Resident-kernel iteration: its GPU tests, a per-iteration timing probe, launch
# overhead probe and a short bench line.
set -o pipefail
O=gpurun_out/res_ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python tools/res_probe.py resident=1,0 dbgs=0 > $O/probe.txt 2>&1 && cat $O/probe.txt &&
timeout -k 10 120 python tools/launch_probe.py > $O/launch.txt 2>&1 && cat $O/launch.txt &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-backward --no-gru > $O/bench.json 2> $O/bench.err && cat $O/bench.json
