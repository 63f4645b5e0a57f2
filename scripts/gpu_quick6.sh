#!/bin/bash
# Resident kernel (whole section, granule hand-offs): its GPU tests, a timing probe,
# the full GPU suite and a bench line.
set -o pipefail
O=gpurun_out/q6; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_resident.py > $O/pytest_res.log 2>&1 || { echo "pytest resident failed"; tail -40 $O/pytest_res.log; exit 1; }
tail -2 $O/pytest_res.log
timeout -k 10 120 python tools/res_probe.py resident=1,0 dbgs=0 > $O/probe.txt 2>&1 && cat $O/probe.txt || exit 1
timeout -k 10 120 python tools/launch_probe.py > $O/launch.txt 2>&1 && cat $O/launch.txt || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-backward --no-gru > $O/bench.json 2> $O/bench.err && cat $O/bench.json
