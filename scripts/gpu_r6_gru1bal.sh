#!/bin/bash
# Round 6: GRU1 workgroup balance — GRU-mode tests, per-layer timing (tools/gc_bench.py) and the
# bench's gru_section leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_gru1bal_${1:-a}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_gru.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gc_bench.py > $O/gc_bench.json 2> $O/gc_bench.err || { tail -5 $O/gc_bench.err; exit 1; }
cat $O/gc_bench.json
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-backward --no-heads --no-extra-configs --no-cpu-baseline \
    > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(json.dumps(d['gru_section']))"
