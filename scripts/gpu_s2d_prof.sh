#!/bin/bash
# S2D front: timing vs torch ops, rocprof kernel stats, and one SQ counter pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s2dp
mkdir -p $O
timeout -k 10 120 python $R/tools/s2d_bench.py > $O/bench.txt 2>&1 && cat $O/bench.txt || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/stats -o s2d --output-format csv -- \
    python3 $R/tools/s2d_bench.py > /dev/null 2>&1 || exit 1
grep -i "s2d_pyramid" $O/stats/s2d_kernel_stats.csv | cut -c1-150
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/pmc -o run --output-format csv -- \
    python3 $R/tools/s2d_bench.py > /dev/null 2>&1 || exit 1
python3 - <<PY
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("$O/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "s2d_pyramid" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({k: round(sum(v) / len(v)) for k, v in acc.items()})
PY
