#!/bin/bash
# Round 6: SQ counters (two passes of <= 8 SQ counters) and HBM traffic (FETCH_SIZE / WRITE_SIZE,
# separate passes) of the backward kernels at C2 (tools/ab_bwd.py, product build, resident form).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_bwdsq_${1:-a}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
n=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
         FETCH_SIZE WRITE_SIZE; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/p$n -o run --output-format csv -- \
      python3 $R/tools/ab_bwd.py --config nyu --rounds 1 --per 2 res= > $O/p$n.log 2>&1 || exit 1
done
python3 $R/tools/sq_summary.py $O/sq_summary.json $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv \
    --kernel bwd_ > $O/sq_summary.txt 2>&1 || exit 1
cat $O/sq_summary.txt
python3 - $O <<'PY'
import csv, collections, json, sys
o = sys.argv[1]
res = {}
for n, c in ((3, "FETCH_SIZE"), (4, "WRITE_SIZE")):
    acc = collections.defaultdict(list)
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f"{o}/p{n}/run_counter_collection.csv")):
        if "bwd_" not in r["Kernel_Name"]:
            continue
        k = (r.get("Dispatch_Id") or r.get("Correlation_Id"))
        per[k] += float(r["Counter_Value"]); names[k] = r["Kernel_Name"].split("(")[0]
    for k, v in per.items():
        acc[names[k]].append(v)
    for kn, v in acc.items():
        res.setdefault(kn, {})[c + "_kB_mean"] = sum(v) / len(v)
print(json.dumps(res, indent=1))
json.dump(res, open(f"{o}/traffic.json", "w"), indent=1)
PY
