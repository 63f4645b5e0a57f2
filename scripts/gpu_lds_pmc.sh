#!/bin/bash
# LDS/issue PMC pass over the resident kernel (res_probe: full run, and with the
# staging switched off so the counters see the taps alone).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ldspmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
for d in 0 2; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/d$d -o run --output-format csv -- \
      python3 $R/tools/res_probe.py resident=1 dbgs=$d reps=5 > $O/d$d.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/ldspmc"
for d in ("d0", "d2"):
    fs = glob.glob(f"{O}/{d}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(list)
    for f in fs:
        for r in csv.DictReader(open(f)):
            if "resident" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d, {k: round(sum(v) / max(1, len(set(range(len(v))))) , 1) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()})
PY
