#!/bin/bash
# Issue / LDS / memory counters over tools/step_bench k16f16 (C5 shape), one pass per group.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sbpmc2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1
grep -oE "SQ_[A-Z_]+" $O/avail.txt | sort -u > $O/sq_names.txt
P1="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY"
i=0
for C in "$P1" "$P2"; do
  i=$((i+1))
  ok=1; for c in $C; do case $c in SQ_*) grep -qx $c $O/sq_names.txt || { echo "missing $c" >> $O/missing.txt; ok=0; };; esac; done
  [ $ok = 1 ] || continue
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d $O/p$i -o run --output-format csv -- \
      $R/tools/step_bench k16f16 16 228 304 3 1 2.0 > $O/p$i.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/sbpmc2"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{O}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:100]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(k, {c: round(sum(x) / len(x)) for c, x in sorted(v.items())})
PY
