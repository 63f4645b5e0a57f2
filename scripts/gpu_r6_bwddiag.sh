#!/bin/bash
# Round 6: where the resident backward pass 1's time goes — ab_bwd.py variants with the
# experiments build's NLSPN_BWD_RES_DBG ablation bits (1 no LDS scatter, 2 no halo flush,
# 4 no waits, 8 no exchange read: results wrong on purpose), and a rocprofv3 kernel summary
# of the resident and step forms.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_bwddiag_${1:-a}; mkdir -p $O
cd $R
export NLSPN_LIB_PATH=$R/nlspn_eccv20_amd/lib/exp/libnlspn_hip_exp.so
timeout -k 10 300 python tools/ab_bwd.py --config ${CFG:-nyu} res= noscat=NLSPN_BWD_RES_DBG=1 noflush=NLSPN_BWD_RES_DBG=2 \
    nowait=NLSPN_BWD_RES_DBG=4 noexch=NLSPN_BWD_RES_DBG=8 skeleton=NLSPN_BWD_RES_DBG=15 steps=NLSPN_BWD_RESIDENT=0 \
    > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.json
timeout -k 10 300 python tools/ab_bwd.py --config ${CFG:-nyu} --T 4 res= skeleton=NLSPN_BWD_RES_DBG=15 steps=NLSPN_BWD_RESIDENT=0 \
    > $O/ab_t4.json 2> $O/ab_t4.err || { tail -5 $O/ab_t4.err; exit 1; }
cat $O/ab_t4.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bwd --output-format csv -- \
    python3 $R/tools/ab_bwd.py --config ${CFG:-nyu} --rounds 3 res= steps=NLSPN_BWD_RESIDENT=0 > $O/prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -c1-160 {} | head -14
