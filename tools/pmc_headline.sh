#!/bin/bash
# SQ / traffic PMC passes on the headline kernel (mfcc_pair_kernel via tools/fp_microbench.py,
# 1 h of C2 PCM, 5 launches), one rocprofv3 run per counter group (never combined with trace
# domains).  Usage (GPU box): bash tools/pmc_headline.sh <tag>   (SONAR_LIB selects the library)
# Summarise: python3 tools/pmc_summary.py gpurun_out/pmc_<tag> mfcc_pair_kernel
set -o pipefail
TAG=$1
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
OUT="$R/gpurun_out/pmc_$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  ITERS=5 SECONDS=3600 timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/tools/fp_microbench.py" mfcc > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$OUT" mfcc_pair_kernel > "$OUT/summary.json" && echo "pmc $TAG ok"
