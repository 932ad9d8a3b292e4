#!/bin/bash
# PMC passes over tools/conv_bench.py (the tower conv kernels at batch 4096),
# or another program with its arguments, each pass its own rocprofv3 run
# (--pmc only).  Usage (GPU box, repo root):
#   bash tools/conv_pmc.sh <out-dir-under-gpurun_out> [<script.py> [args...]]
set -eo pipefail
OUT=$1
PROG=${2:-tools/conv_bench.py}
shift; shift || true
REPO=$(pwd)
export TMPDIR=/tmp
k=0
for C in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_LDS" \
         "GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM_RD"; do
  mkdir -p "$REPO/$OUT/p$k"
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$REPO/$OUT/p$k" -o run -- \
    python3 "$REPO/$PROG" "$@" > "$REPO/$OUT/p$k/bench.json"
  k=$((k+1))
done
python3 "$REPO/tools/pmc_summary.py" "$REPO/$OUT" > "$REPO/$OUT/summary.json"
