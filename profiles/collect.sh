#!/bin/bash
# Everything profiles/<round>/ holds for the default bench, in one GPU call
# (run from the repo root on the GPU box):
#   1. kernel-trace + stats of bench.py (no counters)
#   2. PMC passes, each its own run with --pmc only (gfx950 slots: 8 SQ per
#      pass; FETCH_SIZE and WRITE_SIZE each alone)
#   3. per-kernel counter means (tools/pmc_summary.py) and the HBM traffic
#      of k_rollout per launch (tools/make_traffic.py)
# Usage: bash profiles/collect.sh <round>   (writes gpurun_out/<round>/...)
set -eo pipefail
R=${1:-r01}
REPO=$(pwd)
OUT=$REPO/gpurun_out/$R
mkdir -p "$OUT/stats"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
  python3 "$REPO/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-off-compare --sp-cpu-seconds 0 \
  > "$OUT/stats/bench_under_prof.json"
k=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  mkdir -p "$OUT/pmc/p$k"
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc/p$k" -o run -- \
    python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-off-compare --no-selfplay \
    > "$OUT/pmc/p$k/bench.json"
  k=$((k+1))
done
python3 "$REPO/tools/pmc_summary.py" "$OUT/pmc" > "$OUT/pmc/summary.json"
python3 "$REPO/tools/make_traffic.py" "$OUT/pmc/summary.json" "$OUT/traffic.json"
# the per-dispatch CSVs are large (gpurun copies back at most 64 MiB): keep
# the stats and the summaries only
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" -o -name "*.db" \) -delete
