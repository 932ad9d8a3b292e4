#!/bin/bash
# The two HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE: each its own
# rocprofv3 run) over the default bench without the selfplay sub-object, then
# profiles/<round>_traffic.json's figure.  Usage: bash tools/traffic_passes.sh <out-dir>
set -eo pipefail
OUT=$1
REPO=$(pwd)
export TMPDIR=/tmp
k=0
for C in FETCH_SIZE WRITE_SIZE; do
  mkdir -p "$REPO/$OUT/p$k"
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$REPO/$OUT/p$k" -o run -- \
    python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-off-compare --no-selfplay \
    > "$REPO/$OUT/p$k/bench.json"
  k=$((k+1))
done
python3 "$REPO/tools/pmc_summary.py" "$REPO/$OUT" > "$REPO/$OUT/summary.json"
python3 "$REPO/tools/make_traffic.py" "$REPO/$OUT/summary.json" "$REPO/$OUT/traffic.json"
