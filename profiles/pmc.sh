#!/bin/bash
# PMC passes (counters only with --kernel-trace/--stats; each pass its own run)
# over the default bench.  Usage: bash profiles/pmc.sh <out-dir-under-gpurun_out> "<counters>" ...
set -eo pipefail
OUT=$1; shift
REPO=$(pwd)
export TMPDIR=/tmp
k=0
for C in "$@"; do
  mkdir -p "$REPO/$OUT/p$k"
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$REPO/$OUT/p$k" -o run -- \
    python3 "$REPO/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$REPO/$OUT/p$k/bench.json"
  k=$((k+1))
done
