#!/bin/bash
# Kernel-trace + stats profile of the default bench (run from the repo root on
# the GPU box).  Usage: bash profiles/profile.sh <out-dir-under-gpurun_out>
set -eo pipefail
OUT=${1:-gpurun_out/prof}
REPO=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/$OUT" -o run -- \
  python3 "$REPO/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-off-compare > "$REPO/$OUT/bench_under_prof.json"
