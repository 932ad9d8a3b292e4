#!/bin/bash
# Round-6 counter passes (bash tools/traffic_r06.sh <out-dir>):
#   p0  kernel trace + stats of the command below (durations)
#   p1  --pmc FETCH_SIZE, p2  --pmc WRITE_SIZE (one counter block per run)
# over a short default bench (config 2, the auto-reset leg, one full-batch
# self-play move), then tools/traffic_r06.py -> <out-dir>/traffic.json; and
#   k_play2_only  a kernel trace of the driver's command with every other leg
#   off, so that k_play2's plain rocprof mean is free of the other legs'
#   kernels (256 x mean vs ms_per_step).
set -eo pipefail
OUT=$1
REPO=$(pwd)
export TMPDIR=/tmp
CMD="$REPO/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-off-compare --no-api-path --no-api-caller \
 --sp-warmup 1 --sp-moves 1 --sp-games 0 --sp-steady-moves 0 --sp-cpu-seconds 0 --traffic-json /nonexistent"
mkdir -p "$REPO/$OUT/p0" "$REPO/$OUT/p1" "$REPO/$OUT/p2" "$REPO/$OUT/k_play2_only"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/$OUT/p0" -o run -- python3 $CMD \
  > "$REPO/$OUT/p0/bench.json" 2> "$REPO/$OUT/p0/bench.err"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$REPO/$OUT/p1" -o run -- python3 $CMD \
  > "$REPO/$OUT/p1/bench.json" 2> "$REPO/$OUT/p1/bench.err"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$REPO/$OUT/p2" -o run -- python3 $CMD \
  > "$REPO/$OUT/p2/bench.json" 2> "$REPO/$OUT/p2/bench.err"
python3 "$REPO/tools/traffic_r06.py" "$REPO/$OUT" "$REPO/$OUT/traffic.json" > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/$OUT/k_play2_only" -o run -- \
  python3 "$REPO/bench.py" --gpus 1 --steps 20 --warmup 5 --no-selfplay --no-api-path --no-api-caller \
  --no-auto-reset --no-off-compare > "$REPO/$OUT/k_play2_only/bench.json" 2> "$REPO/$OUT/k_play2_only/bench.err"
find "$REPO/$OUT" -name "*kernel_trace.csv" -delete
find "$REPO/$OUT" -name "*counter_collection.csv" -size +20M -delete
