# The round-end checks on one box, then the driver's own bench command
# untraced and under rocprofv3 (kernel trace + stats, CSV), summarised by
# tools/driver_prof.py into $O (the trace itself stays on the box).
set -e
O=gpurun_out/${1:-final}; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 750 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/dp -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/$O/bench_under_prof.json 2> $R/$O/bench_under_prof.err
TR=$(find /tmp/dp -name 'run_kernel_trace.csv' | head -1)
ST=$(find /tmp/dp -name 'run_kernel_stats.csv' | head -1)
cp $ST $R/$O/run_kernel_stats.csv
python3 $R/tools/driver_prof.py $TR $ST $R/$O/bench_under_prof.json $R/$O/driver_prof.json $R/$O/bench.json > $R/$O/driver_prof.log 2>&1
