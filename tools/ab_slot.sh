# A/B of the gathering expand launch's row-slot forms (HZ_SLOT_WAVE=0: one
# atomic per workgroup after a barrier; 1: one per wave), alternating
# processes; per-kernel stats only (the traces stay on the box)
set -e
mkdir -p gpurun_out/v8
R=$GRAFT_REPO_ROOT
HZ_SLOT_WAVE=1 timeout -k 10 400 python -u -m pytest tests/test_mcts_gpu.py tests/test_selfplay_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/v8/tests_wave.log 2>&1
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do for v in 0 1; do
  HZ_SLOT_WAVE=$v timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/ab$v$i -o tb -- python $R/tools/tree_bench.py 200 2 >> $R/gpurun_out/v8/tb.log 2>&1
  python $R/tools/db_stats.py /tmp/ab$v$i/tb_results.db k_expand_backup > $R/gpurun_out/v8/slot${v}_$i.json
  rm -rf /tmp/ab$v$i
done; done
