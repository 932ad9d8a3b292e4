# key check of the MCTS build, then the expand launch's phase stamps and the
# tree kernels' per-dispatch stats (tree_bench under rocprofv3, twice)
set -e
O=gpurun_out/${1:-v9}; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python tools/kc_search.py > $O/kc.json 2>&1
HZ_LIB=tools/libhz_diag.so timeout -k 10 200 python tools/expand_phases.py 200 6 > $O/phases.json 2> $O/phases.err
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/tb$i -o tb -- python $R/tools/tree_bench.py 200 2 >> $R/$O/tb.log 2>&1
  python $R/tools/db_stats.py /tmp/tb$i/tb_results.db k_expand_backup > $R/$O/expand_$i.json
  rm -rf /tmp/tb$i
done
