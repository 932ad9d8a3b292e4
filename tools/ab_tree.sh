# A/B of the tree kernels between the in-tree libhz.so and another build
# ($1, e.g. abl/libhz_prev.so), alternating processes: tree_bench under
# rocprofv3, per-kernel stats of k_expand_backup only (traces stay on the box)
set -e
O=gpurun_out/${2:-ab}; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do for v in new old; do
  if [ $v = old ]; then export HZ_LIB=$R/$1; else unset HZ_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/ab$v$i -o tb -- python $R/tools/tree_bench.py 200 2 >> $R/$O/tb.log 2>&1
  python $R/tools/db_stats.py /tmp/ab$v$i/tb_results.db k_expand_backup > $R/$O/${v}_$i.json
  rm -rf /tmp/ab$v$i
done; done
