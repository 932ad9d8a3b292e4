# A/B of an environment knob ($1=NAME, $2=value B; A = unset) for the tree
# kernels, alternating processes: tree_bench under rocprofv3, per-kernel
# stats of k_expand_backup (traces stay on the box) into gpurun_out/$3
set -e
O=gpurun_out/${3:-abenv}; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do for v in a b; do
  if [ $v = b ]; then export $1=$2; else unset $1; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/ab$v$i -o tb -- python $R/tools/tree_bench.py 200 2 >> $R/$O/tb.log 2>&1
  python $R/tools/db_stats.py /tmp/ab$v$i/tb_results.db k_expand_backup > $R/$O/${v}_$i.json
  rm -rf /tmp/ab$v$i
done; done
