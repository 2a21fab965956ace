# kernel traces (serialised solo steps and the graph bench) of the W = 400 workloads
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for w in mt10_w400 mt50_w400; do
  O=$R/gpurun_out/w400/$w
  mkdir -p $O
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python $R/bench.py --workload $w --no-cpu-baseline --exec graph --steps 20 --settle-s 0 > $O/bench.json 2> $O/bench.err || exit 1
  python $R/tools/step_timeline.py $O/kt/run_kernel_trace.csv full > $O/timeline.txt
  python $R/tools/kernel_sums.py $O/kt/run_kernel_trace.csv 40 > $O/sums.txt
  rm -rf $O/kt
done
