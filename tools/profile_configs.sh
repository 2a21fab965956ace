# profile_configs.sh TAG -- bench line + rocprofv3 kernel stats for the non-headline workloads
# (C1 mt10_w400, C2 mt10_w2048 in split3, S4 mt50_w400), written to gpurun_out/TAG/<workload>/.
set -o pipefail
TAG=${1:-r2}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for w in mt10_w400 mt10_w2048 mt50_w400; do
  O=$R/gpurun_out/$TAG/$w
  mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/bench.py --workload $w > $O/bench.json 2> $O/bench.err || exit 1
  cp $O/trace/run_kernel_stats.csv $O/kernel_stats.csv
  python $R/tools/step_timeline.py $O/trace/run_kernel_trace.csv > $O/timeline.txt || true
  rm -rf $O/trace
  echo "$w $(python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_step'], d['config']['exec'])")"
done
