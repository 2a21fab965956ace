# exec-mode A/B at S3: graph vs eager, ROCm graph-executor env knobs, and a kernel trace of the eager
# step (does the DAG actually overlap?).  Writes gpurun_out/exec_ab/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/exec_ab
mkdir -p $O
cd $R
for cfg in "graph:" "eager:" "graph_nopkt:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "graph_nopkt_q4:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  mode=graph; [ "$name" = eager ] && mode=eager
  env $envs timeout -k 10 150 python bench.py --steps 30 --warmup 3 --settle-s 1 --no-cpu-baseline --exec $mode > $O/$name.json 2> $O/$name.err || exit 1
  echo "$name $envs $(python -c "import json;d=json.load(open('$O/$name.json'));print(d['value'], d['ms_per_step'])")" | tee -a $O/ab.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/te -o run -- python $R/bench.py --steps 10 --warmup 3 --settle-s 0 --no-cpu-baseline --exec eager > $O/te.log 2>&1 || exit 1
python $R/tools/step_timeline.py $O/te/run_kernel_trace.csv full > $O/eager_timeline.txt
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tg -o run -- python $R/bench.py --steps 10 --warmup 3 --settle-s 0 --no-cpu-baseline --exec graph > $O/tg.log 2>&1 || exit 1
python $R/tools/step_timeline.py $O/tg/run_kernel_trace.csv full > $O/graph_nopkt_timeline.txt
rm -f $O/te/run_kernel_trace.csv $O/tg/run_kernel_trace.csv
echo done
