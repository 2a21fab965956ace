cd $GRAFT_REPO_ROOT
for cfg in "A:" "B:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "C:DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "D:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || exit 1
  echo "$name $envs $(python -c "import json;d=json.load(open('gpurun_out/ab_$name.json'));print(d['value'])")" >> gpurun_out/ab.log
done
