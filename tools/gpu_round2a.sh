# GPU tests + default bench + per-shard step times (what each rank of an N-GPU run computes)
tools/gpu_steps.sh "600 gputests python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests" \
  "240 bench python bench.py --steps 20 --warmup 5 --no-cpu-baseline" \
  "200 shards python -u tools/shard_step.py 50 25 13 7 6"
