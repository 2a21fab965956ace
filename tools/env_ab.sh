# env_ab.sh TAG "ENV=V ..." [bench args] -- parity (x3f + full-batch + update tests), then the bench with
# and without the environment assignment, alternating, three rounds
set -o pipefail
O=gpurun_out/${1:-envab}; mkdir -p $O; E="$2"; shift 2
timeout -k 10 800 python -u -m pytest tests/test_gpu_x3f.py tests/test_gpu_fullbatch.py tests/test_gpu_update.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/base_$i.json 2>/dev/null || exit 1
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/env_$i.json 2>/dev/null || exit 1
done
echo done
