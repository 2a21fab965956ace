# lib_ab.sh TAG [bench args] -- parity of the default library (x3f + full-batch tests), then whole-bench
# A/B against mtrl_amd/libmtsac_ab.so (the same sources built with one switch flipped), alternating
set -o pipefail
O=gpurun_out/${1:-libab}; mkdir -p $O; shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3f.py tests/test_gpu_fullbatch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 "$@" > $O/new_$i.json 2>/dev/null || exit 1
  MTSAC_LIB=mtrl_amd/libmtsac_ab.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 "$@" > $O/old_$i.json 2>/dev/null || exit 1
done
echo done
