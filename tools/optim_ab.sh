# optim_ab.sh TAG -- parity of the default library (update, full-batch, trainer tests), then C1 / S3 bench
# A/B against mtrl_amd/libmtsac_ab.so (built from the previous optim.hip, so its stamp differs), alternating
set -o pipefail
O=gpurun_out/${1:-optimab}; mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 800 python -u -m pytest tests/test_gpu_update.py tests/test_gpu_fullbatch.py tests/test_gpu_trainer.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for w in "mt10_w400 --steps 200" "mt50_w2048 --steps 40"; do
    n=$(echo $w | cut -d' ' -f1)
    timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $O/${n}_new_$i.json 2>/dev/null || exit 1
    MTSAC_ALLOW_STALE_LIB=1 MTSAC_LIB=mtrl_amd/libmtsac_ab.so timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $O/${n}_old_$i.json 2>/dev/null || exit 1
  done
done
echo done
