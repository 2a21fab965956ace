# defer_ab.sh TAG -- the weight-grad finishes deferred to one launch per network (default on one GPU) vs
# MTSAC_DEFER_FINISH=0: parity (update, full-batch, x3p tests), then C1 / S3 / C2-bf16 bench A/B, alternating
set -o pipefail
O=gpurun_out/${1:-defer}; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_gpu_update.py tests/test_gpu_fullbatch.py tests/test_gpu_x3p.py tests/test_gpu_trainer.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  for w in "mt10_w400 --steps 200" "mt50_w2048 --steps 40" "mt10_w2048 --precision bf16 --steps 100"; do
    n=$(echo $w | cut -d' ' -f1)$(echo $w | grep -o bf16)
    timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $O/${n}_on_$i.json 2>/dev/null || exit 1
    MTSAC_DEFER_FINISH=0 timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $O/${n}_off_$i.json 2>/dev/null || exit 1
  done
done
echo done
