# pipe_ab.sh TAG -- cross-step pipelining (MTSAC_PIPELINE=1: step k+1's gather and critic(s, a) forward on
# the prefetch stream beside step k's actor backward) against the one-GPU default (off), alternating
set -o pipefail
O=gpurun_out/${1:-pipeab}; mkdir -p $O
for r in 1 2; do
  for w in mt10_w400 mt50_w2048; do
    timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 40 > $O/${w}_off_$r.json 2>/dev/null || exit 1
    MTSAC_PIPELINE=1 timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 40 > $O/${w}_on_$r.json 2>/dev/null || exit 1
  done
done
echo done
