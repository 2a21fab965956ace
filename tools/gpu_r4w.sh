# gpu_r4w.sh -- round-4: C2 (MT10/W2048) bf16 / split2h with split-K for the one-plane kernel
# (MTSAC_BF16_SPLIT) and the in-launch split-K finish (MTSAC_SPLITK_FIN)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4w
mkdir -p $O
for v in "default" "MTSAC_BF16_SPLIT=1" "MTSAC_SPLITK_FIN=1"; do
  n=${v%%=*}
  env $( [ "$v" = default ] || echo $v ) timeout -k 10 300 python bench.py --workload mt10_w2048 --precision bf16 --no-cpu-baseline > $O/c2_bf16_$n.json 2> $O/c2_bf16_$n.err || exit 1
done
for v in "default" "MTSAC_SPLITK_FIN=1"; do
  n=${v%%=*}
  env $( [ "$v" = default ] || echo $v ) timeout -k 10 300 python bench.py --workload mt10_w2048 --precision split2h --no-cpu-baseline > $O/c2_split2h_$n.json 2> $O/c2_split2h_$n.err || exit 1
done
echo done
