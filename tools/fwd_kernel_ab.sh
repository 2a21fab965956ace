# fwd_kernel_ab.sh TAG -- whole S3 split2h steps with the trunk forward / data grads on gemm_x3f
# (default) vs gemm_x3p at a fixed geometry (MTSAC_X3F_MIN_TILES above any grid turns gemm_x3f off,
# MTSAC_BFRAG=0 keeps the weight planes row-major, which gemm_x3p reads); one process per variant
# (both switches are read once per process), alternating, two rounds.  Output: gpurun_out/TAG/ab.txt
set -o pipefail
O=gpurun_out/${1:-fwdab}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 150 python tools/step_ab.py base:-1 >> $O/ab.txt 2>&1 || exit 1
  MTSAC_X3F_MIN_TILES=1000000 MTSAC_BFRAG=0 timeout -k 10 150 python tools/step_ab.py x3p_g2:2 x3p_g3:3 x3p_auto:-1 >> $O/ab.txt 2>&1 || exit 1
done
echo done
