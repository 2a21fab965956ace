# gpu_r3g.sh -- gemm_x3f 4-wave (64-column slab) variant: correctness under the knob, ablations
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3g
mkdir -p $O
MTSAC_X3F_WV=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_x3f.py -x -q -rf --timeout 200 --timeout-method thread > $O/tests_wv4.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests_wv4.log
[ $rc -ne 0 ] && exit $rc
X3F_ABL="0 131 1000 1131 1002 1064" timeout -k 10 200 python -u tools/x3f_ablate.py 20 > $O/ablate_split3.txt 2>&1 || exit 1
X3F_BF16=1 X3F_ABL="0 131 1000 1131 2000 2131" timeout -k 10 200 python -u tools/x3f_ablate.py 40 > $O/ablate_bf16.txt 2>&1 || exit 1
echo done
