# gpu_r4p.sh -- round-4: the fragment layout beyond S3 (frag_probe: every net whose trunk GEMMs all run
# on gemm_x3f): bitwise tests on S3 / MT10 / shards, C2 and shard-model benches with and without it
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullbatch.py -q -rf -x -s -k fragment --timeout 200 --timeout-method thread > $O/tests_frag.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload mt10_w2048 --no-cpu-baseline > $O/bench_c2_frag.json 2> $O/bench_c2_frag.err || exit 1
MTSAC_BFRAG=0 timeout -k 10 300 python bench.py --workload mt10_w2048 --no-cpu-baseline > $O/bench_c2_rowmajor.json 2> $O/bench_c2_rowmajor.err || exit 1
timeout -k 10 400 python -u tools/shard_model.py 0 300 150 split2h > $O/shard_model_frag.txt 2>&1 || exit 1
MTSAC_BFRAG=0 timeout -k 10 400 python -u tools/shard_model.py 0 300 150 split2h > $O/shard_model_rowmajor.txt 2>&1 || exit 1
X3F_H2=1 X3F_FRAG=1 X3F_ABL="0 1000 1002 1131 131" timeout -k 10 200 python tools/x3f_ablate.py 20 > $O/x3f_h2_frag_wv4.txt 2>&1 || exit 1
echo done
