# gpu_r4q.sh -- round-4: the fragment layout per layer (frag_probe per layer: hidden layers of MT10 /
# task shards too): bitwise tests, C2 split2h / bf16 and shard-model benches with and without it
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullbatch.py tests/test_gpu_x3f.py -q -rf -x -s -k fragment --timeout 200 --timeout-method thread > $O/tests_frag.log 2>&1 || exit 1
for pr in split2h bf16; do
  timeout -k 10 300 python bench.py --workload mt10_w2048 --precision $pr --no-cpu-baseline > $O/bench_c2_${pr}_frag.json 2> $O/bench_c2_${pr}_frag.err || exit 1
  MTSAC_BFRAG=0 timeout -k 10 300 python bench.py --workload mt10_w2048 --precision $pr --no-cpu-baseline > $O/bench_c2_${pr}_rowmajor.json 2> $O/bench_c2_${pr}_rowmajor.err || exit 1
done
timeout -k 10 400 python -u tools/shard_model.py 0 300 150 split2h > $O/shard_model_frag.txt 2>&1 || exit 1
echo done
