# shard_deep_ab.sh TAG -- the split2h deep B ring on the task shards: parity (x3f, full-batch incl. the
# 8-way shards, the 2-process test), then the 7-task shard step (tools/shard_model.py, no collective and
# a modelled 300 GB/s all-reduce) against mtrl_amd/libmtsac_ab.so (-DX3F_DEEP_H2=0), alternating; and
# the S3 bench once each (the 208-row S3 tiles do not change)
set -o pipefail
O=gpurun_out/${1:-sharddeep}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_x3f.py tests/test_gpu_fullbatch.py tests/test_gpu_multiprocess.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  SHARD_N=8 timeout -k 10 200 python tools/shard_model.py 0 300 split2h > $O/new_$i.txt 2>&1 || exit 1
  MTSAC_LIB=mtrl_amd/libmtsac_ab.so SHARD_N=8 timeout -k 10 200 python tools/shard_model.py 0 300 split2h > $O/old_$i.txt 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/s3_new.json 2>/dev/null || exit 1
MTSAC_LIB=mtrl_amd/libmtsac_ab.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/s3_old.json 2>/dev/null || exit 1
echo done
