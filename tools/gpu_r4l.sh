# gpu_r4l.sh -- round-4: the split actor forward beside the critic all-reduce (device-collective runs):
# the modelled / pipelined / sharded tests, the shard model with and without it, per-bucket exposure
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4l
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullbatch.py tests/test_gpu_multiprocess.py tests/test_gpu_shard.py -q -rf -x -k "modelled or pipelined or two_rank or shard" --timeout 250 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/shard_model.py 0 300 150 split2h > $O/shard_model_split.txt 2>&1 || exit 1
MTSAC_SPLIT_ACTOR=0 timeout -k 10 300 python -u tools/shard_model.py 0 300 150 split2h > $O/shard_model_merged.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for bw in 150 300; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/ce$bw -o run -- python $R/tools/coll_exposure.py run 7 $bw split2h > $R/$O/ce$bw.log 2>&1 || exit 1
  python $R/tools/coll_exposure.py parse $R/$O/ce$bw/run_kernel_trace.csv > $R/$O/exposure_t7_${bw}_split2h.txt 2>&1
  gzip -c $R/$O/ce$bw/run_kernel_trace.csv > $R/$O/trace_t7_${bw}_split2h.csv.gz
  rm -rf $R/$O/ce$bw
done
echo done
