# gpu_r4m.sh -- round-4: the sharded trunk optimizer (ZeRO-1 style): parity through the in-process
# collective hook, the sharded / modelled / pipelined tests, the shard model and exposure with it
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4m
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullbatch.py -q -rf -x -k "sharded_optimizer" --timeout 300 --timeout-method thread -s > $O/zero_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullbatch.py tests/test_gpu_multiprocess.py tests/test_gpu_shard.py -q -rf -x -k "modelled or pipelined or two_rank or shard" --timeout 250 --timeout-method thread > $O/tests.log 2>&1 || exit 1
MTSAC_ZERO=1 timeout -k 10 300 python -u tools/shard_model.py 0 300 150 split2h > $O/shard_model_zero.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for bw in 150 300; do
  MTSAC_ZERO=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/ce$bw -o run -- python $R/tools/coll_exposure.py run 7 $bw split2h > $R/$O/ce$bw.log 2>&1 || exit 1
  gzip -c $R/$O/ce$bw/run_kernel_trace.csv > $R/$O/trace_t7_${bw}_zero.csv.gz
  rm -rf $R/$O/ce$bw
done
echo done
