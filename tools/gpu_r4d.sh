# gpu_r4d.sh -- round-4: split2h plane bound + long-run drift, DrQ MFMA convs (pipelined loads), shard
# model and per-bucket collective exposure under split2h
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3f.py tests/test_gpu_fullbatch.py -q -rf -k "split2h_products or long_run" --timeout 200 --timeout-method thread -s > $O/split2h.log 2>&1
echo "split2h exit $?" >> $O/split2h.log
grep -q "Fatal\|core dumped\|Segmentation" $O/split2h.log && exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_drq.py -q -rf --timeout 200 --timeout-method thread -s > $O/drq_tests.log 2>&1
echo "drq exit $?" >> $O/drq_tests.log
grep -q "Fatal\|core dumped\|Segmentation" $O/drq_tests.log && exit 1
timeout -k 10 300 python bench.py --workload atari_drq --no-cpu-baseline > $O/bench_drq_mfma.json 2> $O/bench_drq_mfma.err || exit 1
MTSAC_DRQ_MFMA=4 timeout -k 10 300 python bench.py --workload atari_drq --no-cpu-baseline > $O/bench_drq_wgrad_only.json 2> $O/bench_drq_wgrad_only.err || exit 1
bash tools/drq_kprof.sh r4d/drq_kprof_mfma > /dev/null 2>&1 || exit 1
timeout -k 10 300 python -u tools/shard_model.py 0 300 150 split2h > $O/shard_model_split2h.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for bw in 150 300; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/ce$bw -o run -- python $GRAFT_REPO_ROOT/tools/coll_exposure.py run 7 $bw split2h > $GRAFT_REPO_ROOT/$O/ce$bw.log 2>&1 || exit 1
  python $GRAFT_REPO_ROOT/tools/coll_exposure.py parse $GRAFT_REPO_ROOT/$O/ce$bw/run_kernel_trace.csv > $GRAFT_REPO_ROOT/$O/exposure_t7_${bw}.txt 2>&1
  rm -rf $GRAFT_REPO_ROOT/$O/ce$bw
done
echo done
