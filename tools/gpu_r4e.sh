# gpu_r4e.sh -- round-4: split2h long-run drift (parameters), per-bucket collective exposure, C2 bf16
# per-kernel breakdown, DrQ bench on the restored VALU convs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullbatch.py -q -rf -k "long_run" --timeout 250 --timeout-method thread -s > $O/drift.log 2>&1
echo "drift exit $?" >> $O/drift.log
grep -q "Fatal\|core dumped\|Segmentation" $O/drift.log && exit 1
timeout -k 10 300 python bench.py --workload atari_drq --no-cpu-baseline > $O/bench_drq.json 2> $O/bench_drq.err || exit 1
timeout -k 10 300 python bench.py --workload mt10_w2048 --precision bf16 --no-cpu-baseline > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/c2 -o run -- python $R/tools/shard_prof.py 10 10 2048 2 > $R/$O/c2.log 2>&1 || exit 1
python $R/tools/kernel_sums.py $R/$O/c2/run_kernel_trace.csv 40 > $R/$O/c2_bf16_sums.txt || exit 1
rm -rf $R/$O/c2
for cfg in "150 split2h" "300 split2h" "150 split3"; do
  set -- $cfg
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/ce_$1_$2 -o run -- python $R/tools/coll_exposure.py run 7 $1 $2 > $R/$O/ce_$1_$2.log 2>&1 || exit 1
  python $R/tools/coll_exposure.py parse $R/$O/ce_$1_$2/run_kernel_trace.csv > $R/$O/exposure_t7_$1_$2.txt 2>&1
  python $R/tools/step_timeline.py $R/$O/ce_$1_$2/run_kernel_trace.csv full > $R/$O/timeline_t7_$1_$2.txt 2>&1
  gzip -c $R/$O/ce_$1_$2/run_kernel_trace.csv > $R/$O/trace_t7_$1_$2.csv.gz
  rm -rf $R/$O/ce_$1_$2
done
echo done
