# gpu_r4x.sh -- round-4: head backward one-pass form only at >= 256 workgroups: GPU suite, S3 bench,
# serialised 7-task and S3 sums, the shard model
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4x
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
for cfg in "7 50 2048 3 t7_split2h" "50 50 2048 3 s3_split2h"; do
  set -- $cfg
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/kt_$5 -o run -- python $R/tools/shard_prof.py $1 $2 $3 $4 > $R/$O/kt_$5.log 2>&1 || exit 1
  python $R/tools/kernel_sums.py $R/$O/kt_$5/run_kernel_trace.csv 45 > $R/$O/sums_$5.txt || exit 1
  rm -rf $R/$O/kt_$5
done
cd $R
timeout -k 10 400 python -u tools/shard_model.py 0 300 150 split2h > $O/shard_model.txt 2>&1 || exit 1
echo done
