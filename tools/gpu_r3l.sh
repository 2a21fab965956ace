# gpu_r3l.sh -- serialised kernel lists: S3 split3, S3 bf16, C2 bf16 (MT10 W2048)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in "50 50 2048 1 s3" "50 50 2048 2 s3bf16" "10 10 2048 2 c2bf16" "10 10 2048 1 c2"; do
  set -- $cfg
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_$5 -o run -- python $GRAFT_REPO_ROOT/tools/shard_prof.py $1 $2 $3 $4 > $GRAFT_REPO_ROOT/$O/kt_$5.log 2>&1 || exit 1
  python $GRAFT_REPO_ROOT/tools/kernel_sums.py $GRAFT_REPO_ROOT/$O/kt_$5/run_kernel_trace.csv 60 > $GRAFT_REPO_ROOT/$O/sums_$5.txt || exit 1
  rm -rf $GRAFT_REPO_ROOT/$O/kt_$5
done
echo done
