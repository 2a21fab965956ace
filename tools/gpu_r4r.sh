# gpu_r4r.sh -- round-4: serialised per-kernel step sums on the fragment-layout tree: S3 split2h,
# C2 bf16 and split2h, the 7-task shard split2h
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4r
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for cfg in "50 50 2048 3 s3_split2h" "10 10 2048 2 c2_bf16" "10 10 2048 3 c2_split2h" "7 50 2048 3 t7_split2h"; do
  set -- $cfg
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/kt_$5 -o run -- python $R/tools/shard_prof.py $1 $2 $3 $4 > $R/$O/kt_$5.log 2>&1 || exit 1
  python $R/tools/kernel_sums.py $R/$O/kt_$5/run_kernel_trace.csv 45 > $R/$O/sums_$5.txt || exit 1
  rm -rf $R/$O/kt_$5
done
echo done
