# gpu_r4t.sh -- round-4: head kernels' rows per wave (MTSAC_HEAD_RW 1 / 2 / 4) on serialised S3 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4t
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for rw in 1 2 4; do
  MTSAC_HEAD_RW=$rw timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/kt_$rw -o run -- python $R/tools/shard_prof.py 50 50 2048 3 > $R/$O/kt_$rw.log 2>&1 || exit 1
  python $R/tools/kernel_sums.py $R/$O/kt_$rw/run_kernel_trace.csv 45 > $R/$O/sums_s3_rw$rw.txt || exit 1
  rm -rf $R/$O/kt_$rw
done
echo done
