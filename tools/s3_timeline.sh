# s3_timeline.sh TAG -- kernel timeline of the default bench (S3 split2h, the bench's own exec mode):
# rocprofv3 kernel trace summarised by tools/step_timeline.py (wall vs busy union per step)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-s3tl}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python $R/bench.py --no-cpu-baseline --steps 20 ${2:-} > $O/bench.json 2> $O/bench.err || exit 1
python $R/tools/step_timeline.py $O/tr/run_kernel_trace.csv full > $O/timeline.txt || exit 1
rm -rf $O/tr
