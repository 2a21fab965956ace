# c1_prof.sh TAG -- kernel timeline of MT10/W400 (configs[1]) split2h steps: rocprofv3 kernel trace of
# tools/c1_timeline.py, summarised by tools/step_timeline.py into gpurun_out/TAG/timeline.txt
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-c1}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python $R/tools/c1_timeline.py 10 400 ${2:-3} > $O/c1.txt 2>&1 || exit 1
python $R/tools/step_timeline.py $O/tr/run_kernel_trace.csv full > $O/timeline.txt || exit 1
rm -rf $O/tr
