# gpu_r3w.sh -- MT10/W400 step anatomy: eager vs graph, untimed kernel trace (gaps between launches)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 200 python -u tools/c1_timeline.py > $O/c1_modes.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o run -- python $GRAFT_REPO_ROOT/tools/c1_timeline.py > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/step_timeline.py $O/kt/run_kernel_trace.csv full > $O/c1_timeline.txt || exit 1
rm -rf $O/kt
echo done
