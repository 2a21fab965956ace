# c1_api_trace.sh TAG -- MT10/W400 eager steps under a kernel + HIP runtime API trace (no counters):
# host enqueue times beside the kernels, for the idle gaps of tools/c1_prof.sh's timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-c1api}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/tr -o run -- python $R/tools/c1_timeline.py 10 400 3 > $O/c1.txt 2>&1 || exit 1
ls $O/tr > $O/files.txt
