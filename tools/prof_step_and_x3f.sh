set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof1/kt -o run -- python $R/tools/shard_prof.py 50 > $R/gpurun_out/prof1/kt.log 2>&1 || exit 1
python $R/tools/kernel_sums.py $R/gpurun_out/prof1/kt/run_kernel_trace.csv 45 > $R/gpurun_out/prof1/sums.txt
rm -f $R/gpurun_out/prof1/kt/run_kernel_trace.csv
cd $R && tools/gemm_pmc.sh pmc_x3f 1 257 2 6400 2048 2048 20
