# profile_round.sh TAG -- the evidence behind bench.py's roofline block, written to gpurun_out/TAG/:
#   bench.json / kernel_stats.csv : rocprofv3 --kernel-trace --stats of the DEFAULT bench command
#   fetch.csv / write.csv         : separate --pmc FETCH_SIZE / WRITE_SIZE passes (short eager runs)
#   pmc_traffic.json              : per-family HBM bytes per launch (tools/pmc_traffic.py)
#   clock.csv / clock.txt         : a --pmc GRBM_GUI_ACTIVE pass: the shader clock each family holds (tools/pmc_clock.py)
set -o pipefail
TAG=${1:-r1}
PREC=${2:-split2h}  # the default bench's precision (its PMC family keys)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/bench.py > $O/bench.json 2> $O/bench.err || exit 1
cp $O/trace/run_kernel_stats.csv $O/kernel_stats.csv
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --exec eager --settle-s 0 --precision $PREC > $O/pf.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --exec eager --settle-s 0 --precision $PREC > $O/pw.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d $O/pc -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --exec eager --settle-s 0 --precision $PREC > $O/pc.log 2>&1 || exit 1
cp $O/pc/run_counter_collection.csv $O/clock.csv
python $R/tools/pmc_clock.py $O/clock.csv $O/clock.txt > /dev/null
cp $O/pf/run_counter_collection.csv $O/fetch.csv
cp $O/pw/run_counter_collection.csv $O/write.csv
python $R/tools/pmc_traffic.py $PREC $O/fetch.csv $O/write.csv $O/pmc_traffic.json > /dev/null
rm -rf $O/pf $O/pw $O/pc
echo done
