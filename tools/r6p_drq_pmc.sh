# r6p_drq_pmc.sh TAG: SQ counter passes over the row-tile weight grad (42 x 42, 8 -> 8) and forward (21 x 21)
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
for cfg in "2 256 42 8 8" "0 768 21 16 16" "2 256 21 16 16"; do
  n=$(echo $cfg | tr ' ' _)
  timeout -s KILL 90 rocprofv3 --pmc $C -d $O/pmc_$n -o run --output-format csv -- python tools/drq_conv_one.py $cfg 10 > $O/pmc_$n.log 2>&1 || exit 1
done
echo done
