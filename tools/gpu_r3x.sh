# gpu_r3x.sh -- race hunt: W400 whole vs pipelined in fresh processes, per knob
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3x
mkdir -p $O
timeout -k 10 300 python tools/pipe_repro.py 8 >> $O/repro.txt 2>&1 || exit 1
timeout -k 10 300 python tools/pipe_repro.py 8 MTSAC_LANES_ALT=1 >> $O/repro.txt 2>&1 || exit 1
timeout -k 10 300 python tools/pipe_repro.py 8 MTSAC_EV_ROTATE=1 >> $O/repro.txt 2>&1 || exit 1
echo done
