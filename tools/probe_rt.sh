cd $GRAFT_REPO_ROOT
TL=$(python -c "import torch,os;print(os.path.dirname(torch.__file__))")/lib
mkdir -p /tmp/trt && ln -sf $TL/libamdhip64.so /tmp/trt/libamdhip64.so.7 && ln -sf $TL/libhsa-runtime64.so /tmp/trt/libhsa-runtime64.so.1 && ln -sf $TL/libamd_comgr.so /tmp/trt/libamd_comgr.so.3
LD_LIBRARY_PATH=/tmp/trt:$TL ldd ./tools/capture_probe | grep -E "amdhip|hsa" >> gpurun_out/probe4.log
for v in 0 1 2 4; do LD_LIBRARY_PATH=/tmp/trt:$TL timeout -k 5 30 ./tools/capture_probe $v >> gpurun_out/probe4.log 2>&1; echo "torchrt v$v rc $?" >> gpurun_out/probe4.log; done
