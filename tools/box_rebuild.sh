# box_rebuild.sh TAG -- build provenance: rebuild libmtsac.so from the sources ON the GPU box (into a
# separate directory; the in-tree library is left as it is), compare it with the shipped one, and run
# smoke + the kernel tests + the default bench against the box-built library.  gpurun_out/TAG/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-rebuild}; mkdir -p $O
B=/tmp/mtsac_box_build; rm -rf $B && mkdir -p $B
( cd $R/mtrl_amd/csrc && timeout -k 10 900 make -j16 OBJDIR=$B/obj OUT=$B/libmtsac.so > $O/build.log 2>&1 ) || exit 1
md5sum $R/mtrl_amd/libmtsac.so $B/libmtsac.so > $O/md5.txt
cd $R
MTSAC_LIB=$B/libmtsac.so python -c "from mtrl_amd import _lib as L; print('box-built stamp', L.load().mtsac_build_stamp().decode(), 'tree', L.source_stamp())" > $O/stamp.txt 2>&1 || exit 1
MTSAC_LIB=$B/libmtsac.so timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
MTSAC_LIB=$B/libmtsac.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_x3f.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
MTSAC_LIB=$B/libmtsac.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/bench.json 2> $O/bench.err || exit 1
echo done
