# ab.sh TAG TESTS [WORKLOAD...] -- the GPU tests TESTS (pytest paths, -m gpu) on the default library, then
# a same-box bench A/B per workload against mtrl_amd/libmtsac_ab.so (the same sources built with one
# switch flipped), alternating new / old three times: gpurun_out/TAG/{new,old}_<workload>_<i>.json
set -o pipefail
O=gpurun_out/$1; mkdir -p $O; T=$2; shift 2
if [ -n "$T" ]; then
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
fi
for w in "$@"; do
  for i in 1 2 3; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 --workload $w > $O/new_${w}_$i.json 2>/dev/null || exit 1
    MTSAC_LIB=mtrl_amd/libmtsac_ab.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 --workload $w > $O/old_${w}_$i.json 2>/dev/null || exit 1
  done
done
echo done
