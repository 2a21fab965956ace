#!/bin/bash
# kregs.sh OBJ [pattern] -- per-kernel VGPR/AGPR/spill counts of a hipcc object (gfx950 bundle)
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fb "$1" && \
$B/clang-offload-bundler --unbundle --input=$T/fb --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/co && \
$B/llvm-readelf --notes $T/co > $T/notes
python3 - "$T/notes" "${2:-.}" <<'PY'
import re, sys, subprocess
t = open(sys.argv[1]).read()
# one map per kernel, keys in alphabetical order: split where a map starts (.agpr_count comes first)
for e in t.split('- .agpr_count:')[1:]:
    e = '.agpr_count:' + e
    name = (re.search(r'\.name:\s+(\S+)', e) or [None, ''])[1]
    dm = subprocess.run(['c++filt', name], capture_output=True, text=True).stdout.strip()
    if not re.search(sys.argv[2], dm): continue
    g = lambda k: (re.search(r'\.' + k + r':\s+(\d+)', e) or [None, None])[1]
    print(f"vgpr {g('vgpr_count'):>4} agpr {g('agpr_count'):>4} vspill {g('vgpr_spill_count')} lds {g('group_segment_fixed_size')}  {dm[:170]}")
PY
rm -rf $T
