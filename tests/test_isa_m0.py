"""The LDS-DMA inline asm (mtrl_amd/csrc/gemm_x3p_impl.h glds16) writes M0 without declaring it.

M0 is a reserved register (clang refuses it in a clobber list), so the asm is correct only while the
compiler keeps no value of its own in M0 in the kernels that issue it.  This test reads the gfx950
machine code of the built library and checks exactly that: in every function
that contains an LDS-DMA load, each instruction that names or implicitly uses M0 is either the asm's
``s_mov_b32 m0, sN`` or the LDS-DMA load two instructions after it -- no M0-indexed instruction
(s_movrel / v_movrel / gpr-index mode / GWS) and no other M0 write.  (Functions without LDS-DMA may
use M0 as the compiler likes: drq.hip's jl_project_kernel indexes registers through it.)
CPU only: llvm-objdump disassembles the code objects bundled in libmtsac.so.
"""

from __future__ import annotations

import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mtrl_amd", "libmtsac.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

# instructions that read or write M0 without naming it in the disassembly
IMPLICIT = re.compile(r"^(s_movrel|v_movrel|s_set_gpr_idx|ds_gws|global_load_lds|buffer_load_\w*lds|ds_\w*_addtid)")


def _tools_present() -> bool:
    return all(os.path.exists(os.path.join(LLVM, t)) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump"))


def _disassembly(tmp: str) -> list[list[str]]:
    fb = os.path.join(tmp, "fatbin")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fb, LIB, os.path.join(tmp, "x")],
                   check=True, capture_output=True)
    data = open(fb, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    assert starts, "no offload bundle in libmtsac.so"
    out = []
    for i, s in enumerate(starts):
        chunk = data[s:starts[i + 1] if i + 1 < len(starts) else len(data)]
        bf, co = os.path.join(tmp, f"b{i}"), os.path.join(tmp, f"c{i}.co")
        open(bf, "wb").write(chunk)
        r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + bf,
                            "--targets=" + TARGET, "--output=" + co], capture_output=True)
        if r.returncode != 0 or not os.path.getsize(co):
            continue
        d = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co],
                           check=True, capture_output=True, text=True).stdout
        fn: list[str] = []
        for line in d.splitlines():
            line = line.split("//")[0].strip()
            if re.match(r"^[0-9a-f]+ <.*>:$", line):  # a new function
                if fn:
                    out.append(fn)
                fn = []
                continue
            if not line or line.endswith(":") or line.startswith("Disassembly") or "file format" in line:
                continue
            fn.append(line)
        if fn:
            out.append(fn)
    return out


@pytest.mark.skipif(not os.path.exists(LIB) or not _tools_present(), reason="needs the built library and ROCm llvm tools")
def test_m0_is_only_the_lds_dma_address():
    with tempfile.TemporaryDirectory() as tmp:
        objs = _disassembly(tmp)
    assert objs, "no gfx950 code object found"
    writes = dmas = 0
    for ins in objs:
        if not any(s.startswith("global_load_lds") or re.match(r"buffer_load_\w*lds", s) for s in ins):
            continue
        for i, s in enumerate(ins):
            op = s.split()[0]
            names_m0 = re.search(r"\bm0\b", s) is not None
            if op == "s_mov_b32" and re.match(r"s_mov_b32 m0, s\d+$", s):
                # the asm: s_mov_b32 m0, sN ; s_nop 0 ; global_load_lds_dwordx4 vX, off
                assert i + 2 < len(ins) and ins[i + 1] == "s_nop 0" and ins[i + 2].startswith("global_load_lds_dwordx4"), \
                    f"M0 write not followed by the LDS-DMA: {ins[i:i + 3]}"
                writes += 1
                continue
            if op.startswith("global_load_lds"):
                assert i >= 2 and re.match(r"s_mov_b32 m0, s\d+$", ins[i - 2]) and ins[i - 1] == "s_nop 0", \
                    f"LDS-DMA without the asm's M0 write right before it: {ins[max(0, i - 2):i + 1]}"
                dmas += 1
                continue
            assert not names_m0, f"an instruction other than the LDS-DMA asm uses M0: {s}"
            assert not IMPLICIT.match(op), f"an M0-implicit instruction outside the LDS-DMA asm: {s}"
    assert writes > 0 and writes == dmas
