"""The gfx950 machine code inside libaarmvs.so, for static checks (tests/test_isa_guard.py,
tools/waitcnt_check.py).

The shared object's .hip_fatbin section is the concatenation of one clang offload bundle per
translation unit (each starts with the "__CLANG_OFFLOAD_BUNDLE__" magic; header: entry count,
then per entry its offset, size and target triple).  The gfx950 entries are AMDGPU ELF code
objects; llvm-objdump disassembles them."""
from __future__ import annotations

import os
import struct
import subprocess
import tempfile

LLVM_BIN = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def fatbin(lib_path: str) -> bytes:
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "fat.bin")
        subprocess.run([os.path.join(LLVM_BIN, "llvm-objcopy"), f"--dump-section=.hip_fatbin={out}",
                        lib_path, os.path.join(td, "stripped.so")], check=True, capture_output=True)
        with open(out, "rb") as f:
            return f.read()


def code_objects(lib_path: str, target: str = "gfx950") -> list[bytes]:
    """Every code object for `target` in the library (one per translation unit)."""
    blob = fatbin(lib_path)
    objs = []
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        q = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, q)
            triple = blob[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if triple.endswith(target):
                objs.append(blob[pos + off:pos + off + size])
        pos = blob.find(MAGIC, pos + 24)
    return objs


def disassemble(lib_path: str, target: str = "gfx950") -> str:
    """llvm-objdump -d of every gfx950 code object, concatenated."""
    texts = []
    with tempfile.TemporaryDirectory() as td:
        for i, co in enumerate(code_objects(lib_path, target)):
            p = os.path.join(td, f"co{i}.o")
            with open(p, "wb") as f:
                f.write(co)
            r = subprocess.run([os.path.join(LLVM_BIN, "llvm-objdump"), "-d", f"--mcpu={target}", p],
                               check=True, capture_output=True, text=True)
            texts.append(r.stdout)
    return "\n".join(texts)
