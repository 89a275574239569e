"""Static checks of the shipped gfx950 machine code (CPU).

Packed-fp32 VOP3P instructions (`v_pk_fma_f32`, `v_pk_mul_f32`, `v_pk_add_f32`) made the
backward's results vary from run to run on this toolchain whenever other kernels ran beside it
(round 5: 45 of 96 multi-stream runs differed; 0 of 96 without them).  `csrc/Makefile` compiles
the device code with the feature off; these tests fail if any such instruction reaches
`libaarmvs.so` (a flag dropped from the Makefile, a new unit built another way, a toolchain
that ignores the feature switch), and pin what the round-6 analysis found about the cause: a
dataflow check of every kernel's VMEM loads finds no read of a load's destination before its
`s_waitcnt vmcnt`, in the packed build as in the shipped one (`tools/waitcnt_check.py`)."""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "aa-rmvsnet_amd", "aarmvs", "libaarmvs.so")
CSRC = os.path.join(ROOT, "aa-rmvsnet_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
PACKED = re.compile(r"\bv_pk_(fma|mul|add)_f32\b")

from aarmvs import isa  # noqa: E402

import waitcnt_check  # noqa: E402


def _units():
    mk = open(os.path.join(CSRC, "Makefile")).read()
    return re.search(r"^SRCS := (.*)$", mk, re.M).group(1).split()


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_shipped_code_objects_have_no_packed_fp32_instructions():
    cos = isa.code_objects(LIB)
    assert len(cos) == len(_units()), "one gfx950 code object per .hip unit"
    text = isa.disassemble(LIB)
    assert text.count("v_mfma") > 1000, "the disassembly covers the kernels"
    bad = sorted(set(m.group(0) for m in PACKED.finditer(text)))
    assert not bad, f"packed-fp32 instructions in libaarmvs.so: {bad} (DESIGN.md §6)"


def test_makefile_turns_packed_fp32_off_for_every_unit():
    mk = open(os.path.join(CSRC, "Makefile")).read()
    flags = re.search(r"^FLAGS := (.*?)(?<!\\)$", mk, re.M | re.S).group(1)
    assert "-target-feature -Xclang -packed-fp32-ops" in flags


_MISSING_WAIT = """\
_Zkernel:
	buffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen
	global_load_dword v8, v[2:3], off
	s_waitcnt vmcnt(1)
	v_add_f32_e32 v9, v4, v5
	v_pk_fma_f32 v[10:11], v[8:9], v[4:5], v[6:7]
	s_waitcnt vmcnt(0)
	v_add_f32_e32 v12, v8, v8
	s_endpgm
.Lfunc_end0:
"""


def test_waitcnt_checker_flags_a_read_before_its_wait(tmp_path):
    p = tmp_path / "k.s"
    p.write_text(_MISSING_WAIT)
    (lines,) = waitcnt_check.parse_kernels(str(p)).values()
    hz = waitcnt_check.check_kernel(lines)
    assert [op for op, _, regs in hz] == ["v_pk_fma_f32"] and hz[0][2] == [8]


@pytest.mark.skipif(not os.path.exists(HIPCC) or shutil.which("make") is None, reason="no hipcc")
@pytest.mark.parametrize("unit,packed", [("bptt", True), ("warp_cost", True), ("warp_cost", False)])
def test_no_load_result_is_read_before_its_wait(tmp_path, unit, packed):
    """The two units whose packed builds diverged: no kernel reads a VMEM load's destination
    before the `s_waitcnt vmcnt` that covers it, with or without packed-fp32 code."""
    flags = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "--cuda-device-only", "-S"]
    if unit == "warp_cost":
        flags.append("-ffp-contract=off")
    if not packed:
        flags += ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
    out = tmp_path / f"{unit}.s"
    subprocess.run([HIPCC, *flags, os.path.join(CSRC, f"{unit}.hip"), "-o", str(out)], check=True,
                   capture_output=True)
    text = out.read_text()
    assert (PACKED.search(text) is not None) == packed
    kernels = waitcnt_check.parse_kernels(str(out))
    assert len(kernels) > 10
    found = {n: waitcnt_check.check_kernel(ls) for n, ls in kernels.items()}
    assert not any(found.values()), {n: h[:3] for n, h in found.items() if h}
