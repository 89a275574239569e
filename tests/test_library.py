"""CPU-side checks of the C-ABI library: it loads, and exports every function that
include/aarmvs.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "aarmvs.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(aarmvs_[a-z_]+)\s*\(", text)))


def test_header_declares_the_abi():
    names = declared_functions()
    for n in ("aarmvs_sweep", "aarmvs_homo_warp", "aarmvs_pack_params", "aarmvs_unet_step",
              "aarmvs_softmax_depth", "aarmvs_sweep_workspace_bytes", "aarmvs_last_error"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from aarmvs import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libaarmvs.so is not built (run __graft_entry__.build())")
    handle = ctypes.CDLL(_lib.LIB_PATH)
    for n in declared_functions():
        assert hasattr(handle, n), n
    assert set(_lib.SIGNATURES) == set(declared_functions())


def declared_arity():
    """{function: number of parameters} from the prototypes in include/aarmvs.h."""
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(aarmvs_[a-z_0-9]+)\s*\(([^;{]*?)\)\s*;", text):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_ctypes_signatures_match_the_header_arity():
    """Every ctypes binding passes as many arguments as the C prototype takes (a short
    argtypes list makes ctypes refuse the call only when it runs -- on the GPU box)."""
    from aarmvs import _lib
    arity = declared_arity()
    assert set(arity) == set(_lib.SIGNATURES)
    for name, (_, argtypes) in _lib.SIGNATURES.items():
        assert len(argtypes) == arity[name], (name, len(argtypes), arity[name])


def test_host_only_queries():
    from aarmvs import lib
    L = lib()
    assert L.aarmvs_param_count() == 109970          # omega 1,225 + regulariser 108,745
    assert L.aarmvs_packed_param_bytes() >= 109970 * 4
    assert L.aarmvs_sweep_workspace_bytes(1, 128, 160, 2) > 0
    assert L.aarmvs_sweep_workspace_bytes(1, 130, 160, 2) == 0   # H % 4 != 0 rejected
    assert b"multiple" in L.aarmvs_last_error()


def test_library_calls_run_under_their_tensors_device(monkeypatch):
    """aarmvs.ops enters the device of its first device tensor (or DepthSweep) around every
    library call, so the launch stream and the library's hipGetDevice() are that device's,
    whatever device the caller left current (train/eval ranks on cuda:r)."""
    import contextlib
    import torch
    from aarmvs import ops
    entered = []

    @contextlib.contextmanager
    def fake_device(dev):
        entered.append(dev)
        yield

    monkeypatch.setattr(torch.cuda, "device", fake_device)
    sw = ops.DepthSweep.__new__(ops.DepthSweep)
    sw.device = torch.device("cuda", 3)

    @ops._on_tensor_device
    def f(obj, x=None):
        return "ran"

    assert f(sw) == "ran" and entered == [torch.device("cuda", 3)]
    assert f(torch.zeros(1)) == "ran" and len(entered) == 1          # CPU tensors: no guard
    assert f(None, x=torch.device("cuda", 1)) == "ran" and entered[-1] == torch.device("cuda", 1)


def test_deform_sample_rejects_bad_geometry_before_launching():
    """aarmvs_deform_sample validates on the host (no device work, so it runs here): null
    pointers, C other than 32 and non-positive sizes are refused with a message."""
    from aarmvs import lib
    L = lib()
    fake = 0x1000   # never dereferenced: validation fails first
    assert L.aarmvs_deform_sample(None, fake, None, 1, 32, 8, 8, 8, 8, 1, 1, fake, None) != 0
    assert b"null" in L.aarmvs_last_error()
    assert L.aarmvs_deform_sample(fake, fake, None, 1, 16, 8, 8, 8, 8, 1, 1, fake, None) != 0
    assert b"32" in L.aarmvs_last_error()
    assert L.aarmvs_deform_sample(fake, fake, None, 1, 32, 8, 8, 0, 8, 1, 1, fake, None) != 0
    assert b"geometry" in L.aarmvs_last_error()
    assert L.aarmvs_deform_sample_backward(fake, fake, fake, 1, 32, 8, 8, 8, 8, 1, 1, fake, fake, fake,
                                           None, None) != 0   # mask given, its gradient missing
    assert b"null" in L.aarmvs_last_error()
