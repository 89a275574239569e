"""Torch-facing wrappers of the HIP depth-sweep library.

Tensors stay on the device (PyTorch's caching allocator owns every buffer);
launches go to ``torch.cuda.current_stream()``.  All functions raise
``AarmvsError`` for CPU tensors or when libaarmvs.so is missing: the product
path has no CPU fallback.
"""
from __future__ import annotations

import ctypes
import functools

import torch

from . import _lib
from ._lib import AarmvsError, check, lib
from .synthetic import SWEEP_SHAPES

SWEEP_KEYS = tuple(SWEEP_SHAPES.keys())  # raw-blob order (include/aarmvs.h)


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _device_of(args, kwargs):
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, DepthSweep):
            return a.device
        if torch.is_tensor(a) and a.is_cuda:
            return a.device
        if isinstance(a, torch.device):
            return a
    return None


def _on_tensor_device(fn):
    """Runs ``fn`` with the current device set to its first device tensor's (or its
    DepthSweep's) device, so ``_stream()`` is that device's current stream and the library's
    hipGetDevice() agrees with the tensors, whatever device the caller left current."""
    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        dev = _device_of(args, kwargs)
        if dev is None or dev.type != "cuda" or dev.index is None:
            return fn(*args, **kwargs)
        with torch.cuda.device(dev):
            return fn(*args, **kwargs)
    return wrapper


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _require_device(*ts: torch.Tensor) -> None:
    for t in ts:
        if not t.is_cuda:
            raise AarmvsError("aarmvs: the HIP sweep needs ROCm device tensors (got a CPU tensor); "
                              "there is no CPU fallback")
        if t.dtype != torch.float32:
            raise AarmvsError(f"aarmvs: expected float32 tensors, got {t.dtype}")


def _check_proj(p: torch.Tensor, B: int, what: str) -> None:
    if tuple(p.shape) != (B, 4, 4):
        raise AarmvsError(f"aarmvs: {what} must be [B={B},4,4], got {tuple(p.shape)}")


def relative_projection(src_proj: torch.Tensor, ref_proj: torch.Tensor) -> torch.Tensor:
    """rows 0..2 of src_proj @ inverse(ref_proj) (module.py:16-18), [B,3,4] fp32.

    Computed on the host in fp32, exactly as the reference's CPU path does; the
    4x4 matrices are tiny and this keeps the sampling grid bit-compatible.
    """
    s = src_proj.detach().float().cpu()
    r = ref_proj.detach().float().cpu()
    return torch.matmul(s, torch.inverse(r))[:, :3, :4].contiguous()


@_on_tensor_device
def pack_params(params: dict, device) -> torch.Tensor:
    """Flatten the 48 sweep tensors (checkpoint keys) and pack them on the device."""
    missing = [k for k in SWEEP_KEYS if k not in params]
    if missing:
        raise KeyError(f"aarmvs.pack_params: missing parameters {missing[:3]}...")
    raw = torch.cat([params[k].detach().reshape(-1).float() for k in SWEEP_KEYS]).to(device)
    if raw.numel() != lib().aarmvs_param_count():
        raise AarmvsError("aarmvs.pack_params: parameter count mismatch with libaarmvs")
    nbytes = lib().aarmvs_packed_param_bytes()
    packed = torch.empty(nbytes // 4, dtype=torch.float32, device=device)
    check(lib().aarmvs_pack_params(raw.data_ptr(), packed.data_ptr(), _stream()), "pack_params")
    packed._aarmvs_raw = raw  # keep the source alive until the async pack has run
    return packed


@_on_tensor_device
def homo_warp(src_fea: torch.Tensor, rel: torch.Tensor, depth: torch.Tensor) -> torch.Tensor:
    """homo_warping_depthwise on the GPU for precomputed rel [B,3,4] and depth [B]."""
    _require_device(src_fea)
    src = src_fea.contiguous()
    B, C, H, W = src.shape
    rel_d = rel.reshape(B, 12).to(src.device, torch.float32).contiguous()
    dep = depth.reshape(B).to(src.device, torch.float32).contiguous()
    out = torch.empty_like(src)
    check(lib().aarmvs_homo_warp(src.data_ptr(), rel_d.data_ptr(), dep.data_ptr(), B, C, H, W,
                                 out.data_ptr(), _stream()), "homo_warp")
    return out


@_on_tensor_device
def homo_warp_backward(grad_out: torch.Tensor, rel: torch.Tensor, depth: torch.Tensor,
                       src_shape) -> torch.Tensor:
    """d loss / d src_fea of homo_warp: bilinear scatter-add of grad_out, summed in 64-bit fixed
    point (bit-reproducible, aarmvs_homo_warp_backward; fp32 atomics for a batch element whose
    grad_out is not finite).  Workspace: min(B, 64) * C * H * W * 8 bytes + 256."""
    _require_device(grad_out)
    g = grad_out.contiguous()
    B, C, H, W = src_shape
    rel_d = rel.reshape(B, 12).to(g.device, torch.float32).contiguous()
    dep = depth.reshape(B).to(g.device, torch.float32).contiguous()
    grad_src = torch.zeros(B, C, H, W, device=g.device)
    n = lib().aarmvs_homo_warp_backward_workspace_bytes(B, C, H, W)
    if n == 0:
        raise AarmvsError(f"aarmvs: homo_warp_backward geometry B={B} C={C} H={H} W={W}")
    ws = torch.empty(n, dtype=torch.uint8, device=g.device)
    check(lib().aarmvs_homo_warp_backward(g.data_ptr(), rel_d.data_ptr(), dep.data_ptr(), B, C, H,
                                          W, grad_src.data_ptr(), ws.data_ptr(), _stream()),
          "homo_warp_backward")
    return grad_src


class _GroupNormHip(torch.autograd.Function):
    """GroupNorm on NCHW fp32 device tensors through aarmvs_group_norm_forward/_backward
    (fixed-order fp64 statistics).  Once differentiable (no double backward)."""

    @staticmethod
    @_on_tensor_device
    def forward(ctx, x, weight, bias, groups: int, eps: float):
        _require_device(x)
        xc = x.contiguous()
        B, C = xc.shape[:2]
        HW = xc[0, 0].numel()
        y = torch.empty_like(xc)
        mr = torch.empty(B, groups, 2, device=xc.device)
        scratch = torch.empty(lib().aarmvs_group_norm_scratch_bytes(B, C, HW), dtype=torch.uint8,
                              device=xc.device)
        w = weight.contiguous() if weight is not None else None
        bb = bias.contiguous() if bias is not None else None
        check(lib().aarmvs_group_norm_forward(xc.data_ptr(), w.data_ptr() if w is not None else None,
                                              bb.data_ptr() if bb is not None else None, B, C, HW,
                                              groups, float(eps), y.data_ptr(), mr.data_ptr(),
                                              scratch.data_ptr(), _stream()), "group_norm_forward")
        ctx.save_for_backward(xc, w if w is not None else xc.new_empty(0), mr)
        ctx.groups, ctx.has_w, ctx.has_b = groups, w is not None, bb is not None
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    @_on_tensor_device
    def backward(ctx, gy):
        xc, w, mr = ctx.saved_tensors
        g = gy.contiguous()
        B, C = xc.shape[:2]
        HW = xc[0, 0].numel()
        dx = torch.empty_like(xc)
        s1 = torch.empty(B, C, device=xc.device)
        s2 = torch.empty(B, C, device=xc.device)
        scratch = torch.empty(lib().aarmvs_group_norm_scratch_bytes(B, C, HW), dtype=torch.uint8,
                              device=xc.device)
        check(lib().aarmvs_group_norm_backward(g.data_ptr(), xc.data_ptr(),
                                               w.data_ptr() if ctx.has_w else None, mr.data_ptr(),
                                               B, C, HW, ctx.groups, dx.data_ptr(), s1.data_ptr(),
                                               s2.data_ptr(), scratch.data_ptr(), _stream()),
              "group_norm_backward")
        dw = s1.sum(0) if ctx.has_w else None
        db = s2.sum(0) if ctx.has_b else None
        return dx, dw, db, None, None


class _LstmGatesHip(torch.autograd.Function):
    """ConvLSTMCell gates (module.py:83-90) on the HIP kernels: (z, c_prev) -> (h, c)."""

    @staticmethod
    @_on_tensor_device
    def forward(ctx, z, c_prev):
        _require_device(z, c_prev)
        zc, cp = z.contiguous(), c_prev.contiguous()
        B, C4 = zc.shape[:2]
        hid = C4 // 4
        HW = zc[0, 0].numel()
        if C4 != 4 * hid or tuple(cp.shape) != (B, hid) + tuple(zc.shape[2:]):
            raise AarmvsError(f"aarmvs.lstm_gates: z {tuple(zc.shape)} vs c {tuple(cp.shape)}")
        h = torch.empty_like(cp)
        c = torch.empty_like(cp)
        check(lib().aarmvs_lstm_gates_forward(zc.data_ptr(), cp.data_ptr(), B, hid, HW, h.data_ptr(),
                                              c.data_ptr(), _stream()), "lstm_gates_forward")
        ctx.save_for_backward(zc, cp)
        return h, c

    @staticmethod
    @torch.autograd.function.once_differentiable
    @_on_tensor_device
    def backward(ctx, dh, dc):
        zc, cp = ctx.saved_tensors
        B, C4 = zc.shape[:2]
        hid, HW = C4 // 4, zc[0, 0].numel()
        dh = dh.contiguous() if dh is not None else None
        dc = dc.contiguous() if dc is not None else None
        dz = torch.empty_like(zc)
        dcp = torch.empty_like(cp)
        check(lib().aarmvs_lstm_gates_backward(zc.data_ptr(), cp.data_ptr(),
                                               dh.data_ptr() if dh is not None else None,
                                               dc.data_ptr() if dc is not None else None, B, hid, HW,
                                               dz.data_ptr(), dcp.data_ptr(), _stream()),
              "lstm_gates_backward")
        return dz, dcp


def lstm_gates(z: torch.Tensor, c_prev: torch.Tensor):
    """(h, c) = ConvLSTMCell's gate math on the conv output z [B,4*hid,H,W] and c_prev
    [B,hid,H,W] (fp32 device tensors), forward and backward on the HIP kernels."""
    return _LstmGatesHip.apply(z, c_prev)


def group_norm(x: torch.Tensor, groups: int, weight=None, bias=None, eps: float = 1e-5):
    """F.group_norm(x, groups, weight, bias, eps) for fp32 device tensors on the HIP kernels
    (forward and backward)."""
    if x.dtype != torch.float32:
        raise AarmvsError(f"aarmvs.group_norm: expected float32, got {x.dtype}")
    return _GroupNormHip.apply(x, weight, bias, groups, eps)


@_on_tensor_device
def softmax_depth(cost: torch.Tensor) -> torch.Tensor:
    _require_device(cost)
    c = cost.contiguous()
    B, D = c.shape[:2]
    out = torch.empty_like(c)
    check(lib().aarmvs_softmax_depth(c.data_ptr(), out.data_ptr(), B, D, c[0, 0].numel(),
                                     _stream()), "softmax_depth")
    return out


def _ptr3(ts) -> ctypes.Array:
    return (ctypes.c_void_p * 3)(*[t.data_ptr() for t in ts])


class _EvidentialEpilogue(torch.autograd.Function):
    """The evidential head's epilogue on HIP (aarmvs_evidential_epilogue, evidential/models.py:
    385-459): the three classifier outputs [1,4,D,H,W] -> (evidential [4,H,W], prob_combine
    [1,D,H,W]); backward through aarmvs_evidential_epilogue_backward (no gradient to the depths)."""

    @staticmethod
    def forward(ctx, dv, h0, h1, h2):
        heads = [h.contiguous() for h in (h0, h1, h2)]
        _require_device(*heads)
        B, C, D, H, W = heads[0].shape
        if B != 1 or C != 4 or any(tuple(h.shape) != (1, 4, D, H, W) for h in heads):
            raise ValueError(f"evidential epilogue: heads must be [1, 4, D, H, W], got "
                             f"{[tuple(h.shape) for h in heads]}")
        dev = heads[0].device
        if any(h.device != dev for h in heads):
            raise AarmvsError("aarmvs: evidential epilogue heads must be on one device")
        if not dv.is_cuda or dv.device != dev:
            raise AarmvsError(f"aarmvs: evidential epilogue depth values must be on {dev} "
                              f"(got {dv.device}); the kernel reads them in place")
        dvc = dv.reshape(-1).float().contiguous()
        if dvc.numel() != D:
            raise ValueError(f"evidential epilogue: {dvc.numel()} depth values for D = {D}")
        ev = torch.empty(4, H, W, device=dev, dtype=torch.float32)
        pc = torch.empty(1, D, H, W, device=dev, dtype=torch.float32)
        check(lib().aarmvs_evidential_epilogue(_ptr3(heads), dvc.data_ptr(), D, H * W, ev.data_ptr(),
                                               pc.data_ptr(), _stream()), "evidential_epilogue")
        ctx.save_for_backward(dvc, *heads)
        return ev, pc

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g_ev, g_pc):
        dvc, *heads = ctx.saved_tensors
        D, H, W = heads[0].shape[2:]
        g_ev = g_ev.contiguous() if g_ev is not None else None
        g_pc = g_pc.contiguous() if g_pc is not None else None
        for gt in (g_ev, g_pc):
            if gt is not None:
                _require_device(gt)
                if gt.device != heads[0].device:
                    raise AarmvsError("aarmvs: evidential epilogue gradients on another device")
        gh = [torch.empty_like(h) for h in heads]
        check(lib().aarmvs_evidential_epilogue_backward(_ptr3(heads), dvc.data_ptr(), D, H * W,
                                                        _ptr(g_ev), _ptr(g_pc), _ptr3(gh), _stream()),
              "evidential_epilogue_backward")
        return (None, *gh)


class _DeformSample(torch.autograd.Function):
    """The sampling half of DeformConv2d (aarmvs_deform_sample, the reference's
    models/module.py:160-219): x NHWC [B,H,W,32], offset [B,18,h,w], mask [B,9,h,w] or None ->
    val [B,h*w,9*32], the A operand of the (tap, channel) contraction; differentiable in x,
    offset and mask."""

    @staticmethod
    def forward(ctx, x_nhwc, offset, mask, stride, pad):
        x_nhwc, offset = x_nhwc.contiguous(), offset.contiguous()
        mask = mask.contiguous() if mask is not None else None
        ts = [x_nhwc, offset] + ([mask] if mask is not None else [])
        _require_device(*ts)
        if any(t.device != x_nhwc.device for t in ts):
            raise AarmvsError("aarmvs: deform_sample tensors must be on one device")
        B, H, W, C = x_nhwc.shape
        h, w = offset.shape[2:]
        if tuple(offset.shape) != (B, 18, h, w) or (mask is not None and tuple(mask.shape) != (B, 9, h, w)):
            raise ValueError(f"deform_sample: offset / mask shapes {tuple(offset.shape)} / "
                             f"{None if mask is None else tuple(mask.shape)} for x {tuple(x_nhwc.shape)}")
        val = torch.empty(B, h * w, 9 * C, device=x_nhwc.device, dtype=torch.float32)
        check(lib().aarmvs_deform_sample(x_nhwc.data_ptr(), offset.data_ptr(), _ptr(mask), B, C, H, W,
                                         h, w, stride, pad, val.data_ptr(), _stream()), "deform_sample")
        ctx.save_for_backward(x_nhwc, offset, mask)
        ctx.geom = (stride, pad)
        return val

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g_val):
        x_nhwc, offset, mask = ctx.saved_tensors
        stride, pad = ctx.geom
        g_val = g_val.contiguous()
        _require_device(g_val)
        if g_val.device != x_nhwc.device:
            raise AarmvsError("aarmvs: deform_sample gradient on another device")
        B, H, W, C = x_nhwc.shape
        h, w = offset.shape[2:]
        gx = torch.zeros_like(x_nhwc)
        goff = torch.empty_like(offset)
        gm = torch.empty_like(mask) if mask is not None else None
        check(lib().aarmvs_deform_sample_backward(x_nhwc.data_ptr(), offset.data_ptr(), _ptr(mask), B, C,
                                                  H, W, h, w, stride, pad, g_val.data_ptr(),
                                                  gx.data_ptr(), goff.data_ptr(), _ptr(gm), _stream()),
              "deform_sample_backward")
        return gx, goff, gm, None, None


@_on_tensor_device
def deform_sample(x_nhwc: torch.Tensor, offset: torch.Tensor, mask: torch.Tensor | None, stride: int = 1,
                  pad: int = 1) -> torch.Tensor:
    """val [B, h*w, 9*C] of DeformConv2d's sampling (C == 32), differentiable (see _DeformSample)."""
    return _DeformSample.apply(x_nhwc, offset, mask, int(stride), int(pad))


@_on_tensor_device
def evidential_epilogue(h0: torch.Tensor, h1: torch.Tensor, h2: torch.Tensor, depth_values: torch.Tensor):
    """(evidential [4,H,W], prob_combine [1,D,H,W]) from classif0/1/2's outputs [1,4,D,H,W]
    (D = 32), differentiable w.r.t. the three head outputs."""
    return _EvidentialEpilogue.apply(depth_values, h0, h1, h2)


@_on_tensor_device
def wta_update(cost: torch.Tensor, depth_d: torch.Tensor, max_prob: torch.Tensor,
               depth_map: torch.Tensor, exp_sum: torch.Tensor) -> None:
    """In-place online WTA update of one plane (aarmvs_wta_update, drmvsnet.py:324-334):
    cost/max_prob/depth_map/exp_sum [B,H,W] fp32 device tensors, depth_d [B]."""
    ts = (cost, max_prob, depth_map, exp_sum)
    _require_device(*ts)
    B = cost.shape[0]
    for t in ts:
        if t.shape != cost.shape or not t.is_contiguous():
            raise AarmvsError("aarmvs: wta_update needs contiguous tensors of one [B,H,W] shape")
    dep = depth_d.reshape(-1).to(cost.device, torch.float32).contiguous()
    if dep.numel() != B:
        raise AarmvsError(f"aarmvs: depth_d must hold B={B} values")
    check(lib().aarmvs_wta_update(cost.data_ptr(), dep.data_ptr(), max_prob.data_ptr(),
                                  depth_map.data_ptr(), exp_sum.data_ptr(), B, cost[0].numel(),
                                  _stream()), "wta_update")


def aux_stream(device) -> torch.cuda.ExternalStream:
    """The library's aux stream of ``device`` (aarmvs_aux_stream): one per device, shared by every
    DepthSweep.  The process gets four hardware queues and streams beyond four share them (a
    stream's event wait then stalls its queue partner); with this stream, the default stream and
    the library's two unit / backward streams, a sweep or a training step uses exactly four."""
    device = torch.device(device)
    ptr = ctypes.c_void_p()
    with torch.cuda.device(device):
        check(lib().aarmvs_aux_stream(ctypes.byref(ptr)), "aux_stream")
    return torch.cuda.ExternalStream(ptr.value, device=device)


class DepthSweep:
    """Runs EMVSNet's depth loop (drmvsnet.py:273-291 / :306-342) on the HIP library.

    Holds the packed parameters and a workspace per (B, H, W, nsrc) geometry.
    """

    def __init__(self, params: dict, device, overlap: bool = True):
        """``overlap``: run the next plane group's cost stage on a second stream (the library's
        aux stream, aux_stream()) beside the current group's regulariser steps, and spread each
        plane's U-Net step over the library's streams so that the steps of neighbouring planes
        overlap (four streams in all; small frames move the cost stage to the current stream;
        same results, bit for bit)."""
        self.device = torch.device(device)
        self.packed = pack_params(params, self.device)
        self._ws = {}
        self._aux = None
        self.overlap = overlap

    @property
    def overlap(self) -> bool:
        return self._aux is not None

    @overlap.setter
    def overlap(self, on: bool):
        if on and self._aux is None:
            self._aux = aux_stream(self.device)
        elif not on:
            self._aux = None

    def workspace(self, B, H, W, nsrc) -> torch.Tensor:
        key = (B, H, W, nsrc)
        ws = self._ws.get(key)
        if ws is None:
            n = lib().aarmvs_sweep_workspace_bytes(B, H, W, nsrc)
            if n == 0:
                raise AarmvsError(f"aarmvs: invalid sweep geometry B={B} H={H} W={W} nsrc={nsrc} "
                                  "(H and W must be multiples of 4, 1 <= nsrc <= 16)")
            self._ws = {k: v for k, v in self._ws.items() if k[0] == "bwd" and k[1:] == key}
            # one live geometry at a time keeps HBM use bounded
            ws = torch.empty(n, dtype=torch.uint8, device=self.device)
            self._ws[key] = ws
        return ws

    def relative(self, ref_proj, src_projs, B: int) -> torch.Tensor:
        """[nsrc,B,12] device tensor of rows 0..2 of src_proj @ inv(ref_proj) per source view
        (module.py:16-18): one host round trip, reusable across d_range calls."""
        _check_proj(ref_proj, B, "ref_proj")
        for sp in src_projs:
            _check_proj(sp, B, "src_proj")
        rel = torch.stack([relative_projection(sp, ref_proj) for sp in src_projs])  # [nsrc,B,3,4]
        return rel.reshape(len(src_projs), B, 12).to(self.device).contiguous()

    RECORD_KEYS = ("x", "state", "z", "u", "stats", "t1", "ostats")

    @staticmethod
    def _record_sizes(B: int, H: int, W: int, D: int, nsrc: int) -> dict:
        L = lib()
        counts = (D, D + 1, D, D, D, D * nsrc, D * nsrc)
        out = {}
        for i, (name, count) in enumerate(zip(DepthSweep.RECORD_KEYS, counts)):
            n = L.aarmvs_train_record_bytes(B, H, W, i)
            if n == 0:
                raise AarmvsError(f"aarmvs: invalid record geometry B={B} H={H} W={W}")
            out[name] = n * count
        return out

    @staticmethod
    def record_buffers(B: int, H: int, W: int, D: int, device, *, nsrc: int) -> dict:
        """Device buffers of a training record (aarmvs_train_record) for D planes and nsrc
        source views: the cost slices, D + 1 regulariser state slabs, the gate pre-activations,
        the deconv outputs and their GroupNorm statistics, the omega conv output and its
        statistics (~1 KB per pixel and plane at B = 1, N = 3)."""
        return {k: torch.empty(n, dtype=torch.uint8, device=device)
                for k, n in DepthSweep._record_sizes(B, H, W, D, nsrc).items()}

    @staticmethod
    def _record_struct(rec: dict, B: int, H: int, W: int, D: int, nsrc: int, device=None):
        """ctypes view of a record, after checking every buffer holds this geometry's bytes,
        is contiguous and lives on the sweep's device (the library writes them without bounds)."""
        for k, n in DepthSweep._record_sizes(B, H, W, D, nsrc).items():
            t = rec.get(k)
            if t is None or not t.is_cuda or t.numel() * t.element_size() < n or not t.is_contiguous():
                raise AarmvsError(f"aarmvs: training record '{k}' missing, non-contiguous or smaller "
                                  f"than {n} B (record_buffers(B, H, W, D, nsrc={nsrc}))")
            if device is not None and t.device != torch.device(device):
                raise AarmvsError(f"aarmvs: training record '{k}' is on {t.device}, the sweep on {device}")
        r = _lib.TrainRecord()
        (r.x, r.state, r.z, r.u, r.stats, r.t1, r.ostats) = (rec[k].data_ptr() for k in DepthSweep.RECORD_KEYS)
        return r

    @_on_tensor_device
    def __call__(self, ref_fea, src_feas, ref_proj, src_projs, depth_values, *,
                 want_depth=True, want_cost=False, d_range=None, debug=False, cost_out=None,
                 rel=None, record=None):
        """Returns dict(depth, conf, cost, slice, omega) (entries None when not requested).

        ``d_range=(d0, d1)`` runs planes d0..d1-1 only (d0 == 0 resets the hidden state;
        later ranges continue from the state the previous call left in the workspace).
        ``cost_out`` is an optional caller-owned [B,D,H,W] buffer for the regulariser output.
        ``rel`` is an optional precomputed ``self.relative(ref_proj, src_projs, B)``.
        ``record`` (``record_buffers(B, H, W, D, nsrc=...)``) keeps every plane's tensors for
        ``backward`` (the training forward).
        """
        ref = ref_fea.contiguous()
        srcs = [s.contiguous() for s in src_feas]
        _require_device(ref, *srcs)
        if ref.dim() != 4:
            raise AarmvsError(f"aarmvs: ref_fea must be [B,C,H,W], got {tuple(ref.shape)}")
        B, C, H, W = ref.shape
        nsrc = len(srcs)
        if nsrc < 1 or nsrc > _lib.MAX_SRC:
            raise AarmvsError(f"aarmvs: need 1..{_lib.MAX_SRC} source views, got {nsrc}")
        if len(src_projs) != nsrc:
            raise AarmvsError(f"aarmvs: {nsrc} source features but {len(src_projs)} projections")
        for s in srcs:
            if s.shape != ref.shape:
                raise AarmvsError("aarmvs: source features must match the reference feature shape")
        # the kernels index depth_values[b * D + d] and rel[v][b]: reject mismatches here
        if depth_values.dim() != 2 or depth_values.shape[0] != B or depth_values.shape[1] < 1:
            raise AarmvsError(f"aarmvs: depth_values must be [B={B},D], got {tuple(depth_values.shape)}")
        dv = depth_values.to(ref.device, torch.float32).contiguous()
        D = dv.shape[1]
        if d_range is not None and not (0 <= d_range[0] < d_range[1] <= D):
            raise AarmvsError(f"aarmvs: bad d_range {d_range} for D={D}")
        if rel is None:
            rel = self.relative(ref_proj, src_projs, B)
        elif tuple(rel.shape) != (nsrc, B, 12) or not rel.is_cuda:
            raise AarmvsError(f"aarmvs: rel must be a device [nsrc={nsrc},B={B},12] tensor")
        ws = self.workspace(B, H, W, nsrc)
        out = {"depth": None, "conf": None, "cost": None, "slice": None, "omega": None}
        if want_depth:
            out["depth"] = torch.empty(B, H, W, device=ref.device)
            out["conf"] = torch.empty(B, H, W, device=ref.device)
        if cost_out is not None:
            if tuple(cost_out.shape) != (B, D, H, W) or not cost_out.is_contiguous():
                raise AarmvsError("aarmvs: cost_out must be a contiguous [B,D,H,W] tensor")
            _require_device(cost_out)
            out["cost"] = cost_out
        elif want_cost:
            out["cost"] = torch.empty(B, D, H, W, device=ref.device)
        if debug:
            out["slice"] = torch.empty(B, C, H, W, device=ref.device)
            out["omega"] = torch.empty(nsrc, B, H, W, device=ref.device)
        a = _lib.SweepArgs()
        a.B, a.C, a.H, a.W, a.nsrc, a.D = B, C, H, W, nsrc, D
        d0, d1 = (0, D) if d_range is None else d_range
        a.d_begin, a.d_end = d0, d1
        a.ref_fea = ref.data_ptr()
        for i, s in enumerate(srcs):
            a.src_fea[i] = s.data_ptr()
        a.rel_proj = rel.data_ptr()
        a.depth_values = dv.data_ptr()
        a.packed_params = self.packed.data_ptr()
        a.workspace = ws.data_ptr()
        a.depth_out = _ptr(out["depth"])
        a.conf_out = _ptr(out["conf"])
        a.cost_out = _ptr(out["cost"])
        a.slice_out = _ptr(out["slice"])
        a.omega_out = _ptr(out["omega"])
        a.aux_stream = self._aux.cuda_stream if self._aux is not None else None
        rec_struct = None
        if record is not None:
            rec_struct = self._record_struct(record, B, H, W, D, nsrc, ref.device)
            a.record = ctypes.pointer(rec_struct)
        check(lib().aarmvs_sweep(ctypes.byref(a), _stream()), "sweep")
        out["_keepalive"] = (rel, dv, srcs, ref, rec_struct)
        return out

    @_on_tensor_device
    def backward(self, ref_fea, src_feas, rel, depth_values, record, grad_cost, *,
                 regulariser_only=False, want_grad_x=False):
        """Backward of a recorded training sweep (aarmvs_sweep_backward): from dL/dcost
        [B,D,H,W] to (grad_ref [B,32,H,W], [grad_src [B,32,H,W]] per view, {sweep parameter
        name: gradient}, grad_x [D,B,H,W,32] NHWC or None).  ``regulariser_only`` stops after
        the regulariser (debug: grad_ref/grad_src are None, the omega.* gradients zero)."""
        ref = ref_fea.contiguous()
        srcs = [t.contiguous() for t in src_feas]
        _require_device(ref, *srcs, grad_cost)
        B, C, H, W = ref.shape
        nsrc = len(srcs)
        dv = depth_values.to(ref.device, torch.float32).contiguous()
        D = dv.shape[1]
        g = grad_cost.contiguous()
        if tuple(g.shape) != (B, D, H, W):
            raise AarmvsError(f"aarmvs: grad_cost must be [B={B},D={D},H={H},W={W}], got {tuple(g.shape)}")
        ws = self.workspace(B, H, W, nsrc)
        L = lib()
        key = ("bwd", B, H, W, nsrc)
        scratch = self._ws.get(key)
        if scratch is None:
            n = L.aarmvs_backward_scratch_bytes(B, H, W, nsrc)
            if n == 0:
                raise AarmvsError(f"aarmvs: invalid backward geometry B={B} H={H} W={W} nsrc={nsrc}")
            scratch = torch.empty(n, dtype=torch.uint8, device=ref.device)
            self._ws[key] = scratch
        grad_ref = None if regulariser_only else torch.empty_like(ref)
        grad_src = None if regulariser_only else [torch.empty_like(t) for t in srcs]
        grad_params = torch.empty(L.aarmvs_param_count(), device=ref.device)
        grad_x = torch.empty(D, B, H, W, C, device=ref.device) if want_grad_x else None
        a = _lib.BackwardArgs()
        a.B, a.C, a.H, a.W, a.nsrc, a.D = B, C, H, W, nsrc, D
        a.ref_fea = ref.data_ptr()
        for i, t in enumerate(srcs):
            a.src_fea[i] = t.data_ptr()
            if grad_src is not None:
                a.grad_src[i] = grad_src[i].data_ptr()
        a.rel_proj = rel.data_ptr()
        a.depth_values = dv.data_ptr()
        a.packed_params = self.packed.data_ptr()
        if (not torch.is_tensor(rel) or tuple(rel.shape) != (nsrc, B, 12) or rel.dtype != torch.float32
                or rel.device != ref.device or not rel.is_contiguous()):
            raise AarmvsError(f"aarmvs: rel must be a contiguous float32 [nsrc={nsrc}, B={B}, 12] tensor on "
                              f"{ref.device} (DepthSweep.relative), got "
                              f"{tuple(rel.shape) if torch.is_tensor(rel) else type(rel)}")
        rs = self._record_struct(record, B, H, W, D, nsrc, ref.device)
        a.record = ctypes.pointer(rs)
        a.grad_cost = g.data_ptr()
        a.grad_ref = _ptr(grad_ref)
        a.grad_params = grad_params.data_ptr()
        a.grad_x = _ptr(grad_x)
        a.workspace = ws.data_ptr()
        a.scratch = scratch.data_ptr()
        a.regulariser_only = 1 if regulariser_only else 0
        check(L.aarmvs_sweep_backward(ctypes.byref(a), _stream()), "sweep_backward")
        grads, off = {}, 0
        for k in SWEEP_KEYS:
            n = 1
            for d in SWEEP_SHAPES[k]:
                n *= d
            grads[k] = grad_params[off: off + n].view(SWEEP_SHAPES[k])
            off += n
        return grad_ref, grad_src, grads, grad_x

    def state(self, B, H, W, nsrc, planes, cell, which) -> torch.Tensor:
        """View of a hidden/cell state inside the workspace after the sweep has processed
        ``planes`` planes (or ``unet_step`` steps): the state those planes left."""
        ws = self.workspace(B, H, W, nsrc)
        ptr = lib().aarmvs_state_ptr(ws.data_ptr(), B, H, W, nsrc, planes, cell, which)
        if not ptr:
            raise AarmvsError("aarmvs: bad state query")
        hid = (16, 16, 16, 16, 8)[cell]
        sc = (1, 2, 4, 2, 1)[cell]
        off = ptr - ws.data_ptr()
        # stored NHWC (include/aarmvs.h); returned as the reference's NCHW view
        return ws[off: off + B * hid * (H // sc) * (W // sc) * 4].view(torch.float32).view(
            B, H // sc, W // sc, hid).permute(0, 3, 1, 2)

    @_on_tensor_device
    def cost_slice(self, ref_fea, src_feas, ref_proj, src_projs, depth, want_omega=False):
        """One plane's cost slice x [B,32,H,W] (aarmvs_cost_slice; drmvsnet.py:307-319) at
        depth [B]; returns (x, omega [nsrc,B,H,W] or None).  Uses this object's workspace."""
        ref = ref_fea.contiguous()
        srcs = [s.contiguous() for s in src_feas]
        _require_device(ref, *srcs)
        B, C, H, W = ref.shape
        nsrc = len(srcs)
        if nsrc < 1 or nsrc > _lib.MAX_SRC or len(src_projs) != nsrc:
            raise AarmvsError(f"aarmvs: need 1..{_lib.MAX_SRC} source views with projections")
        for s in srcs:
            if s.shape != ref.shape:
                raise AarmvsError("aarmvs: source features must match the reference feature shape")
        dep = depth.reshape(-1).to(ref.device, torch.float32).contiguous()
        if dep.numel() != B:
            raise AarmvsError(f"aarmvs: depth must hold B={B} values")
        rel = self.relative(ref_proj, src_projs, B)
        ws = self.workspace(B, H, W, nsrc)
        x = torch.empty(B, C, H, W, device=ref.device)
        om = torch.empty(nsrc, B, H, W, device=ref.device) if want_omega else None
        ptrs = (ctypes.c_void_p * nsrc)(*[s.data_ptr() for s in srcs])
        check(lib().aarmvs_cost_slice(ref.data_ptr(), ptrs, rel.data_ptr(), dep.data_ptr(),
                                      self.packed.data_ptr(), B, C, H, W, nsrc, ws.data_ptr(),
                                      x.data_ptr(), _ptr(om), _stream()), "cost_slice")
        return x, om

    @_on_tensor_device
    def unet_step(self, x: torch.Tensor, step: int, nsrc: int = 1) -> torch.Tensor:
        _require_device(x)
        x = x.contiguous()
        B, C, H, W = x.shape
        ws = self.workspace(B, H, W, nsrc)
        cost = torch.empty(B, 1, H, W, device=x.device)
        check(lib().aarmvs_unet_step(x.data_ptr(), B, H, W, nsrc, step, self.packed.data_ptr(),
                                     ws.data_ptr(), cost.data_ptr(), _stream()), "unet_step")
        return cost


# ----------------------------------------------------------------------------------
# opt-in per-kernel timing (aarmvs_profile_*): hipEvents on the launch stream
# ----------------------------------------------------------------------------------
def profile_enable(on: bool = True) -> None:
    lib().aarmvs_profile_enable(1 if on else 0)


def profile_reset() -> None:
    lib().aarmvs_profile_reset()


def profile_read() -> dict:
    """{kernel name: (launches, total device ms)} since the last reset."""
    L = lib()
    out = {}
    for i in range(L.aarmvs_profile_kernel_count()):
        n = ctypes.c_longlong(0)
        ms = ctypes.c_double(0.0)
        check(L.aarmvs_profile_read(i, ctypes.byref(n), ctypes.byref(ms)), "profile_read")
        if n.value:
            out[L.aarmvs_profile_kernel_name(i).decode()] = (int(n.value), float(ms.value))
    return out
