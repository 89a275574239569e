"""Deterministic synthetic inputs and random-init weights (numpy only).

Used by the benchmark, the tests and the golden-fixture generator so that the
reference (run in the build container) and this build (run on the GPU box) see
bit-identical inputs.  Recipe follows SURVEY.md §8(d):

* features ~ N(0,1) ``[B,32,H,W]`` per view, images ~ N(0,1) ``[B,N,3,H,W]``;
* K = [[f,0,W/2],[0,f,H/2],[0,0,1]] with f = W; reference extrinsic = I;
  source view v translated along x by -20*v mm with a small alternating yaw;
  projection = [K @ E[:3,:4]; E[3]] as built by datasets/dtu_yao.py:144-146;
* depth hypotheses linspace(425, 935, D) mm (optionally descending, the
  ``flip_flag`` case of dtu_yao.py:172-173);
* weights: per-tensor ``default_rng([seed, crc32(name)])``, conv weights/biases
  U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (torch's default bound), norm affines near
  (1, 0) so that gamma/beta are exercised.
"""
from __future__ import annotations

import zlib

import numpy as np


def camera_projections(N: int, H: int, W: int, baseline: float = 20.0,
                       yaw: float = 0.02) -> np.ndarray:
    """[N,4,4] float32 projection matrices (view 0 = reference)."""
    f = float(W)
    K = np.array([[f, 0, W / 2.0], [0, f, H / 2.0], [0, 0, 1]], dtype=np.float64)
    out = []
    for v in range(N):
        th = yaw * v * (1 if v % 2 else -1)
        R = np.array([[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]])
        E = np.eye(4)
        E[:3, :3] = R
        E[:3, 3] = [-baseline * v, 0.3 * v, 0.0]
        P = E.copy()
        P[:3, :4] = K @ E[:3, :4]
        out.append(P)
    return np.stack(out).astype(np.float32)


def depth_hypotheses(D: int, lo: float = 425.0, hi: float = 935.0,
                     descending: bool = False, inverse: bool = False) -> np.ndarray:
    if inverse:  # data_eval_transform.py:119-124
        d = 1.0 / np.linspace(1.0 / lo, 1.0 / hi, D)
    else:
        d = np.linspace(lo, hi, D)
    d = d.astype(np.float32)
    return d[::-1].copy() if descending else d


def scene(B: int, N: int, H: int, W: int, D: int, seed: int = 0, C: int = 32,
          descending: bool = False, images: bool = False):
    """Synthetic multi-view sample.  Returns dict of numpy arrays.

    ``features``: [N,B,C,H,W] (view-major; view 0 is the reference) unless
    ``images`` is set, in which case ``imgs`` [B,N,3,H,W] is produced instead.
    """
    rng = np.random.default_rng(seed)
    out = {}
    if images:
        out["imgs"] = rng.standard_normal((B, N, 3, H, W), dtype=np.float32)
    else:
        out["features"] = rng.standard_normal((N, B, C, H, W), dtype=np.float32)
    proj = camera_projections(N, H, W)
    out["proj_matrices"] = np.broadcast_to(proj, (B, N, 4, 4)).copy()
    dv = depth_hypotheses(D, descending=descending)
    out["depth_values"] = np.broadcast_to(dv, (B, D)).copy()
    return out


def depth_targets(depth_values: np.ndarray, H: int, W: int, seed: int):
    """Training targets for a scene (dtu_yao.py's depth / mask, synthetic): depth_gt uniform
    over the hypothesis range, ~70% valid pixels.  Returns (depth_gt [B,H,W], mask [B,H,W])."""
    B = depth_values.shape[0]
    rng = np.random.default_rng(seed + 1000)
    lo, hi = float(depth_values.min()), float(depth_values.max())
    depth_gt = rng.uniform(lo, hi, (B, H, W)).astype(np.float32)
    mask = (rng.uniform(0, 1, (B, H, W)) > 0.3).astype(np.float32)
    return depth_gt, mask


def _fan_in(shape, name: str) -> int:
    if len(shape) <= 1:
        return 1
    if "deconv" in name and name.endswith("conv.weight"):   # ConvTranspose2d: [Cin,Cout,k,k]
        return int(shape[1] * np.prod(shape[2:]))
    return int(np.prod(shape[1:]))


def init_weights(shapes: dict, seed: int = 1) -> dict:
    """Random-init parameters for a state_dict layout ``{name: shape}``."""
    out = {}
    weight_shapes = {n: s for n, s in shapes.items()}
    for name in sorted(shapes):
        shape = tuple(shapes[name])
        rng = np.random.default_rng([seed, zlib.crc32(name.encode())])
        leaf = name.rsplit(".", 1)[-1]
        if leaf in ("running_mean",):
            arr = np.zeros(shape, np.float32)
        elif leaf in ("running_var",):
            arr = np.ones(shape, np.float32)
        elif leaf == "num_batches_tracked":
            arr = np.zeros(shape, np.int64)
        elif len(shape) >= 2:            # conv / deconv weight
            b = 1.0 / np.sqrt(_fan_in(shape, name))
            arr = rng.uniform(-b, b, shape).astype(np.float32)
        else:                            # bias or norm affine
            wname = name[: -len(leaf)] + "weight"
            wshape = weight_shapes.get(wname)
            is_norm = wshape is not None and len(wshape) == 1
            if is_norm and leaf == "weight":
                arr = (1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32)
            elif is_norm:
                arr = (0.1 * rng.standard_normal(shape)).astype(np.float32)
            else:
                fi = _fan_in(wshape, wname) if wshape is not None else 1
                b = 1.0 / np.sqrt(fi)
                arr = rng.uniform(-b, b, shape).astype(np.float32)
        out[name] = arr
    return out


def array_digest(*arrays) -> str:
    """Stable digest of arrays (detects RNG drift between hosts)."""
    h = zlib.crc32(b"")
    for a in arrays:
        h = zlib.crc32(np.ascontiguousarray(a).tobytes(), h)
    return f"{h:08x}"


# state_dict layout of the sweep's parameters (checkpoint keys):
# omega.* (drmvsnet.py:27-38) and cost_regularization.* (drmvsnet.py:66-117).
SWEEP_SHAPES = {
    "omega.reweight_network.0.0.weight": (4, 32, 3, 3),
    "omega.reweight_network.0.0.bias": (4,),
    "omega.reweight_network.0.1.weight": (4,),
    "omega.reweight_network.0.1.bias": (4,),
    "omega.reweight_network.1.stem.0.0.weight": (4, 4, 1, 1),
    "omega.reweight_network.1.stem.0.0.bias": (4,),
    "omega.reweight_network.1.stem.0.1.weight": (4,),
    "omega.reweight_network.1.stem.0.1.bias": (4,),
    "omega.reweight_network.1.stem.1.weight": (4, 4, 1, 1),
    "omega.reweight_network.1.stem.1.bias": (4,),
    "omega.reweight_network.1.stem.2.weight": (4,),
    "omega.reweight_network.1.stem.2.bias": (4,),
    "omega.reweight_network.2.weight": (1, 4, 1, 1),
    "omega.reweight_network.2.bias": (1,),
    "cost_regularization.cell_list.0.conv.weight": (64, 48, 3, 3),
    "cost_regularization.cell_list.0.conv.bias": (64,),
    "cost_regularization.cell_list.1.conv.weight": (64, 32, 3, 3),
    "cost_regularization.cell_list.1.conv.bias": (64,),
    "cost_regularization.cell_list.2.conv.weight": (64, 32, 3, 3),
    "cost_regularization.cell_list.2.conv.bias": (64,),
    "cost_regularization.cell_list.3.conv.weight": (64, 48, 3, 3),
    "cost_regularization.cell_list.3.conv.bias": (64,),
    "cost_regularization.cell_list.4.conv.weight": (32, 40, 3, 3),
    "cost_regularization.cell_list.4.conv.bias": (32,),
    "cost_regularization.deconv_0.conv.weight": (16, 16, 3, 3),
    "cost_regularization.deconv_0.conv.bias": (16,),
    "cost_regularization.deconv_0.gn.weight": (16,),
    "cost_regularization.deconv_0.gn.bias": (16,),
    "cost_regularization.deconv_1.conv.weight": (16, 16, 3, 3),
    "cost_regularization.deconv_1.conv.bias": (16,),
    "cost_regularization.deconv_1.gn.weight": (16,),
    "cost_regularization.deconv_1.gn.bias": (16,),
    "cost_regularization.conv_0.weight": (1, 8, 3, 3),
    "cost_regularization.conv_0.bias": (1,),
}


def sweep_weights(seed: int = 1) -> dict:
    """Random-init sweep parameters (same values init_weights gives the full model)."""
    return init_weights(SWEEP_SHAPES, seed=seed)


def fusion_views(H: int, W: int, nsrc: int, seed: int = 0):
    """Seeded depth maps + DTU-like cameras of one scene (a tilted plane with bumps, seen
    from nsrc + 1 cameras on an arc), for the fusion parity tests and bench
    (depth maps [H,W] float32 with 2% holes, (K, E) per view, a confidence map)."""
    rng = np.random.default_rng(seed)
    f = np.float32(1.2 * W)
    K = np.array([[f, 0, W / 2], [0, f, H / 2], [0, 0, 1]], np.float32)
    cams = []
    for v in range(nsrc + 1):
        th = 0.03 * (v - nsrc / 2)
        R = np.array([[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]])
        t = np.array([-30.0 * (v - nsrc / 2), 2.0 * v, 0.0])
        E = np.eye(4)
        E[:3, :3] = R
        E[:3, 3] = t
        cams.append((K.copy(), E.astype(np.float32)))
    # world surface: z = 600 + 0.05 x + bumps, sampled per camera by ray casting on a grid
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float64)
    depths = []
    for K_, E_ in cams:
        Ki = np.linalg.inv(K_.astype(np.float64))
        rays = Ki @ np.stack([xs.ravel(), ys.ravel(), np.ones(H * W)])
        # camera -> world: X_w = R^T (X_c - t); surface z_w = 600 + 0.05 x_w
        R = E_[:3, :3].astype(np.float64)
        t = E_[:3, 3].astype(np.float64)
        o = -R.T @ t
        dvec = R.T @ rays
        lam = (600.0 + 0.05 * o[0] - o[2]) / (dvec[2] - 0.05 * dvec[0])
        pw = o[:, None] + dvec * lam
        bump = 4.0 * np.sin(pw[0] / 37.0) * np.cos(pw[1] / 23.0)
        depth = (lam * (1.0 + bump / 600.0)).reshape(H, W)
        noise = rng.normal(0, 0.3, (H, W))
        hole = rng.random((H, W)) < 0.02
        d = (depth + noise).astype(np.float32)
        d[hole] = 0.0
        depths.append(d)
    conf = rng.random((H, W)).astype(np.float32)
    return depths, cams, conf
