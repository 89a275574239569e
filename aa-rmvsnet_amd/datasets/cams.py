"""Camera files, pair files and the depth-hypothesis recipes of the reference's dataloaders
(SURVEY §8f-4): they decide which depth_values the sweep sees.

MVSNet camera text format (one file per view): line 0 ``extrinsic``, lines 1-4 the 4x4
world-to-camera matrix, line 6 ``intrinsic``, lines 7-9 the 3x3 K, line 11
``depth_min depth_interval [depth_num depth_max]``.

Reference functions restated (file:line under BuTTerK3ks/AA-RMVSNet/datasets):
  read_cam          dtu_yao.py:64-79, data_eval_transform.py:57-69,
                    data_eval_transform_padding.py:60-81
  projection        dtu_yao.py:144-146, data_eval_transform.py:163-167
  depth hypotheses  dtu_yao.py:149-160 (+ flip :172-173), data_eval_transform.py:117-129,
                    data_eval_transform_padding.py:131-145
"""
from __future__ import annotations

import numpy as np


def _floats(lines) -> np.ndarray:
    return np.array(" ".join(lines).split(), dtype=np.float32)


def read_cam(filename, interval_scale=1.06, image_scale=None, row_shift=0.0, with_depth_end=False):
    """(intrinsics [3,3] f32, extrinsics [4,4] f32, depth_min, depth_interval[, depth_end]).

    ``depth_interval`` is the file's interval times ``interval_scale``.  ``image_scale``
    (training loader): the cameras describe 1/4-resolution images, so K's first two rows
    are multiplied by 2 at 0.5 and by 4 at 1.0 (dtu_yao.py:71-74).  ``row_shift`` adds to
    K[1,2] (the padding loader's +4 rows of zero padding, data_eval_transform_padding.py:68).
    ``with_depth_end`` also returns the file's 4th depth field (padding loader, :79).
    """
    with open(filename) as f:
        lines = [ln.rstrip() for ln in f.readlines()]
    extrinsics = _floats(lines[1:5]).reshape(4, 4)
    intrinsics = _floats(lines[7:10]).reshape(3, 3)
    if image_scale == 0.5:
        intrinsics[:2, :] *= 2
    elif image_scale == 1.0:
        intrinsics[:2, :] *= 4
    if row_shift:
        intrinsics[1, 2] += row_shift
    fields = lines[11].split()
    depth_min = float(fields[0])
    depth_interval = float(fields[1]) * interval_scale
    if with_depth_end:
        return intrinsics, extrinsics, depth_min, depth_interval, float(fields[3])
    return intrinsics, extrinsics, depth_min, depth_interval


def write_cam(filename, intrinsics, extrinsics, depth_min, depth_interval, depth_num=None,
              depth_max=None):
    """Write a camera file in the format read_cam parses (test data, tools)."""
    with open(filename, "w") as f:
        f.write("extrinsic\n")
        for r in np.asarray(extrinsics, dtype=np.float64).reshape(4, 4):
            f.write(" ".join(repr(float(v)) for v in r) + "\n")
        f.write("\nintrinsic\n")
        for r in np.asarray(intrinsics, dtype=np.float64).reshape(3, 3):
            f.write(" ".join(repr(float(v)) for v in r) + "\n")
        extra = "" if depth_num is None else f" {depth_num} {depth_max}"
        f.write(f"\n{depth_min} {depth_interval}{extra}\n")


def read_pair(filename):
    """[(ref_view, [src_views...])] from a pair.txt (dtu_yao.py:43-49, fusion.py:57-68)."""
    out = []
    with open(filename) as f:
        n = int(f.readline())
        for _ in range(n):
            ref = int(f.readline().rstrip())
            srcs = [int(x) for x in f.readline().rstrip().split()[1::2]]
            out.append((ref, srcs))
    return out


def projection(intrinsics, extrinsics) -> np.ndarray:
    """[4,4] f32: rows 0-2 = K @ E[:3,:4], row 3 = E[3] (dtu_yao.py:144-146)."""
    P = np.array(extrinsics, dtype=np.float32, copy=True)
    P[:3, :4] = np.matmul(intrinsics, P[:3, :4])
    return P


def train_depth_values(depth_min, depth_interval, ndepths, inverse=False, fix_range=False,
                       reverse=False):
    """Training loader (dtu_yao.py:149-160): D hypotheses from depth_min to depth_end =
    depth_min + (D-1) interval (935 with ``fix_range``), evenly in depth or in inverse
    depth (``inverse``); ``reverse`` gives the descending order of the flip samples
    (:172-173).  Returns (depth_values f32 [D], depth_end)."""
    depth_end = 935 if fix_range else depth_interval * (ndepths - 1) + depth_min
    if inverse:
        dv = (1.0 / np.linspace(1.0 / depth_min, 1.0 / depth_end, ndepths)).astype(np.float32)
    else:
        dv = np.linspace(depth_min, depth_end, ndepths).astype(np.float32)
    if reverse:
        dv = dv[::-1].copy()
    return dv, depth_end


def eval_depth_values(depth_min, depth_interval, ndepths, inverse=True):
    """Eval loader (data_eval_transform.py:117-129): inverse spacing from 1/depth_min towards
    0 with ``endpoint=False`` (so the far end is depth_min * D, not infinity), or
    ``arange(depth_min, depth_min + D interval, interval)`` in f32.  Returns f32 [D]."""
    if inverse:
        return (1.0 / np.linspace(1.0 / depth_min, 0.0, ndepths, endpoint=False)).astype(np.float32)
    return np.arange(depth_min, depth_interval * ndepths + depth_min, depth_interval, dtype=np.float32)


def padding_depth_values(depth_min, depth_end, ndepths, inverse=True):
    """Padding eval loader (data_eval_transform_padding.py:131-145): D hypotheses between
    depth_min and the camera file's depth_end with ``endpoint=False``, evenly in inverse
    depth or in depth.  Returns f32 [D]."""
    if inverse:
        return (1.0 / np.linspace(1.0 / depth_min, 1.0 / depth_end, ndepths, endpoint=False)
                ).astype(np.float32)
    return np.linspace(depth_min, depth_end, ndepths, endpoint=False).astype(np.float32)
