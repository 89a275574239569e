"""Camera/image rescale and crop of the eval loaders (reference: datasets/preprocess.py).

``scale_camera`` / ``crop_mvs_input`` are plain array arithmetic (restated from
preprocess.py:7-16, 40-74).  The reference resizes images with ``cv2.resize`` (bilinear,
:18-23); OpenCV is not available in this image, so ``scale_image`` resamples with
PyTorch's bilinear interpolation (half-pixel centres, no antialiasing: OpenCV's
INTER_LINEAR grid).  Results agree with OpenCV up to its fixed-point rounding: parity
unpinned for the resize itself (no fixture can be made without OpenCV).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def scale_camera(cam, scale=1):
    """Focal lengths and principal point times ``scale`` (preprocess.py:7-16)."""
    new_cam = np.copy(cam)
    new_cam[0][0] = cam[0][0] * scale
    new_cam[1][1] = cam[1][1] * scale
    new_cam[0][2] = cam[0][2] * scale
    new_cam[1][2] = cam[1][2] * scale
    return new_cam


def scale_image(image, scale=1, interpolation="linear"):
    """[H,W(,C)] image resized by ``scale`` (output size round(H scale), round(W scale))."""
    if scale == 1:
        return np.array(image, copy=True)
    img = np.asarray(image, dtype=np.float32)
    h, w = img.shape[:2]
    size = (int(round(h * scale)), int(round(w * scale)))
    t = torch.from_numpy(np.ascontiguousarray(img))
    t = t.permute(2, 0, 1)[None] if t.dim() == 3 else t[None, None]
    if interpolation == "nearest":
        out = F.interpolate(t, size=size, mode="nearest")
    else:
        out = F.interpolate(t, size=size, mode="bilinear", align_corners=False)
    out = out[0].permute(1, 2, 0) if img.ndim == 3 else out[0, 0]
    return out.numpy()


def scale_mvs_input(images, cams, depth_image=None, scale=1, view_num=5):
    """Resize every view and its camera (preprocess.py:25-38)."""
    new_images = np.array([scale_image(images[v], scale=scale) for v in range(view_num)])
    new_cams = [scale_camera(cams[v], scale=scale) for v in range(view_num)]
    if depth_image is None:
        return new_images, new_cams
    return new_images, cams, scale_image(depth_image, scale=scale, interpolation="nearest")


def crop_mvs_input(images, cams, depth_image=None, view_num=5, max_h=1200, max_w=1600,
                   base_image_size=8):
    """Centre-crop every view to at most (max_h, max_w), else round the size up to a
    multiple of base_image_size, shifting each camera's principal point
    (preprocess.py:40-74; cams are modified in place, as there)."""
    out = []
    for v in range(view_num):
        h, w = images[v].shape[0:2]
        nh = max_h if h > max_h else int(math.ceil(h / base_image_size) * base_image_size)
        nw = max_w if w > max_w else int(math.ceil(w / base_image_size) * base_image_size)
        y0 = int(math.ceil((h - nh) / 2))
        x0 = int(math.ceil((w - nw) / 2))
        out.append(images[v][y0:y0 + nh, x0:x0 + nw])
        cams[v][0][2] = cams[v][0][2] - x0
        cams[v][1][2] = cams[v][1][2] - y0
    out = np.stack(out)
    if depth_image is None:
        return out, cams
    return out, cams, depth_image[y0:y0 + nh, x0:x0 + nw]
