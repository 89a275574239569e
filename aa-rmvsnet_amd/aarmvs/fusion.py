"""Depth-map fusion (the reference's fusion.py) on the HIP library.

``filter_depth_core`` is the per-reference-view core of ``filter_depth``
(fusion.py:174-220): photometric mask, geometric consistency against every source view
(``reproject_with_depth`` / ``check_geometric_consistency``, fusion.py:71-133), the
per-threshold votes, the geometric and final masks and the averaged depth -- one HIP
launch (``aarmvs_fusion_filter``).  ``fuse_points`` back-projects the kept pixels to world
points (fusion.py:235-246), and ``filter_depth`` is the per-scan driver (fusion.py:135-273):
pair file, per reference view the image rescale/crop and camera re-centring, the GPU core
against every source view, the three mask PNGs and the scan's PLY.  The file helpers
read/write the formats the fusion step consumes: PFM maps (``datasets.data_io``, the
reference's datasets/data_io.py:9-74, re-exported here), cam files (fusion.py:27-42), pair files (fusion.py:57-68), images (fusion.py:45-50), masks
(fusion.py:52-56) and a binary PLY writer for the point cloud.
Depth maps must be CUDA float32 tensors; there is no CPU fallback.
"""
from __future__ import annotations

import os

import ctypes

import numpy as np
import torch

from datasets.data_io import read_pfm, save_pfm  # noqa: F401  (fusion.read_pfm / save_pfm)

from . import _lib
from ._lib import AarmvsError, check, lib


def pack_cameras(ref_cam, src_cams) -> np.ndarray:
    """float32 matrices exactly as numpy forms them in fusion.py:71-108 (float32 inverses
    and float32 products), packed for ``aarmvs_fusion_filter`` (include/aarmvs.h)."""
    K_ref = np.asarray(ref_cam[0], np.float32)
    E_ref = np.asarray(ref_cam[1], np.float32)
    parts = [np.linalg.inv(K_ref).ravel(), K_ref.ravel()]
    for K, E in src_cams:
        K = np.asarray(K, np.float32)
        E = np.asarray(E, np.float32)
        parts += [K.ravel(), np.linalg.inv(K).ravel(),
                  np.matmul(E, np.linalg.inv(E_ref))[:3].ravel(),
                  np.matmul(E_ref, np.linalg.inv(E))[:3].ravel()]
    out = np.concatenate(parts).astype(np.float32)
    assert out.size == _lib.fusion_cam_floats(len(src_cams))
    return np.ascontiguousarray(out)


def filter_depth_core(ref_depth: torch.Tensor, confidence: torch.Tensor, ref_cam, src_depths,
                      src_cams, photo_threshold: float):
    """(photo_mask, geo_mask, final_mask [H,W] bool, depth_est_averaged [H,W] float64)."""
    nsrc = len(src_depths)
    if not 1 <= nsrc <= _lib.MAX_FUSION_SRC:
        raise AarmvsError(f"aarmvs: fusion needs 1..{_lib.MAX_FUSION_SRC} source views, got {nsrc}")
    maps = [ref_depth, confidence, *src_depths]
    for t in maps:
        if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32):
            raise AarmvsError("aarmvs: fusion depth maps / confidence must be CUDA float32 tensors")
        if t.shape != ref_depth.shape or t.dim() != 2:
            raise AarmvsError("aarmvs: fusion maps must all be [H,W] of the same size")
    maps = [t.contiguous() for t in maps]
    H, W = ref_depth.shape
    dev = ref_depth.device
    cams = pack_cameras(ref_cam, src_cams)
    photo = torch.empty(H, W, dtype=torch.uint8, device=dev)
    geo = torch.empty_like(photo)
    final = torch.empty_like(photo)
    avg = torch.empty(H, W, dtype=torch.float64, device=dev)
    a = _lib.FusionArgs()
    a.H, a.W, a.nsrc = H, W, nsrc
    a.ref_depth = maps[0].data_ptr()
    a.confidence = maps[1].data_ptr()
    for i, t in enumerate(maps[2:]):
        a.src_depth[i] = t.data_ptr()
    a.cams = cams.ctypes.data
    a.photo_threshold = float(np.float32(photo_threshold))
    a.photo_mask, a.geo_mask, a.final_mask = photo.data_ptr(), geo.data_ptr(), final.data_ptr()
    a.depth_avg = avg.data_ptr()
    check(lib().aarmvs_fusion_filter(ctypes.byref(a), torch.cuda.current_stream().cuda_stream),
          "fusion_filter")
    return photo.bool(), geo.bool(), final.bool(), avg


def fuse_points(depth_est_averaged, final_mask, ref_cam, ref_img=None):
    """World points (float32 [n,3]) and colours (uint8 [n,3] or None) of the kept pixels
    (fusion.py:235-246), host numpy."""
    depth = depth_est_averaged.cpu().numpy() if isinstance(depth_est_averaged, torch.Tensor) else depth_est_averaged
    valid = final_mask.cpu().numpy() if isinstance(final_mask, torch.Tensor) else final_mask
    K, E = (np.asarray(m, np.float32) for m in ref_cam)
    height, width = depth.shape[:2]
    x, y = np.meshgrid(np.arange(0, width), np.arange(0, height))
    x, y, d = x[valid], y[valid], depth[valid]
    xyz_ref = np.matmul(np.linalg.inv(K), np.vstack((x, y, np.ones_like(x))) * d)
    xyz_world = np.matmul(np.linalg.inv(E), np.vstack((xyz_ref, np.ones_like(x))))[:3]
    colors = None if ref_img is None else (np.asarray(ref_img)[valid] * 255).astype(np.uint8)
    return xyz_world.transpose((1, 0)).astype(np.float32), colors


def crop_params(img_hw, depth_hw):
    """(scale, index, index_p, flag) that map an image of size img_hw onto a depth map of size
    depth_hw: resize by scale, then crop index / index_p columns (flag 0) or rows (flag 1)
    (fusion.py:157-165)."""
    (ih, iw), (dh, dw) = img_hw, depth_hw
    scale = float(dh) / ih
    index = int((int(iw * scale) - dw) / 2)
    index_p = (int(iw * scale) - dw) - index
    flag = 0
    if dw / iw > scale:
        scale = float(dw) / iw
        index = int((int(ih * scale) - dh) / 2)
        index_p = (int(ih * scale) - dh) - index
        flag = 1
    return scale, index, index_p, flag


def resize_linear(img, width, height):
    """cv2.resize(img, (width, height)) with the default INTER_LINEAR on a float32 [H,W,C]
    image, restated from OpenCV's published algorithm (imgproc/src/resize.cpp): source
    coordinate (d + 0.5) / scale - 0.5, clamped taps, float32 horizontal then vertical
    passes; an exact 2x downscale takes OpenCV's INTER_AREA path (2x2 mean).  cv2 is not
    installed here, so agreement with cv2 itself is parity unpinned; the common DTU / T&T
    case is scale 1 (the identity)."""
    img = np.asarray(img, np.float32)
    ih, iw = img.shape[:2]
    if (iw, ih) == (width, height):
        return img.copy()
    if iw == 2 * width and ih == 2 * height:
        q = img[0::2, 0::2] + img[0::2, 1::2]
        q = q + img[1::2, 0::2]
        q = q + img[1::2, 1::2]
        return (q * np.float32(0.25)).astype(np.float32)

    def taps(n_src, n_dst):
        scale = float(n_src) / n_dst   # 1 / inv_scale (double), resize.cpp
        d = np.arange(n_dst, dtype=np.float64)
        f = ((d + 0.5) * scale - 0.5).astype(np.float32)
        s0 = np.floor(f).astype(np.int64)
        f = (f - s0.astype(np.float32)).astype(np.float32)
        lo = s0 < 0
        f[lo], s0[lo] = 0.0, 0
        hi = s0 >= n_src - 1
        f[hi], s0[hi] = 0.0, n_src - 1
        s1 = np.minimum(s0 + 1, n_src - 1)
        return s0, s1, (np.float32(1) - f).astype(np.float32), f

    x0, x1, ax0, ax1 = taps(iw, width)
    y0, y1, by0, by1 = taps(ih, height)
    ex = (slice(None), None) if img.ndim == 3 else (slice(None),)
    rows = img[:, x0] * ax0[ex] + img[:, x1] * ax1[ex]          # horizontal pass, float32
    ey = (slice(None), None, None) if img.ndim == 3 else (slice(None), None)
    out = by0[ey] * rows[y0] + by1[ey] * rows[y1]                # vertical pass
    return out.astype(np.float32)


def filter_depth(scan_folder, out_folder, plyfilename, photo_threshold, device="cuda"):
    """fusion.py:135-273 for one scan: for every (ref_view, src_views) of pair.txt with an
    estimated depth map, the geometric / photometric filtering on the GPU
    (``filter_depth_core``), the three mask PNGs under out_folder/mask, and the kept pixels'
    world points (coloured from the rescaled, cropped reference image) written to
    plyfilename.  Returns the number of points written."""
    vertexs, vertex_colors = [], []
    dev = torch.device(device)
    for ref_view, src_views in read_pair_file(os.path.join(scan_folder, "pair.txt")):
        dpath = os.path.join(out_folder, "depth_est_0/{:0>8}.pfm".format(ref_view))
        if not os.path.exists(dpath):
            print("skip", ref_view)
            continue
        ref_img = read_img(os.path.join(scan_folder, "images/{:0>8}.jpg".format(ref_view)))
        ref_depth_est = read_pfm(dpath)[0]
        confidence = read_pfm(os.path.join(out_folder, "confidence_0/{:0>8}.pfm".format(ref_view)))[0]
        scale, index, index_p, flag = crop_params(ref_img.shape[:2], confidence.shape[:2])
        ref_img = resize_linear(ref_img, int(ref_img.shape[1] * scale), int(ref_img.shape[0] * scale))
        if flag == 0:
            ref_img = ref_img[:, index:ref_img.shape[1] - index_p, :]
        else:
            ref_img = ref_img[index:ref_img.shape[0] - index_p, :, :]
        cam_file = os.path.join(scan_folder, "cams/{:0>8}_cam.txt")
        ref_cam = read_camera_parameters(cam_file.format(ref_view), scale, index, flag)
        src_depths, src_cams = [], []
        for src_view in src_views:
            src_depths.append(torch.from_numpy(np.ascontiguousarray(read_pfm(
                os.path.join(out_folder, "depth_est_0/{:0>8}.pfm".format(src_view)))[0])).to(dev))
            src_cams.append(read_camera_parameters(cam_file.format(src_view), scale, index, flag))
        photo, geo, final, avg = filter_depth_core(
            torch.from_numpy(np.ascontiguousarray(ref_depth_est)).to(dev),
            torch.from_numpy(np.ascontiguousarray(confidence)).to(dev), ref_cam, src_depths, src_cams,
            photo_threshold)
        photo, geo, final = (m.cpu().numpy() for m in (photo, geo, final))
        os.makedirs(os.path.join(out_folder, "mask"), exist_ok=True)
        save_mask(os.path.join(out_folder, "mask/{:0>8}_photo.png".format(ref_view)), photo)
        save_mask(os.path.join(out_folder, "mask/{:0>8}_geo.png".format(ref_view)), geo)
        save_mask(os.path.join(out_folder, "mask/{:0>8}_final.png".format(ref_view)), final)
        print("processing {}, ref-view{:0>2}, photo/geo/final-mask:{}/{}/{}".format(
            scan_folder, ref_view, photo.mean(), geo.mean(), final.mean()))
        xyz, rgb = fuse_points(avg.cpu().numpy(), final, ref_cam, ref_img)
        vertexs.append(xyz)
        vertex_colors.append(rgb)
    xyz = np.concatenate(vertexs, axis=0) if vertexs else np.zeros((0, 3), np.float32)
    rgb = np.concatenate(vertex_colors, axis=0) if vertex_colors else np.zeros((0, 3), np.uint8)
    write_ply(plyfilename, xyz, rgb)
    print("saving the final model to", plyfilename)
    return xyz.shape[0]


# ---------------------------------------------------------------------------------
# file formats
# ---------------------------------------------------------------------------------
def read_img(filename):
    """float32 image in [0, 1] (fusion.py:45-50)."""
    from PIL import Image
    return np.array(Image.open(filename), dtype=np.float32) / 255.0


def save_mask(filename, mask):
    """8-bit PNG, 255 where the mask is set (fusion.py:52-56)."""
    from PIL import Image
    mask = np.asarray(mask)
    if mask.dtype != np.bool_:
        raise ValueError("save_mask: mask must be boolean")
    Image.fromarray(mask.astype(np.uint8) * 255).save(filename)
def read_camera_parameters(filename, scale=1.0, index=0, flag=0):
    """(intrinsics float32 3x3, extrinsics float32 4x4) of a cam.txt, intrinsics scaled and
    shifted for the resized / cropped image (fusion.py:27-42)."""
    with open(filename) as f:
        lines = [line.rstrip() for line in f.readlines()]
    extrinsics = np.array(" ".join(lines[1:5]).split(), dtype=np.float32).reshape((4, 4))
    intrinsics = np.array(" ".join(lines[7:10]).split(), dtype=np.float32).reshape((3, 3))
    intrinsics[:2, :] *= scale
    if flag == 0:
        intrinsics[0, 2] -= index
    else:
        intrinsics[1, 2] -= index
    return intrinsics, extrinsics


def read_pair_file(filename):
    """[(ref_view, [src_view, ...]), ...] (fusion.py:57-68)."""
    data = []
    with open(filename) as f:
        num_viewpoint = int(f.readline())
        for _ in range(num_viewpoint):
            ref_view = int(f.readline().rstrip())
            src_views = [int(x) for x in f.readline().rstrip().split()[1::2]]
            data.append((ref_view, src_views))
    return data


def write_ply(filename, xyz, rgb=None):
    """Binary little-endian PLY of float32 x, y, z (+ uint8 red, green, blue) vertices."""
    xyz = np.asarray(xyz, np.float32)
    n = xyz.shape[0]
    fields = [("x", "<f4"), ("y", "<f4"), ("z", "<f4")]
    if rgb is not None:
        fields += [("red", "u1"), ("green", "u1"), ("blue", "u1")]
    v = np.empty(n, dtype=fields)
    v["x"], v["y"], v["z"] = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    if rgb is not None:
        rgb = np.asarray(rgb, np.uint8)
        v["red"], v["green"], v["blue"] = rgb[:, 0], rgb[:, 1], rgb[:, 2]
    props = "".join(f"property {'float' if t == '<f4' else 'uchar'} {name}\n" for name, t in fields)
    header = f"ply\nformat binary_little_endian 1.0\nelement vertex {n}\n{props}end_header\n"
    with open(filename, "wb") as f:
        f.write(header.encode("ascii"))
        f.write(v.tobytes())
