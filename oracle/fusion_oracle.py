"""CPU restatement of AA-RMVSNet's depth-map fusion core (fusion.py) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's CPU leg may import this module; the
product path (aarmvs.fusion) runs the HIP kernel and never falls back to it.

Follows, function by function:
  reproject_with_depth          fusion.py:71-110 (float64 numpy arithmetic on float32 inputs,
                                the float32 casts of the maps and of the reprojected depth)
  check_geometric_consistency   fusion.py:112-133 (masks for i = 2..10, the i = 10 mask
                                zeroing depth_reprojected)
  filter_depth_core             fusion.py:174-220 (photo mask, per-threshold vote counts,
                                geo mask, averaged depth) -- the per-reference-view core of
                                filter_depth without file I/O, image resizing and the PLY write
  remap_linear                  cv2.remap(src, map_x, map_y, INTER_LINEAR) with the default
                                BORDER_CONSTANT 0, restated from OpenCV's published algorithm
                                (imgproc/src/imgwarp.cpp: float maps are rounded to 1/32 pixel,
                                INTER_TAB_SIZE = 32, bilinear weights from that table, the four
                                taps summed left to right in float32; out-of-image taps read the
                                border value).  OpenCV (cv2) is not installed in this image and the
                                reference ships no fusion fixtures, so this function's agreement
                                with cv2 itself is parity unpinned.
Camera matrices are the reference's float32 arrays (read_camera_parameters, fusion.py:27-42);
inverses and products are taken in float32 exactly as numpy does there.
"""
import numpy as np

INTER_BITS = 5
INTER_TAB_SIZE = 1 << INTER_BITS


def remap_linear(src, map_x, map_y):
    """cv2.remap(src, map_x, map_y, cv2.INTER_LINEAR), src float32 [H,W], maps float32."""
    src = np.asarray(src, np.float32)
    H, W = src.shape
    mx = np.asarray(map_x, np.float32)
    my = np.asarray(map_y, np.float32)
    # cvRound: half to even; a non-finite map casts to INT64_MIN (x86), i.e. outside the image,
    # where the taps read the constant border 0 as cv2's INT_MIN does
    with np.errstate(invalid="ignore"):
        X = np.rint(mx * np.float32(INTER_TAB_SIZE)).astype(np.int64)
        Y = np.rint(my * np.float32(INTER_TAB_SIZE)).astype(np.int64)
    sx, sy = X >> INTER_BITS, Y >> INTER_BITS
    fx = (X & (INTER_TAB_SIZE - 1)).astype(np.float32) / np.float32(INTER_TAB_SIZE)
    fy = (Y & (INTER_TAB_SIZE - 1)).astype(np.float32) / np.float32(INTER_TAB_SIZE)
    cx0, cx1 = np.float32(1) - fx, fx
    cy0, cy1 = np.float32(1) - fy, fy
    w = [cy0 * cx0, cy0 * cx1, cy1 * cx0, cy1 * cx1]

    def tap(yy, xx):
        ok = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
        v = np.zeros(xx.shape, np.float32)
        v[ok] = src[yy[ok], xx[ok]]
        return v

    v = [tap(sy, sx), tap(sy, sx + 1), tap(sy + 1, sx), tap(sy + 1, sx + 1)]
    out = v[0] * w[0]
    out = out + v[1] * w[1]
    out = out + v[2] * w[2]
    out = out + v[3] * w[3]
    return out.astype(np.float32)


def reproject_with_depth(depth_ref, intrinsics_ref, extrinsics_ref, depth_src, intrinsics_src,
                         extrinsics_src):
    """fusion.py:71-110."""
    height, width = depth_ref.shape
    x_ref, y_ref = np.meshgrid(np.arange(0, width), np.arange(0, height))
    x_ref, y_ref = x_ref.reshape([-1]), y_ref.reshape([-1])
    xyz_ref = np.matmul(np.linalg.inv(intrinsics_ref),
                        np.vstack((x_ref, y_ref, np.ones_like(x_ref))) * depth_ref.reshape([-1]))
    xyz_src = np.matmul(np.matmul(extrinsics_src, np.linalg.inv(extrinsics_ref)),
                        np.vstack((xyz_ref, np.ones_like(x_ref))))[:3]
    K_xyz_src = np.matmul(intrinsics_src, xyz_src)
    xy_src = K_xyz_src[:2] / K_xyz_src[2:3]
    x_src = xy_src[0].reshape([height, width]).astype(np.float32)
    y_src = xy_src[1].reshape([height, width]).astype(np.float32)
    sampled_depth_src = remap_linear(depth_src, x_src, y_src)
    xyz_src = np.matmul(np.linalg.inv(intrinsics_src),
                        np.vstack((xy_src, np.ones_like(x_ref))) * sampled_depth_src.reshape([-1]))
    xyz_reprojected = np.matmul(np.matmul(extrinsics_ref, np.linalg.inv(extrinsics_src)),
                                np.vstack((xyz_src, np.ones_like(x_ref))))[:3]
    depth_reprojected = xyz_reprojected[2].reshape([height, width]).astype(np.float32)
    K_xyz_reprojected = np.matmul(intrinsics_ref, xyz_reprojected)
    with np.errstate(divide="ignore", invalid="ignore"):   # depth 0 -> inf / nan, as the reference
        xy_reprojected = K_xyz_reprojected[:2] / K_xyz_reprojected[2:3]
    x_reprojected = xy_reprojected[0].reshape([height, width]).astype(np.float32)
    y_reprojected = xy_reprojected[1].reshape([height, width]).astype(np.float32)
    return depth_reprojected, x_reprojected, y_reprojected, x_src, y_src


def check_geometric_consistency(depth_ref, intrinsics_ref, extrinsics_ref, depth_src,
                                intrinsics_src, extrinsics_src):
    """fusion.py:112-133: (masks[i=2..10], mask (i=10), depth_reprojected, x2d_src, y2d_src,
    vis_mask)."""
    height, width = depth_ref.shape
    x_ref, y_ref = np.meshgrid(np.arange(0, width), np.arange(0, height))
    depth_reprojected, x2d_reprojected, y2d_reprojected, x2d_src, y2d_src = reproject_with_depth(
        depth_ref, intrinsics_ref, extrinsics_ref, depth_src, intrinsics_src, extrinsics_src)
    dist = np.sqrt((x2d_reprojected - x_ref) ** 2 + (y2d_reprojected - y_ref) ** 2)
    depth_diff = np.abs(depth_reprojected - depth_ref)
    with np.errstate(divide="ignore", invalid="ignore"):
        relative_depth_diff = depth_diff / depth_ref
    masks = []
    for i in range(2, 11):
        mask = np.logical_and(dist < i / 4, relative_depth_diff < np.float32(i / 1300))
        masks.append(mask)
    vis_mask = np.logical_and(dist < 1, relative_depth_diff < np.float32(0.01))
    depth_reprojected[~mask] = 0
    return masks, mask, depth_reprojected, x2d_src, y2d_src, vis_mask


def filter_depth_core(ref_depth, confidence, ref_cam, src_depths, src_cams, photo_threshold):
    """fusion.py:174-220 for one reference view: (photo_mask, geo_mask, final_mask,
    depth_est_averaged).  Cameras are (intrinsics float32 3x3, extrinsics float32 4x4);
    at most 10 source views (the reference indexes masks[0..n-3])."""
    ref_K, ref_E = ref_cam
    photo_mask = confidence > np.float32(photo_threshold)
    n = 1 + len(src_depths)
    geo_mask_sum = 0
    geo_mask_sums = []
    all_srcview_depth_ests = []
    for ct, (src_depth, (K, E)) in enumerate(zip(src_depths, src_cams), start=1):
        masks, geo_mask, depth_reprojected, _, _, _ = check_geometric_consistency(
            ref_depth, ref_K, ref_E, src_depth, K, E)
        if ct == 1:
            for i in range(2, n):
                geo_mask_sums.append(masks[i - 2].astype(np.int32))
        else:
            for i in range(2, n):
                geo_mask_sums[i - 2] += masks[i - 2].astype(np.int32)
        geo_mask_sum += geo_mask.astype(np.int32)
        all_srcview_depth_ests.append(depth_reprojected)
    geo_mask = geo_mask_sum >= n
    for i in range(2, n):
        geo_mask = np.logical_or(geo_mask, geo_mask_sums[i - 2] >= i)
    depth_est_averaged = (sum(all_srcview_depth_ests) + ref_depth) / (geo_mask_sum + 1)
    final_mask = np.logical_and(photo_mask, geo_mask)
    return photo_mask, geo_mask, final_mask, depth_est_averaged


def filter_depth_scan(pair_data, images, cam_texts, depth_ests, confidences, photo_threshold):
    """fusion.py:135-273 on in-memory inputs: pair_data [(ref, [src...])], images {view: float32
    [H,W,3] in [0,1]}, cam_texts {view: cam.txt text}, depth_ests / confidences {view: float32
    [h,w]} (views without a depth map are skipped).  Returns (masks {ref: (photo, geo, final)},
    xyz float32 [n,3], rgb uint8 [n,3]).  The image rescale is the identity here (the tests
    use scale 1: cv2 is absent, its INTER_LINEAR resize is parity unpinned)."""
    def cam(text, scale, index, flag):                       # fusion.py:27-42
        lines = [ln.rstrip() for ln in text.splitlines()]
        E = np.array(" ".join(lines[1:5]).split(), dtype=np.float32).reshape((4, 4))
        K = np.array(" ".join(lines[7:10]).split(), dtype=np.float32).reshape((3, 3))
        K[:2, :] *= scale
        if flag == 0:
            K[0, 2] -= index
        else:
            K[1, 2] -= index
        return K, E

    masks, verts, cols = {}, [], []
    for ref_view, src_views in pair_data:
        if ref_view not in depth_ests:
            continue
        ref_img = images[ref_view]
        ref_depth = depth_ests[ref_view]
        conf = confidences[ref_view]
        scale = float(conf.shape[0]) / ref_img.shape[0]       # fusion.py:157-171
        index = int((int(ref_img.shape[1] * scale) - conf.shape[1]) / 2)
        index_p = (int(ref_img.shape[1] * scale) - conf.shape[1]) - index
        flag = 0
        if conf.shape[1] / ref_img.shape[1] > scale:
            scale = float(conf.shape[1]) / ref_img.shape[1]
            index = int((int(ref_img.shape[0] * scale) - conf.shape[0]) / 2)
            index_p = (int(ref_img.shape[0] * scale) - conf.shape[0]) - index
            flag = 1
        assert (int(ref_img.shape[1] * scale), int(ref_img.shape[0] * scale)) == ref_img.shape[1::-1]
        if flag == 0:
            ref_img = ref_img[:, index:ref_img.shape[1] - index_p, :]
        else:
            ref_img = ref_img[index:ref_img.shape[0] - index_p, :, :]
        ref_cam = cam(cam_texts[ref_view], scale, index, flag)
        src_d = [depth_ests[s] for s in src_views]
        src_c = [cam(cam_texts[s], scale, index, flag) for s in src_views]
        photo, geo, final, avg = filter_depth_core(ref_depth, conf, ref_cam, src_d, src_c, photo_threshold)
        masks[ref_view] = (photo, geo, final)
        h, w = avg.shape                                       # fusion.py:246-257
        x, y = np.meshgrid(np.arange(0, w), np.arange(0, h))
        x, y, depth = x[final], y[final], avg[final]
        color = ref_img[final]
        xyz_ref = np.matmul(np.linalg.inv(ref_cam[0]), np.vstack((x, y, np.ones_like(x))) * depth)
        xyz_world = np.matmul(np.linalg.inv(ref_cam[1]), np.vstack((xyz_ref, np.ones_like(x))))[:3]
        verts.append(xyz_world.transpose((1, 0)))
        cols.append((color * 255).astype(np.uint8))
    return masks, np.concatenate(verts).astype(np.float32), np.concatenate(cols)
