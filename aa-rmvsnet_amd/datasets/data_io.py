"""PFM depth-map I/O (reference: datasets/data_io.py:9-74): the dataloaders' depth maps, the
eval driver's depth / confidence outputs and the fusion step's inputs.

``save_png`` of the reference (:77-128) is a matplotlib colour-map plot (and fails on
numpy >= 1.24 at its ``np.object`` check, :90): visualisation, out of the §8 scope.
"""
import re
import sys

import numpy as np

__all__ = ["read_pfm", "save_pfm"]


def read_pfm(filename):
    """(data float32 [H,W] or [H,W,3], scale), rows bottom-up in the file (data_io.py:9-45)."""
    with open(filename, "rb") as f:
        header = f.readline().decode("utf-8").rstrip()
        if header not in ("PF", "Pf"):
            raise ValueError("Not a PFM file.")
        m = re.match(r"^(\d+)\s(\d+)\s$", f.readline().decode("utf-8"))
        if not m:
            raise ValueError("Malformed PFM header.")
        width, height = map(int, m.groups())
        scale = float(f.readline().rstrip())
        endian = "<" if scale < 0 else ">"
        data = np.fromfile(f, endian + "f")
    shape = (height, width, 3) if header == "PF" else (height, width)
    return np.flipud(np.reshape(data, shape)), abs(scale)


def save_pfm(filename, image, scale=1):
    """data_io.py:48-74: float32 [H,W] / [H,W,1] / [H,W,3], native byte order."""
    if image.dtype != np.float32:
        raise ValueError("Image dtype must be float32.")
    if image.ndim == 3 and image.shape[2] == 3:
        color = True
    elif image.ndim == 2 or (image.ndim == 3 and image.shape[2] == 1):
        color = False
    else:
        raise ValueError("Image must have H x W x 3, H x W x 1 or H x W dimensions.")
    image = np.flipud(image)
    endian = image.dtype.byteorder
    if endian == "<" or (endian == "=" and sys.byteorder == "little"):
        scale = -scale
    with open(filename, "wb") as f:
        f.write(b"PF\n" if color else b"Pf\n")
        f.write(f"{image.shape[1]} {image.shape[0]}\n".encode("utf-8"))
        f.write(("%f\n" % scale).encode("utf-8"))
        np.ascontiguousarray(image).tofile(f)
