"""PFM depth-map I/O (reference: datasets/data_io.py:9-74), shared with the fusion step.

``save_png`` of the reference (:77-128) is a matplotlib colour-map plot (and fails on
numpy >= 1.24 at its ``np.object`` check, :90): visualisation, out of the §8 scope.
"""
from aarmvs.fusion import read_pfm, save_pfm  # noqa: F401

__all__ = ["read_pfm", "save_pfm"]
