"""Drop-in for the reference's ``models`` package (``from models import *``,
models/__init__.py:1): EMVSNet, mvsnet_cls_loss and the models.module blocks, with the
depth sweep on libaarmvs (gfx950)."""
from models.drmvsnet import *  # noqa: F401,F403
