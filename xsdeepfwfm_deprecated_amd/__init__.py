"""xsdeepfwfm_deprecated_amd -- MI355X-native DeepFwFM forward engine.

The hot path of ShanningLiu/xsDeepFwFM_deprecated (``DeepFMs.forward``) as
hand-written gfx950 HIP kernels behind a C ABI (include/dfwfm.h,
``libdfwfm.so``), surfaced through a drop-in ``DeepFMs`` module.
"""
from ._lib import DfwfmError, build, lib  # noqa: F401
from .DeepFMs import DeepFMs  # noqa: F401
from .QREmbeddingBag import QREmbeddingBag  # noqa: F401
from . import torch_ops  # noqa: F401  -- registers torch.ops.dfwfm.forward

__all__ = ["DeepFMs", "QREmbeddingBag", "DfwfmError", "build", "lib"]
