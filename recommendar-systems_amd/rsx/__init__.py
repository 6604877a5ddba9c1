"""rsx — MI355X-native graph-CF training path (LightGCN / LayerGCN / SMORE).

Hot ops are hand-written HIP kernels for gfx950 behind a flat C ABI
(`include/rsx.h`, `librsx.so`); this package is the host side that mirrors
the reference's `GeneralRecommender` / `Trainer` / YAML surface
(reference `src/common/abstract_recommender.py`, `src/common/trainer.py`).
"""
__version__ = "0.1.0"

from . import torch_ops  # noqa: E402,F401  registers torch.ops.rsx.* 
