"""Small helpers with the reference's semantics (src/utils/utils.py:14-114)."""
from __future__ import annotations

import datetime
import importlib
import random

import numpy as np
import torch

MODELS = {"lightgcn": ("rsx.lightgcn", "LightGCN"), "layergcn": ("rsx.layergcn", "LayerGCN"),
          "smore": ("rsx.smore", "SMORE")}


def get_local_time():
    return datetime.datetime.now().strftime("%b-%d-%Y-%H-%M-%S")


def get_model(model_name: str):
    """Model class by name (reference resolves models.<name.lower()>.<name>)."""
    key = model_name.lower()
    if key not in MODELS:
        raise ValueError(f"rsx implements {sorted(v[1] for v in MODELS.values())}; got {model_name}")
    mod, cls = MODELS[key]
    return getattr(importlib.import_module(mod), cls)


def get_trainer():
    from .trainer import Trainer

    return Trainer


def init_seed(seed):
    random.seed(seed)
    np.random.seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)
    torch.manual_seed(seed)


def early_stopping(value, best, cur_step, max_step, bigger=True):
    """(best, cur_step, stop_flag, update_flag) — reference utils.py:57-98."""
    improved = value > best if bigger else value < best
    if improved:
        return value, 0, False, True
    cur_step += 1
    return best, cur_step, cur_step > max_step, False


def dict2str(result_dict):
    return "".join(f"{k}: " + "%.04f" % v + "    " for k, v in result_dict.items())
