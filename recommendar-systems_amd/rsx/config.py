"""Layered YAML configuration, same surface as the reference's Config
(src/utils/configurator.py:46-149).

Priority (low -> high): configs/overall.yaml, configs/dataset/<dataset>.yaml,
configs/model/<model>.yaml, configs/mg.yaml (when mg=True), then the caller's
config_dict.  `hyper_parameters` lists from every file are concatenated and
"seed" is always part of the grid.  Scientific-notation scalars such as `1e-3`
load as floats.  `config['device']` is the GPU this process drives: LOCAL_RANK
under torchrun, else `gpu_id` (the reference pins CUDA_VISIBLE_DEVICES to
gpu_id, configurator.py:114-118, which would put every rank on one GPU).
"""
from __future__ import annotations

import os
import re

import torch
import yaml

CONFIG_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs")

_FLOAT = re.compile(r"""^(?:
     [-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
    |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
    |\.[0-9_]+(?:[eE][-+][0-9]+)?
    |[-+]?[0-9][0-9_]*(?::[0-5]?[0-9])+\.[0-9_]*
    |[-+]?\.(?:inf|Inf|INF)
    |\.(?:nan|NaN|NAN))$""", re.X)


class _Loader(yaml.SafeLoader):
    pass


_Loader.add_implicit_resolver("tag:yaml.org,2002:float", _FLOAT, list("-+0123456789."))


def load_yaml(path: str) -> dict:
    with open(path, "r", encoding="utf-8") as f:
        return yaml.load(f.read(), Loader=_Loader) or {}


class Config:
    def __init__(self, model=None, dataset=None, config_dict=None, mg=False, config_dir=None):
        config_dict = dict(config_dict or {})
        config_dict["model"] = model
        config_dict["dataset"] = dataset
        self.config_dir = config_dir or os.environ.get("RSX_CONFIG_DIR", CONFIG_DIR)
        files = [os.path.join(self.config_dir, "overall.yaml"),
                 os.path.join(self.config_dir, "dataset", f"{dataset}.yaml"),
                 os.path.join(self.config_dir, "model", f"{model}.yaml")]
        if mg:
            files.append(os.path.join(self.config_dir, "mg.yaml"))
        merged, grid = {}, []
        for path in files:
            if not os.path.isfile(path):
                continue
            data = load_yaml(path)
            grid.extend(data.get("hyper_parameters") or [])
            merged.update(data)
        merged["hyper_parameters"] = grid
        merged.update(config_dict)
        self.final_config_dict = merged
        metric = str(merged.get("valid_metric", "Recall@20")).split("@")[0].lower()
        merged["valid_metric_bigger"] = metric not in ("rmse", "mae", "logloss")
        if "seed" not in merged["hyper_parameters"]:
            merged["hyper_parameters"] = list(merged["hyper_parameters"]) + ["seed"]
        merged["device"] = self._device()

    def _device(self):
        c = self.final_config_dict
        if c.get("use_gpu", True) and torch.cuda.is_available():
            idx = int(os.environ.get("LOCAL_RANK", c.get("gpu_id", 0) or 0))
            return torch.device("cuda", idx)
        return torch.device("cpu")

    # dict-like access (reference configurator.py:120-149)
    def __setitem__(self, key, value):
        if not isinstance(key, str):
            raise TypeError("index must be a str.")
        self.final_config_dict[key] = value

    def __getitem__(self, item):
        return self.final_config_dict.get(item)

    def get(self, key, default=None):
        if not isinstance(key, str):
            raise TypeError("index must be a str.")
        return self.final_config_dict.get(key, default)

    def __contains__(self, key):
        if not isinstance(key, str):
            raise TypeError("index must be a str.")
        return key in self.final_config_dict

    def __str__(self):
        return "\n" + "\n".join(f"{k}={v}" for k, v in self.final_config_dict.items()) + "\n\n"

    __repr__ = __str__
