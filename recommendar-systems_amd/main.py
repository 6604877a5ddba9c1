#!/usr/bin/env python3
"""Entry point with the reference's CLI (src/main.py): `python main.py -m LightGCN -d sports`.

Reads configs/ (overall, dataset, model YAML, same keys as the reference) and the
dataset from data_path/<dataset>/<dataset>.inter; the model runs on the rsx
HIP backend (MI355X).  Extra key=value pairs after the flags override config
entries, e.g. `python main.py -m LightGCN -d sports epochs=5 rsx_sampler=host`.
"""
import argparse
import ast
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from rsx.quick_start import quick_start  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", "-m", type=str, default="LightGCN", help="name of models")
    ap.add_argument("--dataset", "-d", type=str, default="baby", help="name of datasets")
    args, rest = ap.parse_known_args()
    config_dict = {"gpu_id": 0}
    for kv in rest:
        if "=" in kv:
            k, v = kv.split("=", 1)
            try:
                config_dict[k.lstrip("-")] = ast.literal_eval(v)
            except (ValueError, SyntaxError):
                config_dict[k.lstrip("-")] = v
    quick_start(model=args.model, dataset=args.dataset, config_dict=config_dict, save_model=True)
