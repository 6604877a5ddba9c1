"""Logging to stdout and ./log/<model>-<dataset>-<time>.log (reference src/utils/logger.py)."""
import logging
import os

from .utils import get_local_time


def init_logger(config, log_root="./log/"):
    os.makedirs(log_root, exist_ok=True)
    path = os.path.join(log_root, "{}-{}-{}.log".format(config["model"], config["dataset"], get_local_time()))
    fmt = logging.Formatter("%(asctime)-15s %(levelname)s %(message)s", "%a %d %b %Y %H:%M:%S")
    root = logging.getLogger()
    root.setLevel(logging.INFO)
    for h in list(root.handlers):
        root.removeHandler(h)
    fh = logging.FileHandler(path, "w", "utf-8")
    fh.setFormatter(fmt)
    sh = logging.StreamHandler()
    sh.setFormatter(logging.Formatter("%(asctime)-15s %(message)s", "%d %b %H:%M"))
    root.addHandler(fh)
    root.addHandler(sh)
    return path
