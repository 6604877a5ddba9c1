"""Run a model on a dataset over its hyper-parameter grid (reference src/utils/quick_start.py:19-107).

Same flow: Config -> RecDataset -> split -> loaders -> for every combination of
the `hyper_parameters` lists: init_seed, pretrain_setup, model, Trainer.fit.
"""
from __future__ import annotations

import os
import platform
from itertools import product
from logging import getLogger

from .config import Config
from .data import EvalDataLoader, RecDataset, TrainDataLoader
from .logger import init_logger
from .utils import dict2str, get_model, get_trainer, init_seed


def _init_distributed(config):
    """torchrun (WORLD_SIZE > 1): one process per GPU, a process group over RCCL
    ("nccl"; config rsx_dist_backend overrides, e.g. gloo for several ranks on one
    GPU); the user-sharded LightGCN picks it up (rsx.lightgcn)."""
    import torch
    import torch.distributed as dist

    if int(os.environ.get("WORLD_SIZE", "1")) <= 1 or dist.is_initialized():
        return
    backend = config["rsx_dist_backend"] or "nccl"
    dev = config["device"]
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    kw = {"device_id": dev} if backend == "nccl" else {}
    dist.init_process_group(backend, **kw)


def quick_start(model, dataset, config_dict, save_model=True, mg=False, log=True):
    config = Config(model, dataset, config_dict, mg)
    _init_distributed(config)
    if log:
        init_logger(config)
    logger = getLogger()
    if int(os.environ.get("RANK", "0")) != 0:  # one log per job: rank 0's
        logger.setLevel("WARNING")
    logger.info("██Server: \t" + platform.node())
    logger.info("██Dir: \t" + os.getcwd() + "\n")
    logger.info(config)
    ds = RecDataset(config)
    logger.info(str(ds))
    train_ds, valid_ds, test_ds = ds.split()
    logger.info("\n====Training====\n" + str(train_ds))
    logger.info("\n====Validation====\n" + str(valid_ds))
    logger.info("\n====Testing====\n" + str(test_ds))
    train_data = TrainDataLoader(config, train_ds, batch_size=config["train_batch_size"], shuffle=True)
    valid_data = EvalDataLoader(config, valid_ds, additional_dataset=train_ds, batch_size=config["eval_batch_size"])
    test_data = EvalDataLoader(config, test_ds, additional_dataset=train_ds, batch_size=config["eval_batch_size"])
    results = []
    val_metric = config["valid_metric"].lower()
    best_value, best_idx = 0.0, 0
    grid = list(config["hyper_parameters"])
    if "seed" not in grid:
        grid = ["seed"] + grid
        config["hyper_parameters"] = grid
    combos = list(product(*[config[k] or [None] for k in grid]))
    for idx, combo in enumerate(combos):
        for k, v in zip(grid, combo):
            config[k] = v
        init_seed(config["seed"])
        logger.info("========={}/{}: Parameters:{}={}=======".format(idx + 1, len(combos), grid, combo))
        train_data.pretrain_setup()
        mdl = get_model(config["model"])(config, train_data).to(config["device"])
        logger.info(mdl)
        trainer = get_trainer()(config, mdl, mg)
        _, best_valid, best_test = trainer.fit(train_data, valid_data=valid_data, test_data=test_data,
                                               saved=save_model)
        results.append((combo, best_valid, best_test))
        if best_test[val_metric] > best_value:
            best_value, best_idx = best_test[val_metric], idx
        logger.info("best valid result: {}".format(dict2str(best_valid)))
        logger.info("test result: {}".format(dict2str(best_test)))
        logger.info("████Current BEST████:\nParameters: {}={},\nValid: {},\nTest: {}\n\n\n".format(
            grid, results[best_idx][0], dict2str(results[best_idx][1]), dict2str(results[best_idx][2])))
    logger.info("\n============All Over=====================")
    for p, v, t in results:
        logger.info("Parameters: {}={},\n best valid: {},\n best test: {}".format(grid, p, dict2str(v), dict2str(t)))
    logger.info("\n\n█████████████ BEST ████████████████")
    logger.info("\tParameters: {}={},\nValid: {},\nTest: {}\n\n".format(
        grid, results[best_idx][0], dict2str(results[best_idx][1]), dict2str(results[best_idx][2])))
    return results
