"""Interaction data and batch feeders with the reference's surface.

RecDataset mirrors src/utils/dataset.py (TSV `.inter` with user / item / split
label columns, `item_num = max(itemID) + 1`, split by label, cold users dropped
from valid/test).  TrainDataLoader mirrors src/utils/dataloader.py's training
loader: int64 [3, B] (user, positive, negative) batches on the model device.
Two samplers:

* ``rsx_sampler: host`` — the reference's exact random stream: pandas
  `df.sample(frac=1)` shuffle per epoch (numpy global RNG) and one
  `random.sample(all_items, 1)` draw per negative with redraws while the item is
  in the user's history (dataloader.py:226-275,307-309).  Same seeds, same
  triplets as the reference: the parity mode.
* ``rsx_sampler: device`` — one HIP launch per epoch samples every batch
  (rsx_sample_epoch): the throughput mode.

EvalDataLoader mirrors the evaluation loader (`[users, mask]` batches,
dataloader.py:330-416) and additionally exposes the per-user training CSR used
by the fused full-sort kernel.
"""
from __future__ import annotations

import math
import os
import random
from logging import getLogger

import numpy as np
import pandas as pd
import torch
from scipy.sparse import coo_matrix

from . import graph


class RecDataset:
    def __init__(self, config, df: pd.DataFrame | None = None):
        self.config = config
        self.logger = getLogger()
        self.dataset_name = config["dataset"]
        self.dataset_path = os.path.abspath((config["data_path"] or "") + self.dataset_name)
        self.uid_field = config["USER_ID_FIELD"]
        self.iid_field = config["ITEM_ID_FIELD"]
        self.splitting_label = config["inter_splitting_label"]
        if df is not None:
            self.df = df
            return
        path = os.path.join(self.dataset_path, config["inter_file_name"])
        if not os.path.isfile(path):
            raise ValueError(f"File {path} not exist")
        cols = [self.uid_field, self.iid_field, self.splitting_label]
        self.df = pd.read_csv(path, usecols=cols, sep=config["field_separator"])
        if not self.df.columns.isin(cols).all():
            raise ValueError(f"File {path} lost some required columns.")
        self.item_num = int(self.df[self.iid_field].max()) + 1
        self.user_num = int(self.df[self.uid_field].max()) + 1

    @classmethod
    def from_frame(cls, config, df: pd.DataFrame):
        """Dataset from an in-memory table (synthetic data), columns renamed to the config's fields."""
        df = df.rename(columns={"userID": config["USER_ID_FIELD"], "itemID": config["ITEM_ID_FIELD"],
                                "x_label": config["inter_splitting_label"]})
        ds = cls(config, df[[config["USER_ID_FIELD"], config["ITEM_ID_FIELD"], config["inter_splitting_label"]]])
        ds.item_num = int(ds.df[ds.iid_field].max()) + 1
        ds.user_num = int(ds.df[ds.uid_field].max()) + 1
        return ds

    def split(self):
        parts = []
        for label in range(3):
            part = self.df[self.df[self.splitting_label] == label].copy()
            part.drop(self.splitting_label, inplace=True, axis=1)
            parts.append(part)
        if self.config["filter_out_cod_start_users"]:
            known = set(parts[0][self.uid_field].values)
            for k in (1, 2):
                cold = ~parts[k][self.uid_field].isin(known)
                parts[k].drop(parts[k].index[cold], inplace=True)
        return [self.copy(p) for p in parts]

    def copy(self, new_df):
        nxt = RecDataset(self.config, new_df)
        nxt.item_num = self.item_num
        nxt.user_num = self.user_num
        return nxt

    def get_user_num(self):
        return self.user_num

    def get_item_num(self):
        return self.item_num

    def shuffle(self):
        self.df = self.df.sample(frac=1, replace=False).reset_index(drop=True)

    def __len__(self):
        return len(self.df)

    def __getitem__(self, idx):
        return self.df.iloc[idx]

    def __str__(self):
        self.inter_num = len(self.df)
        nu = len(pd.unique(self.df[self.uid_field]))
        ni = len(pd.unique(self.df[self.iid_field]))
        lines = [self.dataset_name,
                 f"The number of users: {nu}", f"Average actions of users: {self.inter_num / max(nu, 1)}",
                 f"The number of items: {ni}", f"Average actions of items: {self.inter_num / max(ni, 1)}",
                 f"The number of inters: {self.inter_num}"]
        if nu and ni:
            lines.append(f"The sparsity of the dataset: {(1 - self.inter_num / nu / ni) * 100}%")
        return "\n".join(lines)

    __repr__ = __str__


class _Loader:
    def __init__(self, config, dataset, batch_size=1, shuffle=False):
        self.config = config
        self.logger = getLogger()
        self.dataset = dataset
        self.dataset_bk = dataset.copy(dataset.df)
        self.batch_size = self.step = batch_size
        self.shuffle = shuffle
        self.device = config["device"]
        self.inter_num = len(dataset.df)
        self.pr = 0
        self.inter_pr = 0

    def __len__(self):
        return math.ceil(self.pr_end / self.step)

    def __iter__(self):
        if self.shuffle:
            self._shuffle()
        return self

    def __next__(self):
        if self.pr >= self.pr_end:
            self.pr = 0
            self.inter_pr = 0
            raise StopIteration()
        return self._next_batch_data()

    def pretrain_setup(self):
        pass


class TrainDataLoader(_Loader):
    """Training batches: LongTensor [3, B] = (user, positive item, negative item) on the device."""

    def __init__(self, config, dataset, batch_size=1, shuffle=False):
        super().__init__(config, dataset, batch_size, shuffle)
        df = dataset.df
        self.all_items = df[dataset.iid_field].unique().tolist()
        self.all_uids = df[dataset.uid_field].unique()
        self.all_item_len = len(self.all_items)
        self.sampler_kind = (config.get("rsx_sampler", "device") or "device").lower()
        if torch.device(self.device).type == "cpu":  # the CPU configuration: the reference's own host stream
            self.sampler_kind = "host"
        self.history_items_per_u = {u: set(g.values) for u, g in df.groupby(dataset.uid_field)[dataset.iid_field]}
        self._dev_sampler = None
        self._epoch = -1
        self._epoch_buf = None

    # -- reference surface ---------------------------------------------------
    def pretrain_setup(self):
        if self.shuffle:
            self.dataset = self.dataset_bk.copy(self.dataset_bk.df)
        self.all_items.sort()
        random.shuffle(self.all_items)

    def inter_matrix(self, form="coo", value_field=None):
        df = self.dataset.df
        src = df[self.dataset.uid_field].values
        tgt = df[self.dataset.iid_field].values
        data = np.ones(len(df)) if value_field is None else df[value_field].values
        mat = coo_matrix((data, (src, tgt)), shape=(self.dataset.user_num, self.dataset.item_num))
        if form == "coo":
            return mat
        if form == "csr":
            return mat.tocsr()
        raise NotImplementedError(f"sparse matrix format [{form}] has not been implemented.")

    @property
    def pr_end(self):
        return len(self.dataset)

    def train_arrays(self):
        df = self.dataset_bk.df
        return (df[self.dataset.uid_field].values.astype(np.int64), df[self.dataset.iid_field].values.astype(np.int64))

    # -- sampling ------------------------------------------------------------
    def _shuffle(self):
        if self.sampler_kind == "host":
            self.dataset.shuffle()
        else:
            self._epoch += 1
            self._epoch_buf = None

    def _next_batch_data(self):
        if self.sampler_kind == "host":
            return self._host_batch()
        return self._device_batch()

    def _host_batch(self):
        """Reference stream: slice of the shuffled table + Python rejection negatives."""
        part = self.dataset.df.iloc[self.pr: self.pr + self.step]
        self.pr += self.step
        users = part[self.dataset.uid_field].values
        items = part[self.dataset.iid_field].values
        negs = []
        for u in users:
            x = random.sample(self.all_items, 1)[0]
            while x in self.history_items_per_u[u]:
                x = random.sample(self.all_items, 1)[0]
            negs.append(x)
        batch = np.vstack([users, items, np.asarray(negs, dtype=np.int64)]).astype(np.int64)
        return torch.from_numpy(batch).to(self.device)

    def _device_batch(self):
        from . import ops

        if self._dev_sampler is None:
            tu, ti = self.train_arrays()
            seed = int(self.config["seed"] or 0)
            self._dev_sampler = ops.DeviceSampler(tu, ti, self.dataset.user_num, self.device, seed=seed)
        s = self._dev_sampler
        if self._epoch < 0:
            self._epoch = 0
        if self._epoch_buf is None:
            self._epoch_buf = s.sample_epoch(self._epoch, self.step, out=None)
        j = self.pr // self.step
        self.pr += self.step
        return ops.DeviceSampler.batch_view(self._epoch_buf, s.n_inter, self.step, j)


class EvalDataLoader(_Loader):
    """Evaluation batches `[users, mask]` (mask = [2, M] batch-row / train-item pairs)."""

    def __init__(self, config, dataset, additional_dataset=None, batch_size=1, shuffle=False):
        super().__init__(config, dataset, batch_size, shuffle)
        if additional_dataset is None:
            raise ValueError("Training datasets is nan")
        self.additional_dataset = additional_dataset
        self.eval_items_per_u = []
        self.eval_len_list = []
        self.train_pos_len_list = []
        eval_u = dataset.df[dataset.uid_field].unique()
        tr = additional_dataset.df.groupby(additional_dataset.uid_field)[additional_dataset.iid_field]
        rows, cols = [], []
        for k, u in enumerate(eval_u):
            its = tr.get_group(u).values
            self.train_pos_len_list.append(len(its))
            rows.append(np.full(len(its), k, dtype=np.int64))
            cols.append(its.astype(np.int64))
        self.pos_items_per_u = torch.from_numpy(
            np.vstack([np.concatenate(rows) if rows else np.zeros(0, np.int64),
                       np.concatenate(cols) if cols else np.zeros(0, np.int64)])).to(self.device)
        ev = dataset.df.groupby(dataset.uid_field)[dataset.iid_field]
        for u in eval_u:
            its = ev.get_group(u).values
            self.eval_len_list.append(len(its))
            self.eval_items_per_u.append(its)
        self.eval_len_list = np.asarray(self.eval_len_list)
        self.eval_u = torch.from_numpy(eval_u.astype(np.int64)).to(self.device)
        # training history CSR over user ids (fused full-sort mask), built once
        tdf = additional_dataset.df
        rp, col = graph.history_csr(tdf[additional_dataset.uid_field].values, tdf[additional_dataset.iid_field].values,
                                    dataset.user_num)
        self.mask_rowptr = torch.from_numpy(rp).to(self.device)
        self.mask_col = torch.from_numpy(col).to(self.device)

    @property
    def pr_end(self):
        return self.eval_u.shape[0]

    def _shuffle(self):
        self.dataset.shuffle()

    def _next_batch_data(self):
        cnt = sum(self.train_pos_len_list[self.pr: self.pr + self.step])
        users = self.eval_u[self.pr: self.pr + self.step]
        mask = self.pos_items_per_u[:, self.inter_pr: self.inter_pr + cnt].clone()
        mask[0] -= self.pr
        self.inter_pr += cnt
        self.pr += self.step
        return [users, mask]

    def eval_csr(self):
        """Held-out items per evaluation user as a device CSR, sorted within each user
        (rsx_topk_metrics' binary search); built on first use."""
        if getattr(self, "_eval_csr", None) is None:
            lens = np.asarray(self.eval_len_list, dtype=np.int64)
            rp = np.zeros(lens.size + 1, dtype=np.int64)
            np.cumsum(lens, out=rp[1:])
            col = (np.concatenate([np.sort(np.asarray(x, dtype=np.int64)) for x in self.eval_items_per_u])
                   if len(self.eval_items_per_u) else np.zeros(0, np.int64)).astype(np.int32)
            self._eval_csr = (torch.from_numpy(rp).to(self.device), torch.from_numpy(col).to(self.device))
        return self._eval_csr

    def get_eval_items(self):
        return self.eval_items_per_u

    def get_eval_len_list(self):
        return self.eval_len_list

    def get_eval_users(self):
        return self.eval_u.cpu()
