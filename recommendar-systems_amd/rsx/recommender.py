"""The plugin API models implement — same surface as the reference's
AbstractRecommender / GeneralRecommender (src/common/abstract_recommender.py:10-103).

A model is constructed as `Cls(config, dataloader)`; the trainer calls
`parameters()`, `train()/eval()`, `pre_epoch_processing()`,
`post_epoch_processing()`, `calculate_loss(interaction)` and
`full_sort_predict([users, mask])`.  rsx models add two optional fast paths the
rsx Trainer uses when present:

* `fused_step(interaction, lr)` — the whole batch (forward, loss, backward,
  Adam) on the device, loss accumulated on the device (no host sync);
* `full_sort_topk(batch, k, eval_data)` — scores, train-item mask and top-k
  fused in one kernel, never materialising the score matrix.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn as nn


class AbstractRecommender(nn.Module):
    supports_fused_step = False

    def pre_epoch_processing(self):
        pass

    def post_epoch_processing(self):
        pass

    def calculate_loss(self, interaction):
        raise NotImplementedError

    def predict(self, interaction):
        raise NotImplementedError

    def full_sort_predict(self, interaction):
        raise NotImplementedError

    def __str__(self):
        n = sum(int(np.prod(p.size())) for p in self.parameters())
        return super().__str__() + f"\nTrainable parameters: {n}"


class GeneralRecommender(AbstractRecommender):
    def __init__(self, config, dataloader):
        super().__init__()
        self.USER_ID = config["USER_ID_FIELD"]
        self.ITEM_ID = config["ITEM_ID_FIELD"]
        self.NEG_ITEM_ID = (config["NEG_PREFIX"] or "neg__") + str(self.ITEM_ID)
        self.n_users = dataloader.dataset.get_user_num()
        self.n_items = dataloader.dataset.get_item_num()
        self.batch_size = config["train_batch_size"]
        self.device = config["device"]
        self.v_feat, self.t_feat = None, None
        if not config["end2end"] and config["is_multimodal_model"]:
            root = os.path.abspath((config["data_path"] or "") + config["dataset"])
            vf = os.path.join(root, config["vision_feature_file"] or "")
            tf = os.path.join(root, config["text_feature_file"] or "")
            if os.path.isfile(vf):
                self.v_feat = torch.from_numpy(np.load(vf)).type(torch.FloatTensor).to(self.device)
            if os.path.isfile(tf):
                self.t_feat = torch.from_numpy(np.load(tf)).type(torch.FloatTensor).to(self.device)
            assert self.v_feat is not None or self.t_feat is not None, "Features all NONE"
