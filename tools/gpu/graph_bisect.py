"""Capture pieces of the SMORE training batch in HIP graphs one at a time (debug)."""
import os
import shutil
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "recommendar-systems_amd"))
from rsx import ops  # noqa: E402
from rsx.config import Config  # noqa: E402
from rsx.data import RecDataset, TrainDataLoader  # noqa: E402
from rsx.smore import SMORE  # noqa: E402
from rsx.trainer import Trainer  # noqa: E402
from rsx.utils import init_seed  # noqa: E402

z = np.load(os.path.join(ROOT, "tests/golden/smore_small.npz"))
tmp = tempfile.mkdtemp()
d = os.path.join(tmp, "baby")
os.makedirs(d)
shutil.copy(os.path.join(ROOT, "tests/golden/gold_small.inter"), os.path.join(d, "baby.inter"))
np.save(os.path.join(d, "image_feat_raw.npy"), z["v_feat"])
np.save(os.path.join(d, "text_feat_raw.npy"), z["t_feat"])
c = Config("SMORE", "baby", dict(data_path=tmp + "/", train_batch_size=512, eval_batch_size=256, rsx_sampler="host",
                                  is_multimodal_model=True, dropout_rate=[0.0], mg_verbose=False, image_knn_k=[10],
                                  text_knn_k=[8], rsx_graph_step=False))
for k in c["hyper_parameters"]:
    if isinstance(c[k], list):
        c[k] = c[k][0]
ds = RecDataset(c)
tr, va, te = ds.split()
train = TrainDataLoader(c, tr, batch_size=512, shuffle=True)
init_seed(c["seed"])
train.pretrain_setup()
m = SMORE(c, train)
if sys.argv[1:] == ["trainer"]:
    c["rsx_graph_step"] = True
    t = Trainer(c, m)
    m.pre_epoch_processing()
    print("epoch", t._train_epoch(train, 0), t._graph.replays, flush=True)
    sys.exit(0)
t = Trainer(c, m)
batch = next(iter(train))
for _ in range(4):
    t._train_batch(batch, 0, m.calculate_loss)
torch.cuda.synchronize()
x = m.item_id_embedding.weight.detach().clone()
ego = torch.cat([m.user_embedding.weight, m.item_id_embedding.weight]).detach().clone()


def cap(name, fn):
    print("capture", name, flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    print("  ok", name, flush=True)


from rsx.smore import _prop_mean  # noqa: E402

only = sys.argv[1:] or None
steps = [
    ("matmul", lambda: x @ x.t()[:, :64]),
    ("spmm_item_graph", lambda: m.image_graph.A.spmm(x)),
    ("prop_mean", lambda: _prop_mean(m.norm_adj_csr, ego, m.n_ui_layers)),
    ("linear_wgrad", lambda: ops.linear_wgrad(x, x)),
    ("forward", lambda: m._forward_all(train=True)),
    ("loss", lambda: m.calculate_loss(batch)),
    ("loss_backward", lambda: m.calculate_loss(batch).backward()),
    ("optimizer", lambda: t.optimizer.step()),
    ("train_batch", lambda: t._train_batch(batch, 0, m.calculate_loss)),
]
for name, fn in steps:
    if only and name not in only:
        continue
    cap(name, fn)
print("done", flush=True)
