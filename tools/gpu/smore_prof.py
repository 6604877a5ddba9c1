"""torch.profiler breakdown of the C3 SMORE training step (op names + input shapes)."""
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "recommendar-systems_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rsx import synth  # noqa: E402
from rsx.config import Config  # noqa: E402
from rsx.data import RecDataset, TrainDataLoader  # noqa: E402
from rsx.trainer import Trainer  # noqa: E402
from rsx.utils import get_model, init_seed  # noqa: E402

root = tempfile.mkdtemp()
df = synth.shaped("baby", seed=0)
synth.write_inter(df, root, "baby")
ni = int(df.itemID.max()) + 1
np.save(os.path.join(root, "baby", "image_feat_raw.npy"), synth.features(ni, 4096, 1))
np.save(os.path.join(root, "baby", "text_feat_raw.npy"), synth.features(ni, 384, 2))
c = Config("SMORE", "baby", dict(data_path=root + "/", rsx_sampler="device", is_multimodal_model=True, mg_verbose=False,
                                  diag_spectrum=False, diag_gate=False, diag_grad=False))
for k in c["hyper_parameters"]:
    if isinstance(c[k], list):
        c[k] = c[k][0]
init_seed(c["seed"])
ds = RecDataset(c)
tr, va, te = ds.split()
for x in (ds, tr, va, te):
    str(x)
train = TrainDataLoader(c, tr, batch_size=2048, shuffle=True)
train.pretrain_setup()
m = get_model("SMORE")(c, train)
t = Trainer(c, m)
m.train()
m.pre_epoch_processing()
it = iter(train)
for i in range(5):
    t._train_batch(next(it), i, m.calculate_loss)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(10):
    t._train_batch(next(it), 5 + i, m.calculate_loss)
torch.cuda.synchronize()
print(f"ms/step {1e3 * (time.perf_counter() - t0) / 10:.2f}", flush=True)
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    for i in range(5):
        t._train_batch(next(it), 20 + i, m.calculate_loss)
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=40, max_name_column_width=50,
                                                         max_shapes_column_width=70))
