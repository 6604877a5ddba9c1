"""VERDICT r05 item 4, second harness: the sequence of tests/test_gpu_dist.py::_order_worker
(one rank over the poisoning latency-injected communicator, the sparse step's
combinations of owner-Adam placement / deferred all-gather / graph replay, one engine and
communicator after another in one process), restricted to COMBOS, with the captured
collectives on the greatest-priority stream (PRIO 1, RSX_COMM_CAPTURE_PRIORITY) or on the
default-priority capture stream (PRIO 0, the round-5 fix).

python tools/gpu/diag_priority2.py PRIO a0d0g1,a0d1g0,...   (a: RSX_SHARDED_COMM_ADAM,
d: RSX_SHARDED_DEFER_AG, g: graph replay)"""
import os
import sys
import tempfile

prio, combos = sys.argv[1], sys.argv[2].split(",")
os.environ.update(RSX_COMM_SIM="4:1.0:100", RSX_COMM_SIM_OPT_IN="1", RSX_COMM_SIM_POISON="1",
                  RSX_COMM_PRIORITY="1", RSX_COMM_CAPTURE_PRIORITY=prio)
os.environ.pop("RSX_COMM_SIM_SHARE", None)
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "recommendar-systems_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

torch.cuda.set_device(0)
store = os.path.join(tempfile.mkdtemp(prefix="rsx_diag_"), "store")
dist.init_process_group("nccl", init_method="file://" + store, rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
from rsx.dist import ShardedLightGCNEngine  # noqa: E402
from test_dist_gloo import D, K, LR, NI, NU, REG  # noqa: E402
from test_gpu_dist import _hub_batches, _hub_graph  # noqa: E402

torch.manual_seed(7)
I0 = torch.nn.init.xavier_uniform_(torch.empty(NI, D)).numpy()
U0 = torch.nn.init.xavier_uniform_(torch.empty(NU, D)).numpy()
tu, ti = _hub_graph()
batches = [torch.from_numpy(b).cuda() for b in _hub_batches(tu, ti)]
for c in combos:
    a, d, g = int(c[1]), int(c[3]), int(c[5])
    os.environ["RSX_SHARDED_COMM_ADAM"] = str(a)
    os.environ["RSX_SHARDED_DEFER_AG"] = str(d)
    eng = ShardedLightGCNEngine(tu, ti, NU, NI, D, K, REG, LR, "cuda:0", U0, I0, batch=16, sparse=True)
    eng.use_graph = bool(g)
    for i, t in enumerate(batches):
        eng.step(triplets=t)
        torch.cuda.synchronize()
        print(f"{c} step {i} ok (graphs {sorted(eng._graphs)})", flush=True)
    eng.flush()
    torch.cuda.synchronize()
    print(f"{c} done finite={bool(np.isfinite(eng.p.cpu().numpy()).all())} err={int(eng.err.item())}", flush=True)
    eng.close()
dist.destroy_process_group()
print("all done", flush=True)
