"""VERDICT r05 item 4, third harness: the pattern of tests/test_gpu_dist.py::_sim_worker, the
test that segfaulted in round 5 (profiles/r05/order/pytest_dist_priority_capture_segfault.txt):
the one-rank sharded engine drawing its own batches (eager, eager, captured, replayed x 5),
first over the real one-rank RCCL communicator, then over the latency-injected one, with
captured collectives on the greatest-priority stream (PRIO 1) or the default-priority
capture stream (PRIO 0).

python tools/gpu/diag_priority3.py PRIO real,sim [CLOSE]   (any sequence of `real` / `sim`;
CLOSE: `plain` = engine.close(), `drain` = drop the graphs, gc, synchronize and wait 1 s before
the communicator is destroyed, `leak` = never destroy it)"""
import os
import sys
import ctypes
import gc
import tempfile
import time

prio, seq = sys.argv[1], sys.argv[2].split(",")
close_mode = sys.argv[3] if len(sys.argv) > 3 else "plain"
os.environ.update(RSX_COMM_SIM_OPT_IN="1", RSX_COMM_CAPTURE_PRIORITY=prio)
for k in ("RSX_COMM_SIM", "RSX_COMM_SIM_POISON", "RSX_COMM_SIM_SHARE", "RSX_SHARDED_COMM_ADAM", "RSX_SHARDED_DEFER_AG"):
    os.environ.pop(k, None)
HERE = os.path.dirname(os.path.abspath(__file__))
if os.environ.get("RSX_DIAG_SEGV_BT") == "1":  # native backtrace of a segfault (tools/gpu/exp/segv_bt.c)
    ctypes.CDLL(os.path.join(HERE, "exp", "segv_bt.so"))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "recommendar-systems_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

torch.cuda.set_device(0)
store = os.path.join(tempfile.mkdtemp(prefix="rsx_diag_"), "store")
dist.init_process_group("nccl", init_method="file://" + store, rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
from rsx.dist import ShardedLightGCNEngine  # noqa: E402
from test_dist_gloo import D, K, LR, NI, NU, REG  # noqa: E402
from test_gpu_dist import _local_graph  # noqa: E402

torch.manual_seed(7)
I0 = torch.nn.init.xavier_uniform_(torch.empty(NI, D)).numpy()
U0 = torch.nn.init.xavier_uniform_(torch.empty(NU, D)).numpy()
tu, ti, trip = _local_graph(0)
for j, what in enumerate(seq):
    if what == "sim":
        os.environ["RSX_COMM_SIM"] = "4:1.0:200"
    else:
        os.environ.pop("RSX_COMM_SIM", None)
    eng = ShardedLightGCNEngine(tu, ti, NU, NI, D, K, REG, LR, "cuda:0", U0, I0, batch=16, sparse=True)
    print(f"[{j}] {what}: sim={eng.sim is not None}", flush=True)
    for s in range(0, 8 * 16, 16):
        eng.step(epoch=0, start=s)
        torch.cuda.synchronize()
        print(f"[{j}] {what} step {s // 16} ok (graphs {sorted(eng._graphs)})", flush=True)
    eng.flush()
    torch.cuda.synchronize()
    if close_mode == "plain":
        eng.close()
    else:
        eng._graphs = {}
        gc.collect()
        torch.cuda.synchronize()
        if close_mode == "drain":
            time.sleep(1.0)
            eng.close()
        else:
            eng._comm = None  # leaked: the captured collectives' communicator stays alive
    print(f"[{j}] {what} closed ({close_mode})", flush=True)
dist.destroy_process_group()
print("all done", flush=True)
