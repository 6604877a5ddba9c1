"""The multi-rank SMORE step (users-sharded and data-parallel) captured as a HIP graph
over the latency-injected communicator (rsx_comm_init_sim, RSX_COMM_SIM=W): this one process is rank 0 of a
modelled W-rank job, every collective is the one-rank identity plus a comm-stream
stand-in holding the modelled time, and with RSX_COMM_SIM_POISON=1 the stand-in fills
the collective's buffer with NaN for that time before restoring it.

This is the configuration of the round-5 capture fault (a segfault in
torch.cuda.graph.capture_end at rsx/trainer.py's _capture, for the sharded SMORE over
the injected communicator: a fork from a torch side stream that had joined the capture,
DESIGN.md §6): the test pins its fix.  Two epochs (plain and mirror-gradient batches,
each run eagerly once, then captured and replayed) must equal the same epochs issued
eagerly, to the tolerance of tests/test_gpu_smore.py's graph-vs-eager test; a step that
read a collective's buffer inside its modelled window would read the poison and turn
the loss NaN.

The oracle is not the comparator here: under latency injection the modelled peers
contribute nothing (their all-reduce terms are the identity's), so no single-process
SMORE computes the same numbers.  The sharded arithmetic itself is checked against
oracle/rsx_oracle.py:SMORECPU with real ranks in tests/test_gpu_smore_dist.py and
tests/test_smore_dist_gloo.py."""
import numpy as np
import pytest
import torch

import test_gpu_smore as T

pytestmark = pytest.mark.gpu


def _run(tmp_path, golden, graph, scheme):
    from rsx.trainer import Trainer

    z, c, train, valid, test = T._setup(tmp_path, golden)
    c["rsx_sharded"] = True
    c["rsx_sampler"] = "device"  # the sharded model samples its own users on the device
    c["rsx_knn"] = "host"
    c["train_batch_size"] = 64  # several steps per epoch on rank 0's 1/W of the fixture
    c["rsx_graph_step"] = graph
    c["rsx_smore_scheme"] = scheme
    m = T._model(c, train)
    assert m.sharded and m.scheme == scheme and m.comm.sim is not None and m.supports_graph_step
    t = Trainer(c, m)
    losses, replays = [], 0
    try:
        for ep in range(2):
            m.pre_epoch_processing()
            loss, _ = t._train_epoch(train, ep)
            losses.append(float(loss))
            replays += t._graph.replays if t._graph is not None else 0
        torch.cuda.synchronize()
        st = [t.optimizer.state[p] for p in m.parameters()]
        return dict(losses=losses, replays=replays, step=m.global_step, steps=m.steps_per_epoch,
                    p={n: p.detach().cpu().numpy() for n, p in m.named_parameters()},
                    m=[s["exp_avg"].cpu().numpy() for s in st], v=[s["exp_avg_sq"].cpu().numpy() for s in st])
    finally:
        m.comm.close()


@pytest.mark.parametrize("world,scheme", [(2, "usershard"), (4, "usershard"), (2, "dp"), (4, "dp")])
def test_sharded_smore_sim_graph_replay_equals_eager(tmp_path, golden, monkeypatch, world, scheme):
    monkeypatch.setenv("RSX_COMM_SIM", f"{world}:1.0:100")  # 1 GB/s, 100 us: wide poison windows
    monkeypatch.setenv("RSX_COMM_SIM_OPT_IN", "1")
    monkeypatch.setenv("RSX_COMM_SIM_POISON", "1")
    eager = _run(tmp_path / "eager", golden, False, scheme)
    graph = _run(tmp_path / "graph", golden, True, scheme)
    assert eager["steps"] >= 4 and eager["replays"] == 0 and graph["replays"] >= 2 * eager["steps"] - 4
    assert graph["step"] == eager["step"]
    assert np.isfinite(eager["losses"]).all() and np.isfinite(graph["losses"]).all()
    np.testing.assert_allclose(graph["losses"], eager["losses"], rtol=1e-5)
    for k in eager["p"]:
        assert np.isfinite(graph["p"][k]).all(), k
        np.testing.assert_allclose(graph["p"][k], eager["p"][k], rtol=0, atol=1e-4, err_msg=k)
    for a, b in zip(graph["m"] + graph["v"], eager["m"] + eager["v"]):
        np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-7)
