#!/usr/bin/env python3
"""Headline benchmark: LightGCN BPR interactions/s (+ full-sort items/s) on MI355X.

Metric (BASELINE.json): "BPR interactions/sec + full-sort items/sec, LightGCN d=64
at 1/2/4/8 MI355X".  Workload at N=1 = configs[1]: LightGCN K=3 d=64 on an
Amazon-sports-shaped synthetic graph (35,598 users, 18,357 items, ~296k
interactions, the reference's split rule; no datasets offline), B=2048.

A step = one training batch end to end on the device: triplet sampling
(shuffle + rejection negatives), 3-layer propagation, BPR loss + backward,
Horner backward propagation, Adam — one `rsx_lightgcn_step` C-ABI call.

N>1 (one process per GPU, torchrun or `--gpus N`): by default the metric's d = 64
LightGCN on the fixed 10M-user graph (`--workload c4 --dim 64`), users row-sharded
over the ranks (rsx.dist / csrc/dist.hip), the global batch of 2048 split
over them: strong scaling, the ranks divide the graph.  Its one-GPU anchor is
`--workload c4 --dim 64 --gpus 1` (the N=1 default stays C2).  The sports graph does
not divide profitably: `--workload c2 --dist rowshard` (every rank its own sports
block, item partials all-reduced per layer) and `--workload c2 --dist dp` (graph and
tables replicated, one triplet all-gather, every rank evaluating the whole global
batch) both lose to one GPU at the same global batch (`--batch N*2048`).
value = all ranks' interactions / max-over-ranks time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "recommendar-systems_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "BPR interactions/sec + full-sort items/sec, LightGCN d=64 at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def spmm_bytes(n_rows, nnz, d):
    """S_spmm = 4(N+1) + 8 nnz + 8 N d (each operand once, Y written once)."""
    return 4 * (n_rows + 1) + 8 * nnz + 8 * n_rows * d


def time_kernel(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps  # ms


def time_graph(fn, reps, stream=None):
    """time_kernel for a multi-launch host sequence: fn captured once as a HIP graph and
    replayed, so the figure is the launches' device time (as in the graph-replayed
    training step), not the host's issue rate of an eager torch.autograd sequence.
    `stream`: the capture stream -- for a torch.autograd backward it must be the stream its
    forward ran on (autograd issues each backward op on its forward op's stream)."""
    with torch.cuda.stream(stream) if stream is not None else torch.cuda.stream(torch.cuda.current_stream()):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def _oracle():
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import rsx_oracle as O

    return O


def _timed_loop(step, budget_s, min_steps=3, max_steps=200):
    """Run step() until budget_s has elapsed (at least min_steps); returns (steps, seconds)."""
    t0 = time.perf_counter()
    steps = 0
    while True:
        step()
        steps += 1
        el = time.perf_counter() - t0
        if (el > budget_s and steps >= min_steps) or steps >= max_steps:
            return steps, el


def cpu_baseline(df_train, nu, ni, budget_s=12.0, d=64, shape="sports", scale=1, K=3):
    """Reference-identical CPU LightGCN (oracle restatement) on this host's cores:
    Python negative sampler + torch.sparse.mm propagation + autograd + Adam.  With
    scale > 1 the graph is a 1/scale slice and the rate is divided by scale."""
    O = _oracle()
    tu, ti = df_train
    A = O.lightgcn_norm_adj_vec(tu, ti, nu, ni)
    torch.manual_seed(999)
    U0 = torch.nn.init.xavier_uniform_(torch.empty(nu, d)).numpy()
    I0 = torch.nn.init.xavier_uniform_(torch.empty(ni, d)).numpy()
    cpu = O.LightGCNCPU(A, U0, I0, K, 1e-2)
    smp = O.ReferenceSampler(tu, ti)
    if scale == 1:
        cpu.step(smp.next(2048))  # warm
    steps, el = _timed_loop(lambda: cpu.step(smp.next(2048)), budget_s, min_steps=1 if scale > 1 else 3)
    what = (f"{steps} LightGCN K={K} d={d} B=2048 steps on the same {shape}-shaped graph" if scale == 1 else
            f"{steps} LightGCN K={K} d={d} B=2048 step(s) on a 1/{scale} user slice ({nu:,} users x {ni:,} items, "
            f"{len(tu):,} train interactions), rate divided by {scale}")
    return {"value": steps * 2048 / el / scale, "unit": "interactions/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{what} ({el:.1f} s; Python sampler + torch.sparse.mm + autograd + Adam, oracle/rsx_oracle.py)"}


def cpu_baseline_layergcn(tu, ti, nu, ni, K, reg, dropout, budget_s, batches_per_epoch):
    """oracle.LayerGCNCPU: per-epoch edge dropout (amortised over the epoch's batches) +
    cosine-gated propagation + BPR/L2 + autograd + Adam."""
    O = _oracle()
    torch.manual_seed(999)
    U0 = torch.nn.init.xavier_uniform_(torch.empty(nu, 64)).numpy()
    I0 = torch.nn.init.xavier_uniform_(torch.empty(ni, 64)).numpy()
    cpu = O.LayerGCNCPU(tu, ti, nu, ni, U0, I0, K, reg, dropout)
    smp = O.ReferenceSampler(tu, ti)
    t0 = time.perf_counter()
    cpu.pre_epoch()
    t_pre = time.perf_counter() - t0
    cpu.step(smp.next(2048))
    steps, el = _timed_loop(lambda: cpu.step(smp.next(2048)), budget_s)
    per = el / steps + t_pre / batches_per_epoch
    return {"value": 2048 / per, "unit": "interactions/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{steps} LayerGCN K={K} d=64 B=2048 steps ({el:.1f} s) + one edge-dropout rebuild "
                      f"({t_pre:.2f} s, amortised over {batches_per_epoch} batches) on the same graph "
                      f"(oracle.LayerGCNCPU: torch.sparse.mm + autograd + Adam)"}


def cpu_baseline_smore(tu, ti, nu, ni, v, t, d, image_k, text_k, dropout, budget_s):
    """oracle.SMORECPU + smore_train_batch: the reference's SMORE batch with the
    model-level mirror gradient (3 forward/backward passes, 2 Adam steps per batch
    once it triggers) on this host's cores; the first two (MG-free) batches untimed."""
    O = _oracle()
    torch.manual_seed(999)
    m = O.SMORECPU(tu, ti, nu, ni, v, t, d=d, image_k=image_k, text_k=text_k, dropout=dropout, batch_size=2048)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    smp = O.ReferenceSampler(tu, ti)
    for _ in range(2):
        O.smore_train_batch(m, opt, smp.next(2048), 1e-3)
    steps, el = _timed_loop(lambda: O.smore_train_batch(m, opt, smp.next(2048), 1e-3), budget_s, min_steps=2)
    return {"value": steps * 2048 / el, "unit": "interactions/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{steps} SMORE d={d} B=2048 batches with the mirror gradient ({el:.1f} s) on the same graph "
                      f"and features (oracle.SMORECPU: torch CPU forward/autograd/Adam)"}


MFMA_F32_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: dense f32 MFMA (no xf32 on gfx950)


def _roof_hbm(name, nbytes, ms, note, calls):
    gbs = nbytes / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": name, "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": gbs / HBM_PEAK_GBS, "traffic": None, "algorithmic_bytes_per_launch": nbytes, "avg_launch_ms": ms,
            "launches_per_pass": calls, "note": note}


def _roof_mfma(name, flops, ms, note, calls):
    tfs = flops / (ms * 1e-3) / 1e12
    return {"bound": "mfma", "kernel": name, "achieved": tfs, "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s",
            "frac": tfs / MFMA_F32_PEAK_TFS, "traffic": None, "algorithmic_flops_per_launch": flops,
            "avg_launch_ms": ms, "launches_per_pass": calls, "note": note}


def smore_kernel_rooflines(model, B, d):
    """SMORE's dominant launches per forward/backward pass, each timed alone (HIP events on
    the stream the kernels use; multi-launch sequences captured once and replayed, as the
    training step runs them) on the model's own operands, with its algorithmic work:
      * the three item views' kNN products in one launch (spmm_batch STORE): per view
        4(NI+1) + 8 nnz + 4 NI d (X read once) + 4 NI d (Y written) bytes;
      * the projections' backward (rsx_linear_bwd, one per modality): dW = g^T X and
        dX = g W, 4 NI d dv flop;
      * the preference block's backward on the 3B batch rows (pref_rows bwd + its batched
        weight gradients): 7 Linear(d, d) x (dX + dW) = 28 (3B) d^2 flop;
      * the InfoNCE backward of both terms (nce_bwd): 2 terms x 2 products (d side,
        d content) x 2 B^2 d flop = 8 B^2 d.
    Sorted by their share of a pass (time x launches per pass)."""
    from rsx import _lib as L
    from rsx import ops
    from rsx import smore_fuse as SF

    dev = model.item_id_embedding.weight.device
    ni = model.n_items
    g = torch.Generator(device="cpu").manual_seed(5)
    out = []
    # views: the item-graph layer of the three views, one launch
    Gs = [model.image_graph.A, model.text_graph.A, model.fusion_graph.A]
    xs = [torch.randn(ni, d, generator=g).to(dev) for _ in range(3)]
    ys = [torch.empty(ni, d, device=dev) for _ in range(3)]
    epis = [ops.epi(L.RSX_EPI_STORE, y=y) for y in ys]
    ms = time_kernel(lambda: ops.spmm_batch(Gs, xs, epis, d), 30)
    nbytes = sum(4 * (ni + 1) + 8 * A.nnz + 8 * ni * d for A in Gs)
    out.append(_roof_hbm(f"spmm_batch<{d},STORE> three kNN item-view products (one launch)", nbytes, ms,
                         "kNN graphs and item tables are Infinity-Cache resident at clothing", 2))
    # projection backward, image modality
    V = model.image_embedding.weight.detach()  # this rank's item rows when the item side is sharded
    W = model.image_trs.weight.detach()
    nv = V.shape[0]
    gi = torch.randn(nv, d, generator=g).to(dev)
    ms = time_graph(lambda: ops.linear_bwd(gi, V, W), 20)
    out.append(_roof_mfma(f"rsx_linear_bwd (wgrad_partial<DX>) projection backward {nv}x{V.shape[1]}->{d}",
                          4.0 * nv * d * V.shape[1], ms, "f32 MFMA 32x32x2 (dW) + 16x16x4 (dX)", 2))
    # preference block backward on 3B rows
    nu = model.n_users if not getattr(model, "sharded", False) else model.user_embedding.weight.shape[0]
    n = nu + ni
    tabs = [torch.randn(n, d, generator=g).to(dev).requires_grad_() for _ in range(4)]
    rows = torch.randint(0, n, (3 * B,), generator=g).to(dev)
    seed = torch.zeros(1, dtype=torch.int64, device=dev)
    cs = torch.cuda.Stream(device=dev)  # the forwards run on the capture stream (time_graph)
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        outs = SF.preference_rows(model, *tabs, rows, seed)
        gos = [torch.randn_like(o) for o in outs]

    def pref_bwd():
        torch.autograd.grad(outs, tabs, gos, retain_graph=True)

    ms = time_graph(pref_bwd, 20, cs)
    out.append(_roof_mfma(f"pref_rows<{d}> backward + weight gradients ({3 * B} batch rows)", 28.0 * 3 * B * d * d,
                          ms, "16x16x4 f32 MFMA row tiles; one 16-row tile per wave", 1))
    # InfoNCE backward of both terms (compact rows)
    side = torch.randn(3 * B, d, generator=g).to(dev).requires_grad_()
    cont = torch.randn(3 * B, d, generator=g).to(dev).requires_grad_()
    allc = torch.randn(3 * B, d, generator=g).to(dev).requires_grad_()
    ar = torch.arange(B, device=dev)
    trip = torch.stack([ar, ar, ar + B]).contiguous()
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        tot, _ = SF.smore_loss_rows(allc, side, cont, trip, ar, B, 1e-5, 2048.0, 0.01, 0.2)

    def nce_bwd():
        torch.autograd.grad(tot, [side, cont], retain_graph=True)

    ms = time_graph(nce_bwd, 20, cs)
    out.append(_roof_mfma(f"nce_bwd_t<{d},2> InfoNCE backward, both terms (B = {B})", 8.0 * B * B * d, ms,
                          "f32 MFMA; the forward's exp(S/tau) tiles and transposed row tiles reused", 1))
    out.sort(key=lambda r: -r["avg_launch_ms"] * r["launches_per_pass"])
    return out


WORKLOADS = {
    "c1": dict(model="LayerGCN", dataset="baby", desc="C1: LayerGCN K=2 d=64, baby-shaped (19,445 users x 7,050 items), "
                                                    "B=2048, device sampler, fused step (reference config: CPU)",
               cfg=dict(n_layers=[2], reg_weight=[1e-2], dropout=[0.1])),
    "c3": dict(model="SMORE", dataset="baby", desc="C3: SMORE d=64, baby-shaped, image 4096 / text 384 N(0,1) features, "
                                                 "kNN 20/15, model-level mirror gradient, B=2048, device sampler",
               cfg=dict(mg_verbose=False, diag_spectrum=False, diag_gate=False, diag_grad=False)),
    "c5": dict(model="SMORE", dataset="clothing", desc="C5: SMORE d=128, clothing-shaped (39,387 users x 23,033 items), "
                                                      "CLIP-like L2-normalised 768/768 N(0,1) features, kNN 20/15, "
                                                      "model-level mirror gradient, B=2048, device sampler, 1 GPU",
               cfg=dict(embedding_size=128, mg_verbose=False, diag_spectrum=False, diag_gate=False, diag_grad=False),
               feats=(768, 768, True), feat_files=("image_feat.npy", "text_feat.npy")),
}


def bench_model(args):
    """C1 / C3 / C5 through the drop-in surface (Config -> RecDataset -> loaders -> model ->
    Trainer): a step = one training batch exactly as Trainer runs it.  SMORE (c3, c5) at
    WORLD_SIZE > 1: data-parallel by default (rsx.smore scheme "dp": every table replicated,
    every rank stepping on its own batch, one batch-row gradient all-gather + one weight
    all-reduce per backward over RCCL); RSX_SMORE_SCHEME=usershard: the users-sharded model
    (rsx.smore_dist: one item all-reduce per UI layer)."""
    import tempfile

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        local = _local_device()
        torch.cuda.set_device(local)
        _init_group(local)
    from rsx import synth
    from rsx.config import Config
    from rsx.data import EvalDataLoader, RecDataset, TrainDataLoader
    from rsx.trainer import Trainer
    from rsx.utils import get_model, init_seed

    w = WORKLOADS[args.workload]
    root = tempfile.mkdtemp(prefix="rsx_bench_")
    df = synth.shaped(w["dataset"], seed=0)
    synth.write_inter(df, root, w["dataset"])
    ni = int(df.itemID.max()) + 1
    feats = None
    if w["model"] == "SMORE":
        dv, dt, l2 = w.get("feats", (4096, 384, False))
        fv, ft = w.get("feat_files", ("image_feat_raw.npy", "text_feat_raw.npy"))  # configs/dataset/<name>.yaml
        feats = (synth.features(ni, dv, 1, l2_normalise=l2), synth.features(ni, dt, 2, l2_normalise=l2))
        np.save(os.path.join(root, w["dataset"], fv), feats[0])
        np.save(os.path.join(root, w["dataset"], ft), feats[1])
    cfg = dict(data_path=root + "/", train_batch_size=args.batch, rsx_sampler="device",
               is_multimodal_model=w["model"] == "SMORE", **w["cfg"])
    if w["model"] == "SMORE" and os.environ.get("RSX_SMORE_SCHEME"):
        cfg["rsx_smore_scheme"] = os.environ["RSX_SMORE_SCHEME"]
    from rsx.dist import sim_comm_params

    sim = sim_comm_params() if (world == 1 and w["model"] == "SMORE") else None
    if sim or (w["model"] == "SMORE" and os.environ.get("RSX_BENCH_SHARDED") == "1"):
        # rank 0 of a modelled W-rank job (rsx.smore_dist.Comm's latency injection), or (diagnosis)
        # the multi-rank model on one rank: its exchange work without a collective
        cfg["rsx_sharded"] = True
    if os.environ.get("RSX_BENCH_GRAPH") == "0":  # diagnosis: the model's batches eagerly
        cfg["rsx_graph_step"] = False
    c = Config(w["model"], w["dataset"], cfg)
    if world > 1:
        c["device"] = torch.device("cuda", _local_device())  # (the rehearsal mode puts every rank on GPU 0)
    for k in c["hyper_parameters"]:
        if isinstance(c[k], list):
            c[k] = c[k][0]
    init_seed(c["seed"])
    ds = RecDataset(c)
    tr, va, te = ds.split()
    for x in (ds, tr, va, te):
        str(x)
    train = TrainDataLoader(c, tr, batch_size=args.batch, shuffle=True)
    valid = EvalDataLoader(c, va, additional_dataset=tr, batch_size=c["eval_batch_size"])
    train.pretrain_setup()
    t_build = time.perf_counter()
    model = get_model(w["model"])(c, train)
    build_s = time.perf_counter() - t_build
    t = Trainer(c, model)
    model.train()
    sharded = bool(getattr(model, "sharded", False))
    if sharded:
        t._gate = t._nan_gate_on()  # as Trainer._train_epoch_autograd arms it
        if t._gate:
            t._arm_nan_gate()

    def batches():
        ep = 0
        while True:
            model.pre_epoch_processing()
            t.reset_graph_step()  # as Trainer._train_epoch does at each epoch start
            for b in (model.local_batches(ep) if sharded else train):
                yield b
            ep += 1

    it = batches()
    idx = {"i": 0}

    def one_step():
        b = next(it)
        if t.fused:
            model.fused_step(b, t.current_lr())
        else:
            t.train_step(b, idx["i"], model.calculate_loss)
        idx["i"] += 1
        return b.shape[1]

    # untimed: the requested warm-up, and for a model with per-epoch work (LayerGCN's edge
    # dropout alternates two draws) two whole epochs, so that each kind of epoch rebuild
    # has run once before the timed steps (which still include their own rebuilds)
    n_warm = args.warmup
    if w["model"] == "LayerGCN":
        n_warm = max(n_warm, 2 * len(train) + 1)
    if sharded:
        # a rank's balanced slices come in two sizes: one whole epoch (+ a few) untimed, so every
        # (slice size, batch kind) graph has been captured before the timed steps, as in the
        # one-GPU line, whose single batch size is captured within its warm-up
        n_warm = max(n_warm, int(model.steps_per_epoch) + 6)
    for _ in range(n_warm):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    n = 0
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        n += one_step()
    ev1.record()
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    log(f"[bench] rank {rank}/{world} {w['model']}: {wall * 1e3 / args.steps:.3f} ms/step wall, host issue "
        f"{t_issue * 1e3 / args.steps:.3f} ms/step, events {ev0.elapsed_time(ev1) / args.steps:.3f} ms/step, "
        f"graph replays {getattr(getattr(t, '_graph', None), 'replays', None)}")
    dev = torch.device("cuda", torch.cuda.current_device())
    per_rank = _rank_report(wall, ev0.elapsed_time(ev1), args.steps, world, dev)
    rccl_world = None
    if world > 1:
        tot = torch.tensor([float(n)], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(tot)
        n = float(tot.item())
        wall = max(p["ms_per_step"] for p in per_rank) * args.steps / 1e3
        if getattr(getattr(model, "comm", None), "handle", None) is not None:
            ones = torch.ones(1, dtype=torch.float32, device=dev)
            model.comm.allreduce_(ones)
            rccl_world = int(round(float(ones.item())))
    model.eval()
    t.evaluate(valid)
    torch.cuda.synchronize()
    te0 = time.perf_counter()
    t.evaluate(valid)
    torch.cuda.synchronize()
    eval_s = time.perf_counter() - te0
    n_eval = int(len(valid.get_eval_users()))
    if world > 1:
        ev_t = torch.tensor([eval_s], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(ev_t, op=torch.distributed.ReduceOp.MAX)
        eval_s = float(ev_t.item())

    # roofline: one propagation SpMM (STORE) over the model's training graph, d columns
    d = int(c["embedding_size"])
    if w["model"] == "SMORE":
        A = model.norm_adj_csr
        x = torch.cat([model.user_embedding.weight, model.item_id_embedding.weight]).detach().contiguous()
        if sharded:  # the full graph over a full-size operand (this rank holds its user rows only)
            x = torch.randn(A.n_cols, d, device=x.device)
        kname = f"spmm_main<{d},STORE> UI-graph propagation layer"
    else:
        A = model.engine.train_adj
        x = model.engine.p
        kname = f"spmm_main<{d},STORE> propagation layer (the epoch's edge-dropout graph)"
    y = torch.empty(A.n_rows, d, device=x.device)
    spmm_ms = time_kernel(lambda: A.spmm(x, out=y), 50)
    alg = spmm_bytes(A.n_rows, A.nnz, d)
    roof = {"bound": "hbm", "kernel": kname, "achieved": alg / (spmm_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": alg / (spmm_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
            "algorithmic_bytes_per_launch": alg, "avg_launch_ms": spmm_ms,
            "note": "baby/clothing working sets are Infinity-Cache resident"}
    kernels = [roof]
    if w["model"] == "SMORE":
        # the step's dominant launches (rocprof: profiles/r02/legs/prof_c{3,5}), each timed
        # alone on the model's own operands; the largest-share one is the line's roofline
        kernels = smore_kernel_rooflines(model, args.batch, d) + [roof]
        roof = kernels[0]
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        tr_df = df[df.x_label == 0]
        tu_, ti_ = tr_df.userID.values.astype(np.int64), tr_df.itemID.values.astype(np.int64)
        nu_ = int(df.userID.max()) + 1
        if w["model"] == "SMORE":
            cpu = cpu_baseline_smore(tu_, ti_, nu_, ni, feats[0], feats[1], d, int(c["image_knn_k"]),
                                     int(c["text_knn_k"]), float(c["dropout_rate"]), args.cpu_budget)
        else:
            cpu = cpu_baseline_layergcn(tu_, ti_, nu_, ni, int(c["n_layers"]), float(c["reg_weight"]),
                                        float(c["dropout"]), args.cpu_budget, -(-tu_.size // args.batch))
    out = {
        "metric": METRIC, "value": n / wall, "unit": "interactions/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "warmup_steps_run": n_warm, "ms_per_step": wall * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic Amazon-{w['dataset']}-shaped graph (rsx.synth seed 0)"
                + ("; N(0,1) features" if w["model"] == "SMORE" else ""),
        "config": {"workload": w["desc"], "model": w["model"], "embedding_size": int(c["embedding_size"]),
                   "global_batch": int(getattr(model, "local_batch", args.batch)) * world,
                   "parallelism": f"{getattr(model, 'scheme', None) or 'usershard'}{world}" if sharded else "single",
                   "fused_step": bool(t.fused),
                   "graph_step": t._graph is not None and t._graph.replays > 0},
        "launcher": os.environ.get("RSX_BENCH_LAUNCHER", "torchrun" if world > 1 else "single process"),
        "rccl_world_size": rccl_world, "per_rank": per_rank,
        "fullsort_items_per_s": n_eval * ni / eval_s,
        "fullsort": {"eval_users": n_eval, "n_items": ni, "s_per_eval_incl_forward_and_metrics": eval_s},
        "model_build_s": build_s, "roofline": roof, "roofline_kernels": kernels, "cpu_baseline": cpu,
    }
    if sim:
        Wm = int(sim["world"])
        out["config"]["parallelism"] = f"{model.scheme}{Wm} (latency-injected, rank 0 of {Wm})"
        out["config"]["global_batch"] = int(getattr(model, "local_batch", args.batch)) * Wm
        out["latency_injection"] = dict(
            sim, modelled_job={"world": Wm, "interactions_per_s": Wm * n / wall, "ms_per_step": wall * 1e3 / args.steps},
            note=("value / ms_per_step: rank 0 of the modelled job (" +
                  ("every table replicated, a batch of its own from its 1/W of the users; the batch-row gradient "
                   "all-gather and the preference weights' all-reduce comm-stream stand-ins of the modelled time, "
                   "the peers' packs copies of its own" if model.scheme == "dp" else
                   "its 1/W of the users and item rows, a batch of its own; every collective a comm-stream "
                   "stand-in of the modelled time") +
                  "): the job's rate is world x value; the fullsort figures are this rank's users only"))
    if rank == 0:
        _json_line(out)
    if world > 1 or sim:
        if getattr(model, "comm", None) is not None:
            model.comm.close()
    if world > 1:
        torch.distributed.destroy_process_group()


def bench_c1_cpu(args):
    """BASELINE config C1 as the reference runs it: LayerGCN K=2 d=64 on a baby-shaped graph
    on the CPU (src/models/layergcn.py:127-177, src/common/trainer.py:186-238), through the
    drop-in rsx LayerGCN with use_gpu False -- its steps go through torch.ops.rsx's C++ CPU
    kernels (rsx.cpu_engine, csrc/cpu_ops.cpp): the reference's host sampler, the per-epoch
    edge-dropout rebuild, propagation, BPR, backward, Adam.  Timed as whole epochs (each
    with its rebuild), beside the CPU port of the reference (oracle.LayerGCNCPU: torch
    sparse ops + autograd + torch Adam) on the same graph and the same host threads."""
    import tempfile

    from rsx import synth
    from rsx.config import Config
    from rsx.data import RecDataset, TrainDataLoader
    from rsx.trainer import Trainer
    from rsx.utils import get_model, init_seed

    threads = torch.get_num_threads()
    root = tempfile.mkdtemp(prefix="rsx_bench_c1_")
    df = synth.shaped("baby", seed=0)
    synth.write_inter(df, root, "baby")
    c = Config("LayerGCN", "baby", dict(data_path=root + "/", train_batch_size=args.batch, use_gpu=False,
                                        is_multimodal_model=False, n_layers=[2], reg_weight=[1e-2], dropout=[0.1]))
    for k in c["hyper_parameters"]:
        if isinstance(c[k], list):
            c[k] = c[k][0]
    assert c["device"].type == "cpu"
    init_seed(c["seed"])
    ds = RecDataset(c)
    tr, va, te = ds.split()
    for x in (ds, tr, va, te):
        str(x)
    train = TrainDataLoader(c, tr, batch_size=args.batch, shuffle=True)
    train.pretrain_setup()
    model = get_model("LayerGCN")(c, train)
    t = Trainer(c, model)
    model.train()

    def epoch(ep):
        model.pre_epoch_processing()
        n = 0
        for b in train:
            if t.fused:
                model.fused_step(b, t.current_lr())
            else:
                t.train_step(b, n, model.calculate_loss)
            n += int(b.shape[1])
        return n

    epoch(0)  # untimed: first use of every kernel
    n_ep = max(1, int(args.steps)) if args.steps is not None else 2
    t0 = time.perf_counter()
    n = sum(epoch(1 + e) for e in range(n_ep))
    wall = time.perf_counter() - t0
    cpu = None
    if not args.no_cpu_baseline:
        tr_df = df[df.x_label == 0]
        tu_, ti_ = tr_df.userID.values.astype(np.int64), tr_df.itemID.values.astype(np.int64)
        cpu = cpu_baseline_layergcn(tu_, ti_, int(df.userID.max()) + 1, int(df.itemID.max()) + 1, 2, 1e-2, 0.1,
                                    args.cpu_budget, -(-tu_.size // args.batch))
    out = {"metric": METRIC, "value": n / wall, "unit": "interactions/s", "n_gpus": 0, "device": "cpu",
           "cores": threads, "epochs": n_ep, "s_per_epoch": wall / n_ep, "ms_per_step": wall * 1e3 / (n / args.batch),
           "higher_is_better": True, "vs_baseline": None, "dtype": "f32",
           "data": "synthetic Amazon-baby-shaped graph (rsx.synth seed 0)",
           "config": {"workload": "C1: LayerGCN K=2 d=64, baby-shaped (19,445 users x 7,050 items), B=2048, "
                                  "edge dropout 0.1, on the CPU through torch.ops.rsx's C++ kernels "
                                  "(rsx.cpu_engine, csrc/cpu_ops.cpp); the reference's host sampler",
                      "model": "LayerGCN", "fused_step": bool(t.fused)},
           "includes": "every epoch's edge-dropout rebuild and host triplet sampling",
           "cpu_baseline": cpu,
           "speedup_vs_cpu_port": (n / wall) / cpu["value"] if cpu else None,
           "reference_measured": {"value": 24776, "unit": "interactions/s", "cores": 8,
                                  "source": "SURVEY.md 6: the reference itself on baby, this container"},
           "roofline": None}
    _json_line(out)


def _c4_chunk(args):
    from rsx import synth

    c, cdf = args
    u, i, lab = synth.chunk_graph(c, synth.C4["chunk_users"], synth.C4["n_items"], synth.C4["avg"], cdf)
    return c, u, i, lab


def relabel_graph(df, how):
    """The interaction frame with users and items renumbered (experiment: SpMM gather locality,
    DESIGN §3): "degree" (each side by descending training degree) or "rcm" (reverse
    Cuthill-McKee of the symmetric bipartite graph, users and items each kept in their RCM
    order).  A permutation of rows only: the propagation's values per node are unchanged."""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import reverse_cuthill_mckee

    u = df.userID.values.astype(np.int64)
    i = df.itemID.values.astype(np.int64)
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    tr = df.x_label.values == 0
    if how == "degree":
        ou = np.argsort(-np.bincount(u[tr], minlength=nu), kind="stable")
        oi = np.argsort(-np.bincount(i[tr], minlength=ni), kind="stable")
    elif how == "rcm":
        n = nu + ni
        a = sp.coo_matrix((np.ones(int(tr.sum()), np.float32), (u[tr], nu + i[tr])), shape=(n, n)).tocsr()
        order = reverse_cuthill_mckee((a + a.T).tocsr(), symmetric_mode=True)
        ou = order[order < nu]
        oi = order[order >= nu] - nu
    else:
        raise SystemExit(f"RSX_BENCH_RELABEL={how!r}: degree or rcm")
    new_u = np.empty(nu, np.int64)
    new_u[ou] = np.arange(nu)
    new_i = np.empty(ni, np.int64)
    new_i[oi] = np.arange(ni)
    out = df.copy()
    out["userID"] = new_u[u]
    out["itemID"] = new_i[i]
    return out


def load_graph(workload, rank, world, c4_chunks=None, replicated=False, c4_dim=256):
    """(train users, train items, valid users, valid items, n_users, n_items, d, desc) of
    this rank.  c2: every rank owns its own sports-shaped block of users (rank-seeded)
    over the same items (row-sharded weak scaling), or with `replicated` every rank the
    same graph (data-parallel).  c4: the fixed 10M-user graph, whose 8 user chunks are
    dealt to the ranks in contiguous ranges (local user ids)."""
    from rsx import synth

    if workload in ("c2", "baby"):
        shape = "sports" if workload == "c2" else "baby"
        nu0, ni, ne0 = synth.SHAPES[shape]
        df = synth.amazon_like(nu0, ni, ne0, seed=0 if replicated else rank)
        relabel = os.environ.get("RSX_BENCH_RELABEL")
        if relabel:  # locality experiment: the same graph under a node relabelling (a permutation)
            df = relabel_graph(df, relabel)
        tr, va = df[df.x_label == 0], df[df.x_label == 1]
        desc = (f"C2: LightGCN K=3 d=64, sports-shaped (35,598 users x 18,357 items per rank), B=2048 per rank, "
                f"device sampler, fused step" if workload == "c2" else
                "north_star baby leg: LightGCN K=3 d=64, baby-shaped (19,445 users x 7,050 items per rank), "
                "B=2048 per rank, device sampler, fused step")
        return (tr.userID.values.astype(np.int64), tr.itemID.values.astype(np.int64),
                va.userID.values.astype(np.int64), va.itemID.values.astype(np.int64),
                int(df.userID.max()) + 1, ni, 64, desc)
    import multiprocessing as mp

    C = synth.C4
    n_chunks = c4_chunks or C["n_users"] // C["chunk_users"]
    c0, c1 = rank * n_chunks // world, (rank + 1) * n_chunks // world
    cdf = synth.zipf_cdf(C["n_items"], 0)
    with mp.get_context("fork").Pool(min(8, c1 - c0)) as pool:  # before any GPU use in this process
        parts = sorted(pool.map(_c4_chunk, [(c, cdf) for c in range(c0, c1)]), key=lambda x: x[0])
    tu, ti, vu, vi = [], [], [], []
    for c, u, i, lab in parts:
        off = (c - c0) * C["chunk_users"]
        tr, va = lab == 0, lab == 1
        tu.append(u[tr] + off)
        ti.append(i[tr])
        vu.append(u[va] + off)
        vi.append(i[va])
    head = ("C4: LightGCN K=3 d=256" if c4_dim == 256 else
            f"C4-d{c4_dim} (the metric's d={c4_dim} on C4's graph): LightGCN K=3 d={c4_dim}")
    return (np.concatenate(tu), np.concatenate(ti), np.concatenate(vu), np.concatenate(vi),
            (c1 - c0) * C["chunk_users"], C["n_items"], c4_dim,
            head + ", synthetic 10M users x 1M items (~10 interactions/user, Zipf(0.8) items; "
            "reference split rule), users row-sharded over the ranks, items replicated, global batch 2048 "
            "split over the ranks")


def replica_hash(t: torch.Tensor) -> torch.Tensor:
    """A position-dependent 64-bit hash of a tensor's words (int64 arithmetic wraps):
    sum_i w_i * (2654435761 i + 1).  A word moved to another index or two differences
    that cancel in a plain sum change it (the plain sum could not tell)."""
    w = t.detach().contiguous().view(torch.int32).reshape(-1).to(torch.int64)
    k = torch.arange(w.numel(), dtype=torch.int64, device=w.device) * 2654435761 + 1
    return (w * k).sum()


def _json_line(out):
    """The one JSON line, on the real stdout (library banners were sent to stderr)."""
    os.write(_STDOUT_FD, (json.dumps(out) + "\n").encode())


_STDOUT_FD = 1


def _local_device() -> int:
    """This rank's GPU: LOCAL_RANK (one process per GPU).  RSX_BENCH_SAME_DEVICE=1 puts every
    rank on GPU 0 -- only with RSX_BENCH_BACKEND=gloo (RCCL refuses two ranks on one GPU):
    a rehearsal of the N-rank code paths on a one-GPU box, not a measurement."""
    if os.environ.get("RSX_BENCH_SAME_DEVICE") == "1":
        return 0
    return int(os.environ.get("LOCAL_RANK", "0"))


def _init_group(local: int):
    import torch.distributed as dist

    backend = os.environ.get("RSX_BENCH_BACKEND", "nccl")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)


def ephemeral_port_range():
    """The kernel's ephemeral (auto-bind) port range, /proc/sys/net/ipv4/ip_local_port_range."""
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            lo, hi = (int(x) for x in f.read().split()[:2])
        return lo, hi
    except (OSError, ValueError):
        return 32768, 60999  # the Linux default


def rendezvous_port():
    """MASTER_PORT for the ranks this launcher starts: a free port OUTSIDE the ephemeral
    range.  A port taken by binding port 0 lies inside that range, so between closing the
    probe socket and rank 0's TCPStore listen the kernel can hand it to any connect() --
    including a peer rank's own retrying client, which then connects to itself
    (GPUTEST_r05: EADDRINUSE).  The kernel never auto-assigns a port outside the range,
    so only an explicit bind elsewhere could take this one."""
    import socket

    lo, hi = ephemeral_port_range()
    pool = list(range(20000, lo)) if lo > 20000 else list(range(hi + 1, 65536))
    if not pool:  # the whole port space is ephemeral: nothing better than a probe
        pool = [29500]
    start = (os.getpid() * 7919) % len(pool)
    for k in range(min(len(pool), 256)):
        p = pool[(start + k) % len(pool)]
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            try:
                s.bind(("127.0.0.1", p))
            except OSError:
                continue
        return p
    return pool[start]


def launch(argv, n):
    """`bench.py --gpus N` without an external launcher: start N rank processes of this
    script (one per GPU, LOCAL_RANK = rank) with the torch.distributed env a torchrun
    launch would give them, relay rank 0's JSON line, and return the worst exit code.
    This process never touches the GPU (no HIP call before or after the children), so
    nothing here initialises a device that a child then shares.  Replaces the
    reference's one-device pinning (src/utils/configurator.py:114-118)."""
    import subprocess
    import tempfile

    port = os.environ.get("MASTER_PORT") or str(rendezvous_port())  # an explicit override wins
    out_path = tempfile.mkstemp(prefix="rsx_bench_rank0_", suffix=".json")[1]
    procs = []
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=port, WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", RSX_BENCH_LAUNCHER="bench.py --gpus")
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL peer maps)
    with open(out_path, "wb") as f0:
        for r in range(n):
            env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                          stdout=f0 if r == 0 else sys.stderr.fileno(), stderr=None))
        rcs = [None] * n
        import time as _t

        while any(rc is None for rc in rcs):
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    rcs[r] = p.poll()
            failed = [r for r, rc in enumerate(rcs) if rc not in (None, 0)]
            if failed:  # one rank died: its peers would block in a collective forever
                for r, p in enumerate(procs):
                    if rcs[r] is None:
                        p.terminate()
                for r, p in enumerate(procs):
                    try:
                        rcs[r] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[r] = p.wait()
                log(f"[bench] launcher: rank(s) {failed} failed, exit codes {rcs}")
                break
            _t.sleep(0.05)
    with open(out_path, "rb") as f0:
        line = f0.read()
    os.unlink(out_path)
    if line:
        os.write(_STDOUT_FD, line)
    bad = [rc for rc in rcs if rc]
    return bad[0] if bad else 0


def _rank_report(wall_s, gpu_ms, steps, world, dev):
    """Every rank's (ms/step wall, ms/step device events), gathered to rank order."""
    mine = torch.tensor([wall_s * 1e3 / steps, gpu_ms / steps], dtype=torch.float64, device=dev)
    if world == 1:
        return [{"rank": 0, "ms_per_step": float(mine[0]), "gpu_ms_per_step_events": float(mine[1])}]
    if torch.distributed.get_backend() != "nccl":
        mine = mine.cpu()  # gloo gathers host tensors only
    parts = [torch.empty_like(mine) for _ in range(world)]
    torch.distributed.all_gather(parts, mine)
    return [{"rank": r, "ms_per_step": float(p[0]), "gpu_ms_per_step_events": float(p[1])}
            for r, p in enumerate(parts)]


def dry_run(args):
    """The N-rank launch and reporting without a GPU (CPU tests): gloo group, the
    world size observed by an all-reduce of ones, K timed CPU 'steps' per rank
    (a fixed small matmul), max-over-ranks time, per-rank report on rank 0."""
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if os.environ.get("RSX_BENCH_DRY_FAIL_RANK") == str(rank):  # test hook: a rank that dies
        raise SystemExit(3)
    if world > 1:
        dist.init_process_group("gloo")
    ones = torch.ones(1)
    if world > 1:
        dist.all_reduce(ones)
    x = torch.randn(64, 64)

    def step():
        return x @ x

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    per_rank = _rank_report(wall, 0.0, args.steps, world, torch.device("cpu"))
    tmax = max(p["ms_per_step"] for p in per_rank) * args.steps / 1e3
    if rank == 0:
        _json_line({"metric": METRIC, "value": None, "unit": "interactions/s", "n_gpus": world,
                    "steps": args.steps, "warmup": args.warmup, "ms_per_step": tmax * 1e3 / args.steps,
                    "dry_run": True, "launcher": os.environ.get("RSX_BENCH_LAUNCHER", "external"),
                    "world_size_observed": int(ones.item()), "per_rank": per_rank,
                    "master_port": int(os.environ["MASTER_PORT"]) if "MASTER_PORT" in os.environ else None})
    if world > 1:
        dist.destroy_process_group()


def main():
    global _STDOUT_FD
    # RCCL / HIP print banners on fd 1 at communicator init: keep fd 1 for the JSON line
    sys.stdout.flush()
    _STDOUT_FD = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default=None, choices=["c2", "baby", "c1", "c3", "c4", "c5"],
                    help="default: c2 at N = 1 (the headline LightGCN sports config), c4 --dim 64 at N > 1 (the "
                         "metric's d = 64 on the 10M-user graph, strong scaling: the ranks divide the graph); "
                         "baby: LightGCN on baby (north_star's 10x leg); c1/c3: LayerGCN / SMORE on baby; "
                         "c5: SMORE d=128 CLIP on clothing; c4: LightGCN d=256 on the 10M-user graph, row-sharded")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default 200 (c4: 20)")
    ap.add_argument("--warmup", type=int, default=None, help="default 20 (c4: 3)")
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sharded", action="store_true",
                    help="use the row-sharded engine even at N=1 (measures its host/launch overhead)")
    ap.add_argument("--dist", choices=["dp", "rowshard"], default=None,
                    help="N>1 scheme for --workload c2/baby: rowshard (default: every rank its own sports-shaped user block "
                         "over the same items, users row-sharded, item partials reduced per layer, rsx.dist: the "
                         "ranks divide the propagation) or dp (the graph replicated, every rank evaluating the "
                         "global batch, rsx.dp); c4 is always rowshard")
    ap.add_argument("--dp", action="store_true",
                    help="use the data-parallel engine even at N=1 (measures its exchange-free overhead)")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--eval-users", type=int, default=None, help="default: all valid users (c4: 32768 per rank)")
    ap.add_argument("--c4-chunks", type=int, default=None,
                    help="c4: build only the first N of the 8 1.25M-user chunks (1 = one rank's share at 8 GPUs)")
    ap.add_argument("--dim", type=int, default=None, choices=[64, 128, 256],
                    help="c4 only: embedding size (default 256 = config C4; 64 = the metric's d on C4's graph, "
                         "the strong-scaling leg whose N=1 anchor fits one GPU)")
    ap.add_argument("--n-layers", type=int, default=3,
                    help="LightGCN depth (c2/baby/c4; default 3 = configs C2/C4; the reference's YAML default is 4)")
    ap.add_argument("--cpu", action="store_true",
                    help="c1 only: the CPU configuration (BASELINE config 1) through torch.ops.rsx's C++ CPU "
                         "kernels, whole epochs timed beside the CPU port; --steps = epochs (default 2)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only: exercise the N-rank launch and report (gloo), no GPU work")
    args = ap.parse_args()
    n_ranks = int(os.environ.get("WORLD_SIZE", args.gpus))
    if args.workload is None:
        # N = 1: C2, the config the metric is quoted on.  N > 1: the metric's d = 64 LightGCN on
        # the 10M-user graph, row-sharded (strong scaling).  The sports graph cannot be divided
        # profitably (0.14 ms a step on one GPU): its row-sharded and data-parallel multi-GPU
        # legs both lose to one GPU at the same global batch
        args.workload = "c2" if n_ranks <= 1 else "c4"
        if args.workload == "c4" and args.dim is None:
            args.dim = 64
    if os.environ.get("RSX_COMM_SIM"):  # the bench is the latency-injection mode's one user
        os.environ.setdefault("RSX_COMM_SIM_OPT_IN", "1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no external launcher (torchrun sets WORLD_SIZE): start the N ranks here
        raise SystemExit(launch(sys.argv[1:], args.gpus))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        log(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}; the world size wins")
    if args.dry_run:
        args.steps = args.steps if args.steps is not None else 3
        args.warmup = args.warmup if args.warmup is not None else 1
        return dry_run(args)
    if args.cpu:
        if args.workload != "c1" or args.gpus != 1:
            raise SystemExit("--cpu is the one-process C1 configuration (--workload c1)")
        return bench_c1_cpu(args)
    big = args.workload == "c4"
    if args.dim is not None and not big:
        raise SystemExit("--dim applies to --workload c4")
    args.steps = args.steps if args.steps is not None else (20 if big else 200)
    args.warmup = args.warmup if args.warmup is not None else (3 if big else 20)
    args.eval_users = args.eval_users if args.eval_users is not None else (32768 if big else 0)
    if args.workload in ("c1", "c3", "c5"):
        if int(os.environ.get("WORLD_SIZE", "1")) != 1 and args.workload == "c1":
            raise SystemExit("--workload c1 is a single-GPU leg")
        return bench_model(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = _local_device()
    # c4 is the strong-scaling leg: the graph AND the global batch (--batch) are fixed, each
    # rank draws its share of the batch from its own users; c2/baby are weak scaling: every
    # rank owns its own sports/baby-shaped user block and a batch of --batch
    # latency injection (RSX_COMM_SIM=W, rsx.dist.sim_comm_params): ONE rank runs the per-rank
    # share of a W-rank c4 job (8/W of the 8 user chunks, batch 2048/W) with every collective
    # replaced by a comm-stream kernel holding the modelled time, CUs and HBM bytes of that
    # collective at W ranks: the step time is the modelled job's critical path
    # (c2 / baby: the data-parallel leg's rank 0 of a W-rank job, csrc/dp.hip's sim mode: the
    # job's global batch and union through the step, the two all-gathers modelled)
    from rsx.dist import sim_comm_params

    sim = sim_comm_params()
    if sim and big:  # time this rank's share of the modelled job (csrc/dist.hip: the owner Adam on 1/W items)
        os.environ.setdefault("RSX_COMM_SIM_SHARE", "1")
    w_eff = sim["world"] if sim else world
    if sim and world != 1:
        raise SystemExit("RSX_COMM_SIM runs one rank")
    if sim and args.c4_chunks is None:
        args.c4_chunks = 8 // w_eff
    B = args.batch // w_eff if big else args.batch
    if big and B * w_eff != args.batch:
        raise SystemExit(f"--batch {args.batch} does not split evenly over {w_eff} ranks")
    # N > 1 default: row-sharded (the ranks divide the propagation); dp is opt-in (--dist dp)
    scheme = args.dist or "rowshard"
    if big and scheme != "rowshard":
        raise SystemExit("--workload c4 is the row-sharded strong-scaling leg")
    dp = not big and not args.sharded and (args.dp or ((world > 1 or sim is not None) and scheme == "dp"))
    tu, ti, vu_all, vi_all, nu, ni, d, desc = load_graph(args.workload, rank, world, args.c4_chunks, replicated=dp,
                                                         c4_dim=args.dim or 256)
    if big and args.c4_chunks:
        desc += f" [only {args.c4_chunks} of 8 user chunks built]"
    if sim and big:
        desc += (f" [latency-injected model of rank 0 of a {sim['world']}-rank job: its {args.c4_chunks}/8 user "
                 f"share, batch {B}, every collective a comm-stream kernel of the modelled time at "
                 f"{sim['busbw_gbs']:.0f} GB/s bus bandwidth + {sim['latency_us']:.0f} us]")
    elif sim and not dp:
        desc += (f" [latency-injected model of rank 0 of a {sim['world']}-rank row-sharded job: its own user "
                 f"block, B={B}, every item-partial collective a comm-stream kernel of the modelled time at "
                 f"{sim['busbw_gbs']:.0f} GB/s bus bandwidth + {sim['latency_us']:.0f} us]")
    elif sim:
        desc += (f" [latency-injected model of rank 0 of a {sim['world']}-rank data-parallel job: the graph "
                 f"replicated, B={B} per rank, global batch {B * sim['world']} (the other ranks' triplets in their "
                 f"slots), both all-gathers comm-stream kernels of the modelled time at {sim['busbw_gbs']:.0f} GB/s "
                 f"bus bandwidth + {sim['latency_us']:.0f} us]")
    if dp:
        desc = desc.replace("per rank), B=2048 per rank", "), the graph replicated on every rank, "
                                                              f"B={B} per rank, global batch {B * world}")
    sharded = (world > 1 or big or args.sharded or (sim is not None and scheme == "rowshard")) and not dp
    if sharded or dp:
        import torch.distributed as dist

        if world == 1:  # a one-rank group for the sharded engine
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(rendezvous_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local)
        _init_group(local)
    dev = torch.device("cuda", local)

    from rsx.engine import LightGCNEngine
    from rsx import _lib as L, graph, ops

    torch.manual_seed(999 + rank)
    if big:  # xavier_uniform_ bound for [n, d]: sqrt(6 / (n + d)); drawn on the device
        U0 = ((torch.rand(nu, d, device=dev) * 2 - 1) * (6.0 / (nu + d)) ** 0.5).cpu()
        I0 = ((torch.rand(ni, d, device=dev) * 2 - 1) * (6.0 / (ni + d)) ** 0.5).cpu()
    else:
        U0 = torch.nn.init.xavier_uniform_(torch.empty(nu, d)).numpy()
        I0 = torch.nn.init.xavier_uniform_(torch.empty(ni, d)).numpy()

    if dp:
        from rsx.dp import DataParallelLightGCNEngine

        eng = DataParallelLightGCNEngine(tu, ti, nu, ni, d, args.n_layers, 1e-2, 1e-3, dev, U0, I0, seed=0,
                                         batch=B)
    elif sharded:
        from rsx.dist import ShardedLightGCNEngine

        eng = ShardedLightGCNEngine(tu, ti, nu, ni, d, args.n_layers, 1e-2, 1e-3, dev, U0, I0, seed=rank,
                                    batch=B)
    else:
        eng = LightGCNEngine(tu, ti, nu, ni, d, args.n_layers, 1e-2, 1e-3, dev, U0, I0, seed=0, batch=B)
    del U0, I0
    E = eng.n_inter
    parts = [eng.adj] if hasattr(eng, "adj") else [eng.A_U, eng.A_I]
    nnz = sum(a.nnz for a in parts)
    log(f"[bench] rank {rank}/{world}: users {nu} items {ni} train {E} nnz {nnz}")

    pos = {"epoch": 0, "start": 0}
    done = {"inter": 0}

    def one_step():
        if dp:  # global step j: this rank's slice j W + rank of the epoch (S W balanced slices)
            S = eng.steps_per_epoch()
            j = pos["start"]
            a, e = ops.DeviceSampler.slice_bounds(E, S * world, j * world + rank)
            eng.step_index(pos["epoch"], j)
            done["inter"] += e - a
            pos["start"] += 1
            if pos["start"] >= S:
                pos["start"] = 0
                pos["epoch"] += 1
            return
        b = min(B, E - pos["start"])
        eng.step(epoch=pos["epoch"], start=pos["start"])
        done["inter"] += b
        pos["start"] += B
        if pos["start"] >= E:
            pos["start"] = 0
            pos["epoch"] += 1

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    done["inter"] = 0
    t0 = time.perf_counter()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(args.steps):
        one_step()
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    per_rank = _rank_report(wall, gpu_ms, args.steps, world, dev)
    rccl_world = None
    if (sharded or dp) and getattr(eng, "_comm", None) is not None and (
            not dp or torch.distributed.get_backend() == "nccl" or sim):
        # the world the step's own communicator spans: an all-reduce of ones on rsx_comm
        # (the DP engine's host hook -- gloo rehearsals -- moves all-gathers only)
        ones = torch.ones(1, dtype=torch.float32, device=dev)
        L.check(L.lib().rsx_comm_allreduce_f32(eng._comm, ones.data_ptr(), 1, ops._stream()),
                "rsx_comm_allreduce_f32")
        rccl_world = int(round(float(ones.item())))
    # data-parallel: the replicas must stay bit-identical with no parameter exchange (§6.1):
    # a position-dependent hash of every rank's parameter table and Adam moments, compared
    # across the ranks after the timed steps (outside the timed region)
    replicas_identical = None
    if dp and world > 1:
        ck = torch.stack([replica_hash(t) for t in (eng.p, eng.m, eng.v)])
        if torch.distributed.get_backend() != "nccl":
            ck = ck.cpu()
        cks = [torch.empty_like(ck) for _ in range(world)]
        torch.distributed.all_gather(cks, ck)
        replicas_identical = all(torch.equal(cks[0], q) for q in cks[1:])
    t_rank = torch.tensor([wall, float(done["inter"])], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = t_rank[:1].clone()
        tot = t_rank[1:].clone()
        torch.distributed.all_reduce(tmax, op=torch.distributed.ReduceOp.MAX)
        torch.distributed.all_reduce(tot, op=torch.distributed.ReduceOp.SUM)
        wall, total_inter = float(tmax.item()), float(tot.item())
    else:
        total_inter = float(done["inter"])
    loss_mean = float(eng.loss_acc.item()) / max(eng.step_count, 1)

    # epoch-inclusive rate: one whole fresh epoch, its sampling launch included
    epoch_rate = None
    if not big:
        pos["epoch"] += 1
        pos["start"] = 0
        ep0 = pos["epoch"]
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        # every rank runs the same number of steps (its collectives pair with its peers'):
        # the largest per-rank batch count; a rank with fewer batches wraps into its next epoch
        nb = torch.tensor([float(eng.steps_per_epoch() if dp else -(-E // B))], dtype=torch.float64, device=dev)
        if world > 1:
            torch.distributed.all_reduce(nb, op=torch.distributed.ReduceOp.MAX)
        nb = int(nb.item())
        done["inter"] = 0
        t_ep = time.perf_counter()
        for _ in range(nb):
            one_step()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        ep_s = time.perf_counter() - t_ep
        er = torch.tensor([ep_s, float(done["inter"])], dtype=torch.float64, device=dev)
        if world > 1:
            torch.distributed.all_reduce(er[:1], op=torch.distributed.ReduceOp.MAX)
            torch.distributed.all_reduce(er[1:], op=torch.distributed.ReduceOp.SUM)
        epoch_rate = {"interactions_per_s": float(er[1] / er[0]), "s_per_epoch": float(er[0]),
                      "batches_per_rank": nb,
                      "includes": "the epoch's device sampling launch (shuffle + negatives), every batch's step"}

    # full-sort evaluation throughput (forward once + fused MFMA scores/mask/top-50)
    vusers = np.unique(vu_all)
    if args.eval_users:
        vusers = vusers[: args.eval_users]
    if dp and world > 1:  # the replicas split the evaluation users (metric sums would be gathered)
        vusers = vusers[rank * vusers.size // world:(rank + 1) * vusers.size // world]
    rp, mc = graph.history_csr(tu, ti, nu)
    rp_d, mc_d = torch.from_numpy(rp).to(dev), torch.from_numpy(mc).to(dev)
    vu_d = torch.from_numpy(vusers.astype(np.int64)).to(dev)

    # held-out (valid) items per evaluation user, sorted: the metric tail's CSR
    sel = np.isin(vu_all, vusers)
    order = np.lexsort((vi_all[sel], vu_all[sel]))
    v_u, v_i = vu_all[sel][order], vi_all[sel][order]
    vlen = np.bincount(np.searchsorted(vusers, v_u), minlength=vusers.size)
    erp = torch.from_numpy(np.concatenate([[0], np.cumsum(vlen)]).astype(np.int64)).to(dev)
    ecol = torch.from_numpy(v_i.astype(np.int32)).to(dev)
    n_pos = int(v_i.size)
    from rsx.evaluator import device_metric_dict

    def evaluate():
        # what Trainer.evaluate does: forward once, one fused scores+mask+top-50 launch over
        # all evaluation users (no score matrix), the metric tail on device, metrics to host
        eng.invalidate()
        f = eng.forward()
        _, idx = ops.fullsort_topk(f[:nu], vu_d, f[nu:], rp_d, mc_d, 50)
        device_metric_dict(idx, erp, ecol, ["recall", "ndcg", "precision", "map"], [5, 10, 20, 50], n_pos)

    evaluate()
    torch.cuda.synchronize()
    te = time.perf_counter()
    reps = 5
    for _ in range(reps):
        evaluate()
    torch.cuda.synchronize()
    eval_s = (time.perf_counter() - te) / reps
    n_eval = float(vusers.size)
    if world > 1:
        ev = torch.tensor([eval_s], dtype=torch.float64, device=dev)
        nev = torch.tensor([n_eval], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(ev, op=torch.distributed.ReduceOp.MAX)
        torch.distributed.all_reduce(nev, op=torch.distributed.ReduceOp.SUM)
        eval_s, n_eval = float(ev.item()), float(nev.item())
    items_per_s = n_eval * ni / eval_s
    # fused scores + mask + top-50 over all evaluation users (MFMA roofline)
    f = eng.forward()
    fs_ms = time_kernel(lambda: ops.fullsort_topk(f[:nu], vu_d, f[nu:], rp_d, mc_d, 50), 10)
    fs_flops = 2.0 * d * ni * vu_d.numel()

    # dominant kernel: one propagation SpMM (STORE epilogue), same stream as the step
    x = eng.p
    ys = [torch.empty(a.n_rows, d, device=dev) for a in parts]

    def run_parts():
        for a, y in zip(parts, ys):
            a.spmm(x, out=y)

    spmm_ms = time_kernel(run_parts, 50)
    alg = spmm_bytes(nu + ni, nnz, d)
    achieved = alg / (spmm_ms * 1e-3) / 1e9

    def pmc_bytes(name):  # PMC bytes per launch measured for the C2 kernel (profiles/*.json)
        tfile = os.path.join(HERE, "profiles", name)
        if os.path.exists(tfile) and args.workload == "c2" and not sharded:
            try:
                return json.load(open(tfile)).get("bytes_per_launch")
            except Exception:  # noqa: BLE001
                return None
        return None

    traffic = pmc_bytes("spmm_traffic.json")
    prior = None
    if big and d == 256:
        # C4: no PMC pass runs inside this process, so `traffic` stays null; the round-3
        # FETCH_SIZE passes of one rank's 1/8 share (1.25M users x 1M items, gfx950-corrected;
        # an older kernel than this HEAD's) are quoted beside it, labelled as such
        tfile = os.path.join(HERE, "profiles", "r03", "c4", "c4_spmm_traffic.json")
        if os.path.exists(tfile) and abs(nu - 1_250_000) <= 1000:
            try:
                per = json.load(open(tfile))["per_kind_fetch_bytes_per_launch"]["spmm_main<256, 0>"]
                prior = {"bytes_per_layer": 2 * per + 4.0 * (nu + ni) * d,
                         "source": "round-3 PMC FETCH_SIZE of the 1/8-share product launches "
                                   "(profiles/r03/c4/c4_spmm_traffic.json) x 2 products + the written rows; "
                                   "measured on the round-3 kernel, not on this HEAD"}
            except Exception:  # noqa: BLE001
                prior = None
    store = {"bound": "hbm", "kernel": f"spmm_main<{d},STORE> (hub-row fixups in-launch) one propagation layer",
             "launches_per_step": 2 if not sharded else None,
             "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
             "traffic": traffic, **({"traffic_prior_profile": prior} if prior else {}),
             "algorithmic_bytes_per_launch": alg, "avg_launch_ms": spmm_ms,
             "note": ("the sports/baby working set (<50 MB) is Infinity-Cache resident" if not big else
                      "C4 shard: tables of GBs, gathers from HBM")}
    roof, kernels = store, [store]
    if not sharded and hasattr(eng, "adj"):
        # the step's largest single launch: the last backward layer with Adam fused into
        # its epilogue, exactly as the tagged step issues it (rows of the last batch
        # tagged; sparse G' and clears on those rows), on scratch copies of p, m, v
        pc, mc, vc, gc = eng.p.clone(), eng.m.clone(), eng.v.clone(), eng.g.clone()
        adam_e = ops.epi(L.RSX_EPI_ADAM, s_in=gc, p=pc, m=mc, v=vc, zero0=gc, row_tag=eng.row_tag,
                         adam=ops.adam_struct(eng.lr, max(eng.step_count, 1)))
        adam_e.tag = max(eng.step_count, 1)
        adam_e.tag_flags = L.RSX_TAG_SPARSE_S | L.RSX_TAG_SPARSE_R | L.RSX_TAG_ZERO
        xh = eng.h1

        def adam_layer():
            eng.adj.spmm_epi(xh, adam_e, d)

        adam_ms = time_kernel(adam_layer, 50)
        # S_spmm + Adam's row streams (reads p, m, v; writes m, v: p's write
        # is S's Y) = S + 20 N d; G' is read on the batch rows only (+ 12 B d per row)
        adam_alg = alg + 20 * (nu + ni) * d + 12 * 3 * B * d
        adam_ach = adam_alg / (adam_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": f"spmm_main<{d},ADAM> (last backward layer + Adam, batch-row tags; "
                                          "the step's largest launch)",
                "launches_per_step": 1, "achieved": adam_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": adam_ach / HBM_PEAK_GBS, "traffic": pmc_bytes("spmm_adam_traffic.json"),
                "algorithmic_bytes_per_launch": adam_alg, "avg_launch_ms": adam_ms,
                "note": store["note"]}
        # the backward's Horner layer H = G' + A H (ADD epilogue, G' read on the batch rows):
        # two per step at K = 3, the first gathering only G's batch rows
        yh = torch.empty_like(eng.h0)
        add_e = ops.epi(L.RSX_EPI_ADD, y=yh, s_in=gc, row_tag=eng.row_tag)
        add_e.tag = max(eng.step_count, 1)
        add_e.tag_flags = L.RSX_TAG_SPARSE_S

        def add_layer():
            eng.adj.spmm_epi(eng.h0, add_e, d)

        add_ms = time_kernel(add_layer, 50)
        add_alg = alg + 12 * 3 * B * d
        add_ach = add_alg / (add_ms * 1e-3) / 1e9
        addk = {"bound": "hbm", "kernel": f"spmm_main<{d},ADD> (a backward Horner layer H = G' + A H, dense X, "
                                         "G' on the batch rows)",
                "launches_per_step": 1 if args.n_layers == 3 else None, "achieved": add_ach, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": add_ach / HBM_PEAK_GBS, "traffic": None,
                "algorithmic_bytes_per_launch": add_alg, "avg_launch_ms": add_ms, "note": store["note"]}
        kernels = [roof, store, addk]
        del pc, mc, vc, gc, yh

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if not big:
            cpu = cpu_baseline((tu, ti), nu, ni, args.cpu_budget, shape="sports" if args.workload == "c2" else "baby",
                               K=args.n_layers)
        else:  # C4: a 1/10 user slice (the first 1M users of the graph) over all 1M items, per step
            m = tu < 1_000_000
            cpu = cpu_baseline((tu[m], ti[m]), 1_000_000, ni, args.cpu_budget, d=d, shape="C4", scale=10,
                               K=args.n_layers)

    if rank == 0:
        ms = wall * 1e3 / args.steps
        out = {
            "metric": METRIC,
            "value": total_inter / wall,
            "unit": "interactions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            # c4: the graph is fixed whatever N (strong), each rank's batch is its own users' 2048
            "scaling": "strong" if big else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": (f"synthetic Amazon-{'sports' if args.workload == 'c2' else 'baby'}-shaped graph (rsx.synth, "
                     "seed=rank; Zipf(0.8) items, 5-core users, reference split rule); xavier-uniform init, seed 999")
                    if not big else
                    ("synthetic C4 graph (rsx.synth.chunk_graph: 8 seeded 1.25M-user chunks, Zipf(0.8) items, "
                     "5+Geometric degrees mean 10, reference split rule); xavier-uniform-bound init"),
            "config": {"workload": desc, "model": "LightGCN", "n_layers": args.n_layers, "embedding_size": d,
                       "global_batch": B * world, "per_rank_batch": B,
                       "leg": ("the metric's leg: C2, weak scaling (per-GPU work fixed as N grows)"
                               if args.workload == "c2" else
                               "strong-scaling leg: the fixed C4 graph and global batch split over the ranks"
                               if big else "baby, weak scaling"),
                       "parallelism": (f"dp{world}" if dp else f"rowshard{world}" if sharded else "single"),
                       "scheme": ("data-parallel: graph + tables replicated, global batch N*B, per step one "
                                  "all-gather of the ranks' triplets (rsx.dp)" if dp else
                                  "row-sharded users, replicated items, item partials all-reduced per layer "
                                  "(rsx.dist)" if sharded else "one GPU"),
                       **({"dp_issue": "graph replay" if eng.use_graph else "eager (one C-ABI call a step)"}
                          if dp else {})},
            "fullsort_items_per_s": items_per_s,
            "fullsort": {"eval_users": int(n_eval), "n_items": ni, "k": 50,
                         "s_per_eval": eval_s,
                         "s_per_eval_includes": "forward + fused top-50 + recall/ndcg/precision/map tail + D2H",
                         "kernel_ms_all_eval_users": fs_ms,
                         # the dense f32 score matrix's flops / kernel time: the screened kernel
                         # (csrc/fullsort.hip fs_screen) runs two bf16 MFMA passes over all pairs and
                         # exact f32 dots for the candidates only, so this is an f32-equivalent rate
                         "algorithmic_tflops_f32_equivalent": fs_flops / (fs_ms * 1e-3) / 1e12,
                         "algorithmic_tflops_note": ("2*d*n_items*users (the dense f32 score GEMM's flops) / "
                                                     "kernel time: an ALGORITHMIC rate of the screened "
                                                     "selection (most pairs never get an f32 dot), not "
                                                     "hardware utilisation; it may exceed the 157.3 TF/s f32 "
                                                     "MFMA peak. Utilisation: mfma_util"),
                         "screen_bf16_mfma_tflops": 2 * 2.0 * (d + 16) * ni * vu_d.numel() / (fs_ms * 1e-3) / 1e12,
                         # north_star's "MFMA utilisation for the full-sort GEMM": the MFMA work the
                         # screened kernel issues (two bf16 passes over every pair) per second over the
                         # dense bf16 peak; the f32-equivalent rate above is the algorithm's, not the
                         # matrix cores' (the kernel is issue-bound on its selection work)
                         "mfma_util": 2 * 2.0 * (d + 16) * ni * vu_d.numel() / (fs_ms * 1e-3) / 1e12 / 2516.6,
                         "mfma_util_note": "bf16 MFMA work / kernel time / 2516.6 TF/s dense bf16 peak",
                         "mfma_f32_peak_tflops": 157.3, "mfma_bf16_dense_peak_tflops": 2516.6},
            "roofline": roof,
            "roofline_kernels": kernels,
            "cpu_baseline": cpu,
            "epoch": epoch_rate,
            "launcher": os.environ.get("RSX_BENCH_LAUNCHER", "torchrun" if world > 1 else "single process"),
            "rccl_world_size": rccl_world,
            "dp_replicas_bit_identical": replicas_identical,
            "per_rank": per_rank,
            "gpu_ms_per_step_events": gpu_ms / args.steps,
            "train_loss_mean": loss_mean,
        }
        if big and d == 64:
            out["scaling_note"] = ("N > 1 default: the metric's d = 64 LightGCN on the fixed 10M-user graph, strong "
                                   "scaling; its one-GPU anchor is `bench.py --workload c4 --dim 64` (round 6: "
                                   "40.5 ms/step, 50.6 k interactions/s, profiles/r06/c4d64/), not the N = 1 default "
                                   "line (C2, the sports graph), so value_N / (N x value_C2) is not an efficiency")
        if sim and dp:
            lib = L.lib()
            Wm = sim["world"]
            out["latency_injection"] = dict(sim, per_collective_ms={
                "allgather_slots": 1e3 * lib.rsx_comm_sim_seconds(eng._comm, L.RSX_COLL_ALLGATHER,
                                                                  float(3 * eng.cap + 1) * 8 * Wm)},
                modelled_job={"world": Wm, "interactions_per_s": Wm * total_inter / wall,
                              "global_batch": B * Wm, "ms_per_step": ms},
                note="value / ms_per_step: rank 0 of the modelled data-parallel job (every rank runs the same "
                     "step on the replicated graph, so the job's rate is world x value)")
        elif sim:
            X = float(ni) * d * 4
            lib = L.lib()
            # one stand-alone injected all-reduce of the item block, timed on the device: the
            # stand-in must take the modelled time (its HBM copy must not be the bound)
            import ctypes as _C
            buf = torch.zeros(ni * d, dtype=torch.float32, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            L.check(lib.rsx_comm_allreduce_f32(eng._comm, _C.c_void_p(buf.data_ptr()), ni * d, ops._stream()),
                    "rsx_comm_allreduce_f32")
            e1.record()
            torch.cuda.synchronize()
            del buf
            Wm = sim["world"]
            out["latency_injection"] = dict(sim, per_collective_ms={
                "allreduce_item_block": 1e3 * lib.rsx_comm_sim_seconds(eng._comm, L.RSX_COLL_ALLREDUCE, X),
                "reduce_scatter_or_all_gather_item_block":
                    1e3 * lib.rsx_comm_sim_seconds(eng._comm, L.RSX_COLL_ALLGATHER, X)},
                measured_allreduce_item_block_ms=e0.elapsed_time(e1),
                modelled_job={"world": Wm, "interactions_per_s": Wm * total_inter / wall, "ms_per_step": ms,
                              "global_batch": B * Wm},
                note="value / ms_per_step: one rank's share of the modelled job (the job's rate is world x value "
                     "when every rank holds the same share)")
        _json_line(out)
    if hasattr(eng, "close"):
        eng.close()
    if sharded or dp:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
