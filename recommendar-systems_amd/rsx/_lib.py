"""ctypes binding of librsx.so (include/rsx.h).

The product path has no CPU fallback: `lib()` raises if the library is missing
or cannot be loaded, and every wrapper raises RuntimeError on a nonzero return
code, as the reference raises Python exceptions for bad inputs.
"""
from __future__ import annotations

import ctypes as C
import os

from . import build as _build

P = C.c_void_p
I64 = C.c_int64
I32 = C.c_int32
F32 = C.c_float

RSX_EPI_STORE = 0
RSX_EPI_LAYERSUM = 1
RSX_EPI_FINAL = 2
RSX_EPI_ADAM = 3
RSX_EPI_LAYERGCN = 4
RSX_EPI_AXPBY = 5
RSX_EPI_LAYERGCN_BWD = 6
RSX_EPI_ADD = 7

RSX_BPR_LIGHTGCN = 0
RSX_BPR_LAYERGCN = 1
RSX_BPR_SMORE = 2
RSX_BPR_SMORE_ROWS = 3

RSX_ERR_UNSUPPORTED = 1002

_ERRORS = {1001: "RSX_ERR_ARG (bad size or null pointer)",
           1002: "RSX_ERR_UNSUPPORTED (embedding width / k not compiled)",
           1003: "RSX_ERR_WORKSPACE (workspace too small)",
           1004: "RSX_ERR_COMM (RCCL missing or a collective failed)"}


class Csr(C.Structure):
    _fields_ = [("n_rows", I64), ("n_cols", I64), ("nnz", I64), ("rowptr", P), ("col", P), ("val", P),
                ("chunk", I32), ("pad0", I32), ("n_work", I64), ("work", P), ("n_long", I64),
                ("long_rows", P), ("n_slots", I64)]


class Adam(C.Structure):
    _fields_ = [("lr", F32), ("beta1", F32), ("beta2", F32), ("eps", F32), ("weight_decay", F32),
                ("pad0", I32), ("step_dev", P), ("step", I64)]


class Epilogue(C.Structure):
    _fields_ = [("kind", I32), ("pad0", I32), ("alpha", F32), ("beta", F32),
                ("y", P), ("s_in", P), ("s_out", P), ("f", P), ("zero0", P), ("zero1", P), ("r_add", P),
                ("p", P), ("m", P), ("v", P), ("g_out", P), ("e0", P), ("aux", P), ("aux_w", P),
                ("adam", Adam), ("row_tag", P), ("tag", I32), ("tag_flags", I32), ("reg_cnt", P), ("reg_k", P),
                ("tag_dev", P), ("halt", P), ("x_tag", P)]


RSX_TAG_ROWS = 1
RSX_TAG_SPARSE_X = 2
RSX_TAG_SPARSE_S = 4
RSX_TAG_SPARSE_R = 8
RSX_TAG_ZERO = 16


class SamplerArgs(C.Structure):
    _fields_ = [("inter_u", P), ("inter_i", P), ("n_inter", I64), ("hist_rowptr", P), ("hist_col", P),
                ("all_items", P), ("n_all_items", I64), ("seed", C.c_uint64), ("epoch", I64), ("start", I64)]


class LgcnStep(C.Structure):
    _fields_ = [("adj", C.POINTER(Csr)), ("n_users", I64), ("n_items", I64), ("d", I32), ("n_layers", I32),
                ("reg", F32), ("pad0", I32),
                ("p", P), ("m", P), ("v", P), ("s", P), ("h0", P), ("h1", P), ("final_emb", P), ("g", P),
                ("r", P), ("slab", P), ("triplets", P), ("batch", I64), ("sample", C.POINTER(SamplerArgs)),
                ("adam", Adam), ("loss_out", P), ("loss_acc", P), ("ws", P), ("ws_bytes", C.c_size_t),
                ("row_tag", P), ("tag", I64), ("reg_cnt", P), ("halt", P)]


class LayerGcnStep(C.Structure):
    _fields_ = [("adj", C.POINTER(Csr)), ("n_users", I64), ("n_items", I64), ("d", I32), ("n_layers", I32),
                ("reg", F32), ("pad0", I32),
                ("p", P), ("m", P), ("v", P), ("out", P), ("g", P), ("r", P), ("acc", P), ("h0", P), ("h1", P),
                ("zs", P), ("cs", P), ("slab", P), ("triplets", P), ("batch", I64), ("adam", Adam),
                ("loss_out", P), ("loss_acc", P), ("ws", P), ("ws_bytes", C.c_size_t)]


class ShardedStep(C.Structure):
    _fields_ = [("adj_u", C.POINTER(Csr)), ("adj_i", C.POINTER(Csr)), ("n_users", I64), ("n_items", I64),
                ("d", I32), ("n_layers", I32), ("reg", F32), ("pad0", I32),
                ("p", P), ("m", P), ("v", P), ("s", P), ("h0", P), ("h1", P), ("final_emb", P), ("g", P),
                ("r", P), ("t", P), ("slab_u", P), ("slab_i", P), ("triplets", P), ("batch", I64),
                ("adam", Adam), ("loss_out", P), ("loss_acc", P), ("ws", P), ("ws_bytes", C.c_size_t),
                ("comm", P), ("row_tag", P), ("tag", I64), ("tag_dev", P), ("reg_cnt", P),
                ("union_items", P), ("item_tag", P), ("cbuf0", P), ("cbuf1", P), ("n_items_pad", I64), ("union_cap", I64),
                ("xch", P), ("n_head", I32), ("pad1", I32), ("head_i", C.POINTER(Csr)), ("head_row0", P),
                ("head_slab", P), ("nbr_items", P), ("nbr_count", P), ("cbufN", P), ("nbr_cap", I64), ("defer_ag", I32), ("pad2", I32),
                ("err", P)]


class DpStep(C.Structure):
    _fields_ = [("adj", C.POINTER(Csr)), ("n_users", I64), ("n_items", I64), ("d", I32), ("n_layers", I32),
                ("reg", F32), ("inc_step", I32), ("p", P), ("m", P), ("v", P), ("s", P), ("h0", P), ("h1", P),
                ("final_emb", P), ("g", P), ("slab", P), ("triplets", P), ("batch", I64), ("adam", Adam),
                ("loss_out", P), ("loss_acc", P), ("comm", P), ("row_tag", P), ("tag_dev", P), ("reg_cnt", P),
                ("halt", P), ("cap", I64), ("slots", P), ("work", P), ("work_bytes", C.c_size_t)]


RSX_COLL_ALLREDUCE, RSX_COLL_ALLGATHER, RSX_COLL_REDUCESCATTER = 0, 1, 2
RSX_COLL_F32, RSX_COLL_I64 = 0, 1
HOST_COLLECTIVE_FN = C.CFUNCTYPE(C.c_int, I32, P, I64, I32, P)


_LIB = None


def _declare(lib):
    sig = {
        "rsx_version": (C.c_char_p, []),
        "rsx_csr_schedule_host": (C.c_int, [P, I64, I32, P, P, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64)]),
        "rsx_spmm": (C.c_int, [C.POINTER(Csr), P, I32, C.POINTER(Epilogue), P, P]),
        "rsx_csr_schedule_rebind": (C.c_int, [C.POINTER(Csr), P, P, P]),
        "rsx_spmm_batch": (C.c_int, [I32, P, P, I32, P, P, P]),
        "rsx_rowwise": (C.c_int, [I64, I32, C.POINTER(Epilogue), P]),
        "rsx_bpr_ws_bytes": (C.c_size_t, [I64]),
        "rsx_bpr": (C.c_int, [I32, P, P, I64, I64, I32, P, I64, F32, F32, P, P, P, P, P, C.c_size_t, P]),
        "rsx_fullsort_ws_bytes": (C.c_size_t, [I64, I64, I32]),
        "rsx_fullsort_plan": (C.c_int, [I64, I64, I32, C.POINTER(I32), C.POINTER(I64)]),
        "rsx_fullsort_topk": (C.c_int, [P, P, I64, P, I64, I32, P, P, I32, P, P, P, C.c_size_t, P]),
        "rsx_score_dense": (C.c_int, [P, P, I64, P, I64, I32, P, P]),
        "rsx_sample_triplets": (C.c_int, [P, P, I64, P, P, P, I64, C.c_uint64, I64, I64, I64, P, P]),
        "rsx_gather_rows": (C.c_int, [P, P, I64, I64, I32, P, P]),
        "rsx_sample_epoch": (C.c_int, [P, P, I64, P, P, P, I64, C.c_uint64, I64, I64, P, P]),
        "rsx_sample_epoch_slices": (C.c_int, [P, P, I64, P, P, P, I64, C.c_uint64, I64, I64, P, P]),
        "rsx_lightgcn_step": (C.c_int, [C.POINTER(LgcnStep), P]),
        "rsx_dp_lightgcn_step": (C.c_int, [C.POINTER(DpStep), P]),
        "rsx_comm_init_sim": (C.c_int, [C.POINTER(P), I32, C.c_double, C.c_double, I32, I64]),
        "rsx_comm_allgather_f32": (C.c_int, [P, P, I64, P]),
        "rsx_comm_allreduce_f32_start": (C.c_int, [P, P, I64, P]),
        "rsx_comm_wait": (C.c_int, [P, P]),
        "rsx_comm_sim_seconds": (C.c_double, [P, I32, C.c_double]),
        "rsx_dp_work_bytes": (C.c_size_t, [I64, I32, I64, I32]),
        "rsx_layergcn_step": (C.c_int, [C.POINTER(LayerGcnStep), P]),
        "rsx_lightgcn_forward": (C.c_int, [C.POINTER(Csr), I32, I32, P, P, P, P, P, P, P]),
        "rsx_smore_spectral_spec_floats": (C.c_size_t, [I64, I32]),
        "rsx_smore_spectral_fwd_ws_bytes": (C.c_size_t, [I64, I32, I32, I32]),
        "rsx_smore_spectral_fwd": (C.c_int, [P, I32, P, P, P, I32, P, P, P, P, P, I64, I32, P, P, P, P, P, P, P,
                                             C.c_size_t, P]),
        "rsx_smore_item_tiles": (C.c_size_t, [I64]),
        "rsx_smore_item_fwd": (C.c_int, [P, I32, P, P, P, I32, P, P, P, P, P, I64, I32, P, P, P, P, P, P, P,
                                         C.c_size_t, P, P, P, P, F32, I32, P, P]),
        "rsx_smore_spectral_bwd": (C.c_int, [P, P, P, P, P, P, P, I64, I32, P, P, P, P, C.c_size_t, P]),
        "rsx_smore_spectral_bwd_ws_bytes": (C.c_size_t, [I64, I32]),
        "rsx_smore_spectral_bwd_partials": (C.c_size_t, [I64, I32]),
        "rsx_topk_metrics_ws_bytes": (C.c_size_t, [I64, I32]),
        "rsx_topk_metrics": (C.c_int, [P, I64, I32, P, P, P, I32, P, P, P, C.c_size_t, P]),
        "rsx_topk_metrics_fast": (C.c_int, [P, I64, I32, P, P, P, I32, P, P, P, C.c_size_t, P]),
        "rsx_linear_wgrad_ws_bytes": (C.c_size_t, [I64, I32, I32]),
        "rsx_linear_wgrad": (C.c_int, [P, P, I64, I32, I32, P, P, C.c_size_t, P]),
        "rsx_linear_bwd_ws_bytes": (C.c_size_t, [I64, I32, I32]),
        "rsx_linear_bwd": (C.c_int, [P, P, P, I64, I32, I32, P, P, P, P, C.c_size_t, P]),
        "rsx_linear_bwd_pair_ws_bytes": (C.c_size_t, [I64, I32, I32, I32]),
        "rsx_linear_bwd_pair": (C.c_int, [P, P, P, I32, P, P, P, P, P, P, I32, P, P, P, I64, I32, P, C.c_size_t, P]),
        "rsx_comm_unique_id_bytes": (C.c_size_t, []),
        "rsx_comm_get_unique_id": (C.c_int, [P]),
        "rsx_comm_init": (C.c_int, [C.POINTER(P), P, I32, I32]),
        "rsx_comm_destroy": (C.c_int, [P]),
        "rsx_comm_init_host": (C.c_int, [C.POINTER(P), I32, I32, HOST_COLLECTIVE_FN, P]),
        "rsx_comm_allreduce_f32": (C.c_int, [P, P, I64, P]),
        "rsx_sharded_lightgcn_step": (C.c_int, [C.POINTER(ShardedStep), P]),
        "rsx_sharded_lightgcn_forward": (C.c_int, [C.POINTER(ShardedStep), P]),
        "rsx_sharded_lightgcn_flush": (C.c_int, [C.POINTER(ShardedStep), P]),
        "rsx_smore_gates": (C.c_int, [I32, P, P, P, P, I64, I32, F32, I32, P, P, P, P, P, P]),
        "rsx_smore_gates_saved": (C.c_int, [I32, P, P, P, P, I64, I32, F32, I32, P, P, P, P, P, P, P]),
        "rsx_smore_pref": (C.c_int, [I32, P, P, P, P, P, P, I64, I32, F32, P, P, P, P, P, P, P, P, P, P, P, P, P]),
        "rsx_smore_pref_rows": (C.c_int, [I32, P, P, P, P, P, P, P, I64, I32, F32, P, P, P, P, P, P, P, P, P, P, P,
                                          P, P, P, P, P, P]),
        "rsx_smore_pref_rows_occ_floats": (C.c_size_t, [I64, I32]),
        "rsx_smore_pref_rows_saved": (C.c_int, [I32, P, P, P, P, P, P, P, I64, I32, F32, P, P, P, P, P, P, P, P, P, P,
                                                P, P, P, P, P, P, P, P, P, P]),
        "rsx_smore_pref_rows_saved_floats": (C.c_size_t, [I64, I32]),
        "rsx_smore_pref_plan_words": (C.c_size_t, [I64]),
        "rsx_tag_rows": (C.c_int, [P, P, I64, P, P]),
        "rsx_tag_rows_next": (C.c_int, [P, P, I64, P, P]),
        "rsx_rowx_entry_floats": (C.c_size_t, [I32, I32]),
        "rsx_rowx_pack": (C.c_int, [P, I64, I64, P, I32, I32, P, P, P, P]),
        "rsx_rowx_combine": (C.c_int, [P, I32, I64, P, I32, I32, P, P]),
        "rsx_smore_wgrad_ws_bytes": (C.c_size_t, [I64, I32, I32]),
        "rsx_smore_wgrad": (C.c_int, [I32, P, P, P, P, I64, I32, P, C.c_size_t, P]),
        "rsx_smore_infonce_ws_bytes": (C.c_size_t, [I64, I32]),
        "rsx_smore_infonce_fwd": (C.c_int, [P, P, P, P, I64, I64, I32, F32, P, P, C.c_size_t, P]),
        "rsx_smore_infonce_bwd": (C.c_int, [P, P, P, P, I64, I64, I32, F32, P, P, P, P, C.c_size_t, P]),
        "rsx_smore_infonce_fwd_total": (C.c_int, [P, P, P, P, I64, I64, I32, F32, P, P, F32, P, P, C.c_size_t, P]),
        "rsx_smore_infonce_bwd_scaled": (C.c_int, [P, P, P, P, I64, I64, I32, F32, P, I32, F32, P, P, P, C.c_size_t,
                                                   P]),
        "rsx_smore_loss_rows_bwd": (C.c_int, [P, P, P, I64, I32, F32, P, F32, P, P, P, P, P, C.c_size_t, P]),
        "rsx_adam_multi": (C.c_int, [I32, P, P, P, P, P, P, F32, F32, F32, F32, F32, P]),
        "rsx_adam_multi_scaled": (C.c_int, [I32, P, P, P, P, P, P, F32, F32, F32, F32, F32, F32, P, P, P]),
        "rsx_adam_multi_mg": (C.c_int, [I32, P, P, P, P, P, P, F32, F32, F32, F32, F32, F32, P, P, P, P, C.c_double,
                                        P]),
        "rsx_nan_gate": (C.c_int, [P, P, P, P]),
        "rsx_smore_unit_weights": (C.c_int, [P, P, P, I32, I32, P, P]),
        "rsx_mg_alpha_ws_bytes": (C.c_size_t, [I32, P]),
        "rsx_mg_alpha": (C.c_int, [I32, P, P, P, C.c_double, C.c_double, C.c_double, C.c_double, P, P, C.c_size_t, P, P]),
        "rsx_axpy_multi": (C.c_int, [I32, P, P, P, P, C.c_double, P, P, P]),
        "rsx_knn_ws_bytes": (C.c_size_t, [I64, I32]),
        "rsx_knn_graph": (C.c_int, [P, I64, I32, I32, P, P, P, P, C.c_size_t, P]),
        "rsx_adj_build_ws_bytes": (C.c_size_t, [I64, I64, I64]),
        "rsx_adj_build": (C.c_int, [P, P, I64, I64, I64, I32, P, I64, P, P, P, P, C.c_size_t, P]),
        "rsx_edge_dropout_ws_bytes": (C.c_size_t, [I64, I64, I64]),
        "rsx_edge_dropout_build": (C.c_int, [P, P, P, I64, I64, I64, P, P, P, P, P, P, P, C.c_size_t, P]),
        "rsx_smore_unit_weights_bwd": (C.c_int, [P, I64, P, P, P, I32, I32, P, P, P, P]),
        "rsx_cpu_spmm": (C.c_int, [P, P, P, I64, P, I32, P]),
        "rsx_cpu_propagate_mean": (C.c_int, [P, P, P, I64, P, I32, I32, P]),
        "rsx_cpu_layergcn_forward": (C.c_int, [P, P, P, I64, P, I32, I32, P, P, P]),
        "rsx_cpu_layergcn_backward": (C.c_int, [P, P, P, I64, P, I32, I32, P, P, P, P]),
        "rsx_cpu_bpr": (C.c_int, [I32, P, P, I64, I64, I32, P, I64, F32, F32, P, P, P]),
        "rsx_cpu_fullsort_topk": (C.c_int, [P, P, I64, P, I64, I32, P, P, I32, P, P]),
        "rsx_cpu_adam": (C.c_int, [P, P, P, P, I64, I64, F32, F32, F32, F32, F32]),
        "rsx_cpu_gcn_step_ws_floats": (C.c_size_t, [I32, I64, I32, I32, I64]),
        "rsx_cpu_gcn_step": (C.c_int, [I32, P, P, P, I64, I64, I32, I32, P, I64, F32, P, P, P, I64, F32, F32, F32,
                                       F32, F32, P, C.c_size_t, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


EXPORTED = ["rsx_version", "rsx_csr_schedule_host", "rsx_csr_schedule_rebind", "rsx_spmm_batch", "rsx_spmm", "rsx_rowwise", "rsx_bpr_ws_bytes", "rsx_bpr",
            "rsx_fullsort_ws_bytes", "rsx_fullsort_plan", "rsx_fullsort_topk", "rsx_score_dense", "rsx_sample_triplets",
            "rsx_gather_rows", "rsx_lightgcn_step", "rsx_layergcn_step", "rsx_lightgcn_forward", "rsx_sample_epoch",
            "rsx_sample_epoch_slices",
            "rsx_smore_spectral_spec_floats", "rsx_smore_spectral_fwd_ws_bytes", "rsx_smore_spectral_fwd",
            "rsx_smore_spectral_bwd",
            "rsx_smore_spectral_bwd_partials", "rsx_smore_spectral_bwd_ws_bytes", "rsx_smore_item_tiles", "rsx_smore_item_fwd",
            "rsx_topk_metrics_ws_bytes", "rsx_topk_metrics", "rsx_topk_metrics_fast", "rsx_linear_wgrad_ws_bytes", "rsx_linear_wgrad", "rsx_linear_bwd_ws_bytes", "rsx_linear_bwd", "rsx_linear_bwd_pair_ws_bytes", "rsx_linear_bwd_pair",
            "rsx_comm_unique_id_bytes", "rsx_comm_get_unique_id", "rsx_comm_init", "rsx_comm_destroy",
            "rsx_comm_init_host",
            "rsx_comm_allreduce_f32", "rsx_sharded_lightgcn_step", "rsx_sharded_lightgcn_forward", "rsx_sharded_lightgcn_flush",
            "rsx_dp_lightgcn_step", "rsx_dp_work_bytes", "rsx_comm_init_sim", "rsx_comm_sim_seconds",
            "rsx_comm_allgather_f32", "rsx_comm_allreduce_f32_start", "rsx_comm_wait",
            "rsx_smore_gates", "rsx_smore_gates_saved", "rsx_smore_pref", "rsx_smore_pref_rows", "rsx_smore_pref_rows_occ_floats", "rsx_smore_pref_rows_saved", "rsx_smore_pref_rows_saved_floats", "rsx_smore_pref_plan_words", "rsx_tag_rows", "rsx_tag_rows_next", "rsx_rowx_entry_floats", "rsx_rowx_pack", "rsx_rowx_combine", "rsx_smore_wgrad_ws_bytes", "rsx_smore_wgrad",
            "rsx_smore_infonce_ws_bytes", "rsx_smore_infonce_fwd", "rsx_smore_infonce_bwd", "rsx_smore_infonce_fwd_total", "rsx_smore_infonce_bwd_scaled", "rsx_smore_loss_rows_bwd", "rsx_adam_multi", "rsx_adam_multi_scaled", "rsx_adam_multi_mg",
            "rsx_smore_unit_weights", "rsx_smore_unit_weights_bwd", "rsx_mg_alpha_ws_bytes", "rsx_mg_alpha",
            "rsx_axpy_multi", "rsx_knn_ws_bytes", "rsx_knn_graph", "rsx_adj_build_ws_bytes", "rsx_adj_build",
            "rsx_edge_dropout_ws_bytes", "rsx_edge_dropout_build", "rsx_nan_gate",
            "rsx_cpu_spmm", "rsx_cpu_propagate_mean", "rsx_cpu_layergcn_forward", "rsx_cpu_layergcn_backward",
            "rsx_cpu_bpr", "rsx_cpu_fullsort_topk", "rsx_cpu_adam", "rsx_cpu_gcn_step_ws_floats", "rsx_cpu_gcn_step"]


def lib_path() -> str:
    return os.environ.get("RSX_LIB", _build.LIB)


def lib():
    """Load librsx.so (building it first if the sources are newer and hipcc exists)."""
    global _LIB
    if _LIB is None:
        path = lib_path()
        if not os.path.exists(path) or _build._needs_build():
            try:
                _build.build()
            except Exception as e:  # noqa: BLE001
                if not os.path.exists(path):
                    raise RuntimeError(f"librsx.so missing at {path} and the build failed: {e}") from e
        _LIB = C.CDLL(path)
        _declare(_LIB)
    return _LIB


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _ERRORS.get(rc, f"hipError {rc}")
        raise RuntimeError(f"{what} failed: {msg}")
