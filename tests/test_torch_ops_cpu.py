"""torch.ops.rsx.* registration (rsx/torch_ops.py) on the CPU: every op
exists with its schema, shape inference works under FakeTensorMode (torch.compile /
meta tracing), and CPU tensors fail loudly (the ops have GPU kernels only)."""
import pytest
import torch

import rsx  # noqa: F401  registers the ops
from rsx import torch_ops

SCHEMAS = {
    "spmm_csr": "rsx::spmm_csr(Tensor rowptr, Tensor col, Tensor val, Tensor x, SymInt n_cols) -> Tensor",
    "propagate_mean": "rsx::propagate_mean(Tensor rowptr, Tensor col, Tensor val, Tensor x, SymInt n_layers) -> Tensor",
    "fullsort_topk": ("rsx::fullsort_topk(Tensor user_emb, Tensor users, Tensor item_emb, Tensor mask_rowptr, "
                      "Tensor mask_col, SymInt k) -> (Tensor, Tensor)"),
}


def test_every_op_registered():
    for name in torch_ops.OPS:
        assert hasattr(torch.ops.rsx, name), name
    for name, schema in SCHEMAS.items():
        assert str(getattr(torch.ops.rsx, name).default._schema) == schema
    assert "Tensor(a0!) p" in str(torch.ops.rsx.adam_.default._schema)


def test_cpu_tensors_raise():
    rp = torch.tensor([0, 1, 2], dtype=torch.int64)
    col = torch.tensor([1, 0], dtype=torch.int32)
    val = torch.ones(2)
    with pytest.raises(NotImplementedError):
        torch.ops.rsx.spmm_csr(rp, col, val, torch.zeros(2, 64), 2)
    with pytest.raises(NotImplementedError):
        torch.ops.rsx.propagate_mean(rp, col, val, torch.zeros(2, 64), 3)


def test_fake_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode

    with FakeTensorMode():
        rp = torch.empty(11, dtype=torch.int64, device="cuda")
        col = torch.empty(40, dtype=torch.int32, device="cuda")
        val = torch.empty(40, device="cuda")
        x = torch.empty(7, 64, device="cuda")
        assert torch.ops.rsx.spmm_csr(rp, col, val, x, 7).shape == (10, 64)
        e = torch.empty(10, 64, device="cuda")
        assert torch.ops.rsx.propagate_mean(rp, col, val, e, 3).shape == (10, 64)
        v, i = torch.ops.rsx.fullsort_topk(torch.empty(5, 64, device="cuda"), torch.empty(3, dtype=torch.int64,
                                           device="cuda"), torch.empty(9, 64, device="cuda"), rp, col, 4)
        assert v.shape == (3, 4) and i.shape == (3, 4) and i.dtype == torch.int64
        cv, ct, cf = torch.ops.rsx.smore_spectral(torch.empty(9, 32, device="cuda"), torch.empty(64, 32, device="cuda"),
                                                  torch.empty(64, device="cuda"), torch.empty(9, 16, device="cuda"),
                                                  torch.empty(64, 16, device="cuda"), torch.empty(64, device="cuda"),
                                                  torch.empty(1, 33, 2, device="cuda"), torch.empty(1, 33, 2, device="cuda"),
                                                  torch.empty(1, 33, 2, device="cuda"), True)
        assert cv.shape == (9, 64)
