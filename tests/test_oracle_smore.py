"""The oracle's SMORE restatement (oracle.SMORECPU + smore_train_batch) against the
reference's own outputs: the d=64 fixture (raw 48/24 features) and the C5-shaped
d=128 fixture (CLIP-like 768/768).  CPU only."""
import numpy as np
import pytest
import torch

import rsx_oracle as O


def _model(z, d):
    init = {k[len("init."):]: z[k] for k in z if k.startswith("init.")}
    return O.SMORECPU(z["train_u"], z["train_i"], int(z["n_users"]), int(z["n_items"]), z["v_feat"], z["t_feat"],
                      d=d, reg_weight=1e-5, image_k=10, text_k=8, dropout=0.0, batch_size=512, init=init)


@pytest.mark.parametrize("fx,d", [("smore_small", 64), ("smore_d128_small", 128)])
def test_smore_oracle_forward_first_step(golden, fx, d):
    z = golden(fx)
    m = _model(z, d)
    with torch.no_grad():
        u, i = m.forward()
    np.testing.assert_allclose(u.numpy(), z["fwd_user"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(i.numpy(), z["fwd_item"], rtol=1e-5, atol=1e-6)
    trip = torch.from_numpy(z["epoch0_triplets"][:, :512].astype(np.int64))
    loss = m.calculate_loss(trip)
    loss.backward()
    assert abs(loss.item() - float(z["step0_loss"])) <= 1e-6 * abs(float(z["step0_loss"]))
    for n, p in m.named_parameters():
        key = "step0_grad." + n
        if key in z:
            scale = max(np.abs(z[key]).max(), 1e-12)
            np.testing.assert_allclose(p.grad.numpy(), z[key], rtol=1e-4, atol=1e-6 * scale, err_msg=n)


@pytest.mark.parametrize("fx,d", [("smore_small", 64), ("smore_d128_small", 128)])
def test_smore_oracle_epoch_with_mirror_gradient(golden, fx, d):
    z = golden(fx)
    m = _model(z, d)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    trip = z["epoch0_triplets"].astype(np.int64)
    total = 0.0
    for s in range(0, trip.shape[1], 512):
        total += O.smore_train_batch(m, opt, torch.from_numpy(trip[:, s:s + 512]), 1e-3)
    assert abs(total - float(z["epoch_losses"][0])) <= 1e-5 * abs(float(z["epoch_losses"][0]))
    for n, p in m.named_parameters():
        np.testing.assert_allclose(p.detach().numpy(), z["epoch0_param." + n], rtol=0, atol=2e-5, err_msg=n)
