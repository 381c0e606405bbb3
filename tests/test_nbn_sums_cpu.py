"""The algebra of the BN-backward sums reduced in a DGRAD epilogue (GF_NBNSUM, gemm3.hip g3_tiled_kernel NS
path; nbn.hip nbn_fin_kernel, phase 6), against torch autograd in fp64.

A raw-input Dense with one input channel (y = act(x w + b) per channel f) feeds a training-mode
BatchNormalization.  The consumer DGRAD produces dy = dL/d(BN output) and, instead of storing it, reduces per
column (position p, channel f) the eight sums

    [0] dy  [1] dy xhat  [2] a dy  [3] a xhat  [4] a  [5] a x dy  [6] a x xhat  [7] a x      (a = act'(y))

over its 128-row m tile; rows past the batch contribute zeros (their dy is zero and a is masked).  Phase 6 adds
the (m tile, position) slots of a channel and forms dgamma, dbeta, dW, db.  This test mirrors both steps in
fp64 and checks them against autograd of the same forward pass, for the three activations the kernel
specialises (reference semantics: common/BatchNormalizationF16.py, training-mode batch statistics).
"""
import numpy as np
import pytest
import torch


def _act(v, act):
    if act == "relu":
        return torch.relu(v)
    if act == "sigmoid":
        return torch.sigmoid(v)
    return v


def _act_grad(y, act):
    if act == "relu":
        return (y > 0).double()
    if act == "sigmoid":
        return y * (1 - y)
    return torch.ones_like(y)


def _epilogue_sums(x, dy, w, b, mean, invstd, act, tile=128):
    """Per (m tile, position, channel) slots of the 8 sums, as the NS epilogue stores them (zero-padded tail)."""
    B, P = x.shape
    F = w.shape[0]
    mt = -(-B // tile)
    pad = mt * tile - B
    xp = torch.cat([x, x[-1:].expand(pad, P)]) if pad else x          # staged rows clamp to the last row
    dyp = torch.cat([dy, torch.zeros(pad, P, F, dtype=dy.dtype)]) if pad else dy
    valid = (torch.arange(mt * tile) < B).double()[:, None, None]
    y = _act(xp[..., None] * w + b, act)
    a = _act_grad(y, act) * valid
    xh = (y - mean) * invstd
    xv = xp[..., None]
    terms = [dyp, dyp * xh, a * dyp, a * xh, a, a * xv * dyp, a * xv * xh, a * xv]
    # [mt][P][F][8]
    return torch.stack([t.reshape(mt, tile, P, F).sum(1) for t in terms], -1)


def _phase6(part, R, gamma, invstd):
    S = part.sum((0, 1))                      # [F][8]
    gg = gamma * invstd
    ma, mb = S[:, 0] / R, S[:, 1] / R
    dgamma, dbeta = S[:, 1], S[:, 0]
    dw = gg * (S[:, 5] - mb * S[:, 6] - ma * S[:, 7])
    db = gg * (S[:, 2] - mb * S[:, 3] - ma * S[:, 4])
    return dw, db, dgamma, dbeta


@pytest.mark.parametrize("act", ["relu", "sigmoid", "linear"])
@pytest.mark.parametrize("B", [128, 750])
def test_nbn_epilogue_sums_give_bn_and_dense_gradients(act, B):
    g = torch.Generator().manual_seed(11)
    P, F, eps = 7, 5, 1e-3
    x = torch.randint(0, 2, (B, P), generator=g).double() + 0.1 * torch.randn(B, P, generator=g, dtype=torch.float64)
    w = torch.randn(F, generator=g, dtype=torch.float64).requires_grad_()
    b = (0.1 * torch.randn(F, generator=g, dtype=torch.float64)).requires_grad_()
    gamma = (1 + 0.2 * torch.randn(F, generator=g, dtype=torch.float64)).requires_grad_()
    beta = (0.1 * torch.randn(F, generator=g, dtype=torch.float64)).requires_grad_()
    dout = torch.randn(B, P, F, generator=g, dtype=torch.float64)

    y = _act(x[..., None] * w + b, act)                       # [B][P][F]
    mean = y.mean((0, 1))
    var = y.var((0, 1), unbiased=False)
    invstd = 1 / torch.sqrt(var + eps)
    out = (y - mean) * invstd * gamma + beta
    (out * dout).sum().backward()

    with torch.no_grad():
        part = _epilogue_sums(x, dout, w, b, mean, invstd, act)
        dw, db, dgamma, dbeta = _phase6(part, B * P, gamma, invstd)
    for got, ref in ((dw, w.grad), (db, b.grad), (dgamma, gamma.grad), (dbeta, beta.grad)):
        np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-9, atol=1e-9)
