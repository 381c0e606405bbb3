"""Ribosomal autoencoder: model semantics, schedules, trainer/checkpoint (CPU) and the HIP encode /
decode inference paths vs. the fp32 PyTorch model (GPU).

Reference: ribosomal_autoencoder/model.py:10-134, ribosomal_autoencoder/training.py:51-101,
evolutionary_experiment/logic/ribosomal_autoencoder.py:116-124.  No trained reference SavedModel ships
with the reference repo, so parity is pinned against the formulas, not against published weights."""
import math
import os

import numpy as np
import pytest
import torch

from serann.models.riboae import ConcreteGAE, DeterministicGAE, build_model, gumbel_log_prob
from serann.riboae import trainer as T
from serann.riboae.io import load_checkpoint, save_checkpoint


def _small(kind="concrete", **kw):
    hp = dict(genotype_length=12, max_phenotype_length=20, vocabulary_size=9, embedding_dim=12)
    hp.update(kw)
    torch.manual_seed(0)
    return build_model(kind, **hp)


def _randomise_bn(model, seed=0):
    g = torch.Generator().manual_seed(seed)
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm1d):
            with torch.no_grad():
                m.running_mean.copy_(torch.randn(m.running_mean.shape, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.running_var.shape, generator=g) + 0.5)
                m.weight.copy_(torch.rand(m.weight.shape, generator=g) + 0.5)
                m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.1)


def test_shapes_and_log_probs():
    m = _small()
    x = torch.randint(0, 9, (3, 20))
    logits = m.inference_net(x)
    assert logits.shape == (3, 12, 2)
    z = torch.softmax(logits, -1)
    logp = m.generative_net(z)
    assert logp.shape == (3, 20, 9)
    assert torch.allclose(logp.exp().sum(-1), torch.ones(3, 20), atol=1e-5)
    # _decode = sum over the sequence of the log-probability of the target token (model.py:54-59)
    ref = torch.gather(logp, -1, x.unsqueeze(-1)).squeeze(-1).sum(-1)
    assert torch.allclose(m._decode(x, z), ref, atol=1e-5)


def test_default_dims_match_reference_flatten_sizes():
    m = ConcreteGAE()
    assert m.inference_net.flat == 342 * 42 * 16 == 229_824          # model.py:29-31
    assert m.generative_net.flat == 96 * 32 == 3072                   # model.py:38-41
    assert m.inference_net.dense.out_features == 200
    assert m.generative_net.dense.out_features == 350 * 40


def test_gumbel_prior_and_loss_formula():
    m = _small(prior_temperature=0.01)
    x = torch.randint(0, 9, (4, 20))
    torch.manual_seed(1)
    out = m.compute_loss(x, temperature=0.3, kld_weight=0.05)
    assert set(out) == {"loss", "nll", "kld"}
    # recompute with the same RNG draw: NELBO = -mean(log p(x|z) - w * KL)  (model.py:88-100)
    torch.manual_seed(1)
    z, logq, logp = m._encode(x, 0.3)
    lpx = m._decode(x, z)
    kl = (logq - logp).flatten(1).sum(1)
    assert torch.allclose(out["loss"], -(lpx - 0.05 * kl).mean(), atol=1e-4)
    assert torch.allclose(out["nll"], -lpx.mean(), atol=1e-4)
    # the prior is Gumbel(log(1/A)/tp, 1/tp) (model.py:70-71)
    s = torch.tensor([0.3])
    tp = 0.01
    expect = gumbel_log_prob(s, math.log(0.5) / tp, 1 / tp)
    zz = (s - math.log(0.5) / tp) * tp
    assert torch.allclose(expect, -(zz + torch.exp(-zz)) - math.log(1 / tp))


def test_deterministic_gae_loss_is_nll():
    m = _small("deterministic")
    assert isinstance(m, DeterministicGAE)
    x = torch.randint(0, 9, (2, 20))
    out = m.compute_loss(x)
    assert torch.allclose(out["loss"], out["nll"]) and float(out["kld"]) == 0.0


def test_schedules_match_reference():
    # training.py:59-64: logspace(log10(.3), -3, 5e6), logspace(log10(3e-4), log10(2e-5), 1e6),
    # linspace(0, .2, 1e7) ** 2, indexed by the 1-based batch number
    assert math.isclose(T.temperature_at(0), 0.3, rel_tol=1e-9)
    assert math.isclose(T.temperature_at(T.TEMPERATURE_STEPS - 1), 1e-3, rel_tol=1e-9)
    assert math.isclose(T.temperature_at(10 ** 9), 1e-3, rel_tol=1e-9)
    assert math.isclose(T.learning_rate_at(0), 3e-4, rel_tol=1e-9)
    assert math.isclose(T.learning_rate_at(T.LEARNING_RATE_STEPS - 1), 2e-5, rel_tol=1e-9)
    assert T.kld_weight_at(0) == 0.0
    assert math.isclose(T.kld_weight_at(T.KLD_STEPS - 1), 0.04, rel_tol=1e-9)
    mid = T.TEMPERATURE_STEPS // 2
    ref = np.logspace(np.log10(0.3), -3, 11)[5]
    assert math.isclose(T.temperature_at(mid), ref, rel_tol=1e-5)


def test_trainer_checkpoint_and_resume(tmp_path):
    m = _small()
    data = np.random.default_rng(0).integers(0, 9, (64, 20))
    logs = []
    hist = T.train("ribo", m, data, None, str(tmp_path), batch_size=16, min_backup_interval=2, max_steps=6,
                   log=lambda *a: logs.append(" ".join(map(str, a))), log_every=2)
    assert len(hist) == 6 and all(np.isfinite(hist))
    cks = sorted(os.listdir(tmp_path))
    assert cks and all(c.startswith("ribo_b") and c.endswith(".pt") for c in cks)
    # best-loss backups replace the previous backup: at most the best + the final checkpoint remain
    assert len(cks) <= 2
    last = max(cks, key=lambda c: int(c[len("ribo_b"):-3]))
    model, ck = load_checkpoint(os.path.join(tmp_path, last))
    assert ck["step"] == 6 and ck["optimizer"]["t"] == 6
    for a, b in zip(model.state_dict().values(), m.state_dict().values()):
        assert torch.equal(a, b)
    hist2 = T.train("ribo", model, data, None, str(tmp_path), batch_size=16, max_steps=2,
                    resume_path=os.path.join(tmp_path, last), log=lambda *a: None)
    assert len(hist2) == 2
    assert any(c.endswith("_b8.pt") for c in os.listdir(tmp_path))


def test_encode_decode_tokens_cpu_roundtrip_shapes():
    m = _small()
    m.eval()
    toks = np.random.default_rng(1).integers(0, 9, (5, 20))
    bits = m.encode_tokens(toks)
    assert bits.shape == (5, 12) and set(np.unique(bits)) <= {0, 1}
    seq = m.decode_tokens(bits)
    assert seq.shape == (5, 20) and seq.max() < 9


def test_checkpoint_roundtrip_weights_only(tmp_path):
    m = _small()
    p = tmp_path / "x.pt"
    save_checkpoint(p, m, "concrete", 3, None, {"loss": 1.0})
    m2, ck = load_checkpoint(p)
    assert ck["kind"] == "concrete" and ck["step"] == 3
    assert m2.hparams == m.hparams


def test_decoder_near_tie_rescoring_cpu():
    """The decoder's fp32 re-decision of near-tie positions, driven by an emulation of the bf16 MFMA
    decode on the CPU (bf16 conv output and weights, fp32 products and sums): the emulated MFMA argmax
    flips some tokens against the fp32 model; after ``_rescore`` none are left."""
    from serann.ops.riboae_ops import HipRiboDecoder
    torch.manual_seed(0)
    m = ConcreteGAE().eval()
    _randomise_bn(m)
    dec = HipRiboDecoder(m, "cpu")
    B, L, V = 96, dec.L, dec.V
    bits = torch.randint(0, 2, (B, 100))
    with torch.no_grad():
        z = torch.nn.functional.one_hot(bits, 2).float()
        ref = m.generative_net(z).argmax(-1)
        h = torch.nn.functional.conv1d(z.permute(0, 2, 1), dec.w1f, dec.b1f).permute(0, 2, 1).reshape(B, -1)
        hb = h.bfloat16()
        logits = hb.float() @ dec.w2.float().T + dec.b2
    raw = logits.view(B, L, V).argmax(-1)
    pl = {"logits": logits.contiguous(), "h": hb.reshape(-1)}
    out = raw.clone()
    dec._rescore(bits, pl, out)
    assert int((raw != ref).sum()) > 0                       # the emulated bf16 path does flip tokens
    assert int((out != ref).sum()) == 0, float((out == ref).float().mean())


# ------------------------------------------------------------------------------------------------
# GPU: HIP inference paths vs. the fp32 PyTorch model (eval mode, randomised BN statistics so the
# BatchNormalization folding is exercised)
@pytest.mark.gpu
def test_hip_decoder_matches_torch():
    """bf16 MFMA decode + fp32 re-decision of near-tie positions agrees with the fp32 model (CPU) on
    >= 99.99 % of tokens (the MFMA path alone flips ~0.3 %)."""
    import copy
    from serann.ops.riboae_ops import HipRiboDecoder
    torch.manual_seed(0)
    m = ConcreteGAE().eval()
    _randomise_bn(m)
    m_cpu = copy.deepcopy(m)
    m = m.cuda()
    bits = torch.randint(0, 2, (512, 100))
    dec = HipRiboDecoder(m, "cuda")
    out = dec(bits.cuda()).cpu()
    with torch.no_grad():
        ref_logp = m_cpu.generative_net(torch.nn.functional.one_hot(bits, 2).float())
    ref = ref_logp.argmax(-1)
    agree = float((out == ref).float().mean())
    assert agree >= 0.9999, agree
    # the MFMA argmax alone (before the rescoring) disagrees where the margin is within bf16 rounding
    raw = dec._plans[512]["out"].long().cpu()
    top2 = ref_logp.topk(2, -1).values
    margin = (top2[..., 0] - top2[..., 1])
    assert int(((raw != ref) & (margin > 0.05)).sum()) == 0


@pytest.mark.gpu
def test_hip_encoder_matches_torch():
    from serann.ops.riboae_ops import HipRiboEncoder
    torch.manual_seed(0)
    m = ConcreteGAE().eval()
    _randomise_bn(m, 3)
    m = m.cuda()
    toks = torch.randint(0, 40, (70, 350), device="cuda")
    enc = HipRiboEncoder(m, "cuda", chunk=48)            # two chunks: 48 + 22 sequences
    torch.cuda.synchronize()
    logits = enc.logits(toks)
    with torch.no_grad():
        ref = m.inference_net(toks)
    assert logits.shape == ref.shape == (70, 100, 2)
    rel = float((logits.double() - ref.double()).norm() / ref.double().norm())
    assert rel < 2e-2, rel
    bits = enc(toks)
    refb = ref.argmax(-1)
    margin = (ref[..., 0] - ref[..., 1]).abs()
    scale = float(ref.abs().mean())
    assert int(((bits != refb) & (margin > 0.05 * scale)).sum()) == 0
    # the numpy API takes the HIP path on a GPU
    np.testing.assert_array_equal(m.encode_tokens(toks.cpu().numpy(), device="cuda"), bits.cpu().numpy())


@pytest.mark.gpu
def test_hip_categorical_loglik_matches_torch():
    """K37: fused log-softmax + gather + sum over the sequence, forward and backward."""
    from serann.ops.riboae_ops import categorical_loglik
    torch.manual_seed(0)
    z = (torch.randn(7, 350, 40, device="cuda") * 3).requires_grad_(True)
    x = torch.randint(0, 40, (7, 350), device="cuda")
    g = torch.randn(7, device="cuda")
    out = categorical_loglik(z, x)
    (out * g).sum().backward()
    dz = z.grad.clone()
    z.grad = None
    ref = torch.gather(torch.log_softmax(z, -1), -1, x.unsqueeze(-1)).squeeze(-1).sum(-1)
    (ref * g).sum().backward()
    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-3)
    assert torch.allclose(dz, z.grad, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_hip_concrete_sample_matches_torch():
    """K36: Gumbel sample + softmax + KL(q||p) forward and the reparameterised backward, on given
    uniforms, vs. the torch formulas of ConcreteGAE._encode (model.py:70-86, 95)."""
    from serann.ops.riboae_ops import concrete_sample
    torch.manual_seed(0)
    B, G, A, t, tp = 9, 100, 2, 0.3, 0.1
    logits = (torch.randn(B, G, A, device="cuda") * 2).requires_grad_(True)
    u = torch.rand(B, G, A, device="cuda")
    gz = torch.randn(B, G, A, device="cuda")
    gk = torch.randn(B, device="cuda")
    z, kl = concrete_sample(logits, t, tp, u)
    ((z * gz).sum() + (kl * gk).sum()).backward()
    d = logits.grad.clone()
    logits.grad = None
    uc = u.clamp(1e-20, 1 - 1e-7)
    s = logits / t - (1 / t) * torch.log(-torch.log(uc))
    logq = gumbel_log_prob(s, logits / t, 1 / t)
    logp = gumbel_log_prob(s, math.log(1 / A) / tp, 1 / tp)
    zr, klr = torch.softmax(s, -1), (logq - logp).flatten(1).sum(1)
    ((zr * gz).sum() + (klr * gk).sum()).backward()
    assert torch.allclose(z, zr, rtol=1e-4, atol=1e-5)
    assert torch.allclose(kl, klr, rtol=1e-4, atol=1e-4 * float(klr.detach().abs().mean()))
    assert torch.allclose(d, logits.grad, rtol=1e-3, atol=1e-3 * float(logits.grad.abs().max()))
    # in-kernel Philox draws: reproducible under torch.manual_seed, different otherwise, and the
    # softmax codes sum to one
    torch.manual_seed(1)
    z1, _ = concrete_sample(logits.detach(), t, tp)
    torch.manual_seed(1)
    z2, _ = concrete_sample(logits.detach(), t, tp)
    z3, _ = concrete_sample(logits.detach(), t, tp)
    assert torch.equal(z1, z2) and not torch.equal(z1, z3)
    assert torch.allclose(z1.sum(-1), torch.ones(B, G, device="cuda"), atol=1e-5)


@pytest.mark.gpu
def test_riboae_loss_uses_hip_path_and_matches(monkeypatch):
    torch.manual_seed(5)
    m = ConcreteGAE().cuda()
    x = torch.randint(0, 40, (16, 350), device="cuda")
    u = torch.rand(16, 100, 2, device="cuda")
    a = m.compute_loss(x, 0.3, 0.05, noise=u)
    ga = torch.autograd.grad(a["loss"], list(m.parameters()))
    monkeypatch.setenv("SERANN_RIBOAE_HIP", "0")
    b = m.compute_loss(x, 0.3, 0.05, noise=u)
    gb = torch.autograd.grad(b["loss"], list(m.parameters()))
    for k in ("loss", "nll", "kld"):
        assert torch.allclose(a[k], b[k], rtol=1e-3, atol=1e-3), (k, a[k], b[k])
    # biases feeding a BatchNorm have a mathematically-zero gradient (rounding noise): absolute
    # tolerance from the largest gradient of the whole model
    gmax = max(float(g.abs().max()) for g in gb)
    for x1, x2 in zip(ga, gb):
        assert torch.allclose(x1, x2, rtol=1e-2, atol=1e-4 * gmax)


def test_arena_only_optimizer_state_restarts_adam_cpu():
    """An arena-only (old HIP) optimizer state on the torch engine: Adam restarts at t = 0 with zero
    moments instead of keeping a large t over fresh moments (trainer.py)."""
    from serann.riboae.trainer import ScheduledKerasAdam
    p = [torch.nn.Parameter(torch.ones(3)), torch.nn.Parameter(torch.ones(2, 2))]
    opt = ScheduledKerasAdam(p, lr=1e-3, eps=1e-7)
    opt.m[0].fill_(5.0)
    opt.t = 7
    opt.load_state_dict({"t": 900, "m_arena": torch.zeros(8), "v_arena": torch.zeros(8)})
    assert opt.t == 0 and float(opt.m[0].abs().sum()) == 0.0
    opt.load_state_dict({"t": 4, "m": [torch.full((3,), 2.0), torch.full((2, 2), 3.0)],
                         "v": [torch.ones(3), torch.ones(2, 2)]})
    assert opt.t == 4 and float(opt.m[1][0, 0]) == 3.0
