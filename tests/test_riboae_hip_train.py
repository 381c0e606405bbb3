"""RiboAE training on the in-house HIP kernels (riboae/hip_trainer.py) against the
fp32 PyTorch model: one step's loss and every parameter gradient, bitwise reproducibility, and a
training run's loss curve against the torch path (reference: ribosomal_autoencoder/training.py:40-48,
model.py:17-104)."""
import copy

import numpy as np
import pytest
import torch

from serann.models.riboae import ConcreteGAE

pytestmark = pytest.mark.gpu


def _model(seed=0):
    torch.manual_seed(seed)
    return ConcreteGAE(genotype_length=20, max_phenotype_length=32, vocabulary_size=12, embedding_dim=16,
                       genotype_alphabet_size=2, prior_temperature=0.1)


def _batch(B=48, seed=1):
    g = torch.Generator().manual_seed(seed)
    x = torch.randint(0, 12, (B, 32), generator=g)
    u = torch.rand(B, 20, 2, generator=g)
    return x, u


SPEC_OF = {"emb": "inference_net.embedding.weight", "c1": "inference_net.conv1.weight",
           "c1_b": "inference_net.conv1.bias", "c2": "inference_net.conv2.weight", "c3": "inference_net.conv3.weight",
           "dense": "inference_net.dense.weight", "dense_b": "inference_net.dense.bias",
           "g1": "generative_net.conv.weight", "g2": "generative_net.dense.weight", "g2_b": "generative_net.dense.bias",
           "bn0_g": "inference_net.bn0.weight", "bn0_be": "inference_net.bn0.bias", "bn1_g": "inference_net.bn1.weight",
           "bn3_be": "inference_net.bn3.bias", "gbn1_g": "generative_net.bn1.weight",
           "gbn2_g": "generative_net.bn2.weight", "gbn2_be": "generative_net.bn2.bias"}


def _grads(model, x, u, autocast):
    out = model.train().compute_loss(x, 0.3, 0.05, noise=u) if not autocast else None
    if autocast:
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
            out = model.train().compute_loss(x, 0.3, 0.05, noise=u)
    g = torch.autograd.grad(out["loss"].float(), list(model.parameters()))
    return {n: t.detach().float().cpu().numpy().astype(np.float64) for (n, _), t in zip(model.named_parameters(), g)}, \
        {k: float(v) for k, v in out.items()}


def _err(got, want):
    err = np.linalg.norm(got - want) / max(np.linalg.norm(want), 1e-30)
    cos = float(np.dot(got.ravel(), want.ravel()) / max(np.linalg.norm(got) * np.linalg.norm(want), 1e-30))
    return err, cos


def test_hip_step_gradients_match_fp32_oracle(monkeypatch):
    """Every parameter gradient of one HIP step against the fp32 CPU oracle: within 5 % (cosine > 0.998),
    with an absolute floor of 0.2 % of the largest gradient element for sums that cancel (the gamma /
    beta of the one-channel BatchNorm after the embedding sum 24k bf16 terms)."""
    from serann.riboae.hip_trainer import HipRiboTrainer
    m = _model()
    x, u = _batch()
    monkeypatch.setenv("SERANN_RIBOAE_HIP", "0")
    ref, out = _grads(copy.deepcopy(m), x, u, autocast=False)                      # CPU fp32
    monkeypatch.delenv("SERANN_RIBOAE_HIP")
    m = m.cuda().train()
    tr = HipRiboTrainer(m, device="cuda")
    hip, res = tr.debug_grads(x.cuda(), 0.3, 0.05, u.cuda())
    assert abs(res["loss"] - out["loss"]) < 1e-2 * abs(out["loss"]), (res, out)
    assert abs(res["kld"] - out["kld"]) < 1e-2 * abs(out["kld"]) + 1e-3
    gmax = max(float(np.abs(g).max()) for g in ref.values())
    for k, tname in SPEC_OF.items():
        want, got = ref[tname], hip[k]
        assert got.shape == want.shape, (k, got.shape, want.shape)
        if np.linalg.norm(want) < 1e-4 * gmax * np.sqrt(want.size):
            assert np.abs(got).max() < 1e-2 * gmax, k           # mathematically ~0 (bias before a BN)
            continue
        e_h, c_h = _err(got, want)
        floor = 2e-3 * gmax * np.sqrt(want.size)
        if np.linalg.norm(got - want) < floor:
            continue
        assert e_h < 0.05 and c_h > 0.998, (k, e_h, c_h)


def test_hip_training_is_bitwise_reproducible():
    from serann.riboae.hip_trainer import HipRiboTrainer
    x, u = _batch(32, seed=3)
    arenas = []
    for _ in range(2):
        m = _model(2).cuda().train()
        tr = HipRiboTrainer(m, device="cuda")
        for i in range(3):
            tr.step(x.cuda(), 0.3, 0.05, 3e-4, noise=u.cuda())
        torch.cuda.synchronize()
        arenas.append((tr.p.cpu(), tr.stats.cpu()))
    assert torch.equal(arenas[0][0], arenas[1][0]) and torch.equal(arenas[0][1], arenas[1][1])


def test_hip_fused_adam_matches_the_arena_pass(monkeypatch):
    """The single-split Dense WGRADs apply Adam in their epilogue (GF_ADAM) and the arena pass skips those
    parameters: after 3 steps every parameter, moment and bf16 copy is bitwise the unfused run's."""
    from serann.riboae.hip_trainer import HipRiboTrainer
    x, u = _batch(32, seed=4)
    out = []
    for fuse in ("1", "0"):
        monkeypatch.setenv("SERANN_FUSE_ADAM", fuse)
        m = _model(5).cuda().train()
        tr = HipRiboTrainer(m, device="cuda")
        for _ in range(3):
            tr.step(x.cuda(), 0.3, 0.05, 3e-4, noise=u.cuda())
        torch.cuda.synchronize()
        pl = tr.plans[(32, True)]
        out.append((tr.p.cpu(), tr.m.cpu(), tr.v.cpu(), tr.pbf.cpu(), pl.skip is not None))
    assert out[0][4] and not out[1][4]                   # the fused run did fuse
    for a, b in zip(out[0][:4], out[1][:4]):
        assert torch.equal(a, b)


def test_hip_loss_curve_matches_torch_path(tmp_path):
    """200 scheduled training steps (trainer.train) on the HIP kernels and on the torch path: the
    smoothed loss at the end agrees within 2 %, and the HIP run leaves a loadable checkpoint."""
    from serann.riboae.io import load_checkpoint
    from serann.riboae.trainer import train
    rng = np.random.default_rng(0)
    # a learnable token distribution: a few templates with random substitutions
    base = rng.integers(0, 12, (6, 32))
    toks = base[rng.integers(0, 6, 2048)]
    flip = rng.random(toks.shape) < 0.1
    toks = np.where(flip, rng.integers(0, 12, toks.shape), toks)
    curves = {}
    for eng in ("hip", "torch"):
        torch.manual_seed(7)
        m = _model(4)
        curves[eng] = np.array(train(f"r_{eng}", m, toks, None, str(tmp_path), batch_size=128, min_backup_interval=10 ** 9,
                                     max_steps=200, device="cuda", log=lambda *a: None, demo_every=0, engine=eng))
    a, b = curves["hip"][-40:].mean(), curves["torch"][-40:].mean()
    assert curves["hip"][-40:].mean() < 0.8 * curves["hip"][:10].mean()       # it learns
    assert abs(a - b) < 0.02 * abs(b), (a, b)
    m2, ck = load_checkpoint(str(tmp_path / "r_hip_b200.pt"))
    assert ck["step"] == 200 and "m" in ck["optimizer"] and "m_arena" not in ck["optimizer"]


def test_checkpoint_moments_cross_engines(tmp_path):
    """A HIP checkpoint resumes on the torch engine and a torch checkpoint on the HIP engine with the
    same Adam moments and step count (the formats used not to convert)."""
    from serann.riboae.hip_trainer import HipRiboTrainer
    from serann.riboae.trainer import ScheduledKerasAdam
    x, u = _batch(32, seed=5)
    m = _model(6).cuda().train()
    tr = HipRiboTrainer(m, device="cuda")
    for _ in range(3):
        tr.step(x.cuda(), 0.3, 0.05, 3e-4, noise=u.cuda())
    st = tr.state_dict()
    assert st["t"] == 3 and len(st["m"]) == len(list(m.parameters()))
    # HIP -> torch: the per-parameter lists are the arena moments in torch layout
    opt = ScheduledKerasAdam(list(m.parameters()), lr=3e-4, eps=1e-7)
    opt.load_state_dict(st)
    assert opt.t == 3
    for a, b in zip(opt.m, tr._moment_views(tr.m)):
        assert torch.equal(a.cpu(), b.cpu())
    # torch -> HIP: a fresh trainer restores the moments from the lists alone
    m2 = _model(6).cuda().train()
    tr2 = HipRiboTrainer(m2, device="cuda")
    tr2.load_state_dict({"t": opt.t, "m": opt.state_dict()["m"], "v": opt.state_dict()["v"]})
    n = tr.pa.size
    assert int(tr2.step_i.item()) == 3
    assert torch.equal(tr2.m[:n].cpu(), tr.m[:n].cpu()) and torch.equal(tr2.v[:n].cpu(), tr.v[:n].cpu())


def test_fused_and_unfused_plans_share_buffers():
    """The training step's plan (fused Adam) and the debug / update=False plan of the same batch size share one set of
    activation buffers and workspaces: a debug_grads call after training allocates no second set."""
    from serann.riboae.hip_trainer import HipRiboTrainer
    m = _model()
    x, u = _batch()
    tr = HipRiboTrainer(m, device="cuda")
    tr.step(x, 0.3, 0.05, 1e-3, noise=u)
    torch.cuda.synchronize()
    before = torch.cuda.memory_allocated()
    tr.debug_grads(x, 0.3, 0.05, u)
    torch.cuda.synchronize()
    assert len(tr.plans) == 2 and len(tr._bufs) == 1
    pf, pu = tr.plans[(48, True)], tr.plans[(48, False)]
    assert pf.buf is pu.buf and pf.mean is pu.mean
    # (only the unfused plan's own descriptors, tile tables and split slabs are new)
    assert torch.cuda.memory_allocated() - before < 16 << 20, torch.cuda.memory_allocated() - before
