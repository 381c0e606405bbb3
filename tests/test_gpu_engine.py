"""HIP grouped engine vs. the torch fp32 oracle (same parameters, same batch).

Numerics contract: bf16 operands / activations with fp32 accumulation and fp32 master weights, so
forward logits and gradients are compared by relative Frobenius error.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from serann.genome.interpreter import interpret
from serann.models.organism import Organism, init_params

from .archs import ARCHS

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-12)


def _batch(B, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.random((B, 28, 28, 1)).astype(np.float32)
    g = rng.integers(0, 2, (B, 100)).astype(np.float32)
    y = rng.integers(0, 10, B).astype(np.int64)
    return x, g, y


def _oracle(ir, params, x, g, y):
    dev = "cpu"          # fp32 oracle on the CPU: independent of the GPU library paths
    org = Organism(ir, params, device=dev)
    xb = torch.as_tensor(x, device=dev)
    gb = torch.as_tensor(g, device=dev)
    yb = torch.as_tensor(y, device=dev)
    cl, rl = org(xb, gb[..., None], training=True)
    lb = ir.loss_balance
    loss = lb * F.cross_entropy(cl, yb) + (1 - lb) * ((torch.sigmoid(rl) - gb) ** 2).mean()
    loss.backward()
    grads = {}
    for k, p in org.params.items():
        nid, name = k[1:].split("_", 1)
        grads.setdefault(int(nid), {})[name] = p.grad.detach().cpu().numpy()
    logits = torch.cat([cl, rl], 1).detach().cpu().numpy()
    return logits, grads


def _oracle_dev(ir, params, x, g, y, device, dtype):
    org = Organism(ir, params, device=device, dtype=dtype)
    xb = torch.as_tensor(x, device=device, dtype=dtype)
    gb = torch.as_tensor(g, device=device, dtype=dtype)
    yb = torch.as_tensor(y, device=device)
    cl, rl = org(xb, gb[..., None], training=True)
    lb = ir.loss_balance
    loss = lb * F.cross_entropy(cl.float(), yb) + (1 - lb) * ((torch.sigmoid(rl.float()) - gb.float()) ** 2).mean()
    loss.backward()
    grads = {}
    for k, p in org.params.items():
        nid, name = k[1:].split("_", 1)
        grads.setdefault(int(nid), {})[name] = p.grad.detach().float().cpu().numpy()
    return grads


def _check_vs_torch_bf16(name, B, seed, perturbed_bound=None):
    from serann.engine.hip_engine import HipPopulationEngine
    ir = interpret(ARCHS[name])
    params = init_params(ir, 7)
    x, g, y = _batch(B, seed=seed)
    eng = HipPopulationEngine([ir], [0], device="cuda", params=[params])
    grads, metrics = eng.debug_train_step(x, g, y)
    ref_logits, ref = _oracle(ir, params, x, g, y)
    assert _rel(eng.debug_logits()[0], ref_logits) < 1e-2
    bf = _oracle_dev(ir, params, x, g, y, "cuda", torch.bfloat16)
    # a second, equally valid bf16 computation: the trainable parameters moved by half a bf16 ulp (random
    # sign).  At B = 96 a gradient is dominated by the few ReLU units whose pre-activation sits within bf16
    # noise of zero: which side a computation lands on is luck, and one flipped unit of one sample moves
    # every upstream gradient by percents (gchain_f64_bn_dense seed 0: the fused chain's forward is as close
    # to fp32 as torch's -- Dense(24) pre-activations 3.3e-3 relative for both -- but it lands four units on
    # the other side of zero, 5.8 % on the first Conv1D kernel against torch's 1.9 %; profiles/r5/
    # relu_knife_edge.txt).  The bound is the worse of the two references.
    # (B = 96 only, where the knife-edge analysis applies: at the production batch the single reference bounds)
    if perturbed_bound is None:
        perturbed_bound = B < 750
    if perturbed_bound:
        rng = np.random.default_rng(1000 + seed)
        params2 = {nid: {k: (v * (1 + 2.0 ** -9 * rng.choice([-1.0, 1.0], size=v.shape))).astype(v.dtype)
                         if k in ("kernel", "bias", "gamma", "beta") else v for k, v in d.items()}
                   for nid, d in params.items()}
        bf2 = _oracle_dev(ir, params2, x, g, y, "cuda", torch.bfloat16)
    else:
        bf2 = bf
    hip = eng.export_arena(0, grads)
    gmax = max(float(np.abs(v).max()) for d in ref.values() for v in d.values())
    for nid, d in ref.items():
        for k, v in d.items():
            a_h = np.linalg.norm(np.asarray(hip[nid][k], np.float64) - v)
            a_b = max(np.linalg.norm(np.asarray(bf[nid][k], np.float64) - v),
                      np.linalg.norm(np.asarray(bf2[nid][k], np.float64) - v))
            floor = 1e-3 * gmax * np.sqrt(v.size)
            if k == "bias" and "kernel" in d:
                # the bias of a layer feeding a BatchNormalization has a mathematically zero gradient; the
                # engine's sum of bf16 BN dx over the batch leaves noise on the layer's scale (as the
                # reference's pure-fp16 Keras does)
                floor = max(floor, 0.02 * np.linalg.norm(d["kernel"]))
            assert a_h < 1.5 * a_b + 0.01 * np.linalg.norm(v) + floor, (name, B, nid, k, a_h, a_b, np.linalg.norm(v))
    assert metrics[0, 3] == B
    eng.close()


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("name", sorted(ARCHS))
def test_train_step_b750_as_accurate_as_torch_bf16(name, seed):
    """Production batch (750): every gradient of the HIP engine is within 1.5x (+1 %) of the error that
    PyTorch's own bf16 computation of the same organism (bf16 GEMM operands on the GPU) makes against the
    fp32 CPU oracle, and the logits within 1 % of the oracle.  Sums that cancel to ~1e-5 of their terms
    (the beta of a BatchNormalization on the raw image: sum dy ~ 3e-5 of sum |dy|) keep an absolute floor
    of 0.1 % of the largest gradient element: the engine stores activations in bf16 (the torch reference
    keeps them fp32), so such a sum is bf16 noise in the engine (scripts/debug_bn_input.py)."""
    _check_vs_torch_bf16(name, 750, seed)


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("name", sorted(ARCHS))
def test_train_step_b96_as_accurate_as_torch_bf16(name, seed):
    """The same criterion at a small batch (96 rows: BatchNorm statistics and the loss mean over few rows,
    remainder-step shapes), every input seed.  (Round 4 pinned one seed per batch and parked the fused
    genotype chain's B = 96 seed-0 miss as an xfail: it is ReLU knife-edge luck, see _check_vs_torch_bf16.)"""
    _check_vs_torch_bf16(name, 96, seed)


def test_population_grouping_matches_single():
    """Grouping heterogeneous organisms into shared launches must not change any organism -- bitwise:
    every reduction split is a function of the organism's own problem (hip_ops: per-problem
    decomposition) and partial sums meet in order-free fixed point (csrc/hip/common.h)."""
    from serann.engine.hip_engine import HipPopulationEngine
    names = sorted(ARCHS)
    irs = [interpret(ARCHS[n]) for n in names]
    params = [init_params(ir, 11 + i) for i, ir in enumerate(irs)]
    x, g, y = _batch(64, seed=3)
    eng = HipPopulationEngine(irs, list(range(len(irs))), device="cuda", params=params)
    grads, _ = eng.debug_train_step(x, g, y)
    logits = eng.debug_logits()
    for i, ir in enumerate(irs):
        single = HipPopulationEngine([ir], [0], device="cuda", params=[params[i]])
        g1, _ = single.debug_train_step(x, g, y)
        l1 = single.debug_logits()[0]
        assert np.array_equal(logits[i], l1), names[i]
        a, b = eng.export_arena(i, grads), single.export_arena(0, g1)
        for nid in b:
            for k in b[nid]:
                assert np.array_equal(a[nid][k], b[nid][k]), (names[i], nid, k)


def test_fit_is_bitwise_reproducible():
    """Two fits from the same seeds (graph capture, 4 stream groups, remainder step, validation) end
    with bitwise-identical master weights, Adam moments, BatchNorm moving statistics and metrics
    (no float atomics anywhere on the training path)."""
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine.base import TrainConfig
    from serann.engine.hip_engine import HipPopulationEngine
    data = get_serann_data(synthetic_encodings(), synthetic_mnist(n_train=3000, n_test=500, seed=6),
                           n_train=3000, n_test=500)
    names = sorted(ARCHS)
    irs = [interpret(ARCHS[n]) for n in names]
    cfg = TrainConfig(epochs=2, batch_size=256)
    runs = []
    for _ in range(2):
        eng = HipPopulationEngine(irs, list(range(len(irs))), device="cuda", cfg=cfg)
        res = eng.fit(data, cfg)
        runs.append((eng.p.cpu(), eng.m.cpu(), eng.v.cpu(), eng.stats.cpu(), res))
        del eng
    (p0, m0, v0, s0, r0), (p1, m1, v1, s1, r1) = runs
    assert torch.equal(p0, p1) and torch.equal(m0, m1) and torch.equal(v0, v1) and torch.equal(s0, s1)
    assert np.array_equal(r0.val_acc, r1.val_acc) and np.array_equal(r0.train_acc, r1.train_acc)
    assert np.array_equal(r0.val_mse, r1.val_mse)


@pytest.mark.parametrize("moments", ["16bit", "fp32"])
def test_fused_adam_matches_the_arena_pass(moments, monkeypatch):
    """WGRAD tiles with a single writer apply Adam in their epilogue (GF_ADAM) and the arena-wide pass skips
    them: after a 2-epoch fit (graph replay, remainder step) weights, moments and bf16 copies are bitwise
    those of the arena pass over every parameter, with either moment storage."""
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine.base import TrainConfig
    from serann.engine.hip_engine import HipPopulationEngine
    data = get_serann_data(synthetic_encodings(), synthetic_mnist(n_train=2200, n_test=300, seed=8),
                           n_train=2200, n_test=300)
    names = sorted(ARCHS)
    irs = [interpret(ARCHS[n]) for n in names]
    cfg = TrainConfig(epochs=2, batch_size=256, adam_moments=moments)
    out = []
    for fuse in ("1", "0"):
        monkeypatch.setenv("SERANN_FUSE_ADAM", fuse)
        eng = HipPopulationEngine(irs, list(range(len(irs))), device="cuda", cfg=cfg)
        res = eng.fit(data, cfg)
        out.append((eng.p.cpu(), eng.m.cpu(), eng.v.cpu(), eng.pbf.cpu(), res, eng._adam_skip))
        del eng
    (p1, m1, v1, b1, r1, sk1), (p0, m0, v0, b0, r0, sk0) = out
    assert sk1[0] is not None and int((sk1[0] != 0).sum()) > 0       # some tiles were fused
    assert sk0[0] is None
    diffs = {k: float((a.float() - b.float()).abs().max()) for k, a, b in (("p", p1, p0), ("m", m1, m0), ("v", v1, v0))}
    assert torch.equal(p1, p0) and torch.equal(m1, m0) and torch.equal(v1, v0) and torch.equal(b1, b0), diffs
    assert np.array_equal(r1.val_acc, r0.val_acc)


def test_fit_graph_replay_learns():
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine.base import TrainConfig
    from serann.engine.hip_engine import HipPopulationEngine
    data = get_serann_data(synthetic_encodings(), synthetic_mnist(n_train=6000, n_test=1000, seed=5),
                           n_train=6000, n_test=1000)
    irs = [interpret(ARCHS[n]) for n in ("conv_pool_dense", "odd_channels_bn", "empty_x_branch")]
    cfg = TrainConfig(epochs=2, batch_size=300)
    eng = HipPopulationEngine(irs, [1, 2, 3], device="cuda", cfg=cfg)
    res = eng.fit(data, cfg)
    assert eng.graph is not None
    assert res.steps == 2 * 19
    assert np.all(np.isfinite(res.val_acc))
    assert res.val_acc.mean() > 0.3, res.val_acc   # synthetic prototypes are easy
    acc = eng.evaluate(data.test_x, data.test_labels, data.test_g, cfg)
    assert np.all(acc > 0.2)
    imgs = [data.test_x[:20]] * 3
    gen = np.random.default_rng(0).integers(0, 2, (3, 100)).astype(np.float32)
    outs = eng.replicate(gen, imgs, cfg)
    assert outs[0].shape == (20, 100) and np.all((outs[0] >= 0) & (outs[0] <= 1))
    # the fused replication epilogue (device bit-pack, K16) gives the host rounding of the same outputs
    from serann.experiment.worker import replication_bits
    packed = eng.replicate_packed(gen, imgs, cfg)
    assert packed.shape == (3, 20, 13) and packed.is_cuda
    bits = np.unpackbits(packed.cpu().numpy(), axis=-1)[..., :100]
    for i in range(3):
        assert np.array_equal(bits[i], replication_bits(outs[i])), i
    # a pool larger than the batch runs in chunks through the same cached plan
    big = [data.test_x[:700]] * 3
    pb = eng.replicate_packed(gen, big, TrainConfig(epochs=2, batch_size=300))
    ob = eng.replicate(gen, big, TrainConfig(epochs=2, batch_size=300))
    assert np.array_equal(np.unpackbits(pb.cpu().numpy(), axis=-1)[..., :100], np.stack([replication_bits(o) for o in ob]))


def test_engines_in_sequence_in_one_process():
    """Several engines built, fitted (captured graph), evaluated, replicated and closed one after another
    in one process -- the driver runs the whole GPU suite as one pytest process -- plus a second fit on one
    engine (its cached inference plan must stay valid), the mutant with host fallbacks included.  Device
    memory returns to its starting level once the engines and datasets are gone."""
    import gc
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine.base import TrainConfig
    from serann.engine.hip_engine import _DEVICE_DATA, HipPopulationEngine
    torch.cuda.synchronize()
    gc.collect()
    base = torch.cuda.memory_allocated()
    cfg = TrainConfig(epochs=1, batch_size=250)
    pops = [("conv_pool_dense", "mutant_neg_sub"), ("odd_channels_bn", "gchain_f64_bn_dense", "rewired_fanout"),
            ("narrow_bn_ancestor", "convpool_bench_a")]
    for k, names in enumerate(pops):
        data = get_serann_data(synthetic_encodings(), synthetic_mnist(n_train=2000, n_test=500, seed=10 + k),
                               n_train=2000, n_test=500)
        irs = [interpret(ARCHS[n]) for n in names]
        eng = HipPopulationEngine(irs, list(range(len(irs))), device="cuda", cfg=cfg)
        for rep in range(2 if k == 0 else 1):
            res = eng.fit(data, cfg)
            assert eng.graph is not None and np.all(np.isfinite(res.val_acc)), (names, rep)
            acc = eng.evaluate(data.test_x, data.test_labels, data.test_g, cfg)
            assert np.all(np.isfinite(acc))
        gen = np.random.default_rng(k).integers(0, 2, (len(irs), 100)).astype(np.float32)
        packed = eng.replicate_packed(gen, [data.test_x[:40]] * len(irs), cfg)
        assert packed.shape == (len(irs), 40, 13)
        eng.close()
        assert eng.graph is None and not eng.plans
        del eng, packed, data
        gc.collect()
        torch.cuda.synchronize()
    assert len(_DEVICE_DATA) == 0                    # uploads died with their datasets
    assert torch.cuda.memory_allocated() - base < 64 << 20, torch.cuda.memory_allocated() - base


def test_fit_remainder_batch_matches_torch():
    """A batch size that does not divide the training split: the last step of each epoch trains on
    the true remainder (Keras semantics), in the HIP engine as in the torch oracle.  BatchNorm moving
    statistics carry ~25 % of their value from the last of 4 steps, so a remainder step padded with
    duplicated rows would show up here."""
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine.base import TrainConfig
    from serann.engine.hip_engine import HipPopulationEngine
    from serann.engine.torch_engine import TorchPopulationEngine
    data = get_serann_data(synthetic_encodings(), synthetic_mnist(n_train=1000, n_test=200, seed=9),
                           n_train=1000, n_test=200)
    names = ("odd_channels_bn", "narrow_bn_x")
    irs = [interpret(ARCHS[n]) for n in names]
    seeds = [21, 22]
    cfg = TrainConfig(epochs=1, batch_size=300)      # split 950 = 3 x 300 + 50
    assert cfg.split(1000) % cfg.batch_size == 50
    hip = HipPopulationEngine(irs, seeds, device="cuda", cfg=cfg,
                              params=[init_params(ir, s) for ir, s in zip(irs, seeds)])
    rh = hip.fit(data, cfg)
    ref = TorchPopulationEngine(irs, seeds, device="cpu", cfg=cfg)
    rr = ref.fit(data, cfg)
    assert rh.steps == rr.steps == 4
    for i, ir in enumerate(irs):
        got = hip.export_params(i)
        org = ref.orgs[i]
        for n in ir.nodes:
            if n.op != "bn":
                continue
            for k in ("moving_mean", "moving_variance"):
                want = org.p(n.id, k).detach().cpu().numpy()
                base = np.zeros_like(want) if k == "moving_mean" else np.ones_like(want)
                # compare the accumulated update (the statistics start at 0 / 1)
                err = _rel(got[n.id][k] - base, want - base)
                assert err < 0.1, (names[i], n.id, k, err)
    assert np.allclose(rh.train_acc, rr.train_acc, atol=0.05), (rh.train_acc, rr.train_acc)


@pytest.mark.parametrize("name", [n for n in sorted(ARCHS) if n.startswith("convpool") or n == "conv_pool_dense"])
def test_convpool_fusion_matches_unfused(name, monkeypatch):
    """Fused first-layer Conv2D + MaxPool2D (one kernel each way, no conv output tensor) against the
    unfused conv GEMM + pool kernels on the same parameters and batch: logits, every gradient (the conv
    weights and bias included), and the pooled activations' argmax-routed gradient."""
    from serann.engine import hip_engine as he
    ir = interpret(ARCHS[name])
    assert he.convpool_pairs(ir), name
    params = init_params(ir, 5)
    x, g, y = _batch(80, seed=4)
    fused = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
    gf, mf = fused.debug_train_step(x, g, y)
    lf = fused.debug_logits()[0]
    monkeypatch.setattr(he, "FUSE_CONVPOOL", False)
    assert not he.convpool_pairs(ir)
    plain = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
    gp, mp = plain.debug_train_step(x, g, y)
    lp = plain.debug_logits()[0]
    assert _rel(lf, lp) < 2e-2, _rel(lf, lp)
    # The unfused conv output is stored in bf16 before the pool, so values within 2^-8 of each other tie
    # inside a window and the first position wins; the fused kernel takes the max of the (nearly) fp32
    # pre-activations.  Both are exact argmaxes of their own inputs, and a few windows route their
    # gradient differently, so the two paths are each compared against the fp32 oracle: the fused one
    # must be at least as accurate as the unfused one (measured: it is more accurate, e.g. conv kernel
    # gradient 0.059 vs 0.082 for convpool_k9_f80), and the two stay close to each other.
    _, ref = _oracle(ir, params, x, g, y)
    a, b = fused.export_arena(0, gf), plain.export_arena(0, gp)
    for nid in ref:
        for k in ref[nid]:
            if np.linalg.norm(ref[nid][k]) < 5e-3:
                continue
            ef, eu = _rel(a[nid][k], ref[nid][k]), _rel(b[nid][k], ref[nid][k])
            assert ef < 1.25 * eu + 1e-2, (name, nid, k, ef, eu)
            assert _rel(a[nid][k], b[nid][k]) < 0.15, (name, nid, k, _rel(a[nid][k], b[nid][k]))
    assert np.allclose(mf, mp, rtol=2e-2, atol=1e-3)


@pytest.mark.parametrize("sign", [1.0, -1.0])
def test_convpool_ties_route_to_the_first_window(sign, monkeypatch):
    """Pool windows whose conv outputs tie exactly (a centre-tap-only filter on a block-constant image) route
    the gradient to the first window in scan order -- for negative values too -- as the unfused pool kernel
    and the reference's MaxPool do; the patches differ off the centre, so the routing shows in dW."""
    from serann.engine import hip_engine as he
    src = ("X_layer = Conv2D(filters=16, kernel_size=3, strides=1)(X_layer)\n"
           "X_layer = MaxPool2D(pool_size=2)(X_layer)\n\n"
           "g_layer = Dense(units=8, activation='relu')(g_layer)\n\n"
           "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
           "con = Dense(units=16, activation='relu')(con)\n\nloss_balance = 0.5")
    ir = interpret(src)
    cid = next(iter(he.convpool_pairs(ir)))
    params = init_params(ir, 3)
    k = np.zeros_like(params[cid]["kernel"])
    k[1, 1, 0, :] = sign * np.linspace(0.5, 1.0, k.shape[-1])
    params[cid]["kernel"] = k
    rng = np.random.default_rng(0)
    B = 32
    # conv output position (i, j) reads image pixel (i + 1, j + 1) at the centre tap: make those pixels
    # constant over every 2 x 2 pool window, and everything else random
    x = rng.random((B, 28, 28, 1)).astype(np.float32)
    blocks = rng.random((B, 13, 13)).astype(np.float32) + 0.1
    x[:, 1:27, 1:27, 0] = np.repeat(np.repeat(blocks, 2, axis=1), 2, axis=2)
    _, g, y = _batch(B, seed=5)
    fused = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
    gf, _ = fused.debug_train_step(x, g, y)
    monkeypatch.setattr(he, "FUSE_CONVPOOL", False)
    plain = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
    gp, _ = plain.debug_train_step(x, g, y)
    a, b = fused.export_arena(0, gf)[cid]["kernel"], plain.export_arena(0, gp)[cid]["kernel"]
    assert _rel(a, b) < 2e-2, _rel(a, b)


@pytest.mark.parametrize("name", [n for n in sorted(ARCHS) if n.startswith("gchain") or n == "convpool_bench_a"])
def test_gchain_fusion_matches_unfused(name, monkeypatch):
    """Fused genotype chain Conv1D(raw genotype) -> Dense -> [BatchNormalization] (gchain.hip: the chain
    is recomputed from the genotype in every pass, no intermediate tensor) against the unfused GEMM / BN
    kernels on the same parameters and batch: logits, every gradient against the fp32 oracle (the fused
    path keeps the pre-BN activations in fp32, the unfused one in bf16), the BatchNorm moving
    statistics, and inference logits through the moving statistics."""
    from serann.engine import hip_engine as he
    ir = interpret(ARCHS[name])
    assert he.gchain_triples(ir), name
    params = init_params(ir, 5)
    x, g, y = _batch(80, seed=4)
    fused = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
    gf, mf = fused.debug_train_step(x, g, y)
    lf = fused.debug_logits()[0]
    monkeypatch.setattr(he, "FUSE_GCHAIN", False)
    assert not he.gchain_triples(ir)
    plain = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
    gp, mp = plain.debug_train_step(x, g, y)
    lp = plain.debug_logits()[0]
    ref_logits, ref = _oracle(ir, params, x, g, y)
    # (a sigmoid Dense's output stored in bf16 before the BN -- unfused -- is the less accurate one)
    assert _rel(lf, ref_logits) < max(1.5 * _rel(lp, ref_logits), 1e-2), (_rel(lf, ref_logits), _rel(lp, ref_logits))
    assert np.allclose(mf[:, 3], mp[:, 3])
    a, b = fused.export_arena(0, gf), plain.export_arena(0, gp)
    for nid in ref:
        for k in ref[nid]:
            if np.linalg.norm(ref[nid][k]) < 5e-3:
                assert np.linalg.norm(a[nid][k]) < 2e-2, (name, nid, k, np.linalg.norm(a[nid][k]))
                continue
            r = np.asarray(ref[nid][k], np.float64)
            ef, eu = np.linalg.norm(a[nid][k] - r), np.linalg.norm(b[nid][k] - r)
            # relu / argmax boundary flips make either path the closer one by chance (measured rel. err.:
            # gchain_f64_bn_dense fused 0.014-0.057 vs unfused 0.017-0.023, convpool_bench_a 0.03-0.12 vs
            # 0.035-0.09 over two seeds; on sigmoid chains the fused path is 2-3x closer): a bound, not an
            # ordering, inside the oracle test's 0.2.  Near-cancelling biases are bounded on their layer's scale.
            kscale = np.linalg.norm(ref[nid]["kernel"]) if "kernel" in ref[nid] else 0.0
            assert ef < max(1.5 * eu, 0.15 * max(np.linalg.norm(r), 0.2 * kscale)), (name, nid, k, ef, eu)
    # moving statistics after one training step, then inference (moving statistics) through both paths
    sf, sp = fused.export_params(0), plain.export_params(0)
    for nid in sp:
        for k in ("moving_mean", "moving_variance"):
            if k in sp[nid]:
                base = np.zeros_like(sp[nid][k]) if k == "moving_mean" else np.ones_like(sp[nid][k])
                assert _rel(sf[nid][k] - base, sp[nid][k] - base) < 2e-2, (name, nid, k)
    from serann.engine.base import TrainConfig
    cfg = TrainConfig(batch_size=40)
    labels = y.astype(np.int64)
    monkeypatch.setattr(he, "FUSE_GCHAIN", True)
    acc_f = fused.evaluate(x, labels, g, cfg)
    monkeypatch.setattr(he, "FUSE_GCHAIN", False)
    acc_p = plain.evaluate(x, labels, g, cfg)
    assert np.allclose(acc_f, acc_p, atol=0.05), (acc_f, acc_p)


@pytest.mark.parametrize("name", ["narrow_bn_ancestor", "narrow_bn_x", "nbn_wide_linear", "nbn_sum_direct"])
def test_nbn_fusion_matches_unfused(name, monkeypatch):
    """Fused raw-input Dense -> BatchNormalization (nbn.hip: the Dense output is recomputed from the raw
    input in every pass, dz stays fp32) against the unfused narrow GEMM + BN kernels: logits, every
    gradient against the fp32 oracle, moving statistics, and inference through the moving statistics."""
    from serann.engine import hip_engine as he
    ir = interpret(ARCHS[name])
    assert he.nbn_pairs(ir), name
    params = init_params(ir, 5)
    x, g, y = _batch(96, seed=4)
    fused = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
    gf, mf = fused.debug_train_step(x, g, y)
    lf = fused.debug_logits()[0]
    monkeypatch.setattr(he, "FUSE_NBN", False)
    assert not he.nbn_pairs(ir)
    plain = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
    gp, mp = plain.debug_train_step(x, g, y)
    lp = plain.debug_logits()[0]
    ref_logits, ref = _oracle(ir, params, x, g, y)
    assert _rel(lf, lp) < 1e-2, _rel(lf, lp)
    assert np.allclose(mf, mp, rtol=2e-2, atol=1e-3)
    a, b = fused.export_arena(0, gf), plain.export_arena(0, gp)
    gmax = max(float(np.abs(v).max()) for d in ref.values() for v in d.values())
    for nid in ref:
        for k in ref[nid]:
            r = np.asarray(ref[nid][k], np.float64)
            ef, eu = np.linalg.norm(a[nid][k] - r), np.linalg.norm(b[nid][k] - r)
            floor = 1e-3 * gmax * np.sqrt(r.size)
            assert ef < 1.25 * eu + 0.02 * np.linalg.norm(r) + floor, (name, nid, k, ef, eu, np.linalg.norm(r))
    sf, sp = fused.export_params(0), plain.export_params(0)
    for nid in sp:
        for k in ("moving_mean", "moving_variance"):
            if k in sp[nid]:
                base = np.zeros_like(sp[nid][k]) if k == "moving_mean" else np.ones_like(sp[nid][k])
                assert _rel(sf[nid][k] - base, sp[nid][k] - base) < 1e-2, (name, nid, k)
    from serann.engine.base import TrainConfig
    cfg = TrainConfig(batch_size=48)
    labels = y.astype(np.int64)
    acc_f = fused.evaluate(x, labels, g, cfg)
    acc_p = plain.evaluate(x, labels, g, cfg)
    assert np.allclose(acc_f, acc_p, atol=0.03), (acc_f, acc_p)


@pytest.mark.parametrize("name", ["narrow_bn_ancestor", "narrow_bn_x", "nbn_sum_direct", "nbn_sum_acts"])
def test_nbn_sums_in_dgrad_match_phases_4_5(name, monkeypatch):
    """The BN backward of a fused raw-input Dense -> BN pair reduced in its consumer's DGRAD epilogue
    (GF_NBNSUM + nbn phase 6, dY never stored) against nbn phases 4 / 5 over the stored bf16 dY: the plan uses
    the fused form, and every gradient is at least as close to the fp32 oracle (1.25x + 1 % slack), at the
    production batch."""
    from serann.engine import hip_engine as he
    from serann.ops import hip_ops as H
    monkeypatch.setattr(he, "BINARY_NBN", False)        # (the GEMM path of the pair: GF_NBNSUM)
    ir = interpret(ARCHS[name])
    params = init_params(ir, 3)
    x, g, y = _batch(750, seed=2)
    fused = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
    gf, _ = fused.debug_train_step(x, g, y)
    kinds = [(la.kind, la.arg) for la in fused._debug_plan.launches]
    assert any(k == "nbn" and a[0] == 6 for k, a in kinds), kinds
    assert not any(k == "nbn" and a[0] in (4, 5) for k, a in kinds), kinds
    assert any(k == "gemm3" and a[0] == H.MODE_DGRAD and 17000 < a[1] < 19000 for k, a in kinds), kinds
    monkeypatch.setattr(he, "NBN_SUM", False)
    plain = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
    gp, _ = plain.debug_train_step(x, g, y)
    assert any(k == "nbn" and a[0] == 5 for k, a in [(la.kind, la.arg) for la in plain._debug_plan.launches])
    _, ref = _oracle(ir, params, x, g, y)
    a, b = fused.export_arena(0, gf), plain.export_arena(0, gp)
    gmax = max(float(np.abs(v).max()) for d in ref.values() for v in d.values())
    for nid in ref:
        for k in ref[nid]:
            r = np.asarray(ref[nid][k], np.float64)
            ef, eu = np.linalg.norm(a[nid][k] - r), np.linalg.norm(b[nid][k] - r)
            floor = 1e-3 * gmax * np.sqrt(r.size)
            assert ef < 1.25 * eu + 0.01 * np.linalg.norm(r) + floor, (name, nid, k, ef, eu, np.linalg.norm(r))
    fused.close()
    plain.close()


def test_adam_kernel_matches_keras_formula():
    from serann.ops import hip_ops as H
    lib = H.lib()
    n = 1003
    dev = "cuda"
    torch.manual_seed(0)
    p = torch.randn(n, device=dev)
    g0 = torch.randn(n, device=dev)
    g = H.to_qg(g0)                                   # the fixed-point gradient arena
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    pbf = torch.zeros(n, dtype=torch.bfloat16, device=dev)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    lr_t = torch.zeros(1, device=dev)
    g0 = H.from_qg(g)                               # the exact value the kernel converts
    p0 = p.clone()
    lib.adam(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), pbf.data_ptr(), step.data_ptr(), lr_t.data_ptr(),
             n, 1e-3, 0.9, 0.999, 1e-4, H.stream_handle())
    torch.cuda.synchronize()
    lr1 = 1e-3 * (1 - 0.999) ** 0.5 / (1 - 0.9)
    m1 = 0.1 * g0
    v1 = 0.001 * g0 * g0
    ref = p0 - lr1 * m1 / (v1.sqrt() + 1e-4)
    assert torch.allclose(p, ref, atol=1e-6, rtol=1e-5)
    assert torch.all(g == 0)
    assert int(step.item()) == 1
    assert torch.allclose(pbf.float(), ref, atol=1e-2, rtol=1e-2)


def _adam_run(mode, steps, grads, p0):
    """``steps`` arena Adam steps (hip adam kernel, moment storage ``mode``) on the gradient sequence ``grads``."""
    from serann.ops import hip_ops as H
    lib = H.lib()
    n = p0.numel()
    p = p0.clone()
    m16 = mode == H.MOM_16
    m = torch.zeros(n, dtype=torch.bfloat16 if m16 else torch.float32, device="cuda")
    v = torch.zeros(n, dtype=torch.int16 if m16 else torch.float32, device="cuda")
    pbf = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
    step = torch.zeros(1, dtype=torch.int32, device="cuda")
    lr_t = torch.zeros(1, device="cuda")
    for t in range(steps):
        g = H.to_qg(grads(t))
        lib.adam(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), pbf.data_ptr(), step.data_ptr(),
                 lr_t.data_ptr(), n, 1e-3, 0.9, 0.999, 1e-4, H.stream_handle(), mode)
    torch.cuda.synchronize()
    return p, m, v


def test_adam_16bit_moments_track_fp32_moments():
    """bf16 m + log16 v (csrc/hip/common.h MOM_16) against fp32 moments over a generation's 380 steps of noisy
    gradients whose scales span 1e-7 .. 10 (the eps = 1e-4 regime and above): the parameter displacement of each
    element stays within a few percent of the fp32-moment run, and the moments decode to the fp32 moments."""
    from serann.ops import hip_ops as H
    n = 4096
    gen = torch.Generator(device="cuda").manual_seed(3)
    scale = 10.0 ** torch.empty(n, device="cuda").uniform_(-7, 1, generator=gen)
    bias = torch.randn(n, device="cuda", generator=gen)
    p0 = torch.randn(n, device="cuda", generator=gen)
    noise = torch.randn(380, n, device="cuda", generator=gen)

    def grads(t):
        return scale * (0.5 * bias + noise[t])
    p32, m32, v32 = _adam_run(H.MOM_F32, 380, grads, p0)
    p16, m16, v16 = _adam_run(H.MOM_16, 380, grads, p0)
    d32, d16 = p32 - p0, p16 - p0
    rel = (d16 - d32).abs() / d32.abs().clamp_min(1e-12)
    big = d32.abs() > 1e-6                        # displacements that are not ~0 (every scale >= ~1e-6)
    # elements whose noisy updates nearly cancel (a random walk back to ~0) are measured against 5 % of the
    # largest path an Adam step sequence can take (~ lr per step)
    rel_path = (d16 - d32).abs() / (d32.abs() + 0.05 * 380 * 1e-3)
    stats = dict(median=float(rel[big].median()), q99_path=float(torch.quantile(rel_path, 0.99)),
                 norm=float((d16 - d32).norm() / d32.norm()))
    assert stats["median"] < 0.01 and stats["q99_path"] < 0.05 and stats["norm"] < 0.02, stats
    mf, vf = H.moments_f32(m16, v16)
    live = v32 > 2.0 ** -30
    assert float(((vf - v32).abs() / v32)[live].max()) < 0.03
    mrel = (mf - m32).abs() / m32.abs().clamp_min(1e-30)
    assert float(mrel[m32.abs() > 1e-3 * m32.abs().max()].median()) < 0.01


def test_fit_16bit_moments_vs_fp32_moments():
    """Fits (graph replay, 4 stream groups, fused-Adam WGRAD and finalize epilogues; 4 epochs = 132 Adam steps) with
    16-bit moments against the same fits with fp32 moments: every organism's validation accuracy within 0.03, the
    population mean within 0.01.  (Mid-curve organisms after 2 epochs move by up to 0.26 under ANY perturbation --
    fp32 moments with the learning rate x 1.001 as much as 16-bit moments: profiles/r6/moments_16bit_vs_fp32.txt --
    so the comparison is made once they have converged.  The reference itself keeps fp16 moments.)"""
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine.base import TrainConfig
    from serann.engine.hip_engine import HipPopulationEngine
    data = get_serann_data(synthetic_encodings(), synthetic_mnist(n_train=8000, n_test=500, seed=12),
                           n_train=8000, n_test=500)
    names = sorted(ARCHS)
    irs = [interpret(ARCHS[n]) for n in names]
    acc = {}
    for mode in ("fp32", "16bit"):
        cfg = TrainConfig(epochs=4, batch_size=256, adam_moments=mode, val_every_epoch=False)
        eng = HipPopulationEngine(irs, list(range(len(irs))), device="cuda", cfg=cfg)
        res = eng.fit(data, cfg)
        assert res.steps >= 50 and (eng.m.dtype == torch.bfloat16) == (mode == "16bit")
        acc[mode] = res.val_acc
        del eng
    d = acc["16bit"] - acc["fp32"]
    table = "\n".join(f"{n:30s} {a:.4f} {b:.4f}" for n, a, b in zip(names, acc["fp32"], acc["16bit"]))
    assert np.all(np.abs(d) <= 0.03) and abs(d.mean()) <= 0.01, table


def test_exploding_organism_is_flagged_diverged():
    """An organism whose gradients leave fp16's range (weights scaled x1000 per layer: activations ~1e9) is flagged
    by the Adam passes (csrc/hip/common.h flag_diverged) and its metrics come back NaN -- the reference's float16
    graph turns it into NaN weights -- while its neighbour in the same shard trains normally."""
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine.base import TrainConfig
    from serann.engine.hip_engine import HipPopulationEngine
    data = get_serann_data(synthetic_encodings(), synthetic_mnist(n_train=1500, n_test=300, seed=13),
                           n_train=1500, n_test=300)
    names = ("conv_pool_dense", "empty_x_branch")
    irs = [interpret(ARCHS[n]) for n in names]
    params = [init_params(ir, 7 + i) for i, ir in enumerate(irs)]
    for nid in params[1]:
        if "kernel" in params[1][nid]:
            params[1][nid]["kernel"] = params[1][nid]["kernel"] * 1000.0
    cfg = TrainConfig(epochs=1, batch_size=250)
    eng = HipPopulationEngine(irs, [0, 1], device="cuda", cfg=cfg, params=params)
    res = eng.fit(data, cfg)
    assert res.extra["diverged"] == [1], res.extra["diverged"]
    assert np.isfinite(res.val_acc[0]) and np.isnan(res.val_acc[1]) and np.isnan(res.val_mse[1])
    acc = eng.evaluate(data.test_x, data.test_labels, data.test_g, cfg)
    assert np.isfinite(acc[0]) and np.isnan(acc[1])
    eng.close()


@pytest.mark.parametrize("act", ["relu", "sigmoid"])
def test_bn_statistics_of_a_far_from_zero_input(act):
    """GF_BNUSTAT sums the producer's stored bf16 outputs unshifted (fp32 per wave, then wide fixed point,
    finished in double: gemm3.hip bn_ustat_flush).  On a BatchNormalization input whose mean is ~100x its spread
    (a Dense with bias 100, or a saturated sigmoid) the batch mean and inverse std the engine uses match a two-pass
    computation over the very same stored bf16 tensor."""
    from serann.engine.hip_engine import HipPopulationEngine
    src = ("X_layer = Conv2D(filters=48, kernel_size=3, strides=2)(X_layer)\n"
           f"X_layer = Dense(units=24, activation='{act}')(X_layer)\nX_layer = BatchNormalization()(X_layer)\n\n"
           "g_layer = Dense(units=16, activation='relu')(g_layer)\n\n"
           "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
           "con = Dense(units=40, activation='relu')(con)\n\nloss_balance = 0.4")
    ir = interpret(src)
    params = init_params(ir, 3)
    dense = next(n for n in ir.nodes if n.op == "gemm" and n.attrs["kind"] != "head_cls" and n.attrs["cin"] == 48)
    bn = next(n for n in ir.nodes if n.op == "bn")
    x, g, y = _batch(750, seed=5)
    eng = HipPopulationEngine([ir], [0], device="cuda", params=[params])
    off = eng.layouts[0].b[dense.id]                 # (the engine initialises biases to zero, as Keras does)
    with torch.no_grad():
        eng.p[off:off + 24] = 100.0 if act == "relu" else 6.0
        eng.pbf[off:off + 24] = eng.p[off:off + 24].to(torch.bfloat16)
    eng.debug_train_step(x, g, y)
    mem = eng._debug_mem
    rec = mem["orgs"][0]
    C = bn.attrs["channels"]
    _, off = rec["act"][dense.id]
    import math
    xin = mem["act"].view(off, 750 * math.prod(dense.shape)).view(-1, C).double().cpu()   # the stored bf16 BN input
    # (the LDS-tiled 1x1 FWD with the BN statistics in its epilogue: a Dense over 48 channels, no k splits)
    f32 = mem["f32"]
    mean = f32.view(rec["bn"][bn.id]["mean"], C).double().cpu()
    invstd = f32.view(rec["bn"][bn.id]["invstd"], C).double().cpu()
    want_mean = xin.mean(0)
    want_var = ((xin - want_mean) ** 2).mean(0)                              # two-pass
    assert float((xin.std(0) / xin.mean(0).abs()).max()) < 0.05            # |mean| / std > 20 on every channel
    assert torch.allclose(mean, want_mean, rtol=1e-6, atol=0)
    want_invstd = 1.0 / torch.sqrt(want_var + 1e-3)
    assert float(((invstd - want_invstd).abs() / want_invstd).max()) < 1e-3, (invstd, want_invstd)
    eng.close()


@pytest.mark.parametrize("name", ["narrow_bn_ancestor", "empty_x_branch", "nbn_sum_acts", "conv_pool_dense"])
def test_tiled_n_tile_groups_are_bitwise_neutral(name, monkeypatch):
    """LDS-tiled FWD / DGRAD blocks walking several n tiles (hip_ops.tiled_ngroup, forced on here for every launch)
    give bitwise the logits and gradients of one tile per block: every output tile is still one block's."""
    from serann.engine.hip_engine import HipPopulationEngine
    from serann.ops import hip_ops as H
    ir = interpret(ARCHS[name])
    params = init_params(ir, 11)
    x, g, y = _batch(750, seed=2)
    out = []
    for ng, mn in ((1, 1 << 30), (3, 1)):
        monkeypatch.setattr(H, "TILED_NGROUP", ng)
        monkeypatch.setattr(H, "TILED_NGROUP_MIN", mn)
        eng = HipPopulationEngine([ir], [0], device="cuda", params=[params])
        grads, metrics = eng.debug_train_step(x, g, y)
        tiled = [la for la in eng._debug_plan.launches if la.kind == "gemm3" and 7000 <= la.arg[1] % 10000 < 9000]
        out.append((grads.cpu(), eng.debug_logits()[0], metrics, len(tiled)))
        eng.close()
    (g1, l1, m1, n1), (g3, l3, m3, n3) = out
    assert n1 > 0 and n3 == n1
    assert torch.equal(g1, g3) and np.array_equal(l1, l3) and np.array_equal(m1, m3)


@pytest.mark.parametrize("name", ["narrow_bn_ancestor", "nbn_sum_acts", "bnbn_g_first_linear"])
def test_binary_genotype_factorisation_matches_the_gemm_path(name, monkeypatch):
    """The factorised genotype slice (csrc/hip/bnbn.hip: bin_prep / bin_fwd / the H WGRAD / bin_s / bin_wg; the BN
    output never written) against the GEMM path of the same pair (K-slice FWD, GF_NBNSUM DGRAD, slice WGRAD) on one
    production-batch step: logits and every gradient at least as close to the fp32 oracle (1.25x + 1 % slack)."""
    from serann.engine import hip_engine as he
    ir = interpret(ARCHS[name])
    params = init_params(ir, 4)
    x, g, y = _batch(750, seed=3)
    fact = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
    gf, mf = fact.debug_train_step(x, g, y)
    assert sorted({la.arg for la in fact._debug_plan.launches if la.kind == "bin"}) == [0, 1, 3]
    lf = fact.debug_logits()[0]
    monkeypatch.setattr(he, "BINARY_NBN", False)
    plain = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
    gp, mp = plain.debug_train_step(x, g, y)
    assert not any(la.kind == "bin" for la in plain._debug_plan.launches)
    lp = plain.debug_logits()[0]
    ref_logits, ref = _oracle(ir, params, x, g, y)
    assert _rel(lf, ref_logits) < 1.25 * _rel(lp, ref_logits) + 1e-3, (_rel(lf, ref_logits), _rel(lp, ref_logits))
    a, b = fact.export_arena(0, gf), plain.export_arena(0, gp)
    gmax = max(float(np.abs(v).max()) for d in ref.values() for v in d.values())
    for nid in ref:
        for k in ref[nid]:
            r = np.asarray(ref[nid][k], np.float64)
            ef, eu = np.linalg.norm(a[nid][k] - r), np.linalg.norm(b[nid][k] - r)
            floor = 1e-3 * gmax * np.sqrt(r.size)
            assert ef < 1.25 * eu + 0.01 * np.linalg.norm(r) + floor, (name, nid, k, ef, eu, np.linalg.norm(r))
    assert np.array_equal(mf[:, 3], mp[:, 3])
    fact.close()
    plain.close()


def test_binary_genotype_factorisation_fit_matches_the_gemm_path(monkeypatch):
    """Three-epoch fits (graph replay, 4 stream groups, fused Adam in bin_wg with 16-bit moments) of binary-path
    organisms against the GEMM path: validation accuracies within 0.03 once converged, and the factorised fit is
    bitwise reproducible."""
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine import hip_engine as he
    from serann.engine.base import TrainConfig
    data = get_serann_data(synthetic_encodings(), synthetic_mnist(n_train=6000, n_test=300, seed=21),
                           n_train=6000, n_test=300)
    names = ["narrow_bn_ancestor", "nbn_sum_acts", "bnbn_g_first_linear", "conv_pool_dense"]
    irs = [interpret(ARCHS[n]) for n in names]
    cfg = TrainConfig(epochs=3, batch_size=250, val_every_epoch=False)
    out = []
    for binary in (True, True, False):
        monkeypatch.setattr(he, "BINARY_NBN", binary)
        eng = he.HipPopulationEngine(irs, list(range(len(irs))), device="cuda", cfg=cfg)
        res = eng.fit(data, cfg)
        out.append((eng.p.cpu(), res.val_acc))
        del eng
    (p1, a1), (p2, a2), (_, a3) = out
    assert torch.equal(p1, p2) and np.array_equal(a1, a2)
    assert np.all(np.abs(a1 - a3) <= 0.03), (a1, a3)
