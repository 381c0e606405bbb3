"""LPT cost model (experiment/cost_model.py): features, both coefficient formats, and the LPT partition's
predicted balance on a generator population (replaces reference experiment.py:170-178 round-robin)."""
import numpy as np

from serann.experiment import cost_model as CM
from serann.genome.interpreter import interpret

from .archs import ARCHS


def test_features_split_conv_and_dense():
    ir = interpret(ARCHS["conv_pool_dense"])
    f = CM.features(ir)
    assert f["Fc"] > 0 and f["Fd"] > 0
    assert abs(f["Fc"] + f["Fd"] - f["F"]) < 1e-6 * f["F"]
    assert f["Ab"] == 0 and f["Aa"] > 0
    g = CM.features(interpret(ARCHS["narrow_bn_ancestor"]))
    assert g["Fc"] == 0 and g["Ab"] == 2 * 100 * 75      # BN input + output, per sample


def test_named_and_legacy_coefficients():
    ir = interpret(ARCHS["odd_channels_bn"])
    f = CM.features(ir)
    named = {"coef": {"Fc": 1e-15, "Fd": 2e-15, "Ab": 3e-12, "Aa": 4e-12, "N": 5e-6}, "d_s": 1e-3}
    t = CM.organism_time(ir, 750, named)
    want = (1e-15 * f["Fc"] * 3 * 750 + 2e-15 * f["Fd"] * 3 * 750 + 3e-12 * f["Ab"] * 750
            + 4e-12 * f["Aa"] * 750 + 5e-6 * f["N"])
    assert abs(t - want) < 1e-12 * max(1.0, want)
    legacy = {"a_s_per_flop": 1e-15, "b_s_per_byte": 1e-13, "c_s_per_node": 1e-6, "d_s": 0.0}
    tl = CM.organism_time(ir, 750, legacy)
    assert abs(tl - (1e-15 * 3 * f["F"] * 750 + 1e-13 * f["A"] * 750 + 1e-6 * f["N"])) < 1e-12
    assert CM.shard_time([ir, ir], 750, named) == 2 * t + 1e-3


def test_lpt_balances_a_generator_population():
    from serann.genome.generator import generate
    from serann.parallel.partition import lpt_partition
    df = generate(160, seed=3, validation_genotype_size=100)
    irs = [interpret(c) for c in df["code"]]
    coef = CM.coefficients()
    costs = np.array([CM.organism_time(ir, 750, coef) for ir in irs])
    parts = lpt_partition(costs, 8, [ir.arch_hash() for ir in irs])
    loads = np.array([costs[p].sum() for p in parts])
    assert sorted(i for p in parts for i in p) == list(range(len(irs)))
    assert loads.max() / loads.mean() < 1.05
