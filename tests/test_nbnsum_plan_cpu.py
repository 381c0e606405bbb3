"""Planner side of the BN-backward sums in the consumer DGRAD (GF_NBNSUM), on the CPU: which fused raw-input
Dense -> BatchNormalization pairs get the NS DGRAD (variants 17000 + BN / 18000 + BN) and the phase-6 finalize,
and which keep nbn phases 4 / 5 (hip_engine.py: one input channel, one consumer GEMM whose DGRAD runs on the
LDS-tiled kernel, K of that DGRAD > 32).  The plan is built without launching anything; the GPU tests
(test_gpu_engine.py::test_nbn_sums_in_dgrad_match_phases_4_5) check the numbers."""
import pytest

from .archs import ARCHS
from serann.genome.interpreter import interpret


def _plan_kinds(name, batch=96):
    from serann.engine.hip_engine import HipPopulationEngine
    ir = interpret(ARCHS[name])
    eng = HipPopulationEngine([ir], [0], device="cpu")
    mem = eng._alloc_buffers(batch, with_grads=True)
    pl = eng._build_plan("train", batch, mem, [{"X": 0, "g": 0}], 0, [0], None, adam_ctx=1)
    return [(la.kind, la.arg) for la in pl.launches if la.kind != "fn"]


def _nbn_phases(kinds):
    return sorted({a[0] for k, a in kinds if k == "nbn"})


def _ns_dgrads(kinds):
    from serann.ops import hip_ops as H
    return [a for k, a in kinds if k == "gemm3" and a[0] == H.MODE_DGRAD and 17000 < a[1] < 19000]


@pytest.mark.parametrize("name", ["narrow_bn_ancestor", "nbn_sum_direct", "nbn_sum_acts"])
def test_eligible_pairs_use_the_dgrad_sums(name):
    kinds = _plan_kinds(name)
    assert _nbn_phases(kinds) == [2, 6], kinds
    assert _ns_dgrads(kinds), kinds


def test_short_consumer_keeps_phases_4_5():
    # nbn_wide_linear: the sigmoid pair's consumer is Dense(10) (DGRAD K = 10 <= 32): phases 4 / 5 stay
    kinds = _plan_kinds("nbn_wide_linear")
    assert 5 in _nbn_phases(kinds) and 4 in _nbn_phases(kinds), kinds


def test_switch_off_restores_phases_4_5(monkeypatch):
    from serann.engine import hip_engine as he
    monkeypatch.setattr(he, "NBN_SUM", False)
    kinds = _plan_kinds("narrow_bn_ancestor")
    assert _nbn_phases(kinds) == [2, 4, 5], kinds
    assert not _ns_dgrads(kinds), kinds
