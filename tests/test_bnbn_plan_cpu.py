"""Plan structure of the binary-genotype factorisation (csrc/hip/bnbn.hip) on the CPU: a raw-genotype Dense -> BN
pair read by a merged-Dense K slice runs as the factorised kernels when the genotype batches are binary, and as
the GF_NBNSUM DGRAD / GEMM slices otherwise (nothing is launched here)."""
import numpy as np
import pytest

from serann.genome.interpreter import interpret
from serann.ops import hip_ops as H

from .archs import ARCHS


def _plan(name, binary, B=750):
    from serann.engine.hip_engine import HipPopulationEngine
    try:
        H.lib()
    except ImportError:
        pytest.skip("serann_hip not built")
    ir = interpret(ARCHS[name])
    eng = HipPopulationEngine([ir, ir], [0, 1], device="cpu")
    eng._g_binary = binary
    mem = eng._alloc_buffers(B, with_grads=True)
    pl = eng._build_plan("train", B, mem, [{"X": 0, "g": 0}] * 2, 0, [0] * 2, None, adam_ctx=1)
    return eng, pl


def test_binary_pairs_take_the_factorised_kernels():
    eng, pl = _plan("narrow_bn_ancestor", True)
    kinds = [(la.kind, la.arg) for la in pl.launches]
    assert [a for k, a in kinds if k == "bin"] == [0, 1, 3]
    assert ("memset", None) not in kinds and any(k == "memset" for k, _ in kinds)
    # no DGRAD carries the BN-backward-sums epilogue any more, and no 7500-column slice GEMM remains
    for la in pl.launches:
        if la.kind == "gemm3":
            d = np.frombuffer(la.descs.numpy().tobytes(), dtype=H.GEMM_DTYPE)
            assert not np.any(d["flags"] & H.GF_NBNSUM)
            assert not np.any(d["K"] == 7500) and not np.any(d["N"] == 7500)
    # nbn phase 7: one statistics block per problem from the count of ones (the BN output is never written,
    # and the pair's Dense has no FWD launch at all: no statistics-only narrow kernel); phase 6 still runs
    nbn = [la for la in pl.launches if la.kind == "nbn"]
    assert not [la for la in nbn if la.arg[0] == 2]
    p7 = [la for la in nbn if la.arg[0] == 7]
    assert len(p7) == 1 and p7[0].n == 2
    for la in pl.launches[:pl.fwd_count]:
        if la.kind == "gemm3":
            d = np.frombuffer(la.descs.numpy().tobytes(), dtype=H.GEMM_DTYPE)
            assert not np.any(d["flags"] & H.GF_BNSTAT)
    assert any(la.arg[0] == 6 for la in nbn)
    # the factorised slice's dW is applied by bin_wg (Adam region), not by the arena pass
    assert any(r[2] == 7500 for r in pl.adam_regions)
    # part buffers of phase 6 hold one m slot per bin_sw row split (two organisms: few column blocks, so the
    # 152 rows are split towards BIN_SW_BLOCKS blocks of >= 32 rows)
    rows = np.frombuffer([la for la in nbn if la.arg[0] == 6][0].descs.numpy().tobytes(), dtype=H.NBN_DTYPE)
    sw = [la for la in pl.launches if la.kind == "bin" and la.arg == 3][0]
    brows = np.frombuffer(sw.descs.numpy().tobytes(), dtype=H.BIN_DTYPE)
    cols = np.where(brows["flags"] & H.BIN_VEC4, 256, 64)
    assert np.all(brows["ns"] == 4) and sw.n == int(np.sum(4 * -(-brows["L"] * brows["F"] // cols)))
    assert np.all(rows["mtiles"] == 4) and np.all(rows["np"] == 100)


def test_non_binary_genotypes_keep_the_nbnsum_path():
    eng, pl = _plan("narrow_bn_ancestor", False)
    assert not any(la.kind == "bin" for la in pl.launches)
    flags = [np.frombuffer(la.descs.numpy().tobytes(), dtype=H.GEMM_DTYPE)["flags"] for la in pl.launches
             if la.kind == "gemm3"]
    assert any(np.any(f & H.GF_NBNSUM) for f in flags)


def test_binary_check():
    from serann.engine.hip_engine import _is_binary
    assert _is_binary(np.array([[0, 1, 1], [1, 0, 0]], np.float32))
    assert not _is_binary(np.array([[0, 1, 0.5]], np.float32))
    assert not _is_binary(np.zeros((0, 3)))
