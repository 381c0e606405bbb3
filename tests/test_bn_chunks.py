"""Host-side BatchNorm block sizing (mirror of aux.hip bn_vec / bn_stat_mult): the grid the engine
launches must cover exactly the super-rows each block walks on the device."""
from serann.ops import hip_ops as H


def _device_blocks(R, C, stats):
    # aux.hip bn_vec: srb super-rows per block, 1x below BN_STAT_SMALL blocks, BN_RED_MULT x above
    nsr = (R + 7) // 8
    srb1 = max(1, (H.BN_VEC_ELEMS // 8) // C)
    base = (nsr + srb1 - 1) // srb1
    mult = (1 if base < H.BN_STAT_SMALL else H.BN_RED_MULT) if stats else 1
    srb = srb1 * mult
    return (nsr + srb - 1) // srb, srb, nsr


def test_bn_chunks_cover_rows():
    for R, C in [(750, 128), (750, 37), (96000, 128), (363000, 16), (588000, 67), (5000, 1), (4096, 256)]:
        for stats in (False, True):
            n = H.bn_chunks(R, C, stats=stats)
            nb, srb, nsr = _device_blocks(R, C, stats)
            assert n == nb
            assert (n - 1) * srb < nsr <= n * srb      # every super-row owned by exactly one block


def test_bn_stats_multiplier_threshold():
    # small problems keep one block per 16K elements; large ones take BN_RED_MULT x the rows
    assert H.bn_chunks(96000, 128, stats=True) == H.bn_chunks(96000, 128)
    big = H.bn_chunks(588000, 67)
    assert big >= H.BN_STAT_SMALL
    assert H.bn_chunks(588000, 67, stats=True) == -(-big // H.BN_RED_MULT)
    assert H.BN_WS_STRIPES >= 1
