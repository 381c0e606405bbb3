"""Host-side launch planning (no GPU): tile-table permutations, shared column widths, kernel variant
selection and the fused conv + pool eligibility rules."""
import numpy as np
import pytest

from serann.genome.interpreter import interpret
from serann.ops import hip_ops as H

from .archs import ARCHS


@pytest.mark.parametrize("n,g", [(24, 3), (50, 3), (200, 6), (97, 12), (5, 2)])
def test_xcd_swizzle_is_a_permutation_grouping_runs_on_one_xcd(n, g):
    tiles = np.stack([np.arange(n)] * 4, 1).astype(np.int32)
    out = H.xcd_swizzle(tiles, g)
    assert sorted(out[:, 0].tolist()) == list(range(n))
    full = (n // (H.XCDS * g)) * H.XCDS * g
    pos = {int(t): i for i, t in enumerate(out[:, 0])}
    for c in range(full // g):
        assert len({pos[c * g + j] % H.XCDS for j in range(g)}) == 1
    assert (out[full:] == tiles[full:]).all()                 # the tail keeps its natural order


def _dense_rows(shapes):
    return [dict(M=M, N=N, K=K, KH=1, KW=1, SH=1, SW=1, C=K, flags=0) for M, N, K in shapes]


def test_tiled_widths_are_shared_per_launch_group():
    shapes = [(750, 135, 784), (750, 110, 200), (750, 190, 500), (750, 40, 300)]
    plans = H.gemm3_plan(H.MODE_FWD, _dense_rows(shapes), shapes)
    widths = [v for v, _, _ in plans if 7000 < v < 7300]
    assert 7064 in widths                                    # N <= 64 keeps its own narrow tile
    assert len([w for w in widths if w != 7064]) == 1         # one width for every N > 64 problem
    one = H.gemm3_plan(H.MODE_FWD, _dense_rows(shapes[:1]), shapes[:1])
    assert [v for v, _, _ in one] == [7160]                    # N = 135 alone: one 160-column tile


def test_wgrad_variants_default_to_64_row_tiles():
    assert H.gemm3_variant(H.MODE_WGRAD, 135, 4896, 750, {}) == 64128
    # F in (64, 96]: 64-row tiles (the 96-row / wide / tail-32 tiles measured slower and were removed)
    assert H.gemm3_variant(H.MODE_WGRAD, 73, 64, 432000, {}) == 64064
    assert H.gemm3_variant(H.MODE_WGRAD, 97, 64, 432000, {}) == 64064


def _split_signature(mode, rows, dims):
    """Per problem: the k ranges / row blocks its blocks cover (what decides its fp32 partial sums)."""
    out = {}
    for v, rws, tiles in H.gemm3_plan(mode, [dict(r) for r in rows], dims, splitk=True):
        for p, r in enumerate(rws):
            t = tiles[tiles[:, 0] == p]
            key = r["out"]
            out[key] = (sorted(set(int(x) for x in t[:, 3])), int(r.get("_split", 1)), int(r.get("flags", 0)) & H.GF_WSTORE)
    return out


def test_decomposition_is_per_problem():
    """Deterministic sharding: a problem's reduction splits (WGRAD m-splits, FWD k-splits, fused-chain row
    blocks, conv+pool images per block) are the same alone as inside any grouped launch, so an organism
    trains bit-identically whatever shard / stream group it lands in."""
    geo = dict(H=1, W=1, OH=1, OW=1, KH=1, KW=1, SH=1, SW=1)
    wg = [dict(a=0, b=0, out=1000 + i, C=K, F=F, M=F, N=K, K=R, flags=0, **geo)
          for i, (F, K, R) in enumerate([(70, 98, 75000), (128, 300, 750), (16, 40, 588000), (64, 3000, 96000)])]
    wdims = [(r["M"], r["N"], r["K"]) for r in wg]
    full = _split_signature(H.MODE_WGRAD, wg, wdims)
    for r, d in zip(wg, wdims):
        assert _split_signature(H.MODE_WGRAD, [r], [d])[r["out"]] == full[r["out"]]
    fw = [dict(a=0, b=0, out=2000 + i, C=K, F=N, M=750, N=N, K=K, act=0, flags=H.GF_VEC_A | H.GF_VEC_B, **geo)
          for i, (N, K) in enumerate([(135, 12000), (200, 6000), (40, 9000), (190, 2100)])]
    fdims = [(750, r["N"], r["K"]) for r in fw]
    full = _split_signature(H.MODE_FWD, fw, fdims)
    for r, d in zip(fw, fdims):
        assert _split_signature(H.MODE_FWD, [r], [d])[r["out"]] == full[r["out"]]
    # shared-input first layers: the kernel family (and so the arithmetic of every column) is the same alone as in
    # a run with other organisms' filter banks
    rows, dims = _imcol_rows([(0, 432000, 32, 25, 16), (0, 432000, 32, 25, 40), (0, 432000, 32, 25, 8)])
    fam = lambda v: (5100 < v < 5200, (v // 10) % 10)                        # (shared kernel, k steps)
    together = {r["out"]: fam(v) for v, rws, _ in H.gemm3_plan(H.MODE_FWD, [dict(r) for r in rows], dims) for r in rws}
    for r, d in zip(rows, dims):
        (v, _, _), = H.gemm3_plan(H.MODE_FWD, [dict(r)], [d])
        assert fam(v) == together[r["out"]] == (True, 1)
    # fused chain and conv+pool: functions of the problem alone
    assert H.gchain_rpb(72000, H.GC_BFULL, 96, 100) == H.gchain_rpb(72000, H.GC_BFULL, 96, 100)
    assert H.convpool_wgrad_imgs(750, 32) == 4 and H.convpool_wgrad_imgs(80, 16) == 4
    assert H.convpool_imgs(750, 80, False) == 8 and H.convpool_imgs(4000, 32, True) == 16


def test_gchain_large_genotype_is_not_fused():
    """A fused chain stages the genotype rows of a block in LDS (GCHAIN_GMAX elements); chains whose
    smallest block (64 rows) cannot fit stay on the unfused kernels (advisor finding, round 2)."""
    assert H.gchain_fits(96, 100)
    assert not H.gchain_fits(1, 8192)            # 65 batch rows x 8192 genotype elements
    with pytest.raises(ValueError):
        H.gchain_rpb(64 * 1000, H.GC_FSTAT, 1, 8192)
    src = ("g_layer=Conv1D(filters=8,kernel_size=3,strides=2)(g_layer)\n"
           "g_layer=Dense(units=16,activation='relu')(g_layer)\n"
           "con=concatenate([Reshape((1,-1))(X_layer),Reshape((1,-1))(g_layer)])\n"
           "loss_balance=0.5")
    from serann.engine.hip_engine import gchain_triples
    assert gchain_triples(interpret(src, genotype_size=100))
    assert not gchain_triples(interpret(src, genotype_size=16000))


def test_convpool_pool_window_limit():
    """The fused conv+pool kernel packs the pool-window offset into 8 bits: at most 256 windows."""
    assert H.convpool_ok(28, 28, 5, 5, 2, 2)
    assert H.convpool_ok(28, 28, 3, 3, 16, 16)
    assert not H.convpool_ok(28, 28, 3, 3, 17, 16)


@pytest.mark.parametrize("name,fused", [("convpool_bench_a", True), ("convpool_k9_f80", True),
                                        ("conv_pool_dense", True), ("odd_channels_bn", False),
                                        ("conv1d_rank4_and_strided_pool", False), ("bn_first_and_pool3", False)])
def test_convpool_eligibility(name, fused):
    from serann.engine.hip_engine import convpool_pairs
    ir = interpret(ARCHS[name])
    pairs = convpool_pairs(ir)
    assert bool(pairs) == fused
    for cid, pid in pairs.items():
        c, p = ir.node(cid), ir.node(pid)
        assert c.attrs["cin"] == 1 and ir.node(c.inputs[0]).op == "input"
        assert p.inputs == [cid] and H.convpool_ok(c.attrs["h"], c.attrs["w"], c.attrs["kh"], c.attrs["kw"])


def test_convpool_variant_encoding():
    assert H.convpool_variant(5, 5, 32) == 1 * 8 + 2
    assert H.convpool_variant(7, 7, 40) == 2 * 8 + 3
    assert H.convpool_variant(9, 9, 80) == 3 * 8 + 4
    assert H.convpool_chunks(750, 80, backward=False) == -(-750 // H.CONVPOOL_FWD_IMGS) * 2
    assert not H.convpool_ok(28, 28, 11, 11)                  # > 96 taps


@pytest.mark.parametrize("name,expect", [
    ("convpool_bench_a", "bn"), ("gchain_sigmoid_stride2", "bn"), ("gchain_f64_bn_dense", "bn"),
    ("gchain_nobn_k9_f100", "dense"), ("gchain_relu_conv_fanout", "dense"), ("bn_first_and_pool3", "dense"),
    ("odd_channels_bn", None), ("conv1d_rank4_and_strided_pool", None), ("narrow_bn_ancestor", None)])
def test_gchain_eligibility(name, expect):
    """Conv1D on the raw genotype whose only consumer is a Dense; the BatchNormalization joins only when
    it is the Dense's sole consumer (a fan-out Dense output stays materialised)."""
    from serann.engine.hip_engine import gchain_triples
    ir = interpret(ARCHS[name])
    tr = gchain_triples(ir)
    if expect is None:
        assert not tr
        return
    assert len(tr) == 1
    last, (cid, did, bid) = next(iter(tr.items()))
    c, dn = ir.node(cid), ir.node(did)
    assert c.attrs["kind"] == "conv1d" and ir.node(c.inputs[0]).op == "input" and dn.inputs == [cid]
    assert (bid is not None) == (expect == "bn")
    assert last == (bid if bid is not None else did)
    assert H.gchain_variant(c.attrs["f"], dn.attrs["f"], c.attrs["kh"]) is not None


@pytest.mark.parametrize("name,expect", [
    ("narrow_bn_ancestor", [75]), ("narrow_bn_x", [24]), ("nbn_wide_linear", [8, 200]),
    ("odd_channels_bn", []),            # the BN's Dense reads a conv output (needs a DGRAD)
    ("gchain_sigmoid_stride2", []),     # the BN belongs to the genotype chain's Dense
    ("empty_x_branch", [])])
def test_nbn_eligibility(name, expect):
    """Raw-input Dense (K <= 4) -> BatchNormalization pairs fused in training plans (nbn.hip)."""
    from serann.engine.hip_engine import nbn_pairs
    ir = interpret(ARCHS[name])
    pairs = nbn_pairs(ir)
    assert sorted(ir.node(d).attrs["f"] for d in pairs.values()) == expect
    for bid, did in pairs.items():
        d = ir.node(did)
        assert ir.node(bid).inputs == [did] and ir.node(d.inputs[0]).op == "input" and d.attrs["cin"] <= 4


def test_nbn_chunking_covers_rows():
    for rows, f in ((75000, 75), (588000, 24), (750 * 100, 200), (17, 8)):
        for phase in (2, 4, 5):
            s1 = max(1, (H.NBN_ELEMS // 8) // f)
            srb = max(1, (H.NBN_P2_ELEMS // 8) // f) if phase == 2 else s1 * H.NBN_RED_MULT
            assert H.nbn_chunks(rows, f, phase) * srb * 8 >= rows > (H.nbn_chunks(rows, f, phase) - 1) * srb * 8


def test_gchain_variant_and_block_sizing():
    assert H.gchain_variant(32, 51, 5) == 1 * 8 + 2
    assert H.gchain_variant(8, 100, 9) == 1 * 8 + 4
    assert H.gchain_variant(64, 64, 1) == 2 * 8 + 2
    assert H.gchain_variant(64, 100, 1) is None          # F1 > 32 needs F2 <= 64
    assert H.gchain_variant(16, 129, 3) is None          # F2 > 128
    assert H.gchain_variant(16, 64, 17) is None          # > 16 taps
    for mode in range(4):
        for rows, l1 in ((72000, 96), (750, 1), (8000, 100), (363000, 484)):
            rpb = H.gchain_rpb(rows, mode, l1, 100)
            assert rpb % 64 == 0 and rpb >= 64
            # the block's genotype rows fit the kernel's LDS staging buffer
            assert (-(-rpb // l1) + 1) * 100 <= H.GCHAIN_GMAX


def test_conv_wgrad_multi_image_chunks():
    """Small conv outputs pack whole images into the 128-row chunks of the conv WGRAD kernel; the
    tier is chosen to hold as many as a chunk can take, and large outputs keep per-image tiles."""
    g = dict(KH=7, KW=7, C=64, H=11, W=11, OH=5, OW=5, SH=1)
    bmf, bnk, tier = H.conv_wgrad_config(g, 16)
    assert H.conv_wgrad_ipc(g, tier) == 3                    # 3 x 11*11*72 <= 32768 < 4 x ...
    g = dict(KH=5, KW=5, C=32, H=12, W=12, OH=8, OW=8, SH=1)
    assert H.conv_wgrad_ipc(g, H.conv_wgrad_config(g, 16)[2]) == 2
    g = dict(KH=3, KW=3, C=73, H=24, W=24, OH=22, OW=22, SH=1)
    assert H.conv_wgrad_ipc(g, H.conv_wgrad_config(g, 16)[2]) == 1
    # the tile table covers every image exactly once
    rows = [dict(a=0, b=0, out=0, H=11, W=11, C=64, OH=5, OW=5, F=16, KH=7, KW=7, SH=1, SW=1, M=16, N=3136,
                 K=17 * 25, flags=0)]
    (v, rws, tiles), = H.gemm3_plan(H.MODE_WGRAD, rows, [(16, 3136, 17 * 25)])
    assert v >= 3000000
    assert int(tiles[:, 3].max()) == 6 and int(tiles[:, 2].min()) == 0      # ceil(17 / 3) chunks


def test_adam_skip_mask():
    """One byte per 4-parameter group of the arena-wide Adam pass; bit j = parameter 4i + j is updated by its
    WGRAD epilogue.  Regions are strided blocks (a column slice of a merged Dense's weights)."""
    n = 50
    m = H.adam_skip_mask(n, [(3, 2, 3, 10), (40, 1, 6, 6)])
    assert m.dtype == np.uint8 and len(m) == -(-n // 4)
    want = np.zeros(52, bool)
    for e in (3, 4, 5, 13, 14, 15, 40, 41, 42, 43, 44, 45):
        want[e] = True
    bits = np.unpackbits(m[:, None], axis=1, bitorder="little")[:, :4].ravel().astype(bool)
    assert np.array_equal(bits, want)


def test_conv_wgrad_splits_per_problem():
    """Tap-shifted conv WGRAD (round 5): a block covers the whole padded (tap, Cp) width up to 1024 columns;
    the chunk-range splits are bounded by MFMAs per wave and by chunks per block, are a function of the
    problem alone, and split problems get fp32 slabs (``_wgfin``: one per split, summed in order by the
    finalize) while single-split problems store their Q40 gradient (GF_WSTORE)."""
    def row(B, Hh, Ww, C, F, K):
        OH, OW = Hh - K + 1, Ww - K + 1
        return dict(a=0, b=0, out=1, H=Hh, W=Ww, C=C, OH=OH, OW=OW, F=F, KH=K, KW=K, SH=1, SW=1, M=F,
                    N=K * K * C, K=B * OH * OW, flags=0), (F, K * K * C, B * OH * OW)
    big, dbig = row(750, 28, 28, 74, 16, 5)       # 2000 reduction columns: two 1024-column blocks
    small, dsmall = row(8, 12, 12, 16, 16, 3)
    assert H.conv_wgrad_config(big, 16)[1] == 2048 and H.conv_wgrad_config(small, 16)[1] == 256
    alone = {}
    for rows, dims in (([big], [dbig]), ([small], [dsmall])):
        for v, rws, tiles in H.gemm3_plan(H.MODE_WGRAD, [dict(r) for r in rows], dims):
            alone[rws[0]["N"]] = (v, rws[0].get("_wgfin"), rws[0]["kper"], rws[0]["flags"], tiles[:, 1:].tolist())
    together = {}
    for v, rws, tiles in H.gemm3_plan(H.MODE_WGRAD, [dict(big), dict(small)], [dbig, dsmall]):
        for p, r in enumerate(rws):
            together[r["N"]] = (v, r.get("_wgfin"), r["kper"], r["flags"], tiles[tiles[:, 0] == p][:, 1:].tolist())
    assert alone == together
    v, ns, per, flags, tl = alone[25 * 74]
    nchunks = 750 * 5                                    # 576 pixels per image: 5 chunks of 128
    assert ns == -(-nchunks // per) > 1 and per <= H.CONV_WGRAD_MAX_CHUNKS and not flags & H.GF_WSTORE
    assert len(tl) == ns                                 # one 2048-column block (25 x 80 padded) per split
    v, ns, per, flags, tl = alone[144]
    assert ns is None and flags & H.GF_WSTORE            # 16 chunks: one block


def test_adam_skip_mask_device_matches_host():
    """The device-built skip mask (difference array over whole groups + edge bits) equals the per-parameter
    host construction on random disjoint regions: contiguous blocks, strided column slices, ranges inside
    one 4-parameter group, and ranges that end or start mid-group next to each other."""
    import torch
    rng = np.random.default_rng(3)
    for trial in range(40):
        n = int(rng.integers(8, 3000))
        regions, used = [], np.zeros(n, bool)
        for _ in range(int(rng.integers(1, 12))):
            rows, cols = int(rng.integers(1, 6)), int(rng.integers(1, 40))
            ld = cols if rng.random() < 0.5 else cols + int(rng.integers(1, 9))
            off = int(rng.integers(0, n))
            idx = off + np.arange(rows)[:, None] * ld + np.arange(cols)[None, :]
            if idx.max() >= n or used[idx.ravel()].any():
                continue
            used[idx.ravel()] = True
            regions.append((off, rows, cols, ld))
        want = H.adam_skip_mask(n, regions)
        got = H.adam_skip_mask_device(n, regions, torch.device("cpu")).numpy()
        assert np.array_equal(got, want), (trial, regions)


def test_wgrad_row_groups_are_per_problem():
    """Dense / 1x1 WGRAD: m-split problems get two row groups per block (variant + 500, twice the k-steps
    per block, half the fixed-point flushes); single-split problems (plain store / fused Adam) keep one.
    The choice and the split boundaries are functions of the problem alone, whatever shares the launch."""
    geo = dict(H=1, W=1, OH=1, OW=1, KH=1, KW=1, SH=1, SW=1, a=0, b=0, flags=0)
    probs = [(60, 16, 300000), (152, 7500, 750), (64, 44, 588000), (150, 300, 75000), (60, 16, 750)]
    rows = [dict(geo, out=1000 + i, C=N, F=M, M=M, N=N, K=K, adam=1) for i, (M, N, K) in enumerate(probs)]
    full = {}
    for v, rws, tiles in H.gemm3_plan(H.MODE_WGRAD, [dict(r) for r in rows], probs):
        for p, r in enumerate(rws):
            t = tiles[tiles[:, 0] == p]
            full[r["out"]] = (v, r["flags"], sorted(set(int(x) for x in t[:, 3])))
    assert full[1001][0] % 1000 < 500 and full[1001][1] & H.GF_ADAM          # single split: one group, Adam
    for out in (1000, 1002, 1003):
        assert full[out][0] % 1000 >= 500 and not full[out][1] & H.GF_WSTORE  # m-split: two groups
    for r, d in zip(rows, probs):
        (v, rws, tiles), = H.gemm3_plan(H.MODE_WGRAD, [dict(r)], [d])
        assert (v, rws[0]["flags"], sorted(set(int(x) for x in tiles[:, 3]))) == full[r["out"]]


def _imcol_rows(specs):
    """FWD rows of first-layer convolutions over materialised im2col matrices: (matrix id, M, K8, K, N)."""
    rows, dims = [], []
    for i, (a, M, C, K, N) in enumerate(specs):
        rows.append(dict(a=1000 * (a + 1), out=10 ** 6 * (i + 1), M=M, N=N, K=K, C=C, H=1, W=M, OH=1, OW=M,
                         KH=1, KW=1, SH=1, SW=1, flags=0, _imcol=1))
        dims.append((M, N, K))
    return rows, dims


def test_shared_input_fwd_runs_cover_every_tile_once():
    """Shared-input FWD (g3_shared_fwd_kernel): the problems of one im2col matrix are consecutive in the launch's
    descriptor table and every (problem, 256-row tile) is computed by exactly one run."""
    specs = [(0, 432000, 32, 25, 16), (1, 126750, 16, 9, 16), (0, 432000, 32, 25, 8), (2, 300000, 56, 49, 32),
             (0, 432000, 32, 25, 16), (1, 126750, 16, 9, 16), (2, 300000, 56, 49, 8), (3, 9000, 88, 81, 60)]
    rows, dims = _imcol_rows(specs)
    rows.append(dict(rows[0], _imcol=0, out=5))          # not an im2col first layer: the usual kernels
    dims.append(dims[0])
    plans = H.gemm3_plan(H.MODE_FWD, [dict(r) for r in rows], dims)
    shared = [(v, rws, t) for v, rws, t in plans if 5100 < v < 5200]
    assert sorted(v for v, _, _ in shared) == [5111, 5122, 5134]     # (NT, KS) by the widest bank, K8
    seen = {}
    for v, rws, tiles in shared:
        a = [r["a"] for r in rws]
        assert a == sorted(a)                             # one matrix's problems are consecutive
        for p0, mt, n, z in tiles.tolist():
            assert n >= 1 and z == 0 and len({rws[p]["a"] for p in range(p0, p0 + n)}) == 1
            for p in range(p0, p0 + n):
                key = (rws[p]["out"], mt)
                assert key not in seen
                seen[key] = 1
    expect = {(r["out"], m) for r, (M, _, _) in zip(rows[:-1], dims) for m in range(-(-M // 256))}
    assert set(seen) == expect
    assert all(5 not in [r["out"] for r in rws] for _, rws, _ in shared)


def test_shared_input_fwd_eligibility():
    rows, dims = _imcol_rows([(0, 432000, 32, 25, 16)])
    assert H.shared_fwd_ok(rows[0], *dims[0])
    assert not H.shared_fwd_ok(dict(rows[0], N=65), 432000, 65, 25)            # > 4 column tiles
    assert not H.shared_fwd_ok(dict(rows[0], C=104), 432000, 16, 100)          # > 3 register-held k steps
    assert not H.shared_fwd_ok(dict(rows[0], flags=H.GF_ACCUM), 432000, 16, 25)
    assert not H.shared_fwd_ok(dict(rows[0], _imcol=0), 432000, 16, 25)
    # a lone problem takes the same kernel (its bits do not depend on who shares its launch)
    (v, _, _), = H.gemm3_plan(H.MODE_FWD, [dict(rows[0])], dims)
    assert v == 5111


def test_shared_wgrad_order_is_a_permutation_grouping_row_ranges():
    """First-layer WGRADs over one im2col matrix: the tiles of its problems that reduce the same row range are
    dispatched to one XCD (its L2 serves the matrix rows to every organism); the table stays a permutation and the
    other problems' tiles keep their order."""
    rows = [dict(b=1000, _imcol=1), dict(b=2000, _imcol=1), dict(b=1000, _imcol=1), dict(b=1000, _imcol=1),
            dict(b=1000, _imcol=0)]
    tl = []
    for p in range(len(rows)):
        for k in range(40):                               # 40 row ranges of 16 k steps, one (m, n) tile
            tl.append((p, 0, 0, (16 * k) | ((16 * k + 16) << 16)))
    tiles = np.array(tl, np.int32)
    out = H.shared_wgrad_order(rows, tiles)
    assert sorted(map(tuple, out.tolist())) == sorted(map(tuple, tiles.tolist()))
    pos = {tuple(t): i for i, t in enumerate(out.tolist())}
    nfull = (3 * 40 // (H.XCDS * 3)) * H.XCDS * 3 // 3      # row ranges inside whole swizzle groups
    for k in range(nfull):
        w = (16 * k) | ((16 * k + 16) << 16)
        assert len({pos[(p, 0, 0, w)] % H.XCDS for p in (0, 2, 3)}) == 1
    keep = [t for t in out.tolist() if t[0] in (1, 4)]
    assert keep == [t for t in tiles.tolist() if t[0] in (1, 4)]


def test_small_bank_wgrad_selection():
    """g3_wgrad_tiny_kernel takes 1x1 WGRADs of <= 16 filters and <= 64 columns over >= 64 k steps (8000000 + NK),
    with one row group; conv geometries, wide banks and short reductions keep the other kernels."""
    geo = dict(H=26, W=26, OH=26, OW=26, KH=1, KW=1, SH=1, SW=1, flags=0)
    cases = [((16, 9, 507000), 8000001), ((8, 25, 432000), 8000002), ((13, 49, 300000), 8000004),
             ((32, 9, 507000), None), ((16, 81, 300000), None), ((16, 9, 750), None)]
    for (M, N, K), want in cases:
        r = dict(a=1, b=2, out=3, M=M, N=N, K=K, C=N, F=M, **geo)
        (v, rws, tiles), = H.gemm3_plan(H.MODE_WGRAD, [r], [(M, N, K)])
        if want is None:
            assert not 8000000 < v < 8000010
        else:
            assert v == want and H.gemm3_block(H.MODE_WGRAD, v) == (16, 16 * (want - 8000000))
            assert (tiles[:, 1] == 0).all() and (tiles[:, 2] == 0).all()
            spans = sorted((t & 0xffff, t >> 16) for t in tiles[:, 3].tolist())
            assert spans[0][0] == 0 and spans[-1][1] == -(-K // H.BK)
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))          # the k ranges tile the reduction
    r = dict(a=1, b=2, out=3, M=16, N=9, K=507000, C=9, F=16, **dict(geo, KH=3, KW=3))
    (v, _, _), = H.gemm3_plan(H.MODE_WGRAD, [r], [(16, 81, 507000)])
    assert not 8000000 < v < 8000010
