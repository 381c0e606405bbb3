"""Python side of the HIP/CDNA4 kernels: descriptor dtypes (mirroring ``csrc/hip/serann_hip.h``)
and thin launch wrappers that pass raw device pointers and the current HIP stream.

The kernels are loaded from the in-tree ``serann/_native/serann_hip*.so``.  On a machine with a GPU
the engine *requires* the extension (it fails loudly instead of silently falling back).
"""
from __future__ import annotations

import functools
import os as _os
import numpy as np

from ..utils.native import load

_I = np.int64
GEMM_FIELDS = ["a", "b", "out", "bias", "aux", "H", "W", "C", "OH", "OW", "F", "KH", "KW", "SH", "SW",
               "M", "N", "K", "act", "flags",
               # fast-division magics for the v3 kernels (filled by fill_gemm_divisors)
               "dvC", "dvKW", "dvOW", "dvOHW", "dvF", "dvW", "dvHW", "dvSH", "dvSW", "dvCp",
               "kper",      # GF_SPLITWS: k steps per split
               "ldb",       # LDS-tiled kernel: B row stride (0: K)
               "sbase",     # GF_SPLITWS: first workspace slot
               "ldo",       # 64-row WGRAD: output row stride (0: N)
               "adam",      # GF_ADAM: device AdamCtx
               "ext"]       # GF_NBNSUM: device NbnDesc of the fused Dense -> BN pair
GEMM_DTYPE = np.dtype([(f, _I) for f in GEMM_FIELDS])
BN_DTYPE = np.dtype([(f, _I) for f in ["x", "y", "dy", "dx", "gamma", "beta", "mm", "mv", "mean", "invstd", "ws",
                                       "dgamma", "dbeta", "pdb", "R", "C", "flags"]] + [("eps", np.float64),
                                                                                ("momentum", np.float64)])
POOL_DTYPE = np.dtype([(f, _I) for f in ["x", "y", "idx", "dy", "dx", "B", "H", "W", "C", "OH", "OW", "PH", "PW",
                                         "SH", "SW", "flags"]])
COPY_DTYPE = np.dtype([(f, _I) for f in ["src", "dst", "rows", "cols", "src_stride", "dst_stride", "flags"]])
EW_DTYPE = np.dtype([("a", _I), ("b", _I), ("out", _I), ("D", _I, (4,)), ("R", _I, (4,)), ("aJ", _I, (4,)),
                     ("aR", _I, (4,)), ("bJ", _I, (4,)), ("bR", _I, (4,)), ("ca", np.float32), ("cb", np.float32),
                     ("c", np.float32), ("pad", np.float32), ("flags", _I)])
EW_ELEMS = 2048        # ew.hip: destination elements per block
SPLITFIN_DTYPE = np.dtype([(f, _I) for f in ["ws", "out", "bias", "M", "N", "S", "act", "flags"]])
SPLITFIN_ELEMS = 2048  # aux.hip: outputs per block of the split-K finalize kernel
WGFIN_DTYPE = np.dtype([(f, _I) for f in ["ws", "out", "adam", "M", "N", "C", "Cp", "S", "ldo", "flags"]])
BIN_DTYPE = np.dtype([(f, _I) for f in ["g", "w", "bias", "gamma", "beta", "mean", "invstd", "act", "flags", "wc", "ldw",
                                        "Nc", "L", "F", "B", "E", "C0", "slab", "Hm", "cs", "part", "dw", "dbias",
                                        "adam", "ns"]])
BIN_VEC4 = 4           # bnbn.hip BinDesc::flags: bin_sw reads / writes 4 columns per lane
WGFIN_ELEMS = 64       # aux.hip: outputs per block of the split WGRAD finalize kernel
CONVPOOL_DTYPE = np.dtype([(f, _I) for f in ["x", "w", "bias", "y", "idx", "dy", "dw", "dbias", "B", "H", "W", "F",
                                             "KH", "KW", "SH", "SW", "OH", "OW", "PH", "PW", "PSH", "PSW", "POH",
                                             "POW", "act", "flags"]])
CONVPOOL_FWD_IMGS, CONVPOOL_WGRAD_IMGS, CONVPOOL_MAXPIX = 16, 32, 1024   # convpool.hip
GCHAIN_DTYPE = np.dtype([(f, _I) for f in ["g", "w1", "b1", "w2", "b2", "y", "dy", "dw1", "db1", "dw2", "db2",
                                           "gamma", "beta", "mm", "mv", "mean", "invstd", "ws", "wsb", "dgamma",
                                           "dbeta", "B", "L0", "L1", "T", "S", "F1", "F2", "act1", "act2", "flags",
                                           "rpb", "dvL1"]] + [("eps", np.float64), ("momentum", np.float64)])
GC_BN, GC_GAMMA, GC_BETA, GC_TRAIN = 1, 2, 4, 8          # gchain.hip GChainFlags
GC_FSTAT, GC_FAPPLY, GC_BSTAT, GC_BFULL = 0, 1, 2, 3     # gchain.hip modes
REPBITS_DTYPE = np.dtype([(f, _I) for f in ["logits", "out", "rows", "NC", "L"]])
LOSS_DTYPE = np.dtype([(f, _I) for f in ["logits", "dlogits", "labels", "target", "metrics", "NC", "L", "B", "flags"]]
                      + [("lb", np.float64)])

GF_VEC_A, GF_VEC_B, GF_ACCUM, GF_OUT_F32, GF_WSTORE, GF_SPLITWS, GF_BNSTAT = 1, 2, 4, 8, 16, 64, 128
GF_BNUSTAT = 1024      # FWD epilogue accumulates the consuming BN's unshifted phase-0 sums (BnDesc flag BN_USTAT)
BN_USTAT = 512
GF_NBNSUM = 512
GF_NOSTORE = 32
GF_ADAM = 256
GF_WSLAB = 2048        # Dense / 1x1 WGRAD m-split: fp32 slab per split + ordered wgrad_finalize (serann_hip.h)
ADAM_CTX_DTYPE = np.dtype([(f, _I) for f in ['p', 'm', 'v', 'pbf', 'g', 'lr_t', 'org_off', 'diverged', 'norg']]
                          + [(f, np.float32) for f in ['b1', 'b2', 'eps']]
                          + [("mode", np.int32)])
MOM_F32, MOM_16 = 0, 1            # AdamCtx.mode: fp32 moments, or bf16 m + log16 v (csrc/hip/common.h)
MODE_FWD, MODE_DGRAD, MODE_WGRAD = 0, 1, 2
ACT_CODES = {"linear": 0, "relu": 1, "sigmoid": 2}

BM, BN, BK = 64, 64, 32
RED_ELEMS = 16384      # aux.hip: elements per block of the channel-strided reductions (BN with C > 256)
POOL_ELEMS = 1024
COPY_ROWS = 16


@functools.lru_cache(maxsize=4096)
def fast_div_magic(d: int) -> int:
    """Packed (multiplier | shift << 32) for q = (umulhi(n, mul) + n) >> shift == n // d, exact for
    0 <= n < 2**31 (gemm3.hip fdiv)."""
    d = max(int(d), 1)
    sh = (d - 1).bit_length()
    mul = ((1 << 32) * ((1 << sh) - d)) // d + 1
    return int(mul | (sh << 32))


_DIVISOR_FIELDS = (("dvC", lambda a: a["C"]), ("dvKW", lambda a: a["KW"]), ("dvOW", lambda a: a["OW"]),
                   ("dvOHW", lambda a: a["OH"] * a["OW"]), ("dvF", lambda a: a["F"]), ("dvW", lambda a: a["W"]),
                   ("dvHW", lambda a: a["H"] * a["W"]), ("dvSH", lambda a: a["SH"]), ("dvSW", lambda a: a["SW"]),
                   ("dvCp", lambda a: -(-a["C"] // 8) * 8))


def fill_gemm_divisors(a: np.ndarray) -> np.ndarray:
    """Fill the dv* fields of a GEMM_DTYPE record array from its geometry fields (in place)."""
    for name, src in _DIVISOR_FIELDS:
        a[name] = [fast_div_magic(int(v)) for v in src(a)]
    return a


def record_array(rows, dtype) -> np.ndarray:
    """dict rows -> structured records of ``dtype`` (keys starting with '_' are planner annotations and
    skipped; missing fields are 0; an unknown field raises), filled column by column."""
    a = np.zeros(len(rows), dtype=dtype)
    keys = set()
    for r in rows:
        keys.update(r)
    names = set(dtype.names)
    for k in keys:
        if k.startswith("_"):
            continue
        if k not in names:
            raise ValueError(f"no field of name {k}")
        a[k] = [r.get(k, 0) for r in rows]
    return a


def gemm_desc_array(rows) -> np.ndarray:
    """dict rows -> GEMM_DTYPE records with the fast-division fields filled."""
    return fill_gemm_divisors(record_array(rows, GEMM_DTYPE))


BN_VEC_ELEMS = 16384   # aux.hip: elements per block of the vectorised (C <= 256) BatchNorm kernel

NBN_DTYPE = np.dtype([(f, _I) for f in ["x", "w", "bias", "y", "dy", "gamma", "beta", "mm", "mv", "mean", "invstd",
                                        "ws", "wsb", "dw", "db", "dgamma", "dbeta", "R", "F", "K", "ldx", "act",
                                        "flags"]] + [("eps", np.float64), ("momentum", np.float64)]
                     + [(f, _I) for f in ["part", "mtiles", "np"]])
# nbn.hip block sizes: elements per block of phase 2 (a streaming write; each block first rebuilds the
# per-channel scale / shift from the statistics workspace, so short blocks pay that prologue often), and
# the multiple of it taken by the reduction phases 4 / 5
NBN_ELEMS = int(_os.environ.get("SERANN_NBN_ELEMS", "16384"))
NBN_RED_MULT = int(_os.environ.get("SERANN_NBN_RED_MULT", "4"))
# phase 2 alone (no reduction, so its block boundaries do not touch the numerics): 131072 elements per block
# repeat its per-channel prologue 8x less often; ancestor step 5.40 -> 5.20 ms on one stream, 5.54 -> 5.40 at
# 4 stream groups, generation-3 mix neutral (profiles/r4/ab_nbn_phase2_elems.txt)
NBN_P2_ELEMS = int(_os.environ.get("SERANN_NBN_P2_ELEMS", "131072"))


def nbn_super_rows(units: int, phase: int) -> int:
    """Super-rows (8 rows) per nbn block: a function of the problem alone (the phase 4 / 5 block partial
    sums meet in fixed point, so their boundaries fix the rounding)."""
    if phase == 2:
        return max(1, (NBN_P2_ELEMS // 8) // int(units))
    return max(1, (NBN_ELEMS // 8) // int(units)) * NBN_RED_MULT


def nbn_chunks(rows: int, units: int, phase: int) -> int:
    """Blocks of a fused raw-input Dense -> BatchNormalization problem [rows][units] (nbn.hip)."""
    return -(-(-(-int(rows) // 8)) // nbn_super_rows(units, phase))


NBN_FIN_CH = 8      # nbn.hip nbn_fin_kernel: channels per block
NBN_NSUM = 8        # serann_hip.h: GF_NBNSUM sums per column


def nbn_fin_tiles(channels) -> np.ndarray:
    """int32 (ntiles, 4) tile table of an nbn phase-6 launch: (problem, first channel, 0, 0)."""
    out = [(p, f0, 0, 0) for p, F in enumerate(channels) for f0 in range(0, int(F), NBN_FIN_CH)]
    return np.asarray(out, dtype=np.int32).reshape(-1, 4)


def nbn_tiles(rows_units, phase: int) -> np.ndarray:
    """int32 (ntiles, 4) tile table of one nbn launch: (problem, first super-row, end super-row, first flag)
    for problems of (rows, units)."""
    out = []
    for p, (rows, units) in enumerate(rows_units):
        nsr = -(-int(rows) // 8)
        srb = nbn_super_rows(units, phase)
        s0 = np.arange(0, nsr, srb)
        if len(s0):
            out.append(np.stack([np.full(len(s0), p), s0, np.minimum(nsr, s0 + srb), (s0 == 0).astype(int)], 1))
    return np.concatenate(out).astype(np.int32) if out else np.zeros((0, 4), np.int32)


BN_RED_MULT = 4        # aux.hip: the statistics phases (0, 4) take BN_RED_MULT x the rows per block
BN_WS_STRIPES = 8      # serann_hip.h: copies of the [2C] BN statistics workspace (wide fixed point)
BN_STAT_SMALL = 2048    # aux.hip: ... unless the problem spans fewer blocks than this at 1x


def bn_ws_words(channels: int) -> int:
    """int64 words of one BatchNorm statistics workspace: BN_WS_STRIPES copies x 2C sums x (hi, lo)
    (csrc/hip/common.h fxw_add / fxw_sum)."""
    return BN_WS_STRIPES * 2 * int(channels) * 2


Q32 = float(2 ** 32)   # csrc/hip/common.h fxm_add: the loss metrics are int64 in 2^-32 units
QG = float(2 ** 40)    # csrc/hip/common.h fx_*: the gradient arena is int64 in 2^-40 units
QG_CLAMP = 2.0 ** 22   # fx_q clamps every contribution to +-2^22


def to_qg(t):
    """float tensor -> int64 gradient-arena fixed point (the kernels' fx_q: clamp, round to nearest)."""
    import torch
    return torch.round(t.double().clamp(-QG_CLAMP, QG_CLAMP) * QG).to(torch.int64)


def from_qg(t):
    """int64 gradient-arena tensor (device or host) -> float32 torch tensor on the same device."""
    return (t.double() / QG).float()


def moments_f32(m, v) -> tuple:
    """The Adam moment arenas as fp32 tensors, whatever their storage (csrc/hip/common.h MOM_*): fp32 as is,
    bf16 m widened, log16 v (16-bit code q held in int16: v = 2^(q / 819.2 - 48), q = 0: 0) decoded."""
    import torch
    if v.dtype == torch.int16:
        q = v.to(torch.int32) & 0xffff
        vf = torch.exp2(q.double() / 819.2 - 48.0).float()
        vf = torch.where(q == 0, torch.zeros_like(vf), vf)
        return m.float(), vf
    return m.float(), v.float()


def from_q32(t) -> np.ndarray:
    """int64 Q32 tensor (loss metrics) -> float64 numpy array."""
    return t.detach().cpu().numpy().astype(np.float64) / Q32


def adam_skip_mask(n: int, regions) -> np.ndarray:
    """Skip mask of the arena-wide Adam pass (adam.hip): one uint8 per 4-parameter group (plus the tail
    group), bit j = parameter 4i + j is updated by its WGRAD epilogue (GF_ADAM).  ``regions``: (first
    element, rows, cols, row stride) blocks of the parameter arena."""
    fused = np.zeros(((int(n) + 3) // 4) * 4, dtype=bool)
    for off, rows, cols, ld in regions:
        off, rows, cols, ld = int(off), int(rows), int(cols), int(ld)
        if rows <= 0 or cols <= 0:
            continue
        if ld == cols:
            fused[off:off + rows * cols] = True
        else:
            idx = off + np.arange(rows)[:, None] * ld + np.arange(cols)[None, :]
            fused[idx.ravel()] = True
    b = fused.reshape(-1, 4).astype(np.uint8)
    return (b[:, 0] | (b[:, 1] << 1) | (b[:, 2] << 2) | (b[:, 3] << 3)).astype(np.uint8)


def adam_skip_mask_device(n: int, regions, device):
    """:func:`adam_skip_mask` built on ``device`` without materialising a per-parameter array on the host
    (a 100M-parameter shard made that ~0.1 s of numpy per generation).  Every region row is a parameter
    range [s, e): the 4-parameter groups it covers whole get 0xF (a difference array + cumsum marks them),
    its at most 3 + 3 edge parameters their own bit.  Regions are disjoint parameter sets, so no bit is set
    twice and the edge bits add up to their OR."""
    import torch
    ng = (int(n) + 3) // 4
    starts, ends = [], []
    for off, rows, cols, ld in regions:
        off, rows, cols, ld = int(off), int(rows), int(cols), int(ld)
        if rows <= 0 or cols <= 0:
            continue
        if ld == cols:
            starts.append(np.array([off], np.int64))
            ends.append(np.array([off + rows * cols], np.int64))
        else:
            r0 = off + np.arange(rows, dtype=np.int64) * ld
            starts.append(r0)
            ends.append(r0 + cols)
    if not starts:
        return torch.zeros(ng, dtype=torch.uint8, device=device)
    s_, e_ = np.concatenate(starts), np.concatenate(ends)
    ga, gb = (s_ + 3) // 4, e_ // 4                  # whole groups [ga, gb)
    full = ga < gb
    idx = np.concatenate([ga[full], gb[full]])
    val = np.concatenate([np.ones(int(full.sum()), np.int32), -np.ones(int(full.sum()), np.int32)])
    edge_e = []
    for k in range(3):
        e = s_ + k                                   # head: before the first whole group
        edge_e.append(e[(e < e_) & (e < ga * 4)])
        e = gb * 4 + k                               # tail: after the last whole group
        edge_e.append(e[(e >= s_) & (e < e_) & (e >= ga * 4)])
    ee = np.unique(np.concatenate(edge_e))
    d = torch.zeros(ng + 1, dtype=torch.int32, device=device)
    d.index_add_(0, torch.as_tensor(idx, device=device), torch.as_tensor(val, device=device))
    m = (torch.cumsum(d[:ng], 0) > 0).to(torch.int32) * 15
    if len(ee):
        m.index_add_(0, torch.as_tensor(ee // 4, device=device),
                     torch.as_tensor((1 << (ee % 4)).astype(np.int32), device=device))
    return m.to(torch.uint8)


def bn_chunks(rows: int, channels: int, stats: bool = False) -> int:
    """Blocks of a BatchNorm problem [rows][channels] (aux.hip bn_kernel chunking); ``stats``: a
    statistics phase (0 or 4)."""
    c = max(int(channels), 1)
    if c > 256:
        return red_chunks(rows, c)
    nsr = -(-int(rows) // 8)
    srb1 = max(1, (BN_VEC_ELEMS // 8) // c)
    srb = srb1 * (1 if not stats or -(-nsr // srb1) < BN_STAT_SMALL else BN_RED_MULT)
    return -(-nsr // srb)


def pool_units(elements: int, channels: int) -> int:
    """Work units of a MaxPool problem (aux.hip: 8-channel vectors when C % 8 == 0)."""
    return int(elements) // (8 if int(channels) % 8 == 0 else 1)


def convpool_kt(kh: int, kw: int) -> int:
    """32-tap k steps of a fused conv+pool problem (convpool.hip instantiations 1..3)."""
    return -(-int(kh) * int(kw) // 32)


def convpool_variant(kh: int, kw: int, filters: int) -> int:
    """Kernel instantiation of a fused conv+pool problem: k steps * 8 + 16-filter tiles per block."""
    return convpool_kt(kh, kw) * 8 + min(4, -(-int(filters) // 16))


def convpool_ok(h: int, w: int, kh: int, kw: int, ph: int = 1, pw: int = 1) -> bool:
    """Shapes the fused first-layer Conv2D + MaxPool2D kernels accept (convpool.hip limits): the image
    fits the LDS copy, at most 3 k steps of taps, and at most 256 pool-window offsets (the argmax code
    is 8 bits, packed into the low mantissa bits of the max key)."""
    return (int(h) * int(w) <= CONVPOOL_MAXPIX and 1 <= convpool_kt(kh, kw) <= 3
            and int(ph) * int(pw) <= 256)


def gchain_variant(f1: int, f2: int, taps: int):
    """Instantiation (F1K * 8 + F2K) of the fused genotype chain for a Conv1D with ``f1`` filters and
    ``taps`` taps followed by a Dense of ``f2`` units, or None when gchain.hip has none: T <= 16,
    F1 <= 32 with F2 <= 128, or F1 <= 64 with F2 <= 64."""
    f1, f2 = int(f1), int(f2)
    f1k, f2k = -(-f1 // 32), -(-f2 // 32)
    if not 1 <= int(taps) <= 16 or f1 < 1 or f2 < 1:
        return None
    if (f1k == 1 and f2k <= 4) or (f1k == 2 and f2k <= 2):
        return f1k * 8 + f2k
    return None


# target blocks per PROBLEM per mode (gchain.hip; FSTAT, FAPPLY, BSTAT, BFULL).  Per problem, not per
# launch: a problem's row blocking -- and so the grouping of its fp32 partial sums before they meet in the
# fixed-point workspaces -- must not depend on which other organisms share the launch, or an organism would
# train differently in a 2-rank shard than in the whole population (deterministic sharding)
GCHAIN_BLOCKS = {0: 96, 1: 96, 2: 192, 3: int(_os.environ.get("SERANN_GCHAIN_BFULL_BLOCKS", "48"))}
GCHAIN_GMAX = 8192                                        # gchain.hip GC_GMAX: staged genotype elements


def gchain_genotype_elems(rpb: int, l1: int, l0: int) -> int:
    """Upper bound of the genotype elements one fused-chain block stages in LDS (gchain.hip
    gc_prologue): the rows [R0, R0 + rpb) of the [B * L1] conv output touch at most
    ceil(rpb / L1) + 1 batch rows of L0 genotype elements."""
    return (-(-int(rpb) // max(1, int(l1))) + 1) * int(l0)


def gchain_fits(l1: int, l0: int) -> bool:
    """A fused chain is eligible only when a block of the smallest row count (64) stages its genotype
    rows within GCHAIN_GMAX elements (otherwise the unfused kernels run it)."""
    return gchain_genotype_elems(64, l1, l0) <= GCHAIN_GMAX


def gchain_rpb(rows: int, mode: int, l1: int = 1, l0: int = 0) -> int:
    """Rows per block of one fused-chain problem of ``rows`` rows (conv output length ``l1``, genotype
    length ``l0``): a multiple of 64 (128 when the genotype staging allows; 4 waves x 32-row backward
    super-tiles) sized so the problem gets about GCHAIN_BLOCKS[mode] blocks (the full backward has fewer,
    longer blocks: one fixed-point atomic flush per gradient element and block), and small enough that the
    block's genotype rows fit the LDS staging buffer (raises when even 64 rows do not: gchain_fits must
    have excluded the chain).  A function of the problem alone (deterministic sharding)."""
    per = -(-int(rows) // GCHAIN_BLOCKS[int(mode)])
    rpb = max(128, -(-per // 128) * 128)
    rpb = min(rpb, -(-int(rows) // 128) * 128)
    if l0 > 0:
        while rpb > 64 and gchain_genotype_elems(rpb, l1, l0) > GCHAIN_GMAX:
            rpb -= 64
        if gchain_genotype_elems(rpb, l1, l0) > GCHAIN_GMAX:
            raise ValueError(f"fused genotype chain: {rpb} rows of L1={l1}, L0={l0} exceed the LDS staging "
                             f"buffer ({GCHAIN_GMAX} elements)")
    return rpb


def convpool_chunks(batch: int, filters: int, backward: bool, imgs: int = 0) -> int:
    """Blocks of one fused conv+pool problem: image chunks x groups of 64 filters (``imgs``: images
    per block, default CONVPOOL_WGRAD_IMGS / CONVPOOL_FWD_IMGS)."""
    per = imgs or (CONVPOOL_WGRAD_IMGS if backward else CONVPOOL_FWD_IMGS)
    return -(-int(batch) // per) * -(-int(filters) // 64)


# blocks one fused conv+pool problem should have at least.  At 16 (round 2) a B = 750 problem ran in 24
# WGRAD / 47 FWD blocks -- one block per CU on under a fifth of the chip, 150-260 us each on the bench
# population (profiles/r3b/launch_table_before.txt); 160 takes both down to 4 images per block (188 blocks)
CONVPOOL_MIN_CHUNKS = int(_os.environ.get("SERANN_CONVPOOL_MIN_CHUNKS", "160"))


def convpool_imgs(batch: int, filters: int, backward: bool) -> int:
    """Images per block of one fused conv+pool problem: 32 (WGRAD) / 16 (FWD), halved (down to 4: one
    image per wave) while the problem alone has fewer than CONVPOOL_MIN_CHUNKS blocks.  Per problem, so
    the grouping of the WGRAD partial sums does not depend on the other problems of the launch
    (deterministic sharding)."""
    imgs = CONVPOOL_WGRAD_IMGS if backward else CONVPOOL_FWD_IMGS
    while imgs > 4 and convpool_chunks(batch, filters, backward, imgs) < CONVPOOL_MIN_CHUNKS:
        imgs //= 2
    return imgs


def convpool_wgrad_imgs(batch: int, filters: int) -> int:
    return convpool_imgs(batch, filters, True)


def red_chunks(rows: int, channels: int) -> int:
    """Blocks needed by a BN / act_bwd problem of shape [rows][channels]."""
    per = max(1, RED_ELEMS // max(int(channels), 1))
    return -(-int(rows) // per)


def lib(required: bool = True):
    return load("serann_hip", required=required)


def available() -> bool:
    try:
        import torch
        if not torch.cuda.is_available():
            return False
        m = lib(required=False)
        return m is not None
    except Exception:
        return False


def check_layouts():
    sizes = lib().desc_sizes()
    for name, dt in [("GemmDesc", GEMM_DTYPE), ("BnDesc", BN_DTYPE), ("EwDesc", EW_DTYPE),
                     ("PoolDesc", POOL_DTYPE), ("CopyDesc", COPY_DTYPE), ("LossDesc", LOSS_DTYPE),
                     ("TransDesc", TRANS_DTYPE), ("ImcolDesc", IMCOL_DTYPE), ("SplitFinDesc", SPLITFIN_DTYPE),
                     ("WgFinDesc", WGFIN_DTYPE),
                     ("ConvPoolDesc", CONVPOOL_DTYPE), ("GChainDesc", GCHAIN_DTYPE),
                     ("RepBitsDesc", REPBITS_DTYPE), ("NbnDesc", NBN_DTYPE), ("AdamCtx", ADAM_CTX_DTYPE),
                     ("BinDesc", BIN_DTYPE)]:
        if sizes[name] != dt.itemsize:
            raise RuntimeError(f"descriptor layout mismatch for {name}: C++ {sizes[name]} vs numpy {dt.itemsize}")


# ---- strided elementwise rows (ew.hip): the interpreter's rare ops --------------------------------------
def _pad4(v, fill):
    v = [int(x) for x in v]
    if len(v) > 4:
        raise ValueError(f"ew: rank {len(v)} > 4")
    return [fill] * (4 - len(v)) + v


def _dense_strides(shape):
    st, acc = [], 1
    for d in reversed([int(x) for x in shape]):
        st.append(acc)
        acc *= d
    return list(reversed(st))


def _bcast_strides(src_shape, shape):
    """Element strides reading a dense ``src_shape`` tensor broadcast to ``shape`` (same rank)."""
    if len(src_shape) != len(shape):
        raise ValueError("ew: broadcast operands need equal ranks")
    st = _dense_strides(src_shape)
    return [0 if int(s) == 1 and int(d) != 1 else st[k] for k, (s, d) in enumerate(zip(src_shape, shape))]


def ew_map_row(out, shape, a, a_shape, ca=1.0, b=0, b_shape=None, cb=0.0, c=0.0, accum=False) -> dict:
    """out[shape] (+)= ca * A + cb * B + c, A / B dense tensors of ``a_shape`` / ``b_shape`` broadcast to
    ``shape`` (full shapes, batch included).  Row for EW_DTYPE; count = ew_count(row)."""
    one = [1, 1, 1, 1]
    return dict(a=a, b=b, out=out, D=_pad4(shape, 1), R=one, aJ=_pad4(_bcast_strides(a_shape, shape), 0),
                aR=[0] * 4, bJ=_pad4(_bcast_strides(b_shape, shape), 0) if b else [0] * 4, bR=[0] * 4,
                ca=float(ca), cb=float(cb), c=float(c), pad=0.0, flags=1 if accum else 0)


def ew_reduce_row(out, out_shape, src, src_shape, scale=1.0, accum=False) -> dict:
    """out[out_shape] (+)= scale * (src summed over the dimensions where ``out_shape`` is 1 and
    ``src_shape`` is not): the gradient of an operand broadcast to ``src_shape``."""
    st = _dense_strides(src_shape)
    red = [int(o) == 1 and int(s) != 1 for o, s in zip(out_shape, src_shape)]
    return dict(a=src, b=0, out=out, D=_pad4(out_shape, 1),
                R=_pad4([int(s) if r else 1 for s, r in zip(src_shape, red)], 1),
                aJ=_pad4([0 if r else st[k] for k, r in enumerate(red)], 0),
                aR=_pad4([st[k] if r else 0 for k, r in enumerate(red)], 0),
                bJ=[0] * 4, bR=[0] * 4, ca=float(scale), cb=0.0, c=0.0, pad=0.0, flags=1 if accum else 0)


def ew_permute_row(out, src, dims, perm, accum=False) -> dict:
    """out (dense, dims permuted by ``perm``) (+)= src (dense ``dims``): out[i_perm] = src[i]."""
    st = _dense_strides(dims)
    return dict(a=src, b=0, out=out, D=_pad4([dims[p] for p in perm], 1), R=[1, 1, 1, 1],
                aJ=_pad4([st[p] for p in perm], 0), aR=[0] * 4, bJ=[0] * 4, bR=[0] * 4,
                ca=1.0, cb=0.0, c=0.0, pad=0.0, flags=1 if accum else 0)


def ew_count(row) -> int:
    n = 1
    for d in row["D"]:
        n *= int(d)
    return -(-n // EW_ELEMS)


OPERAND_SLACK_BYTES = 256   # readable memory every kernel operand must have behind its last element


def operand(shape, dtype, device, zero: bool = True):
    """A kernel operand of ``shape``: contiguous, followed by OPERAND_SLACK_BYTES of zeroed memory.

    Contract of every gemm3 / conv / BN kernel: a 16-B fragment load may start at any valid element,
    so up to 14 bytes past an operand's last element are read (the over-read lanes are masked, never
    used).  Plain ``torch.empty`` tensors can end at the last mapped byte of an allocator segment, where
    that read faults the GPU; every buffer handed to these kernels comes from here (or an engine arena,
    which keeps the same slack)."""
    import torch
    shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list, torch.Size)) else (shape,)))
    n = 1
    for s in shape:
        n *= s
    esz = torch.empty(0, dtype=dtype).element_size()
    extra = -(-OPERAND_SLACK_BYTES // esz)
    buf = (torch.zeros if zero else torch.empty)(n + extra, dtype=dtype, device=device)
    if not zero:
        buf[n:].zero_()
    return buf[:n].view(shape)


def padded(t):
    """``t``'s values as a kernel operand (see :func:`operand`)."""
    out = operand(t.shape, t.dtype, t.device, zero=False)
    out.copy_(t)
    return out


def stream_handle():
    import torch
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


# ------------------------------------------------------------------------------------------------
# tile tables
# ------------------------------------------------------------------------------------------------
TRANS_DTYPE = np.dtype([(f, _I) for f in ["src", "dst", "F", "P", "C"]])
IMCOL_DTYPE = np.dtype([(f, _I) for f in ["x", "out", "B", "H", "W", "OH", "OW", "KH", "KW", "SH", "SW", "K8"]])
IMCOL_ROWS = 64
TRANS_ELEMS = 4096


# rows per wave (16-row tiles) of the direct-fragment DGRAD onto <= 16 channels (instantiated: 2, 4, 8; 2 measured
# 3 % slower on the generation-15 mix, profiles/r6/ab_dgrad_nt1_rt2_rejected.txt)
DGRAD_NT1_RT = int(_os.environ.get("SERANN_DGRAD_NT1_RT", "4"))


def gemm3_variant(mode: int, M: int, N: int, K: int, geo: dict) -> int:
    """Kernel instantiation of the v3 kernels (gemm3.hip launch_gemm3 encoding) for one problem.

    FWD/DGRAD: NT (BN/16) + 10*RT + 100*KW + 1000*GEN; WGRAD: BMF*1000 + BNK + 1000000*GEN.
    GEN (element-gather fallback) only for problems whose reduction chunks can wrap more than one
    kernel row (KW*C < 8) or straddle output pixels in DGRAD (F % 8 != 0 on a KHxKW > 1 kernel)."""
    KH, KW, C, W, F = (int(geo.get(k, 1)) for k in ("KH", "KW", "C", "W", "F"))
    im2col_gen = KW * C < 8 and W != KW and KH > 1
    if mode == MODE_WGRAD:
        bmf = 16 if M <= 16 else (32 if M <= 32 else 64)
        # (wider f tiles -- 96-row, 128 / 160 / 192-row with 4 or 8 waves -- and 32-row tail tiles were
        # measured slower on the bench population in round 2 and removed: profiles/r2e/ab_wgrad96.txt,
        # ab_wgrad_tail32.txt, profiles/r2_wide_ab.txt)
        if N <= 16:                      # narrow reduction width: waves split f, one 16-column tile
            return 64 * 1000 + 16 + (1000000 if im2col_gen else 0)
        if bmf == 16:
            bnk = 256 if N > 128 else (128 if N > 64 else 64)
        else:
            bnk = 128 if N > 64 else 64
        return bmf * 1000 + bnk + (1000000 if im2col_gen else 0)
    gen = im2col_gen if mode == MODE_FWD else (F % 8 != 0 and KH * KW > 1)
    nt = 1 if N <= 16 else (2 if N <= 32 else (4 if N <= 64 else 8))
    if K <= 32 and not gen and M >= 16384 and "sk" not in _OFF:       # single k step: store-bound, keep registers low
        return 5000 + nt + 10 * (2 if nt == 8 else 4)
    kw = M <= 8192 and -(-K // BK) >= 16
    rt = 2 if (kw or nt == 8 or M < 16384) else 4
    if mode == MODE_DGRAD and nt == 1 and rt == 4:
        rt = DGRAD_NT1_RT                  # conv DGRAD onto <= 16 channels (A/B knob)
    return nt + 10 * rt + (100 if kw else 0) + (1000 if gen else 0)


def gemm3_block(mode: int, variant: int):
    """(rows, cols) of the output tile one block of a v3 launch covers."""
    if mode == MODE_WGRAD:
        if 8000000 < variant < 8000010:
            return (16, 16 * (variant - 8000000))      # small-bank WGRAD: the whole [F x N] tile
        v = variant % 1000000
        return (v // 1000, (v % 1000) % 500)
    if mode == MODE_FWD and 5100 < variant < 5200:
        return (256, 16 * (variant % 10))           # shared-input FWD: 256 rows, one column tile
    if 7000 < variant % 10000 < 7300 and variant < 20000:
        return (128, variant % 10000 - 7000)
    if 8000 < variant % 10000 < 8300 and variant < 20000:
        return (128, variant % 10000 - 8000)
    if variant >= 5000:
        return (64 * ((variant // 10) % 10), 16 * (variant % 10))
    nt, rt, kw = variant % 10, (variant // 10) % 10, (variant % 1000) >= 100
    return (16 * rt if kw else 64 * rt, 16 * nt)


CONV_PATCH_TIERS = (8192, 16384, 32768)   # gemm3.hip: LDS patch capacities (bf16 elements)


def conv_lds_config(geo: dict, N: int):
    """(RT, patch tier) for the LDS-halo FWD conv kernel (64*RT output pixels per block), or None
    when the problem is not a KHxKW > 1 convolution or its input patch does not fit in 64 KB.
    Prefers the largest RT (more MFMA work per staged patch and per barrier) whose padding of the
    per-image pixel count stays within 20% of the smallest tiling, then the smallest patch tier that
    holds it (more blocks resident per CU)."""
    KH, KW, C, W, OH, OW, SH = (int(geo[k]) for k in ("KH", "KW", "C", "W", "OH", "OW", "SH"))
    if KH * KW <= 1 or "conv_fwd" in _OFF:
        return None
    cp = -(-C // 8) * 8
    cs = cp if (cp // 8) % 2 == 1 else cp + 8
    ohw = OH * OW
    min_pad = -(-ohw // 64) * 64
    for rt in (4, 2, 1):
        tm = 64 * rt
        if -(-ohw // tm) * tm > 1.2 * min_pad and rt > 1:
            continue
        span = (OW - 1 + tm - 1) // OW
        need = (span * SH + KH) * W * cs
        for tier, cap in enumerate(CONV_PATCH_TIERS):
            if need <= cap:
                return rt, tier
    return None


def conv_wgrad_cs(C: int, SW: int) -> int:
    """Channel stride of a conv WGRAD patch pixel in LDS (gemm3.hip conv_wgrad_cs): Cp = ceil8(C) rounded up to
    an odd number of 16-B slots."""
    cp = -(-int(C) // 8) * 8
    return cp if (cp // 8) % 2 == 1 else cp + 8


def conv_wgrad_ipc(geo: dict, tier: int) -> int:
    """Whole images per 128-row chunk of the conv WGRAD kernel (gemm3.hip g3_conv_wgrad_kernel):
    min(128 // (OH*OW), patch capacity // (H*W*Cs)) when that is >= 2, else 1 (per-image pixel tiles)."""
    H, W, C, OH, OW = (int(geo[k]) for k in ("H", "W", "C", "OH", "OW"))
    cs = conv_wgrad_cs(C, int(geo.get("SW", 1)))
    ohw = OH * OW
    ipc = min(128 // ohw, CONV_PATCH_TIERS[tier] // (H * W * cs)) if ohw < 128 else 0
    return ipc if ipc >= 2 else 1


def conv_wgrad_config(geo: dict, F: int):
    """(BMF, BNK, patch tier) for the LDS-halo conv WGRAD kernel (128-pixel chunks), or None.  Small
    outputs take the smallest tier that packs all the images a chunk can hold (multi-image chunks)."""
    KH, KW, C, W, OH, OW, SH = (int(geo[k]) for k in ("KH", "KW", "C", "W", "OH", "OW", "SH"))
    if KH * KW <= 1 or "conv_wgrad" in _OFF:
        return None
    cp = -(-C // 8) * 8
    cs = conv_wgrad_cs(C, int(geo.get("SW", 1)))
    # output rows a 128-pixel chunk spans beyond its first (at most the image's), and the input rows they read
    span = min((OW - 1 + 127) // OW, OH - 1)
    need = (span * SH + KH) * W * cs
    tier = next((i for i, cap in enumerate(CONV_PATCH_TIERS) if need <= cap), None)
    if tier is None:
        return None
    # the 64 KB tier is built for 16-filter blocks only (two LDS-DMA stages of it fill the LDS): wider layers keep
    # their whole-F blocks (4 filter tiles per B fragment) on the smaller tiers whenever the patch fits them
    tiers = range(len(CONV_PATCH_TIERS)) if F <= 16 or tier == 2 else range(2)
    if OH * OW < 128 and "conv_wgrad_multi" not in _OFF:
        want = 128 // (OH * OW)
        best = max(tiers, key=lambda t_: (min(conv_wgrad_ipc(geo, t_), want), -t_))
        if conv_wgrad_ipc(geo, best) >= 2:
            tier = best
    # (the 64 KB patch tier is built for 16-filter blocks only: two LDS-DMA stages of it fill the CU's LDS)
    bmf = 16 if F <= 16 or tier == 2 else (32 if F <= 32 else 64)
    return bmf, conv_wgrad_bnk(KH * KW * cp, bmf), tier


def conv_wgrad_bnk(kp: int, bmf: int) -> int:
    """Columns of the padded (tap, Cp) reduction space one conv WGRAD block covers (gemm3.hip: 4 waves x
    NTW = BNK / 64 column tiles of 16, every wave all BMF filters): the whole width when the accumulators
    allow it (TF x NTW <= 32 tiles of 4 registers per lane), so the staged patch of a chunk -- the kernel's
    dominant traffic -- is read once for every tap; at least 2 tiles per wave."""
    ntw_max = max(2, min(CONV_WGRAD_BNK_MAX // 64, 32 // (bmf // 16)))
    ntw = 2
    while ntw < ntw_max and 64 * ntw < kp:
        ntw *= 2
    return 64 * ntw


def conv_wgrad_splits(nchunks: int, wave_mfmas_per_chunk: int, tiles: int = 1, slab_bytes: int = 0) -> int:
    """Chunk-range splits of one conv WGRAD problem (gemm3.hip g3_conv_wgrad_kernel): enough that no block
    runs more than CONV_WGRAD_WAVE_MFMAS MFMAs per wave or CONV_WGRAD_MAX_CHUNKS chunks (a chunk's patch
    staging is latency-bound, so narrow problems are bounded by chunks, wide ones by MFMAs), and at least
    CONV_WGRAD_MIN_CHUNKS chunks per block.  The splits meet in per-split fp32 slabs summed in order by the
    wgrad_finalize launch, so their cost is slab bytes (plain stores), not fixed-point atomics.  A function of
    the problem alone (deterministic: the split boundaries decide the partial sums)."""
    want = max(-(-nchunks * wave_mfmas_per_chunk // CONV_WGRAD_WAVE_MFMAS), -(-nchunks // CONV_WGRAD_MAX_CHUNKS))
    # ... but no more than CONV_WGRAD_MAX_BLOCKS blocks per problem (tiles = its f x column tiles) and
    # CONV_WGRAD_MAX_SLAB_MB of fp32 slabs (slab_bytes = one split's slab): a problem with thousands of chunks
    # (the RiboAE's 350 x 50 maps at batch 512: 8000) fills the GPU with long chunk ranges instead of
    # thousands of splits whose slabs the finalize must read back (205 MB per step there)
    cap = max(1, CONV_WGRAD_MAX_BLOCKS // max(1, tiles))
    if slab_bytes > 0:
        cap = min(cap, max(1, (CONV_WGRAD_MAX_SLAB_MB << 20) // slab_bytes))
    return max(1, min(want, cap, nchunks // CONV_WGRAD_MIN_CHUNKS))


NARROW_ROWS, NARROW_WROWS = 256, 1024   # gemm3.hip narrow (K <= 4) kernels: rows per block
# rows per block of a statistics-only narrow FWD (GF_BNSTAT | GF_NOSTORE, super-row kernel; a multiple of 8)
NARROW_NOSTORE_ROWS = int(_os.environ.get("SERANN_NARROW_NOSTORE_ROWS", "2048"))

# A/B switches for measurements and fault isolation (all paths are on by default)
_OFF = set(filter(None, _os.environ.get("SERANN_GEMM3_OFF", "").split(",")))   # conv_fwd,conv_wgrad,narrow,sk


def narrow_k(geo: dict, mode: int, M: int, N: int, K: int):
    """Reduction width of a 1x1 / Dense problem that the narrow VALU kernels take (K <= 4, N <= 256,
    no stride, no accumulate), else None."""
    if int(geo.get("KH", 1)) * int(geo.get("KW", 1)) != 1 or int(geo.get("SH", 1)) * int(geo.get("SW", 1)) != 1:
        return None
    if int(geo.get("flags", 0)) & (GF_ACCUM | GF_OUT_F32) or "narrow" in _OFF:
        return None
    if mode == MODE_FWD and K <= 4 and N <= 256:
        return K
    if mode == MODE_WGRAD and N <= 4 and M <= 256:
        return N
    return None


# Shared-input FWD (gemm3.hip g3_shared_fwd_kernel): first-layer problems over one materialised im2col matrix
# (rows annotated ``_imcol`` by the engine) run as runs of problems per 256-row block; a launch aims at this many
# blocks (problem runs are split until it is reached, or one problem per run)
SHARED_FWD_BLOCKS = int(_os.environ.get("SERANN_SHARED_FWD_BLOCKS", "1024"))
SHARED_FWD_MAXC, SHARED_FWD_MAXN = 96, 64
# problems per matrix to share (1: every eligible row, so the kernel that computes a problem -- and its bits -- do
# not depend on which organisms share its launch, shard or stream group)
SHARED_FWD_MIN = int(_os.environ.get("SERANN_SHARED_FWD_MIN", "1"))


def shared_fwd_ok(r: dict, M: int, N: int, K: int) -> bool:
    """True when FWD row ``r`` may join a shared-input run: an im2col first layer (``_imcol``) whose row stride
    (C = K8) fits the kernel's 3 register-held k steps, one column tile of at most 64 filters, plain bf16 output."""
    if "shared" in _OFF or not r.get("_imcol"):
        return False
    flags = int(r.get("flags", 0))
    return (int(r["C"]) <= SHARED_FWD_MAXC and N <= SHARED_FWD_MAXN and K <= int(r["C"])
            and not flags & (GF_ACCUM | GF_OUT_F32 | GF_SPLITWS) and not r.get("_force_tiled") and not r.get("_split"))


def shared_fwd_variant(C: int, maxN: int) -> int:
    """gemm3.hip g3_shared_fwd_kernel<NT, KS> encoding: 5100 + 10 * KS + NT."""
    nt = 1 if maxN <= 16 else (2 if maxN <= 32 else 4)
    return 5100 + 10 * -(-int(C) // 32) + nt


def shared_fwd_tiles(items) -> tuple:
    """Tile table of one shared-input FWD launch: ``items`` (row, (M, N, K)) reordered so the problems of one
    im2col matrix are consecutive, then per matrix its m tiles x runs of problems, the runs of one m tile on one
    XCD (they read the same A rows).  Returns (items, int32 (n, 4) tiles (first problem, m tile, count, 0))."""
    order = sorted(range(len(items)), key=lambda i: (int(items[i][0]["a"]), i))
    items = [items[i] for i in order]
    tl = []
    p = 0
    while p < len(items):
        a = int(items[p][0]["a"])
        q = p
        while q < len(items) and int(items[q][0]["a"]) == a:
            q += 1
        n, M = q - p, int(items[p][1][0])
        mt = -(-M // 256)
        nch = max(1, min(n, -(-SHARED_FWD_BLOCKS // mt)))
        per = -(-n // nch)
        starts = np.arange(p, q, per)
        t_ = np.empty((mt, len(starts), 4), np.int64)
        t_[..., 0] = starts[None, :]
        t_[..., 1] = np.arange(mt)[:, None]
        t_[..., 2] = np.minimum(per, q - starts)[None, :]
        t_[..., 3] = 0
        tl.append(xcd_swizzle(t_.reshape(-1, 4), len(starts)))
        p = q
    return items, np.concatenate(tl).astype(np.int32)


# k steps (32 rows) per small-bank WGRAD block; 0: the Dense WGRAD rule (wgrad_target)
TINY_WGRAD_TARGET = int(_os.environ.get("SERANN_TINY_WGRAD_TARGET", "0"))


def tiny_wgrad_ok(r: dict, M: int, N: int, K: int) -> bool:
    """WGRAD row for g3_wgrad_tiny_kernel: a 1x1 stride-1 problem whose whole [F x N] output is one 16-row MFMA
    tile of at most 4 column tiles (F <= 16, N <= 64) over a reduction long enough to split (>= 64 k steps: the
    first layers over the shared im2col matrix); a function of the problem alone."""
    if "tiny" in _OFF or M > 16 or N > 64 or -(-K // BK) < 64:
        return False
    return all(int(r.get(k, 1)) == 1 for k in ("KH", "KW", "SH", "SW"))


def shared_wgrad_order(rows, tiles: np.ndarray) -> np.ndarray:
    """WGRAD tiles of first layers over one im2col matrix (rows annotated ``_imcol``, the matrix at ``b``): the
    tiles of all its problems that read the same row range are made consecutive and dispatched to one XCD, so the
    matrix rows are fetched into that XCD's L2 once for every organism's filter bank instead of once per organism.
    Tiles are independent (plain stores, per-split slabs or fixed-point atomics), so only the order changes."""
    if "wshare" in _OFF or len(tiles) == 0:
        return tiles
    first, sid = {}, np.full(len(rows), -1, np.int64)
    for p, r in enumerate(rows):
        if r.get("_imcol"):
            sid[p] = first.setdefault(int(r["b"]), p)
    counts = np.bincount(sid[sid >= 0], minlength=len(rows)) if (sid >= 0).any() else np.zeros(len(rows), int)
    shared = counts[sid.clip(0)] >= 2
    shared &= sid >= 0
    ts = shared[tiles[:, 0]]
    if not ts.any():
        return tiles
    rest, sh = tiles[~ts], tiles[ts]
    k0 = sh[:, 3].astype(np.int64) & 0xffff
    order = np.lexsort((sh[:, 0], sh[:, 1], sh[:, 2], k0, sid[sh[:, 0]]))
    sh = sh[order]
    out = []
    g0 = sid[sh[:, 0]]
    for s in np.unique(g0):
        blk = sh[g0 == s]
        out.append(xcd_swizzle(blk, int(counts[s])))
    return np.concatenate([rest] + out).astype(tiles.dtype)


TILED_BNS = (64, 128, 160, 192)               # gemm3.hip g3_tiled_kernel instantiations


def tiled_bn(N: int) -> int:
    """Column tile of the LDS-tiled 1x1 / Dense kernel: the smallest instantiation covering N (one n tile
    reads the A panel once), 128-column tiles beyond 192."""
    if "wide" in _OFF:
        return 128 if N > 64 else 64
    for bn in TILED_BNS:
        if N <= bn:
            return bn
    return 128


def _merge_tiled_widths(groups: dict) -> None:
    """All LDS-tiled problems of one launch group with N > 64 share ONE column-tile width (128, 160 or
    192): every distinct width is a separate launch, and a launch of a few dozen blocks costs its full
    latency -- on a generator population, per-problem widths turned 12 tiled launches per step into 30
    and the step 0.6 ms slower.  The shared width minimises the computed columns (ceil(N / bn) * bn per
    problem, weighted by M * K), with wider tiles charged for their lower occupancy."""
    for base in (7000, 8000):
        keys = [k for k in groups if k in (base + 128, base + 160, base + 192)]
        if len(keys) <= 1:
            continue
        items = [it for k in keys for it in groups.pop(k)]
        best, best_cost = 128, None
        for bn, penalty in ((128, 1.0), (160, 1.15), (192, 1.2)):
            cost = penalty * sum(-(-N // bn) * bn * float(M) * float(K) for _, (M, N, K) in items)
            if best_cost is None or cost < best_cost:
                best, best_cost = bn, cost
        groups[base + best] = items


def gemm3_plan(mode: int, rows, dims, splitk: bool = False):
    """Group the problems of one grouped launch by v3 kernel instantiation.

    Returns [(variant, rows, tiles int32 (n, 4))].  FWD convolutions whose input patch fits in LDS go
    to the halo kernel (tiles (prob, image, first pixel, column tile)); everything else to the
    direct / WGRAD kernels (tiles (prob, m tile, n tile, k range)).
    ``splitk``: LDS-tiled FWD problems with few output tiles and a long reduction get k splits (rows
    marked ``_split`` = number of splits, plus GF_SPLITWS and kper); the caller provides the fp32
    workspace (``aux``) and runs splitk_finalize after the launch."""
    groups = {}
    # shared-input runs: im2col first layers of >= 2 problems over one matrix (widest filter bank sets the variant)
    share = {}
    if mode == MODE_FWD:
        for r, (M, N, K) in zip(rows, dims):
            if narrow_k(r, mode, M, N, K) is None and shared_fwd_ok(r, M, N, K):
                n_, mx = share.get(int(r["a"]), (0, 0))
                share[int(r["a"])] = (n_ + 1, max(mx, N))
    for r, dm in zip(rows, dims):
        M, N, K = dm
        v = None
        nk = narrow_k(r, mode, M, N, K) if mode in (MODE_FWD, MODE_WGRAD) and not r.get("_nonarrow") else None
        sh = share.get(int(r.get("a", 0))) if share and nk is None and shared_fwd_ok(r, M, N, K) else None
        if r.get("_force_tiled"):
            v = 7000 + tiled_bn(N)                # K slice of a concat input: LDS-tiled + workspace
        elif sh is not None and sh[0] >= SHARED_FWD_MIN:
            v = shared_fwd_variant(int(r["C"]), sh[1])
        elif nk is not None:
            # + 100: LDS-staged rows when the narrow kernel's row width (N, or F for WGRAD) is not a
            # multiple of 8 (unaligned 16-B row chunks); measured faster for K <= 2 (Dense on the raw
            # genotype / image: FWD 3-4x), slower for K = 3, 4
            # + 200: the super-row form (aligned 16-B accesses, no staging; row width > 8, any K)
            wide = N if mode == MODE_FWD else M
            st = wide % 8 != 0 and nk <= 2 and "nst" not in _OFF
            sr = wide % 8 != 0 and wide > 8 and "sr" not in _OFF
            v = (6000 if mode == MODE_FWD else 4000000) + nk + (200 if sr else 100 if st else 0)
        elif (mode in (MODE_FWD, MODE_DGRAD) and "tiled" not in _OFF and K > 32
              and int(r.get("KH", 1)) * int(r.get("KW", 1)) == 1 and int(r.get("SH", 1)) * int(r.get("SW", 1)) == 1):
            v = 7000 + tiled_bn(N)                # LDS-tiled 1x1 / Dense GEMM
            if mode == MODE_DGRAD and r.get("_bnat") and "bt" not in _OFF:
                # natural-layout weights read k-major (no transposed copy needed)
                v += 1000
                r["b"] = r["_bnat"]
                r["ldb"] = int(r.get("_bnat_ld", 0))
            if mode == MODE_DGRAD and int(r.get("flags", 0)) & GF_NBNSUM:
                v += 10000                        # the instantiation with the BN-backward-sums epilogue
            if mode == MODE_FWD and splitk:
                # (split count from the problem's own column tile, not the launch's shared width below:
                # the split boundaries decide the fp32 partial sums, so they must not depend on the
                # other problems of the launch)
                ns = tiled_fwd_splits(M, N, K, tiled_bn(N), int(r.get("flags", 0)))
                if ns > 1:
                    r["_split"] = ns
        elif mode == MODE_FWD and not (r.get("flags", 0) & GF_ACCUM):
            cfg = conv_lds_config(r, N)
            if cfg is not None:
                nt = 1 if N <= 16 else (2 if N <= 32 else 4)
                v = 2000 + nt + 10 * cfg[0] + 100 * cfg[1]
        if mode == MODE_WGRAD and v is None:
            cfg = conv_wgrad_config(r, M)
            if cfg is not None:
                v = 3000000 + 100000 * cfg[2] + cfg[0] * 1000 + cfg[1] // 64   # (BNK / 64: column tiles per wave)
        if mode == MODE_WGRAD and v is None and tiny_wgrad_ok(r, M, N, K):
            v = 8000000 + (1 if N <= 16 else (2 if N <= 32 else 4))     # small-bank WGRAD (g3_wgrad_tiny_kernel)
        if v is None:
            v = gemm3_variant(mode, M, N, K, r)
            if mode == MODE_WGRAD and WGRAD_WIDE and 64 < M <= 192 and N > 16 and v < 1000000 \
                    and -(-K // BK) <= WGRAD_WIDE_MAXK:
                # one f tile over the whole layer: the X panel of a column tile is read once, not once per
                # 64-row f tile (a function of the problem alone: its single split is kept)
                v = next(b for b in (96, 128, 160, 192) if M <= b) * 1000 + 64
            if mode == MODE_WGRAD and dwgrad_ok(r, M, N, v):
                # LDS-DMA ring kernel (+ 500: act' from a staged Y tile)
                v = 5000000 + v + (500 if int(r.get("act", 0)) else 0)
            elif mode == MODE_WGRAD:
                bm_, bn_ = gemm3_block(mode, v)
                if wgrad_row_groups(M, N, K, bm_, bn_) == 2:
                    v += 500
        groups.setdefault(v, []).append((r, dm))
    _merge_tiled_widths(groups)
    out = []
    for v in sorted(groups):
        items = groups[v]
        if (mode == MODE_FWD and 6000 <= v < 7000) or (mode == MODE_WGRAD and 4000000 <= v < 5000000):
            tl = []
            for p, (r, (M, N, K)) in enumerate(items):
                per = NARROW_ROWS if mode == MODE_FWD else NARROW_WROWS
                if mode == MODE_FWD and v % 1000 >= 200 and int(r.get("flags", 0)) & GF_NOSTORE:
                    # statistics-only super-row pass: longer row blocks (the kernel reads them from kper)
                    per = NARROW_NOSTORE_ROWS
                    r["kper"] = per
                nrows = M if mode == MODE_FWD else K
                nb = -(-nrows // per)
                tl.append(np.stack([np.full(nb, p), np.arange(nb), np.zeros(nb, int), np.zeros(nb, int)], 1))
            tiles = np.concatenate(tl).astype(np.int32)
        elif mode == MODE_FWD and 5100 < v < 5200:
            items, tiles = shared_fwd_tiles(items)
        elif 2000 <= v < 3000 and mode in (MODE_FWD, MODE_DGRAD):
            nt, rt = v % 10, (v // 10) % 10
            tm, bn = 64 * rt, 16 * nt
            tl = []
            for p, (r, (M, N, K)) in enumerate(items):
                ohw = int(r["OH"]) * int(r["OW"])
                nb = M // ohw
                tpi = -(-ohw // tm)
                ntn = -(-N // bn)
                bb, jj, nn = np.meshgrid(np.arange(nb), np.arange(tpi), np.arange(ntn), indexing="ij")
                tl.append(np.stack([np.full(bb.size, p), bb.ravel(), jj.ravel() * tm, nn.ravel()], 1))
            tiles = np.concatenate(tl).astype(np.int32)
        elif 3000000 <= v < 4000000 and mode == MODE_WGRAD:
            bmf, bnk = (v % 100000) // 1000, 64 * (v % 1000)
            tl = []
            tier = (v // 100000) % 10
            geo = []
            for p, (r, (M, N, K)) in enumerate(items):
                ohw = int(r["OH"]) * int(r["OW"])
                ipc = conv_wgrad_ipc(r, tier)
                nchunks = -(-(K // ohw) // ipc) if ipc >= 2 else (K // ohw) * (-(-ohw // 128))
                cp = -(-int(r["C"]) // 8) * 8
                ldp = int(r["KH"]) * int(r["KW"]) * cp
                nkt = -(-ldp // bnk)
                nft = -(-M // bmf)
                # MFMAs per wave and chunk of the widest block: 4 k steps x f tiles x its column tiles, taken
                # in groups of 4 per wave
                ntw = bnk // 64
                nvj = -(-min(4 * ntw, -(-ldp // 16)) // 4)
                per = -(-nchunks // conv_wgrad_splits(nchunks, 4 * (bmf // 16) * 4 * -(-nvj // 4), nft * nkt,
                                                      4 * M * ldp))
                ns = -(-nchunks // per)
                r["kper"] = per
                if ns > 1:
                    r["_wgfin"] = ns                # fp32 slabs + wgrad_finalize (the caller allocates ext)
                    r["_ldp"] = ldp
                else:
                    r["flags"] = int(r.get("flags", 0)) | GF_WSTORE
                geo.append((nchunks, nkt, nft, per))
            # (chunks per block 8..64: unlike the GEMM WGRAD, more and shorter blocks measured slower --
            # every block restages its patches and the cross-chunk prefetch needs a long chunk range)
            for p, (r, (M, N, K)) in enumerate(items):
                nchunks, nkt, nft, per = geo[p]
                # tiles ordered (chunk range, f tile, k' tile), vectorised over all three
                c0 = np.arange(0, nchunks, per)
                fk = ((np.arange(nft)[:, None] << 16) | np.arange(nkt)[None, :]).ravel()
                t_ = np.empty((len(c0), len(fk), 4), np.int64)
                t_[..., 0] = p
                t_[..., 1] = fk[None, :]
                t_[..., 2] = c0[:, None]
                t_[..., 3] = np.minimum(nchunks, c0 + per)[:, None]
                # the f x k' tiles of one chunk range stage the same input patches: one XCD (its L2) for them
                tl.append(xcd_swizzle(t_.reshape(-1, 4), len(fk)))
            tiles = np.concatenate(tl).astype(np.int32)
        else:
            bm, bn = gemm3_block(mode, v)
            dms = [dm for _, dm in items]
            if mode == MODE_WGRAD:
                rg = 1 if v >= 8000000 else (DWGRAD_RG if v >= 5000000 else (2 if (v % 1000000) % 1000 >= 500 else 1))
                tg = [wgrad_target(M, N, K, bm, bn, rg) for (M, N, K) in dms]
                if 8000000 < v < 8000010 and TINY_WGRAD_TARGET > 0:
                    tg = [TINY_WGRAD_TARGET] * len(dms)       # k steps per small-bank WGRAD block (A/B knob)
                tiles = gemm_tiles(dms, mode, target_ksteps=tg, bm=bm, bn=bn, swizzle=True)
                tiles = shared_wgrad_order([r for r, _ in items], tiles)
                for (r, (M, N, K)), t_ in zip(items, tg):
                    ns = wgrad_splits(K, t_, min(32, t_))
                    if ns == 1:
                        r["flags"] = int(r.get("flags", 0)) | GF_WSTORE
                        if r.get("adam"):
                            r["flags"] |= GF_ADAM      # sole writer: apply the optimizer step in the epilogue
                    elif WGRAD_SLABS:
                        # m-split: fp32 slab per split, summed in split order by wgrad_finalize (which also applies
                        # Adam when the row carries an AdamCtx); the caller allocates the slabs (ext)
                        kt = -(-K // BK)
                        r["kper"] = -(-kt // ns)
                        r["_wgfin"] = -(-kt // r["kper"])
                        r["_ldp"] = N
                        r["flags"] = int(r.get("flags", 0)) | GF_WSLAB
                    else:
                        r["adam"] = 0
            elif mode == MODE_FWD and 7000 < v < 7300:
                tl = []
                for p, (r, (M, N, K)) in enumerate(items):
                    kt = -(-K // BK)
                    ns = int(r.get("_split", 1))
                    per = -(-kt // ns)
                    if ns > 1 or r.get("_ws"):
                        r["kper"] = max(per, 1)
                        r["flags"] = int(r.get("flags", 0)) | GF_SPLITWS
                    t = gemm_tiles([(M, N, K)], mode, bm=bm, bn=bn, ngroup=tiled_ngroup(items, bm, bn))
                    spl = []
                    for s_ in range(ns):
                        k0, k1 = s_ * per, min(kt, (s_ + 1) * per)
                        if k0 >= k1:
                            continue
                        ts = t.copy()
                        ts[:, 0] = p
                        ts[:, 3] = k0 | (k1 << 16)
                        spl.append(ts)
                    # the m x n tiles of one k split share its X and W panels: one XCD per split
                    if spl:
                        tl.append(xcd_swizzle(np.concatenate(spl), len(t)))
                tiles = np.concatenate(tl).astype(np.int32) if tl else np.zeros((0, 4), np.int32)
            else:
                tiled = 7000 <= v < 9000 or 17000 <= v < 19000
                tiles = gemm_tiles(dms, mode, bm=bm, bn=bn, swizzle=mode == MODE_DGRAD and v >= 7000,
                                   ngroup=tiled_ngroup(items, bm, bn) if tiled else 1)
        out.append((v, [r for r, _ in items], tiles))
    return out


def fwd_bnustat_ok(r: dict, M: int, N: int, K: int, splitk: bool = True) -> bool:
    """True when the FWD kernel gemm3_plan picks for row ``r`` accumulates a consuming BatchNorm's statistics in its
    epilogue (GF_BNUSTAT): the conv-halo kernel, the LDS-tiled kernel without k splits, or the direct kernel without
    the wave-split-K form -- mirrors gemm3_plan's selection (narrow rows have their own GF_BNSTAT)."""
    flags = int(r.get("flags", 0))
    if flags & (GF_ACCUM | GF_OUT_F32 | GF_SPLITWS) or r.get("_force_tiled") or r.get("_split"):
        return False
    if narrow_k(r, MODE_FWD, M, N, K) is not None and not r.get("_nonarrow"):
        return False
    one = int(r.get("KH", 1)) * int(r.get("KW", 1)) == 1 and int(r.get("SH", 1)) * int(r.get("SW", 1)) == 1
    if "tiled" not in _OFF and K > 32 and one:
        return not (splitk and tiled_fwd_splits(M, N, K, tiled_bn(N), flags) > 1)
    if conv_lds_config(r, N) is not None:
        return True
    v = gemm3_variant(MODE_FWD, M, N, K, r)
    return v >= 5000 or (v % 1000) < 100          # single-step, or the direct kernel without wave-split K


def dwgrad_ok(geo: dict, M: int, N: int, v: int) -> bool:
    """A Dense / 1x1 stride-1 WGRAD the LDS-DMA ring kernel takes (gemm3.hip g3_dwgrad_kernel): a regular
    (non-gather) tile of >= 64 columns, and 16-B aligned rows of dY (F % 8 == 0) and X (C % 8 == 0)."""
    if not DWGRAD or v >= 1000000 or v // 1000 not in (16, 32, 64) or v % 1000 not in (64, 128, 256):
        return False
    if int(geo.get("KH", 1)) * int(geo.get("KW", 1)) != 1 or int(geo.get("SH", 1)) * int(geo.get("SW", 1)) != 1:
        return False
    # X rows need only 8-B alignment (C % 4 == 0): a 16-B piece past a row's end carries the next row's first
    # elements into columns >= N, whose accumulators are never stored
    return int(M) % 8 == 0 and int(N) % DWGRAD_CALIGN == 0 and int(geo.get("C", N)) == int(N)


def wgrad_finalize_row(r: dict, ws_ptr: int, adam: int = 0) -> dict:
    """WgFinDesc of a split WGRAD row (``_wgfin`` set by gemm3_plan: a conv WGRAD's padded (tap, Cp) slabs, or a
    Dense / 1x1 WGRAD's [M][N] slabs, GF_WSLAB) whose slabs live at ``ws_ptr`` (``wgrad_slab_elems(r)`` fp32); sets
    the row's ``ext``.  ``adam``: device AdamCtx -- the finalize applies the optimizer step (sole writer)."""
    r["ext"] = ws_ptr
    if int(r.get("flags", 0)) & GF_WSLAB:
        C = Cp = int(r["N"])                     # one "tap" of N columns, unpadded
    else:
        C = int(r["C"])
        Cp = -(-C // 8) * 8
    return dict(ws=ws_ptr, out=int(r["out"]), adam=adam, M=int(r["M"]), N=int(r["N"]), C=C, Cp=Cp,
                S=int(r["_wgfin"]), ldo=int(r.get("ldo", 0) or 0), flags=0)


def wgrad_slab_elems(r: dict) -> int:
    return int(r["_wgfin"]) * int(r["M"]) * int(r["_ldp"])


def dgrad_reads_natural(KH: int, KW: int, SH: int, SW: int, F: int) -> bool:
    """True when a layer's DGRAD runs on the LDS-tiled kernel reading the natural [F][C] weights (BT,
    variants 8064 / 8128), i.e. it needs no transposed weight copy (mirrors gemm3_plan)."""
    return ("tiled" not in _OFF and "bt" not in _OFF and KH * KW == 1 and SH * SW == 1 and F > BK)


# target k steps per split (0: off; round 2: 48, round 3: 32; 24 from the round-4 sweep, profiles/r4/ab_split_targets.txt)
SPLIT_KSTEPS = int(_os.environ.get("SERANN_SPLIT_KSTEPS", "24"))


def tiled_fwd_splits(M: int, N: int, K: int, bn: int, flags: int) -> int:
    """k splits of an LDS-tiled FWD problem.  Merged-Dense layers have few output tiles (M = batch
    rows, N <= 256) and a long reduction (K up to ~20k): unsplit, a handful of blocks each walk hundreds
    of latency-bound k steps.  Split so every block walks about SPLIT_KSTEPS k steps (at most 16
    splits); bf16 problems only (GF_OUT_F32 / GF_ACCUM outputs are never split)."""
    if SPLIT_KSTEPS <= 0 or flags & (GF_OUT_F32 | GF_ACCUM):
        return 1
    kt = -(-K // BK)
    tiles = -(-M // 128) * -(-N // bn)
    if tiles >= 256 or kt < 2 * SPLIT_KSTEPS:
        return 1
    return int(min(16, kt // SPLIT_KSTEPS))


def wgrad_splits(K: int, target_ksteps: int = 128, min_ksteps: int = 32) -> int:
    """Number of m-splits (blocks along the reduction) of a WGRAD problem with K reduction rows."""
    kt = -(-K // BK)
    if kt <= target_ksteps:
        return 1
    return max(1, min(-(-kt // min_ksteps), -(-kt // target_ksteps), _WGRAD_MAXSPLIT))


def wgrad_row_groups(M: int, N: int, K: int, bm: int, bn: int) -> int:
    """Row groups per block of a Dense / 1x1 WGRAD problem: 2 when it is m-split at one group per block
    (the groups halve its fixed-point flushes), 1 for single-split problems (plain store / fused Adam).
    A function of the problem alone (deterministic sharding)."""
    if WGRAD_ROW_GROUPS < 2:
        return 1
    tg = wgrad_target(M, N, K, bm, bn)
    return 2 if wgrad_splits(K, tg, min(32, tg)) > 1 else 1


def wgrad_target(M: int, N: int, K: int = 0, bm: int = 64, bn: int = 64, rg: int = 1) -> int:
    """k-steps (32 rows) per WGRAD block: SERANN_WGRAD_TARGET (64), halved (down to 16) while the
    problem alone has fewer than WGRAD_MIN_BLOCKS blocks -- a small weight matrix over many rows
    (measured: two [70 x 98] Dense WGRADs over 75000 rows in 57 blocks ran at 0.2 TB/s) splits its
    reduction finer.  A function of the problem alone: the m-split boundaries decide the fp32 partial
    sums that meet in the fixed-point arena, so they must not depend on the launch (deterministic
    sharding)."""
    tg = _WGRAD_TARGET * rg
    tiles = -(-int(M) // bm) * -(-int(N) // bn)
    if K and -(-int(K) // BK) <= WGRAD_NOSPLIT_KSTEPS:
        # a short reduction (the batch-750 rows of a merged-Dense / head WGRAD) stays one split: its blocks walk
        # 24 k steps either way, and the split cost a partial-sum round trip and the fused Adam epilogue (round 6:
        # the ancestor's X-slice and head WGRADs; 13 % of the round-5 bench kernel time was such m-splits)
        return max(tg, -(-int(K) // BK))
    while tg > 16 and K and tiles * wgrad_splits(K, tg, min(32, tg)) < WGRAD_MIN_BLOCKS // rg:
        tg //= 2
    return tg


# target k steps per WGRAD split (rounds 2-3: 128; 64 from the round-4 sweep: generation-3 mix 17.5 -> 17.0 ms per
# step on one stream, ancestor neutral, profiles/r4/ab_split_targets.txt)
_WGRAD_TARGET = int(_os.environ.get("SERANN_WGRAD_TARGET", "64"))
# whole-F WGRAD tiles (BMF 96..192 x 64 columns) for Dense problems with F in (64, 192] and a short reduction
# (<= WGRAD_WIDE_MAXK 32-row k steps: the batch-750 Dense layers, single split -> plain store / fused Adam)
WGRAD_WIDE = _os.environ.get("SERANN_WGRAD_WIDE", "0") != "0"
WGRAD_WIDE_MAXK = int(_os.environ.get("SERANN_WGRAD_WIDE_MAXK", "64"))
# m-split WGRAD problems run two row groups of 4 waves per block (gemm3.hip, variant + 500): a block walks
# 2 x 128 k-steps, so an m-split costs one fixed-point flush per 256 k-steps at the same parallelism
WGRAD_ROW_GROUPS = int(_os.environ.get("SERANN_WGRAD_ROW_GROUPS", "2"))
# conv-halo WGRAD chunk-range splits (conv_wgrad_splits): per-block bounds on MFMAs per wave and on chunks
CONV_WGRAD_WAVE_MFMAS = int(_os.environ.get("SERANN_CONV_WGRAD_WAVE_MFMAS", "4096"))
CONV_WGRAD_MAX_CHUNKS = int(_os.environ.get("SERANN_CONV_WGRAD_MAX_CHUNKS", "8"))
CONV_WGRAD_MIN_CHUNKS = int(_os.environ.get("SERANN_CONV_WGRAD_MIN_CHUNKS", "4"))
CONV_WGRAD_MAX_BLOCKS = int(_os.environ.get("SERANN_CONV_WGRAD_MAX_BLOCKS", "2048"))
CONV_WGRAD_MAX_SLAB_MB = int(_os.environ.get("SERANN_CONV_WGRAD_MAX_SLAB_MB", "64"))
# column width cap of a conv WGRAD block (round 5: 1024, i.e. 16 column tiles per wave for 16-filter problems)
CONV_WGRAD_BNK_MAX = int(_os.environ.get("SERANN_CONV_WGRAD_BNK_MAX", "2048"))
# LDS-DMA Dense / 1x1 WGRAD kernel (round 5) and its k steps per block as a multiple of the WGRAD target.  Off by
# default: on the fixed populations it measured slower than the register-staged kernel (an act' m-split problem
# 271 -> 420 us: one 128 KB block per CU against three 8-wave blocks; the big single-split Dense WGRADs have
# C % 8 != 0 and cannot take it; profiles/r5/ab_dma_dense_wgrad.txt)
DWGRAD = _os.environ.get("SERANN_DWGRAD", "0") != "0"
DWGRAD_RG = int(_os.environ.get("SERANN_DWGRAD_RG", "2"))
DWGRAD_CALIGN = int(_os.environ.get("SERANN_DWGRAD_CALIGN", "8"))
WGRAD_MIN_BLOCKS = int(_os.environ.get("SERANN_WGRAD_MIN_BLOCKS", "32"))     # per problem (round 2: 64)
# WGRAD reductions of at most this many 32-row k steps are never m-split (wgrad_target)
WGRAD_NOSPLIT_KSTEPS = int(_os.environ.get("SERANN_WGRAD_NOSPLIT_KSTEPS", "32"))
# Dense / 1x1 WGRAD m-splits meet in fp32 slabs + an ordered finalize (GF_WSLAB, round 6) instead of Q40 atomics
WGRAD_SLABS = _os.environ.get("SERANN_WGRAD_SLABS", "1") != "0"
_WGRAD_MAXSPLIT = int(_os.environ.get("SERANN_WGRAD_MAXSPLIT", "1000000"))


# LDS-tiled FWD / DGRAD: n tiles per block (g3_tiled_kernel walks them in turn) when a launch has at least
# TILED_NGROUP_MIN tiles -- tens of thousands of 5-k-step blocks (the ancestor's merged-Dense DGRAD: 44,250) spend
# their time in block prologues and epilogues (profiles/r5/ab_nbnsum_epilogue_sums.txt)
TILED_NGROUP = int(_os.environ.get("SERANN_TILED_NGROUP", "4"))
TILED_NGROUP_MIN = int(_os.environ.get("SERANN_TILED_NGROUP_MIN", "4096"))


def tiled_ngroup(items, bm: int, bn: int) -> int:
    """n tiles per block of one LDS-tiled launch (``items``: its (row, (M, N, K)) problems; k splits included)."""
    if TILED_NGROUP <= 1:
        return 1
    total = 0
    for r, (M, N, K) in items:
        total += -(-int(M) // bm) * -(-int(N) // bn) * max(1, int(r.get("_split", 1)))
    return TILED_NGROUP if total >= TILED_NGROUP_MIN else 1


def gemm_tiles(dims, mode: int, target_ksteps=128, min_ksteps: int = 32, bm: int = BM,
               bn: int = BN, swizzle: bool = False, ngroup: int = 1) -> np.ndarray:
    """dims: list of (M, N, K) per problem -> int32 (ntiles, 4) table (prob, tm, tn, kt0|kt1<<16).
    target_ksteps: int, or one value per problem (WGRAD m-split granularity).  Vectorised over the k
    splits of a problem (a WGRAD over 432k rows has hundreds): plans are rebuilt every generation.
    ``ngroup`` > 1 (LDS-tiled kernel): a block walks up to ngroup consecutive n tiles of its row tile; the n entry
    is then first tile | (tiles << 16)."""
    rows = []
    for p, (M, N, K) in enumerate(dims):
        tm, tn = -(-M // bm), -(-N // bn)
        kt = -(-K // BK)
        if tm == 0 or tn == 0:
            continue
        ng = max(1, min(int(ngroup), tn))
        tn_full = tn
        tn = -(-tn_full // ng)                      # n groups
        nsplit = 1
        tgt = target_ksteps[p] if isinstance(target_ksteps, (list, tuple)) else target_ksteps
        if mode == MODE_WGRAD:
            nsplit = wgrad_splits(K, tgt, min(min_ksteps, tgt))
        per = -(-kt // nsplit)
        k0 = np.arange(nsplit, dtype=np.int64) * per
        k1 = np.minimum(kt, k0 + per)
        packed = (k0 | (k1 << 16))[k0 < k1]
        # k-split outermost, then n, then m: consecutive blocks share the weight (B) panel
        T = tm * tn
        idx = np.arange(T)
        blk = np.empty((len(packed), T, 4), np.int64)
        blk[:, :, 0] = p
        blk[:, :, 1] = idx % tm
        g = idx // tm
        blk[:, :, 2] = g * ng if ng == 1 else (g * ng) | (np.minimum(ng, tn_full - g * ng) << 16)
        blk[:, :, 3] = packed[:, None]
        if swizzle:
            # m fastest: the tm tiles of one n column share its B panel (WGRAD: the X columns,
            # DGRAD: the weight columns) -> keep them on one XCD
            blk = blk[:, xcd_order(T, tm)]
        rows.append(blk.reshape(-1, 4))
    if not rows:
        return np.zeros((0, 4), np.int32)
    return np.concatenate(rows).astype(np.int32)


XCDS = 8                                   # MI355X: 8 XCDs, blockIdx.x -> XCD blockIdx.x % 8 (round robin)
XCD_SWIZZLE = "xcd" not in _OFF


def xcd_swizzle(tiles: np.ndarray, group: int) -> np.ndarray:
    """Reorder one problem's tile table so that every run of ``group`` consecutive tiles (tiles that
    share an operand panel: the m tiles of one WGRAD column tile, the m x n tiles of one FWD k split)
    is dispatched to ONE XCD, in consecutive rounds of the round-robin dispatch: their panel re-reads
    hit that XCD's L2 instead of going to the Infinity Cache / HBM once per XCD.  Tiles are independent
    (disjoint outputs or atomics), so the order is a pure performance choice; the tail that does not
    fill 8 whole groups keeps its natural order."""
    return tiles[xcd_order(len(tiles), group)]


def xcd_order(n: int, group: int) -> np.ndarray:
    """Gather order of xcd_swizzle: swizzled = tiles[xcd_order(len(tiles), group)]."""
    g = int(group)
    order = np.arange(n)
    if not XCD_SWIZZLE or g <= 1 or n < XCDS * g:
        return order
    full = (n // (XCDS * g)) * XCDS * g
    i = np.arange(full)
    k, j = i // g, i % g
    pos = ((k // XCDS) * g + j) * XCDS + (k % XCDS)
    order[pos] = i
    return order


def chunk_tiles(counts, chunk: int) -> np.ndarray:
    """counts: elements/rows per problem -> int32 (ntiles, 2) table (prob, chunk index)."""
    rows = []
    for p, n in enumerate(counts):
        c = -(-int(n) // chunk)
        if c > 0:
            rows.append(np.stack([np.full(c, p), np.arange(c)], 1))
    if not rows:
        return np.zeros((0, 2), np.int32)
    return np.concatenate(rows).astype(np.int32)
