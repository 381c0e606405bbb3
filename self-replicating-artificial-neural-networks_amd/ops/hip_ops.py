"""Python side of the HIP/CDNA4 kernels: descriptor dtypes (mirroring ``csrc/hip/serann_hip.h``)
and thin launch wrappers that pass raw device pointers and the current HIP stream.

The kernels are loaded from the in-tree ``serann/_native/serann_hip*.so``.  On a machine with a GPU
the engine *requires* the extension (it fails loudly instead of silently falling back).
"""
from __future__ import annotations

import numpy as np

from ..utils.native import load

_I = np.int64
GEMM_FIELDS = ["a", "b", "out", "bias", "aux", "H", "W", "C", "OH", "OW", "F", "KH", "KW", "SH", "SW",
               "M", "N", "K", "act", "flags"]
GEMM_DTYPE = np.dtype([(f, _I) for f in GEMM_FIELDS])
ACTBWD_DTYPE = np.dtype([(f, _I) for f in ["dy", "y", "dz", "dbias", "M", "N", "act", "flags"]])
BN_DTYPE = np.dtype([(f, _I) for f in ["x", "y", "dy", "dx", "gamma", "beta", "mm", "mv", "mean", "invstd", "ws",
                                       "dgamma", "dbeta", "R", "C", "flags"]] + [("eps", np.float64),
                                                                                ("momentum", np.float64)])
POOL_DTYPE = np.dtype([(f, _I) for f in ["x", "y", "idx", "dy", "dx", "B", "H", "W", "C", "OH", "OW", "PH", "PW",
                                         "SH", "SW", "flags"]])
COPY_DTYPE = np.dtype([(f, _I) for f in ["src", "dst", "rows", "cols", "src_stride", "dst_stride", "flags"]])
LOSS_DTYPE = np.dtype([(f, _I) for f in ["logits", "dlogits", "labels", "target", "metrics", "NC", "L", "B", "flags"]]
                      + [("lb", np.float64)])

GF_VEC_A, GF_VEC_B, GF_ACCUM, GF_OUT_F32 = 1, 2, 4, 8
MODE_FWD, MODE_DGRAD, MODE_WGRAD = 0, 1, 2
ACT_CODES = {"linear": 0, "relu": 1, "sigmoid": 2}

BM, BN, BK = 64, 64, 32
RED_ELEMS = 16384      # aux.hip: elements per block of the channel-strided reductions (BN, act_bwd)
POOL_ELEMS = 1024
COPY_ROWS = 16


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
    for name, dt in [("GemmDesc", GEMM_DTYPE), ("ActBwdDesc", ACTBWD_DTYPE), ("BnDesc", BN_DTYPE),
                     ("PoolDesc", POOL_DTYPE), ("CopyDesc", COPY_DTYPE), ("LossDesc", LOSS_DTYPE),
                     ("TransDesc", TRANS_DTYPE), ("ImcolDesc", IMCOL_DTYPE)]:
        if sizes[name] != dt.itemsize:
            raise RuntimeError(f"descriptor layout mismatch for {name}: C++ {sizes[name]} vs numpy {dt.itemsize}")


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


def gemm2_variant(mode: int, M: int, N: int, K: int = 0) -> int:
    """Tile variant of the v2 kernels: the column tile (FWD/DGRAD) or f tile (WGRAD) in {16, 32, 64};
    FWD/DGRAD problems with few rows and a long k loop use the wave-split-K form (+1000)."""
    dim = M if mode == MODE_WGRAD else N
    v = 16 if dim <= 16 else (32 if dim <= 32 else 64)
    if mode != MODE_WGRAD and M <= 8192 and -(-K // BK) >= 16:
        v += 1000
    return v


def gemm2_block(mode: int, variant: int):
    if mode == MODE_WGRAD:
        return (variant, 64)
    return (32, variant % 1000) if variant >= 1000 else (128, variant)


def gemm_tiles(dims, mode: int, target_ksteps: int = 128, min_ksteps: int = 32, bm: int = BM,
               bn: int = BN) -> np.ndarray:
    """dims: list of (M, N, K) per problem -> int32 (ntiles, 4) table (prob, tm, tn, kt0|kt1<<16)."""
    rows = []
    for p, (M, N, K) in enumerate(dims):
        tm, tn = -(-M // bm), -(-N // bn)
        kt = -(-K // BK)
        if tm == 0 or tn == 0:
            continue
        nsplit = 1
        if mode == MODE_WGRAD and kt > target_ksteps:
            nsplit = max(1, min(-(-kt // min_ksteps), -(-kt // target_ksteps)))
        per = -(-kt // nsplit)
        # k-split outermost, then n, then m: consecutive blocks share the weight (B) panel
        for s in range(nsplit):
            k0, k1 = s * per, min(kt, (s + 1) * per)
            if k0 >= k1:
                continue
            packed = k0 | (k1 << 16)
            mm, nn = np.meshgrid(np.arange(tm), np.arange(tn), indexing="xy")
            blk = np.stack([np.full(tm * tn, p), mm.ravel(), nn.ravel(), np.full(tm * tn, packed)], 1)
            rows.append(blk)
    if not rows:
        return np.zeros((0, 4), np.int32)
    return np.concatenate(rows).astype(np.int32)


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
