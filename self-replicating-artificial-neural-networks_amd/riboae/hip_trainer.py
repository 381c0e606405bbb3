"""RiboAE (ConcreteGAE) training on the in-house HIP kernels.

Reference: ribosomal_autoencoder/training.py:40-48 (GradientTape -> Adam) over model.py:17-104.  The
whole training step -- forward, NELBO, backward and Keras Adam -- runs on this repository's kernels, no
MIOpen / hipBLASLt / rocBLAS:

  tokens -> embed_gather (K30) -> BN(1) -> Conv2D 5x5 1->32 -> BN -> Conv2D 3x3 32->16 -> BN
         -> Conv2D 3x3 16->16 -> BN -> Dense 229,824 -> 200 (split-K, K32) -> concrete sample + KL (K36)
         -> Conv1D 2->32 k5 -> BN -> Dense 3072 -> 350 V -> BN(V) -> log-softmax / gather / sum (K37)

Convolutions and Dense layers are gemm3 FWD / DGRAD / WGRAD launches (NHWC bf16 activations, fp32
accumulation), BatchNormalization the bn_kernel phases (train statistics in wide fixed point, moving
statistics with the standard n / (n - 1) factor), the embedding gradient a WGRAD of the one-hot token
matrix against the embedding-output gradient, and Adam the fused arena kernel (K13/K38) over a flat fp32
parameter arena with a Q40 fixed-point gradient arena -- so a step is bitwise reproducible.

The torch model's parameters and BatchNorm running statistics are re-pointed into the arenas
(convolution kernels as permuted views of the output-major layout the kernels use), so the model object
keeps working for checkpoints, eval-mode encode / decode and the torch reference path.

Descriptors, tile tables and every activation / gradient buffer are built once per batch size: a step is
~40 kernel launches and no host work beyond the per-step scalars (temperature, KL weight, lr).
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops import hip_ops as H

SLACK = 64


def _zeros(n, dtype, dev):
    return torch.zeros(int(n) + SLACK, dtype=dtype, device=dev)


class _Arena:
    def __init__(self):
        self.size = 0
        self.items: Dict[str, tuple] = {}

    def add(self, name, n):
        off = self.size
        self.items[name] = (off, int(n))
        self.size += (int(n) + 15) // 16 * 16
        return off


class _Plan:
    """Buffers and launch lists of one batch size."""


# attributes _build_buffers sets (one set per batch size, shared by the fused and unfused plans)
_BUF_ATTRS = ("geo", "shapes", "flat", "gflat", "buf", "wt", "wsa", "mean", "invstd")


class HipRiboTrainer:
    def __init__(self, model, device="cuda", beta1=0.9, beta2=0.999, eps=1e-7, ksplit: int = 32):
        self.model = model
        self.dev = torch.device(device)
        self.b1, self.b2, self.eps = beta1, beta2, eps
        self.ksplit = int(ksplit)                 # k splits of the 229,824-wide Dense FWD (>= 256 blocks at B=512)
        self.fuse_bn_stats = os.environ.get("SERANN_FUSE_BN_USTATS", "1") != "0"
        # the large single-split Dense WGRADs apply Adam in their epilogue (SERANN_FUSE_ADAM=0: the arena pass)
        self.fuse_adam = os.environ.get("SERANN_FUSE_ADAM", "1") != "0"
        self.fused_adam = False
        self.adam_regions: List[tuple] = []
        self.lib = H.lib(required=True)
        H.check_layouts()
        inf, gen = model.inference_net, model.generative_net
        self.L, self.E, self.G, self.A, self.V = inf.max_len, inf.emb_dim, inf.genotype_length, inf.alphabet, gen.vocab
        self._build_params()
        self.plans: Dict[int, _Plan] = {}
        self._bufs: Dict[int, dict] = {}             # per batch size: the buffers both plans of that size use
        self.keep: List[torch.Tensor] = []          # split-WGRAD slabs referenced by the launch descriptors

    def _plan(self, B: int, fused: bool = False) -> _Plan:
        """Buffers and launches of one batch size; ``fused``: single-split WGRAD tiles apply Adam in their epilogue
        (GF_ADAM) and the arena pass skips them -- the training step's plan.  The unfused plan keeps every gradient
        in the arena (debug_grads / update=False)."""
        key = (int(B), bool(fused))
        if key not in self.plans:
            self.B = int(B)
            self.fused_adam = bool(fused) and self.fuse_adam
            self.adam_regions = []
            # the fused and unfused plans of one batch size share every buffer (only their WGRAD descriptors
            # differ): a debug_grads / update=False call after training allocates no second activation set
            if int(B) in self._bufs:
                for k, v in self._bufs[int(B)].items():
                    setattr(self, k, v)
            else:
                self._build_buffers()
                self._bufs[int(B)] = {k: getattr(self, k) for k in _BUF_ATTRS}
            self._build_launches()
            pl = _Plan()
            for k in ("buf", "wsa", "mean", "invstd", "fwd_enc", "fwd_dec", "bwd_dec", "bwd_enc", "trans", "wt"):
                setattr(pl, k, getattr(self, k))
            pl.B = int(B)
            pl.skip = H.adam_skip_mask_device(self.pa.size, self.adam_regions, self.dev) if self.adam_regions else None
            self.plans[key] = pl
        return self.plans[key]

    # ------------------------------------------------------------------------------------------------
    # parameter arena: fp32 master, Q40 int64 gradients, Adam moments, bf16 compute copy
    # ------------------------------------------------------------------------------------------------
    def _build_params(self):
        m, dev = self.model, self.dev
        inf, gen = m.inference_net, m.generative_net
        pa, sa = _Arena(), _Arena()
        # (name, module parameter, kernel layout shape, permutation kernel layout -> torch layout)
        self.specs = [("emb", inf.embedding, "weight", None, None)]
        convs = [("c1", inf.conv1, inf.bn1), ("c2", inf.conv2, inf.bn2), ("c3", inf.conv3, inf.bn3)]
        self.bns = {"bn0": inf.bn0, "bn1": inf.bn1, "bn2": inf.bn2, "bn3": inf.bn3, "gbn1": gen.bn1,
                    "gbn2": gen.bn2}
        for name, conv, _ in convs:
            F_, C_, KH, KW = conv.weight.shape
            self.specs.append((name, conv, "weight", (F_, KH, KW, C_), (0, 3, 1, 2)))
            self.specs.append((name + "_b", conv, "bias", None, None))
        self.specs += [("dense", inf.dense, "weight", None, None), ("dense_b", inf.dense, "bias", None, None)]
        F_, C_, T = gen.conv.weight.shape
        self.specs += [("g1", gen.conv, "weight", (F_, T, C_), (0, 2, 1)), ("g1_b", gen.conv, "bias", None, None),
                       ("g2", gen.dense, "weight", None, None), ("g2_b", gen.dense, "bias", None, None)]
        for bname, bn in self.bns.items():
            self.specs += [(bname + "_g", bn, "weight", None, None), (bname + "_be", bn, "bias", None, None)]
        for name, mod, attr, klayout, _ in self.specs:
            pa.add(name, getattr(mod, attr).numel())
        for bname, bn in self.bns.items():
            sa.add(bname + "_mm", bn.running_mean.numel())
            sa.add(bname + "_mv", bn.running_var.numel())
        self.pa, self.sa = pa, sa
        n = pa.size
        self.p = _zeros(n, torch.float32, dev)
        self.g = _zeros(n, torch.int64, dev)
        self.m = _zeros(n, torch.float32, dev)
        self.v = _zeros(n, torch.float32, dev)
        self.pbf = _zeros(n, torch.bfloat16, dev)
        self.stats = _zeros(sa.size, torch.float32, dev)
        self.step_i = torch.zeros(1, dtype=torch.int32, device=dev)
        self.lr_t = torch.zeros(1, dtype=torch.float32, device=dev)
        actx = np.zeros(1, dtype=H.ADAM_CTX_DTYPE)
        actx[0] = (self.p.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), self.pbf.data_ptr(), self.g.data_ptr(),
                   self.lr_t.data_ptr(), 0, 0, 0, self.b1, self.b2, self.eps, H.MOM_F32)
        self._adam_ctx = torch.as_tensor(np.frombuffer(actx.tobytes(), dtype=np.uint8).copy(), device=dev)
        with torch.no_grad():
            for name, mod, attr, klayout, perm in self.specs:
                off, cnt = pa.items[name]
                old = getattr(mod, attr)
                flat = self.p.narrow(0, off, cnt)
                if klayout is None:
                    view = flat.view(old.shape)
                    view.copy_(old.detach().to(dev))
                else:
                    kv = flat.view(klayout)
                    inv = [0] * len(perm)
                    for i, p_ in enumerate(perm):
                        inv[p_] = i
                    kv.copy_(old.detach().to(dev).permute(*inv))      # torch layout -> kernel layout
                    view = kv.permute(*perm)                           # torch-layout view of the arena
                setattr(mod, attr, torch.nn.Parameter(view, requires_grad=old.requires_grad))
            for bname, bn in self.bns.items():
                for key, buf in (("_mm", "running_mean"), ("_mv", "running_var")):
                    off, cnt = sa.items[bname + key]
                    v = self.stats.narrow(0, off, cnt)
                    v.copy_(getattr(bn, buf).detach().to(dev))
                    setattr(bn, buf, v)
            self.pbf[:n].copy_(self.p[:n].to(torch.bfloat16))

    def pptr(self, name):
        return self.p.data_ptr() + 4 * self.pa.items[name][0]

    def gptr(self, name):
        return self.g.data_ptr() + 8 * self.pa.items[name][0]

    def bptr(self, name):
        return self.pbf.data_ptr() + 2 * self.pa.items[name][0]

    def sptr(self, name):
        return self.stats.data_ptr() + 4 * self.sa.items[name][0]

    # ------------------------------------------------------------------------------------------------
    def _build_buffers(self):
        B, L, E, G, A, V, dev = self.B, self.L, self.E, self.G, self.A, self.V, self.dev
        bf = torch.bfloat16
        self.geo = {}
        h, w = L, E
        shapes = {"e0": (B, L, E, 1)}
        cin = 1
        for name in ("c1", "c2", "c3"):
            conv = getattr(self.model.inference_net, {"c1": "conv1", "c2": "conv2", "c3": "conv3"}[name])
            F_, _, KH, KW = conv.weight.shape
            oh, ow = h - KH + 1, w - KW + 1
            self.geo[name] = dict(H=h, W=w, C=cin, OH=oh, OW=ow, F=F_, KH=KH, KW=KW)
            shapes[name] = (B, oh, ow, F_)
            h, w, cin = oh, ow, F_
        self.flat = h * w * cin
        gconv = self.model.generative_net.conv
        F1, _, T = gconv.weight.shape
        self.geo["g1"] = dict(H=G, W=1, C=A, OH=G - T + 1, OW=1, F=F1, KH=T, KW=1)
        self.gflat = (G - T + 1) * F1
        buf = {}
        for k, shp in shapes.items():
            n = math.prod(shp)
            buf[k] = _zeros(n, bf, dev)                    # layer output (pre-BN)
            buf["y" + k] = _zeros(n, bf, dev)              # BN output
            buf["d" + k] = _zeros(n, bf, dev)              # gradient wrt the BN output
            buf["dz" + k] = _zeros(n, bf, dev)             # gradient wrt the layer output (BN dx)
        self.shapes = shapes
        # (the kernels read and write the dtypes their neighbours use: int32 tokens, a bf16 one-hot from a kernel,
        # bf16 z / dz / dlogits and the generative BN's bf16 output read in place by the log-likelihood kernels --
        # no dtype-shuttling copies in the step)
        buf["tok"] = torch.zeros(B * L + SLACK, dtype=torch.int32, device=dev)
        buf["onehot"] = _zeros(B * L * V, bf, dev)
        buf["logits"] = _zeros(B * G * A, torch.float32, dev)
        buf["s"] = _zeros(B * G * A, torch.float32, dev)
        buf["z"] = _zeros(B * G * A, torch.float32, dev)
        buf["kl"] = _zeros(B, torch.float32, dev)
        buf["zb"] = _zeros(B * G * A, bf, dev)
        buf["dzb"] = _zeros(B * G * A, bf, dev)
        buf["dlogitsb"] = _zeros(B * G * A, bf, dev)
        n1 = B * self.gflat
        for k in ("h1", "yh1", "dh1", "dzh1"):
            buf[k] = _zeros(n1, bf, dev)
        n2 = B * L * V
        for k in ("h2", "yh2", "dh2", "dzh2"):
            buf[k] = _zeros(n2, bf, dev)
        buf["logpx"] = _zeros(B, torch.float32, dev)
        buf["gout"] = _zeros(B, torch.float32, dev)
        buf["gkl"] = _zeros(B, torch.float32, dev)
        # conv DGRAD transposed weights Wt[C][KH][KW][F] (bf16), refreshed every step
        wt = _Arena()
        for name in ("c1", "c2", "c3", "g1"):
            wt.add(name, self.pa.items[name][1])
        buf["wt"] = _zeros(wt.size, bf, dev)
        self.wt = wt
        # split-K workspace of the 229,824 -> 200 Dense (fp32 slabs, ordered finalize)
        buf["ws_dense"] = _zeros(self.ksplit * B * G * A, torch.float32, dev)
        # BN statistics workspaces (wide fixed point)
        ws = _Arena()
        for bname in self.bns:
            c = self.bns[bname].num_features
            ws.add(bname, H.bn_ws_words(c))
            ws.add(bname + "_b", H.bn_ws_words(c))
        buf["ws"] = _zeros(ws.size, torch.int64, dev)
        self.wsa = ws
        self.mean = {k: _zeros(self.bns[k].num_features, torch.float32, dev) for k in self.bns}
        self.invstd = {k: _zeros(self.bns[k].num_features, torch.float32, dev) for k in self.bns}
        self.buf = buf

    def _ptr(self, k):
        return self.buf[k].data_ptr()

    # ------------------------------------------------------------------------------------------------
    def _gemm(self, mode, rows, dims, splitk=False):
        out = []
        for v, rws, tiles in H.gemm3_plan(mode, [dict(r) for r in rows], dims, splitk=splitk):
            # split conv WGRADs: fp32 slabs per split, summed in split order by one wgrad_finalize launch
            # after the GEMM (without them the splits would meet in fixed-point atomics: 3x slower here)
            fin = []
            for r in rws:
                if r.get("_wgfin"):
                    ws = _zeros(H.wgrad_slab_elems(r), torch.float32, self.dev)
                    self.keep.append(ws)
                    fin.append(H.wgrad_finalize_row(r, ws.data_ptr()))
            if mode == H.MODE_WGRAD:
                for r in rws:
                    if int(r.get("flags", 0)) & H.GF_ADAM:
                        self.adam_regions.append(((int(r["out"]) - self.g.data_ptr()) // 8, int(r["M"]), int(r["N"]),
                                                  int(r.get("ldo") or r["N"])))
            clean = [{k: val for k, val in r.items() if not k.startswith("_")} for r in rws]
            d = torch.as_tensor(np.frombuffer(H.gemm_desc_array(clean).tobytes(), dtype=np.uint8).copy(), device=self.dev)
            out.append(("gemm3", (mode, v), d, torch.as_tensor(np.ascontiguousarray(tiles), device=self.dev)))
            if fin:
                a = np.zeros(len(fin), dtype=H.WGFIN_DTYPE)
                for i, f in enumerate(fin):
                    for k, val in f.items():
                        a[i][k] = val
                fd = torch.as_tensor(np.frombuffer(a.tobytes(), dtype=np.uint8).copy(), device=self.dev)
                ft = torch.as_tensor(H.chunk_tiles([f["M"] * f["N"] for f in fin], H.WGFIN_ELEMS), device=self.dev)
                out.append(("wgfin", 0, fd, ft))
        return out

    def _bn_row(self, bname, x, y, dy, dx, R):
        c = self.bns[bname].num_features
        wsb = self.buf["ws"].data_ptr() + 8 * self.wsa.items[bname][0]
        wsb2 = self.buf["ws"].data_ptr() + 8 * self.wsa.items[bname + "_b"][0]
        base = dict(x=x, y=y, dy=dy, dx=dx, gamma=self.pptr(bname + "_g"), beta=self.pptr(bname + "_be"),
                    mm=self.sptr(bname + "_mm"), mv=self.sptr(bname + "_mv"), mean=self.mean[bname].data_ptr(),
                    invstd=self.invstd[bname].data_ptr(), dgamma=self.gptr(bname + "_g"),
                    dbeta=self.gptr(bname + "_be"), R=R, C=c, flags=1 | 2 | 64, eps=1e-3, momentum=0.99)
        return dict(base, ws=wsb), dict(base, ws=wsb2)

    def _bn_launch(self, phase, row):
        R, C = int(row["R"]), int(row["C"])
        a = np.zeros(1, dtype=H.BN_DTYPE)
        for k, v in row.items():
            a[0][k] = v
        d = torch.as_tensor(np.frombuffer(a.tobytes(), dtype=np.uint8).copy(), device=self.dev)
        t = torch.as_tensor(H.chunk_tiles([H.bn_chunks(R, C, stats=phase in (0, 4))], 1), device=self.dev)
        return ("bn", phase, d, t)

    def _build_launches(self):
        B, L, E, G, A, V = self.B, self.L, self.E, self.G, self.A, self.V
        P = self._ptr
        fwd, bwd = [], []
        # --- encoder -------------------------------------------------------------------------------
        bn0f, bn0b = self._bn_row("bn0", P("e0"), P("ye0"), P("de0"), P("dze0"), B * L * E)
        fwd += [self._bn_launch(0, bn0f), self._bn_launch(2, bn0f)]
        prev, prev_d = "ye0", "de0"
        enc_bwd = []
        for name, bname in (("c1", "bn1"), ("c2", "bn2"), ("c3", "bn3")):
            g_ = self.geo[name]
            M = B * g_["OH"] * g_["OW"]
            K = g_["KH"] * g_["KW"] * g_["C"]
            geo = dict(g_, SH=1, SW=1)
            vec = (H.GF_VEC_A if g_["C"] % 8 == 0 else 0) | (H.GF_VEC_B if K % 8 == 0 else 0)
            frow = dict(a=P(prev), b=self.bptr(name), out=P(name), bias=self.pptr(name + "_b"),
                        M=M, N=g_["F"], K=K, act=0, flags=vec, **geo)
            bf_, bb_ = self._bn_row(bname, P(name), P("y" + name), P("d" + name), P("dz" + name), M)
            # the conv's FWD epilogue accumulates the BN's statistics (GF_BNUSTAT): no phase-0 pass over its output
            ustat = self.fuse_bn_stats and g_["F"] <= 256 and H.fwd_bnustat_ok(frow, M, g_["F"], K, splitk=False)
            if ustat:
                frow.update(aux=self.buf["ws"].data_ptr() + 8 * self.wsa.items[bname][0],
                            flags=vec | H.GF_BNUSTAT)
                bf_["flags"] |= H.BN_USTAT
            fwd += self._gemm(H.MODE_FWD, [frow], [(M, g_["F"], K)])
            fwd += ([] if ustat else [self._bn_launch(0, bf_)]) + [self._bn_launch(2, bf_)]
            # backward of this block (appended in reverse below)
            blk = [self._bn_launch(4, bb_), self._bn_launch(5, bb_)]
            blk += self._gemm(H.MODE_WGRAD, [dict(a=P("dz" + name), b=P(prev), out=self.gptr(name),
                                                  bias=self.gptr(name + "_b"), aux=0, act=0, M=g_["F"], N=K, K=M,
                                                  flags=vec, **geo)],
                              [(g_["F"], K, M)])
            Mi = B * g_["H"] * g_["W"]
            blk += self._gemm(H.MODE_DGRAD, [dict(a=P("dz" + name), b=self.buf["wt"].data_ptr() + 2 * self.wt.items[name][0],
                                                  _bnat=self.bptr(name), aux=0, act=0, out=P(prev_d), M=Mi, N=g_["C"],
                                                  K=g_["KH"] * g_["KW"] * g_["F"],
                                                  flags=(H.GF_VEC_A if g_["F"] % 8 == 0 else 0) |
                                                  (H.GF_VEC_B if g_["C"] % 8 == 0 else 0), **geo)],
                              [(Mi, g_["C"], g_["KH"] * g_["KW"] * g_["F"])])
            enc_bwd.append(blk)
            prev, prev_d = "y" + name, "d" + name
        # Dense 229,824 -> G*A: split-K FWD (fp32 slabs) + ordered finalize to fp32 logits
        K, N = self.flat, G * A
        dense_geo = dict(H=1, W=1, OH=1, OW=1, KH=1, KW=1, SH=1, SW=1)
        kt = -(-K // H.BK)
        per = -(-kt // self.ksplit)
        row = dict(a=P(prev), b=self.bptr("dense"), out=P("logits"), bias=0, aux=P("ws_dense"), C=K, F=N, M=B, N=N,
                   K=K, act=0, kper=per, sbase=0, flags=H.GF_SPLITWS | H.GF_VEC_A | H.GF_VEC_B, **dense_geo)
        tl = []
        for s_ in range(self.ksplit):
            k0, k1 = s_ * per, min(kt, (s_ + 1) * per)
            for tm in range(-(-B // 128)):
                for tn in range(-(-N // 128)):
                    tl.append((0, tm, tn, k0 | (k1 << 16)))
        d = torch.as_tensor(np.frombuffer(H.gemm_desc_array([row]).tobytes(), dtype=np.uint8).copy(), device=self.dev)
        fwd.append(("gemm3", (H.MODE_FWD, 7128), d, torch.as_tensor(np.asarray(tl, np.int32), device=self.dev)))
        fin = np.zeros(1, dtype=H.SPLITFIN_DTYPE)
        fin[0] = (P("ws_dense"), P("logits"), self.pptr("dense_b"), B, N, self.ksplit, 0, 1)
        fwd.append(("splitfin", 0, torch.as_tensor(np.frombuffer(fin.tobytes(), dtype=np.uint8).copy(), device=self.dev),
                    torch.as_tensor(H.chunk_tiles([B * N], H.SPLITFIN_ELEMS), device=self.dev)))
        self.fwd_enc = fwd
        # --- decoder (after the concrete sample) -------------------------------------------------
        dec = []
        g1 = self.geo["g1"]
        M1, K1 = B * g1["OH"], g1["KH"] * g1["C"]
        geo1 = dict(g1, SH=1, SW=1)
        g1row = dict(a=P("zb"), b=self.bptr("g1"), out=P("h1"), bias=self.pptr("g1_b"),
                     M=M1, N=g1["F"], K=K1, act=0, flags=H.GF_VEC_B if K1 % 8 == 0 else 0, **geo1)
        gb1f, gb1b = self._bn_row("gbn1", P("h1"), P("yh1"), P("dh1"), P("dzh1"), M1)
        ustat = self.fuse_bn_stats and g1["F"] <= 256 and H.fwd_bnustat_ok(g1row, M1, g1["F"], K1, splitk=False)
        if ustat:
            g1row.update(aux=self.buf["ws"].data_ptr() + 8 * self.wsa.items["gbn1"][0],
                         flags=g1row["flags"] | H.GF_BNUSTAT)
            gb1f["flags"] |= H.BN_USTAT
        dec += self._gemm(H.MODE_FWD, [g1row], [(M1, g1["F"], K1)])
        dec += ([] if ustat else [self._bn_launch(0, gb1f)]) + [self._bn_launch(2, gb1f)]
        K2, N2 = self.gflat, L * V
        dec += self._gemm(H.MODE_FWD, [dict(a=P("yh1"), b=self.bptr("g2"), out=P("h2"), bias=self.pptr("g2_b"),
                                            C=K2, F=N2, M=B, N=N2, K=K2, act=0, flags=H.GF_VEC_A | H.GF_VEC_B,
                                            **dense_geo)], [(B, N2, K2)], splitk=False)
        gb2f, gb2b = self._bn_row("gbn2", P("h2"), P("yh2"), P("dh2"), P("dzh2"), B * L)
        dec += [self._bn_launch(0, gb2f), self._bn_launch(2, gb2f)]
        self.fwd_dec = dec
        # --- decoder backward ----------------------------------------------------------------------
        db = [self._bn_launch(4, gb2b), self._bn_launch(5, gb2b)]
        # (DGRAD first: with fused Adam the WGRAD epilogue updates the weights the DGRAD reads)
        db += self._gemm(H.MODE_DGRAD, [dict(a=P("dzh2"), b=0, _bnat=self.bptr("g2"), aux=0, act=0, out=P("dh1"),
                                             C=K2, F=N2, M=B, N=K2, K=N2, flags=H.GF_VEC_A | H.GF_VEC_B,
                                             **dense_geo)], [(B, K2, N2)])
        db += self._gemm(H.MODE_WGRAD, [dict(a=P("dzh2"), b=P("yh1"), out=self.gptr("g2"), bias=self.gptr("g2_b"),
                                             adam=self._adam_ctx.data_ptr() if self.fused_adam else 0,
                                             aux=0, act=0, C=K2, F=N2, M=N2, N=K2, K=B,
                                             flags=H.GF_VEC_A | (H.GF_VEC_B if K2 % 8 == 0 else 0),
                                             **dense_geo)], [(N2, K2, B)])
        db += [self._bn_launch(4, gb1b), self._bn_launch(5, gb1b)]
        db += self._gemm(H.MODE_WGRAD, [dict(a=P("dzh1"), b=P("zb"), out=self.gptr("g1"), bias=self.gptr("g1_b"),
                                             aux=0, act=0, M=g1["F"], N=K1, K=M1,
                                             flags=H.GF_VEC_A if g1["F"] % 8 == 0 else 0, **geo1)], [(g1["F"], K1, M1)])
        Mi = B * g1["H"]
        db += self._gemm(H.MODE_DGRAD, [dict(a=P("dzh1"), b=self.buf["wt"].data_ptr() + 2 * self.wt.items["g1"][0],
                                             _bnat=self.bptr("g1"), aux=0, act=0, out=P("dzb"), M=Mi, N=g1["C"],
                                             K=g1["KH"] * g1["F"], flags=H.GF_VEC_A, **geo1)],
                         [(Mi, g1["C"], g1["KH"] * g1["F"])])
        self.bwd_dec = db
        # --- encoder backward (after the concrete backward) ----------------------------------------
        eb = []
        # (DGRAD first: with fused Adam the WGRAD epilogue updates the weights the DGRAD reads)
        eb += self._gemm(H.MODE_DGRAD, [dict(a=P("dlogitsb"), b=0, _bnat=self.bptr("dense"), aux=0, act=0,
                                             out=P("dc3"), C=K, F=N, M=B, N=K, K=N,
                                             flags=(H.GF_VEC_A if N % 8 == 0 else 0) | H.GF_VEC_B, **dense_geo)],
                         [(B, K, N)])
        actx = self._adam_ctx.data_ptr() if self.fused_adam else 0
        eb += self._gemm(H.MODE_WGRAD, [dict(a=P("dlogitsb"), b=P("yc3"), out=self.gptr("dense"), adam=actx,
                                             bias=self.gptr("dense_b"), aux=0, act=0, C=K, F=N, M=N, N=K, K=B,
                                             flags=(H.GF_VEC_A if N % 8 == 0 else 0) | (H.GF_VEC_B if K % 8 == 0 else 0),
                                             **dense_geo)], [(N, K, B)])
        for blk in reversed(enc_bwd):
            eb += blk
        eb += [self._bn_launch(4, bn0b), self._bn_launch(5, bn0b)]
        # embedding gradient: dTable[V][E] = onehot(tokens)^T . dE  (a WGRAD of the one-hot matrix)
        eb += self._gemm(H.MODE_WGRAD, [dict(a=P("onehot"), b=P("dze0"), out=self.gptr("emb"), bias=0, aux=0, act=0,
                                             C=E, F=V, M=V, N=E, K=B * L,
                                             flags=H.GF_VEC_A if V % 8 == 0 else 0, **dense_geo)], [(V, E, B * L)])
        self.bwd_enc = eb
        # transposes of the conv weights for their DGRAD (from the bf16 copy)
        tr = []
        for name in ("c1", "c2", "c3", "g1"):
            off, cnt = self.pa.items[name]
            shp = self.p.narrow(0, off, cnt)
            if name == "g1":
                F_, T_, C_ = self.geo["g1"]["F"], self.geo["g1"]["KH"], self.geo["g1"]["C"]
                P_ = T_
            else:
                F_, C_, P_ = self.geo[name]["F"], self.geo[name]["C"], self.geo[name]["KH"] * self.geo[name]["KW"]
            tr.append((self.bptr(name), self.buf["wt"].data_ptr() + 2 * self.wt.items[name][0], F_, P_, C_))
        a = np.array(tr, dtype=H.TRANS_DTYPE)
        self.trans = (torch.as_tensor(np.frombuffer(a.tobytes(), dtype=np.uint8).copy(), device=self.dev),
                      torch.as_tensor(H.chunk_tiles([-(-(r[2] * r[3] * r[4]) // H.TRANS_ELEMS) for r in tr], 1),
                                      device=self.dev))
        torch.cuda.synchronize(self.dev)

    # ------------------------------------------------------------------------------------------------
    def _run(self, launches):
        L_, s = self.lib, H.stream_handle()
        for kind, arg, d, t in launches:
            if kind == "gemm3":
                L_.gemm3(arg[0], arg[1], d.data_ptr(), t.data_ptr(), len(t), s)
            elif kind == "bn":
                L_.bn(arg, d.data_ptr(), t.data_ptr(), len(t), s)
            elif kind == "splitfin":
                L_.splitk_finalize(d.data_ptr(), t.data_ptr(), len(t), s)
            elif kind == "wgfin":
                L_.wgrad_finalize(d.data_ptr(), t.data_ptr(), len(t), s)

    def step(self, tokens: torch.Tensor, temperature: float, kld_weight: float, lr: float,
             prior_temperature: Optional[float] = None, noise: Optional[torch.Tensor] = None,
             seed: Optional[int] = None, update: bool = True) -> Dict[str, torch.Tensor]:
        """One NELBO training step on a [B][L] token batch; returns device scalars (loss, nll, kld).
        ``update=False`` leaves the Q40 gradient arena filled and skips Adam (numerics tests)."""
        B = int(tokens.shape[0])
        L, E, G, A, V = self.L, self.E, self.G, self.A, self.V
        if tuple(tokens.shape) != (B, L):
            raise ValueError(f"expected a (B, {L}) token batch, got {tuple(tokens.shape)}")
        pl = self._plan(B, fused=update)
        tp = float(prior_temperature if prior_temperature is not None else self.model.prior_temperature)
        lib, s = self.lib, H.stream_handle()
        if update and pl.skip is not None:
            # step counter and lr_t first: the fused-Adam WGRAD epilogues read lr_t during the backward
            lib.adam_scalars(self.step_i.data_ptr(), self.lr_t.data_ptr(), float(lr), self.b1, self.b2, s)
        buf = pl.buf
        buf["tok"][:B * L].copy_(tokens.reshape(-1))      # (device-resident int32 batches: a device copy)
        lib.onehot(buf["tok"].data_ptr(), buf["onehot"].data_ptr(), B * L, V, s)
        lib.memset32(buf["ws"].data_ptr(), 2 * buf["ws"].numel(), s)
        lib.transpose_weights(pl.trans[0].data_ptr(), pl.trans[1].data_ptr(), len(pl.trans[1]), s)
        lib.embed_gather(buf["tok"].data_ptr(), self.bptr("emb"), buf["e0"].data_ptr(), B * L, E, V, s)
        self._run(pl.fwd_enc)
        # K36: concrete sample + KL (Philox from torch's CPU generator, as riboae_ops.concrete_sample)
        if noise is None:
            if seed is None:
                seed = int(torch.randint(0, 2 ** 31 - 1, (1,))) << 31 | int(torch.randint(0, 2 ** 31 - 1, (1,)))
            uptr, off = 0, 0
        else:
            noise = noise.to(self.dev, torch.float32).contiguous()
            uptr, seed, off = noise.data_ptr(), 0, 0
        lib.concrete_fwd(buf["logits"].data_ptr(), uptr, buf["s"].data_ptr(), buf["z"].data_ptr(), buf["kl"].data_ptr(),
                         B, G, A, float(temperature), tp, int(seed), off, s, buf["zb"].data_ptr())
        self._run(pl.fwd_dec)
        lib.cat_loglik_fwd(buf["yh2"].data_ptr(), buf["tok"].data_ptr(), buf["logpx"].data_ptr(), B, L, V, s, 1)
        logpx, kl = buf["logpx"][:B], buf["kl"][:B]
        nelbo = -(logpx - kld_weight * kl).mean()
        # backward: d nelbo / d logpx = -1/B, d / d kl = w/B
        buf["gout"][:B].fill_(-1.0 / B)
        buf["gkl"][:B].fill_(float(kld_weight) / B)
        lib.cat_loglik_bwd(buf["yh2"].data_ptr(), buf["tok"].data_ptr(), buf["gout"].data_ptr(),
                           buf["dh2"].data_ptr(), B, L, V, s, 1)
        self._run(pl.bwd_dec)
        lib.concrete_bwd(buf["s"].data_ptr(), buf["z"].data_ptr(), buf["dzb"].data_ptr(), buf["gkl"].data_ptr(),
                         buf["dlogitsb"].data_ptr(), B, G, A, float(temperature), tp, s, 1)
        self._run(pl.bwd_enc)
        if update and pl.skip is not None:
            lib.adam_update(self.p.data_ptr(), self.g.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                            self.pbf.data_ptr(), self.lr_t.data_ptr(), self.pa.size, self.b1, self.b2, self.eps,
                            pl.skip.data_ptr(), s)
        elif update:
            lib.adam(self.p.data_ptr(), self.g.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), self.pbf.data_ptr(),
                     self.step_i.data_ptr(), self.lr_t.data_ptr(), self.pa.size, float(lr), self.b1, self.b2,
                     self.eps, s)
        return {"loss": nelbo, "nll": -logpx.mean(), "kld": kl.mean()}

    # checkpoint interface of the trainer's optimizer (riboae/trainer.py saves ``opt.state_dict()``)
    def _moment_views(self, arena: torch.Tensor) -> List[torch.Tensor]:
        """Torch-layout views of ``arena`` (an Adam moment arena) in ``model.parameters()`` order -- the
        per-parameter list format of the torch engine's optimizer (ScheduledKerasAdam.state_dict)."""
        where = {}
        for name, mod, attr, klayout, perm in self.specs:
            off, cnt = self.pa.items[name]
            flat = arena.narrow(0, off, cnt)
            where[id(getattr(mod, attr))] = flat.view(getattr(mod, attr).shape) if klayout is None else \
                flat.view(klayout).permute(*perm)
        out = []
        for p in self.model.parameters():
            if id(p) not in where:
                raise RuntimeError("model parameter outside the HIP trainer's arena")
            out.append(where[id(p)])
        return out

    def state_dict(self):
        """Per-parameter moment lists in ``model.parameters()`` order (the torch engine's format), so a HIP
        checkpoint resumes on either engine; the flat arenas are not stored a second time (load_state_dict
        still reads the arena form of older checkpoints)."""
        return {"t": int(self.step_i.item()),
                "m": [v.detach().cpu().contiguous() for v in self._moment_views(self.m)],
                "v": [v.detach().cpu().contiguous() for v in self._moment_views(self.v)]}

    def load_state_dict(self, st):
        """Accepts this engine's arenas or the torch engine's per-parameter moment lists.  A state with
        neither restarts Adam from scratch (t = 0 with zero moments: keeping a large t over zero moments
        would skew the bias correction and inflate the first updates)."""
        n = self.pa.size
        t = int(st.get("t", 0))
        with torch.no_grad():
            if "m_arena" in st:
                self.m[:n].copy_(st["m_arena"].to(self.dev))
                self.v[:n].copy_(st["v_arena"].to(self.dev))
            elif "m" in st and "v" in st:
                for arena, key in ((self.m, "m"), (self.v, "v")):
                    views = self._moment_views(arena)
                    if len(views) != len(st[key]):
                        raise ValueError(f"optimizer state has {len(st[key])} moments, model has {len(views)}")
                    for dst, src in zip(views, st[key]):
                        dst.copy_(src.to(self.dev).reshape(dst.shape))
            else:
                self.m.zero_()
                self.v.zero_()
                t = 0
        self.step_i.fill_(t)

    def debug_grads(self, tokens, temperature, kld_weight, noise):
        """Gradients of one step without the Adam update (numerics tests): {param name: torch-layout
        array}, plus the step's (loss, nll, kld).  The BatchNorm moving statistics are restored."""
        st0 = self.stats.clone()
        res = self.step(tokens, temperature, kld_weight, 0.0, noise=noise, update=False)
        g = H.from_qg(self.g)
        self.g.zero_()
        with torch.no_grad():
            self.stats.copy_(st0)
        out = {}
        for name, mod, attr, klayout, perm in self.specs:
            off, cnt = self.pa.items[name]
            flat = g.narrow(0, off, cnt)
            t = flat.view(getattr(mod, attr).shape) if klayout is None else flat.view(klayout).permute(*perm)
            out[name] = t.cpu().numpy().copy()
        return out, {k: float(v) for k, v in res.items()}
