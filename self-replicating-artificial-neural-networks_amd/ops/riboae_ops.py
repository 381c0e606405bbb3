"""HIP inference paths of the ribosomal autoencoder (reference ribosomal_autoencoder/model.py:17-52,
evolutionary_experiment/logic/ribosomal_autoencoder.py:116-124).

* Decode (K33-K35): genotype bits -> token ids.  Eval-mode BatchNormalization layers are folded into
  the preceding Conv1D / Dense weights, so decode is two gemm3 MFMA launches (Conv1D 2->32 k5 on the
  LDS-halo implicit-GEMM conv kernel; Dense 3072 -> 350*V on the LDS-tiled kernel with fp32 output) and
  one fused group-argmax launch.  log_softmax is monotone, so it is never materialised.
  Positions whose top-2 margin lies within the bf16 error bound (~4 % of them on random genotypes) are
  re-decided in fp32 (``HipRiboDecoder._rescore``), so decode agrees with the fp32 model: a flipped
  token would be a spurious phenotype mutation in the evolution loop.
* Training (K37): ``categorical_loglik`` -- log-softmax over the vocabulary, gather at the target
  tokens and the sum over the sequence in one HIP kernel (and its backward), instead of materialising
  the [B][L][V] log-probabilities (model.py:45-46, 54-59).
* Encode (K30-K32, K35): token ids -> genotype bits.  The one-channel BatchNormalization after the
  embedding is folded into the embedding table, the BatchNormalizations after the three Conv2Ds into
  their weights and biases.  Encode is an embedding-gather launch, three LDS-halo MFMA convolutions
  (350x50x1 -> 346x46x32 -> 344x44x16 -> 342x42x16, NHWC bf16), the split-K LDS-tiled Dense
  229,824 -> 200 (K >> M, N: per-split fp32 partial slabs + an ordered finalize, no atomics, so encode is
  deterministic) and a group-argmax over the alphabet.
"""
from __future__ import annotations

import numpy as np
import torch

from . import hip_ops as H


def available() -> bool:
    return H.available()


class HipRiboDecoder:
    def __init__(self, model, device):
        self.device = torch.device(device)
        self.version = getattr(model, "_param_version", 0)
        self.model_id = id(model)
        gn = model.generative_net
        G, A, V, L = model.genotype_length, model.alphabet, model.vocab, model.max_len
        self.G, self.A, self.V, self.L = G, A, V, L
        with torch.no_grad():
            bn1, bn2 = gn.bn1, gn.bn2
            s1 = bn1.weight / torch.sqrt(bn1.running_var + bn1.eps)
            t1 = bn1.bias - bn1.running_mean * s1
            w = gn.conv.weight                          # (32, A, 5)
            w1 = (w * s1[:, None, None]).permute(0, 2, 1).contiguous()      # Wm [F][KH=5][KW=1][C=A]
            b1 = gn.conv.bias * s1 + t1
            s2 = bn2.weight / torch.sqrt(bn2.running_var + bn2.eps)
            t2 = bn2.bias - bn2.running_mean * s2
            wd = gn.dense.weight                        # (L*V, 3072) == Wm [N][K]
            s2f = s2.repeat(L)
            w2 = wd * s2f[:, None]
            b2 = gn.dense.bias * s2f + t2.repeat(L)
            # kernel operands carry the fragment-load slack (hip_ops.operand)
            self.w1 = H.padded(w1.to(self.device, torch.bfloat16).contiguous())
            self.b1 = H.padded(b1.to(self.device, torch.float32).contiguous())
            self.w2 = H.padded(w2.to(self.device, torch.bfloat16).contiguous())
            self.b2 = H.padded(b2.to(self.device, torch.float32).contiguous())
            # fp32 copies for the near-tie rescoring (``_rescore``)
            self.w1f = (w * s1[:, None, None]).to(self.device, torch.float32).contiguous()   # (32, A, 5)
            self.b1f = b1.to(self.device, torch.float32).contiguous()
            self.w2f = w2.to(self.device, torch.float32).contiguous()                      # (L*V, 3072)
            self.w2n = self.w2f.norm(dim=1).view(L, V).amax(1)                             # (L,)
        self.C1 = w.shape[0]
        self._plans = {}

    def stale(self, model) -> bool:
        return id(model) != self.model_id or getattr(model, "_param_version", 0) != self.version

    def _plan(self, B: int):
        """Buffers and gemm3 launches for a batch of B genotypes (cached per B)."""
        if B in self._plans:
            return self._plans[B]
        G, A, V, L, C1 = self.G, self.A, self.V, self.L, self.C1
        OL, dev = G - 4, self.device
        x = H.operand(B * G * A, torch.bfloat16, dev)
        h = H.operand(B * OL * C1, torch.bfloat16, dev)
        logits = H.operand((B, L * V), torch.float32, dev)
        out = H.operand((B, L), torch.int32, dev)
        K1, K2 = 5 * A, OL * C1
        launches = []
        for row, dims in ((dict(a=x.data_ptr(), b=self.w1.data_ptr(), out=h.data_ptr(), bias=self.b1.data_ptr(),
                                H=G, W=1, C=A, OH=OL, OW=1, F=C1, KH=5, KW=1, SH=1, SW=1, M=B * OL, N=C1, K=K1,
                                act=0, flags=(H.GF_VEC_B if K1 % 8 == 0 else 0)), (B * OL, C1, K1)),
                          (dict(a=h.data_ptr(), b=self.w2.data_ptr(), out=logits.data_ptr(), bias=self.b2.data_ptr(),
                                H=1, W=1, C=K2, OH=1, OW=1, F=L * V, KH=1, KW=1, SH=1, SW=1, M=B, N=L * V, K=K2,
                                act=0, flags=H.GF_OUT_F32 | (H.GF_VEC_A | H.GF_VEC_B if K2 % 8 == 0 else 0)),
                           (B, L * V, K2))):
            for v, rws, tiles in H.gemm3_plan(H.MODE_FWD, [row], [dims]):
                d = torch.as_tensor(np.frombuffer(H.gemm_desc_array(rws).tobytes(), dtype=np.uint8).copy(), device=dev)
                launches.append((v, d, torch.as_tensor(np.ascontiguousarray(tiles), device=dev)))
        pl = dict(x=x, h=h, logits=logits, out=out, launches=launches)
        self._plans[B] = pl
        return pl

    @torch.no_grad()
    def __call__(self, bits: torch.Tensor) -> torch.Tensor:
        B = bits.shape[0]
        pl = self._plan(B)
        lib, s = H.lib(), H.stream_handle()
        n = B * self.G * self.A
        pl["x"][:n].view(B, self.G, self.A).copy_(
            torch.nn.functional.one_hot(bits.to(self.device).long(), self.A).to(torch.bfloat16))
        for v, d, t in pl["launches"]:
            lib.gemm3(H.MODE_FWD, v, d.data_ptr(), t.data_ptr(), len(t), s)
        lib.group_argmax(pl["logits"].data_ptr(), pl["out"].data_ptr(), B * self.L, self.V, s)
        out = pl["out"].long().clone()
        self._rescore(bits, pl, out)
        return out

    # bf16 operands round each product h_k * w_k by a relative ~2^-9 (input and weight); over the K = 3072
    # products of a logit that is a random walk of std ~ 2^-9 * sqrt(2/3) * ||h|| ||w|| / sqrt(K).  A position
    # whose top-2 margin is within TIE_SIGMAS of it (both logits moving) is re-decided in fp32.
    TIE_SIGMAS = 8.0

    def _rescore(self, bits: torch.Tensor, pl: dict, out: torch.Tensor) -> None:
        """Re-decide near-tie positions in fp32 so decode matches the fp32 model (the bf16 MFMA path flips
        ~0.3 % of tokens on random genotypes, each a spurious phenotype mutation in the evolution loop).
        Flagged positions (usually well under 1 %) get the fp32 conv of their sequence and fp32 dot
        products for the candidate tokens within the error bound of the top logit."""
        B, L, V, C1 = out.shape[0], self.L, self.V, self.C1
        OL = self.G - 4
        K = OL * C1
        logits = pl["logits"].view(B, L, V)
        top = logits.topk(2, dim=-1).values                                   # (B, L, 2)
        h = pl["h"][:B * K].view(B, K).float()
        sig = (2.0 ** -9) * (2.0 / 3.0) ** 0.5 * h.norm(dim=1)[:, None] * self.w2n[None, :] / K ** 0.5
        tau = self.TIE_SIGMAS * 2 ** 0.5 * sig                                # (B, L)
        flag = (top[..., 0] - top[..., 1]) < tau
        if not bool(flag.any()):
            return
        fb, fl = flag.nonzero(as_tuple=True)
        ub, inv = torch.unique(fb, return_inverse=True)
        z = torch.nn.functional.one_hot(bits.to(self.device).long()[ub], self.A).float()     # (nb, G, A)
        h32 = torch.nn.functional.conv1d(z.permute(0, 2, 1), self.w1f, self.b1f)             # (nb, C1, OL)
        h32 = h32.permute(0, 2, 1).reshape(len(ub), K)
        cand = logits[fb, fl] >= (top[fb, fl, 0] - 2 * tau[fb, fl])[:, None]                 # (n, V)
        ci, cv = cand.nonzero(as_tuple=True)
        rows = fl[ci] * V + cv
        vals = torch.empty(len(ci), device=self.device)
        for c0 in range(0, len(ci), 8192):
            r = rows[c0:c0 + 8192]
            vals[c0:c0 + 8192] = (h32[inv[ci[c0:c0 + 8192]]] * self.w2f[r]).sum(1) + self.b2[r]
        best = torch.full((len(fb), V), float("-inf"), device=self.device)
        best[ci, cv] = vals
        out[fb, fl] = best.argmax(1)


def _fold_bn(bn):
    s_ = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    return s_, bn.bias - bn.running_mean * s_


class HipRiboEncoder:
    """Eval-mode ``inference_net`` + argmax on the HIP kernels (see the module docstring)."""

    SPLIT_KSTEPS = 48           # 32-wide k steps per split-K block of the flatten Dense

    def __init__(self, model, device, chunk: int = 128):
        self.device = torch.device(device)
        self.version = getattr(model, "_param_version", 0)
        self.model_id = id(model)
        self.chunk = int(chunk)
        net = model.inference_net
        self.L, self.E = net.max_len, net.emb_dim
        self.G, self.A = net.genotype_length, net.alphabet
        with torch.no_grad():
            s0, t0 = _fold_bn(net.bn0)
            table = net.embedding.weight * s0[0] + t0[0]                    # (V, E)
            self.V = table.shape[0]
            self.table = H.padded(table.to(self.device, torch.bfloat16).contiguous())
            self.convs = []
            for conv, bn in ((net.conv1, net.bn1), (net.conv2, net.bn2), (net.conv3, net.bn3)):
                sc, sh = _fold_bn(bn)
                w = (conv.weight * sc[:, None, None, None]).permute(0, 2, 3, 1).contiguous()  # [F][KH][KW][C]
                b = conv.bias * sc + sh
                self.convs.append((H.padded(w.to(self.device, torch.bfloat16).contiguous()),
                                   H.padded(b.to(self.device, torch.float32).contiguous()), conv.kernel_size))
            self.wd = H.padded(net.dense.weight.to(self.device, torch.bfloat16).contiguous())          # [N][K]
            self.bd = H.padded(net.dense.bias.to(self.device, torch.float32).contiguous())
        self._plans = {}

    def stale(self, model) -> bool:
        return id(model) != self.model_id or getattr(model, "_param_version", 0) != self.version

    def _plan(self, B: int):
        """Buffers, descriptors and tile tables for a chunk of B sequences (cached per B)."""
        if B in self._plans:
            return self._plans[B]
        dev = self.device
        Hh, Ww, C = self.L, self.E, 1
        x = H.operand((B, Hh, Ww, C), torch.bfloat16, dev)
        bufs, launches = [x], []
        cur = x
        for w, b, (kh, kw) in self.convs:
            F = w.shape[0]
            OH, OW = Hh - kh + 1, Ww - kw + 1
            y = H.operand((B, OH, OW, F), torch.bfloat16, dev)
            K = kh * kw * C
            row = dict(a=cur.data_ptr(), b=w.data_ptr(), out=y.data_ptr(), bias=b.data_ptr(), H=Hh, W=Ww, C=C,
                       OH=OH, OW=OW, F=F, KH=kh, KW=kw, SH=1, SW=1, M=B * OH * OW, N=F, K=K, act=0,
                       flags=(H.GF_VEC_B if C % 8 == 0 else 0) | (H.GF_VEC_A if C % 8 == 0 else 0))
            for v, rws, tiles in H.gemm3_plan(H.MODE_FWD, [row], [(B * OH * OW, F, K)]):
                d = torch.as_tensor(np.frombuffer(H.gemm_desc_array(rws).tobytes(), dtype=np.uint8).copy(),
                                    device=dev)
                t = torch.as_tensor(np.ascontiguousarray(tiles), device=dev)
                launches.append((v, d, t))
            bufs.append(y)
            cur, Hh, Ww, C = y, OH, OW, F
        K = Hh * Ww * C
        N = self.G * self.A
        logits = H.operand((B, N), torch.float32, dev)
        kt = -(-K // H.BK)
        per = self.SPLIT_KSTEPS
        ns = -(-kt // per)
        # split-K: split s writes its fp32 partial tile to ws[s] (GF_SPLITWS); splitk_finalize sums the
        # splits in order and adds the bias (deterministic, no atomics)
        ws = H.operand(ns * B * N, torch.float32, dev)
        row = dict(a=cur.data_ptr(), b=self.wd.data_ptr(), out=logits.data_ptr(), bias=0, aux=ws.data_ptr(),
                   H=1, W=1, C=K, OH=1, OW=1, F=N, KH=1, KW=1, SH=1, SW=1, M=B, N=N, K=K, act=0, kper=per, sbase=0,
                   flags=H.GF_SPLITWS | (H.GF_VEC_A | H.GF_VEC_B if K % 8 == 0 else 0))
        d = torch.as_tensor(np.frombuffer(H.gemm_desc_array([row]).tobytes(), dtype=np.uint8).copy(), device=dev)
        tl = []
        for k0 in range(0, kt, per):
            packed = k0 | (min(kt, k0 + per) << 16)
            for tm in range(-(-B // 128)):
                for tn in range(-(-N // 128)):
                    tl.append((0, tm, tn, packed))
        t = torch.as_tensor(np.asarray(tl, dtype=np.int32), device=dev)
        fin = np.zeros(1, dtype=H.SPLITFIN_DTYPE)
        fin[0] = (ws.data_ptr(), logits.data_ptr(), self.bd.data_ptr(), B, N, ns, 0, 1)
        fd = torch.as_tensor(np.frombuffer(fin.tobytes(), dtype=np.uint8).copy(), device=dev)
        ft = torch.as_tensor(H.chunk_tiles([B * N], H.SPLITFIN_ELEMS), device=dev)
        bufs.append(ws)
        dense = (7128, d, t, fd, ft)
        bits = H.operand(B * self.G, torch.int32, dev)
        plan = dict(x=x, bufs=bufs, convs=launches, dense=dense, logits=logits, bits=bits)
        self._plans[B] = plan
        return plan

    @torch.no_grad()
    def logits(self, tokens: torch.Tensor) -> torch.Tensor:
        """(n, L) token ids -> (n, G, A) fp32 logits of the eval-mode inference net."""
        return self._run(tokens, want_logits=True)

    @torch.no_grad()
    def __call__(self, tokens: torch.Tensor) -> torch.Tensor:
        return self._run(tokens, want_logits=False)

    def _run(self, tokens: torch.Tensor, want_logits: bool):
        tok = tokens.to(self.device).to(torch.int32)
        n = tok.shape[0]
        if tok.shape[1] != self.L:
            raise ValueError(f"token sequences must have length {self.L}, got {tok.shape[1]}")
        lib, s = H.lib(), H.stream_handle()
        outs = []
        for c0 in range(0, n, self.chunk):
            part = tok[c0:c0 + self.chunk].contiguous()
            B = part.shape[0]
            pl = self._plan(B)
            lib.embed_gather(part.data_ptr(), self.table.data_ptr(), pl["x"].data_ptr(), B * self.L, self.E,
                             self.V, s)
            for v, d, t in pl["convs"]:
                lib.gemm3(H.MODE_FWD, v, d.data_ptr(), t.data_ptr(), len(t), s)
            v, d, t, fd, ft = pl["dense"]
            lib.gemm3(H.MODE_FWD, v, d.data_ptr(), t.data_ptr(), len(t), s)
            lib.splitk_finalize(fd.data_ptr(), ft.data_ptr(), len(ft), s)
            if want_logits:
                outs.append(pl["logits"].view(B, self.G, self.A).clone())
            else:
                lib.group_argmax(pl["logits"].data_ptr(), pl["bits"].data_ptr(), B * self.G, self.A, s)
                outs.append(pl["bits"].view(B, self.G).long().clone())
        return torch.cat(outs, 0)


class _Concrete(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, t, tp, u):
        logits = logits.float().contiguous()
        B, G, A = logits.shape
        s = torch.empty_like(logits)
        z = torch.empty_like(logits)
        kl = torch.zeros(B, dtype=torch.float32, device=logits.device)
        if u is None:
            # Philox key/offset drawn from torch's CPU generator: torch.manual_seed reproduces the sample
            seed, off = (int(v) for v in torch.randint(0, 2 ** 31 - 1, (2,)))
            seed = (seed << 31) | int(torch.randint(0, 2 ** 31 - 1, (1,)))
            uptr = 0
        else:
            u = u.float().contiguous()
            uptr, seed, off = u.data_ptr(), 0, 0
        H.lib().concrete_fwd(logits.data_ptr(), uptr, s.data_ptr(), z.data_ptr(), kl.data_ptr(), B, G, A, float(t),
                             float(tp), seed, off, H.stream_handle())
        ctx.save_for_backward(s, z)
        ctx.t, ctx.tp = float(t), float(tp)
        return z, kl

    @staticmethod
    def backward(ctx, gz, gkl):
        s, z = ctx.saved_tensors
        B, G, A = s.shape
        d = torch.empty_like(s)
        gz = gz.float().contiguous() if gz is not None else None
        gkl = gkl.float().contiguous() if gkl is not None else None
        H.lib().concrete_bwd(s.data_ptr(), z.data_ptr(), gz.data_ptr() if gz is not None else 0,
                             gkl.data_ptr() if gkl is not None else 0, d.data_ptr(), B, G, A, ctx.t, ctx.tp,
                             H.stream_handle())
        return d, None, None, None


def concrete_sample(logits: torch.Tensor, temperature: float, prior_temperature: float, u=None):
    """K36: (softmax of a Gumbel(logits/t, 1/t) sample, per-row KL sum_{g,a} log q - log p) on the HIP
    kernels; ``u`` (same shape as logits) replaces the in-kernel Philox uniforms when given."""
    return _Concrete.apply(logits, temperature, prior_temperature, u)


class _CatLogLik(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, x):
        z = z.float().contiguous()
        x = x.to(torch.int64).contiguous()
        B, L, V = z.shape
        out = torch.zeros(B, dtype=torch.float32, device=z.device)
        H.lib().cat_loglik_fwd(z.data_ptr(), x.data_ptr(), out.data_ptr(), B, L, V, H.stream_handle())
        ctx.save_for_backward(z, x)
        return out

    @staticmethod
    def backward(ctx, g):
        z, x = ctx.saved_tensors
        B, L, V = z.shape
        dz = torch.empty_like(z)
        H.lib().cat_loglik_bwd(z.data_ptr(), x.data_ptr(), g.float().contiguous().data_ptr(), dz.data_ptr(), B, L, V,
                               H.stream_handle())
        return dz, None


def categorical_loglik(z: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """sum_l log_softmax(z[b, l])[x[b, l]] -> (B,) on the HIP kernels (z: [B][L][V] pre-softmax)."""
    return _CatLogLik.apply(z, x)
