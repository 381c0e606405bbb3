"""HIP decode path of the ribosomal autoencoder (K33-K35): genotype bits -> token ids.

Eval-mode BatchNormalization layers are folded into the preceding Conv1D / Dense weights, so decode
is two grouped MFMA GEMM launches (Conv1D 2->32 k5 as an implicit-GEMM conv; Dense 3072 -> 350*V
with fp32 output) and one fused group-argmax launch.  log_softmax is monotone, so it is never
materialised (inference never materialises log-probs).
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
            self.w1 = w1.to(self.device, torch.bfloat16).contiguous()
            self.b1 = b1.to(self.device, torch.float32).contiguous()
            self.w2 = w2.to(self.device, torch.bfloat16).contiguous()
            self.b2 = b2.to(self.device, torch.float32).contiguous()
        self.C1 = w.shape[0]

    def stale(self, model) -> bool:
        return id(model) != self.model_id or getattr(model, "_param_version", 0) != self.version

    def _desc(self, row):
        a = np.zeros(1, dtype=H.GEMM_DTYPE)
        for k, v in row.items():
            a[0][k] = v
        return torch.as_tensor(np.frombuffer(a.tobytes(), dtype=np.uint8).copy(), device=self.device)

    @torch.no_grad()
    def __call__(self, bits: torch.Tensor) -> torch.Tensor:
        B = bits.shape[0]
        G, A, V, L, C1 = self.G, self.A, self.V, self.L, self.C1
        OL = G - 4
        lib, s = H.lib(), H.stream_handle()
        x = torch.nn.functional.one_hot(bits.to(self.device).long(), A).to(torch.bfloat16).contiguous()
        h = torch.empty(B, OL, C1, dtype=torch.bfloat16, device=self.device)
        logits = torch.empty(B, L * V, dtype=torch.float32, device=self.device)
        out = torch.empty(B, L, dtype=torch.int32, device=self.device)
        K1 = 5 * A
        d1 = self._desc(dict(a=x.data_ptr(), b=self.w1.data_ptr(), out=h.data_ptr(), bias=self.b1.data_ptr(),
                             H=G, W=1, C=A, OH=OL, OW=1, F=C1, KH=5, KW=1, SH=1, SW=1, M=B * OL, N=C1, K=K1,
                             act=0, flags=(H.GF_VEC_B if K1 % 8 == 0 else 0)))
        t1 = torch.as_tensor(H.gemm_tiles([(B * OL, C1, K1)], H.MODE_FWD), device=self.device)
        lib.grouped_gemm(H.MODE_FWD, d1.data_ptr(), t1.data_ptr(), len(t1), s)
        K2 = OL * C1
        d2 = self._desc(dict(a=h.data_ptr(), b=self.w2.data_ptr(), out=logits.data_ptr(), bias=self.b2.data_ptr(),
                             H=1, W=1, C=K2, OH=1, OW=1, F=L * V, KH=1, KW=1, SH=1, SW=1, M=B, N=L * V, K=K2,
                             act=0, flags=H.GF_OUT_F32 | (H.GF_VEC_A if K2 % 8 == 0 else 0) |
                             (H.GF_VEC_B if K2 % 8 == 0 else 0)))
        t2 = torch.as_tensor(H.gemm_tiles([(B, L * V, K2)], H.MODE_FWD), device=self.device)
        lib.grouped_gemm(H.MODE_FWD, d2.data_ptr(), t2.data_ptr(), len(t2), s)
        lib.group_argmax(logits.data_ptr(), out.data_ptr(), B * L, V, s)
        return out.long()
