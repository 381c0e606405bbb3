"""Ribosomal autoencoder (RiboAE): token sequence <-> binary genotype.

Reference: ribosomal_autoencoder/model.py:10-134 (GeneticAutoencoder, ConcreteGAE, DeterministicGAE,
load_ribosomal_autoencoder).  Same architecture, Keras defaults re-created in PyTorch:

inference_net  : Embedding(V, 50) -> (350, 50, 1) -> BN -> Conv2D(32, 5) -> BN -> Conv2D(16, 3) -> BN
                 -> Conv2D(16, 3) -> BN -> Flatten (229,824) -> Dense(200) -> (100, 2)
generative_net : (100, 2) -> Conv1D(32, 5) -> BN -> Flatten (3,072) -> Dense(350 * V) -> (350, V) -> BN
                 -> log_softmax

* ``ConcreteGAE`` -- binary-concrete VAE with a Gumbel prior Gumbel(log(1/A)/tp, 1/tp); the encoder
  samples Gumbel(logits/t, 1/t) and feeds softmax(sample) to the decoder; NELBO = -mean(log p(x|z) -
  w * KL), KL estimated by log q(z|x) - log p(z) summed over the 100 x 2 latent (model.py:62-104).
* ``DeterministicGAE`` -- softmax codes, loss = -mean log p(x|z) (model.py:107-120).

Inference (``encode_tokens`` / ``decode_tokens``) runs in eval mode; on a GPU the decode path uses
the HIP kernels (BN folded into the conv/dense weights, grouped MFMA GEMM, fused group-argmax), and so
does the encode path (embedding gather, LDS-halo convolutions, split-K Dense, group-argmax).
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


class KerasBN(nn.BatchNorm1d):
    """Keras BatchNormalization defaults (momentum 0.99, epsilon 1e-3) over the LAST axis of an
    arbitrary-rank channels-last tensor."""

    def __init__(self, channels: int):
        super().__init__(channels, eps=1e-3, momentum=0.01)

    def forward(self, x):
        shp = x.shape
        y = super().forward(x.reshape(-1, shp[-1]))
        return y.reshape(shp)


def _glorot_(w: torch.Tensor, fan_in: int, fan_out: int):
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        w.uniform_(-lim, lim)


class InferenceNet(nn.Module):
    def __init__(self, genotype_length, max_len, vocab, emb, alphabet):
        super().__init__()
        self.max_len, self.emb_dim = max_len, emb
        self.genotype_length, self.alphabet = genotype_length, alphabet
        self.embedding = nn.Embedding(vocab, emb)
        nn.init.uniform_(self.embedding.weight, -0.05, 0.05)
        self.bn0 = KerasBN(1)
        self.conv1 = nn.Conv2d(1, 32, 5)
        self.bn1 = KerasBN(32)
        self.conv2 = nn.Conv2d(32, 16, 3)
        self.bn2 = KerasBN(16)
        self.conv3 = nn.Conv2d(16, 16, 3)
        self.bn3 = KerasBN(16)
        h, w = max_len - 8, emb - 8
        self.flat = h * w * 16
        self.dense = nn.Linear(self.flat, genotype_length * alphabet)
        for conv in (self.conv1, self.conv2, self.conv3):
            k = conv.kernel_size[0] * conv.kernel_size[1]
            _glorot_(conv.weight, k * conv.in_channels, k * conv.out_channels)
            nn.init.zeros_(conv.bias)
        _glorot_(self.dense.weight, self.flat, genotype_length * alphabet)
        nn.init.zeros_(self.dense.bias)

    def forward(self, tokens):
        x = self.embedding(tokens.long())                          # (B, L, E)
        x = self.bn0(x.unsqueeze(-1))                              # (B, L, E, 1)  channels-last
        x = x.permute(0, 3, 1, 2)                                  # NCHW
        x = self.conv1(x)
        x = self.bn1(x.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
        x = self.conv2(x)
        x = self.bn2(x.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
        x = self.conv3(x)
        x = self.bn3(x.permute(0, 2, 3, 1))                        # (B, h, w, 16) Keras flatten order
        x = self.dense(x.reshape(x.shape[0], -1))
        return x.view(-1, self.genotype_length, self.alphabet)


class GenerativeNet(nn.Module):
    def __init__(self, genotype_length, max_len, vocab, alphabet):
        super().__init__()
        self.max_len, self.vocab = max_len, vocab
        self.conv = nn.Conv1d(alphabet, 32, 5)
        self.bn1 = KerasBN(32)
        self.flat = (genotype_length - 4) * 32
        self.dense = nn.Linear(self.flat, max_len * vocab)
        self.bn2 = KerasBN(vocab)
        _glorot_(self.conv.weight, 5 * alphabet, 5 * 32)
        nn.init.zeros_(self.conv.bias)
        _glorot_(self.dense.weight, self.flat, max_len * vocab)
        nn.init.zeros_(self.dense.bias)

    def logits(self, z):                                           # pre-softmax (B, L, V)
        x = self.conv(z.permute(0, 2, 1))                          # (B, 32, G-4)
        x = self.bn1(x.permute(0, 2, 1))                           # (B, G-4, 32)
        x = self.dense(x.reshape(x.shape[0], -1))
        return self.bn2(x.view(-1, self.max_len, self.vocab))

    def forward(self, z):                                          # z: (B, G, A)
        return F.log_softmax(self.logits(z), dim=-1)


class GeneticAutoencoder(nn.Module):
    def __init__(self, genotype_length=100, max_phenotype_length=350, vocabulary_size=40, embedding_dim=50,
                 genotype_alphabet_size=2):
        super().__init__()
        self.genotype_length = genotype_length
        self.max_len = max_phenotype_length
        self.vocab = vocabulary_size
        self.alphabet = genotype_alphabet_size
        self.hparams = dict(genotype_length=genotype_length, max_phenotype_length=max_phenotype_length,
                            vocabulary_size=vocabulary_size, embedding_dim=embedding_dim,
                            genotype_alphabet_size=genotype_alphabet_size)
        self.inference_net = InferenceNet(genotype_length, max_phenotype_length, vocabulary_size, embedding_dim,
                                          genotype_alphabet_size)
        self.generative_net = GenerativeNet(genotype_length, max_phenotype_length, vocabulary_size,
                                            genotype_alphabet_size)
        self._hip_decoder = None
        self._hip_encoder = None

    def decode(self, z_bits: torch.Tensor) -> torch.Tensor:
        logits = self.generative_net(F.one_hot(z_bits.long(), self.alphabet).float())
        return logits.argmax(-1)

    def _decode(self, x, z):
        if z.is_cuda and os.environ.get("SERANN_RIBOAE_HIP", "1") != "0":
            from ..ops.riboae_ops import available, categorical_loglik
            if available():
                # fused log-softmax + gather + sum over the sequence (HIP)
                return categorical_loglik(self.generative_net.logits(z), x)
        logp = self.generative_net(z)                               # (B, L, V) log-probs
        return torch.gather(logp, -1, x.long().unsqueeze(-1)).squeeze(-1).sum(-1)

    def encode(self, x):
        return self.inference_net(x).argmax(-1)

    # -- numpy inference API used by the codec ----------------------------------------------------
    @torch.no_grad()
    def encode_tokens(self, tokens: np.ndarray, device="cpu") -> np.ndarray:
        self.eval()
        t = torch.as_tensor(np.asarray(tokens), device=device)
        if str(device).startswith("cuda"):
            from ..ops.riboae_ops import HipRiboEncoder, available
            if available():
                if self._hip_encoder is None or self._hip_encoder.stale(self):
                    self._hip_encoder = HipRiboEncoder(self, device)
                return self._hip_encoder(t).cpu().numpy()
        return self.encode(t).cpu().numpy()

    @torch.no_grad()
    def decode_tokens(self, genotypes: np.ndarray, device="cpu") -> np.ndarray:
        self.eval()
        g = torch.as_tensor((np.asarray(genotypes) > 0.5).astype(np.int64), device=device)
        if str(device).startswith("cuda"):
            from ..ops.riboae_ops import HipRiboDecoder, available
            if available():
                if self._hip_decoder is None or self._hip_decoder.stale(self):
                    self._hip_decoder = HipRiboDecoder(self, device)
                return self._hip_decoder(g).cpu().numpy()
        return self.decode(g).cpu().numpy()


def gumbel_log_prob(x, loc, scale):
    z = (x - loc) / scale
    return -(z + torch.exp(-z)) - math.log(scale) if isinstance(scale, float) else -(z + torch.exp(-z)) - torch.log(scale)


class ConcreteGAE(GeneticAutoencoder):
    def __init__(self, genotype_length=100, max_phenotype_length=350, vocabulary_size=40, embedding_dim=50,
                 genotype_alphabet_size=2, prior_temperature=0.1):
        super().__init__(genotype_length, max_phenotype_length, vocabulary_size, embedding_dim, genotype_alphabet_size)
        self.prior_temperature = prior_temperature
        self.hparams["prior_temperature"] = prior_temperature

    def _encode(self, x, temperature=0.2, noise=None):
        logits = self.inference_net(x)
        loc = logits / temperature
        scale = 1.0 / temperature
        u = (torch.rand_like(loc) if noise is None else noise.to(loc)).clamp(1e-20, 1 - 1e-7)
        sample = loc - scale * torch.log(-torch.log(u))            # Gumbel(loc, scale) sample
        logq = gumbel_log_prob(sample, loc, scale)
        ploc = math.log(1.0 / self.alphabet) / self.prior_temperature
        logp = gumbel_log_prob(sample, ploc, 1.0 / self.prior_temperature)
        return torch.softmax(sample, -1), logq, logp

    def compute_loss(self, x, temperature, kld_weight, noise=None) -> Dict[str, torch.Tensor]:
        """NELBO (model.py:88-100).  ``noise``: optional uniforms of the logits' shape (B, G, A) replacing
        the random draw, so two runs (or the HIP and the torch path) see the same sample."""
        if x.is_cuda and os.environ.get("SERANN_RIBOAE_HIP", "1") != "0":
            from ..ops.riboae_ops import available, concrete_sample
            if available():                                        # K36 fused sample + softmax + KL
                z, kl = concrete_sample(self.inference_net(x), temperature, self.prior_temperature, noise)
                logpx_z = self._decode(x, z)
                nelbo = -(logpx_z - kld_weight * kl).mean()
                return {"loss": nelbo, "nll": -logpx_z.mean(), "kld": kl.mean()}
        z, logq, logp = self._encode(x, temperature, noise)
        logpx_z = self._decode(x, z)
        kl = (logq - logp).flatten(1).sum(1)
        nelbo = -(logpx_z - kld_weight * kl).mean()
        return {"loss": nelbo, "nll": -logpx_z.mean(), "kld": kl.mean()}


class DeterministicGAE(GeneticAutoencoder):
    def _encode(self, x):
        return torch.softmax(self.inference_net(x), -1)

    def compute_loss(self, x, *args, **kw):
        z = self._encode(x)
        nll = -self._decode(x, z).mean()
        return {"loss": nll, "nll": nll, "kld": torch.zeros((), device=nll.device)}


def build_model(kind: str = "concrete", **hp) -> GeneticAutoencoder:
    return ConcreteGAE(**hp) if kind == "concrete" else DeterministicGAE(**{k: v for k, v in hp.items()
                                                                            if k != "prior_temperature"})
