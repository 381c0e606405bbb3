"""RiboAE checkpoints: ``torch.save`` of model hyper-parameters + state + optimizer state + step
(the reference keeps only a TF SavedModel of the best model and cannot resume, training.py:92-101).
Loading uses ``weights_only=True``."""
from __future__ import annotations

import os
from typing import Optional

import torch

from ..genome.codec import RiboAECodec
from ..genome.tokenizer import Vocabulary
from ..models.riboae import build_model


def save_checkpoint(path, model, kind: str, step: int, optimizer_state: Optional[dict] = None,
                    extra: Optional[dict] = None):
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    payload = {"kind": kind, "hparams": dict(model.hparams), "state_dict": model.state_dict(), "step": int(step),
               "optimizer": optimizer_state or {}, "extra": extra or {}}
    tmp = str(path) + ".tmp"
    torch.save(payload, tmp)
    os.replace(tmp, path)


def load_checkpoint(path, device="cpu"):
    ck = torch.load(path, map_location=device, weights_only=True)
    model = build_model(ck["kind"], **ck["hparams"])
    model.load_state_dict(ck["state_dict"])
    model.to(device).eval()
    return model, ck


def load_codec(path, vocabulary_path, device="cpu", max_tokens: int = 350) -> RiboAECodec:
    model, ck = load_checkpoint(path, device)
    vocab = Vocabulary.load_csv(vocabulary_path)
    name = os.path.splitext(os.path.basename(str(path)))[0]
    return RiboAECodec(model, vocab, max_tokens=max_tokens, device=device, name=name)


def load_ribosomal_autoencoder(path, device="cpu"):
    """(encode, decode) numpy closures (reference: ribosomal_autoencoder/model.py:123-134)."""
    model, _ = load_checkpoint(path, device)

    def encode(tokens):
        return model.encode_tokens(tokens, device=device)

    def decode(genotype):
        return model.decode_tokens(genotype, device=device)

    return encode, decode
