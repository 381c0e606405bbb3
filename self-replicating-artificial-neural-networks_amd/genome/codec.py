"""Genetic codecs: genotype (bit vector) <-> decoded SeRANN source code.

The reference's only codec is the learned ribosomal autoencoder (RiboAE), queried through a CPU
side-process (evolutionary_experiment/logic/ribosomal_autoencoder.py:12-126).  Here codecs are
in-process objects with the same public API (``decode_to_string``, ``encode_string``,
``decode_to_sequence``, ``encode_sequence``, ``sequence_to_string``):

* :class:`RiboAECodec` -- the ribosomal autoencoder (``serann.models.riboae``) running on the GPU
  (HIP decode kernels) or CPU;
* :class:`TableCodec`  -- a *synthetic* codec for benchmarking and plumbing without a trained
  RiboAE: genotypes are hashed into a table of generator-sampled nets, so decoded
  populations follow the reference architecture distribution.  The ancestor genotype(s) can be
  pinned to a chosen valid, trainable net.  ``sensitive_bits`` restricts the hash to the first k
  loci so that mutations elsewhere are silent (a knob for clonal-population studies).
"""
from __future__ import annotations

import hashlib
from typing import Dict, List, Optional, Sequence

import numpy as np

from .tokenizer import PAD_TOKEN, Vocabulary, tokenize


def decoded_form(source: str) -> str:
    """The form a source takes after a RiboAE round trip: tokens joined with '' (no spaces)."""
    return "".join(tokenize(source))


class GeneticCodec:
    genotype_size: int = 100
    max_tokens: int = 350
    name: str = "codec"

    def decode_to_string(self, genotypes) -> List[str]:
        raise NotImplementedError

    def encode_string(self, sources: Sequence[str]) -> np.ndarray:
        raise NotImplementedError

    def get_model_name(self) -> str:
        return self.name


def pack_bits(genotypes: np.ndarray) -> np.ndarray:
    g = (np.asarray(genotypes) > 0.5).astype(np.uint8)
    return np.packbits(g, axis=-1)


class TableCodec(GeneticCodec):
    def __init__(self, sources: Sequence[str], genotype_size: int = 100, max_tokens: int = 350,
                 anchors: Optional[Dict[bytes, str]] = None, sensitive_bits: Optional[int] = None,
                 salt: str = "serann"):
        self.table = [decoded_form(s) for s in sources]
        self.genotype_size = genotype_size
        self.max_tokens = max_tokens
        # anchors are stored in decoded form: the ancestor's unmutated clones are a large share of every
        # early generation, and re-tokenising the source per clone cost ~2 ms each (pop 1000: ~1 s/gen)
        self.anchors = {k: decoded_form(v) for k, v in (anchors or {}).items()}
        self.sensitive_bits = sensitive_bits or genotype_size
        self.salt = salt.encode()
        self.name = f"table{len(self.table)}"
        self._vocab = None

    @classmethod
    def from_generator(cls, n: int = 4096, seed: int = 0, genotype_size: int = 100,
                       ancestor: Optional[Sequence[int]] = None, anchor_max_params: float = 2e6,
                       **kw) -> "TableCodec":
        from .generator import generate
        from .interpreter import try_interpret
        df = generate(n, seed=seed)
        sources = list(df["code"])
        anchors = {}
        if ancestor is not None:
            # pin the ancestor to the first net that is valid and trainable at this genotype size
            for s in sources:
                r = try_interpret(decoded_form(s), genotype_size=genotype_size)
                if r.ok and r.parameters_count <= anchor_max_params:
                    anchors[pack_bits(np.asarray(ancestor)[None])[0].tobytes()] = s
                    break
        return cls(sources, genotype_size=genotype_size, anchors=anchors, **kw)

    def _index(self, key: bytes) -> int:
        h = hashlib.blake2b(key, digest_size=8, key=self.salt[:64]).digest()
        return int.from_bytes(h, "little") % len(self.table)

    def decode_to_string(self, genotypes) -> List[str]:
        g = np.asarray(genotypes)
        if g.ndim == 1:
            g = g[None]
        packed_full = pack_bits(g)
        packed_sens = pack_bits(g[:, :self.sensitive_bits])
        out = []
        for full, sens in zip(packed_full, packed_sens):
            a = self.anchors.get(full.tobytes())
            out.append(a if a is not None else self.table[self._index(sens.tobytes())])
        return out

    # a table codec has no inverse: encoding returns the genotype of a table row when known
    def encode_string(self, sources: Sequence[str]) -> np.ndarray:
        raise NotImplementedError("TableCodec is decode-only")


class RiboAECodec(GeneticCodec):
    """Ribosomal-autoencoder codec (in-process; replaces RiboAeProcess + queues)."""

    def __init__(self, model, vocabulary: Vocabulary, max_tokens: int = 350, device="cpu",
                 name: str = "riboae", batch_size: int = 4096):
        self.model = model
        self.vocab = vocabulary
        self.max_tokens = max_tokens
        self.genotype_size = model.genotype_length
        self.device = device
        self.name = name
        self.batch_size = batch_size
        self.PADDING_TOKEN = vocabulary.pad_index

    def decode_to_sequence(self, genotypes) -> np.ndarray:
        g = np.asarray(genotypes)
        if g.ndim == 1:
            g = g[None]
        outs = []
        for i in range(0, len(g), self.batch_size):
            outs.append(self.model.decode_tokens(g[i:i + self.batch_size], device=self.device))
        return np.concatenate(outs, 0) if outs else np.zeros((0, self.max_tokens), np.int64)

    def encode_sequence(self, tokens) -> np.ndarray:
        t = np.asarray(tokens)
        outs = []
        for i in range(0, len(t), self.batch_size):
            outs.append(self.model.encode_tokens(t[i:i + self.batch_size], device=self.device))
        return np.concatenate(outs, 0)

    def sequence_to_string(self, sequences) -> List[str]:
        return self.vocab.decode(np.asarray(sequences))

    def decode_to_string(self, genotypes) -> List[str]:
        return self.sequence_to_string(self.decode_to_sequence(genotypes))

    def encode_string(self, sources: Sequence[str]) -> np.ndarray:
        return self.encode_sequence(self.vocab.encode_strings(sources, self.max_tokens))

    def remove_sequences_padding(self, sequences):
        sequences = np.asarray(sequences)
        lengths = sequences.shape[1] - np.sum(sequences == self.vocab.pad_index, axis=1)
        return [sequences[i, :lengths[i]] for i in range(len(sequences))]
