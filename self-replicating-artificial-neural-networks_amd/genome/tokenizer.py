"""Bit-exact SeRANN source-code tokenizer and vocabulary IO.

Behavioural contract (reference: evolutionary_experiment/logic/ribosomal_autoencoder.py:129-152,
helpers/source_codes_to_tokens.py:21-36):

* blank lines are collapsed (``\\n\\n`` -> ``\\n``, applied twice) and all spaces removed at every
  recursion level;
* the string is split on ``\\n = ' ( ) [ ] , .`` in that priority order, separators kept as tokens;
* at the leaf level a piece that parses as a Python ``int`` is split into single characters
  (so ``-1`` -> ``-``, ``1``), anything else (including the empty string) is one token;
* an empty string at a non-leaf level produces no tokens.

The implementation here is an explicit work-list version (no recursion, no quadratic
``sum(list, [])``) that yields the same token stream.
"""
from __future__ import annotations

from typing import Iterable, List, Sequence

import numpy as np

SPLIT_CHARACTERS: Sequence[str] = ("\n", "=", "'", "(", ")", "[", "]", ",", ".")
PAD_TOKEN = "<PAD>"


def _is_python_int(s: str) -> bool:
    try:
        int(s)
        return True
    except ValueError:
        return False


def _normalise(s: str) -> str:
    return s.replace("\n\n", "\n").replace("\n\n", "\n").replace(" ", "")


def tokenize(source: str, split_characters: Sequence[str] = SPLIT_CHARACTERS) -> List[str]:
    """Tokenize one SeRANN source code string."""
    out: List[str] = []
    # stack of (piece, level); processed depth-first, left to right
    stack = [(source, 0)]
    n_levels = len(split_characters)
    while stack:
        s, level = stack.pop()
        if level == n_levels:
            if _is_python_int(s):
                out.extend(s)
            else:
                out.append(s)
            continue
        s = _normalise(s)
        if s == "":
            continue
        c = split_characters[level]
        pieces = s.split(c)
        seq = []
        for i, p in enumerate(pieces):
            if i:
                seq.append(c)
            seq.append(p)
        # push in reverse so the leftmost piece is processed first
        for p in reversed(seq):
            stack.append((p, level + 1))
    return out


class Tokenizer:
    """Callable tokenizer object (API of the reference ``Tokenizer``)."""

    def __init__(self, split_characters: Sequence[str] = SPLIT_CHARACTERS):
        self._split_characters = tuple(split_characters)

    def __call__(self, s: str, split_characters: Sequence[str] | None = None) -> List[str]:
        return tokenize(s, self._split_characters if split_characters is None else split_characters)


class Vocabulary:
    """Token <-> index mapping; ``<PAD>`` is the last index (source_codes_to_tokens.py:73-77)."""

    def __init__(self, tokens: Sequence[str]):
        tokens = list(tokens)
        if PAD_TOKEN not in tokens:
            tokens.append(PAD_TOKEN)
        self.index2token = np.array(tokens, dtype=object)
        self.token2index = {t: i for i, t in enumerate(tokens)}
        self.pad_index = self.token2index[PAD_TOKEN]

    def __len__(self) -> int:
        return len(self.index2token)

    @classmethod
    def build(cls, token_lists: Iterable[Sequence[str]]) -> "Vocabulary":
        unique = set()
        for toks in token_lists:
            unique.update(toks)
        unique.discard(PAD_TOKEN)
        return cls(sorted(unique) + [PAD_TOKEN])

    @classmethod
    def load_csv(cls, path) -> "Vocabulary":
        import pandas as pd
        df = pd.read_csv(path, keep_default_na=False)
        df = df.sort_values("index")
        return cls(list(df["token"]))

    def save_csv(self, path) -> None:
        import pandas as pd
        df = pd.DataFrame({"token": list(self.index2token), "index": np.arange(len(self))})
        df.to_csv(path, index=False)

    def encode(self, tokens: Sequence[str], max_tokens: int) -> np.ndarray:
        out = np.full(max_tokens, self.pad_index, dtype=np.int64)
        idx = [self.token2index[t] for t in tokens[:max_tokens]]
        out[:len(idx)] = idx
        return out

    def encode_strings(self, sources: Sequence[str], max_tokens: int) -> np.ndarray:
        """Tokenize, truncate to ``max_tokens`` and pad (ribosomal_autoencoder.py:49-57)."""
        out = np.full((len(sources), max_tokens), self.pad_index, dtype=np.int64)
        for i, s in enumerate(sources):
            toks = tokenize(s)[:max_tokens]
            out[i, :len(toks)] = [self.token2index[t] for t in toks]
        return out

    def decode(self, sequences: np.ndarray) -> List[str]:
        """Join tokens with '' and ``rstrip('<PAD>')`` -- a *character-set* strip, exactly like the
        reference (ribosomal_autoencoder.py:69-78)."""
        sequences = np.asarray(sequences)
        words = self.index2token[sequences]
        return ["".join(w).rstrip(PAD_TOKEN) for w in words]
