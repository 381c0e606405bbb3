"""Population statistics (reference: evolutionary_experiment/logic/experiment.py:240-267).

Definitions kept exactly:
* ``mean_pairwise_euclidean_distance`` = mean of scipy ``pdist(genotypes)`` (i < j pairs);
* ``mean_pairwise_hamming_distance``   = mean of pairwise Hamming *fractions*;
* ``nucleotide_diversity``             = **sum** of the full ``cdist`` Hamming-fraction matrix
  (ordered pairs, diagonal zeros, not normalised);
* ``shannon_index`` = -sum p log p over the genotype (or source) distribution;
* ``species_richness`` = number of distinct genotypes (sources).

Genotypes are {0,1}, so Euclidean = sqrt(Hamming count): one popcount pass over bit-packed
genotypes (native C++, ``csrc/host/serann_host_core.h``) replaces the reference's ~1.5 M Python
callbacks per generation at pop=1000.
"""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np

from .native import load


def _pack64(genotypes: np.ndarray) -> np.ndarray:
    g = (np.asarray(genotypes) > 0.5).astype(np.uint8)
    p = np.packbits(g, axis=-1)
    pad = (-p.shape[1]) % 8
    if pad:
        p = np.pad(p, ((0, 0), (0, pad)))
    return np.ascontiguousarray(p).view(np.uint64)


def pairwise_sums(genotypes: np.ndarray):
    """(sum_{i<j} hamming_count, sum_{i<j} sqrt(hamming_count))."""
    g = np.asarray(genotypes)
    n = len(g)
    if n < 2:
        return 0.0, 0.0
    h = load("serann_host")
    if h is not None:
        return h.genotype_pair_stats(_pack64(g))
    gb = (g > 0.5).astype(np.float64)
    d = gb @ (1 - gb).T + (1 - gb) @ gb.T
    iu = np.triu_indices(n, 1)
    return float(d[iu].sum()), float(np.sqrt(d[iu]).sum())


def _entropy_and_richness(keys: Sequence) -> tuple:
    _, counts = np.unique(np.asarray(keys), return_counts=True)
    p = counts / counts.sum()
    return float(-(p * np.log(p)).sum()), int(len(counts))


def genotype_stats(genotypes: np.ndarray, euclid_from_parent, hamming_from_parent) -> Dict[str, float]:
    g = np.asarray(genotypes)
    n, L = g.shape
    npairs = n * (n - 1) // 2
    sh, se = pairwise_sums(g)
    keys = [row.tobytes() for row in (g > 0.5).astype(np.uint8)]
    shannon, richness = _entropy_and_richness(keys)
    return {
        "mean_pairwise_euclidean_distance": se / npairs if npairs else float("nan"),
        "mean_pairwise_hamming_distance": sh / L / npairs if npairs else float("nan"),
        "mean_euclidean_distance_from_parent": float(np.nanmean(euclid_from_parent))
        if np.isfinite(np.asarray(euclid_from_parent, float)).any() else float("nan"),
        "mean_hamming_distance_from_parent": float(np.nanmean(hamming_from_parent))
        if np.isfinite(np.asarray(hamming_from_parent, float)).any() else float("nan"),
        "shannon_index": shannon,
        "nucleotide_diversity": 2.0 * sh / L,
        "species_richness": richness,
    }


def source_code_stats(source_codes: Sequence[str], levenshtein_from_parent) -> Dict[str, float]:
    lev = np.asarray(levenshtein_from_parent, dtype=float)
    shannon, richness = _entropy_and_richness(list(source_codes))
    return {
        "median_levenshtein_distance_from_parent": float(np.nanmedian(lev)) if np.isfinite(lev).any()
        else float("nan"),
        "shannon_index": shannon,
        "species_richness": richness,
    }


def fertility(classification_performance: np.ndarray, selection_pressure: float):
    """Absolute fertility = acc ** lambda; relative = normalised, NaN -> 0 (experiment.py:110-117).

    If no organism is fertile the relative fertility is all zeros (the reference produces NaN here
    and crashes in ``np.random.multinomial``)."""
    acc = np.asarray(classification_performance, dtype=np.float64)
    absolute = acc ** selection_pressure
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = absolute / np.nansum(absolute) if np.nansum(absolute) > 0 else np.zeros_like(absolute)
    rel = np.nan_to_num(rel)
    s = rel.sum()
    if s > 0:
        rel = rel / s
    return absolute, rel
