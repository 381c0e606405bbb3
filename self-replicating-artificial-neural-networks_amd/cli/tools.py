"""Dataset-bootstrap CLIs (README stages 1-4 of the reference):

* ``generator``              -- synthetic SeRANN dataset (synthetic_serann_generator/generator.py:128-143)
* ``source_codes_to_tokens`` -- tokenize, build the vocabulary, pad (helpers/source_codes_to_tokens.py)
* ``tokens_to_genotypes``    -- encode a token dataset with a RiboAE (helpers/tokens_to_genotypes.py);
                                the reference encodes the whole dataset once per batch (SURVEY §2.9
                                item 3) -- here each batch is encoded once, on the GPU when present
* ``training``               -- RiboAE trainer (ribosomal_autoencoder/training.py:104-133)
File formats are the reference's: zip-compressed CSV, ``sequences`` npz, ``token,index`` CSV,
``encodings`` npz.
"""
from __future__ import annotations

import argparse
import json
import os
from pathlib import Path

import numpy as np
import pandas as pd

from ..config import global_config, riboae_config


def generator_main(argv=None):
    p = argparse.ArgumentParser(description="Generate a synthetic SeRANN dataset")
    p.add_argument("-d", "--dataset-name", required=True, help="Output dataset name")
    p.add_argument("-n", "--num-of-examples", default=10000, type=int, help="Number of examples to generate")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--workers", type=int, default=min(8, os.cpu_count() or 1))
    p.add_argument("--validation-genotype-size", type=int, default=350,
                   help="genotype length used to validate nets (reference: 350)")
    a = p.parse_args(argv)
    from ..genome.generator import generate
    out = Path(global_config["synthetic_datasets_dir"]) / f"{a.dataset_name}.csv"
    out.parent.mkdir(parents=True, exist_ok=True)
    df = generate(a.num_of_examples, seed=a.seed, validation_genotype_size=a.validation_genotype_size,
                  workers=a.workers)
    df.to_csv(out, index=False, compression="zip")
    print(f"{len(df)} unique nets written to {out}")
    return out


def source_codes_to_tokens_main(argv=None):
    p = argparse.ArgumentParser(description="Tokenize a synthetic SeRANN dataset")
    p.add_argument("-d", "--dataset-name", required=True, help="Synthetic SeRANN dataset name")
    p.add_argument("-m", "--max-tokens", default=350, type=int, help="Maximum tokens sequence length")
    a = p.parse_args(argv)
    from ..genome.tokenizer import Vocabulary, tokenize
    df = pd.read_csv(Path(global_config["synthetic_datasets_dir"]) / f"{a.dataset_name}.csv", compression="zip")
    tokens = [tokenize(s) for s in df["code"]]
    vocab = Vocabulary.build(tokens)
    keep = [t for t in tokens if len(t) <= a.max_tokens]
    seqs = np.stack([vocab.encode(t, a.max_tokens) for t in keep]) if keep else np.zeros((0, a.max_tokens), np.int64)
    tok_dir, voc_dir = Path(global_config["token_sequences_dir"]), Path(global_config["vocabularies_dir"])
    tok_dir.mkdir(parents=True, exist_ok=True)
    voc_dir.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(tok_dir / f"{a.dataset_name}.npz", sequences=seqs)
    vocab.save_csv(voc_dir / f"{a.dataset_name}.csv")
    print(f"{len(seqs)} sequences (dropped {len(tokens) - len(keep)} > {a.max_tokens} tokens), "
          f"vocabulary of {len(vocab)}")


def tokens_to_genotypes_main(argv=None):
    p = argparse.ArgumentParser(description="Encode token sequences into genotypes with a RiboAE")
    p.add_argument("-d", "--dataset-name", required=True, help="Synthetic SeRANN dataset name")
    p.add_argument("-r", "--riboae-name", required=True, help="Ribosomal autoencoder model name")
    p.add_argument("-b", "--batch-size", default=256, type=int, help="Batch size for the RiboAE inference")
    p.add_argument("--device", default=None)
    a = p.parse_args(argv)
    import torch
    from ..riboae.io import load_checkpoint
    device = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    seqs = np.load(Path(global_config["token_sequences_dir"]) / f"{a.dataset_name}.npz")["sequences"]
    ck = Path(global_config["ribosomal_autoencoders_dir"]) / a.riboae_name
    ck = ck if ck.suffix == ".pt" else ck.with_suffix(".pt")
    model, _ = load_checkpoint(ck, device)
    out = [model.encode_tokens(seqs[i:i + a.batch_size], device=device) for i in range(0, len(seqs), a.batch_size)]
    enc = np.concatenate(out, 0).astype(np.int8) if out else np.zeros((0, model.genotype_length), np.int8)
    d = Path(global_config["encodings_datasets_dir"])
    d.mkdir(parents=True, exist_ok=True)
    path = d / f"{a.dataset_name}__{a.riboae_name}.npz"
    np.savez_compressed(path, encodings=enc)
    print(f"{len(enc)} genotypes written to {path}")


def training_main(argv=None):
    p = argparse.ArgumentParser(description="Train the ribosomal autoencoder")
    p.add_argument("-p", "--parameters", required=True, help="Experiment parameters file path")
    p.add_argument("-n", "--name", required=True, help="Output model name")
    p.add_argument("--dataset", default=None, help="token sequences npz (default: config path)")
    p.add_argument("--vocabulary", default=None, help="vocabulary csv (default: config path)")
    p.add_argument("--max-steps", type=int, default=None, help="stop after N batches (reference: infinite)")
    p.add_argument("--resume", default=None, help="checkpoint to resume from")
    p.add_argument("--device", default=None)
    p.add_argument("--deterministic", action="store_true", help="train the DeterministicGAE variant")
    a = p.parse_args(argv)
    import torch
    from ..genome.tokenizer import Vocabulary
    from ..models.riboae import ConcreteGAE, DeterministicGAE
    from ..riboae.trainer import get_dataset, train
    with open(a.parameters) as f:
        params = json.load(f)
    device = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    torch.manual_seed(riboae_config["random_seed"])
    vocab = Vocabulary.load_csv(a.vocabulary or riboae_config["vocabulary_path"])
    seqs = np.load(a.dataset or riboae_config["token_sequences_dataset_path"])["sequences"]
    hp = dict(genotype_length=params["genotype_size"], max_phenotype_length=params["source_code_length"],
              vocabulary_size=len(vocab), embedding_dim=params["embedding_size"],
              genotype_alphabet_size=params["genotype_alphabet_size"])
    model = DeterministicGAE(**hp) if a.deterministic else ConcreteGAE(**hp,
                                                                       prior_temperature=params["prior_temperature"])
    train_set, _ = get_dataset(seqs, params["train_test_ratio"])
    train(a.name, model, train_set, vocab, riboae_config["ribosomal_autoencoders_dir"], batch_size=params["batch_size"],
          min_backup_interval=params["min_backup_interval"], max_steps=a.max_steps, device=device,
          resume_path=a.resume)
