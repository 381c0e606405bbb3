"""Genome layer: tokenizer (bit-exact vs. golden outputs of the reference tokenizer), interpreter
(Keras-2.6 validity / shape / parameter-count semantics), generator distribution, codecs."""
import json
import math
import os

import numpy as np
import pytest

from serann.genome.codec import TableCodec, decoded_form, pack_bits
from serann.genome.generator import TRANSITIONS, generate, generate_source
from serann.genome.interpreter import interpret, layer_counts, try_interpret
from serann.genome.tokenizer import PAD_TOKEN, Tokenizer, Vocabulary, tokenize

FIX = os.path.join(os.path.dirname(__file__), "fixtures")


def test_tokenizer_matches_reference_golden():
    gold = json.load(open(os.path.join(FIX, "tokenizer_golden.json")))
    for case in gold:
        assert tokenize(case["source"]) == case["tokens"], repr(case["source"])


def test_tokenizer_details():
    t = Tokenizer()
    assert t("Reshape((1, -1))") == ["Reshape", "(", "(", "1", ",", "-", "1", ")", ")"]
    assert t("units=128") == ["units", "=", "1", "2", "8"]
    assert t("a\n\n\nb") == ["a", "\n", "b"]


def test_vocabulary_roundtrip(tmp_path):
    srcs = [generate_source(np.random.default_rng(i))["code"] for i in range(30)]
    vocab = Vocabulary.build(tokenize(s) for s in srcs)
    assert vocab.index2token[-1] == PAD_TOKEN
    enc = vocab.encode_strings(srcs, 350)
    dec = vocab.decode(enc)
    assert dec == [decoded_form(s) for s in srcs]
    p = tmp_path / "v.csv"
    vocab.save_csv(p)
    v2 = Vocabulary.load_csv(p)
    assert list(v2.index2token) == list(vocab.index2token)


def test_rstrip_is_character_set_strip():
    vocab = Vocabulary(["a", "P", "x"])
    seq = np.array([[vocab.token2index["x"], vocab.token2index["a"], vocab.token2index["P"], vocab.pad_index]])
    # 'xaP<PAD>' -> rstrip of the character set {<,P,A,D,>} removes 'P' too but keeps 'a'
    assert vocab.decode(seq) == ["xa"]


BASE = ("X_layer = Conv2D(filters=8, kernel_size=5, strides=1)(X_layer)\n"
        "g_layer = Dense(units=10, activation='relu')(g_layer)\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n"
        "con = Dense(units=32, activation='relu')(con)\n"
        "loss_balance = 0.25")


def test_param_count_matches_keras_formula():
    r = try_interpret(BASE)
    assert r.ok
    conv = 5 * 5 * 1 * 8 + 8
    gd = 1 * 10 + 10
    D = 24 * 24 * 8 + 100 * 10
    md = D * 32 + 32
    heads = 32 * 10 + 10 + 32 * 100 + 100
    assert r.parameters_count == conv + gd + md + heads
    assert r.loss_balance == 0.25


def test_decoded_form_is_valid_python():
    r = try_interpret(decoded_form(BASE))
    assert r.ok


def test_bn_counts_moving_stats():
    src = BASE.replace("con = Dense(units=32, activation='relu')(con)", "con = BatchNormalization()(con)")
    r = try_interpret(src)
    D = 24 * 24 * 8 + 100 * 10
    assert r.ok and r.parameters_count == (5 * 5 * 8 + 8) + 20 + 4 * D + (D * 10 + 10 + D * 100 + 100)


@pytest.mark.parametrize("src,why", [
    ("X_layer=Conv2D(filters=08,kernel_size=3)(X_layer)\ncon=X_layer\nloss_balance=0.5", "syntax"),
    ("g_layer=Conv2D(filters=8,kernel_size=3)(g_layer)\ncon=g_layer\nloss_balance=0.5", "conv2d rank"),
    ("X_layer=Conv2D(filters=8,kernel_size=29)(X_layer)\ncon=X_layer\nloss_balance=0.5", "negative dim"),
    ("X_layer=MaxPool2D(pool_size=2)(g_layer)\ncon=X_layer\nloss_balance=0.5", "pool rank"),
    ("X_layer=Dense(units=8,filters=3)(X_layer)\ncon=X_layer\nloss_balance=0.5", "bad kwarg"),
    ("X_layer=Dense(units=8,activation='relurelu')(X_layer)\ncon=X_layer\nloss_balance=0.5", "activation"),
    ("X_layer=Dense(units=8)(X_layer)\nloss_balance=0.5", "missing con"),
    ("con=X_layer", "missing loss_balance"),
    ("con=X_layer\nloss_balance=X_layer", "tensor loss balance"),
    ("con=Dense\nloss_balance=0.5", "con not tensor"),
    ("con=concatenate([X_layer,g_layer])\nloss_balance=0.5", "concat rank mismatch"),
    ("con=Reshape((5,-1))(X_layer)\nloss_balance=0.5", "reshape divisibility"),
    ("con=relu\nloss_balance=0.5", "name error"),
    ("con=X_layer(X_layer)\nloss_balance=0.5", "tensor not callable"),
])
def test_invalid_sources(src, why):
    assert not try_interpret(src).ok, why


@pytest.mark.parametrize("src", [
    "X_layer,g_layer=g_layer,X_layer\ncon=Conv1D(4,3,2)(X_layer)\nloss_balance=1",
    "con=concatenate([Reshape((1,-1))(X_layer)])\nloss_balance=0.5",
    "X_layer=Conv1D(filters=4,kernel_size=3)(X_layer)\ncon=X_layer\nloss_balance='5'",
    "con=X_layer=Dense(5,'sigmoid',0)(X_layer)\nloss_balance=-0.5",
    "X_layer=MaxPool2D(pool_size=(2,3),strides=1)(X_layer)\ncon=X_layer\nloss_balance=0.1",
    "Dense(units=3)(g_layer)\ncon=-X_layer\nloss_balance=0.5",
    "con=BatchNormalization(1)(g_layer)\nloss_balance=0.5",
])
def test_valid_mutants(src):
    r = try_interpret(src)
    assert r.ok, r.error


def test_dangling_layers_not_counted():
    a = try_interpret("con=X_layer\nloss_balance=0.5")
    b = try_interpret("g_layer=Dense(units=50)(g_layer)\ncon=X_layer\nloss_balance=0.5")
    assert a.ok and b.ok and a.parameters_count == b.parameters_count


def test_conv_shapes_and_strides():
    ir = interpret("X_layer=Conv2D(filters=4,kernel_size=(3,5),strides=(2,1))(X_layer)\ncon=X_layer\nloss_balance=0")
    conv = [n for n in ir.nodes if n.op == "gemm" and n.attrs["kind"] == "conv2d"][0]
    assert conv.shape == ((28 - 3) // 2 + 1, 28 - 5 + 1, 4)


def test_layer_counts():
    src = decoded_form(BASE)
    assert layer_counts(src) == {"classification_layers": 1, "replication_layers": 1, "merged_layers": 2}


def test_generator_distribution_matches_reference_survey():
    # SURVEY §2.2 (derived from the reference chain): ~9.2% invalid, p50 0.95M params, ~23.8% overweight
    rng = np.random.default_rng(0)
    ok, params, flops = 0, [], []
    N = 3000
    for _ in range(N):
        r = try_interpret(generate_source(rng)["code"], genotype_size=100)
        if r.ok:
            ok += 1
            params.append(r.parameters_count)
            if r.parameters_count <= 2e6:
                flops.append(r.ir.flops_per_sample())
    params = np.array(params)
    assert 0.06 < 1 - ok / N < 0.12
    assert 0.7e6 < np.median(params) < 1.25e6
    assert 0.19 < (params > 2e6).mean() < 0.28
    assert 1.8e6 < np.median(flops) < 2.9e6


def test_effective_g_row():
    # the reference's g row sums to 1.1; the effective (sorted-cumsum) distribution is 0.4/0.4/0.2
    assert dict(TRANSITIONS["g"]) == {"g_Dense": 0.4, "g_Conv1D": 0.4, "M_Concatenate": 0.2}
    for k, v in TRANSITIONS.items():
        assert math.isclose(sum(p for _, p in v), 1.0), k


def test_generate_dataframe_columns():
    df = generate(20, seed=1)
    assert list(df.columns) == ["code", "parameters_count", "last_layer", "net_hash", "x_layers", "g_layers",
                                "m_layers", "loss_balance"]
    assert df["net_hash"].is_unique


def test_table_codec_deterministic_and_anchored():
    anc = np.zeros(100, dtype=int)
    c = TableCodec.from_generator(64, seed=2, ancestor=anc)
    g = np.random.default_rng(0).integers(0, 2, (5, 100))
    assert c.decode_to_string(g) == c.decode_to_string(g)
    a = try_interpret(c.decode_to_string(anc[None])[0])
    assert a.ok and a.parameters_count <= 2e6
    assert pack_bits(anc[None]).shape == (1, 13)
