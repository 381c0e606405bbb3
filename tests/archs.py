"""Architecture corpus for engine/kernel parity tests (decoded, no-space form and template form)."""

ARCHS = {
    # the example.json ancestor's shape (table codec): narrow Dense on the raw genotype feeding a
    # BatchNormalization (fused BN statistics), concat with the raw image (fused concat, no DGRAD slice)
    "narrow_bn_ancestor": (
        "g_layer = Dense(units=75, activation='relu')(g_layer)\n"
        "g_layer = BatchNormalization()(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=152, activation='relu')(con)\n\nloss_balance = 0.85"),
    # (relu, not sigmoid: a BN right after a sigmoid of the raw image normalises outputs whose spread is
    # ~0.05, where bf16 storage (2^-9 near 0.5) alone is a ~4 % error -- an ill-conditioned parity case)
    "narrow_bn_x": (
        "X_layer = Dense(units=24, activation='relu')(X_layer)\n"
        "X_layer = BatchNormalization()(X_layer)\n\n"
        "g_layer = Dense(units=16, activation='relu')(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=40, activation='relu')(con)\n\nloss_balance = 0.4"),
    "conv_pool_dense": (
        "X_layer = Conv2D(filters=16, kernel_size=5, strides=1)(X_layer)\n"
        "X_layer = MaxPool2D(pool_size=2)(X_layer)\n"
        "X_layer = Dense(units=24, activation='relu')(X_layer)\n\n"
        "g_layer = Dense(units=40, activation='sigmoid')(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=64, activation='relu')(con)\n\nloss_balance = 0.7"),
    "odd_channels_bn": (
        "X_layer = Conv2D(filters=8, kernel_size=3, strides=2)(X_layer)\n"
        "X_layer = Dense(units=13, activation='relu')(X_layer)\n"
        "X_layer = BatchNormalization()(X_layer)\n"
        "X_layer = Conv2D(filters=4, kernel_size=3, strides=1)(X_layer)\n\n"
        "g_layer = Conv1D(filters=8, kernel_size=5, strides=2)(g_layer)\n"
        "g_layer = BatchNormalization()(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=37, activation='sigmoid')(con)\ncon = BatchNormalization()(con)\n\nloss_balance = 0.3"),
    "empty_x_branch": (
        "g_layer = Dense(units=64, activation='relu')(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=128, activation='relu')(con)\n\nloss_balance = 0.5"),
    "bn_first_and_pool3": (
        "X_layer = BatchNormalization()(X_layer)\n"
        "X_layer = Conv2D(filters=32, kernel_size=7, strides=1)(X_layer)\n"
        "X_layer = MaxPool2D(pool_size=3)(X_layer)\n\n"
        "g_layer = Conv1D(filters=16, kernel_size=3, strides=1)(g_layer)\n"
        "g_layer = Dense(units=9, activation='relu')(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=48, activation='relu')(con)\ncon = Dense(units=32, activation='sigmoid')(con)\n\n"
        "loss_balance = 0.9"),
    "rewired_fanout": (
        "X_layer = Conv2D(filters=8, kernel_size=5, strides=2)(X_layer)\n"
        "g_layer = Dense(units=16, activation='relu')(g_layer)\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n"
        "con = Dense(units=20, activation='relu')(con)\nloss_balance = 0.6"),
    "mutant_neg_sub": (
        "X_layer = Conv2D(filters=8, kernel_size=3, strides=2)(X_layer)\n"
        "X_layer = -X_layer\n"
        "g_layer = Dense(units=16, activation='relu')(g_layer)\n"
        "g_layer = g_layer-1\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n"
        "con = Dense(units=20, activation='relu')(con)\nloss_balance = 0.4"),
    # BatchNormalization on non-last axes (of a conv output and of a genotype feature map) and a broadcasting
    # tensor - tensor subtraction: ew.hip transposes / maps / broadcast-gradient reductions
    "mutant_bn_axis_bsub": (
        "X_layer = Conv2D(filters=8, kernel_size=3, strides=2)(X_layer)\n"
        "X_layer = BatchNormalization(axis=1)(X_layer)\n"
        "g_layer = Dense(units=16, activation='relu')(g_layer)\n"
        "con = Dense(units=1)(g_layer)\n"
        "g_layer = g_layer-con\n"
        "g_layer = BatchNormalization(axis=-2)(g_layer)\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n"
        "con = Dense(units=20, activation='relu')(con)\nloss_balance = 0.4"),
    "conv1d_rank4_and_strided_pool": (
        "X_layer = Conv2D(filters=8, kernel_size=3, strides=1)(X_layer)\n"
        "X_layer = Conv1D(filters=8, kernel_size=3, strides=2)(X_layer)\n"
        "X_layer = MaxPool2D(pool_size=3, strides=2)(X_layer)\n"
        "g_layer = Conv1D(filters=3, kernel_size=1)(g_layer)\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n"
        "con = Dense(units=24, activation='relu')(con)\nloss_balance = 0.5"),
    # fused first-layer Conv2D + MaxPool2D (csrc/hip/convpool.hip): the bench's dominant clone ...
    "convpool_bench_a": (
        "X_layer=Conv2D(filters=32,kernel_size=5,strides=1)(X_layer)\nX_layer=MaxPool2D(pool_size=3)(X_layer)\n"
        "g_layer=Conv1D(filters=32,kernel_size=5,strides=1)(g_layer)\ng_layer=Dense(units=51,activation='relu')(g_layer)\n"
        "g_layer=BatchNormalization()(g_layer)\n"
        "con=concatenate([Reshape((1,-1))(X_layer),Reshape((1,-1))(g_layer)])\n"
        "con=Dense(units=135,activation='relu')(con)\nloss_balance=0.1329"),
    # ... overlapping windows, relu on the conv, a partial 16-filter tile, 2 k steps of taps
    "convpool_relu_overlap": (
        "X_layer = Conv2D(filters=40, kernel_size=7, strides=2, activation='relu')(X_layer)\n"
        "X_layer = MaxPool2D(pool_size=3, strides=2)(X_layer)\n\n"
        "g_layer = Dense(units=24, activation='relu')(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=64, activation='relu')(con)\n\nloss_balance = 0.6"),
    # ... 9x9 taps (3 k steps), 80 filters (two 64-filter groups), a Dense after the pool
    "convpool_k9_f80": (
        "X_layer = Conv2D(filters=80, kernel_size=9, strides=1)(X_layer)\n"
        "X_layer = MaxPool2D(pool_size=4)(X_layer)\n"
        "X_layer = Dense(units=12, activation='relu')(X_layer)\n\n"
        "g_layer = Dense(units=8, activation='sigmoid')(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=32, activation='relu')(con)\n\nloss_balance = 0.5"),
    # ... sigmoid conv, pool stride larger than the window (gaps)
    "convpool_sigmoid_gap": (
        "X_layer = Conv2D(filters=16, kernel_size=3, strides=1, activation='sigmoid')(X_layer)\n"
        "X_layer = MaxPool2D(pool_size=2, strides=3)(X_layer)\n\n"
        "g_layer = Dense(units=16, activation='relu')(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=24, activation='relu')(con)\n\nloss_balance = 0.7"),
    # fused raw-input Dense -> BatchNormalization (csrc/hip/nbn.hip): a linear 8-unit image Dense, a
    # 200-unit sigmoid genotype Dense (one super-row group per block), a Dense after the BN
    # fused Dense -> BN whose BN output feeds one Dense directly (not through a concat) on the LDS-tiled DGRAD:
    # the BN backward sums are reduced in that DGRAD's epilogue (GF_NBNSUM, nbn phase 6).  (relu: a sigmoid of
    # the 0/1 genotype has a ~0.07 spread per channel, which the BN turns into an ill-conditioned parity case)
    "nbn_sum_direct": (
        "g_layer = Dense(units=64, activation='relu')(g_layer)\n"
        "g_layer = BatchNormalization()(g_layer)\n"
        "g_layer = Dense(units=48, activation='relu')(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=40, activation='relu')(con)\n\nloss_balance = 0.5"),
    # the DGRAD-epilogue BN sums (GF_NBNSUM) under the sigmoid and linear activations of the raw-input Dense
    "nbn_sum_acts": (
        "X_layer = Dense(units=16)(X_layer)\n"
        "X_layer = BatchNormalization()(X_layer)\n\n"
        "g_layer = Dense(units=64, activation='sigmoid')(g_layer)\n"
        "g_layer = BatchNormalization()(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=48, activation='relu')(con)\n\nloss_balance = 0.5"),
    # the binary-genotype factorisation (csrc/hip/bnbn.hip) with the genotype slice FIRST in the concat (it carries
    # the merged Dense's bias gradient) and a linear raw-genotype Dense
    "bnbn_g_first_linear": (
        "X_layer = Conv2D(filters=8, kernel_size=3, strides=2)(X_layer)\n\n"
        "g_layer = Dense(units=32)(g_layer)\n"
        "g_layer = BatchNormalization()(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(g_layer), Reshape((1, -1))(X_layer)])\n\n"
        "con = Dense(units=40, activation='sigmoid')(con)\n\nloss_balance = 0.35"),
    "nbn_wide_linear": (
        "X_layer = Dense(units=8)(X_layer)\n"
        "X_layer = BatchNormalization()(X_layer)\n\n"
        "g_layer = Dense(units=200, activation='sigmoid')(g_layer)\n"
        "g_layer = BatchNormalization()(g_layer)\n"
        "g_layer = Dense(units=10, activation='relu')(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=24, activation='relu')(con)\n\nloss_balance = 0.55"),
    # fused genotype chains (csrc/hip/gchain.hip): Conv1D(raw genotype) -> Dense -> [BN] ...
    "gchain_sigmoid_stride2": (
        "X_layer = Dense(units=20, activation='relu')(X_layer)\n"
        "g_layer = Conv1D(filters=16, kernel_size=3, strides=2)(g_layer)\n"
        "g_layer = Dense(units=40, activation='sigmoid')(g_layer)\n"
        "g_layer = BatchNormalization()(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=32, activation='relu')(con)\n\nloss_balance = 0.4"),
    # ... no BN, 9 taps, 100 units (4 k steps over the Dense output)
    "gchain_nobn_k9_f100": (
        "X_layer = MaxPool2D(pool_size=4)(X_layer)\n"
        "g_layer = Conv1D(filters=8, kernel_size=9, strides=1)(g_layer)\n"
        "g_layer = Dense(units=100, activation='relu')(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=48, activation='relu')(con)\n\nloss_balance = 0.3"),
    # ... 64 filters (two k steps into the Dense), 1 tap, a Dense after the BN (dy not from a concat)
    "gchain_f64_bn_dense": (
        "g_layer = Conv1D(filters=64, kernel_size=1, strides=1)(g_layer)\n"
        "g_layer = Dense(units=64, activation='relu')(g_layer)\n"
        "g_layer = BatchNormalization()(g_layer)\n"
        "g_layer = Dense(units=10, activation='relu')(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=24, activation='relu')(con)\n\nloss_balance = 0.6"),
    # ... activated Conv1D, stride 3, Dense output read by two consumers (no BN fused, dy accumulated)
    "gchain_relu_conv_fanout": (
        "g_layer = Conv1D(filters=24, kernel_size=7, strides=3, activation='relu')(g_layer)\n"
        "g_layer = Dense(units=20, activation='sigmoid')(g_layer)\n"
        "X_layer = Dense(units=12, activation='relu')(g_layer)\n\n"
        "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
        "con = Dense(units=16, activation='relu')(con)\n\nloss_balance = 0.5"),
}
