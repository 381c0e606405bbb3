"""Per-kernel numerics on bf16-exact operands vs. plain PyTorch fp32 references of the same op.

Operands are drawn as bf16 values, so the only differences are fp32 accumulation order and the
final bf16 rounding of the output (<~0.4% relative).  Gradients land in the deterministic fixed-point
fixed-point arena (csrc/hip/common.h fx_*), BatchNorm statistics in the wide fixed-point workspace;
the determinism tests re-run a kernel and require bitwise-identical results."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from serann.ops import hip_ops as H

pytestmark = pytest.mark.gpu
DEV = "cuda"


# fp32 PyTorch references run on the CPU: exact fp32 convolution math, independent of the GPU
# library paths (MIOpen solver selection) the kernels under test are compared against
def _cpu(t):
    return t.detach().float().cpu() if torch.is_tensor(t) else t


def ref_conv2d(x, w, b, stride):
    return F.conv2d(_cpu(x), _cpu(w), _cpu(b), stride).to(DEV)


def ref_conv2d_input(shape, w, dz, stride):
    return torch.nn.grad.conv2d_input(shape, _cpu(w), _cpu(dz), stride).to(DEV)


def ref_conv2d_weight(x, wshape, dz, stride):
    return torch.nn.grad.conv2d_weight(_cpu(x), wshape, _cpu(dz), stride).to(DEV)


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def _desc(rows, dtype):
    a = np.zeros(len(rows), dtype=dtype)
    for i, r in enumerate(rows):
        for k, v in r.items():
            a[i][k] = v
    if dtype == H.GEMM_DTYPE:
        H.fill_gemm_divisors(a)
    return torch.as_tensor(np.frombuffer(a.tobytes(), dtype=np.uint8).copy(), device=DEV)


def _run_gemm(mode, rows, dims):
    # reference ops (MIOpen / hipBLASLt) may still be in flight, and the descriptor tables below are
    # uploaded from pageable memory: start every launch from an idle device
    torch.cuda.synchronize()
    keep = []
    for v, rws, tiles in H.gemm3_plan(mode, [dict(r) for r in rows], dims):
        fin = []
        for r in rws:
            if r.get("_wgfin"):                   # split conv WGRAD: fp32 slabs + the ordered finalize
                ws = torch.empty(H.wgrad_slab_elems(r) + 64, dtype=torch.float32, device=DEV)
                keep.append(ws)
                fin.append(H.wgrad_finalize_row(r, ws.data_ptr()))
        d = _desc([{k: val for k, val in r.items() if not k.startswith("_")} for r in rws], H.GEMM_DTYPE)
        t = torch.as_tensor(tiles, device=DEV)
        H.lib().gemm3(mode, v, d.data_ptr(), t.data_ptr(), len(t), H.stream_handle())
        if fin:
            fd = _desc(fin, H.WGFIN_DTYPE)
            ft = torch.as_tensor(H.chunk_tiles([f["M"] * f["N"] for f in fin], H.WGFIN_ELEMS), device=DEV)
            H.lib().wgrad_finalize(fd.data_ptr(), ft.data_ptr(), len(ft), H.stream_handle())
            keep += [fd, ft]
    torch.cuda.synchronize()


def _q(t):
    """Gradient-arena fixed point (int64, 2^-40 units) -> fp32."""
    return H.from_qg(t)


SHAPES = [  # B, H, W, C, F, KH, KW, SH, SW, act
    (3, 28, 28, 1, 16, 5, 5, 1, 1, "relu"),
    (2, 13, 13, 13, 4, 3, 3, 1, 1, "linear"),
    (4, 12, 12, 16, 37, 3, 3, 2, 2, "sigmoid"),
    (2, 9, 7, 64, 64, 1, 1, 1, 1, "relu"),
    (5, 100, 1, 1, 32, 5, 1, 2, 1, "linear"),
    (7, 1, 1, 868, 110, 1, 1, 1, 1, "linear"),
    (2, 26, 26, 8, 8, 1, 3, 1, 2, "relu"),
    (3, 10, 10, 24, 9, 7, 7, 1, 1, "linear"),
    # v3 paths: RT=4 rows/wave (M >= 16384), odd C with kernel-row wraps, NT=8 (N > 64), stride 3,
    # KW*C < 8 gathers (GEN), F % 8 != 0 conv DGRAD (GEN)
    (48, 24, 24, 20, 32, 5, 5, 1, 1, "relu"),
    (6, 28, 28, 55, 64, 7, 7, 1, 1, "linear"),
    (4, 6, 6, 40, 100, 3, 3, 1, 1, "relu"),
    (3, 20, 20, 16, 16, 3, 3, 3, 3, "linear"),
    (2, 11, 11, 2, 13, 3, 3, 2, 2, "linear"),
    (30, 30, 1, 3, 24, 7, 1, 1, 1, "relu"),
    # single-k-step FWD/DGRAD (K <= 32, M >= 16384) and the narrow (N <= 16) WGRAD layout
    (30, 28, 28, 1, 100, 1, 1, 1, 1, "relu"),
    (25, 26, 26, 24, 40, 1, 1, 1, 1, "sigmoid"),
    # narrow VALU kernels (K <= 4 input channels, 1x1): FWD and WGRAD
    (4, 9, 9, 3, 200, 1, 1, 1, 1, "sigmoid"),
    (6, 10, 10, 2, 13, 1, 1, 1, 1, "linear"),
    (30, 100, 1, 1, 75, 1, 1, 1, 1, "relu"),      # narrow + LDS-staged rows (N % 8 != 0): g Dense(75)
    (30, 100, 1, 2, 37, 1, 1, 1, 1, "sigmoid"),   # staged, K = 2, multi-pass blocks with a ragged tail
    (13, 100, 1, 1, 130, 1, 1, 1, 1, "relu"),     # staged, N > 128 (several FWD passes per block)
    # small conv outputs: the conv WGRAD kernel packs several whole images into one 128-row chunk
    # (5x5 outputs: 3 images per chunk, a ragged last chunk; 8x8 outputs: 2 images per chunk)
    (17, 11, 11, 64, 16, 7, 7, 1, 1, "relu"),
    (9, 12, 12, 32, 24, 5, 5, 1, 1, "linear"),
    # tap-shifted conv WGRAD (round 5): a whole 2000-column reduction in two 1024-column blocks (16 column
    # tiles per wave, odd C), 49 taps x 32 channels, 64 filters x 4 column tiles per wave with odd C
    (6, 28, 28, 74, 16, 5, 5, 1, 1, "relu"),
    (5, 24, 24, 32, 16, 7, 7, 1, 1, "linear"),
    (4, 14, 14, 61, 64, 5, 5, 1, 1, "relu"),
    (3, 24, 24, 16, 16, 5, 5, 2, 2, "sigmoid"),
    # small-bank WGRAD (F <= 16, <= 64 columns, 1x1): one MFMA row tile per block, waves on their own row steps
    (10, 26, 26, 9, 16, 1, 1, 1, 1, "relu"),
    (12, 20, 20, 49, 8, 1, 1, 1, 1, "linear"),
    # production-batch first layers on a one-channel input (RT = 4 DGRAD into C = 1)
    (750, 28, 28, 1, 32, 7, 7, 1, 1, "linear"),
    (48, 32, 16, 1, 32, 5, 5, 1, 1, "linear"),
    # wide-f WGRAD tiles (F > 64: one 128- or 256-row f tile per layer)
    (9, 1, 1, 300, 200, 1, 1, 1, 1, "relu"),
    (40, 5, 1, 96, 120, 1, 1, 1, 1, "sigmoid"),
]


@pytest.mark.parametrize("shape", SHAPES)
def test_grouped_conv_fwd_dgrad_wgrad(shape):
    B, Hh, Ww, C, Fo, KH, KW, SH, SW, act = shape
    OH, OW = (Hh - KH) // SH + 1, (Ww - KW) // SW + 1
    g = torch.Generator(device=DEV).manual_seed(0)
    x = H.padded(torch.randn(B, Hh, Ww, C, device=DEV, generator=g).bfloat16())
    w = H.padded((torch.randn(Fo, KH, KW, C, device=DEV, generator=g) / math.sqrt(KH * KW * C)).bfloat16())  # Wm layout
    bias = H.padded(torch.randn(Fo, device=DEV, generator=g))
    dz = H.padded(torch.randn(B, OH, OW, Fo, device=DEV, generator=g).bfloat16())
    xr = x.float().permute(0, 3, 1, 2)
    wr = w.float().permute(0, 3, 1, 2)            # (F, C, KH, KW)
    ref = ref_conv2d(xr, wr, bias, (SH, SW)).permute(0, 2, 3, 1)
    ref = {"relu": torch.relu, "sigmoid": torch.sigmoid, "linear": lambda t: t}[act](ref)
    # FWD
    y = H.padded(torch.zeros(B, OH, OW, Fo, dtype=torch.bfloat16, device=DEV))
    K = KH * KW * C
    flags = (H.GF_VEC_A if C % 8 == 0 else 0) | (H.GF_VEC_B if K % 8 == 0 else 0)
    geo = dict(H=Hh, W=Ww, C=C, OH=OH, OW=OW, F=Fo, KH=KH, KW=KW, SH=SH, SW=SW)
    _run_gemm(H.MODE_FWD, [dict(a=x.data_ptr(), b=w.data_ptr(), out=y.data_ptr(), bias=bias.data_ptr(),
                                M=B * OH * OW, N=Fo, K=K, act=H.ACT_CODES[act], flags=flags, **geo)],
              [(B * OH * OW, Fo, K)])
    assert _rel(y.float(), ref) < 6e-3
    # DGRAD
    dx = H.padded(torch.zeros(B, Hh, Ww, C, dtype=torch.bfloat16, device=DEV))
    ref_dx = ref_conv2d_input(xr.shape, wr, dz.float().permute(0, 3, 1, 2), (SH, SW)).permute(0, 2, 3, 1)
    flags = (H.GF_VEC_A if Fo % 8 == 0 else 0) | (H.GF_VEC_B if C % 8 == 0 else 0)
    wt = H.padded(w.permute(3, 1, 2, 0).contiguous())  # Wt[C][KH][KW][F] for the register-fragment DGRAD kernel
    _run_gemm(H.MODE_DGRAD, [dict(a=dz.data_ptr(), b=wt.data_ptr(), _bnat=w.data_ptr(), out=dx.data_ptr(),
                                  M=B * Hh * Ww, N=C, K=KH * KW * Fo, flags=flags, **geo)],
              [(B * Hh * Ww, C, KH * KW * Fo)])
    assert _rel(dx.float(), ref_dx) < 6e-3
    # WGRAD (accumulates into a zeroed fixed-point buffer, split over m); run twice: bitwise equal
    ref_dw = ref_conv2d_weight(xr, wr.shape, dz.float().permute(0, 3, 1, 2), (SH, SW)).permute(0, 2, 3, 1)
    res = []
    for _ in range(2):
        dw = H.padded(torch.zeros(Fo, KH, KW, C, dtype=torch.int64, device=DEV))
        _run_gemm(H.MODE_WGRAD, [dict(a=dz.data_ptr(), b=x.data_ptr(), out=dw.data_ptr(), M=Fo, N=K, K=B * OH * OW,
                                      flags=flags, **geo)], [(Fo, K, B * OH * OW)])
        res.append(dw)
    assert torch.equal(res[0], res[1])
    assert _rel(_q(res[0]), ref_dw) < 2e-5


def test_tiled_fwd_split_k_with_finalize():
    """Merged-Dense FWD with a long reduction: k split over blocks (fp32 partials in a workspace),
    then the grouped finalize (sum of splits + bias + activation) -- the engine's GF_SPLITWS path."""
    torch.cuda.synchronize()
    # N = 148 / 135 / 190: one 160- / 192-column tile; 250: two 128-column tiles
    probs = [(750, 148, 12444, "relu"), (750, 110, 3776, "sigmoid"), (300, 40, 5000, "linear"), (750, 110, 130, "relu"),
             (750, 135, 6944, "relu"), (750, 190, 2100, "sigmoid"), (500, 250, 3000, "linear")]
    rows, dims, refs, outs, keep = [], [], [], [], []
    for M, N, K, act in probs:
        x = H.padded(torch.randn(M, K, device=DEV).bfloat16())
        w = H.padded((torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16())
        b = H.padded(torch.randn(N, device=DEV))
        y = H.padded(torch.zeros(M, N, dtype=torch.bfloat16, device=DEV))
        keep += [x, w, b, y]
        rows.append(dict(a=x.data_ptr(), b=w.data_ptr(), out=y.data_ptr(), bias=b.data_ptr(), H=1, W=1, C=K, OH=1, OW=1,
                         F=N, KH=1, KW=1, SH=1, SW=1, M=M, N=N, K=K, act=H.ACT_CODES[act],
                         flags=H.GF_VEC_A | H.GF_VEC_B if K % 8 == 0 else 0))
        dims.append((M, N, K))
        r = x.float() @ w.float().t() + b
        refs.append({"relu": torch.relu, "sigmoid": torch.sigmoid, "linear": lambda t: t}[act](r))
        outs.append(y)
    plans = H.gemm3_plan(H.MODE_FWD, rows, dims, splitk=True)
    nsplit = 0
    for v, rws, tiles in plans:
        fin = []
        for r in rws:
            ns = int(r.pop("_split", 1))
            if ns > 1:
                nsplit += 1
                wsb = H.padded(torch.full((ns * r["M"] * r["N"],), float("nan"), device=DEV))  # every slot is written
                keep.append(wsb)
                r["aux"] = wsb.data_ptr()
                fin.append(dict(ws=r["aux"], out=r["out"], bias=r["bias"], M=r["M"], N=r["N"], S=ns, act=r["act"]))
        d = _desc(rws, H.GEMM_DTYPE)
        t = torch.as_tensor(tiles, device=DEV)
        H.lib().gemm3(H.MODE_FWD, v, d.data_ptr(), t.data_ptr(), len(t), H.stream_handle())
        if fin:
            fd = _desc(fin, H.SPLITFIN_DTYPE)
            ft = torch.as_tensor(H.chunk_tiles([f["M"] * f["N"] for f in fin], H.SPLITFIN_ELEMS), device=DEV)
            H.lib().splitk_finalize(fd.data_ptr(), ft.data_ptr(), len(ft), H.stream_handle())
    torch.cuda.synchronize()
    assert nsplit >= 3
    assert {v for v, _, _ in plans} & {7160, 7192}          # one shared wide width for the N > 64 group
    for y, r in zip(outs, refs):
        assert _rel(y.float(), r) < 6e-3


@pytest.mark.parametrize("M,N,F,D,col,act", [(750, 300, 152, 300, 0, "relu"), (96, 77, 40, 77, 0, "sigmoid"),
                                               (64, 130, 33, 130, 0, "linear"), (200, 57, 110, 200, 100, "relu"),
                                               (750, 180, 135, 200, 20, "relu")])
def test_tiled_dgrad_natural_weights(M, N, F, D, col, act):
    """Dense DGRAD on the LDS-tiled kernel reading the natural [F][D] weights k-major (BT variant, no
    transposed copy), optionally a column slice [col, col + N) of a wider weight matrix (fused concat),
    with dZ = dY * act'(Y) fused on load."""
    torch.cuda.synchronize()
    dy = H.padded(torch.randn(M, F, device=DEV).bfloat16())
    y = H.padded(torch.randn(M, F, device=DEV).bfloat16())
    if act == "relu":
        y = H.padded(torch.relu(y))
    elif act == "sigmoid":
        y = H.padded(torch.sigmoid(y.float()).bfloat16())
    w = H.padded((torch.randn(F, D, device=DEV) / math.sqrt(F)).bfloat16())
    dx = H.padded(torch.zeros(M, N, dtype=torch.bfloat16, device=DEV))
    row = dict(a=dy.data_ptr(), b=0, _bnat=w.data_ptr() + 2 * col, _bnat_ld=D, aux=y.data_ptr(), act=H.ACT_CODES[act],
               out=dx.data_ptr(), H=1, W=1, C=N, OH=1, OW=1, F=F, KH=1, KW=1, SH=1, SW=1, M=M, N=N, K=F, flags=0)
    plans = H.gemm3_plan(H.MODE_DGRAD, [row], [(M, N, F)])
    assert [v for v, _, _ in plans] == [8000 + H.tiled_bn(N)]
    for v, rws, tiles in plans:
        d = _desc([{k: val for k, val in r.items() if not k.startswith("_")} for r in rws], H.GEMM_DTYPE)
        t = torch.as_tensor(tiles, device=DEV)
        H.lib().gemm3(H.MODE_DGRAD, v, d.data_ptr(), t.data_ptr(), len(t), H.stream_handle())
    torch.cuda.synchronize()
    yf = y.float()
    g = {"relu": (yf > 0).float(), "sigmoid": yf * (1 - yf), "linear": torch.ones_like(yf)}[act]
    ref = (dy.float() * g) @ w.float()[:, col:col + N]
    assert _rel(dx.float(), ref) < 6e-3


def test_transpose_weights_kernel():
    w = H.padded(torch.randn(37, 3, 5, 13, device=DEV).bfloat16())
    out = H.padded(torch.zeros(13, 3, 5, 37, dtype=torch.bfloat16, device=DEV))
    d = _desc([dict(src=w.data_ptr(), dst=out.data_ptr(), F=37, P=15, C=13)], H.TRANS_DTYPE)
    t = torch.as_tensor(H.chunk_tiles([-(-w.numel() // H.TRANS_ELEMS)], 1), device=DEV)
    H.lib().transpose_weights(d.data_ptr(), t.data_ptr(), len(t), H.stream_handle())
    torch.cuda.synchronize()
    assert torch.equal(out, w.permute(3, 1, 2, 0).contiguous())


def test_grouped_gemm_many_problems_one_launch():
    rows, dims, refs, outs = [], [], [], []
    keep = []
    for i, (B, Hh, Ww, C, Fo, KH, KW, SH, SW, act) in enumerate(SHAPES):
        OH, OW = (Hh - KH) // SH + 1, (Ww - KW) // SW + 1
        x = H.padded(torch.randn(B, Hh, Ww, C, device=DEV).bfloat16())
        w = H.padded((torch.randn(Fo, KH, KW, C, device=DEV) / math.sqrt(KH * KW * C)).bfloat16())
        y = H.padded(torch.zeros(B, OH, OW, Fo, dtype=torch.bfloat16, device=DEV))
        keep += [x, w, y]
        K = KH * KW * C
        rows.append(dict(a=x.data_ptr(), b=w.data_ptr(), out=y.data_ptr(), H=Hh, W=Ww, C=C, OH=OH, OW=OW, F=Fo, KH=KH,
                         KW=KW, SH=SH, SW=SW, M=B * OH * OW, N=Fo, K=K, act=0,
                         flags=(H.GF_VEC_A if C % 8 == 0 else 0) | (H.GF_VEC_B if K % 8 == 0 else 0)))
        dims.append((B * OH * OW, Fo, K))
        refs.append(ref_conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, (SH, SW)).permute(0, 2, 3, 1))
        outs.append(y)
    _run_gemm(H.MODE_FWD, rows, dims)
    for y, r in zip(outs, refs):
        assert _rel(y.float(), r) < 6e-3


@pytest.mark.parametrize("RC", [(3000, 13), (20001, 67), (4096, 256), (999, 300), (5000, 1), (3001, 3), (588000, 1),
                                (24576, 1), (96000, 128), (363000, 16)])
def test_bn_train_infer_backward(RC):
    R, C = RC
    x = H.padded((torch.randn(R, C, device=DEV) * 3 + 1).bfloat16())
    gamma = H.padded(torch.rand(C, device=DEV) + 0.5)
    beta = H.padded(torch.randn(C, device=DEV))
    mm, mv = H.padded(torch.zeros(C, device=DEV)), H.padded(torch.ones(C, device=DEV))
    mean, invstd = H.padded(torch.zeros(C, device=DEV)), H.padded(torch.zeros(C, device=DEV))
    ws = H.padded(torch.zeros(H.bn_ws_words(C), dtype=torch.int64, device=DEV))
    y = H.padded(torch.zeros(R, C, dtype=torch.bfloat16, device=DEV))
    dy = H.padded(torch.randn(R, C, device=DEV).bfloat16())
    dx = H.padded(torch.zeros(R, C, dtype=torch.bfloat16, device=DEV))
    dg, db = (H.operand(C, torch.int64, DEV) for _ in range(2))     # Q40 gradient arena
    row = dict(x=x.data_ptr(), y=y.data_ptr(), dy=dy.data_ptr(), dx=dx.data_ptr(), gamma=gamma.data_ptr(),
               beta=beta.data_ptr(), mm=mm.data_ptr(), mv=mv.data_ptr(), mean=mean.data_ptr(), invstd=invstd.data_ptr(),
               ws=ws.data_ptr(), dgamma=dg.data_ptr(), dbeta=db.data_ptr(), R=R, C=C, flags=3, eps=1e-3, momentum=0.99)
    d = _desc([row], H.BN_DTYPE)
    t = torch.as_tensor(H.chunk_tiles([H.bn_chunks(R, C)], 1), device=DEV)
    ts = torch.as_tensor(H.chunk_tiles([H.bn_chunks(R, C, stats=True)], 1), device=DEV)   # phases 0 / 4
    L, s = H.lib(), H.stream_handle()
    L.bn(0, d.data_ptr(), ts.data_ptr(), len(ts), s)
    torch.cuda.synchronize()
    ws0 = H.padded(ws.clone())
    ws.zero_()
    L.bn(0, d.data_ptr(), ts.data_ptr(), len(ts), s)        # statistics again: bitwise identical
    torch.cuda.synchronize()
    assert torch.equal(ws, ws0)
    L.bn(2, d.data_ptr(), t.data_ptr(), len(t), s)
    torch.cuda.synchronize()
    xf = x.float().requires_grad_(True)
    g_ = gamma.clone().requires_grad_(True)
    b_ = beta.clone().requires_grad_(True)
    mu, var = xf.mean(0), xf.var(0, unbiased=False)
    ref = (xf - mu) / torch.sqrt(var + 1e-3) * g_ + b_
    assert _rel(y.float(), ref.detach()) < 6e-3
    assert torch.allclose(mm, 0.01 * mu.detach(), atol=1e-5)
    assert torch.allclose(mv, 0.99 + 0.01 * var.detach() * R / (R - 1.001), atol=1e-4)
    # backward (workspace re-zeroed, as the engine's per-step memset does)
    ws.zero_()
    for ph in (4, 5):
        tt = ts if ph == 4 else t
        L.bn(ph, d.data_ptr(), tt.data_ptr(), len(tt), s)
    torch.cuda.synchronize()
    ref.backward(dy.float())
    assert _rel(dx.float(), xf.grad) < 1e-2
    assert _rel(_q(dg), g_.grad) < 1e-3 and _rel(_q(db), b_.grad) < 1e-3
    # inference
    L.bn(3, d.data_ptr(), t.data_ptr(), len(t), s)
    torch.cuda.synchronize()
    ref_inf = (x.float() - mm) / torch.sqrt(mv + 1e-3) * gamma + beta
    assert _rel(y.float(), ref_inf) < 6e-3


@pytest.mark.parametrize("C", [5, 16])
@pytest.mark.parametrize("p", [(2, 2, 2, 2), (3, 3, 3, 3), (3, 3, 2, 2), (2, 3, 1, 2)])
def test_maxpool_fwd_bwd(p, C, shape=(3, 13, 11)):
    """C=5: element units; C=16: 8-channel vector units (aux.hip pool_vec)."""
    PH, PW, SH, SW = p
    B, Hh, Ww = shape
    OH, OW = (Hh - PH) // SH + 1, (Ww - PW) // SW + 1
    x = H.padded(torch.randn(B, Hh, Ww, C, device=DEV).bfloat16())
    y = H.padded(torch.zeros(B, OH, OW, C, dtype=torch.bfloat16, device=DEV))
    idx = H.padded(torch.zeros(B * OH * OW * C, dtype=torch.uint8, device=DEV))
    dy = H.padded(torch.randn(B, OH, OW, C, device=DEV).bfloat16())
    dx = torch.zeros_like(x)
    row = dict(x=x.data_ptr(), y=y.data_ptr(), idx=idx.data_ptr(), dy=dy.data_ptr(), dx=dx.data_ptr(), B=B, H=Hh, W=Ww,
               C=C, OH=OH, OW=OW, PH=PH, PW=PW, SH=SH, SW=SW, flags=0)
    d = _desc([row], H.POOL_DTYPE)
    L, s = H.lib(), H.stream_handle()
    t = torch.as_tensor(H.chunk_tiles([H.pool_units(B * OH * OW * C, C)], H.POOL_ELEMS), device=DEV)
    L.pool(0, d.data_ptr(), t.data_ptr(), len(t), s)
    t2 = torch.as_tensor(H.chunk_tiles([H.pool_units(B * Hh * Ww * C, C)], H.POOL_ELEMS), device=DEV)
    L.pool(1, d.data_ptr(), t2.data_ptr(), len(t2), s)
    torch.cuda.synchronize()
    xf = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    ref = F.max_pool2d(xf, (PH, PW), (SH, SW))
    assert torch.equal(y.float(), ref.detach().permute(0, 2, 3, 1))
    ref.backward(dy.float().permute(0, 3, 1, 2))
    assert _rel(dx.float(), xf.grad.permute(0, 2, 3, 1)) < 6e-3


@pytest.mark.parametrize("C", [37, 8])
@pytest.mark.parametrize("p", [(2, 2, 2, 2), (3, 3, 2, 2)])
def test_maxpool_large_unit_indices(p, C):
    """~2^24 element units (a batch-750 conv output with an odd filter count): the fp64-reciprocal index math of
    aux.hip's pool kernels stays exact past float32's integer range."""
    test_maxpool_fwd_bwd(p, C, shape=(750, 27, 25))


def test_loss_kernel_matches_keras_losses():
    B, NC, L_ = 50, 10, 100
    z = H.padded(torch.randn(B, NC + L_, device=DEV))
    labels = H.padded(torch.randint(0, NC, (B,), device=DEV, dtype=torch.int32))
    tgt = H.padded(torch.randint(0, 2, (B, L_), device=DEV).bfloat16())
    dz = H.padded(torch.zeros(B, NC + L_, dtype=torch.bfloat16, device=DEV))
    metrics = H.padded(torch.zeros(4, dtype=torch.int64, device=DEV))  # Q32 fixed point
    lb = 0.3
    row = dict(logits=z.data_ptr(), dlogits=dz.data_ptr(), labels=labels.data_ptr(), target=tgt.data_ptr(),
               metrics=metrics.data_ptr(), NC=NC, L=L_, B=B, lb=lb)
    d = _desc([row], H.LOSS_DTYPE)
    H.lib().loss(1, d.data_ptr(), 1, B, H.stream_handle(), B)
    torch.cuda.synchronize()
    zz = z.clone().requires_grad_(True)
    ce = F.cross_entropy(zz[:, :NC], labels.long())
    mse = ((torch.sigmoid(zz[:, NC:]) - tgt.float()) ** 2).mean()
    loss = lb * ce + (1 - lb) * mse
    loss.backward()
    assert _rel(dz.float(), zz.grad) < 6e-3
    m = torch.as_tensor(H.from_q32(metrics))      # the metrics stay Q32 (common.h fxm_add)
    assert abs(m[0].item() / B - loss.item()) < 1e-4
    assert m[1].item() == (zz[:, :NC].argmax(1) == labels.long()).sum().item()
    assert abs(m[2].item() / B - mse.item()) < 1e-5


@pytest.mark.parametrize("shape", [(3, 9, 9, 8, 13, 3, 3), (3, 9, 9, 2, 13, 1, 1), (50, 12, 12, 1, 70, 1, 1),
                                   # small-bank WGRAD (g3_wgrad_tiny_kernel: F <= 16, N = 9 / 25 / 49 columns, as the
                                   # first layers over an im2col matrix), odd row widths and F = 13
                                   (40, 16, 16, 9, 16, 1, 1), (30, 14, 14, 25, 13, 1, 1), (20, 20, 20, 49, 8, 1, 1)])
@pytest.mark.parametrize("act", ["relu", "sigmoid"])
def test_fused_act_grad_and_bias_grad(act, shape):
    """WGRAD/DGRAD apply dZ = dY * act'(Y) on load; WGRAD also reduces the bias gradient
    (1x1 shapes with C <= 4 take the narrow VALU kernels)."""
    B, Hh, Ww, C, Fo, KH, KW = shape
    SH = SW = 1
    OH, OW = Hh - KH + 1, Ww - KW + 1
    x = H.padded(torch.randn(B, Hh, Ww, C, device=DEV).bfloat16())
    w = H.padded((torch.randn(Fo, KH, KW, C, device=DEV) / 6).bfloat16())
    ypre = H.padded(torch.randn(B, OH, OW, Fo, device=DEV))
    y = H.padded((torch.relu(ypre) if act == "relu" else torch.sigmoid(ypre)).bfloat16())
    dy = H.padded(torch.randn(B, OH, OW, Fo, device=DEV).bfloat16())
    yf = y.float()
    dz = dy.float() * ((yf > 0).float() if act == "relu" else yf * (1 - yf))
    dz = dz.bfloat16().float()
    geo = dict(H=Hh, W=Ww, C=C, OH=OH, OW=OW, F=Fo, KH=KH, KW=KW, SH=SH, SW=SW)
    K = KH * KW * C
    dw = H.padded(torch.zeros(Fo, KH, KW, C, dtype=torch.int64, device=DEV))
    db = H.padded(torch.zeros(Fo, dtype=torch.int64, device=DEV))
    _run_gemm(H.MODE_WGRAD, [dict(a=dy.data_ptr(), b=x.data_ptr(), out=dw.data_ptr(), bias=db.data_ptr(),
                                  aux=y.data_ptr(), act=H.ACT_CODES[act], M=Fo, N=K, K=B * OH * OW, **geo)],
              [(Fo, K, B * OH * OW)])
    dw, db = _q(dw), _q(db)
    xr = x.float().permute(0, 3, 1, 2)
    wr = w.float().permute(0, 3, 1, 2)
    ref_dw = ref_conv2d_weight(xr, wr.shape, dz.permute(0, 3, 1, 2), (SH, SW)).permute(0, 2, 3, 1)
    assert _rel(dw, ref_dw) < 1e-3
    assert _rel(db, dz.sum((0, 1, 2))) < 1e-3
    dx = H.padded(torch.zeros(B, Hh, Ww, C, dtype=torch.bfloat16, device=DEV))
    wt = H.padded(w.permute(3, 1, 2, 0).contiguous())
    _run_gemm(H.MODE_DGRAD, [dict(a=dy.data_ptr(), b=wt.data_ptr(), _bnat=w.data_ptr(), out=dx.data_ptr(),
                                  aux=y.data_ptr(), act=H.ACT_CODES[act], M=B * Hh * Ww, N=C, K=KH * KW * Fo, **geo)],
              [(B * Hh * Ww, C, KH * KW * Fo)])
    ref_dx = ref_conv2d_input(xr.shape, wr, dz.permute(0, 3, 1, 2), (SH, SW)).permute(0, 2, 3, 1)
    assert _rel(dx.float(), ref_dx) < 6e-3


def test_wave_split_k_dense():
    """Few rows, long K (the Dense-on-merge shape): the wave-split-K form must match."""
    M, K, N = 750, 5003, 110
    x = H.padded(torch.randn(M, K, device=DEV).bfloat16())
    w = H.padded((torch.randn(N, K, device=DEV) / 70).bfloat16())
    b = H.padded(torch.randn(N, device=DEV))
    y = H.padded(torch.zeros(M, N, device=DEV))
    geo = dict(H=1, W=1, C=K, OH=1, OW=1, F=N, KH=1, KW=1, SH=1, SW=1)
    assert 100 <= H.gemm3_variant(H.MODE_FWD, M, N, K, geo) % 1000
    _run_gemm(H.MODE_FWD, [dict(a=x.data_ptr(), b=w.data_ptr(), out=y.data_ptr(), bias=b.data_ptr(), M=M, N=N, K=K,
                                flags=H.GF_OUT_F32, **geo)],
              [(M, N, K)])
    assert _rel(y, x.float() @ w.float().t() + b) < 1e-4


@pytest.mark.parametrize("shape", [(4, 12, 12, 16, 32, 3, 3, 1, 1), (3, 1, 1, 200, 37, 1, 1, 1, 1),
                                   (40, 10, 10, 24, 64, 1, 1, 1, 1)])
def test_v3_accumulating_outputs(shape):
    """GF_ACCUM (a tensor with several consumers): DGRAD and FWD add into the existing bf16 output,
    through both the coalesced LDS-staged epilogue and the scattered one."""
    B, Hh, Ww, C, Fo, KH, KW, SH, SW = shape
    OH, OW = (Hh - KH) // SH + 1, (Ww - KW) // SW + 1
    x = H.padded(torch.randn(B, Hh, Ww, C, device=DEV).bfloat16())
    w = H.padded((torch.randn(Fo, KH, KW, C, device=DEV) / math.sqrt(KH * KW * C)).bfloat16())
    dz = H.padded(torch.randn(B, OH, OW, Fo, device=DEV).bfloat16())
    xr, wr = x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2)
    geo = dict(H=Hh, W=Ww, C=C, OH=OH, OW=OW, F=Fo, KH=KH, KW=KW, SH=SH, SW=SW)
    prev = H.padded(torch.randn(B, Hh, Ww, C, device=DEV).bfloat16())
    dx = H.padded(prev.clone())
    wt = H.padded(w.permute(3, 1, 2, 0).contiguous())
    _run_gemm(H.MODE_DGRAD, [dict(a=dz.data_ptr(), b=wt.data_ptr(), out=dx.data_ptr(), M=B * Hh * Ww, N=C,
                                  K=KH * KW * Fo, flags=H.GF_ACCUM, **geo)], [(B * Hh * Ww, C, KH * KW * Fo)])
    ref = prev.float() + ref_conv2d_input(xr.shape, wr, dz.float().permute(0, 3, 1, 2), (SH, SW)).permute(0, 2, 3, 1)
    assert _rel(dx.float(), ref) < 6e-3
    prev_y = H.padded(torch.randn(B, OH, OW, Fo, device=DEV).bfloat16())
    y = H.padded(prev_y.clone())
    _run_gemm(H.MODE_FWD, [dict(a=x.data_ptr(), b=w.data_ptr(), out=y.data_ptr(), M=B * OH * OW, N=Fo,
                                K=KH * KW * C, flags=H.GF_ACCUM, **geo)], [(B * OH * OW, Fo, KH * KW * C)])
    ref_y = prev_y.float() + ref_conv2d(xr, wr, None, (SH, SW)).permute(0, 2, 3, 1)
    assert _rel(y.float(), ref_y) < 6e-3


def _ew_run(rows):
    d = _desc(rows, H.EW_DTYPE)
    t = torch.as_tensor(H.chunk_tiles([H.ew_count(r) for r in rows], 1), device=DEV)
    H.lib().ew(d.data_ptr(), t.data_ptr(), len(t), H.stream_handle())
    torch.cuda.synchronize()


def test_ew_map_reduce_permute():
    """ew.hip (rare ops: neg / broadcasting sub / non-last-axis BatchNormalization transposes) against
    torch: a broadcast binary map, the gradient reduction of each broadcast operand (with accumulate), and
    the [outer][C][inner] -> [outer][inner][C] permutation."""
    g = torch.Generator(device=DEV).manual_seed(3)
    sa, sb = (5, 6, 1, 7), (5, 1, 3, 1)
    out_shape = (5, 6, 3, 7)
    a = H.padded(torch.randn(sa, device=DEV, generator=g).bfloat16())
    b = H.padded(torch.randn(sb, device=DEV, generator=g).bfloat16())
    y = H.operand(out_shape, torch.bfloat16, DEV)
    _ew_run([H.ew_map_row(y.data_ptr(), out_shape, a.data_ptr(), sa, ca=1.0, b=b.data_ptr(), b_shape=sb, cb=-1.0, c=0.5)])
    ref = a.float() - b.float() + 0.5
    assert _rel(y.float(), ref) < 6e-3
    # d/da of (a - b) broadcast: sum over the broadcast axis, accumulated onto an existing gradient
    dy = H.padded(torch.randn(out_shape, device=DEV, generator=g).bfloat16())
    prev = torch.randn(sa, device=DEV, generator=g).bfloat16()
    da = H.padded(prev.clone())
    db = H.operand(sb, torch.bfloat16, DEV)
    _ew_run([H.ew_reduce_row(da.data_ptr(), sa, dy.data_ptr(), out_shape, 1.0, accum=True),
             H.ew_reduce_row(db.data_ptr(), sb, dy.data_ptr(), out_shape, -1.0)])
    assert _rel(da.float(), prev.float() + dy.float().sum(2, keepdim=True)) < 6e-3
    assert _rel(db.float(), -dy.float().sum((1, 3), keepdim=True)) < 6e-3
    # neg and the channels-last permutation of a BN over axis 1 of (B, C, H, W)
    x = H.padded(torch.randn(4, 9, 5, 3, device=DEV, generator=g).bfloat16())
    xt = H.operand(4 * 5 * 3 * 9, torch.bfloat16, DEV)
    _ew_run([H.ew_permute_row(xt.data_ptr(), x.data_ptr(), (4, 9, 15), (0, 2, 1))])
    assert torch.equal(xt.view(4, 15, 9), x.view(4, 9, 15).permute(0, 2, 1))
    n = H.operand((4, 9, 5, 3), torch.bfloat16, DEV)
    _ew_run([H.ew_map_row(n.data_ptr(), (4, 9, 5, 3), x.data_ptr(), (4, 9, 5, 3), ca=-1.0)])
    assert torch.equal(n, -x)


@pytest.mark.parametrize("F,N", [(146, 300), (95, 1504), (190, 77), (118, 64)])
def test_wide_f_dense_wgrad(F, N, monkeypatch):
    """Whole-F WGRAD tiles (hip_ops.WGRAD_WIDE: BMF 96..192 x 64) on batch-750 Dense problems: Q40 gradient
    and bias gradient against fp32, single split (plain store), bitwise repeatable."""
    monkeypatch.setattr(H, "WGRAD_WIDE", True)
    M = 750
    g = torch.Generator(device=DEV).manual_seed(5)
    x = H.padded(torch.randn(M, N, device=DEV, generator=g).bfloat16())
    dz = H.padded(torch.randn(M, F, device=DEV, generator=g).bfloat16())
    geo = dict(H=1, W=1, C=N, OH=1, OW=1, F=F, KH=1, KW=1, SH=1, SW=1)
    row = dict(a=dz.data_ptr(), b=x.data_ptr(), M=F, N=N, K=M, flags=H.GF_VEC_A if F % 8 == 0 else 0, **geo)
    plans = H.gemm3_plan(H.MODE_WGRAD, [dict(row)], [(F, N, M)])
    assert plans[0][0] % 1000000 // 1000 >= 96, plans[0][0]
    res = []
    for _ in range(2):
        dw = H.operand((F, N), torch.int64, DEV)
        db = H.operand(F, torch.int64, DEV)
        _run_gemm(H.MODE_WGRAD, [dict(row, out=dw.data_ptr(), bias=db.data_ptr())], [(F, N, M)])
        res.append((dw.clone(), db.clone()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    ref = dz.float().t() @ x.float()
    assert _rel(_q(res[0][0]), ref) < 2e-5
    assert _rel(_q(res[0][1]), dz.float().sum(0)) < 1e-5


def test_small_gradients_reach_adam_unquantised():
    """Gradients of 1e-10 .. 1e-8 (the RiboAE's dead embedding / Dense tail under Keras' eps = 1e-7 Adam):
    a Dense WGRAD writes them into the fixed-point gradient arena and the arena Adam applies them; every
    update matches fp32 Adam on the exact gradient of the same bf16 operands within 1 %.  (The round-4 Q32
    arena, 2^-32 = 2.3e-10 units, is off by up to 100 % here -- checked below on the same gradients.)"""
    torch.cuda.synchronize()
    F_, C_, B_ = 16, 64, 256
    g = torch.Generator(device=DEV).manual_seed(5)
    dz = H.padded((torch.randn(B_, F_, device=DEV, generator=g) * 4e-5).bfloat16())
    scale = torch.logspace(-6, -4, C_, device=DEV)                 # column scales: |dW| spans ~1e-10 .. 1e-8
    x = H.padded((torch.randn(B_, C_, device=DEV, generator=g) * scale / math.sqrt(B_)).bfloat16())
    ref_g = (dz.double().t() @ x.double()).float()                 # exact gradient of the bf16 operands
    absg = ref_g.abs()
    assert float(absg.min()) < 1e-10 and float(absg.max()) > 5e-9
    dw = H.padded(torch.zeros(F_, C_, dtype=torch.int64, device=DEV))
    geo = dict(H=1, W=1, C=C_, OH=1, OW=1, F=F_, KH=1, KW=1, SH=1, SW=1)
    _run_gemm(H.MODE_WGRAD, [dict(a=dz.data_ptr(), b=x.data_ptr(), out=dw.data_ptr(), M=F_, N=C_, K=B_,
                                  flags=H.GF_VEC_A | H.GF_VEC_B, **geo)], [(F_, C_, B_)])
    n = F_ * C_
    p = H.padded(torch.randn(n, device=DEV, generator=g) * 1e-6)   # small: p's fp32 rounding stays << the update
    p0 = p.clone()
    m, v = H.padded(torch.zeros(n, device=DEV)), H.padded(torch.zeros(n, device=DEV))
    pbf = H.padded(torch.zeros(n, dtype=torch.bfloat16, device=DEV))
    step = torch.zeros(1, dtype=torch.int32, device=DEV)
    lr_t = torch.zeros(1, device=DEV)
    lr, eps = 1e-3, 1e-7
    H.lib().adam(p.data_ptr(), dw.data_ptr(), m.data_ptr(), v.data_ptr(), pbf.data_ptr(), step.data_ptr(),
                 lr_t.data_ptr(), n, lr, 0.9, 0.999, eps, H.stream_handle())
    torch.cuda.synchronize()

    def adam_update(gr):
        gr = gr.double().reshape(-1)
        lr1 = lr * (1 - 0.999) ** 0.5 / (1 - 0.9)
        return lr1 * (0.1 * gr) / ((0.001 * gr * gr).sqrt() + eps)

    want = adam_update(ref_g)
    got = (p0.double() - p.double())[:n]
    big = ref_g.reshape(-1).double().abs() >= 1e-10
    assert int(big.sum()) > n // 2
    rel = ((got - want).abs() / want.abs().clamp_min(1e-30))[big]
    tol = 0.01 * want.abs()[big] + 1e-12
    assert bool(((got - want).abs()[big] <= tol).all()), float(rel.max())
    q32 = torch.round(ref_g.double() * 2.0 ** 32) / 2.0 ** 32
    q32_err = ((adam_update(q32) - want).abs() / want.abs().clamp_min(1e-30))[big]
    assert float(q32_err.max()) > 0.2          # the test discriminates: the Q32 arena fails it


@pytest.mark.parametrize("F,C,rows,act", [(16, 264, 750, "linear"), (24, 96, 750, "relu"), (64, 64, 20000, "sigmoid"),
                                          (120, 200, 3000, "linear"), (8, 64, 100, "relu"), (40, 128, 75000, "linear"),
                                          (64, 136, 750, "linear"), (32, 72, 4100, "sigmoid"),
                                          (152, 8284, 750, "linear"), (64, 100, 3000, "relu")])
def test_dma_dense_wgrad(F, C, rows, act, monkeypatch):
    """The LDS-DMA ring Dense WGRAD (gemm3.hip g3_dwgrad_kernel): every (BMF, BNK) instantiation with and without
    the staged Y tile (act' on the A fragments), ragged f / column tiles and 64-row steps, single split (plain
    store) and m-splits (fixed-point atomics); gradient and bias gradient against fp32, bitwise repeatable."""
    monkeypatch.setattr(H, "DWGRAD", True)                  # (off by default: hip_ops.DWGRAD)
    monkeypatch.setattr(H, "DWGRAD_CALIGN", 4)              # X rows 8-B aligned (C % 4 == 0) allowed
    g = torch.Generator(device=DEV).manual_seed(11)
    x = H.padded(torch.randn(rows, C, device=DEV, generator=g).bfloat16())
    dy = H.padded(torch.randn(rows, F, device=DEV, generator=g).bfloat16())
    ypre = torch.randn(rows, F, device=DEV, generator=g)
    y = H.padded((torch.relu(ypre) if act == "relu" else torch.sigmoid(ypre)).bfloat16())
    yf = y.float()
    dz = dy.float() * {"relu": (yf > 0).float(), "sigmoid": yf * (1 - yf), "linear": torch.ones_like(yf)}[act]
    dz = dz.bfloat16().float()
    geo = dict(H=1, W=1, C=C, OH=1, OW=1, F=F, KH=1, KW=1, SH=1, SW=1)
    row = dict(a=dy.data_ptr(), b=x.data_ptr(), aux=y.data_ptr() if act != "linear" else 0, act=H.ACT_CODES[act],
               M=F, N=C, K=rows, flags=H.GF_VEC_A | H.GF_VEC_B, **geo)
    plans = H.gemm3_plan(H.MODE_WGRAD, [dict(row)], [(F, C, rows)])
    assert len(plans) == 1 and plans[0][0] >= 5000000, plans[0][0]
    assert (plans[0][0] % 1000 >= 500) == (act != "linear")
    res = []
    for _ in range(2):
        dw = H.operand((F, C), torch.int64, DEV)
        db = H.operand(F, torch.int64, DEV)
        dw.zero_()
        db.zero_()
        _run_gemm(H.MODE_WGRAD, [dict(row, out=dw.data_ptr(), bias=db.data_ptr())], [(F, C, rows)])
        res.append((dw.clone(), db.clone()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    ref = dz.double().t() @ x.double()
    assert _rel(_q(res[0][0]), ref.float()) < 2e-5
    assert _rel(_q(res[0][1]), dz.double().sum(0).float()) < 1e-5


@pytest.mark.parametrize("shape", [
    (4, 12, 12, 16, 32, 3, 3, "relu"),        # conv-halo FWD
    (3, 9, 7, 64, 24, 1, 1, "sigmoid"),       # 1x1, K = 64: LDS-tiled FWD
    (5, 6, 6, 16, 40, 1, 1, "linear"),        # 1x1, K = 16: single-step direct FWD
    (2, 13, 13, 13, 20, 3, 3, "linear"),      # odd channels, conv-halo
    (6, 10, 10, 8, 70, 3, 3, "relu"),         # several column tiles
])
def test_fwd_epilogue_bn_statistics(shape):
    """GF_BNUSTAT: the FWD epilogue (conv-halo, LDS-tiled, direct kernels) accumulates sum y and sum y^2 of its stored
    bf16 outputs per channel into a BatchNorm statistics workspace (wide fixed point, BN_WS_STRIPES copies) -- what
    BN phase 2 reads with flag 512 -- and the output itself is unchanged."""
    B, Hh, Ww, C, Fo, KH, KW, act = shape
    OH, OW = Hh - KH + 1, Ww - KW + 1
    g = torch.Generator(device=DEV).manual_seed(4)
    x = H.padded(torch.randn(B, Hh, Ww, C, device=DEV, generator=g).bfloat16())
    w = H.padded((torch.randn(Fo, KH, KW, C, device=DEV, generator=g) / math.sqrt(KH * KW * C)).bfloat16())
    bias = H.padded(torch.randn(Fo, device=DEV, generator=g) + 2.0)      # |mean| >> std: no cancellation either
    M, K = B * OH * OW, KH * KW * C
    geo = dict(H=Hh, W=Ww, C=C, OH=OH, OW=OW, F=Fo, KH=KH, KW=KW, SH=1, SW=1)
    flags = (H.GF_VEC_A if C % 8 == 0 else 0) | (H.GF_VEC_B if K % 8 == 0 else 0)
    row = dict(a=x.data_ptr(), b=w.data_ptr(), bias=bias.data_ptr(), M=M, N=Fo, K=K, act=H.ACT_CODES[act], **geo)
    assert H.fwd_bnustat_ok(dict(row, flags=flags), M, Fo, K)
    outs = []
    for extra in (0, H.GF_BNUSTAT):
        y = H.padded(torch.zeros(B, OH, OW, Fo, dtype=torch.bfloat16, device=DEV))
        ws = H.operand(H.bn_ws_words(Fo), torch.int64, DEV)
        ws.zero_()
        _run_gemm(H.MODE_FWD, [dict(row, out=y.data_ptr(), aux=ws.data_ptr() if extra else 0, flags=flags | extra)],
                  [(M, Fo, K)])
        outs.append((y.clone(), ws.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    yv = outs[1][0].double().reshape(M, Fo)
    w4 = outs[1][1][:H.bn_ws_words(Fo)].reshape(H.BN_WS_STRIPES, 2 * Fo, 2).cpu()
    sums = (w4[..., 0].double() + w4[..., 1].double() / 2.0 ** 32).sum(0)
    torch.testing.assert_close(sums[:Fo], yv.sum(0).cpu(), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(sums[Fo:], (yv * yv).sum(0).cpu(), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("geom", [(28, 28, 5, 5, 1), (28, 28, 3, 3, 2), (28, 28, 7, 7, 1), (24, 20, 9, 9, 1),
                                  (100, 1, 5, 1, 1)])
def test_shared_input_fwd_many_filter_banks(geom, monkeypatch):
    """g3_shared_fwd_kernel: first layers of several organisms over ONE im2col matrix of the shared input batch
    (filter banks of 8 - 60 filters, mixed activations, BN statistics in the epilogue for some): each output
    against the fp32 convolution, the statistics against the stored outputs, and bitwise against the same
    problems run one by one on the unshared kernels (direct single-step / LDS-tiled)."""
    Hh, Ww, KH, KW, S = geom
    B = 40
    OH, OW = (Hh - KH) // S + 1, (Ww - KW) // S + 1
    M, K = B * OH * OW, KH * KW
    K8 = -(-K // 8) * 8
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(B, 1, Hh, Ww, device=DEV, generator=g).bfloat16()
    cols = F.unfold(x.float().cpu(), (KH, KW), stride=S)                 # [B, K, OH*OW], taps (kh, kw)
    A = torch.zeros(M, K8)
    A[:, :K] = cols.permute(0, 2, 1).reshape(M, K)
    A = H.padded(A.to(DEV).bfloat16())
    banks = [(16, "relu", True), (8, "linear", False), (32, "sigmoid", True), (13, "relu", False), (60, "linear", True)]
    ws_, bs_, rows = [], [], []
    for Fo, act, stat in banks:
        w = H.padded((torch.randn(Fo, K, device=DEV, generator=g) / math.sqrt(K)).bfloat16())
        b = H.padded(torch.randn(Fo, device=DEV, generator=g) * 0.3)
        ws_.append(w)
        bs_.append(b)
        rows.append(dict(a=A.data_ptr(), b=w.data_ptr(), bias=b.data_ptr(), M=M, N=Fo, K=K, C=K8, H=OH, W=OW, OH=OH,
                         OW=OW, F=Fo, KH=1, KW=1, SH=1, SW=1, act=H.ACT_CODES[act], flags=H.GF_BNUSTAT if stat else 0,
                         _imcol=1))
    results = []
    for off in (set(), {"shared"}):
        monkeypatch.setattr(H, "_OFF", off)
        plans = H.gemm3_plan(H.MODE_FWD, [dict(r) for r in rows], [(M, r["N"], K) for r in rows])
        assert any(5100 < v < 5200 for v, _, _ in plans) == (not off)
        outs = []
        for r in rows:
            y = H.padded(torch.zeros(M, r["N"], dtype=torch.bfloat16, device=DEV))
            wsb = H.operand(H.bn_ws_words(r["N"]), torch.int64, DEV)
            wsb.zero_()
            outs.append((y, wsb))
        run = [dict(r, out=y.data_ptr(), aux=wsb.data_ptr() if r["flags"] else 0) for r, (y, wsb) in zip(rows, outs)]
        if off:
            for r in run:                                  # one by one on the usual kernels (outputs only)
                _run_gemm(H.MODE_FWD, [dict(r, flags=0, aux=0)], [(M, r["N"], K)])
        else:
            _run_gemm(H.MODE_FWD, run, [(M, r["N"], K) for r in run])
        results.append(outs)
    for i, ((Fo, act, stat), w, b) in enumerate(zip(banks, ws_, bs_)):
        y, wsb = results[0][i]
        ref = ref_conv2d(x, w.view(Fo, 1, KH, KW), b, S)                    # [B, F, OH, OW]
        ref = {"relu": torch.relu, "sigmoid": torch.sigmoid, "linear": lambda t: t}[act](ref)
        got = y.view(B, OH, OW, Fo).permute(0, 3, 1, 2).float()
        assert _rel(got, ref) < 6e-3, (i, _rel(got, ref))
        assert torch.equal(y, results[1][i][0]), f"bank {i}: shared and unshared outputs differ"
        if stat:
            yv = y.double()
            w4 = wsb[:H.bn_ws_words(Fo)].reshape(H.BN_WS_STRIPES, 2 * Fo, 2).cpu()
            sums = (w4[..., 0].double() + w4[..., 1].double() / 2.0 ** 32).sum(0)
            torch.testing.assert_close(sums[:Fo], yv.sum(0).cpu(), rtol=1e-5, atol=1e-3)
            torch.testing.assert_close(sums[Fo:], (yv * yv).sum(0).cpu(), rtol=1e-5, atol=1e-3)
