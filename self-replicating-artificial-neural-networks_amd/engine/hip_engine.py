"""HIP grouped population engine (MI355X / gfx950).

A shard of P heterogeneous organisms is compiled into a *plan*: per dependency level, one grouped
launch per op kind covering every organism (grouped implicit-GEMM for Dense/Conv2D/Conv1D/heads,
fused BatchNormalizationF16, MaxPool, concat copies), one fused heads-loss launch, the mirrored
backward levels, and one fused Keras-Adam launch over a flat fp32 parameter arena.  Architectures
are fixed for a whole generation, so the training step is captured once into a HIP graph and
replayed for every one of the ~380 steps (no host work inside the training loop).

Memory (288 GB HBM per MI355X): bf16 activations and activation-gradients for every node at the
training batch (aliased for reshapes), fp32 master weights + Adam moments + gradients in one arena,
bf16 compute copy refreshed by the Adam kernel, device-resident datasets (bf16).

Weights use the output-major layout ``Wm[F][KH][KW][C]`` (the forward GEMM's B operand is then
k-contiguous); the two heads of an organism are stored adjacently as one ``[NC+L][D]`` matrix so
they run as a single GEMM with an fp32 output.

Rare ops reachable only by mutation (unary / binary minus with broadcasting, BatchNormalization on a
non-last axis) run on the strided elementwise kernel (csrc/hip/ew.hip): maps, broadcast-gradient
reductions and the [outer][C][inner] <-> [outer][inner][C] transposes around the channels-last BN
kernels -- no host-driven torch op anywhere in a plan.
"""
from __future__ import annotations

import os
import math
import threading
import time
import weakref
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..experiment.cost_model import organism_time
from ..genome.ir import Node, OrganismIR
from ..models.organism import glorot_limit, init_params
from ..ops import hip_ops as H
from .base import FitResult, PopulationEngine, TrainConfig, epoch_permutation

import os

ALIGN = 16  # elements; keeps every buffer 32-B aligned for bf16 and 64-B for fp32
SLACK = 64  # elements of zeroed tail on every arena
FUSE_BN_STATS = os.environ.get("SERANN_FUSE_BN_STATS", "1") != "0"
# BN phase-0 statistics in the producing conv-halo / direct / LDS-tiled FWD epilogue (GF_BNUSTAT, round 5)
FUSE_BN_USTATS = os.environ.get("SERANN_FUSE_BN_USTATS", "1") != "0"
FUSE_CONVPOOL = os.environ.get("SERANN_FUSE_CONVPOOL", "1") != "0"
FUSE_GCHAIN = os.environ.get("SERANN_FUSE_GCHAIN", "1") != "0"


def convpool_pairs(ir: OrganismIR) -> Dict[int, int]:
    """Conv2D nodes on the raw single-channel image whose only consumer is a MaxPool2D: conv id -> pool
    id.  Such a pair runs as one fused kernel (csrc/hip/convpool.hip) and the conv output -- and its
    gradient -- is never materialised (SERANN_FUSE_CONVPOOL=0 turns it off)."""
    if not FUSE_CONVPOOL:
        return {}
    consumers: Dict[int, List[int]] = {}
    for n in ir.nodes:
        for i in n.inputs:
            consumers.setdefault(i, []).append(n.id)
    out = {}
    for n in ir.nodes:
        if n.op != "gemm" or n.attrs["kind"] != "conv2d":
            continue
        a = n.attrs
        src = ir.node(n.inputs[0])
        if src.op != "input" or a["cin"] != 1 or a["act"] not in H.ACT_CODES:
            continue
        cons = consumers.get(n.id, [])
        if len(cons) != 1 or ir.node(cons[0]).op != "pool" or ir.cls_head == n.id:
            continue
        pa = ir.node(cons[0]).attrs
        if pa["c"] != a["f"] or pa["h"] != a["oh"] or pa["w"] != a["ow"]:
            continue
        if not H.convpool_ok(a["h"], a["w"], a["kh"], a["kw"], pa["ph"], pa["pw"]):
            continue
        out[n.id] = cons[0]
    return out


def gchain_triples(ir: OrganismIR) -> Dict[int, Tuple[int, int, Optional[int]]]:
    """Replication-branch chains ``Conv1D(raw genotype) -> Dense -> [BatchNormalization]`` run by the
    fused kernels of csrc/hip/gchain.hip: last node id -> (conv id, dense id, BN id or None).

    Eligible: a Conv1D on the raw single-channel genotype whose only consumer is a Dense on its output
    (<= 16 taps and a gchain_variant for the filter / unit counts); the BatchNormalization joins when it
    is the Dense's only consumer and normalises its last axis.  The conv output -- and, with the BN, the
    Dense output -- and their gradients are never materialised (SERANN_FUSE_GCHAIN=0 turns it off)."""
    if not FUSE_GCHAIN:
        return {}
    consumers: Dict[int, List[int]] = {}
    for n in ir.nodes:
        for i in n.inputs:
            consumers.setdefault(i, []).append(n.id)
    out = {}
    for n in ir.nodes:
        if n.op != "gemm" or n.attrs["kind"] != "conv1d":
            continue
        a = n.attrs
        src = ir.node(n.inputs[0])
        if src.op != "input" or a["cin"] != 1 or a["w"] != 1 or a["kw"] != 1 or a["act"] not in H.ACT_CODES:
            continue
        cons = consumers.get(n.id, [])
        if len(cons) != 1:
            continue
        dn = ir.node(cons[0])
        if dn.op != "gemm" or dn.attrs["kind"] != "dense" or list(dn.inputs) != [n.id]:
            continue
        da = dn.attrs
        if (da["cin"] != a["f"] or da["h"] != a["oh"] or da["w"] != 1 or da["act"] not in H.ACT_CODES
                or H.gchain_variant(a["f"], da["f"], a["kh"]) is None or not H.gchain_fits(a["oh"], a["h"])):
            continue
        bn = None
        dc = consumers.get(dn.id, [])
        if len(dc) == 1:
            b = ir.node(dc[0])
            if b.op == "bn" and b.attrs["last"] and b.attrs["channels"] == da["f"]:
                bn = b.id
        out[bn if bn is not None else dn.id] = (n.id, dn.id, bn)
    return out


FUSE_NBN = os.environ.get("SERANN_FUSE_NBN", "1") != "0"
# binary-genotype factorisation of raw-genotype Dense -> BN pairs read by a merged-Dense K slice (csrc/hip/bnbn.hip)
BINARY_NBN = os.environ.get("SERANN_BINARY_NBN", "1") != "0"
BIN_VEC4 = os.environ.get("SERANN_BIN_VEC4", "1") != "0"
BIN_SW_BLOCKS = int(os.environ.get("SERANN_BIN_SW_BLOCKS", "1024"))   # row-split target of a bin_sw launch
# fused pairs whose BN output feeds one LDS-tiled DGRAD: BN backward sums in that DGRAD's epilogue (nbn phase 6)
NBN_SUM = os.environ.get("SERANN_NBNSUM", "1") != "0"


def nbn_pairs(ir: OrganismIR) -> Dict[int, int]:
    """Raw-input Dense -> BatchNormalization pairs fused in training plans (csrc/hip/nbn.hip): BN id ->
    Dense id.  Eligible: a Dense with K <= 4 input channels on a raw input (the genotype or the image:
    no DGRAD), 8 <= units <= 256, whose only consumer is a last-axis BatchNormalization of its units; the
    Dense then runs as the narrow statistics-only kernel and its output -- and its gradient -- is never
    materialised in training (SERANN_FUSE_NBN=0 turns it off)."""
    if not (FUSE_NBN and FUSE_BN_STATS) or "narrow" in H._OFF:
        return {}
    consumers: Dict[int, List[int]] = {}
    for n in ir.nodes:
        for i in n.inputs:
            consumers.setdefault(i, []).append(n.id)
    out = {}
    for b in ir.nodes:
        if b.op != "bn" or not b.attrs["last"]:
            continue
        n = ir.node(b.inputs[0])
        if n.op != "gemm" or n.attrs["kind"] != "dense" or ir.cls_head == n.id:
            continue
        a = n.attrs
        if (a["kh"] * a["kw"] != 1 or a["sh"] * a["sw"] != 1 or a["cin"] > 4 or not 8 <= a["f"] <= 256
                or a["f"] != b.attrs["channels"] or a["act"] not in H.ACT_CODES):
            continue
        if ir.node(n.inputs[0]).op != "input" or consumers.get(n.id, []) != [b.id]:
            continue
        out[b.id] = n.id
    return out


class _Deferred:
    """A device address inside a buffer allocated later: element offset ``off`` (int64 words) plus a byte delta."""

    def __init__(self, off: int, delta: int = 0):
        self.off, self.delta = int(off), int(delta)

    def __add__(self, nbytes: int) -> "_Deferred":
        return _Deferred(self.off, self.delta + int(nbytes))

    def resolve(self, base: int) -> int:
        return int(base) + 8 * self.off + self.delta


def _is_binary(a) -> bool:
    """True when every element of the genotype array ``a`` is 0 or 1 (the factorised genotype-slice path's
    precondition; the reference's genotypes always are)."""
    arr = np.asarray(a)
    return bool(arr.size) and bool(np.all((arr == 0) | (arr == 1)))


def _padded_zeros(shape, dtype, device) -> torch.Tensor:
    """Zeroed tensor followed by SLACK zeroed elements (GEMM fragment loads may over-read)."""
    n = math.prod(shape)
    return torch.zeros(n + SLACK, dtype=dtype, device=device)[:n].view(shape)


def _al(n: int) -> int:
    return (int(n) + ALIGN - 1) // ALIGN * ALIGN


# split WGRADs' ordered finalize applies Adam to the weights it writes (SERANN_FINALIZE_ADAM=0: the arena pass does)
FINALIZE_ADAM = os.environ.get("SERANN_FINALIZE_ADAM", "1") != "0"


class Arena:
    """Bump allocator over one device tensor."""

    def __init__(self, dtype, device):
        self.dtype, self.device = dtype, device
        self.size = 0
        self.t: Optional[torch.Tensor] = None

    def alloc(self, n: int) -> int:
        off = self.size
        self.size += _al(max(1, n))
        return off

    def materialize(self, zero=True):
        # +SLACK: the GEMM kernels' 16-B fragment loads may run a few elements past a tensor's end
        self.t = (torch.zeros if zero else torch.empty)(max(self.size, ALIGN) + SLACK, dtype=self.dtype,
                                                        device=self.device)
        return self.t

    def view(self, off: int, n: int) -> torch.Tensor:
        return self.t.narrow(0, off, n)

    def ptr(self, off: int) -> int:
        return self.t.data_ptr() + off * self.t.element_size()


# Device copies of the shared training / test arrays, owned by their source objects: a weak-keyed map
# from the host object to its uploads, so an upload lives exactly as long as the dataset (or test array)
# it mirrors -- no process-lifetime device cache, no id() reuse hazard.
class _UploadCache:
    """Identity-keyed map host object -> {device: uploads} that holds its keys weakly (numpy arrays and
    dataclasses are unhashable, so WeakKeyDictionary does not apply): an entry dies with its key."""

    def __init__(self):
        self._d: Dict[int, tuple] = {}

    def setdefault(self, key, default):
        k = id(key)
        ent = self._d.get(k)
        if ent is not None and ent[0]() is key:
            return ent[1]

        def _drop(_ref, k=k):
            cur = self._d.get(k)
            if cur is not None and cur[0] is _ref:
                del self._d[k]
        self._d[k] = (weakref.ref(key, _drop), default)
        return default

    def clear(self):
        self._d.clear()

    def __len__(self):
        return len(self._d)


_DEVICE_DATA = _UploadCache()


def device_data(data, device) -> dict:
    """Upload the (shared) training/test arrays once per dataset object and device, as bf16 / int32."""
    per_dev = _DEVICE_DATA.setdefault(data, {})
    d = per_dev.get(str(device))
    if d is None:
        def bf(a):
            return torch.as_tensor(np.ascontiguousarray(a.reshape(len(a), -1)), dtype=torch.float32).to(
                device).to(torch.bfloat16).contiguous()

        d = {
            "train_x": bf(data.train_x), "train_g": bf(data.train_g),
            "train_y": torch.as_tensor(data.train_labels.astype(np.int32), device=device),
            "test_x": bf(data.test_x), "test_g": bf(data.test_g),
            "test_y": torch.as_tensor(data.test_labels.astype(np.int32), device=device),
        }
        per_dev[str(device)] = d
    return d


def release_device_data() -> None:
    """Drop every cached upload (the OOM path frees them before a retry)."""
    _DEVICE_DATA.clear()


# ------------------------------------------------------------------------------------------------
@dataclass
class OrgLayout:
    """Per-organism parameter / buffer layout (offsets into the arenas)."""
    ir: OrganismIR
    w: Dict[int, int] = field(default_factory=dict)       # gemm node -> Wm offset (param arena)
    b: Dict[int, int] = field(default_factory=dict)       # gemm node -> bias offset
    gamma: Dict[int, int] = field(default_factory=dict)
    beta: Dict[int, int] = field(default_factory=dict)
    mm: Dict[int, int] = field(default_factory=dict)      # moving stats (stat arena)
    mv: Dict[int, int] = field(default_factory=dict)
    head: int = -1                                         # fused head pseudo-node id


@dataclass
class Launch:
    kind: str
    arg: int
    descs: Optional[torch.Tensor]
    tiles: Optional[torch.Tensor]
    n: int


_NP_TO_TORCH = {np.dtype(np.uint8): torch.uint8, np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64,
                np.dtype(np.float32): torch.float32}


# Measurement only: launches of these "kind:arg" chunked kinds (e.g. "bn:0,bn:5") are left out of every plan, to
# bound what fusing them away could save.  The results are wrong with it set; nothing sets it by default.
_TIMING_SKIP = frozenset(filter(None, os.environ.get("SERANN_TIMING_SKIP", "").split(",")))

class _TableArena:
    """The descriptor and tile tables of one plan, packed into a few device buffers.  A table gets its
    device address when it is added (descriptors embed the addresses of other descriptors, e.g. GF_NBNSUM's
    NbnDesc), and the tables reach the device with ONE host-to-device copy per buffer when the plan is
    complete (:meth:`flush`) instead of one small pageable copy per table (~1500 per generation-3 plan set:
    a fifth of its build time)."""
    ALIGN = 256

    def __init__(self, device, chunk: int = 1 << 21):
        self.device, self.chunk = device, chunk
        self.bufs: List[list] = []                  # [host uint8 array, device uint8 tensor, bytes used]

    def put(self, arr: np.ndarray) -> torch.Tensor:
        a = np.ascontiguousarray(arr)
        nb = a.nbytes
        if not self.bufs or self.bufs[-1][2] + nb + SLACK > len(self.bufs[-1][0]):
            size = max(self.chunk, _al(nb) + 2 * SLACK)
            self.bufs.append([np.zeros(size, np.uint8), torch.empty(size, dtype=torch.uint8, device=self.device), 0])
        b = self.bufs[-1]
        off = b[2]
        b[0][off:off + nb] = a.reshape(-1).view(np.uint8)
        b[2] = off + -(-max(nb, 1) // self.ALIGN) * self.ALIGN
        return b[1][off:off + nb].view(_NP_TO_TORCH[a.dtype]).view(a.shape)

    def flush(self, keep: list) -> None:
        for host, dev, used in self.bufs:
            if used:
                dev[:used].copy_(torch.from_numpy(host[:used]))
            keep.append(dev)
        self.bufs = []


class Plan:
    """A compiled list of launches for one (mode, batch) configuration."""

    def __init__(self):
        self.launches: List[Launch] = []
        self.keep: List[torch.Tensor] = []

    def run(self):
        L = H.lib()
        s = H.stream_handle()
        for la in self.launches:
            k = la.kind
            if k == "gemm3":
                L.gemm3(la.arg[0], la.arg[1], la.descs.data_ptr(), la.tiles.data_ptr(), la.n, s)
            elif k == "transpose":
                L.transpose_weights(la.descs.data_ptr(), la.tiles.data_ptr(), la.n, s)
            elif k == "imcol":
                L.imcol(la.descs.data_ptr(), la.tiles.data_ptr(), la.n, s)
            elif k == "bn":
                L.bn(la.arg, la.descs.data_ptr(), la.tiles.data_ptr(), la.n, s)
            elif k == "pool":
                L.pool(la.arg, la.descs.data_ptr(), la.tiles.data_ptr(), la.n, s)
            elif k == "convpool":
                L.convpool(la.arg[0], la.arg[1], la.descs.data_ptr(), la.tiles.data_ptr(), la.n, s)
            elif k == "gchain":
                L.gchain(la.arg[0], la.arg[1], la.descs.data_ptr(), la.tiles.data_ptr(), la.n, s)
            elif k == "nbn":
                L.nbn(la.arg[0], la.arg[1], la.descs.data_ptr(), la.tiles.data_ptr(), la.n, s)
            elif k == "copy":
                L.copy2d(la.descs.data_ptr(), la.tiles.data_ptr(), la.n, s)
            elif k == "ew":
                L.ew(la.descs.data_ptr(), la.tiles.data_ptr(), la.n, s)
            elif k == "splitfin":
                L.splitk_finalize(la.descs.data_ptr(), la.tiles.data_ptr(), la.n, s)
            elif k == "wgfin":
                L.wgrad_finalize(la.descs.data_ptr(), la.tiles.data_ptr(), la.n, s)
            elif k == "bin":
                L.bin(la.arg, la.descs.data_ptr(), la.tiles.data_ptr(), la.n, s)
            elif k == "memset":
                L.memset32(la.arg[0], la.arg[1], s)
            else:
                raise ValueError(k)


class HipPopulationEngine(PopulationEngine):
    def __init__(self, irs: Sequence[OrganismIR], seeds: Sequence[int], device="cuda", cfg: Optional[TrainConfig] = None,
                 params: Optional[List[Dict[int, Dict[str, np.ndarray]]]] = None):
        self.lib = H.lib(required=True)
        H.check_layouts()
        self.device = torch.device(device)
        self.cfg = cfg or TrainConfig()
        self.irs = list(irs)
        self.num_organisms = len(self.irs)
        self.lb = [float(ir.loss_balance) for ir in self.irs]
        self._build_param_layout()
        self._init_params(seeds, params)
        self.plans: Dict[tuple, Plan] = {}
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.timings: Dict[str, float] = {}
        self._bg = threading.local()                 # fit's background plan builder (_upload_fence)

    # ---------------------------------------------------------------------------------------------
    # parameters
    # ---------------------------------------------------------------------------------------------
    def _build_param_layout(self):
        dev = self.device
        self.parena = Arena(torch.float32, dev)
        self.sarena = Arena(torch.float32, dev)     # BN moving statistics
        self.layouts: List[OrgLayout] = []
        org_off = []
        for ir in self.irs:
            lay = OrgLayout(ir)
            org_off.append(self.parena.size)              # organisms are contiguous in the parameter arena
            for n in ir.nodes:
                if n.op == "gemm" and n.attrs["kind"] not in ("head_cls", "head_rep"):
                    a = n.attrs
                    lay.w[n.id] = self.parena.alloc(a["f"] * a["kh"] * a["kw"] * a["cin"])
                    if a["use_bias"]:
                        lay.b[n.id] = self.parena.alloc(a["f"])
                elif n.op == "bn":
                    c = n.attrs["channels"]
                    if n.attrs["scale"]:
                        lay.gamma[n.id] = self.parena.alloc(c)
                    if n.attrs["center"]:
                        lay.beta[n.id] = self.parena.alloc(c)
                    lay.mm[n.id] = self.sarena.alloc(c)
                    lay.mv[n.id] = self.sarena.alloc(c)
            # fused heads: [NC + L][D] contiguous, bias [NC + L]
            D, NC, L = ir.head_features, ir.num_classes, ir.genotype_size
            lay.head = ir.cls_head
            lay.w[ir.cls_head] = self.parena.alloc((NC + L) * D)
            lay.b[ir.cls_head] = self.parena.alloc(NC + L)
            self.layouts.append(lay)
        org_off.append(self.parena.size)
        # divergence flags (csrc/hip/common.h flag_diverged): the Adam passes flag an organism with a gradient
        # element beyond fp16's range; fit / evaluate report its metrics as NaN
        self.org_off = torch.as_tensor(np.asarray(org_off, np.int64), device=dev)
        self.diverged = torch.zeros(max(len(self.irs), 1), dtype=torch.int32, device=dev)
        # transposed bf16 weights for DGRAD (v2): Wt[C][KH][KW][F]
        self.wt_off = []
        wt_size = 0
        for lay in self.layouts:
            d = {}
            for nid, off in lay.w.items():
                n = lay.ir.node(nid)
                a = n.attrs
                if a["kind"] == "head_cls":
                    cnt = (lay.ir.num_classes + lay.ir.genotype_size) * lay.ir.head_features
                else:
                    cnt = a["f"] * a["kh"] * a["kw"] * a["cin"]
                d[nid] = wt_size
                wt_size += _al(cnt)
            self.wt_off.append(d)
        self.wt = torch.zeros(max(wt_size, ALIGN) + SLACK, dtype=torch.bfloat16, device=dev)
        self.p = self.parena.materialize()
        # gradients: deterministic Q40 fixed-point accumulator (csrc/hip/common.h fx_*), converted by Adam
        self.g = torch.zeros(self.p.numel(), dtype=torch.int64, device=dev)
        # Adam moments: fp32, or 16 bits -- bf16 m, log16 v (TrainConfig.adam_moments; csrc/hip/common.h MOM_16)
        if self.cfg.adam_moments not in ("16bit", "fp32"):
            raise ValueError(f"adam_moments must be '16bit' or 'fp32', not {self.cfg.adam_moments!r}")
        self.mom_mode = H.MOM_16 if self.cfg.adam_moments == "16bit" else H.MOM_F32
        m16 = self.mom_mode == H.MOM_16
        self.m = torch.zeros(self.p.numel(), dtype=torch.bfloat16 if m16 else torch.float32, device=dev)
        # (log16 v: 16-bit codes held in int16, code 0 is v = 0)
        self.v = torch.zeros(self.p.numel(), dtype=torch.int16 if m16 else torch.float32, device=dev)
        self.pbf = torch.zeros(self.p.numel() + SLACK, dtype=torch.bfloat16, device=dev)
        self.stats = self.sarena.materialize()
        self.step_i = torch.zeros(1, dtype=torch.int32, device=dev)
        self.lr_t = torch.zeros(1, dtype=torch.float32, device=dev)

    def _init_params(self, seeds, params):
        """Keras defaults: glorot-uniform kernels, zero bias, gamma 1, beta 0, moving var 1.
        With ``params`` (numpy, Keras layout) the exact values are loaded (parity tests)."""
        P = self.p
        with torch.no_grad():
            for i, lay in enumerate(self.layouts):
                ir = lay.ir
                gen = torch.Generator(device=self.device)
                gen.manual_seed(int(seeds[i]) if seeds is not None else i)
                src = params[i] if params is not None else None
                for n in ir.nodes:
                    if n.op == "gemm":
                        a = n.attrs
                        if a["kind"] == "head_rep":
                            continue
                        if a["kind"] == "head_cls":
                            D, NC, L = ir.head_features, ir.num_classes, ir.genotype_size
                            rep = ir.node(ir.rep_head)
                            blocks = []
                            for hn in (n, rep):
                                ha = hn.attrs
                                if src is not None:
                                    k = torch.as_tensor(src[hn.id]["kernel"], device=self.device)   # (1,1,D,f)
                                    blocks.append(k.reshape(D, ha["f"]).t())
                                else:
                                    lim = glorot_limit(hn)
                                    blocks.append((torch.rand(ha["f"], D, generator=gen, device=self.device) * 2 - 1) * lim)
                            w = torch.cat(blocks, 0)
                            P.narrow(0, lay.w[n.id], (NC + L) * D).copy_(w.reshape(-1))
                            P.narrow(0, lay.b[n.id], NC + L).zero_()
                            continue
                        cnt = a["f"] * a["kh"] * a["kw"] * a["cin"]
                        if src is not None:
                            k = torch.as_tensor(src[n.id]["kernel"], device=self.device)   # (kh,kw,c,f)
                            w = k.permute(3, 0, 1, 2).reshape(-1)
                        else:
                            w = (torch.rand(cnt, generator=gen, device=self.device) * 2 - 1) * glorot_limit(n)
                        P.narrow(0, lay.w[n.id], cnt).copy_(w)
                        if n.id in lay.b:
                            P.narrow(0, lay.b[n.id], a["f"]).zero_()
                    elif n.op == "bn":
                        c = n.attrs["channels"]
                        if n.id in lay.gamma:
                            P.narrow(0, lay.gamma[n.id], c).fill_(1.0)
                        if n.id in lay.beta:
                            P.narrow(0, lay.beta[n.id], c).zero_()
                        self.stats.narrow(0, lay.mm[n.id], c).zero_()
                        self.stats.narrow(0, lay.mv[n.id], c).fill_(1.0)
            self.pbf[:P.numel()].copy_(P.to(torch.bfloat16))

    def export_params(self, i: int) -> Dict[int, Dict[str, np.ndarray]]:
        """Organism ``i`` parameters in Keras layout (for parity tests / checkpoints)."""
        lay = self.layouts[i]
        ir = lay.ir
        out: Dict[int, Dict[str, np.ndarray]] = {}
        P, S = self.p.detach().cpu(), self.stats.detach().cpu()
        for n in ir.nodes:
            a = n.attrs
            if n.op == "gemm":
                if a["kind"] in ("head_cls", "head_rep"):
                    D, NC, L = ir.head_features, ir.num_classes, ir.genotype_size
                    w = P.narrow(0, lay.w[ir.cls_head], (NC + L) * D).reshape(NC + L, D)
                    b = P.narrow(0, lay.b[ir.cls_head], NC + L)
                    sl = slice(0, NC) if a["kind"] == "head_cls" else slice(NC, NC + L)
                    out[n.id] = {"kernel": w[sl].t().reshape(1, 1, D, -1).numpy().copy(), "bias": b[sl].numpy().copy()}
                    continue
                cnt = a["f"] * a["kh"] * a["kw"] * a["cin"]
                w = P.narrow(0, lay.w[n.id], cnt).reshape(a["f"], a["kh"], a["kw"], a["cin"]).permute(1, 2, 3, 0)
                d = {"kernel": w.numpy().copy()}
                if n.id in lay.b:
                    d["bias"] = P.narrow(0, lay.b[n.id], a["f"]).numpy().copy()
                out[n.id] = d
            elif n.op == "bn":
                c = a["channels"]
                d = {"moving_mean": S.narrow(0, lay.mm[n.id], c).numpy().copy(),
                     "moving_variance": S.narrow(0, lay.mv[n.id], c).numpy().copy()}
                if n.id in lay.gamma:
                    d["gamma"] = P.narrow(0, lay.gamma[n.id], c).numpy().copy()
                if n.id in lay.beta:
                    d["beta"] = P.narrow(0, lay.beta[n.id], c).numpy().copy()
                out[n.id] = d
        return out

    # ---------------------------------------------------------------------------------------------
    # activation buffers
    # ---------------------------------------------------------------------------------------------
    def _alloc_buffers(self, B: int, with_grads: bool):
        """Activation (and gradient) buffers for batch B; aliases for reshapes."""
        dev = self.device
        act = Arena(torch.bfloat16, dev)
        grad = Arena(torch.bfloat16, dev)
        f32 = Arena(torch.float32, dev)
        u8 = Arena(torch.uint8, dev)
        bufs = []
        for lay in self.layouts:
            ir = lay.ir
            bmap = {}
            owner = {}
            for n in ir.nodes:
                size = B * math.prod(n.shape)
                if n.op == "input":
                    owner[n.id] = n.id
                    continue
                if n.op == "reshape":
                    owner[n.id] = owner[n.inputs[0]]
                    bmap[n.id] = bmap.get(n.inputs[0])
                    continue
                if n.op == "gemm" and n.attrs["kind"] == "head_rep":
                    continue
                owner[n.id] = n.id
                if n.op == "gemm" and n.attrs["kind"] == "head_cls":
                    NC, L = ir.num_classes, ir.genotype_size
                    bmap[n.id] = ("f32", f32.alloc(B * (NC + L)))
                    continue
                bmap[n.id] = ("act", act.alloc(size))
            fused_convs = set(convpool_pairs(ir))
            gch = gchain_triples(ir)
            no_tensor = set(fused_convs)     # outputs (and gradients) never materialised
            gc_nodes = set()
            for cid, did, bid in gch.values():
                gc_nodes.update(i for i in (cid, did, bid) if i is not None)
                no_tensor.add(cid)
                if bid is not None:
                    no_tensor.add(did)
            for cid in no_tensor:
                bmap.pop(cid, None)          # fused conv + pool, fused genotype chain
            rec = {"owner": owner, "act": bmap, "grad": {}, "idx": {}, "bn": {}, "fused_convs": fused_convs,
                   "gchain": gch, "gc_nodes": gc_nodes}
            for n in ir.nodes:
                if n.op == "pool":
                    rec["idx"][n.id] = u8.alloc(B * math.prod(n.shape))
                if n.op == "bn":
                    c = n.attrs["channels"]
                    rec["bn"][n.id] = {"mean": f32.alloc(c), "invstd": f32.alloc(c), "ws": None, "wsb": None}
                    if not n.attrs["last"]:
                        # a BatchNormalization on a non-last axis runs channels-last on transposed copies
                        # (ew.hip permutes): input / output [outer][inner][C], their gradients likewise
                        size = B * math.prod(n.shape)
                        rec["bn"][n.id].update(xt=act.alloc(size), yt=act.alloc(size))
            if with_grads:
                req = self._requires_grad(ir)
                for n in ir.nodes:
                    if n.op in ("input", "reshape") or (n.op == "gemm" and n.attrs["kind"] == "head_rep"):
                        continue
                    if n.id in no_tensor:
                        continue
                    if n.op == "gemm" and n.attrs["kind"] == "head_cls":
                        NC, L = ir.num_classes, ir.genotype_size
                        rec["grad"][n.id] = grad.alloc(B * (NC + L))
                    elif req[n.id]:
                        rec["grad"][n.id] = grad.alloc(B * math.prod(n.shape))
                    if n.op == "bn" and not n.attrs["last"] and req[n.id]:
                        size = B * math.prod(n.shape)
                        rec["bn"][n.id].update(dyt=grad.alloc(size), dxt=grad.alloc(size))
                rec["req"] = req
            bufs.append(rec)
        # BN statistics workspaces (wide fixed point: [stripe][2C][hi, lo] int64, csrc/hip/common.h fxw_*),
        # contiguous so one memset zeroes them all
        ws = Arena(torch.int64, dev)
        for lay, rec in zip(self.layouts, bufs):
            for nid, d in rec["bn"].items():
                c = lay.ir.node(nid).attrs["channels"]
                d["ws"] = ws.alloc(H.bn_ws_words(c))
                d["wsb"] = ws.alloc(H.bn_ws_words(c))
        act.materialize(zero=True)
        grad.materialize(zero=True)
        f32.materialize(zero=True)
        u8.materialize(zero=True)
        ws.materialize(zero=True)
        return {"act": act, "grad": grad, "f32": f32, "u8": u8, "ws": ws, "orgs": bufs, "B": B}

    @staticmethod
    def _requires_grad(ir: OrganismIR) -> Dict[int, bool]:
        req = {}
        for n in ir.nodes:
            if n.op == "input":
                req[n.id] = False
            elif n.op == "reshape":
                req[n.id] = req[n.inputs[0]]
            else:
                has_params = n.op == "gemm" or (n.op == "bn" and (n.attrs["scale"] or n.attrs["center"]))
                req[n.id] = has_params or any(req[i] for i in n.inputs)
        return req

    # ---------------------------------------------------------------------------------------------
    # plan compilation
    # ---------------------------------------------------------------------------------------------
    def _act_ptr(self, mem, org: int, nid: int, inputs: dict) -> int:
        rec = mem["orgs"][org]
        ir = self.layouts[org].ir
        own = rec["owner"][nid]
        node = ir.node(own)
        if node.op == "input":
            return inputs[org][node.attrs["name"]]
        kind, off = rec["act"][own]
        return mem["act"].ptr(off) if kind == "act" else mem["f32"].ptr(off)

    def _grad_ptr(self, mem, org: int, nid: int) -> int:
        rec = mem["orgs"][org]
        own = rec["owner"][nid]
        off = rec["grad"].get(own)
        return None if off is None else mem["grad"].ptr(off)

    def _fused_concats(self, mem, org_iter):
        """Concatenations read in place by their consumers (no concat copy).

        Eligible: a concat along the last axis whose every consumer (through reshapes) is a Dense /
        classification-head GEMM that takes the concat's rows as its input rows -- the Keras pattern
        ``Dense(concatenate([Reshape((1, -1))(X), Reshape((1, -1))(g)]))``.  The consumer then runs one
        K slice per concat input (A = that input in place, B = its column range of the weights).
        Returns (fcat[o]: concat id -> [(input id, first column, width)], fcons[o]: gemm id -> concat id).
        SERANN_FUSE_CONCAT=0 turns it off."""
        P = self.num_organisms
        fcat = [dict() for _ in range(P)]
        fcons = [dict() for _ in range(P)]
        if os.environ.get("SERANN_FUSE_CONCAT", "1") == "0":
            return fcat, fcons
        for o, lay in org_iter():
            ir = lay.ir
            owner = mem["orgs"][o]["owner"]
            for c in ir.nodes:
                if c.op != "concat" or owner.get(c.id) != c.id or c.attrs["axis"] != len(c.shape):
                    continue
                D, rows = c.shape[-1], math.prod(c.shape[:-1])
                cons, ok = [], True
                for n in ir.nodes:
                    if n.op == "reshape" or not any(owner.get(i) == c.id for i in n.inputs):
                        continue
                    if n.op == "gemm" and n.attrs["kind"] == "head_rep":
                        continue
                    a = n.attrs
                    if n.op == "gemm" and a["kind"] == "dense" and a["cin"] == D and a["h"] == rows:
                        cons.append(n.id)
                    elif n.op == "gemm" and a["kind"] == "head_cls" and ir.head_features == D and rows == 1:
                        cons.append(n.id)
                    else:
                        ok = False
                        break
                if not ok or not cons:
                    continue
                parts, col = [], 0
                for i in c.inputs:
                    w = ir.node(i).shape[-1]
                    parts.append((i, col, w))
                    col += w
                if col != D:
                    continue
                fcat[o][c.id] = parts
                for g in cons:
                    fcons[o][g] = c.id
        return fcat, fcons

    def _stream_groups(self, nstreams: int) -> List[List[int]]:
        """Partition the organisms into <= nstreams groups of similar predicted step time (LPT on the
        calibrated cost model; SERANN_STREAM_COST=flops: on training FLOPs, the round-2 rule)."""
        P = self.num_organisms
        k = max(1, min(int(nstreams), P))
        if k == 1:
            return [list(range(P))]
        if os.environ.get("SERANN_STREAM_COST", "model") == "flops":
            costs = [float(lay.ir.cost_per_sample()) + 1.0 for lay in self.layouts]
        else:       # calibrated per-organism step time (experiment/cost_model.py), as for the rank partition
            costs = [organism_time(lay.ir, self.cfg.batch_size) for lay in self.layouts]
        order = sorted(range(P), key=lambda o: -costs[o])
        loads = [0.0] * k
        groups: List[List[int]] = [[] for _ in range(k)]
        for o in order:
            i = min(range(k), key=lambda j: loads[j])
            groups[i].append(o)
            loads[i] += costs[o]
        return [sorted(g) for g in groups if g]

    def _build_plan(self, mode: str, B: int, mem, inputs: List[dict], label_ptr: int = 0, target_ptrs=None,
                    metrics: Optional[torch.Tensor] = None, orgs: Optional[Sequence[int]] = None,
                    adam_ctx: int = 0) -> Plan:
        """mode in {'train', 'infer'}; inputs[org] = {'X': ptr, 'g': ptr} bf16 device pointers.
        ``orgs``: build the plan for this subset of organisms only (one plan per stream group).
        ``adam_ctx``: device AdamCtx -- WGRAD launches that are the sole writer of their weight tile apply the
        optimizer step in their epilogue (GF_ADAM; ``plan.adam_regions`` lists those parameters, which the
        arena-wide Adam pass then skips)."""
        train = mode == "train"
        plan = Plan()
        plan.adam_regions = []
        P = self.num_organisms
        sel = None if orgs is None else set(int(o) for o in orgs)

        def org_iter():
            for o_, lay_ in enumerate(self.layouts):
                if sel is None or o_ in sel:
                    yield o_, lay_

        depth_of = []
        maxd = 0
        for o_, lay in enumerate(self.layouts):
            dd = {}
            for n in lay.ir.nodes:
                dd[n.id] = 0 if n.op == "input" else 1 + max(dd[i] for i in n.inputs)
            depth_of.append(dd)
            if sel is None or o_ in sel:
                maxd = max(maxd, max(dd.values()))

        tables = _TableArena(self.device)

        def T(arr):
            return tables.put(np.asarray(arr))

        def desc_tensor(rows, dtype):
            a = H.record_array(rows, dtype)
            if dtype == H.GEMM_DTYPE:
                H.fill_gemm_divisors(a)
            return T(np.frombuffer(a.tobytes(), dtype=np.uint8).copy())

        def add_gemm(mode_, rows, dims, extra_fin=None):
            if not rows:
                return
            assert len(rows) == len(dims), (len(rows), len(dims))
            # split WGRADs of every variant group of this call are finalized by ONE grouped launch after the
            # last of them (not one per group: a finalize launch is mostly its own latency)
            wfin_all = []
            for v, rws, tiles in H.gemm3_plan(mode_, rows, dims, splitk=True):
                if not len(tiles):
                    continue
                if mode_ == H.MODE_WGRAD:
                    for r in rws:
                        if int(r.get("flags", 0)) & H.GF_ADAM:
                            plan.adam_regions.append(((int(r["out"]) - self.g.data_ptr()) // 8, int(r["M"]),
                                                      int(r["N"]), int(r.get("ldo") or r["N"])))
                # split-K FWD problems (merged Dense): fp32 partials per split in a workspace of
                # the plan, then one grouped finalize launch (ordered sum of splits + bias + activation)
                fin = []
                for r in rws:
                    ns = int(r.pop("_split", 1))
                    if ns > 1 and not r.get("_pre"):
                        wsb = torch.zeros(ns * int(r["M"]) * int(r["N"]), dtype=torch.float32, device=self.device)
                        plan.keep.append(wsb)
                        r["aux"] = wsb.data_ptr()
                        fin.append(dict(ws=r["aux"], out=r["out"], bias=r.get("bias", 0), M=r["M"], N=r["N"],
                                        S=ns, act=r.get("act", 0)))
                # split conv WGRADs: fp32 slabs per split (every element written), summed in split order by
                # one grouped wgrad_finalize launch after the GEMM (no fixed-point atomics)
                # (conv WGRADs' padded slabs, Dense / 1x1 m-splits' [M][N] slabs: GF_WSLAB); the finalize is the
                # sole writer of those weights, so it applies Adam too when the plan fuses the optimizer
                wfin = []
                for r in rws:
                    if r.get("_wgfin"):
                        wsw = torch.empty(H.wgrad_slab_elems(r) + SLACK, dtype=torch.float32, device=self.device)
                        plan.keep.append(wsw)
                        fadam = int(r.get("adam") or 0) if FINALIZE_ADAM else 0
                        wfin.append(H.wgrad_finalize_row(r, wsw.data_ptr(), fadam))
                        if fadam:
                            plan.adam_regions.append(((int(r["out"]) - self.g.data_ptr()) // 8, int(r["M"]),
                                                      int(r["N"]), int(r.get("ldo") or r["N"])))
                plan.launches.append(Launch("gemm3", (mode_, v), desc_tensor(rws, H.GEMM_DTYPE), T(tiles),
                                            len(tiles)))
                wfin_all += wfin
                if fin:
                    add_chunked("splitfin", 0, fin, H.SPLITFIN_DTYPE, [f["M"] * f["N"] for f in fin],
                                H.SPLITFIN_ELEMS)
            if wfin_all:
                add_chunked("wgfin", 0, wfin_all, H.WGFIN_DTYPE, [f["M"] * f["N"] for f in wfin_all], H.WGFIN_ELEMS)
            if extra_fin:
                # K slices of fused-concat consumers (every variant launched above): one finalize
                add_chunked("splitfin", 0, extra_fin, H.SPLITFIN_DTYPE, [f["M"] * f["N"] for f in extra_fin],
                            H.SPLITFIN_ELEMS)

        def add_chunked(kind, arg, rows, dtype, counts, chunk):
            if not rows or f"{kind}:{arg}" in _TIMING_SKIP:
                return
            tiles = H.chunk_tiles(counts, chunk)
            if len(tiles) == 0:
                return
            plan.launches.append(Launch(kind, arg, desc_tensor(rows, dtype), T(tiles), len(tiles)))

        pa, pbf = self.parena, self.pbf

        def wptr_bf(off):
            return pbf.data_ptr() + off * 2

        def pptr(off):
            return self.p.data_ptr() + off * 4

        def gptr(off):
            return self.g.data_ptr() + off * 8          # Q40 int64 gradient arena

        def sptr(off):
            return self.stats.data_ptr() + off * 4

        f32a = mem["f32"]

        # Shared im2col of the raw inputs: when every organism reads the same input batch, all
        # first-layer convolutions with the same (KH, KW, SH, SW) that are not fused with their pool
        # share one materialised im2col matrix, and their FWD / WGRAD become aligned 1x1 problems.
        shared_inputs = all(inp == inputs[0] for inp in inputs)
        imcol: Dict[tuple, dict] = {}

        def raw_conv_imcol(o, n):
            if not shared_inputs:
                return None
            a = n.attrs
            ir_ = self.layouts[o].ir
            src = ir_.node(mem["orgs"][o]["owner"][n.inputs[0]])
            if src.op != "input" or a["kh"] * a["kw"] == 1 or a["kind"] not in ("conv2d", "conv1d") or a["cin"] != 1:
                return None
            key = (src.attrs["name"], a["h"], a["w"], a["kh"], a["kw"], a["sh"], a["sw"])
            if key not in imcol:
                k8 = -(-(a["kh"] * a["kw"]) // 8) * 8
                rows = B * a["oh"] * a["ow"]
                buf = torch.zeros(rows * k8 + 8, dtype=torch.bfloat16, device=self.device)
                plan.keep.append(buf)
                imcol[key] = dict(buf=buf, K8=k8, rows=rows,
                                  desc=dict(x=inputs[0][src.attrs["name"]], out=buf.data_ptr(), B=B, H=a["h"], W=a["w"],
                                            OH=a["oh"], OW=a["ow"], KH=a["kh"], KW=a["kw"], SH=a["sh"], SW=a["sw"],
                                            K8=k8))
            return imcol[key]

        plan.imcol_lookup = raw_conv_imcol

        fcat, fcons = self._fused_concats(mem, org_iter)
        cpool = [dict() for _ in range(P)]            # pool id -> fused conv id
        for o, lay in org_iter():
            cpool[o] = {pid: cid for cid, pid in convpool_pairs(lay.ir).items()}

        def convpool_row(o, pool_node, conv_id):
            lay_ = self.layouts[o]
            rec_ = mem["orgs"][o]
            c = lay_.ir.node(conv_id).attrs
            pa = pool_node.attrs
            src_ = lay_.ir.node(lay_.ir.node(conv_id).inputs[0]).attrs["name"]
            return dict(x=inputs[o][src_], w=wptr_bf(lay_.w[conv_id]),
                        bias=pptr(lay_.b[conv_id]) if conv_id in lay_.b else 0,
                        y=self._act_ptr(mem, o, pool_node.id, inputs), idx=mem["u8"].ptr(rec_["idx"][pool_node.id]),
                        dy=mem["grad"].ptr(rec_["grad"][pool_node.id]) if train else 0,
                        dw=gptr(lay_.w[conv_id]) if train else 0,
                        dbias=gptr(lay_.b[conv_id]) if train and conv_id in lay_.b else 0,
                        B=B, H=c["h"], W=c["w"], F=c["f"], KH=c["kh"], KW=c["kw"], SH=c["sh"], SW=c["sw"],
                        OH=c["oh"], OW=c["ow"], PH=pa["ph"], PW=pa["pw"], PSH=pa["sh"], PSW=pa["sw"],
                        POH=pa["oh"], POW=pa["ow"], act=H.ACT_CODES[c["act"]], flags=0,
                        _kt=H.convpool_variant(c["kh"], c["kw"], c["f"]))

        def add_convpool(rows, backward):
            by_kt: Dict[int, list] = {}
            for r in rows:
                by_kt.setdefault(r.pop("_kt"), []).append(r)
            for kt in sorted(by_kt):
                rws = by_kt[kt]
                for r in rws:
                    r["flags"] = H.convpool_imgs(r["B"], r["F"], backward)
                add_chunked("convpool", (1 if backward else 0, kt), rws, H.CONVPOOL_DTYPE,
                            [H.convpool_chunks(r["B"], r["F"], backward, r["flags"]) for r in rws], 1)
        def gchain_row(o, last):
            """Descriptor of the fused genotype chain ending at node ``last`` of organism ``o``."""
            lay_ = self.layouts[o]
            rec_ = mem["orgs"][o]
            ir_ = lay_.ir
            cid, did, bid = rec_["gchain"][last]
            c = ir_.node(cid).attrs
            dn = ir_.node(did).attrs
            src_ = ir_.node(ir_.node(cid).inputs[0]).attrs["name"]
            gl = rec_["grad"].get(last) if train else None
            row = dict(g=inputs[o][src_], w1=wptr_bf(lay_.w[cid]), b1=pptr(lay_.b[cid]) if cid in lay_.b else 0,
                       w2=wptr_bf(lay_.w[did]), b2=pptr(lay_.b[did]) if did in lay_.b else 0,
                       y=self._act_ptr(mem, o, last, inputs), dy=mem["grad"].ptr(gl) if gl is not None else 0,
                       dw1=gptr(lay_.w[cid]) if train else 0, db1=gptr(lay_.b[cid]) if train and cid in lay_.b else 0,
                       dw2=gptr(lay_.w[did]) if train else 0, db2=gptr(lay_.b[did]) if train and did in lay_.b else 0,
                       B=B, L0=c["h"], L1=c["oh"], T=c["kh"], S=c["sh"], F1=c["f"], F2=dn["f"],
                       dvL1=H.fast_div_magic(c["oh"]),
                       act1=H.ACT_CODES[c["act"]], act2=H.ACT_CODES[dn["act"]], flags=H.GC_TRAIN if train else 0,
                       eps=1e-3, momentum=0.99, _bn=bid is not None,
                       _v=H.gchain_variant(c["f"], dn["f"], c["kh"])
                       + 64 * (3 * (c["act"] != "linear") + H.ACT_CODES[dn["act"]]))
            if bid is not None:
                bd = rec_["bn"][bid]
                ba = ir_.node(bid).attrs
                row.update(gamma=pptr(lay_.gamma[bid]) if bid in lay_.gamma else 0,
                           beta=pptr(lay_.beta[bid]) if bid in lay_.beta else 0,
                           mm=sptr(lay_.mm[bid]), mv=sptr(lay_.mv[bid]), mean=f32a.ptr(bd["mean"]),
                           invstd=f32a.ptr(bd["invstd"]), ws=mem["ws"].ptr(bd["ws"]), wsb=mem["ws"].ptr(bd["wsb"]),
                           dgamma=gptr(lay_.gamma[bid]) if train and bid in lay_.gamma else 0,
                           dbeta=gptr(lay_.beta[bid]) if train and bid in lay_.beta else 0,
                           eps=ba["epsilon"], momentum=ba["momentum"])
                row["flags"] |= H.GC_BN | (H.GC_GAMMA if bid in lay_.gamma else 0) | (H.GC_BETA if bid in lay_.beta else 0)
            return row

        def add_gchain(rows, mode_):
            """One launch per kernel instantiation; rows per block sized to the launch's grid."""
            by_v: Dict[int, list] = {}
            for r in rows:
                by_v.setdefault(r["_v"], []).append(dict(r))
            for v in sorted(by_v):
                rws = by_v[v]
                counts = []
                for r in rws:
                    R_ = int(r["B"]) * int(r["L1"])
                    r["rpb"] = H.gchain_rpb(R_, mode_, int(r["L1"]), int(r["L0"]))
                    counts.append(-(-R_ // r["rpb"]))
                tiles = H.chunk_tiles(counts, 1)
                if len(tiles):
                    plan.launches.append(Launch("gchain", (mode_, v), desc_tensor(rws, H.GCHAIN_DTYPE), T(tiles),
                                                len(tiles)))

        # fused raw-input Dense -> BatchNormalization (training): BN id -> Dense id, and the Dense ids
        nbn = [nbn_pairs(lay.ir) if train and (sel is None or o in sel) else {} for o, lay in enumerate(self.layouts)]
        nbn_src = [set(m.values()) for m in nbn]
        # pairs whose BN output has ONE consumer GEMM, whose DGRAD runs on the LDS-tiled kernel: that DGRAD reduces
        # the BN / Dense backward sums in its epilogue (GF_NBNSUM) instead of storing dY, and nbn phase 6 replaces
        # phases 4 and 5 (which read the stored dY twice)
        nbnsum = [set() for _ in range(P)]
        if train and NBN_SUM and "tiled" not in H._OFF:
            for o, lay in org_iter():
                ir = lay.ir
                owner = mem["orgs"][o]["owner"]
                for bid, did in nbn[o].items():
                    if ir.node(did).attrs["cin"] != 1:
                        continue                        # the DGRAD epilogue form covers 1-channel raw inputs
                    uses = [n for n in ir.nodes if n.op != "reshape" and any(owner.get(i, i) == bid for i in n.inputs)]
                    if len(uses) != 1:
                        continue
                    u = uses[0]
                    if u.op == "concat" and u.id in fcat[o]:
                        cons = [g for g, c in fcons[o].items() if c == u.id]
                        if len(cons) != 1 or sum(owner.get(pid, pid) == bid for pid, _, _ in fcat[o][u.id]) != 1:
                            continue
                        cn = ir.node(cons[0])
                        kdg = ir.num_classes + ir.genotype_size if cn.attrs["kind"] == "head_cls" else cn.attrs["f"]
                        ok = kdg > H.BK
                    elif (u.op == "gemm" and u.attrs["kind"] == "dense" and owner.get(u.inputs[0], u.inputs[0]) == bid):
                        a_ = u.attrs
                        ok = a_["kh"] * a_["kw"] == 1 and a_["sh"] * a_["sw"] == 1 and a_["f"] > H.BK
                    else:
                        ok = False
                    if ok:
                        nbnsum[o].add(bid)
        nbnsum_rows = [dict() for _ in range(P)]
        # binary-genotype pairs (bnbn.hip): an nbnsum pair on the raw genotype whose BN output is one K slice of a
        # merged Dense -- the slice's FWD / DGRAD / WGRAD become the factorised kernels and its BN output is never
        # written.  Only when this engine's genotype batches are binary (fit / debug_train_step check the data).
        binpair = [dict() for _ in range(P)]           # bid -> consumer gemm id
        if train and BINARY_NBN and getattr(self, "_g_binary", False):
            for o, lay in org_iter():
                ir = lay.ir
                for bid in nbnsum[o]:
                    did = nbn[o][bid]
                    if ir.node(ir.node(did).inputs[0]).attrs["name"] != "g":
                        continue
                    own_ = mem["orgs"][o]["owner"]
                    cons = [(g_, c_) for g_, c_ in fcons[o].items()
                            if any(own_.get(pid, pid) == bid for pid, _, _ in fcat[o].get(c_, []))]
                    if len(cons) != 1:
                        continue
                    cn = ir.node(cons[0][0])
                    Lg, Fb = ir.genotype_size, ir.node(did).attrs["f"]
                    if (cn.attrs["kind"] == "dense" and cn.attrs["f"] <= 256 and Lg <= 256 and Fb <= 256
                            and math.prod(ir.node(bid).shape) == Lg * Fb):
                        binpair[o][bid] = cons[0][0]

        def binslice(o, pid, cid):
            """The binary pair whose BN output is K slice ``pid`` (a concat input: the BN's reshape) of consumer
            ``cid``, or None."""
            bid = mem["orgs"][o]["owner"].get(pid, pid)
            return bid if binpair[o].get(bid) == cid else None

        def bin_desc(o, bid, cid, col, width):
            """BinDesc of pair ``bid`` and its consumer ``cid`` (K slice at column ``col``), with its E / C0
            workspaces; the FWD slab, the H / cs / part buffers and dW are filled in by the callers."""
            lay_ = self.layouts[o]
            ir_ = lay_.ir
            did = nbn[o][bid]
            Nc = ir_.node(cid).attrs["f"]
            Lg, Fb = ir_.genotype_size, ir_.node(did).attrs["f"]
            Ew = torch.empty(Lg * Nc + Nc, dtype=torch.float32, device=self.device)
            plan.keep.append(Ew)
            bd_ = mem["orgs"][o]["bn"][bid]
            return dict(g=inputs[o]["g"], w=wptr_bf(lay_.w[did]), bias=pptr(lay_.b[did]) if did in lay_.b else 0,
                        gamma=pptr(lay_.gamma[bid]) if bid in lay_.gamma else 0,
                        beta=pptr(lay_.beta[bid]) if bid in lay_.beta else 0,
                        mean=f32a.ptr(bd_["mean"]), invstd=f32a.ptr(bd_["invstd"]),
                        act=H.ACT_CODES[ir_.node(did).attrs["act"]],
                        flags=(1 if bid in lay_.gamma else 0) | (2 if bid in lay_.beta else 0),
                        wc=wptr_bf(lay_.w[cid]) + 2 * col, ldw=ir_.node(cid).attrs["cin"], Nc=Nc, L=Lg, F=Fb, B=B,
                        E=Ew.data_ptr(), C0=Ew.data_ptr() + 4 * Lg * Nc)

        def add_bin(phase, rows):
            if not rows:
                return
            if phase == 0:                             # (problem, n)
                counts = [int(r["Nc"]) for r in rows]
            elif phase == 1:                           # (problem, 32-row block)
                counts = [-(-int(r["B"]) // 32) for r in rows]
            else:                                      # (problem, (64 V-column block) * ns + split)
                counts = [-(-int(r["L"]) * int(r["F"]) // (256 if r["flags"] & H.BIN_VEC4 else 64)) * int(r["ns"])
                          for r in rows]
            tiles = H.chunk_tiles(counts, 1)
            plan.launches.append(Launch("bin", phase, desc_tensor(rows, H.BIN_DTYPE), T(tiles), len(tiles)))

        def add_bin_sw(rows):
            """bin_sw over this depth's factorised slices.  A launch of few column blocks (a lone organism's
            slice) splits its rows too, towards BIN_SW_BLOCKS blocks of >= 32 rows each; split s writes its
            partial sums into NbnDesc::part slot s, which phase 6 adds with the others."""
            if not rows:
                return
            jbl = [-(-int(r["L"]) * int(r["F"]) // (256 if r["flags"] & H.BIN_VEC4 else 64)) for r in rows]
            want = -(-BIN_SW_BLOCKS // sum(jbl))
            for r in rows:
                r["ns"] = max(1, min(want, int(r["Nc"]) // 32))
                nbnsum_ext(r["_o"], r["_bid"], 128 * r["ns"], int(r["L"]) * int(r["F"]))   # ns m slots
                r["part"] = nbnsum_rows[r["_o"]][r["_bid"]]["part"]
            add_bin(3, rows)

        def nbnsum_ext(o, bid, M_, N_):
            """Device NbnDesc (with its partial-sum workspace) for the GF_NBNSUM DGRAD of pair ``bid``."""
            row = nbn_row(o, bid)
            Fb = int(row["F"])
            if N_ % Fb:
                raise RuntimeError(f"organism {o}: BN {bid} gradient columns {N_} not a multiple of its {Fb} channels")
            mt = -(-M_ // 128)                          # the LDS-tiled kernel's m tile
            part = torch.empty(mt * N_ * H.NBN_NSUM, dtype=torch.float32, device=self.device)
            plan.keep.append(part)
            row.update(part=part.data_ptr(), mtiles=mt, np=N_ // Fb)
            nbnsum_rows[o][bid] = row
            return desc_tensor([row], H.NBN_DTYPE).data_ptr()

        def nbn_row(o, bid):
            lay_ = self.layouts[o]
            rec_ = mem["orgs"][o]
            ir_ = lay_.ir
            did = nbn[o][bid]
            a_ = ir_.node(did).attrs
            ba = ir_.node(bid).attrs
            bd = rec_["bn"][bid]
            bflags = (1 if bid in lay_.gamma else 0) | (2 if bid in lay_.beta else 0)
            R_ = B * math.prod(ir_.node(bid).shape) // ba["channels"]
            src_ = ir_.node(ir_.node(did).inputs[0]).attrs["name"]
            return dict(x=inputs[o][src_], w=wptr_bf(lay_.w[did]), bias=pptr(lay_.b[did]) if did in lay_.b else 0,
                        y=self._act_ptr(mem, o, bid, inputs),
                        dy=mem["grad"].ptr(rec_["grad"][bid]) if bid in rec_["grad"] else 0,
                        gamma=pptr(lay_.gamma[bid]) if bid in lay_.gamma else 0,
                        beta=pptr(lay_.beta[bid]) if bid in lay_.beta else 0,
                        mm=sptr(lay_.mm[bid]), mv=sptr(lay_.mv[bid]), mean=f32a.ptr(bd["mean"]),
                        invstd=f32a.ptr(bd["invstd"]), ws=mem["ws"].ptr(bd["ws"]), wsb=mem["ws"].ptr(bd["wsb"]),
                        dw=gptr(lay_.w[did]), db=gptr(lay_.b[did]) if did in lay_.b else 0,
                        dgamma=gptr(lay_.gamma[bid]) if bid in lay_.gamma else 0,
                        dbeta=gptr(lay_.beta[bid]) if bid in lay_.beta else 0,
                        R=R_, F=a_["f"], K=a_["cin"], ldx=a_["cin"], act=H.ACT_CODES[a_["act"]], flags=bflags,
                        eps=ba["epsilon"], momentum=ba["momentum"])

        def add_nbn(rows, phase, stats_only=False):
            by_k: Dict[int, list] = {}
            for r in rows:
                by_k.setdefault(int(r["K"]), []).append({k: v for k, v in r.items() if not k.startswith("_")})
            for k_ in sorted(by_k):
                rws = by_k[k_]
                if stats_only:
                    # phase 2's first block of each problem only: statistics, moving averages, mean / invstd
                    tiles = np.array([(p_, 0, 0, 1) for p_ in range(len(rws))], np.int32)
                else:
                    tiles = H.nbn_fin_tiles([r["F"] for r in rws]) if phase == 6 else \
                        H.nbn_tiles([(r["R"], r["F"]) for r in rws], phase)
                if len(tiles):
                    plan.launches.append(Launch("nbn", (phase, k_), desc_tensor(rws, H.NBN_DTYPE), T(tiles),
                                                len(tiles)))

        # gemm node -> the (first) last-axis BatchNormalization reading its output with matching channels
        bn_consumer = [dict() for _ in range(P)]
        bn_prefused = set()
        for o, lay in org_iter():
            owner = mem["orgs"][o]["owner"]
            for n in lay.ir.nodes:
                if n.op == "bn" and n.attrs["last"] and n.id not in mem["orgs"][o]["gc_nodes"]:
                    src = lay.ir.node(owner[n.inputs[0]])
                    if (src.op == "gemm" and src.attrs["kind"] not in ("head_cls", "head_rep")
                            and src.attrs["f"] == n.attrs["channels"] and src.id not in bn_consumer[o]):
                        bn_consumer[o][src.id] = n.id

        def concat_slices(o, n, F):
            """K slices (input node, first column, width, k splits, first workspace slot) of a fused-concat
            consumer, and the number of workspace slots."""
            out, S = [], 0
            for pid, col, width in fcat[o][fcons[o][n.id]]:
                kt = -(-width // H.BK)
                ns = max(1, min(16, kt // H.SPLIT_KSTEPS)) if H.SPLIT_KSTEPS > 0 else 1
                if binslice(o, pid, n.id) is not None:
                    ns = 1                              # the factorised slice writes one fp32 partial (bin_fwd)
                out.append((pid, col, width, ns, S))
                S += ns
            return out, S

        bn_ustat = set()

        def bnustat(o, n, row, M, F, K):
            """The FWD row of a GEMM whose output feeds a BatchNormalization accumulates that BN's phase-0 statistics
            (unshifted) in its epilogue when its kernel can (hip_ops.fwd_bnustat_ok); the BN's phase-0 launch is
            dropped and its phase 2 reads the sums with BnDesc flag 512."""
            bnc = bn_consumer[o].get(n.id)
            if not (train and bnc is not None and FUSE_BN_USTATS and F <= 256 and H.fwd_bnustat_ok(row, M, F, K)):
                return
            row["aux"] = mem["ws"].ptr(mem["orgs"][o]["bn"][bnc]["ws"])
            row["flags"] |= H.GF_BNUSTAT
            bn_prefused.add((o, bnc))
            bn_ustat.add((o, bnc))

        # ---- forward ---------------------------------------------------------------------------
        for d in range(1, maxd + 1):
            fin_rows = []
            bin_rows = []
            g_rows, g_dims = [], []
            p_rows, p_cnt = [], []
            bn_rows, bn_cnt, bn_cnt_st, bn_stat = [], [], [], []
            nbn_rows = []
            c_rows, c_cnt = [], []
            cp_rows = []
            gc_rows = []
            ew_pre, ew_post = [], []          # rare ops (ew.hip): maps / transposes in, transposes out
            for o, lay in org_iter():
                ir = lay.ir
                rec = mem["orgs"][o]
                for n in ir.nodes:
                    if depth_of[o][n.id] != d or n.op in ("input", "reshape"):
                        continue
                    a = n.attrs
                    if n.id in rec["gc_nodes"]:
                        if n.id in rec["gchain"]:
                            gc_rows.append(gchain_row(o, n.id))   # the whole chain, at its last node's depth
                        continue
                    if n.id in rec["fused_convs"]:
                        continue                      # computed by the fused conv + pool kernel
                    if n.op == "pool" and n.id in cpool[o]:
                        cp_rows.append(convpool_row(o, n, cpool[o][n.id]))
                        continue
                    if n.op == "gemm":
                        if a["kind"] == "head_rep":
                            continue
                        xin = self._act_ptr(mem, o, n.inputs[0], inputs)
                        out = self._act_ptr(mem, o, n.id, inputs)
                        if a["kind"] == "head_cls":
                            NC, L, D = ir.num_classes, ir.genotype_size, ir.head_features
                            F, C, flags, act = NC + L, D, H.GF_OUT_F32, 0
                            Hh = Ww = OH = OW = 1
                            KH = KW = SH = SW = 1
                        else:
                            F, C = a["f"], a["cin"]
                            Hh, Ww, OH, OW = a["h"], a["w"], a["oh"], a["ow"]
                            KH, KW, SH, SW = a["kh"], a["kw"], a["sh"], a["sw"]
                            flags, act = 0, H.ACT_CODES[a["act"]]
                        K = KH * KW * C
                        M = B * OH * OW
                        if C % 8 == 0:
                            flags |= H.GF_VEC_A
                        if K % 8 == 0:
                            flags |= H.GF_VEC_B
                        bias = pptr(lay.b[n.id]) if n.id in lay.b else 0
                        ic = raw_conv_imcol(o, n) if a["kind"] != "head_cls" else None
                        if n.id in fcons[o]:
                            # consumer of a fused concat: one K slice per concat input, read in place
                            # (no concat copy); fp32 partials + one finalize (bias, activation)
                            D = ir.head_features if a["kind"] == "head_cls" else C
                            sl, S = concat_slices(o, n, F)
                            wsb = torch.zeros(S * M * F, dtype=torch.float32, device=self.device)
                            plan.keep.append(wsb)
                            for pid, col, width, ns, sb in sl:
                                if binslice(o, pid, n.id) is not None:
                                    bin_rows.append(dict(bin_desc(o, binslice(o, pid, n.id), n.id, col, width),
                                                         slab=wsb.data_ptr() + 4 * sb * M * F))
                                    continue
                                g_rows.append(dict(a=self._act_ptr(mem, o, pid, inputs), b=wptr_bf(lay.w[n.id]) + 2 * col,
                                                   out=out, bias=0, H=1, W=1, C=width, OH=1, OW=1, F=F, KH=1, KW=1,
                                                   SH=1, SW=1, M=M, N=F, K=width, act=0, flags=0, ldb=D,
                                                   aux=wsb.data_ptr(), sbase=sb, _split=ns, _ws=1, _force_tiled=1,
                                                   _pre=1))
                                g_dims.append((M, F, width))
                            fin_rows.append(dict(ws=wsb.data_ptr(), out=out, bias=bias, M=M, N=F, S=S, act=act,
                                                 flags=1 if a["kind"] == "head_cls" else 0))
                        elif ic is not None:
                            g_rows.append(dict(a=ic["buf"].data_ptr(), b=wptr_bf(lay.w[n.id]), out=out, bias=bias, H=OH,
                                               W=OW, C=ic["K8"], OH=OH, OW=OW, F=F, KH=1, KW=1, SH=1, SW=1, M=M, N=F,
                                               K=K, act=act, flags=flags, _imcol=1))
                            bnustat(o, n, g_rows[-1], M, F, K)
                        else:
                            g_rows.append(dict(a=xin, b=wptr_bf(lay.w[n.id]), out=out, bias=bias, H=Hh, W=Ww, C=C, OH=OH,
                                               OW=OW, F=F, KH=KH, KW=KW, SH=SH, SW=SW, M=M, N=F, K=K, act=act,
                                               flags=flags))
                            # a narrow-kernel output that feeds a BatchNormalization: the BN statistics
                            # (phase 0) are accumulated by the producing kernel itself
                            bnc = bn_consumer[o].get(n.id)
                            if (train and bnc is not None and FUSE_BN_STATS and F <= 256
                                    and H.narrow_k(g_rows[-1], H.MODE_FWD, M, F, K) is not None):
                                g_rows[-1]["aux"] = mem["ws"].ptr(rec["bn"][bnc]["ws"])
                                g_rows[-1]["flags"] |= H.GF_BNSTAT
                                bn_prefused.add((o, bnc))
                                if n.id in nbn_src[o]:
                                    g_rows[-1]["flags"] |= H.GF_NOSTORE     # recomputed by nbn.hip
                                    if bnc in binpair[o]:
                                        # binary input: nbn phase 7 derives the statistics from the count
                                        # of ones; nothing of this Dense runs in the FWD
                                        g_rows.pop()
                                        continue
                            elif n.id in nbn_src[o]:
                                raise RuntimeError(f"organism {o}: Dense {n.id} fused with its BatchNormalization "
                                                   f"but not on the narrow statistics kernel")
                            else:
                                bnustat(o, n, g_rows[-1], M, F, K)
                        if n.id not in fcons[o]:
                            g_dims.append((M, F, K))      # (K slices appended their own dims)
                    elif n.op == "pool":
                        p_rows.append(dict(x=self._act_ptr(mem, o, n.inputs[0], inputs),
                                           y=self._act_ptr(mem, o, n.id, inputs),
                                           idx=mem["u8"].ptr(rec["idx"][n.id]), B=B, H=a["h"], W=a["w"], C=a["c"],
                                           OH=a["oh"], OW=a["ow"], PH=a["ph"], PW=a["pw"], SH=a["sh"], SW=a["sw"]))
                        p_cnt.append(H.pool_units(B * math.prod(n.shape), a["c"]))
                    elif n.op == "bn" and a["last"] and n.id in nbn[o]:
                        nbn_rows.append(dict(nbn_row(o, n.id), _bin=n.id in binpair[o]))
                    elif n.op == "bn" and a["last"]:
                        bd = rec["bn"][n.id]
                        c = a["channels"]
                        flags = (1 if n.id in lay.gamma else 0) | (2 if n.id in lay.beta else 0)
                        if (o, n.id) in bn_ustat:
                            flags |= H.BN_USTAT
                        bn_rows.append(dict(x=self._act_ptr(mem, o, n.inputs[0], inputs),
                                            y=self._act_ptr(mem, o, n.id, inputs),
                                            gamma=pptr(lay.gamma[n.id]) if n.id in lay.gamma else 0,
                                            beta=pptr(lay.beta[n.id]) if n.id in lay.beta else 0,
                                            mm=sptr(lay.mm[n.id]), mv=sptr(lay.mv[n.id]),
                                            mean=f32a.ptr(bd["mean"]), invstd=f32a.ptr(bd["invstd"]),
                                            ws=mem["ws"].ptr(bd["ws"]), R=B * math.prod(n.shape) // c, C=c,
                                            flags=flags, eps=a["epsilon"], momentum=a["momentum"]))
                        bn_cnt.append(H.bn_chunks(B * math.prod(n.shape) // c, c))
                        bn_cnt_st.append(H.bn_chunks(B * math.prod(n.shape) // c, c, stats=True))
                        bn_stat.append((o, n.id) not in bn_prefused)
                    elif n.op == "concat":
                        if n.id in fcat[o]:
                            continue                  # read in place by its consumers' K slices
                        ax = a["axis"]
                        outer = B * math.prod(n.shape[:ax - 1])
                        out_inner = math.prod(n.shape[ax - 1:])
                        col = 0
                        for i in n.inputs:
                            sh = ir.node(i).shape
                            inner = math.prod(sh[ax - 1:])
                            c_rows.append(dict(src=self._act_ptr(mem, o, i, inputs),
                                               dst=self._act_ptr(mem, o, n.id, inputs) + col * 2,
                                               rows=outer, cols=inner, src_stride=inner, dst_stride=out_inner))
                            c_cnt.append(-(-outer // H.COPY_ROWS))
                            col += inner
                    elif n.op == "bn":
                        # non-last axis: [outer][C][inner] -> [outer][inner][C], the channels-last BN kernels,
                        # and back (SURVEY §2.7 mutants; the reference runs it inside its Keras graph)
                        bd = rec["bn"][n.id]
                        c = a["channels"]
                        full = (B,) + tuple(n.shape)
                        outer, inner = math.prod(full[:a["axis"]]), math.prod(full[a["axis"] + 1:])
                        xt, yt = mem["act"].ptr(bd["xt"]), mem["act"].ptr(bd["yt"])
                        ew_pre.append(H.ew_permute_row(xt, self._act_ptr(mem, o, n.inputs[0], inputs),
                                                       (outer, c, inner), (0, 2, 1)))
                        ew_post.append(H.ew_permute_row(self._act_ptr(mem, o, n.id, inputs), yt, (outer, inner, c),
                                                        (0, 2, 1)))
                        flags = (1 if n.id in lay.gamma else 0) | (2 if n.id in lay.beta else 0)
                        bn_rows.append(dict(x=xt, y=yt,
                                            gamma=pptr(lay.gamma[n.id]) if n.id in lay.gamma else 0,
                                            beta=pptr(lay.beta[n.id]) if n.id in lay.beta else 0,
                                            mm=sptr(lay.mm[n.id]), mv=sptr(lay.mv[n.id]),
                                            mean=f32a.ptr(bd["mean"]), invstd=f32a.ptr(bd["invstd"]),
                                            ws=mem["ws"].ptr(bd["ws"]), R=outer * inner, C=c,
                                            flags=flags, eps=a["epsilon"], momentum=a["momentum"]))
                        bn_cnt.append(H.bn_chunks(outer * inner, c))
                        bn_cnt_st.append(H.bn_chunks(outer * inner, c, stats=True))
                        bn_stat.append(True)
                    elif n.op in ("neg", "sub"):
                        full = (B,) + tuple(n.shape)
                        out = self._act_ptr(mem, o, n.id, inputs)
                        x0 = self._act_ptr(mem, o, n.inputs[0], inputs)
                        s0 = (B,) + tuple(ir.node(n.inputs[0]).shape)
                        if n.op == "neg":
                            ew_pre.append(H.ew_map_row(out, full, x0, s0, ca=-1.0))
                        elif a["mode"] == "tt":
                            ew_pre.append(H.ew_map_row(out, full, x0, s0, ca=1.0,
                                                       b=self._act_ptr(mem, o, n.inputs[1], inputs),
                                                       b_shape=(B,) + tuple(ir.node(n.inputs[1]).shape), cb=-1.0))
                        elif a["mode"] == "tc":
                            ew_pre.append(H.ew_map_row(out, full, x0, s0, ca=1.0, c=-a["c"]))
                        else:
                            ew_pre.append(H.ew_map_row(out, full, x0, s0, ca=-1.0, c=a["c"]))
                    else:
                        raise ValueError(f"organism {o}: no kernel for op {n.op!r}")
            add_chunked("ew", 0, ew_pre, H.EW_DTYPE, [H.ew_count(r) for r in ew_pre], 1)
            # factorised genotype slices: E / C0 from the weights, then their partial (before the finalize)
            add_bin(0, bin_rows)
            add_bin(1, bin_rows)
            add_gemm(H.MODE_FWD, g_rows, g_dims, extra_fin=fin_rows)
            add_chunked("pool", 0, p_rows, H.POOL_DTYPE, p_cnt, H.POOL_ELEMS)
            add_convpool(cp_rows, False)
            if train:
                add_gchain([r for r in gc_rows if r["_bn"]], H.GC_FSTAT)
            add_gchain(gc_rows, H.GC_FAPPLY)
            add_nbn([r for r in nbn_rows if not r.get("_bin")], 2)
            add_nbn([r for r in nbn_rows if r.get("_bin")], 7, stats_only=True)
            if bn_rows:
                if train:
                    need0 = [i for i, need in enumerate(bn_stat) if need]      # (``sel`` is the organism filter)
                    add_chunked("bn", 0, [bn_rows[i] for i in need0], H.BN_DTYPE, [bn_cnt_st[i] for i in need0], 1)
                    add_chunked("bn", 2, bn_rows, H.BN_DTYPE, bn_cnt, 1)
                else:
                    add_chunked("bn", 3, bn_rows, H.BN_DTYPE, bn_cnt, 1)
            add_chunked("copy", 0, c_rows, H.COPY_DTYPE, c_cnt, 1)
            add_chunked("ew", 0, ew_post, H.EW_DTYPE, [H.ew_count(r) for r in ew_post], 1)

        if imcol:
            rows_ = [v["desc"] for v in imcol.values()]
            cnt_ = [-(-v["rows"] // H.IMCOL_ROWS) for v in imcol.values()]
            tiles_ = H.chunk_tiles(cnt_, 1)
            plan.launches.insert(0, Launch("imcol", 0, desc_tensor(rows_, H.IMCOL_DTYPE), T(tiles_), len(tiles_)))

        # ---- loss ------------------------------------------------------------------------------
        if metrics is not None:
            rows = []
            for o, lay in org_iter():
                ir = lay.ir
                rec = mem["orgs"][o]
                NC, L = ir.num_classes, ir.genotype_size
                rows.append(dict(logits=self._act_ptr(mem, o, ir.cls_head, inputs),
                                 dlogits=mem["grad"].ptr(rec["grad"][ir.cls_head]) if train else 0,
                                 labels=label_ptr, target=target_ptrs[o], metrics=metrics.data_ptr() + 32 * o,
                                 NC=NC, L=L, B=B, lb=self.lb[o]))
            plan.loss = (desc_tensor(rows, H.LOSS_DTYPE), len(rows), B)
        else:
            plan.loss = None

        plan.fwd_count = len(plan.launches)
        if not train:
            tables.flush(plan.keep)
            self._upload_fence()                     # as at the end of the train plan
            return plan

        # ---- backward --------------------------------------------------------------------------
        # Gradient buffers are written by several op kinds; the first writer of a buffer (in
        # execution order) overwrites it and later writers accumulate.  Two writers of one buffer
        # never share a launch.
        written = [set() for _ in range(P)]

        def target(o, nid):
            rec = mem["orgs"][o]
            own = rec["owner"][nid]
            if not rec["req"].get(own, False):
                return None
            return own

        trows, tcnt = [], []
        for o, lay in org_iter():
            ir = lay.ir
            for nid, off in lay.w.items():
                a = ir.node(nid).attrs
                if nid in mem["orgs"][o]["gc_nodes"]:
                    continue                      # fused genotype chain: no DGRAD launch
                if a["kind"] == "head_cls":
                    F_, P_, C_ = ir.num_classes + ir.genotype_size, 1, ir.head_features
                else:
                    F_, P_, C_ = a["f"], a["kh"] * a["kw"], a["cin"]
                # the transposed copy Wt[C][KH][KW][F] only feeds DGRAD kernels that cannot read the
                # natural layout, and only layers whose input needs a gradient have a DGRAD at all
                if nid in fcons[o]:
                    needs_dgrad = any(target(o, pid) is not None for pid, _, _ in fcat[o][fcons[o][nid]])
                else:
                    needs_dgrad = target(o, ir.node(nid).inputs[0]) is not None
                if not needs_dgrad or H.dgrad_reads_natural(a["kh"], a["kw"], a["sh"], a["sw"], F_):
                    continue
                trows.append(dict(src=wptr_bf(off), dst=self.wt.data_ptr() + 2 * self.wt_off[o][nid], F=F_, P=P_,
                                  C=C_))
                tcnt.append(-(-(F_ * P_ * C_) // H.TRANS_ELEMS))
        add_chunked("transpose", 0, trows, H.TRANS_DTYPE, tcnt, 1)

        # BatchNormalization whose input is the output of an activated GEMM used by nothing else: its
        # backward (phase 5) writes that GEMM's dZ = dx * act'(x) directly, so the GEMM's WGRAD / DGRAD
        # read dZ alone instead of dY and Y (SERANN_FOLD_BN_ACT=0 turns it off).  The same BN backward
        # reduces that GEMM's bias gradient from its fp32 dZ (BnDesc.pdb), so the WGRAD skips it
        dz_folded = [dict() for _ in range(P)]          # gemm id -> act code folded into the BN dx
        if os.environ.get("SERANN_FOLD_BN_ACT", "1") != "0":
            for o, lay in org_iter():
                ir = lay.ir
                rec = mem["orgs"][o]
                owner = rec["owner"]
                uses: Dict[int, int] = {}
                for n in ir.nodes:
                    if n.op == "reshape":
                        continue
                    for i in n.inputs:
                        uses[owner.get(i, i)] = uses.get(owner.get(i, i), 0) + 1
                for n in ir.nodes:
                    if n.op != "bn" or not n.attrs["last"] or n.id in rec["gc_nodes"]:
                        continue
                    src = ir.node(owner[n.inputs[0]])
                    if (src.op == "gemm" and src.attrs["kind"] not in ("head_cls", "head_rep")
                            and src.id not in rec["fused_convs"] and src.id not in rec["gc_nodes"]
                            and src.attrs["act"] in ("linear", "relu", "sigmoid")
                            and uses.get(src.id, 0) == 1 and rec["req"].get(src.id, False)):
                        dz_folded[o][src.id] = H.ACT_CODES[src.attrs["act"]]

        # A Dense(units=1) combined into a BatchNormalization's input by a subtraction (x = a - Dense(..): a mutant
        # form): its bias gradient is -sum(dx) of the BN, mathematically ~0 for a centred BN.  The BN
        # backward takes that sum in fp32 (BnDesc flags 128 / 256) and the Dense's WGRAD skips its bias: summed
        # from the bf16 dx the sub's broadcast reduction sees, it carried ~1000x torch-bf16's error
        sub_pdb = [dict() for _ in range(P)]            # bn id -> (gemm id, BnDesc flag)
        pdb_gemms = [set() for _ in range(P)]
        for o, lay in org_iter():
            ir = lay.ir
            rec = mem["orgs"][o]
            owner = rec["owner"]
            uses: Dict[int, int] = {}
            for n in ir.nodes:
                if n.op == "reshape":
                    continue
                for i in n.inputs:
                    uses[owner.get(i, i)] = uses.get(owner.get(i, i), 0) + 1
            for n in ir.nodes:
                if n.op != "bn":
                    continue
                sn = ir.node(owner[n.inputs[0]])
                if sn.op != "sub" or sn.attrs["mode"] != "tt" or uses.get(sn.id, 0) != 1:
                    continue
                srcs = [owner.get(i, i) for i in sn.inputs]
                if srcs[0] == srcs[1]:
                    continue
                for pos, gid in enumerate(srcs):
                    gn = ir.node(gid)
                    if (gn.op == "gemm" and gn.attrs["kind"] == "dense" and gid in lay.b
                            and gn.attrs["act"] == "linear" and gn.shape[-1] == 1 and uses.get(gid, 0) == 1
                            and gid not in rec["fused_convs"] and gid not in rec["gc_nodes"] and rec["req"].get(gid)):
                        sub_pdb[o][n.id] = (gid, 128 if pos == 1 else 256)
                        pdb_gemms[o].add(gid)
                        break

        STAGES = ("dgrad", "pool", "bn", "copy", "ew")
        for d in range(maxd, 0, -1):
            wg_rows, wg_dims = [], []
            bn_red, bn_red_cnt = [], []
            cpw_rows = []
            gcb_rows = []
            nbnb_rows, nbnf_rows = [], []
            bw_bin, bin_need = [], []           # factorised genotype slices of this depth (bnbn.hip)

            def bin_ws(n64, need=bin_need):
                """Reserve n64 int64 words of this depth's zeroed factorised-slice workspace (one memset launch);
                returns a deferred address: the workspace is allocated once the depth's sizes are known."""
                off = sum(need)
                need.append(-(-n64 // 32) * 32 + 32)
                return _Deferred(off)
            tasks = {s: [] for s in STAGES}     # stage -> [(o, owner|None, make_row(acc), count)]
            ew_bpre = []                        # non-last-axis BN: dy -> channels-last dyt
            for o, lay in org_iter():
                ir = lay.ir
                rec = mem["orgs"][o]
                for n in ir.nodes:
                    if depth_of[o][n.id] != d or n.op in ("input", "reshape"):
                        continue
                    if n.op == "gemm" and n.attrs["kind"] == "head_rep":
                        continue
                    a = n.attrs
                    if n.id in rec["gc_nodes"]:
                        if n.id in rec["gchain"]:
                            gcb_rows.append(gchain_row(o, n.id))
                        continue
                    if not rec["req"].get(n.id, False) or n.id in rec["fused_convs"] or n.id in nbn_src[o]:
                        continue
                    if n.op == "bn" and n.id in nbn[o]:
                        if n.id in nbnsum_rows[o]:
                            nbnf_rows.append(nbnsum_rows[o][n.id])   # sums reduced by the consumer's DGRAD
                        else:
                            nbnb_rows.append(nbn_row(o, n.id))     # BN backward + the Dense's WGRAD (nbn.hip)
                        continue
                    if n.op == "pool" and n.id in cpool[o]:
                        # fused pool backward + conv WGRAD + bias gradient (no DGRAD: raw image input)
                        cpw_rows.append(convpool_row(o, n, cpool[o][n.id]))
                        continue
                    if n.op == "gemm":
                        head = a["kind"] == "head_cls"
                        dz = mem["grad"].ptr(rec["grad"][n.id])
                        yv = self._act_ptr(mem, o, n.id, inputs)
                        if head:
                            NC, L, D = ir.num_classes, ir.genotype_size, ir.head_features
                            F, C, act = NC + L, D, 0
                            Hh = Ww = OH = OW = 1
                            KH = KW = SH = SW = 1
                        else:
                            F, C = a["f"], a["cin"]
                            Hh, Ww, OH, OW = a["h"], a["w"], a["oh"], a["ow"]
                            KH, KW, SH, SW = a["kh"], a["kw"], a["sh"], a["sw"]
                            # dZ already carries act' (written by the consuming BN's backward)
                            act = 0 if n.id in dz_folded[o] else H.ACT_CODES[a["act"]]
                        M = B * OH * OW
                        K = KH * KW * C
                        # a producer folded into its BN's backward gets its bias gradient from there (as does a
                        # Dense(units=1) subtracted from a BN input: sub_pdb)
                        dbias = gptr(lay.b[n.id]) if (n.id in lay.b and n.id not in dz_folded[o]
                                                      and n.id not in pdb_gemms[o]) else 0
                        xin = self._act_ptr(mem, o, n.inputs[0], inputs)
                        vec = (H.GF_VEC_A if F % 8 == 0 else 0) | (H.GF_VEC_B if C % 8 == 0 else 0)
                        ic = raw_conv_imcol(o, n) if not head else None
                        if n.id in fcons[o]:
                            # fused-concat consumer: WGRAD and DGRAD per K slice, in place on the concat
                            # inputs and their gradient buffers (no concat copy, no DGRAD for inputs
                            # without a gradient, e.g. the raw image)
                            D = C
                            sl, _ = concat_slices(o, n, F)
                            for q, (pid, col, width, ns, sb) in enumerate(sl):
                                bpid = binslice(o, pid, n.id)
                                if bpid is not None:
                                    # factorised genotype slice: H = dZ^T g and cs = column sums of dZ by one
                                    # WGRAD launch (Q40, plan-private zeroed buffers), then bin_s (the BN / Dense
                                    # backward sums for nbn phase 6) and bin_wg (dW, Adam) after this depth's WGRADs
                                    Lg = ir.genotype_size
                                    hq = bin_ws(F * Lg + F)                 # Q40 H [F][L], then cs [F]
                                    csq = hq + 8 * F * Lg
                                    wg_rows.append(dict(a=dz, b=inputs[o]["g"], out=hq, bias=csq, aux=yv, act=act,
                                                        H=Hh, W=1, C=Lg, OH=OH, OW=1, F=F, KH=1, KW=1, SH=1, SW=1, M=F,
                                                        N=Lg, K=M, flags=(H.GF_VEC_A if F % 8 == 0 else 0),
                                                        _nonarrow=1, _noadam=1))
                                    wg_dims.append((F, Lg, M))
                                    brow = dict(bin_desc(o, bpid, n.id, col, width), Hm=hq, cs=csq,
                                                dw=gptr(lay.w[n.id] + col), dbias=dbias if q == 0 else 0,
                                                adam=adam_ctx, _o=o, _bid=bpid)   # (part, ns: add_bin_sw)
                                    if (BIN_VEC4 and brow["F"] >= 4 and brow["ldw"] % 4 == 0 and brow["wc"] % 8 == 0
                                            and brow["dw"] % 32 == 0 and (brow["L"] * brow["F"]) % 4 == 0):
                                        brow["flags"] |= H.BIN_VEC4      # 4 columns per lane in bin_sw
                                    bw_bin.append(brow)
                                    if adam_ctx:
                                        plan.adam_regions.append(((gptr(lay.w[n.id] + col) - self.g.data_ptr()) // 8,
                                                                  F, width, D))
                                    continue
                                wg_rows.append(dict(a=dz, b=self._act_ptr(mem, o, pid, inputs), out=gptr(lay.w[n.id] + col),
                                                    bias=dbias if q == 0 else 0, aux=yv, act=act, H=Hh, W=1, C=width,
                                                    OH=OH, OW=1, F=F, KH=1, KW=1, SH=1, SW=1, M=F, N=width, K=M,
                                                    flags=(H.GF_VEC_A if F % 8 == 0 else 0), ldo=D, _nonarrow=1))
                                wg_dims.append((F, width, M))
                                own_p = target(o, pid)
                                if own_p is not None:
                                    base = dict(a=dz, b=self.wt.data_ptr() + 2 * (self.wt_off[o][n.id] + col * F),
                                                _bnat=wptr_bf(lay.w[n.id]) + 2 * col, _bnat_ld=D,
                                                aux=yv, act=act, out=mem["grad"].ptr(rec["grad"][own_p]), H=Hh, W=1,
                                                C=width, OH=OH, OW=1, F=F, KH=1, KW=1, SH=1, SW=1, M=M, N=width, K=F)
                                    sf = 0
                                    if own_p in nbnsum[o]:
                                        base["ext"] = nbnsum_ext(o, own_p, M, width)
                                        sf = H.GF_NBNSUM
                                    tasks["dgrad"].append((o, own_p, lambda acc, r=base, sf=sf: dict(r, flags=(H.GF_ACCUM if acc else 0) | sf),
                                                           (M, width, F)))
                            continue
                        if ic is not None:
                            wg_rows.append(dict(a=dz, b=ic["buf"].data_ptr(), out=gptr(lay.w[n.id]), bias=dbias,
                                                aux=yv, act=act, H=OH, W=OW, C=ic["K8"], OH=OH, OW=OW, F=F, KH=1, KW=1,
                                                SH=1, SW=1, M=F, N=K, K=M, flags=vec, _imcol=1))
                            wg_dims.append((F, K, M))
                        else:
                            # dZ = dY * act'(Y) on load; the bias gradient is reduced inside WGRAD
                            wg_rows.append(dict(a=dz, b=xin, out=gptr(lay.w[n.id]), bias=dbias, aux=yv, act=act,
                                                H=Hh, W=Ww, C=C, OH=OH, OW=OW, F=F, KH=KH, KW=KW, SH=SH, SW=SW,
                                                M=F, N=K, K=M, flags=vec))
                            wg_dims.append((F, K, M))
                        own = target(o, n.inputs[0])
                        if own is not None:
                            Mi = B * Hh * Ww
                            base = dict(a=dz, b=self.wt.data_ptr() + 2 * self.wt_off[o][n.id],
                                        _bnat=wptr_bf(lay.w[n.id]), aux=yv, act=act,
                                        out=mem["grad"].ptr(rec["grad"][own]), H=Hh,
                                        W=Ww, C=C, OH=OH, OW=OW, F=F, KH=KH, KW=KW, SH=SH, SW=SW, M=Mi, N=C,
                                        K=KH * KW * F)
                            sf = 0
                            if own in nbnsum[o]:
                                base["ext"] = nbnsum_ext(o, own, Mi, C)
                                sf = H.GF_NBNSUM
                            tasks["dgrad"].append((o, own, lambda acc, r=base, v=vec, sf=sf: dict(r, flags=v | sf | (H.GF_ACCUM if acc else 0)),
                                                   (Mi, C, KH * KW * F)))
                    elif n.op == "pool":
                        own = target(o, n.inputs[0])
                        if own is not None:
                            base = dict(idx=mem["u8"].ptr(rec["idx"][n.id]), dy=mem["grad"].ptr(rec["grad"][n.id]),
                                        dx=mem["grad"].ptr(rec["grad"][own]), B=B, H=a["h"], W=a["w"], C=a["c"],
                                        OH=a["oh"], OW=a["ow"], PH=a["ph"], PW=a["pw"], SH=a["sh"], SW=a["sw"])
                            tasks["pool"].append((o, own, lambda acc, r=base: dict(r, flags=1 if acc else 0),
                                                  H.pool_units(B * a["h"] * a["w"] * a["c"], a["c"])))
                    elif n.op == "bn" and a["last"]:
                        bd = rec["bn"][n.id]
                        c = a["channels"]
                        R = B * math.prod(n.shape) // c
                        own = target(o, n.inputs[0])
                        pflags = (1 if n.id in lay.gamma else 0) | (2 if n.id in lay.beta else 0)
                        base = dict(x=self._act_ptr(mem, o, n.inputs[0], inputs),
                                    dy=mem["grad"].ptr(rec["grad"][n.id]),
                                    dx=mem["grad"].ptr(rec["grad"][own]) if own is not None else 0,
                                    gamma=pptr(lay.gamma[n.id]) if n.id in lay.gamma else 0,
                                    mean=f32a.ptr(bd["mean"]), invstd=f32a.ptr(bd["invstd"]),
                                    ws=mem["ws"].ptr(bd["wsb"]),
                                    dgamma=gptr(lay.gamma[n.id]) if n.id in lay.gamma else 0,
                                    dbeta=gptr(lay.beta[n.id]) if n.id in lay.beta else 0,
                                    R=R, C=c, eps=a["epsilon"], momentum=a["momentum"])
                        bn_red.append(dict(base, flags=pflags))
                        bn_red_cnt.append(H.bn_chunks(R, c, stats=True))
                        if own is not None and own in dz_folded[o]:
                            pflags |= dz_folded[o][own] << 4
                            if own in lay.b:
                                base = dict(base, pdb=gptr(lay.b[own]))
                        elif n.id in sub_pdb[o]:
                            gid, pf = sub_pdb[o][n.id]
                            pflags |= pf
                            base = dict(base, pdb=gptr(lay.b[gid]))
                        if own is None:
                            tasks["bn"].append((o, None, lambda acc, r=base, f=pflags: dict(r, flags=f | 8),
                                                H.bn_chunks(R, c)))
                        else:
                            tasks["bn"].append((o, own, lambda acc, r=base, f=pflags: dict(r, flags=f | (4 if acc else 0)),
                                                H.bn_chunks(R, c)))
                    elif n.op == "concat":
                        if n.id in fcat[o]:
                            continue                  # its consumers' DGRAD slices wrote the input gradients
                        ax = a["axis"]
                        outer = B * math.prod(n.shape[:ax - 1])
                        out_inner = math.prod(n.shape[ax - 1:])
                        col = 0
                        dyp = mem["grad"].ptr(rec["grad"][n.id])
                        for i in n.inputs:
                            inner = math.prod(ir.node(i).shape[ax - 1:])
                            own = target(o, i)
                            if own is not None:
                                base = dict(src=dyp + col * 2, dst=mem["grad"].ptr(rec["grad"][own]), rows=outer,
                                            cols=inner, src_stride=out_inner, dst_stride=inner)
                                tasks["copy"].append((o, own, lambda acc, r=base: dict(r, flags=1 if acc else 0),
                                                      -(-outer // H.COPY_ROWS)))
                            col += inner
                    elif n.op == "bn":
                        # non-last axis (see the forward): BN backward on the channels-last copies, dx
                        # transposed back into the input's gradient
                        bd = rec["bn"][n.id]
                        c = a["channels"]
                        full = (B,) + tuple(n.shape)
                        outer, inner = math.prod(full[:a["axis"]]), math.prod(full[a["axis"] + 1:])
                        R = outer * inner
                        dyt, dxt = mem["grad"].ptr(bd["dyt"]), mem["grad"].ptr(bd["dxt"])
                        ew_bpre.append(H.ew_permute_row(dyt, mem["grad"].ptr(rec["grad"][n.id]), (outer, c, inner),
                                                        (0, 2, 1)))
                        own = target(o, n.inputs[0])
                        pflags = (1 if n.id in lay.gamma else 0) | (2 if n.id in lay.beta else 0)
                        base = dict(x=mem["act"].ptr(bd["xt"]), dy=dyt, dx=dxt,
                                    gamma=pptr(lay.gamma[n.id]) if n.id in lay.gamma else 0,
                                    mean=f32a.ptr(bd["mean"]), invstd=f32a.ptr(bd["invstd"]),
                                    ws=mem["ws"].ptr(bd["wsb"]),
                                    dgamma=gptr(lay.gamma[n.id]) if n.id in lay.gamma else 0,
                                    dbeta=gptr(lay.beta[n.id]) if n.id in lay.beta else 0,
                                    R=R, C=c, eps=a["epsilon"], momentum=a["momentum"])
                        bn_red.append(dict(base, flags=pflags))
                        bn_red_cnt.append(H.bn_chunks(R, c, stats=True))
                        # dxt is private to this BN: overwritten (no accumulate); no dx at all without a target
                        if n.id in sub_pdb[o] and own is not None:
                            gid, pf = sub_pdb[o][n.id]
                            base = dict(base, pdb=gptr(lay.b[gid]), flags=pflags | pf)
                            pf5 = pflags | pf
                        else:
                            pf5 = pflags
                        tasks["bn"].append((o, None, lambda acc, r=base, f=pf5, t=own: dict(r, flags=f | (8 if t is None else 0)),
                                            H.bn_chunks(R, c)))
                        if own is not None:
                            tasks["ew"].append((o, own, lambda acc, r=(mem["grad"].ptr(rec["grad"][own]), dxt, (outer, inner, c)):
                                                H.ew_permute_row(r[0], r[1], r[2], (0, 2, 1), accum=acc),
                                                -(-B * math.prod(n.shape) // H.EW_ELEMS)))
                    elif n.op in ("neg", "sub"):
                        dy = mem["grad"].ptr(rec["grad"][n.id])
                        full = (B,) + tuple(n.shape)
                        if n.op == "neg":
                            scales = [-1.0]
                        elif a["mode"] == "tt":
                            scales = [1.0, -1.0]
                        else:
                            scales = [1.0 if a["mode"] == "tc" else -1.0]
                        for i, sc in zip(n.inputs, scales):
                            own = target(o, i)
                            if own is None:
                                continue
                            oshape = (B,) + tuple(ir.node(i).shape)
                            tasks["ew"].append((o, own, lambda acc, r=(mem["grad"].ptr(rec["grad"][own]), oshape, dy, full, sc):
                                                H.ew_reduce_row(r[0], r[1], r[2], r[3], r[4], accum=acc),
                                                -(-math.prod(oshape) // H.EW_ELEMS)))
                    else:
                        raise ValueError(f"organism {o}: no backward kernel for op {n.op!r}")
            add_convpool(cpw_rows, True)
            add_gchain([r for r in gcb_rows if r["_bn"]], H.GC_BSTAT)
            add_gchain(gcb_rows, H.GC_BFULL)
            add_chunked("ew", 0, ew_bpre, H.EW_DTYPE, [H.ew_count(r) for r in ew_bpre], 1)
            if bn_red:
                add_chunked("bn", 4, bn_red, H.BN_DTYPE, bn_red_cnt, 1)
            add_nbn(nbnb_rows, 4)
            add_nbn(nbnb_rows, 5)
            add_nbn(nbnf_rows, 6)
            for stage in STAGES:
                batches = [[]]
                used = [set()]
                for o, own, make, cnt in tasks[stage]:
                    key = (o, own) if own is not None else None
                    if key is not None and key in used[-1]:
                        batches.append([])
                        used.append(set())
                    acc = own is not None and own in written[o]
                    batches[-1].append((make(acc), cnt))
                    if key is not None:
                        used[-1].add(key)
                        written[o].add(own)
                for b in batches:
                    if not b:
                        continue
                    rows = [r for r, _ in b]
                    cnts = [c for _, c in b]
                    if stage == "dgrad":
                        add_gemm(H.MODE_DGRAD, rows, cnts)
                    elif stage == "pool":
                        add_chunked("pool", 1, rows, H.POOL_DTYPE, cnts, H.POOL_ELEMS)
                    elif stage == "bn":
                        add_chunked("bn", 5, rows, H.BN_DTYPE, cnts, 1)
                    elif stage == "ew":
                        add_chunked("ew", 0, rows, H.EW_DTYPE, cnts, 1)
                    else:
                        add_chunked("copy", 0, rows, H.COPY_DTYPE, cnts, 1)
            # WGRAD after this depth's DGRAD: a WGRAD that applies Adam to its tile (GF_ADAM) rewrites the
            # bf16 weights the layer's DGRAD reads
            if adam_ctx:
                for r in wg_rows:
                    if not r.get("_noadam"):
                        r["adam"] = adam_ctx
            if bin_need:
                wsz = torch.empty(sum(bin_need) + 64, dtype=torch.int64, device=self.device)
                plan.keep.append(wsz)
                base_ = wsz.data_ptr()
                for r in wg_rows:
                    for k_ in ("out", "bias"):
                        if isinstance(r.get(k_), _Deferred):
                            r[k_] = r[k_].resolve(base_)
                for r in bw_bin:
                    for k_ in ("Hm", "cs"):
                        r[k_] = r[k_].resolve(base_)
                plan.launches.append(Launch("memset", (base_, 2 * wsz.numel()), None, None, 0))
            add_gemm(H.MODE_WGRAD, wg_rows, wg_dims)
            add_bin_sw(bw_bin)
        # descriptor / tile tables are uploaded from pageable host memory: fence them before a launch can
        # read them.  Plans are built once per generation, so this costs nothing on the training hot path.
        tables.flush(plan.keep)
        self._upload_fence()
        return plan

    def _upload_fence(self):
        """Device-wide synchronize (uploads and any outstanding work on other streams) -- or, for a plan
        built by fit's background thread while the captured training graph runs, only the building thread's
        upload stream."""
        if self.device.type != "cuda":
            return
        if getattr(self._bg, "stream_only", False):
            torch.cuda.current_stream(self.device).synchronize()
        else:
            torch.cuda.synchronize(self.device)

    # ---------------------------------------------------------------------------------------------
    # execution
    # ---------------------------------------------------------------------------------------------
    def _run_loss(self, plan: Plan, train: bool, nvalid: int):
        if plan.loss is None:
            return
        descs, P, B = plan.loss
        self.lib.loss(1 if train else 0, descs.data_ptr(), P, B, H.stream_handle(), nvalid)

    def fit(self, data, cfg: Optional[TrainConfig] = None) -> FitResult:
        cfg = cfg or self.cfg
        dev = self.device
        dd = device_data(data, dev)
        P = self.num_organisms
        n = dd["train_x"].shape[0]
        split = cfg.split(n)
        steps = cfg.steps_per_epoch(split)
        B = cfg.batch_size
        xcols, gcols = dd["train_x"].shape[1], dd["train_g"].shape[1]

        # shared batch buffers
        xb = _padded_zeros((B, xcols), torch.bfloat16, dev)
        gb = _padded_zeros((B, gcols), torch.bfloat16, dev)
        yb = torch.zeros(B, dtype=torch.int32, device=dev)
        perm_t = torch.zeros(max(split, 1), dtype=torch.int32, device=dev)
        counter = torch.zeros(1, dtype=torch.int32, device=dev)
        metrics = torch.zeros(P, 4, dtype=torch.int64, device=dev)      # Q32 fixed point (aux.hip loss_kernel)

        self.diverged.zero_()                       # (flags of this fit only)
        # binary genotype batches enable the factorised genotype-slice path (bnbn.hip); checked on the host data
        self._g_binary = _is_binary(data.train_g)
        t_plan = time.perf_counter()
        mem = self._alloc_buffers(B, with_grads=True)
        self.timings["alloc_s"] = time.perf_counter() - t_plan
        self._train_mem = mem
        inputs = [{"X": xb.data_ptr(), "g": gb.data_ptr()} for _ in range(P)]
        targets = [gb.data_ptr()] * P
        # Organisms are independent: split them into stream groups (LPT on FLOPs) with one plan each,
        # so the level-by-level launches of different groups overlap on the GPU (fork/join inside the
        # captured graph).  One group = the single-stream schedule.
        groups = self._stream_groups(int(os.environ.get("SERANN_STREAMS", "4")))
        # WGRAD tiles with a single writer apply Adam in their epilogue (SERANN_FUSE_ADAM=0: the arena pass
        # does every parameter)
        actx = np.zeros(1, dtype=H.ADAM_CTX_DTYPE)
        actx[0] = (self.p.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), self.pbf.data_ptr(), self.g.data_ptr(),
                   self.lr_t.data_ptr(), self.org_off.data_ptr(), self.diverged.data_ptr(), self.num_organisms,
                   cfg.beta1, cfg.beta2, cfg.eps, self.mom_mode)
        self._adam_ctx = torch.as_tensor(np.frombuffer(actx.tobytes(), dtype=np.uint8).copy(), device=dev)
        actx_ptr = self._adam_ctx.data_ptr() if os.environ.get("SERANN_FUSE_ADAM", "1") != "0" else 0
        plans = [self._build_plan("train", B, mem, inputs, yb.data_ptr(), targets, metrics, orgs=g_, adam_ctx=actx_ptr)
                 for g_ in groups]

        def skip_mask(pls):
            regions = [r for pl in pls for r in pl.adam_regions]
            if not regions:
                return None
            return H.adam_skip_mask_device(self.p.numel(), regions, dev)
        skip_main = skip_mask(plans)
        if not hasattr(self, "_streams") or len(self._streams) < len(plans):
            self._streams = [torch.cuda.Stream(device=dev) for _ in plans]
        streams = self._streams[:len(plans)]
        L = self.lib
        ws = mem["ws"].t

        def run_plan(pl):
            tmp = Plan()
            tmp.launches = pl.launches[:pl.fwd_count]
            tmp.run()
            if pl.loss is not None:
                self._run_loss(pl, True, pl.loss[2])
            tmp.launches = pl.launches[pl.fwd_count:]
            tmp.run()

        # Keras trains the last step of an epoch on the true remainder (split % B rows), so that step has
        # its own plan (BatchNorm batch statistics, loss mean, gradients and accuracy over Br rows) and
        # its own activation buffers; it reads the first Br rows of the shared batch buffers.
        full_steps = split // B
        Br = split - full_steps * B
        rem = {"plans": None, "ws": None, "skip": None}

        def build_rest():
            """The remainder step's plans (and the validation plan): built while the captured graph runs
            the first epoch's full steps when possible (:func:`start_rest`), else before training."""
            if Br > 0 and steps > full_steps:
                mem_r = self._alloc_buffers(Br, with_grads=True)
                self._train_mem_rem = mem_r
                rem["plans"] = [self._build_plan("train", Br, mem_r, inputs, yb.data_ptr(), targets, metrics,
                                                 orgs=g_, adam_ctx=actx_ptr) for g_ in groups]
                rem["ws"] = mem_r["ws"].t
                rem["skip"] = skip_mask(rem["plans"])
            self._infer_plan(B)
        bg = {"thread": None, "err": None, "stream": None}

        def start_rest():
            if dev.type != "cuda":
                build_rest()
                return
            side = bg["stream"] = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream())

            def work():
                self._bg.stream_only = True
                try:
                    with torch.cuda.stream(side):
                        build_rest()
                except BaseException as e:        # re-raised by join_rest on the fitting thread
                    bg["err"] = e
                finally:
                    self._bg.stream_only = False
            bg["thread"] = threading.Thread(target=work, name="serann-plan-build", daemon=True)
            self._plan_thread = bg["thread"]                  # close() joins it if fit() is left early
            bg["thread"].start()

        def join_rest():
            if bg["thread"] is not None:
                bg["thread"].join()
                bg["thread"] = None
                if bg["err"] is not None:
                    raise bg["err"]
                torch.cuda.current_stream().wait_stream(bg["stream"])
            self._adam_skip = (skip_main, rem["skip"])       # referenced by the captured graph

        def step(pls=plans, nb=B, wsb=ws, base=0, ctr=True, skip=skip_main):
            s = H.stream_handle()
            L.gather_batch(dd["train_x"].data_ptr(), dd["train_g"].data_ptr(), dd["train_y"].data_ptr(),
                           perm_t.data_ptr(), counter.data_ptr() if ctr else 0, base, nb, split, xcols, gcols,
                           xb.data_ptr(), gb.data_ptr(), yb.data_ptr(), s)
            L.memset32(wsb.data_ptr(), 2 * wsb.numel(), s)          # int64 workspace
            # step counter and lr_t first: the fused WGRAD epilogues read lr_t during the backward
            L.adam_scalars(self.step_i.data_ptr(), self.lr_t.data_ptr(), cfg.lr, cfg.beta1, cfg.beta2, s)
            if len(pls) == 1:
                run_plan(pls[0])
            else:
                main = torch.cuda.current_stream()
                for st in streams:
                    st.wait_stream(main)
                for pl, st in zip(pls, streams):
                    with torch.cuda.stream(st):
                        run_plan(pl)
                for st in streams:
                    main.wait_stream(st)
            s = H.stream_handle()
            L.adam_update(self.p.data_ptr(), self.g.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                          self.pbf.data_ptr(), self.lr_t.data_ptr(), self.p.numel(), cfg.beta1, cfg.beta2, cfg.eps,
                          skip.data_ptr() if skip is not None else 0, s, self.mom_mode, self.org_off.data_ptr(),
                          self.diverged.data_ptr(), self.num_organisms)
            L.counter_add(counter.data_ptr(), 1, s)

        def remainder_step():
            step(rem["plans"], Br, rem["ws"], full_steps * B, False, rem["skip"])

        use_graph = full_steps > 1
        graph = None
        if not (use_graph and cfg.epochs > 0 and min(steps, full_steps) > 1):
            build_rest()                        # no captured graph to overlap with
            join_rest()
        self.timings["plan_s"] = time.perf_counter() - t_plan
        self.timings["launches_per_step"] = sum(len(pl.launches) for pl in plans) + 5
        self.timings["stream_groups"] = len(plans)

        t0 = time.perf_counter()
        train_acc = np.zeros(P)
        val_acc = np.full(P, np.nan)
        val_mse = np.full(P, np.nan)
        total = 0
        try:
            train_acc, val_acc, val_mse, total, graph = self._fit_epochs(
                cfg, split, n, steps, full_steps, use_graph, perm_t, counter, metrics, dd, step, remainder_step,
                start_rest, join_rest, rem, train_acc, val_acc, val_mse, total, graph)
        finally:
            if bg["thread"] is not None:                   # left early (HIP error, interrupt): never leave the
                bg["thread"].join()                        # builder thread allocating behind our back
                bg["thread"] = None
        torch.cuda.synchronize(dev)
        self._train_mem = mem
        self.graph = graph
        # every buffer the captured graph addresses lives as long as the graph does
        self._fit_bufs = (xb, gb, yb, perm_t, counter, metrics, plans, rem["plans"])
        div = self.diverged_mask()
        if div.any():
            # a gradient beyond fp16's range: the reference's float16 graph ends such an organism with NaN weights
            # and NaN metrics (common.h flag_diverged)
            train_acc, val_acc, val_mse = (np.where(div, np.nan, a) for a in (train_acc, val_acc, val_mse))
        return FitResult(train_acc, val_acc, val_mse, time.perf_counter() - t0, total,
                         extra={"plan_s": self.timings["plan_s"], "alloc_s": self.timings["alloc_s"],
                                "diverged": np.flatnonzero(div).tolist(),
                                "launches_per_step": self.timings["launches_per_step"]})

    def _fit_epochs(self, cfg, split, n, steps, full_steps, use_graph, perm_t, counter, metrics, dd, step,
                    remainder_step, start_rest, join_rest, rem, train_acc, val_acc, val_mse, total, graph):
        """The epoch loop of :meth:`fit`: capture on the first full step, replay the rest, remainder step,
        validation.  Returns (train_acc, val_acc, val_mse, steps run, graph)."""
        dev = self.device
        for epoch in range(cfg.epochs):
            perm = epoch_permutation(cfg.seed, epoch, split).astype(np.int32)
            perm_t.copy_(torch.from_numpy(perm))
            counter.zero_()
            metrics.zero_()
            nfull = min(steps, full_steps)
            if use_graph and graph is None and nfull > 1:
                # warm one step eagerly (first-touch), then capture
                step()
                total += 1
                s_ = torch.cuda.Stream(device=dev)
                s_.wait_stream(torch.cuda.current_stream())
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.stream(s_):
                    with torch.cuda.graph(graph, stream=s_):
                        step()
                torch.cuda.current_stream().wait_stream(s_)
                remaining = nfull - 1
                start_rest()                    # CPU-side plan building overlaps the replays below
            else:
                remaining = nfull
            ev = None
            if graph is not None and remaining > 0 and "replay_ms_per_step" not in self.timings:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            for _ in range(remaining):
                if graph is not None:
                    graph.replay()
                else:
                    step()
                total += 1
            if ev is not None:
                # device time per replayed training step of this shard (cost-model calibration, profiling)
                ev[1].record()
                ev[1].synchronize()
                self.timings["replay_ms_per_step"] = ev[0].elapsed_time(ev[1]) / remaining
            join_rest()
            if rem["plans"] is not None and steps > nfull:
                remainder_step()
                total += 1
            m = H.from_q32(metrics)
            train_acc = m[:, 1] / np.maximum(m[:, 3], 1)
            if cfg.val_every_epoch or epoch == cfg.epochs - 1:
                val_acc, val_mse = self._evaluate_rows(dd["train_x"], dd["train_g"], dd["train_y"], split, n, cfg)
        return train_acc, val_acc, val_mse, total, graph

    # ---------------------------------------------------------------------------------------------
    def export_arena(self, i: int, arena: torch.Tensor) -> Dict[int, Dict[str, np.ndarray]]:
        """Export organism ``i``'s slice of an arena shaped like the parameters (e.g. gradients)."""
        saved = self.p
        try:
            self.p = arena
            out = self.export_params(i)
        finally:
            self.p = saved
        return out

    def debug_train_step(self, x: np.ndarray, g: np.ndarray, y: np.ndarray, apply_adam: bool = False):
        """One training step on an explicit batch WITHOUT graph capture; returns (grad arena copy,
        metrics).  Used by the numerics tests against the torch oracle."""
        dev = self.device
        B = len(x)
        # kernel operands keep the fragment-load slack behind them (hip_ops.operand)
        xb = H.padded(torch.as_tensor(np.ascontiguousarray(x.reshape(B, -1)), dtype=torch.float32, device=dev).to(torch.bfloat16))
        gb = H.padded(torch.as_tensor(np.ascontiguousarray(g), dtype=torch.float32, device=dev).to(torch.bfloat16))
        yb = H.padded(torch.as_tensor(y.astype(np.int32), device=dev))
        metrics = torch.zeros(self.num_organisms, 4, dtype=torch.int64, device=dev)
        mem = self._alloc_buffers(B, with_grads=True)
        inputs = [{"X": xb.data_ptr(), "g": gb.data_ptr()} for _ in range(self.num_organisms)]
        self._g_binary = _is_binary(g)
        plan = self._build_plan("train", B, mem, inputs, yb.data_ptr(), [gb.data_ptr()] * self.num_organisms, metrics)
        s = H.stream_handle()
        self.g.zero_()
        self.lib.memset32(mem["ws"].t.data_ptr(), 2 * mem["ws"].t.numel(), s)
        fwd = Plan()
        fwd.launches = plan.launches[:plan.fwd_count]
        fwd.run()
        self._run_loss(plan, True, B)
        bwd = Plan()
        bwd.launches = plan.launches[plan.fwd_count:]
        bwd.run()
        grads = H.from_qg(self.g)
        if apply_adam:
            c = self.cfg
            self.lib.adam(self.p.data_ptr(), self.g.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), self.pbf.data_ptr(),
                          self.step_i.data_ptr(), self.lr_t.data_ptr(), self.p.numel(), c.lr, c.beta1, c.beta2, c.eps, s,
                          self.mom_mode)
        torch.cuda.synchronize(dev)
        self._debug_mem = mem
        self._debug_plan = plan                          # (tests inspect its launches)
        return grads, H.from_q32(metrics)

    def debug_logits(self, mem=None) -> List[np.ndarray]:
        mem = mem or self._debug_mem
        out = []
        for i, lay in enumerate(self.layouts):
            ir = lay.ir
            NC, L = ir.num_classes, ir.genotype_size
            kind, off = mem["orgs"][i]["act"][ir.cls_head]
            out.append(mem["f32"].view(off, mem["B"] * (NC + L)).view(mem["B"], NC + L).cpu().numpy())
        return out

    # ---------------------------------------------------------------------------------------------
    def _infer_plan(self, B):
        key = ("infer", B)
        if key not in self.plans:
            dev = self.device
            xcols = self.layouts[0].ir.nodes[0].shape[0] * self.layouts[0].ir.nodes[0].shape[1]
            gcols = self.layouts[0].ir.genotype_size
            xb = _padded_zeros((B, xcols), torch.bfloat16, dev)
            gb = _padded_zeros((B, gcols), torch.bfloat16, dev)
            yb = torch.zeros(B, dtype=torch.int32, device=dev)
            metrics = torch.zeros(self.num_organisms, 4, dtype=torch.int64, device=dev)
            mem = getattr(self, "_train_mem", None)
            if mem is None or mem["B"] != B:
                mem = self._alloc_buffers(B, with_grads=False)
            inputs = [{"X": xb.data_ptr(), "g": gb.data_ptr()} for _ in range(self.num_organisms)]
            plan = self._build_plan("infer", B, mem, inputs, yb.data_ptr(), [gb.data_ptr()] * self.num_organisms,
                                    metrics)
            self.plans[key] = (plan, xb, gb, yb, metrics, mem)
        return self.plans[key]

    def _evaluate_rows(self, X, G, Y, start, end, cfg):
        P = self.num_organisms
        n = end - start
        if n <= 0:
            return np.full(P, np.nan), np.full(P, np.nan)
        B = cfg.batch_size
        plan, xb, gb, yb, metrics, mem = self._infer_plan(B)
        metrics.zero_()
        perm = torch.arange(start, end, dtype=torch.int32, device=self.device)
        L = self.lib
        for base in range(0, n, B):
            s = H.stream_handle()
            L.gather_batch(X.data_ptr(), G.data_ptr(), Y.data_ptr(), perm.data_ptr(), 0, base, B, n, X.shape[1],
                           G.shape[1], xb.data_ptr(), gb.data_ptr(), yb.data_ptr(), s)
            plan.run()
            self._run_loss(plan, False, min(B, n - base))
        m = H.from_q32(metrics)
        return m[:, 1] / np.maximum(m[:, 3], 1), m[:, 2] / np.maximum(m[:, 3], 1)

    def evaluate(self, x, labels, g, cfg: Optional[TrainConfig] = None) -> np.ndarray:
        cfg = cfg or self.cfg
        dd = device_data_for_arrays(x, labels, g, self.device)
        acc, _ = self._evaluate_rows(dd["x"], dd["g"], dd["y"], 0, len(x), cfg)
        return np.where(self.diverged_mask(), np.nan, acc)

    def diverged_mask(self) -> np.ndarray:
        """Organisms whose last fit produced a gradient element beyond fp16's range (csrc/hip/common.h
        flag_diverged): bool [P]."""
        return self.diverged[:self.num_organisms].cpu().numpy() != 0

    def _rep_plan(self, B: int):
        """Forward-only plan of the replication step at batch B, cached per B: per-organism input
        buffers (each organism runs on its OWN rows), the inference plan over them,
        and the fused replication epilogue's descriptors (sigmoid -> fp16 -> round -> bit-pack, K16)."""
        key = ("rep", B)
        if key not in self.plans:
            P, dev = self.num_organisms, self.device
            n0 = self.layouts[0].ir.nodes[0]
            xcols = int(math.prod(n0.shape))
            L = self.layouts[0].ir.genotype_size
            xs = _padded_zeros((P, B, xcols), torch.bfloat16, dev)
            gs = _padded_zeros((P, B, L), torch.bfloat16, dev)
            mem = self._alloc_buffers(B, with_grads=False)
            inputs = [{"X": xs[i].data_ptr(), "g": gs[i].data_ptr()} for i in range(P)]
            plan = self._build_plan("infer", B, mem, inputs)
            nbytes = (L + 7) // 8
            bits = torch.zeros(P, B, nbytes, dtype=torch.uint8, device=dev)
            rows = []
            for i, lay in enumerate(self.layouts):
                ir = lay.ir
                kind, off = mem["orgs"][i]["act"][ir.cls_head]
                rows.append((mem["f32"].ptr(off), bits[i].data_ptr(), B, ir.num_classes, ir.genotype_size))
            d = np.array(rows, dtype=H.REPBITS_DTYPE)
            descs = torch.as_tensor(np.frombuffer(d.tobytes(), dtype=np.uint8).copy(), device=dev)
            torch.cuda.synchronize(dev)
            self.plans[key] = dict(plan=plan, xs=xs, gs=gs, mem=mem, bits=bits, descs=descs)
        return self.plans[key]

    def _replicate_chunks(self, genotypes, images, cfg, packed: bool):
        cfg = cfg or self.cfg
        P = self.num_organisms
        pool = len(images[0]) if P else 0
        B = min(pool, cfg.batch_size)
        rp = self._rep_plan(B)
        dev = self.device
        L = self.layouts[0].ir.genotype_size
        g = torch.as_tensor(np.asarray(genotypes, np.float32), device=dev).to(torch.bfloat16)
        rp["gs"][:] = g[:, None, :]
        outs = []
        for c0 in range(0, pool, B):
            nb = min(B, pool - c0)
            rp["xs"][:, :nb] = torch.as_tensor(np.stack([im[c0:c0 + nb].reshape(nb, -1) for im in images]),
                                               dtype=torch.float32, device=dev).to(torch.bfloat16)
            rp["plan"].run()
            if packed:
                self.lib.rep_bits(rp["descs"].data_ptr(), P, B, (L + 7) // 8, H.stream_handle())
                outs.append(rp["bits"][:, :nb].clone())
            else:
                mem = rp["mem"]
                chunk = []
                for i, lay in enumerate(self.layouts):
                    ir = lay.ir
                    NC = ir.num_classes
                    kind, off = mem["orgs"][i]["act"][ir.cls_head]
                    logits = mem["f32"].view(off, B * (NC + L)).view(B, NC + L)
                    chunk.append(torch.sigmoid(logits[:nb, NC:]).half().float())
                outs.append(torch.stack(chunk))
        return torch.cat(outs, 1)

    def replicate(self, genotypes, images, cfg: Optional[TrainConfig] = None) -> List[np.ndarray]:
        """Sigmoid replication outputs (fp16-rounded, as Keras predicts in fp16) per organism."""
        P = self.num_organisms
        if P == 0 or len(images[0]) == 0:
            return [np.zeros((0, self.layouts[i].ir.genotype_size), np.float32) for i in range(P)]
        out = self._replicate_chunks(genotypes, images, cfg, packed=False).cpu().numpy()
        return [out[i] for i in range(P)]

    def replicate_packed(self, genotypes, images, cfg: Optional[TrainConfig] = None) -> torch.Tensor:
        """Offspring genotypes as packed bits straight from the fused epilogue: a device tensor
        [P][pool][ceil(L / 8)] uint8 (numpy.packbits order) that feeds the all-gather without a host hop."""
        P = self.num_organisms
        L = self.layouts[0].ir.genotype_size if P else 0
        if P == 0 or len(images[0]) == 0:
            return torch.zeros(P, 0, (L + 7) // 8, dtype=torch.uint8, device=self.device)
        return self._replicate_chunks(genotypes, images, cfg, packed=True)

    def close(self):
        """Release every device resource the engine owns besides its parameters: the captured graph first
        (its replay addresses the buffers below), then plans, activation / gradient buffers, descriptor
        tables and side streams.  Waits for the device first, so nothing in flight still reads them."""
        th = getattr(self, "_plan_thread", None)
        if th is not None:                      # a plan-builder thread of an interrupted fit() still running
            th.join()
            self._plan_thread = None
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.graph = None
        self.plans.clear()
        for name in ("_fit_bufs", "_train_mem", "_train_mem_rem", "_debug_mem", "_debug_plan", "_adam_skip", "_adam_ctx", "_streams"):
            if hasattr(self, name):
                delattr(self, name)


def device_data_for_arrays(x, labels, g, device):
    """Upload an evaluation set (x, labels, g) once per x array and device (weak-keyed on x: freed with
    it); labels / g are matched by identity through weak references."""
    per_x = _DEVICE_DATA.setdefault(x, {})
    d = per_x.get(str(device))
    if d is not None and not (d["_labels"]() is labels and d["_g"]() is g):
        d = None
    if d is None:
        d = {"x": torch.as_tensor(np.ascontiguousarray(x.reshape(len(x), -1)), dtype=torch.float32).to(device).to(
            torch.bfloat16),
             "g": torch.as_tensor(np.ascontiguousarray(g), dtype=torch.float32).to(device).to(torch.bfloat16),
             "y": torch.as_tensor(labels.astype(np.int32), device=device),
             "_labels": weakref.ref(labels), "_g": weakref.ref(g)}
        per_x[str(device)] = d
    return d
