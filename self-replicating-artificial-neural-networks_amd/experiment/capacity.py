"""Shard capacity: GPU-memory admission, training waves and the out-of-memory fallback.

Reference behaviour being replaced:

* ``run_experiment.py:100-104`` admits a worker to the pool only with >= 6000 MB of free GPU memory
  (``min_gpu_memory_required``) and sizes jobs by ``max_serann_per_gpu = 112`` organisms
  (``evolutionary_experiment/config.py:8``) -- a V100-era constant: a pop-1000 generation becomes 9 jobs.
* ``experiment_worker.py:121-126`` catches *any* exception of ``fit`` and retries once at half the batch.

Here a rank trains its whole shard in one engine when the shard fits in HBM (288 GB per MI355X: a
125-organism shard needs a few GB), and otherwise in *waves*: consecutive groups of organisms, each
trained by its own engine, sized from an estimate of every organism's device bytes
(:func:`organism_device_bytes`) against the free HBM.  Waves change nothing numerically -- every
reduction split is a function of the organism's own problem (``ops/hip_ops.py``) and partial sums meet
in order-free fixed point (``csrc/hip/common.h``), and the epoch permutation is per generation -- so an
organism trains bit-identically in any wave.  An out-of-memory error (the estimate is conservative but
not a guarantee) splits the failing wave in two and retries; a single organism that still does not fit
falls back to the reference's half-batch retry, and after that is reported as failed (NaN metrics, no
offspring) instead of crashing the generation.
"""
from __future__ import annotations

import math
import os
from typing import Callable, List, Optional, Sequence

ENV_BUDGET = "SERANN_HBM_BUDGET_GB"        # override the per-rank device budget (tests, shared GPUs)
HBM_FRACTION = 0.85                        # of the free HBM a rank plans with
MIN_GPU_MEMORY_MB = 6000                   # reference admission threshold (run_experiment.py:103)


def organism_device_bytes(ir, batch: int, replication_batch: int = 0) -> int:
    """Conservative device footprint of one organism in the HIP engine at training batch ``batch``.

    Parameters: fp32 master + Q40 int64 gradient + 2 fp32 Adam moments + bf16 compute copy + bf16
    transposed copy = 24 B per weight.  Activations: bf16 output and bf16 gradient of every node at the
    batch (fused producers never materialise theirs, which this estimate ignores), the uint8 pool
    argmax, fp32 head logits, the split-K FWD workspaces of long-K merged Dense layers (<= 16 fp32
    slabs of the output), and the fp32 split slabs of every KH x KW > 1 convolution's WGRAD (at most one slab per
    CONV_WGRAD_MIN_CHUNKS 128-pixel chunks, capped at CONV_WGRAD_MAX_SLAB_MB per layer: ops/hip_ops.py
    conv_wgrad_splits).  ``replication_batch``: the forward-only buffers of the replication plan."""
    from ..ops.hip_ops import CONV_WGRAD_MAX_SLAB_MB, CONV_WGRAD_MIN_CHUNKS
    weights = 0
    act = 0
    slabs = 0
    for n in ir.nodes:
        if n.op == "gemm":
            a = n.attrs
            if a["kind"] in ("head_cls", "head_rep"):
                continue
            weights += a["f"] * a["kh"] * a["kw"] * a["cin"] + (a["f"] if a["use_bias"] else 0)
            if a["kh"] * a["kw"] > 1:
                chunks = -(-batch * math.prod(n.shape[:-1]) // 128)
                one = 4 * a["f"] * a["kh"] * a["kw"] * (-(-a["cin"] // 8) * 8)
                slabs += min(CONV_WGRAD_MAX_SLAB_MB << 20, max(1, chunks // CONV_WGRAD_MIN_CHUNKS) * one)
        elif n.op == "bn":
            weights += 4 * n.attrs["channels"]
        if n.op in ("input", "reshape"):
            continue
        elems = math.prod(n.shape)
        act += 2 * 2 * elems                     # bf16 activation + bf16 gradient
        if n.op == "pool":
            act += elems                         # argmax bytes
        if n.op == "gemm" and n.attrs["kind"] == "dense" and elems == n.attrs["f"] and n.attrs["cin"] >= 3072:
            act += 16 * 4 * elems                # split-K FWD slabs of a long-K merged Dense (<= 16 splits)
    heads = ir.head_features * (ir.num_classes + ir.genotype_size)
    weights += heads + ir.num_classes + ir.genotype_size
    act += 3 * 4 * (ir.num_classes + ir.genotype_size)          # fp32 logits + bf16 dlogits (+ slack)
    per_sample_fwd = sum(2 * math.prod(n.shape) for n in ir.nodes if n.op not in ("input", "reshape"))
    total = 24 * weights + batch * act + slabs + replication_batch * per_sample_fwd
    return int(1.25 * total) + (1 << 20)         # allocator rounding, descriptor tables


def device_budget(device) -> Optional[float]:
    """Bytes this rank may plan with: ``SERANN_HBM_BUDGET_GB`` when set, else HBM_FRACTION of the free
    device memory; None on the CPU (no budget: one wave)."""
    env = os.environ.get(ENV_BUDGET)
    if env:
        return float(env) * 1e9
    if not str(device).startswith("cuda"):
        return None
    import torch
    free, _total = torch.cuda.mem_get_info(torch.device(device))
    return HBM_FRACTION * float(free)


def admit(device, min_mb: float = MIN_GPU_MEMORY_MB) -> None:
    """GPU-memory admission (reference run_experiment.py:103): refuse to start a rank whose device has
    less than ``min_mb`` MB free, with a clear error instead of an out-of-memory failure mid-generation."""
    if not str(device).startswith("cuda"):
        return
    import torch
    free, total = torch.cuda.mem_get_info(torch.device(device))
    if free < min_mb * 1e6:
        raise RuntimeError(f"{device}: {free / 1e6:.0f} MB free of {total / 1e6:.0f} MB, below the "
                           f"{min_mb:.0f} MB admission threshold (reference min_gpu_memory_required)")


def plan_waves(sizes: Sequence[int], budget: Optional[float], max_per_wave: Optional[int] = None) -> List[List[int]]:
    """Split organisms 0..n-1 (in order) into consecutive waves whose summed ``sizes`` stay within
    ``budget`` (at least one organism per wave) and hold at most ``max_per_wave`` organisms."""
    n = len(sizes)
    if n == 0:
        return []
    waves, cur, acc = [], [], 0.0
    for i, s in enumerate(sizes):
        full = (budget is not None and cur and acc + s > budget) or (max_per_wave and len(cur) >= max_per_wave)
        if full:
            waves.append(cur)
            cur, acc = [], 0.0
        cur.append(i)
        acc += float(s)
    waves.append(cur)
    return waves


def is_oom(exc: BaseException) -> bool:
    """True for a device allocation failure (torch's OutOfMemoryError or a HIP out-of-memory error)."""
    try:
        import torch
        if isinstance(exc, torch.cuda.OutOfMemoryError):
            return True
    except Exception:
        pass
    msg = str(exc).lower()
    return "out of memory" in msg or "hiperroroutofmemory" in msg.replace(" ", "")


def free_device_memory(device) -> None:
    if str(device).startswith("cuda"):
        import gc
        import torch
        gc.collect()
        torch.cuda.empty_cache()


def run_with_fallback(members: List[int], run: Callable[[List[int], Optional[int]], object],
                      batch: int, device, log: Callable[[str], None] = print,
                      on_fail: Optional[Callable[[List[int]], object]] = None) -> list:
    """Run ``run(members, batch_override)`` for one wave; on an out-of-memory error split the wave in
    two and recurse; a single organism that still fails is retried once at half the batch (reference
    experiment_worker.py:121-126) and then handed to ``on_fail``.  Returns the list of results."""
    try:
        return [run(members, None)]
    except Exception as e:            # noqa: BLE001 -- classified below
        if not is_oom(e):
            raise
        free_device_memory(device)
        if len(members) > 1:
            h = len(members) // 2
            log(f"out of device memory with {len(members)} organisms in a wave: splitting into {h} + {len(members) - h}")
            return (run_with_fallback(members[:h], run, batch, device, log, on_fail)
                    + run_with_fallback(members[h:], run, batch, device, log, on_fail))
        half = max(1, batch // 2)
        log(f"out of device memory for a single organism: retrying at batch {half} (reference behaviour)")
        try:
            return [run(members, half)]
        except Exception as e2:       # noqa: BLE001
            if not is_oom(e2) or on_fail is None:
                raise
            free_device_memory(device)
            log("the organism does not fit even at half batch: reporting it as failed")
            return [on_fail(members)]
