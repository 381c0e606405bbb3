"""SPMD communication layer (replaces the external ``distributed_computing`` job pool).

One process per GPU, launched by ``torch.distributed.run`` (or the CLI's ``--nproc`` spawner).
The control plane (generation table, RNG, selection) is *replicated* on every rank; the data plane
(training a shard of organisms) is sharded.  Per generation there is exactly one packed
all-gather of fixed-width records (M3) -- metrics + bit-packed offspring genotypes -- instead of
the reference's pickled pandas objects over TCP.

* GPU: backend ``nccl`` (= RCCL over xGMI on ROCm), payload tensors live on the local GPU.
* CPU: backend ``gloo`` (tests, world_size > 1 emulation).
"""
from __future__ import annotations

import os
import pickle
from datetime import timedelta
from typing import Any, List, Optional

import numpy as np


class Comm:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    def barrier(self):
        pass

    def allgather_bytes(self, payload: bytes) -> List[bytes]:
        return [payload]

    def allgather_payload(self, head: bytes, body=None) -> List[bytes]:
        """All-gather one record per rank made of a small host ``head`` and a ``body`` that may be a
        device tensor (the packed offspring bits from the replication epilogue): on RCCL the body never
        visits the host before the collective."""
        return self.allgather_bytes(head + _host_bytes(body))

    def broadcast_bytes(self, payload: Optional[bytes], src: int = 0) -> bytes:
        return payload

    def allgather_object(self, obj: Any) -> List[Any]:
        return [pickle.loads(b) for b in self.allgather_bytes(pickle.dumps(obj))]

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        b = self.broadcast_bytes(pickle.dumps(obj) if self.rank == src else None, src)
        return pickle.loads(b)

    def allreduce_max(self, value: float) -> float:
        return value

    def device_index(self) -> int:
        """Index of the GPU this rank computes on, or -1 (CPU)."""
        try:
            import torch
            if torch.cuda.is_available():
                return int(torch.cuda.current_device())
        except ImportError:
            pass
        return -1

    def shutdown(self):
        pass


class LocalComm(Comm):
    """world_size == 1."""


class TorchDistComm(Comm):
    """torch.distributed communicator.  Uses byte tensors so that one all-gather moves all
    of a rank's results; on RCCL the tensors are device tensors (no host staging in RCCL)."""

    def __init__(self, backend: Optional[str] = None, device=None, timeout_s: Optional[float] = None):
        import torch
        import torch.distributed as dist
        self.dist = dist
        self.torch = torch
        if timeout_s is None:
            timeout_s = collective_timeout_s()
        if not dist.is_initialized():
            if backend is None:
                backend = os.environ.get("SERANN_COMM_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29511")
            if backend == "nccl":
                # bind this rank to its GPU before RCCL creates communicators
                lr = int(os.environ.get("LOCAL_RANK", "0"))
                torch.cuda.set_device(lr % max(1, torch.cuda.device_count()))
            dist.init_process_group(backend=backend, timeout=timedelta(seconds=timeout_s))
        self.backend = dist.get_backend()
        self.rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        self.local_rank = int(os.environ.get("LOCAL_RANK", self.rank))
        if device is None:
            device = torch.device("cuda", self.local_rank) if self.backend == "nccl" else torch.device("cpu")
        self.device = torch.device(device)

    def barrier(self):
        if self.backend == "nccl":
            self.dist.barrier(device_ids=[self.device.index])
        else:
            self.dist.barrier()

    def _tensor(self, payload: bytes):
        t = self.torch.frombuffer(bytearray(payload), dtype=self.torch.uint8) if payload else \
            self.torch.zeros(0, dtype=self.torch.uint8)
        return t.to(self.device)

    def allgather_bytes(self, payload: bytes) -> List[bytes]:
        return self._allgather_tensor(self._tensor(payload))

    def allgather_payload(self, head: bytes, body=None) -> List[bytes]:
        torch = self.torch
        parts = [self._tensor(head)]
        if body is not None and len(body):
            if torch.is_tensor(body):
                parts.append(body.reshape(-1).to(self.device, torch.uint8))      # device -> device on RCCL
            else:
                parts.append(self._tensor(np.ascontiguousarray(body, np.uint8).tobytes()))
        return self._allgather_tensor(torch.cat(parts) if len(parts) > 1 else parts[0])

    def _allgather_tensor(self, t) -> List[bytes]:
        """One length exchange + one ``all_gather_into_tensor`` of the records padded to the longest;
        the gathered buffer comes to the host once, after the collective."""
        torch = self.torch
        n = torch.tensor([t.numel()], dtype=torch.int64, device=self.device)
        sizes = [torch.zeros_like(n) for _ in range(self.world_size)]
        self.dist.all_gather(sizes, n)
        sizes = [int(s.item()) for s in sizes]
        mx = max(sizes)
        buf = torch.zeros(mx, dtype=torch.uint8, device=self.device)
        if t.numel():
            buf[:t.numel()] = t
        out = torch.empty(self.world_size * mx, dtype=torch.uint8, device=self.device)
        self.dist.all_gather_into_tensor(out, buf)
        host = out.cpu().numpy()
        return [host[r * mx:r * mx + sizes[r]].tobytes() for r in range(self.world_size)]

    def broadcast_bytes(self, payload: Optional[bytes], src: int = 0) -> bytes:
        torch = self.torch
        n = torch.tensor([len(payload) if self.rank == src else 0], dtype=torch.int64, device=self.device)
        self.dist.broadcast(n, src)
        size = int(n.item())
        buf = self._tensor(payload) if self.rank == src else torch.empty(size, dtype=torch.uint8,
                                                                          device=self.device)
        if size:
            self.dist.broadcast(buf, src)
        return buf.cpu().numpy().tobytes()

    def allreduce_max(self, value: float) -> float:
        t = self.torch.tensor([float(value)], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def device_index(self) -> int:
        return int(self.device.index) if self.device.type == "cuda" else -1

    def shutdown(self):
        if self.dist.is_initialized():
            self.dist.destroy_process_group()


def collective_timeout_s() -> float:
    """Collective timeout: the per-generation job timeout (``worker_pool_job_timeout``, the reference's
    1080 s pool job timeout) plus a margin for the replicated control plane.  A stalled rank is ended by
    its own watchdog at the job timeout (utils/faults.py); this bounds how long the others wait."""
    from ..config import experiment_config
    return float(experiment_config["worker_pool_job_timeout"]) + 300.0


def make_comm(distributed: Optional[bool] = None, backend: Optional[str] = None) -> Comm:
    """Create the communicator from the environment (``WORLD_SIZE`` set by torchrun)."""
    if distributed is None:
        distributed = int(os.environ.get("WORLD_SIZE", "1")) > 1
    if not distributed:
        return LocalComm()
    return TorchDistComm(backend=backend)


# ------------------------------------------------------------------------------------------------
# fixed-width result records (M3): metrics + bit-packed offspring pools
# ------------------------------------------------------------------------------------------------
METRIC_FIELDS = ("classification_validation_accuracy", "classification_training_accuracy",
                 "classification_test_accuracy", "replication_mse")


def _host_bytes(body) -> bytes:
    if body is None:
        return b""
    try:
        import torch
        if torch.is_tensor(body):
            return body.detach().cpu().numpy().astype(np.uint8).tobytes()
    except ImportError:
        pass
    return np.ascontiguousarray(body, np.uint8).tobytes()


_HEAD_INTS, _HEAD_TIMES = 4, 3       # (n, pool, L, device index), (learning, replication, shard wall) seconds


def pack_header(indices: np.ndarray, metrics: np.ndarray, pool: int, L: int,
                learning_time: float, replication_time: float, device: int = -1, shard_s: float = 0.0) -> bytes:
    """The host part of a result record: (n, pool, L, the rank's GPU index), three timings (learning,
    replication, the whole shard's wall time), the organism indices and the (n, 4) float64 metrics.  The
    packed offspring bits [n][pool][ceil(L / 8)] follow it."""
    n = len(indices)
    header = np.array([n, pool if n else 0, L if n else 0, device], dtype=np.int64).tobytes()
    times = np.array([learning_time, replication_time, shard_s], dtype=np.float64).tobytes()
    return header + times + np.asarray(indices, np.int32).tobytes() + np.asarray(metrics, np.float64).tobytes()


def pack_results(indices: np.ndarray, metrics: np.ndarray, offspring: np.ndarray,
                 learning_time: float, replication_time: float) -> bytes:
    """indices: (n,) int32 organism indices in the generation table; metrics: (n, 4) float64;
    offspring: (n, pool, L) {0,1} -> bit-packed (host form of the record)."""
    n = len(indices)
    head = pack_header(indices, metrics, offspring.shape[1] if n else 0, offspring.shape[2] if n else 0,
                       learning_time, replication_time)
    bits = np.packbits(np.asarray(offspring, np.uint8), axis=-1).tobytes() if n else b""
    return head + bits


def unpack_header(payload: bytes) -> dict:
    """The rank-level fields of a result record: organisms, GPU index and timings."""
    n, pool, L, dev = np.frombuffer(payload[:8 * _HEAD_INTS], dtype=np.int64)
    lt, rt, sh = np.frombuffer(payload[8 * _HEAD_INTS:8 * (_HEAD_INTS + _HEAD_TIMES)], dtype=np.float64)
    return dict(organisms=int(n), device=int(dev), learning_s=float(lt), replication_s=float(rt), shard_s=float(sh))


def unpack_results(payload: bytes):
    n, pool, L, _dev = np.frombuffer(payload[:8 * _HEAD_INTS], dtype=np.int64)
    lt, rt, _sh = np.frombuffer(payload[8 * _HEAD_INTS:8 * (_HEAD_INTS + _HEAD_TIMES)], dtype=np.float64)
    off = 8 * (_HEAD_INTS + _HEAD_TIMES)
    idx = np.frombuffer(payload[off:off + 4 * n], dtype=np.int32)
    off += 4 * n
    metrics = np.frombuffer(payload[off:off + 8 * n * 4], dtype=np.float64).reshape(n, 4)
    off += 8 * n * 4
    if n:
        nbytes = (L + 7) // 8
        bits = np.frombuffer(payload[off:off + n * pool * nbytes], dtype=np.uint8).reshape(n, pool, nbytes)
        offspring = np.unpackbits(bits, axis=-1)[..., :L]
    else:
        offspring = np.zeros((0, 0, 0), np.uint8)
    return idx, metrics, offspring, float(lt), float(rt)
