"""Multi-GPU batch split: one process per GPU over torch.distributed (RCCL on ROCm).

The reference decodes on one OpenCL device (``discrete_LDPC_decoder_irreg.py:174-175``) and
has no communication backend. Decoding independent codewords partitions perfectly, so the
multi-GPU design has exactly two exchanges, both off the data path:

* setup: rank 0's code graph (CSR of H) and decoder tables are broadcast once
  (:func:`broadcast_arrays` — three broadcasts: the header's size, the header, one packed
  payload; over xGMI with the ``nccl``=RCCL backend, or over TCP with ``gloo``);
* per Eb/N0 point: one all-reduce of the counters {errors, bits, codewords, iterations}
  (:func:`allreduce_counts`).

Codeword ranges are contiguous per rank (:func:`shard_range`); each shard is its own decode
call, so the batch-global early stop of the reference is applied per shard.
"""
from __future__ import annotations

import os
from typing import Dict, Tuple

import numpy as np
import torch
import torch.distributed as dist

__all__ = ["init_from_env", "shard_range", "broadcast_arrays", "allreduce_counts", "allreduce_max"]

_DTYPES = [np.dtype(x) for x in ("int8", "uint8", "int16", "int32", "int64", "float32", "float64")]


def init_from_env(backend: str | None = None) -> Tuple[int, int, torch.device]:
    """Initialise the process group from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).

    Returns (rank, world_size, device). Single-process runs (no WORLD_SIZE) skip the group.
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (not for production runs): IBL_SHARE_DEVICE=1 maps ranks onto the visible
    # devices round-robin (several ranks on one GPU), IBL_DIST_BACKEND overrides the backend
    # (RCCL needs one GPU per rank, so shared-device rehearsals use gloo)
    if os.environ.get("IBL_SHARE_DEVICE") == "1" and torch.cuda.device_count() > 0:
        local = local % torch.cuda.device_count()
    backend = backend or os.environ.get("IBL_DIST_BACKEND") or None
    use_gpu = torch.cuda.is_available()
    device = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or ("nccl" if use_gpu else "gloo")
        if backend == "gloo" and use_gpu and os.environ.get("IBL_SHARE_DEVICE") != "1":
            # one GPU per rank is the production layout: its collectives belong on RCCL over xGMI
            raise RuntimeError("refusing the gloo backend with one GPU per rank: use nccl (RCCL), or set "
                               "IBL_SHARE_DEVICE=1 for a shared-device rehearsal")
        kwargs = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kwargs)
    return rank, world, device


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, start+count) codeword range of ``rank`` (sizes differ by at most 1)."""
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def _comm_device() -> torch.device:
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def broadcast_arrays(arrays: Dict[str, np.ndarray] | None, src: int = 0) -> Dict[str, np.ndarray]:
    """Broadcast a dict of numpy arrays from ``src`` to every rank: three broadcasts in total — the header's
    length, the header (keys, dtypes, shapes, payload size) and one packed uint8 payload.

    Non-source ranks pass ``None``. Key order, dtypes and shapes travel in a small header. An initialised
    group of size 1 still runs the collectives (so a 1-GPU ``nccl`` group exercises the device path).
    """
    if not dist.is_initialized():
        return {k: np.ascontiguousarray(v) for k, v in (arrays or {}).items()}
    dev = _comm_device()
    rank = dist.get_rank()
    if rank == src:
        keys = list(arrays.keys())
        header = [len(keys)]
        blobs = []
        for k in keys:
            a = np.ascontiguousarray(arrays[k])
            kb = k.encode()
            header += [len(kb), *kb, _DTYPES.index(a.dtype), a.ndim, *a.shape]
            blobs.append(a.view(np.uint8).ravel())
        payload = np.concatenate(blobs) if blobs else np.zeros(0, np.uint8)
        hdr = torch.tensor([len(header), payload.size] + header, dtype=torch.int64, device=dev)
        size = torch.tensor([hdr.numel()], dtype=torch.int64, device=dev)
    else:
        size = torch.zeros(1, dtype=torch.int64, device=dev)
    dist.broadcast(size, src)
    if rank != src:
        hdr = torch.zeros(int(size.item()), dtype=torch.int64, device=dev)
    dist.broadcast(hdr, src)
    h = hdr.cpu().numpy().tolist()
    n_payload = h[1]
    buf = (torch.from_numpy(payload).to(dev) if rank == src
           else torch.empty(n_payload, dtype=torch.uint8, device=dev))
    dist.broadcast(buf, src)
    raw = buf.cpu().numpy()
    out, pos, off = {}, 3, 0
    for _ in range(h[2]):
        klen = h[pos]; pos += 1
        key = bytes(h[pos:pos + klen]).decode(); pos += klen
        dt = _DTYPES[h[pos]]; nd = h[pos + 1]; pos += 2
        shape = tuple(h[pos:pos + nd]); pos += nd
        nbytes = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
        out[key] = raw[off:off + nbytes].view(dt).reshape(shape).copy()
        off += nbytes
    return out


def allreduce_counts(counts: Dict[str, int]) -> Dict[str, int]:
    """Sum integer counters over ranks (one all-reduce)."""
    keys = sorted(counts)
    t = torch.tensor([int(counts[k]) for k in keys], dtype=torch.int64, device=_comm_device())
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return dict(zip(keys, (int(x) for x in t.cpu().tolist())))


def allreduce_max(x: float) -> float:
    t = torch.tensor([float(x)], dtype=torch.float64, device=_comm_device())
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
