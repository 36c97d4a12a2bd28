"""Multi-GPU plumbing for the ACL path: one process per GPU (torch.distributed,
RCCL on the GPU box, gloo for CPU rehearsal).

The path shards trivially: packets are independent and every
GPU holds the full rule table, so the data path needs no collective.  The only
real exchange is the rule file itself — rank 0 loads it and broadcasts its
bytes once per rule swap (the reference's rule hot-swap, tutorial/step08.go:33-44,
is a local pointer store; across GPUs it becomes this broadcast).  For the
"root-scattered" deployment (packets arriving on one GPU) scatter_slots /
gather_verdicts move packet shards and verdict shards with one RCCL
collective each (dist.scatter / dist.gather: the root's peer transfers run
concurrently over its xGMI links, not one recv at a time).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def world():
    """(rank, world_size, local_rank) from the torch.distributed.run env."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str, device: torch.device | None):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=device)
    else:
        dist.init_process_group(backend)


def comm_device(device: torch.device | None) -> torch.device:
    """Tensors for collectives live on the GPU under RCCL, on the CPU under gloo."""
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return device
    return torch.device("cpu")


def broadcast_rules(text: str | None, device: torch.device | None, src: int = 0) -> str:
    """Rank `src` passes the rule-file text; every rank returns it."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return text
    cd = comm_device(device)
    rank = dist.get_rank()
    size = torch.zeros(1, dtype=torch.int64, device=cd)
    if rank == src:
        raw = torch.frombuffer(bytearray(text.encode()), dtype=torch.uint8).to(cd)
        size[0] = raw.numel()
    dist.broadcast(size, src)
    if rank != src:
        raw = torch.empty(int(size.item()), dtype=torch.uint8, device=cd)
    dist.broadcast(raw, src)
    return bytes(raw.cpu().numpy()).decode()


def max_over_ranks(x: float, device: torch.device | None) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=comm_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard(n_total: int, rank: int, world_size: int):
    """Contiguous shard [start, start + count) of a batch of n_total packets,
    64-packet aligned so permit words never straddle ranks."""
    waves = (n_total + 63) // 64
    per, rem = divmod(waves, world_size)
    first = rank * per + min(rank, rem)
    cnt = per + (1 if rank < rem else 0)
    start = min(n_total, first * 64)
    return start, min(n_total, (first + cnt) * 64) - start


def _even_shard(n_total: int, world_size: int) -> int:
    """Packets per rank for the collectives: equal 64-aligned shards (the
    last rank's tail is padding when n_total does not divide evenly)."""
    waves = (n_total + 63) // 64
    return (waves + world_size - 1) // world_size * 64


def scatter_slots(slots: torch.Tensor | None, n_total: int, stride: int, device: torch.device | None,
                  src: int = 0) -> torch.Tensor:
    """Root-scattered ingest: rank `src` holds all n_total slots; every rank
    receives its shard through ONE collective (dist.scatter — under RCCL the
    root's sends to all peers run concurrently, one per xGMI link; ncclScatter
    semantics, rccl.h:767).  Shards are equal 64-packet-aligned pieces;
    returns this rank's slots trimmed to its real packets (shard_even())."""
    rank, ws = dist.get_rank(), dist.get_world_size()
    cd = comm_device(device)
    per = _even_shard(n_total, ws)
    start, cnt = shard_even(n_total, rank, ws)
    out = torch.empty(per * stride, dtype=torch.uint8, device=cd)
    pieces = None
    if rank == src:
        flat = slots.reshape(-1)
        if flat.device != cd:
            flat = flat.to(cd)
        need = per * ws * stride
        if flat.numel() < need:  # ragged batch: pad the root's copy (zero slots, never reported)
            pad = torch.zeros(need, dtype=torch.uint8, device=cd)
            pad[:n_total * stride] = flat[:n_total * stride]
            flat = pad
        pieces = list(flat[:need].view(ws, per * stride).unbind(0))
    dist.scatter(out, pieces, src=src)
    return out[:cnt * stride]


def gather_verdicts(port: torch.Tensor, n_total: int, device: torch.device | None, dst: int = 0):
    """Inverse of scatter_slots for the u32 verdict vector, through ONE
    dist.gather (ncclGather semantics, rccl.h:745): returns the full vector
    on `dst`, None elsewhere."""
    rank, ws = dist.get_rank(), dist.get_world_size()
    cd = comm_device(device)
    per = _even_shard(n_total, ws)
    buf = torch.zeros(per, dtype=port.dtype, device=cd)
    buf[:port.numel()] = port.to(cd)
    if rank == dst:
        full = torch.empty(per * ws, dtype=port.dtype, device=cd)
        dist.gather(buf, list(full.view(ws, per).unbind(0)), dst=dst)
        return full[:n_total]
    dist.gather(buf, None, dst=dst)
    return None


def shard_even(n_total: int, rank: int, world_size: int):
    """(start, count) of rank's piece under the equal-shard collectives."""
    per = _even_shard(n_total, world_size)
    start = min(n_total, rank * per)
    return start, min(n_total, start + per) - start


def scatter_classify_gather(slots_root, n_total: int, stride: int, classify, device, src: int = 0):
    """The root-scattered deployment end to end (SURVEY.md §8e curve 2): rank
    `src` holds all n_total slots, every rank receives its 64-aligned shard,
    runs `classify(shard_slots, count) -> u32/i32 port tensor` on it, and the
    verdicts come back to `src`.  Returns (full verdict vector on src / None,
    seconds between the opening and closing barriers, max over ranks)."""
    import time
    dev = comm_device(device)
    dist.barrier()
    if dev is not None and dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    mine = scatter_slots(slots_root, n_total, stride, device, src)
    _, cnt = shard_even(n_total, dist.get_rank(), dist.get_world_size())
    port = classify(mine, cnt) if cnt else torch.empty(0, dtype=torch.int32, device=dev)
    full = gather_verdicts(port, n_total, device, src)
    if dev is not None and dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dist.barrier()
    return full, max_over_ranks(time.perf_counter() - t0, device)
