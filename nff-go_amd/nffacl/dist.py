"""Multi-GPU plumbing for the ACL path: one process per GPU (torch.distributed,
RCCL on the GPU box, gloo for CPU rehearsal).

The path shards trivially: packets are independent and every
GPU holds the full rule table, so the data path needs no collective.  The only
real exchange is the rule file itself — rank 0 loads it and broadcasts its
bytes once per rule swap (the reference's rule hot-swap, tutorial/step08.go:33-44,
is a local pointer store; across GPUs it becomes this broadcast).  For the
"root-scattered" deployment (packets arriving on one GPU) scatter_slots /
gather_verdicts move packet shards and verdict shards over RCCL.
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


def scatter_slots(slots: torch.Tensor | None, n_total: int, stride: int, device: torch.device | None,
                  src: int = 0) -> torch.Tensor:
    """Root-scattered ingest: rank `src` holds all n_total slots; every rank
    receives its shard (point-to-point sends, one per peer)."""
    rank, ws = dist.get_rank(), dist.get_world_size()
    cd = comm_device(device)
    start, cnt = shard(n_total, rank, ws)
    if rank == src:
        reqs = []
        for r in range(ws):
            if r == src:
                continue
            s, c = shard(n_total, r, ws)
            if c:
                reqs.append(dist.isend(slots[s * stride:(s + c) * stride].to(cd).contiguous(), r))
        for q in reqs:
            q.wait()
        return slots[start * stride:(start + cnt) * stride].to(cd)
    buf = torch.empty(cnt * stride, dtype=torch.uint8, device=cd)
    if cnt:
        dist.recv(buf, src)
    return buf


def gather_verdicts(port: torch.Tensor, n_total: int, device: torch.device | None, dst: int = 0):
    """Inverse of scatter_slots for the u32 verdict vector (returns the full
    vector on `dst`, None elsewhere)."""
    rank, ws = dist.get_rank(), dist.get_world_size()
    cd = comm_device(device)
    if rank == dst:
        out = torch.empty(n_total, dtype=port.dtype, device=cd)
        s0, c0 = shard(n_total, rank, ws)
        out[s0:s0 + c0] = port.to(cd)
        for r in range(ws):
            if r == dst:
                continue
            s, c = shard(n_total, r, ws)
            if c:
                tmp = torch.empty(c, dtype=port.dtype, device=cd)
                dist.recv(tmp, r)
                out[s:s + c] = tmp
        return out
    s, c = shard(n_total, rank, ws)
    if c:
        dist.send(port.to(cd).contiguous(), dst)
    return None


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
    _, cnt = shard(n_total, dist.get_rank(), dist.get_world_size())
    port = classify(mine, cnt) if cnt else torch.empty(0, dtype=torch.int32, device=dev)
    full = gather_verdicts(port, n_total, device, src)
    if dev is not None and dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dist.barrier()
    return full, max_over_ranks(time.perf_counter() - t0, device)
