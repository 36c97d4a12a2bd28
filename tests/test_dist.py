"""Multi-process (world_size 2, gloo, CPU) coverage of the N>1 path: rule
broadcast, sharding, max-over-ranks timing, root scatter / verdict gather.
The classify step itself is per-rank and identical to N=1 (tested on GPU)."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world_size, port, q):
    sys.path.insert(0, str(ROOT / "nff-go_amd"))
    sys.path.insert(0, str(ROOT))
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world_size), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from nffacl import dist as nd, synth
    from oracle import oracle, rules_oracle as ro
    try:
        nd.init("gloo", None)
        g = synth.gen_rules(synth.RuleSpec(200), 77)
        text = nd.broadcast_rules(g.text if rank == 0 else None, None)
        ok_rules = text == g.text
        n_total = 64 * 37 + 5
        slots = torch.from_numpy(synth.gen_slots(g, n_total, 78)) if rank == 0 else None
        mine = nd.scatter_slots(slots, n_total, 64, None)
        start, cnt = nd.shard_even(n_total, rank, world_size)
        full = synth.gen_slots(g, n_total, 78)
        ok_shard = mine.numel() == cnt * 64 and bytes(mine.numpy()) == bytes(full[start * 64:(start + cnt) * 64])
        # per-rank classify (oracle here: no GPU on this container), then gather
        a4, a6 = ro.parse_text_table(text.encode()).arrays()
        port_local = torch.from_numpy(oracle.classify_slots(mine.numpy(), 64, cnt, a4, a6).view(np.int32))
        gathered = nd.gather_verdicts(port_local, n_total, None)
        ok_gather = True
        if rank == 0:
            want = oracle.classify_slots(full, 64, n_total, a4, a6).view(np.int32)
            ok_gather = bool((gathered.numpy() == want).all())
        # the same through scatter_classify_gather (bench.py's N>1 scatter-inclusive line)
        def classify(sl, cnt):
            return torch.from_numpy(oracle.classify_slots(sl.numpy(), 64, cnt, a4, a6).view(np.int32))
        full_v, secs = nd.scatter_classify_gather(slots, n_total, 64, classify, None)
        if rank == 0:
            ok_gather = ok_gather and bool((full_v.numpy() == want).all()) and secs > 0
        else:
            ok_gather = ok_gather and full_v is None
        t = nd.max_over_ranks(float(rank + 1), None)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, ok_rules, ok_shard, ok_gather, t))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


@pytest.mark.parametrize("ws", [2, 3])
def test_gloo_pipeline(ws):
    """Rule broadcast, dist.scatter of slots / dist.gather of verdicts (the
    collectives RCCL runs at N>1), max-over-ranks timing; 3 ranks make the
    equal shards ragged (padding on the last rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert len(r) == 5, r
        rank, ok_rules, ok_shard, ok_gather, t = r
        assert ok_rules and ok_shard and ok_gather, r
        assert t == float(ws)


@pytest.mark.parametrize("n,ws", [(0, 2), (1, 2), (64, 2), (65, 2), (1 << 24, 8), (1000003, 8), (100, 3)])
@pytest.mark.parametrize("even", [False, True])
def test_shards_partition_the_batch(n, ws, even):
    sys.path.insert(0, str(ROOT / "nff-go_amd"))
    from nffacl import dist as nd
    fn = nd.shard_even if even else nd.shard
    covered = 0
    prev_end = 0
    for r in range(ws):
        s, c = fn(n, r, ws)
        assert s == prev_end and (s % 64 == 0 or s == n)
        prev_end = s + c
        covered += c
    assert covered == n
