#!/usr/bin/env python3
"""bench.py — device-resident L3 ACL classification throughput on MI355X.

Headline (BASELINE.json "metric"): Mpackets/s of device-resident L3 ACL
classify, 64 B packets, 1 k rules (config C2), with the fraction of the HBM
roofline.  One step = one classify launch (nffacl_classify_device, the HIP
path) over the whole per-GPU batch of synthetic 64-byte slots already
resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1|c3|c4|c5|l2] [--algo auto|linear|indexed]

(`--config l2` measures the L2 ACL kernel, SURVEY.md §8f row 4 — not a
BASELINE.json config: 256 GetL2ACLFromTextTable rules over 64 B slots.)

N > 1 runs under torch.distributed.run (one rank per GPU, RCCL): rank 0
generates the rule file and broadcasts its bytes over RCCL (the path's one real
exchange step, outside the timed region); every rank classifies its own
resident shard — no data-path collective ("scaling": "weak").

The JSON line carries:
  roofline     achieved = 68 algorithmic bytes/packet (64 B read + 4 B port
               write) x packets per launch / mean kernel time
               (HIP events on the launch stream); peak = 8 TB/s HBM3E;
               traffic = PMC bytes per launch from profiles/ (if collected)
  cpu_baseline the oracle (oracle/acl_oracle.c, reference algorithm restated
               in C) on a bounded sample of the same packets, on this host's
               cores, rank 0 at N = 1 only
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "nff-go_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

METRIC = "Mpackets/s device-resident L3 ACL classify, 64B pkts @1k rules; % HBM roofline"
METRIC_L2 = "Mpackets/s device-resident L2 ACL classify, 64B pkts @256 rules (SURVEY.md §8f, not a BASELINE metric)"
BYTES_PER_PACKET = 68  # 64 B slot read + 4 B verdict write
HBM_PEAK_GBPS = 8000.0
WORKLOADS = {
    "c1": "C1 firewall.conf (4 text rules -> 4 ip4 + 1 ip6), 64B packets, device-resident",
    "c2": "C2 1k-rule L3 ACL, 64B packets, device-resident",
    "c3": "C3 10k-rule L3+L4 ACL, IMIX 64/570/1518 (7:4:1) packed frames, device-resident",
    "c4": "C4 1k-rule L3 ACL, 64B packets, packet batch sharded across GPUs",
    "c5": "C5 100k-rule L3+L4 ACL with port ranges, 64B packets, device-resident",
    "l2": "L2 ACL (acl.go l2ACL), 256 MAC/EtherType rules, 64B packets, device-resident",
}
ALGO_NAMES = {1: "linear", 2: "indexed", 3: "hybrid"}  # nffacl.ALGO_*
L2_RULES = 256
# L2 reads the 16-byte line holding the Ethernet header and writes 4 B
BYTES_PER_PACKET_L2 = 20
# C3 reads each frame's first 64-byte line + its 8-byte descriptor and writes 4 B
BYTES_PER_PACKET_FRAMES = 76


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_rules(cfg: str):
    from nffacl import synth
    if cfg == "l2":
        g = synth.gen_l2_rules(L2_RULES)
        return g.text, g
    if cfg == "c1":
        text = (ROOT / "tests" / "golden" / "rules" / "firewall.conf").read_text()
        return text, synth.firewall_rules(text)
    g = synth.gen_rules(synth.SPECS[cfg if cfg != "c4" else "c2"], synth.RULE_SEEDS[cfg])
    return g.text, g


def pmc_traffic(cfg: str, algo: str, n: int):
    """HBM bytes per launch from the committed PMC summary, if one matches."""
    path = ROOT / "profiles" / "pmc_traffic.json"
    if not path.exists():
        return None
    try:
        d = json.loads(path.read_text())
        e = d.get(f"{cfg}:{algo}:{n}")
        return None if e is None else float(e["bytes_per_launch"])
    except Exception:
        return None


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_frames(frames: np.ndarray, desc: np.ndarray, a4, a6, budget_s: float):
    """C3: the oracle over the same packed IMIX frames (descriptor order)."""
    from oracle import oracle
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    n = len(desc)
    cal = min(n, 1 << 15)
    t = time.perf_counter()
    oracle.classify_frames(frames, desc[:cal], a4, a6, threads=cores)
    rate = cal / max(time.perf_counter() - t, 1e-6)
    sample = int(min(n, max(cal, rate * budget_s)))
    passes, done, dt = 0, 0, 0.0
    while True:
        t = time.perf_counter()
        ports = oracle.classify_frames(frames, desc[:sample], a4, a6, threads=cores)
        dt += time.perf_counter() - t
        passes += 1
        done += sample
        if dt >= budget_s or passes >= 50:
            break
    one = min(sample, 1 << 15)
    t1 = time.perf_counter()
    oracle.classify_frames(frames, desc[:one], a4, a6, threads=1)
    dt1 = time.perf_counter() - t1
    return {
        "value": round(done / dt / 1e6, 3), "unit": "Mpps", "cores": cores, "kind": "port",
        "sample": f"first {sample} IMIX frames x {passes} pass(es) (oracle/acl_oracle.c = acl.go l3ACL "
                  f"restated in C, {cores} threads, {dt:.1f}s)",
        "single_core_mpps": round(one / dt1 / 1e6, 3),
    }, ports[:sample]


def cpu_baseline(slots: np.ndarray, n: int, a4, a6, budget_s: float, eth=None):
    from oracle import oracle
    if eth is not None:
        return cpu_baseline_l2(slots, n, eth, budget_s)
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))  # the GPU box's CPU share for one GPU
    # calibrate on a small prefix, then size the sample for ~budget_s
    cal = min(n, 1 << 15)
    t = time.perf_counter()
    oracle.classify_slots(slots, 64, cal, a4, a6, threads=cores)
    rate = cal / max(time.perf_counter() - t, 1e-6)
    sample = int(min(n, max(cal, rate * budget_s)))
    passes, done, dt = 0, 0, 0.0
    while True:  # whole passes over the sample until ~budget_s of CPU work
        t = time.perf_counter()
        ports, which = oracle.classify_slots_which(slots, 64, sample, a4, a6, threads=cores)
        dt += time.perf_counter() - t
        passes += 1
        done += sample
        if dt >= budget_s or passes >= 50:
            break
    t1 = time.perf_counter()
    one = min(sample, 1 << 16)
    oracle.classify_slots(slots, 64, one, a4, a6, threads=1)
    dt1 = time.perf_counter() - t1
    hit = which >= 0
    return {
        "value": round(done / dt / 1e6, 3), "unit": "Mpps", "cores": cores, "kind": "port",
        "sample": f"first {sample} packets of rank 0's batch x {passes} pass(es) "
                  f"(oracle/acl_oracle.c = acl.go l3ACL restated in C, {cores} threads, {dt:.1f}s)",
        "single_core_mpps": round(one / dt1 / 1e6, 3),
        "mean_first_match_index": round(float(which[hit].mean()), 1) if hit.any() else None,
        "match_fraction": round(float(hit.mean()), 4),
    }, ports[:sample]


def cpu_baseline_l2(slots: np.ndarray, n: int, eth, budget_s: float):
    from oracle import oracle
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    cal = min(n, 1 << 16)
    t = time.perf_counter()
    oracle.l2_classify_slots(slots, 64, cal, eth, threads=cores)
    rate = cal / max(time.perf_counter() - t, 1e-6)
    sample = int(min(n, max(cal, rate * budget_s)))
    passes, done, dt = 0, 0, 0.0
    while True:
        t = time.perf_counter()
        ports = oracle.l2_classify_slots(slots, 64, sample, eth, threads=cores)
        dt += time.perf_counter() - t
        passes += 1
        done += sample
        if dt >= budget_s or passes >= 50:
            break
    one = min(sample, 1 << 16)
    t1 = time.perf_counter()
    oracle.l2_classify_slots(slots, 64, one, eth, threads=1)
    dt1 = time.perf_counter() - t1
    return {
        "value": round(done / dt / 1e6, 3), "unit": "Mpps", "cores": cores, "kind": "port",
        "sample": f"first {sample} packets x {passes} pass(es) (oracle/acl_oracle.c = acl.go l2ACL "
                  f"restated in C, {cores} threads, {dt:.1f}s)",
        "single_core_mpps": round(one / dt1 / 1e6, 3),
    }, ports[:sample]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "l2"])
    ap.add_argument("--algo", default="auto", choices=["auto", "linear", "indexed", "hybrid"])
    ap.add_argument("--packets", type=int, default=1 << 24, help="packets per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--timing", default="region", choices=["launch", "region"],
                    help="HIP events around every launch, or one pair around the K launches "
                         "(kernel_ms = region / K, inter-launch gaps included)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host", action="store_true", help="skip the PCIe-inclusive measurement")
    ap.add_argument("--no-scatter", action="store_true",
                    help="N>1: skip the root-scattered (scatter+classify+gather) measurement")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N>1 (nccl = RCCL on ROCm)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import nffacl
    from nffacl import dist as nd

    rank, world, local = nd.world()
    if os.environ.get("NFFACL_BENCH_ONE_GPU") == "1":  # rehearse N ranks on one GPU (gloo)
        local = 0
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        nd.init(args.backend, dev)

    cfg = args.config
    n = args.packets
    algo_id = {"auto": nffacl.ALGO_AUTO, "linear": nffacl.ALGO_LINEAR, "indexed": nffacl.ALGO_INDEXED,
               "hybrid": nffacl.ALGO_HYBRID}[args.algo]

    # ---- rules: rank 0 generates, RCCL broadcast of the rule file bytes ----
    text, gen = build_rules(cfg)
    text = nd.broadcast_rules(text if rank == 0 else None, dev)
    l2_mode = cfg == "l2"
    if l2_mode:
        rules = nffacl.L2Rules.parse_text(text)
        n4, n6 = rules.count(), 0
        eng = nffacl.L2Engine(rules, device=local, algo=algo_id)
        algo_name = ALGO_NAMES[eng.algo]
    else:
        rules = nffacl.L3Rules.parse_text(text)
        n4, n6 = rules.counts()
        eng = nffacl.Engine(rules, device=local, algo=algo_id)
        algo_name = ALGO_NAMES[eng.algo]

    # ---- packets: per-rank shard, resident in HBM before timing ----
    from nffacl import synth
    t0 = time.perf_counter()
    frames_mode = cfg == "c3"
    if frames_mode:
        frames, desc = synth.gen_imix(gen, n, synth.PACKET_SEEDS[cfg] + 7919 * rank)
        d_frames = torch.from_numpy(frames).to(dev)
        d_desc = torch.from_numpy(desc.view(np.int64)).to(dev)
        slots = None
    elif l2_mode:
        slots = synth.gen_l2_slots(gen, n, synth.L2_PACKET_SEED + 7919 * rank)
        d_slots = torch.from_numpy(slots).to(dev)
    else:
        slots = synth.gen_slots(gen, n, synth.PACKET_SEEDS[cfg] + 7919 * rank)
        d_slots = torch.from_numpy(slots).to(dev)
    log(f"[rank {rank}] generated {n} packets in {time.perf_counter() - t0:.1f}s; rules ip4={n4} ip6={n6}; algo={algo_name}")
    port = torch.empty(n, dtype=torch.int32, device=dev)
    permit = torch.empty((n + 63) // 64, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def launch():
        if frames_mode:
            eng.classify_frames_device(d_frames, d_desc, n, port, permit, stream)
        else:
            eng.classify_device(d_slots, 64, n, port, permit, stream)

    for _ in range(args.warmup):
        launch()
    torch.cuda.synchronize(dev)

    # ---- timed region ----
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    if args.timing == "region":
        evs[0][0].record(stream)
        for s in range(args.steps):
            launch()
        evs[0][1].record(stream)
    else:
        for s in range(args.steps):
            evs[s][0].record(stream)
            launch()
            evs[s][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if args.timing == "region":  # mean launch duration over the region, gaps included
        kms = np.full(args.steps, evs[0][0].elapsed_time(evs[0][1]) / args.steps)
        # per-launch spread (min/p50/max) from a separate, untimed pass with an
        # event pair around each launch; the region mean stays the roofline basis
        m = min(args.steps, 20)
        for s in range(m):
            evs[s][0].record(stream)
            launch()
            evs[s][1].record(stream)
        torch.cuda.synchronize(dev)
        spread = np.array([a.elapsed_time(b) for a, b in evs[:m]])
    else:
        kms = np.array([a.elapsed_time(b) for a, b in evs])  # per-launch kernel time (ms)
        spread = kms
    elapsed = nd.max_over_ranks(elapsed, dev)

    # ---- spot parity check (outside timing): GPU verdicts vs oracle sample ----
    from oracle import oracle, rules_oracle as ro
    got = port.cpu().numpy().view(np.uint32)
    rng = np.random.default_rng(rank)
    idx = np.sort(rng.choice(n, min(n, 4096), replace=False))
    eth = a4 = a6 = None
    if l2_mode:
        eth = ro.parse_l2_text_table(text.encode()).array()
        want = oracle.l2_classify_slots(slots.reshape(n, 64)[idx].reshape(-1), 64, len(idx), eth, threads=4)
    else:
        a4, a6 = ro.parse_text_table(text.encode()).arrays()
    if l2_mode:
        pass
    elif frames_mode:
        want = oracle.classify_frames(frames, desc[idx], a4, a6, threads=4)
    else:
        want = oracle.classify_slots(slots.reshape(n, 64)[idx].reshape(-1), 64, len(idx), a4, a6, threads=4)
    bit_exact = bool((got[idx] == want).all())

    total = n * world * args.steps
    value = total / elapsed / 1e6
    mean_k = float(kms.mean()) / 1e3
    bpp = BYTES_PER_PACKET_FRAMES if frames_mode else BYTES_PER_PACKET_L2 if l2_mode else BYTES_PER_PACKET
    achieved = bpp * n / mean_k / 1e9
    out = {
        "metric": METRIC_L2 if l2_mode else METRIC,
        "value": round(value, 1),
        "unit": "Mpps",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (deterministic seeds; SURVEY.md §8d mix)",
        "config": {
            "workload": WORKLOADS.get(cfg, cfg), "rules_ip4": n4, "rules_ip6": n6,
            "packets_per_gpu": n, "slot_bytes": None if frames_mode else 64,
            "algorithmic_bytes_per_packet": bpp, "algo": algo_name, "parallelism": f"dp{world}",
            "table_bytes": None if l2_mode else eng.table_bytes,
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": pmc_traffic(cfg, algo_name, n),
            "kernel_ms_mean": round(float(kms.mean()), 5), "kernel_ms_min": round(float(spread.min()), 5),
            "kernel_ms_p50": round(float(np.median(spread)), 5), "kernel_ms_max": round(float(spread.max()), 5),
            "kernel_ms_all": [round(float(x), 4) for x in spread],
            "timing": args.timing,
        },
        "bit_exact_sample": bit_exact,
    }

    # ---- N>1: root-scattered curve (SURVEY.md §8e curve 2; not `value`) ----
    # rank 0's resident batch is scattered over RCCL/xGMI, classified on every
    # rank, verdicts gathered back; bit-exact vs rank 0's own classify above.
    if world > 1 and not args.no_scatter and not frames_mode and not l2_mode:
        def classify_shard(sl, cnt):
            sl = sl.to(dev)  # gloo rehearsal: shards arrive in host memory
            p = torch.empty(cnt, dtype=torch.int32, device=dev)
            eng.classify_device(sl, 64, cnt, p, None, stream)
            return p
        root = d_slots if rank == 0 else None
        nd.scatter_classify_gather(root, n, 64, classify_shard, dev)  # warm-up
        times = []
        for _ in range(3):
            full, secs = nd.scatter_classify_gather(root, n, 64, classify_shard, dev)
            times.append(secs)
        if rank == 0:
            best = min(times)
            out["scatter_inclusive"] = {
                "mpps": round(n / best / 1e6, 1), "ms": round(best * 1e3, 3), "packets": n,
                "bytes_scattered": n * 64, "bit_exact_vs_local": bool(torch.equal(full.cpu(), port.cpu())),
            }

    # ---- PCIe-inclusive rate (not `value`) ----
    if rank == 0 and not args.no_host and not frames_mode:
        m = min(n, 1 << 22)
        pinned = torch.from_numpy(slots[: m * 64]).pin_memory().numpy()
        eng.classify_host(pinned, 64, m)
        t = time.perf_counter()
        hp, _ = eng.classify_host(pinned, 64, m)
        dt = time.perf_counter() - t
        out["host_inclusive_mpps"] = round(m / dt / 1e6, 1)
        out["host_inclusive_bit_exact_sample"] = bool((hp[idx[idx < m]] == got[idx[idx < m]]).all())

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if frames_mode:
            cb, cports = cpu_baseline_frames(frames, desc, a4, a6, args.cpu_seconds)
        else:
            cb, cports = cpu_baseline(slots, n, a4, a6, args.cpu_seconds, eth)
        cb["bit_exact_vs_gpu"] = bool((cports == got[: len(cports)]).all())
        cb["cpu_model"] = cpu_model()
        out["cpu_baseline"] = cb
    elif rank == 0:
        out["cpu_baseline"] = None

    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()
    return 0 if bit_exact else 1


if __name__ == "__main__":
    sys.exit(main())
