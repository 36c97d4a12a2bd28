#!/usr/bin/env python3
"""bench.py — device-resident L3 ACL classification throughput on MI355X.

Headline (BASELINE.json "metric"): Mpackets/s of device-resident L3 ACL
classify, 64 B packets, 1 k rules (config C2), with the fraction of the HBM
roofline.  One step = one classify launch (nffacl_classify_device, the HIP
path) over the whole per-GPU batch of synthetic 64-byte slots already
resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1|c3|c4|c5|l2]
                  [--extra c1,c3,c5|none] [--algo auto|linear|indexed|hybrid]

At N = 1 the same process then measures the other single-GPU BASELINE.json
configs named by --extra (default C1: examples/firewall's firewall.conf, C3:
10 k rules on IMIX frames, C5: 100 k rules with port ranges — the "LDS
rule-table tiling stress") and reports them under "configs", each with its
own metric, roofline and CPU baseline; `value` stays the C2 headline.

Key order of the one JSON line: the contract's keys, "configs", the compact
"call_shapes", the PCIe-inclusive rate, and last a "summary" of every headline
figure, so that a reader who keeps only the line's tail still has them all.  (`--config l2` measures the L2 ACL kernel, SURVEY.md
§8f row 4 — not a BASELINE.json config.)

N > 1 runs under torch.distributed.run (one rank per GPU, RCCL): rank 0
generates the rule file and broadcasts its bytes over RCCL (the path's one real
exchange step, outside the timed region); every rank classifies its own
resident shard — no data-path collective ("scaling": "weak").  The
root-scattered deployment (dist.scatter of slots / dist.gather of verdicts)
is reported beside it as "scatter_inclusive".

Every JSON record carries:
  roofline     achieved = algorithmic bytes/packet (C2/C5: 64 B slot read +
               4 B port write; C3: 64 B first frame line + 8 B descriptor +
               4 B) x packets per launch / mean kernel time
               (HIP events on the launch stream); peak = 8 TB/s HBM3E;
               traffic = PMC bytes per launch from profiles/ (if collected)
  cpu_baseline the oracle (oracle/acl_oracle.c, the reference algorithm
               restated in C) on a bounded sample of the same packets, on
               this host's cores: the GPU box's CPU share (<= 16 threads,
               `value`), all visible cores, and 1 core; rank 0 at N = 1 only
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
METRICS = {
    "c1": "Mpackets/s device-resident L3 ACL classify, 64B pkts @firewall.conf (4 ip4 + 1 ip6 rules); % HBM roofline",
    "c2": METRIC,
    "c3": "Mpackets/s device-resident L3+L4 ACL classify, IMIX 64/570/1518B (7:4:1) frames @10k rules; % HBM roofline",
    "c4": METRIC,
    "c5": "Mpackets/s device-resident L3+L4 ACL classify, 64B pkts @100k rules with port ranges; % HBM roofline",
    "l2": "Mpackets/s device-resident L2 ACL classify, 64B pkts @256 rules (SURVEY.md §8f, not a BASELINE metric)",
}
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
# bytes per packet: 64 B slot + 4 B verdict; L2 reads the 16-byte Ethernet
# line + 4 B; C3 reads each frame's first 64-byte line + its 8-byte descriptor + 4 B
BYTES_PER_PACKET = {"l2": 20, "c3": 76}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def c3_bytes_per_packet(frames: np.ndarray, desc: np.ndarray) -> float:
    """Algorithmic bytes per IMIX packet: its first 64-byte line + 8-byte
    descriptor + 4-byte verdict, plus a second 64-byte line for IPv4 frames
    whose ports lie past byte 63 (IHL >= 12: L4 at 14 + 4 IHL >= 62) and that
    are longer than 64 bytes (bytes past a frame read as 0)."""
    off = (desc >> np.uint64(16)).astype(np.int64)
    ln = (desc & np.uint64(0xFFFF)).astype(np.int64)
    et = frames[off + 12].astype(np.int64) << 8 | frames[off + 13]
    ihl = frames[off + 14] & 0x0F
    second = (et == 0x0800) & (ihl >= 12) & (ln > 64)
    return round(64 + 8 + 4 + 64 * float(second.mean()), 3)


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
    """(HBM bytes per launch, where they come from) from the committed PMC
    summary of this config's kernel, if one matches: profile-derived (a
    separate rocprofv3 --pmc run of the same command, FETCH_SIZE x 2 +
    WRITE_SIZE per the MI355X guide), not measured by this run."""
    path = ROOT / "profiles" / "pmc_traffic.json"
    if not path.exists():
        return None, None
    try:
        d = json.loads(path.read_text())
        e = d.get(f"{cfg}:{algo}:{n}")
        if e is None:
            return None, None
        return float(e["bytes_per_launch"]), f"profile-derived: {e.get('source', '?')} (rocprofv3 --pmc, not this run)"
    except Exception:
        return None, None


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_topology():
    """(visible cores, sockets, cgroup CPU quota in cores or None)."""
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:
        visible = os.cpu_count() or 1
    sockets = set()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                sockets.add(line.split(":", 1)[1].strip())
    except OSError:
        pass
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    return visible, max(1, len(sockets)), quota


def cpu_leg(run, n: int, budget_s: float, what: str, all_budget_s: float = 2.0):
    """CPU baseline of the oracle: `run(count, threads)` classifies the first
    `count` packets of the workload and returns their ports.  Timed at the GPU
    box's CPU share (<= 16 threads, the reported `value`), on all visible
    cores, and on 1 core, each over a sample sized for its time budget."""
    visible, sockets, quota = cpu_topology()
    box = max(1, min(visible, 16))

    def timed(threads, budget):
        cal = min(n, 1 << 14)
        t = time.perf_counter()
        run(cal, threads)
        rate = cal / max(time.perf_counter() - t, 1e-6)
        sample = int(min(n, max(cal, rate * budget)))
        passes, done, dt, ports = 0, 0, 0.0, None
        while True:  # whole passes over the sample until ~budget of CPU work
            t = time.perf_counter()
            ports = run(sample, threads)
            dt += time.perf_counter() - t
            passes += 1
            done += sample
            if dt >= budget or passes >= 50:
                break
        return done / dt / 1e6, sample, passes, dt, ports

    v, sample, passes, dt, ports = timed(box, budget_s)
    out = {
        "value": round(v, 3), "unit": "Mpps", "cores": box, "kind": "port",
        "sample": f"first {sample} {what} x {passes} pass(es) (oracle/acl_oracle.c = acl.go l3ACL "
                  f"restated in C, {box} threads, {dt:.1f}s)",
    }
    v1, s1, _, _, _ = timed(1, min(budget_s, 3.0))
    out["single_core_mpps"] = round(v1, 3)
    if visible > box:
        va, sa, pa, da, _ = timed(visible, all_budget_s)
        out.update(value_all_cores=round(va, 3), cores_all=visible,
                   sample_all_cores=f"first {sa} {what} x {pa} pass(es), {visible} threads, {da:.1f}s")
    else:
        out.update(value_all_cores=round(v, 3), cores_all=visible)
    out.update(cpu_model=cpu_model(), sockets=sockets, cgroup_cpu_quota=quota)
    return out, ports[:sample]


def run_config(cfg: str, args, rank: int, world: int, local: int, dev, nd, headline: bool):
    """Measure one config on this rank: returns (record dict, state for the
    headline's extra legs)."""
    import torch
    import torch.distributed as dist
    import nffacl
    from nffacl import synth
    from oracle import oracle, rules_oracle as ro

    n = args.packets
    algo_id = {"auto": nffacl.ALGO_AUTO, "linear": nffacl.ALGO_LINEAR, "indexed": nffacl.ALGO_INDEXED,
               "hybrid": nffacl.ALGO_HYBRID}[args.algo if headline else "auto"]
    # ---- rules: rank 0 generates, RCCL broadcast of the rule file bytes ----
    text, gen = build_rules(cfg)
    text = nd.broadcast_rules(text if rank == 0 else None, dev)
    l2_mode = cfg == "l2"
    frames_mode = cfg == "c3"
    if l2_mode:
        rules = nffacl.L2Rules.parse_text(text)
        n4, n6 = rules.count(), 0
        eng = nffacl.L2Engine(rules, device=local, algo=algo_id)
    else:
        rules = nffacl.L3Rules.parse_text(text)
        n4, n6 = rules.counts()
        eng = nffacl.Engine(rules, device=local, algo=algo_id)
    algo_name = ALGO_NAMES[eng.algo]

    # ---- packets: per-rank shard, resident in HBM before timing ----
    t0 = time.perf_counter()
    seed = synth.PACKET_SEEDS.get(cfg, 0) + 7919 * rank
    slots = frames = desc = None
    if frames_mode:
        frames, desc = synth.gen_imix(gen, n, seed)
        d_frames = torch.from_numpy(frames).to(dev)
        d_desc = torch.from_numpy(desc.view(np.int64)).to(dev)
    elif l2_mode:
        slots = synth.gen_l2_slots(gen, n, synth.L2_PACKET_SEED + 7919 * rank)
        d_slots = torch.from_numpy(slots).to(dev)
    else:
        slots = synth.gen_slots(gen, n, seed)
        d_slots = torch.from_numpy(slots).to(dev)
    log(f"[rank {rank}] {cfg}: generated {n} packets in {time.perf_counter() - t0:.1f}s; "
        f"rules ip4={n4} ip6={n6}; algo={algo_name}")
    port = torch.empty(n, dtype=torch.int32, device=dev)
    permit = torch.empty((n + 63) // 64, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def launch():
        if frames_mode:
            eng.classify_frames_device(d_frames, d_desc, n, port, permit, stream)
        else:
            eng.classify_device(d_slots, 64, n, port, permit, stream)

    # headline: exactly W untimed launches (the driver's contract); the extra
    # configs (their own engine, tables and kernels, first used here) at least
    # 20, so that their K timed launches start on a warmed-up kernel too
    warm = args.warmup if headline else max(args.warmup, EXTRA_MIN_WARMUP)
    for _ in range(warm):
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
        for _ in range(args.steps):
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
    got = port.cpu().numpy().view(np.uint32)
    rng = np.random.default_rng(rank)
    idx = np.sort(rng.choice(n, min(n, 4096), replace=False))
    eth = a4 = a6 = None
    if l2_mode:
        eth = ro.parse_l2_text_table(text.encode()).array()
        want = oracle.l2_classify_slots(slots.reshape(n, 64)[idx].reshape(-1), 64, len(idx), eth, threads=4)
    else:
        a4, a6 = ro.parse_text_table(text.encode()).arrays()
        if frames_mode:
            want = oracle.classify_frames(frames, desc[idx], a4, a6, threads=4)
        else:
            want = oracle.classify_slots(slots.reshape(n, 64)[idx].reshape(-1), 64, len(idx), a4, a6, threads=4)
    bit_exact = bool((got[idx] == want).all())

    total = n * world * args.steps
    value = total / elapsed / 1e6
    mean_k = float(kms.mean()) / 1e3
    bpp = BYTES_PER_PACKET.get(cfg, 68)
    if frames_mode:  # exact per-config average: + the second line of IPv4 IHL >= 12 frames
        bpp = c3_bytes_per_packet(frames, desc)
    achieved = bpp * n / mean_k / 1e9
    rec = {
        "metric": METRICS[cfg],
        "value": round(value, 1),
        "unit": "Mpps",
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "steps": args.steps,
        "warmup": warm,
        "config": {
            "workload": WORKLOADS.get(cfg, cfg), "rules_ip4": n4, "rules_ip6": n6,
            "packets_per_gpu": n, "slot_bytes": None if frames_mode else 64,
            "algorithmic_bytes_per_packet": bpp, "algo": algo_name, "parallelism": f"dp{world}",
            "table_bytes": None if l2_mode else eng.table_bytes,
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": pmc_traffic(cfg, algo_name, n)[0],
            "traffic_source": pmc_traffic(cfg, algo_name, n)[1],
            "kernel_ms_mean": round(float(kms.mean()), 5), "kernel_ms_min": round(float(spread.min()), 5),
            "kernel_ms_p50": round(float(np.median(spread)), 5), "kernel_ms_max": round(float(spread.max()), 5),
            "timing": args.timing,
        },
        "bit_exact_sample": bit_exact,
    }
    state = dict(eng=eng, n=n, port=port, got=got, idx=idx, slots=slots, frames=frames, desc=desc,
                 d_slots=None if frames_mode else d_slots, a4=a4, a6=a6, eth=eth, stream=stream,
                 frames_mode=frames_mode, l2_mode=l2_mode)
    return rec, state


def cpu_baseline_for(cfg: str, st: dict, budget_s: float):
    from oracle import oracle
    a4, a6, n = st["a4"], st["a6"], st["n"]
    if st["l2_mode"]:
        slots, eth = st["slots"], st["eth"]
        return cpu_leg(lambda c, t: oracle.l2_classify_slots(slots, 64, c, eth, threads=t), n, budget_s,
                       "packets")
    if st["frames_mode"]:
        frames, desc = st["frames"], st["desc"]
        return cpu_leg(lambda c, t: oracle.classify_frames(frames, desc[:c], a4, a6, threads=t), n, budget_s,
                       "IMIX frames")
    slots = st["slots"]
    cb, ports = cpu_leg(lambda c, t: oracle.classify_slots(slots, 64, c, a4, a6, threads=t), n, budget_s,
                        "packets of rank 0's batch")
    m = min(n, 1 << 20)  # match statistics of the workload
    _, which = oracle.classify_slots_which(slots, 64, m, a4, a6, threads=16)
    hit = which >= 0
    cb["mean_first_match_index"] = round(float(which[hit].mean()), 1) if hit.any() else None
    cb["match_fraction"] = round(float(hit.mean()), 4)
    return cb, ports


EXTRA_MIN_WARMUP = 20  # untimed launches before an extra config's timed region (headline: --warmup)

SHAPE_RUNS = (  # (name, service kind, threads, packets per call, seconds)
    ("scalar_1_thread", "scalar", 1, 0, 1.0),
    ("scalar_32_threads", "scalar", 32, 0, 1.5),
    ("burst32_16_clones", "burst", 16, 32, 1.5),
    ("burst32_32_clones", "burst", 32, 32, 1.5),
)


def shape_runs():
    """SHAPE_RUNS, or NFFACL_BENCH_SHAPES="kind:threads:per_call:seconds,..." (experiments)."""
    spec = os.environ.get("NFFACL_BENCH_SHAPES")
    if not spec:
        return SHAPE_RUNS
    runs = []
    for item in spec.split(","):
        kind, threads, per, secs = item.split(":")
        runs.append((f"{kind}{per}_{threads}_threads", kind, int(threads), int(per), float(secs)))
    return tuple(runs)


def call_shapes(cfg: str, text: str, gen, cpu_mpps, local: int):
    """The reference's own call shapes through the resident consumer, on this
    config's rules: one packet per call from 1 and 32
    threads (SetSeparator / SetSplitter, firewall.go:54-57) and 32-packet
    bursts from 16 clones (VectorSeparateFunction, flow.go:131, 1487-1520),
    callers pinned to the GPU's NUMA node, every verdict checked against the
    oracle; beside them the oracle on the same CPUs (cpu_baseline.value: the
    box's 16-CPU share) — the same-CPU comparison.  Host-driven: packets and
    verdicts cross PCIe per call (never `value`)."""
    import ctypes
    import nffacl
    from nffacl import synth
    from oracle import oracle, rules_oracle as ro
    lib = ctypes.CDLL(str(ROOT / "nff-go_amd" / "libnffshapes.so"))
    lib.nffshapes_run.restype = ctypes.c_int
    lib.nffshapes_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p,  # the loaded libnffacl's entry points
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                  ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_double, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    n = 1 << 16
    slots = synth.gen_slots(gen, n, synth.PACKET_SEEDS.get(cfg, 0) + 31, stride=80)
    a4, a6 = ro.parse_text_table(text.encode()).arrays()
    expect = oracle.classify_slots(slots, 80, n, a4, a6, threads=16).astype(np.uint32)
    rules = nffacl.L3Rules.parse_text(text)
    node = nffacl.device_numa_node(local)
    res = {"packets_distinct": n, "slot_bytes": 80, "pinned_numa_node": node if node >= 0 else None,
           "cpu_same_cpus_mpps": cpu_mpps}
    svcs = {"scalar": nffacl.Service(local, mailboxes=128), "burst": nffacl.Service(local, mailboxes=32, burst=True)}
    try:
        for name, kind, threads, per, secs in shape_runs():
            o = (ctypes.c_double * 9)()
            fns = (ctypes.cast(nffacl._lib.nffacl_service_classify, ctypes.c_void_p),
                   ctypes.cast(nffacl._lib.nffacl_service_classify_burst, ctypes.c_void_p))
            before = svcs[kind].stats()
            st = lib.nffshapes_run(fns[0], fns[1], svcs[kind]._h, rules.handle, slots.ctypes.data, 80, n,
                                   expect.ctypes.data, threads, per, secs, node, o)
            if st != 0:
                res[name] = {"error": st}
                continue
            sst = svcs[kind].stats()
            d = {k: sst[k] - before[k] for k in ("polls", "groups", "timeouts", "retries", "launches", "torn")}
            res[name] = {"mpps": round(o[0], 3), "lat_us_p50": round(o[1], 2), "lat_us_p99": round(o[2], 2),
                         "wrong": int(o[3]), "calls": int(o[4]), "errors": int(o[8]),
                         "cpu_us_per_packet": round(o[5], 3), "cpus_busy": round(o[6], 2), "pinned": bool(o[7]),
                         "timeouts": d["timeouts"], "retries": d["retries"], "table_oob": sst["table_oob"],
                         # the consumer's view (means over its launches so far: poll = PCIe read
                         # issue -> data, group = classify + answer one request)
                         "consumer_poll_us": round(sst["poll_ns"] / 1e3, 2),
                         "consumer_group_us": round(sst["group_ns"] / 1e3, 2),
                         "polls_per_call": round(d["polls"] / max(1, d["groups"]), 2),
                         "torn_per_call": round(d["torn"] / max(1, d["groups"]), 3)}
            if cpu_mpps:
                res[name]["vs_cpu_same_cpus"] = round(o[0] / cpu_mpps, 3)
    finally:
        for v in svcs.values():
            v.close()
    res["bit_exact"] = all(isinstance(v, dict) and v.get("wrong") == 0 and v.get("errors") == 0
                           for k, v in res.items() if k in {r[0] for r in shape_runs()})
    return res


def text_of(cfg: str) -> str:
    return build_rules(cfg)[0]


def group_leg(st: dict, args, engine_ms: float, text: str, local: int) -> dict:
    """The C-ABI device group (nffacl_group_classify_device, one process
    driving every visible GPU: the reference's clones-in-one-process
    deployment, flow/scheduler.go:283-289) over the same resident batch:
    K launches timed like the headline, for groups of the first 1, 2, 4, ...
    visible devices (root = this rank's device).  At one device it must match
    the Engine's rate (no collective runs); on a multi-GPU node it is the
    curve a Go host would get (RCCL scatter / gather over xGMI, DESIGN.md
    §6).  Verdicts bit-exact vs the Engine's own classify of the batch."""
    import torch
    import nffacl
    ndev = torch.cuda.device_count()
    devs = [local] + [d for d in range(ndev) if d != local]
    rules = nffacl.L3Rules.parse_text(text)
    n, stream, d_slots = st["n"], st["stream"], st["d_slots"]
    dev = d_slots.device
    port = torch.empty(n, dtype=torch.int32, device=dev)
    permit = torch.empty((n + 63) // 64, dtype=torch.int64, device=dev)
    def timed(launch):
        for _ in range(max(args.warmup, 3)):
            launch()
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(args.steps):
            launch()
        b.record(stream)
        torch.cuda.synchronize(dev)
        return a.elapsed_time(b) / args.steps

    # the Engine again, timed the same way right before the groups (apples to apples)
    eng_ms = timed(lambda: st["eng"].classify_device(d_slots, 64, n, port, permit, stream))
    res = {"devices_visible": ndev, "packets": n, "engine_ms_bench": engine_ms, "engine_ms": round(eng_ms, 4),
           "curve": []}
    sizes = sorted({min(ndev, 1 << k) for k in range(8)})
    exact = True
    for size in sizes:
        try:
            grp = nffacl.Group(devs[:size], rules)
        except nffacl.NFError as e:
            res["curve"].append({"devices": size, "error": str(e)})
            exact = False
            break
        with grp:
            ms = timed(lambda: grp.classify_device(d_slots, 64, n, port, permit, stream))
        same = bool(torch.equal(port.cpu(), st["port"].cpu()))
        exact = exact and same
        res["curve"].append({"devices": size, "ms": round(ms, 4), "mpps": round(n / ms / 1e3, 1),
                             "vs_engine": round(eng_ms / ms, 4), "bit_exact_vs_engine": same})
    res["bit_exact_vs_engine"] = exact
    return res


def compact_shapes(res: dict) -> dict:
    """One config's call-shape record as it goes into the JSON line: per
    shape the rate, latency, exactness and same-CPU ratio (the consumer's
    counters stay out of the line)."""
    out = {k: res[k] for k in ("cpu_same_cpus_mpps", "pinned_numa_node", "bit_exact") if k in res}
    for name, v in res.items():
        if isinstance(v, dict):
            out[name] = {k: v[k] for k in ("mpps", "lat_us_p50", "lat_us_p99", "wrong", "errors", "timeouts",
                                           "vs_cpu_same_cpus", "error") if k in v}
    return out


def summary(out: dict, ok: bool, cfg: str) -> dict:
    """Every headline figure of the line in one small block (emitted last)."""
    def leg(r):
        rf = r.get("roofline", {})
        cb = r.get("cpu_baseline") or {}
        return {"gpps": round(r["value"] / 1e3, 2), "ms": r["ms_per_step"], "frac": rf.get("frac"),
                "exact": r.get("bit_exact_sample"), "cpu16_mpps": cb.get("value")}
    s = {cfg: leg(out)}
    for c, r in (out.get("configs") or {}).items():
        s[c] = leg(r)
    for k in ("host_inclusive_mpps", "host_inclusive_bit_exact_sample"):
        if k in out:
            s[k] = out[k]
    grp = out.get("device_group") or {}
    if grp.get("curve"):
        s["device_group"] = [{k: c.get(k) for k in ("devices", "mpps", "vs_engine")} for c in grp["curve"]]
    for c, r in (out.get("call_shapes") or {}).items():
        b = r.get("burst32_16_clones") or {}
        b32 = r.get("burst32_32_clones") or {}
        sc = r.get("scalar_32_threads") or {}
        s[f"shapes_{c}"] = {"burst16_mpps": b.get("mpps"), "burst16_vs_cpu": b.get("vs_cpu_same_cpus"),
                            "burst32_mpps": b32.get("mpps"), "scalar32_mpps": sc.get("mpps"),
                            "scalar32_vs_cpu": sc.get("vs_cpu_same_cpus"), "exact": r.get("bit_exact")}
    s["all_bit_exact"] = bool(ok)
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "l2"])
    ap.add_argument("--extra", default="c1,c3,c5",
                    help="N=1: further configs measured in the same process (comma list, or 'none')")
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
    ap.add_argument("--no-shapes", action="store_true",
                    help="N=1: skip the call-shape record (scalar calls / bursts through the resident consumer)")
    ap.add_argument("--no-group", action="store_true",
                    help="N=1: skip the C-ABI device-group leg (nffacl_group_classify_device)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N>1 (nccl = RCCL on ROCm)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
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
    rec, st = run_config(cfg, args, rank, world, local, dev, nd, headline=True)
    out = {
        "metric": rec["metric"], "value": rec["value"], "unit": "Mpps", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": rec["ms_per_step"],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (deterministic seeds; SURVEY.md §8d mix)",
        "config": rec["config"], "roofline": rec["roofline"], "bit_exact_sample": rec["bit_exact_sample"],
    }
    ok = rec["bit_exact_sample"]
    eng, n, got, idx = st["eng"], st["n"], st["got"], st["idx"]
    host = {}

    # ---- N>1: root-scattered curve (SURVEY.md §8e curve 2; not `value`) ----
    # rank 0's resident batch goes out with one dist.scatter (RCCL: the
    # root's sends to all peers concurrently over xGMI), every rank classifies
    # its shard, verdicts come back with one dist.gather; bit-exact vs rank
    # 0's own classify of the whole batch above.
    if world > 1:
        out["ranks"] = dist.get_world_size()
        out["backend"] = dist.get_backend()
        if out["backend"] == "nccl":  # RCCL on ROCm
            out["rccl_ranks"] = out["ranks"]
    if world > 1 and not args.no_scatter and not st["frames_mode"] and not st["l2_mode"]:
        stream = st["stream"]

        def classify_shard(sl, cnt):
            sl = sl.to(dev)  # gloo rehearsal: shards arrive in host memory
            p = torch.empty(cnt, dtype=torch.int32, device=dev)
            eng.classify_device(sl, 64, cnt, p, None, stream)
            return p
        root = st["d_slots"] if rank == 0 else None
        nd.scatter_classify_gather(root, n, 64, classify_shard, dev)  # warm-up
        times = []
        for _ in range(3):
            full, secs = nd.scatter_classify_gather(root, n, 64, classify_shard, dev)
            times.append(secs)
        if rank == 0:
            best = min(times)
            out["scatter_inclusive"] = {
                "mpps": round(n / best / 1e6, 1), "ms": round(best * 1e3, 3), "packets": n,
                "bytes_scattered": n * 64, "collectives": "dist.scatter + dist.gather",
                "bit_exact_vs_local": bool(torch.equal(full.cpu(), st["port"].cpu())),
            }

    # ---- PCIe-inclusive rate (not `value`) ----
    # L3ACLPort over host slots: pinned 64-byte slots in, the verdict array
    # in pinned memory too (the kernels read the slots and write the verdicts
    # over PCIe, nffacl_classify_host); best of 3 calls of 2^23 packets
    if rank == 0 and not args.no_host and not st["frames_mode"]:
        m = min(n, 1 << 23)
        pinned = torch.from_numpy(st["slots"][: m * 64]).pin_memory().numpy()
        hout = torch.empty(m, dtype=torch.int32).pin_memory().numpy().view(np.uint32)
        eng.classify_host(pinned, 64, m, out=hout, permit=False)
        best = float("inf")
        for _ in range(3):
            t = time.perf_counter()
            hp, _ = eng.classify_host(pinned, 64, m, out=hout, permit=False)
            best = min(best, time.perf_counter() - t)
        host = {"host_inclusive": {"packets": m, "gbps_in": round(m * 64 / best / 1e9, 1),
                                   "input": "pinned host 64 B slots", "output": "pinned host u32 verdicts"},
                "host_inclusive_mpps": round(m / best / 1e6, 1),
                "host_inclusive_bit_exact_sample": bool((hp[idx[idx < m]] == got[idx[idx < m]]).all())}
        ok = ok and host["host_inclusive_bit_exact_sample"]

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb, cports = cpu_baseline_for(cfg, st, args.cpu_seconds)
        cb["bit_exact_vs_gpu"] = bool((cports == got[: len(cports)]).all())
        out["cpu_baseline"] = cb
        ok = ok and cb["bit_exact_vs_gpu"]
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0 and world == 1 and not args.no_group and not st["frames_mode"] and not st["l2_mode"]:
        out["device_group"] = group_leg(st, args, rec["ms_per_step"], text_of(cfg), local)
        ok = ok and out["device_group"].get("bit_exact_vs_engine", False)
    shapes = {}
    do_shapes = rank == 0 and world == 1 and not args.no_shapes and cfg in ("c1", "c2", "c3", "c5")
    if do_shapes:
        text, gen = build_rules(cfg)
        shapes[cfg] = call_shapes(cfg, text, gen, (out.get("cpu_baseline") or {}).get("value"), local)
        ok = ok and shapes[cfg]["bit_exact"]
    eng.close()
    del st

    # ---- further single-GPU configs in the same process (N = 1) ----
    extras = [] if args.extra in ("", "none") or world > 1 else [c for c in args.extra.split(",") if c != cfg]
    if extras:
        out["configs"] = {}
    for c in extras:
        rec, st = run_config(c, args, rank, world, local, dev, nd, headline=False)
        if not args.no_cpu_baseline:
            cb, cports = cpu_baseline_for(c, st, max(3.0, args.cpu_seconds * 0.6))
            cb["bit_exact_vs_gpu"] = bool((cports == st["got"][: len(cports)]).all())
            rec["cpu_baseline"] = cb
            ok = ok and cb["bit_exact_vs_gpu"]
        ok = ok and rec["bit_exact_sample"]
        if do_shapes and c in ("c1", "c2", "c3", "c5"):
            text, gen = build_rules(c)
            shapes[c] = call_shapes(c, text, gen, (rec.get("cpu_baseline") or {}).get("value"), local)
            ok = ok and shapes[c]["bit_exact"]
        out["configs"][c] = rec
        st["eng"].close()
        del st
        torch.cuda.empty_cache()

    if shapes:
        out["call_shapes"] = {c: compact_shapes(v) for c, v in shapes.items()}
    out.update(host)
    if rank == 0:
        out["summary"] = summary(out, ok, cfg)
        print(json.dumps(out, separators=(",", ":")), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
