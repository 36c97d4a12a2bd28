"""Deterministic synthetic workloads for the benchmark configs.

Rules are produced as text rule files (the GetL3ACLFromTextTable format,
packet/acl.go:148) so every run exercises the real parser; packets as dense
64-byte slots (C1/C2/C4/C5) or packed IMIX frames (C3) laid out like DPDK mbuf
data rooms.  Everything is numpy-vectorised so 2^24-packet batches build in
seconds.

Config table (BASELINE.json "configs"):
  C1 firewall   examples/firewall/firewall.conf (4 text rules -> 4 ip4 + 1 ip6), 64 B
  C2 l3_1k      1 000 L3 rules (90% IPv4), ports ANY, 64 B           <- headline
  C3 l3l4_10k   10 000 L3+L4 rules, IMIX 64/570/1518 at 7:4:1
  C4 l3_1k x8   C2 sharded over 8 GPUs
  C5 l3l4_100k  100 000 rules with port ranges on both ports, 64 B

Rule distribution (§8d): prefix lengths uniform /8-/32 (IPv6 /16-/128);
each address field is ANY with p=0.2, but never both (a src=ANY dst=ANY
ports-ANY rule shadows every later rule of its protocol, which would collapse
the workload to a few dozen live rules); ID ANY/TCP/UDP at 2:1:1; outputs
Accept 60% / Reject 30% / numeric 2..15 10%.
Packet mix: 85% IPv4 (TCP/UDP/ICMP 45/45/10; IHL 5, 2% IHL 6..15),
12% IPv6 (TCP/UDP), 3% non-IP (ARP / VLAN); 50% of IP packets are built to
match a uniformly chosen rule of their family (the oracle decides the real
first match), 50% are uniformly random.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

RULE_SEEDS = {"c1": 0x5EED0001, "c2": 0x5EED0002, "c3": 0x5EED0003, "c4": 0x5EED0004, "c5": 0x5EED0005}
PACKET_SEEDS = {"c1": 0x9AC70001, "c2": 0x9AC70002, "c3": 0x9AC70003, "c4": 0x9AC70004, "c5": 0x9AC70005}


@dataclass
class RuleSpec:
    n_rules: int
    v6_frac: float = 0.10
    any_frac: float = 0.20
    # port modes per direction: (p_single, p_range, p_any)
    sport: tuple = (0.0, 0.0, 1.0)
    dport: tuple = (0.0, 0.0, 1.0)


SPECS = {
    "c2": RuleSpec(1000),
    "c3": RuleSpec(10000, sport=(0.0, 0.2, 0.8), dport=(0.5, 0.3, 0.2)),
    "c4": RuleSpec(1000),
    "c5": RuleSpec(100000, sport=(0.0, 0.7, 0.3), dport=(0.5, 0.4, 0.1)),
}


@dataclass
class GenRules:
    """Generator-side view of the rules (network-order integers)."""
    text: str
    # per family arrays, in file order of that family
    v4_src: np.ndarray      # uint32 BE value
    v4_src_len: np.ndarray  # prefix length, -1 = ANY
    v4_dst: np.ndarray
    v4_dst_len: np.ndarray
    v4_proto: np.ndarray    # 0 = ANY
    v4_sp: np.ndarray       # (n, 2) min, max
    v4_dp: np.ndarray
    v6_src: np.ndarray      # (n, 2) uint64 hi, lo
    v6_src_len: np.ndarray
    v6_dst: np.ndarray
    v6_dst_len: np.ndarray
    v6_proto: np.ndarray
    v6_sp: np.ndarray
    v6_dp: np.ndarray


def _ip4_text(v: int) -> str:
    return f"{v >> 24 & 255}.{v >> 16 & 255}.{v >> 8 & 255}.{v & 255}"


def _ip6_text(hi: int, lo: int) -> str:
    x = (hi << 64) | lo
    groups = [(x >> (112 - 16 * k)) & 0xFFFF for k in range(8)]
    return ":".join(f"{g:x}" for g in groups)


def _mask32(length: np.ndarray) -> np.ndarray:
    length = np.asarray(length, np.int64)
    m = np.where(length <= 0, 0, (0xFFFFFFFF << (32 - np.clip(length, 1, 32))) & 0xFFFFFFFF)
    return m.astype(np.uint64).astype(np.uint32)


def _mask64(length: np.ndarray) -> np.ndarray:
    """Mask of the top `length` bits of a 64-bit half (length clipped 0..64)."""
    length = np.clip(np.asarray(length, np.int64), 0, 64)
    out = np.zeros(length.shape, np.uint64)
    nz = length > 0
    out[nz] = (np.uint64(0xFFFFFFFFFFFFFFFF) << (np.uint64(64) - length[nz].astype(np.uint64)))
    return out


def _ports(rng, n, mode):
    p_single, p_range, _ = mode
    u = rng.random(n)
    lo = rng.integers(0, 65536, n)
    width = rng.integers(1, 4097, n)
    hi = np.minimum(lo + width, 65535)
    kind = np.where(u < p_single, 1, np.where(u < p_single + p_range, 2, 0))
    mn = np.where(kind == 0, 0, lo)
    mx = np.where(kind == 0, 65535, np.where(kind == 1, lo, hi))
    return np.stack([mn, mx], 1).astype(np.int64), kind


def _port_text(mn, mx, kind):
    if kind == 0:
        return "ANY"
    if kind == 1:
        return str(mn)
    return f"{mn}:{mx}"


def gen_rules(spec: RuleSpec, seed: int) -> GenRules:
    rng = np.random.default_rng(seed)
    n = spec.n_rules
    is6 = rng.random(n) < spec.v6_frac
    # address fields: ANY w.p. any_frac each, never both
    s_any = rng.random(n) < spec.any_frac
    d_any = rng.random(n) < spec.any_frac
    both = s_any & d_any
    d_any[both] = False
    proto_pick = rng.choice(np.array([0, 0, 6, 17]), n)
    sp, sk = _ports(rng, n, spec.sport)
    dp, dk = _ports(rng, n, spec.dport)
    u = rng.random(n)
    outs = np.where(u < 0.6, 1, np.where(u < 0.9, 0, rng.integers(2, 16, n)))
    len4s = rng.integers(8, 33, n)
    len4d = rng.integers(8, 33, n)
    len6s = rng.integers(16, 129, n)
    len6d = rng.integers(16, 129, n)
    a4s = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    a4d = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    a6s = rng.integers(0, np.iinfo(np.uint64).max, (n, 2), dtype=np.uint64, endpoint=True)
    a6d = rng.integers(0, np.iinfo(np.uint64).max, (n, 2), dtype=np.uint64, endpoint=True)
    # canonical network addresses
    a4s &= _mask32(len4s)
    a4d &= _mask32(len4d)
    for a, ln in ((a6s, len6s), (a6d, len6d)):
        a[:, 0] &= _mask64(ln)
        a[:, 1] &= _mask64(ln - 64)

    lines = ["# synthetic rules: src dst proto sport dport output"]
    for i in range(n):
        if is6[i]:
            src = "ANY" if s_any[i] else f"{_ip6_text(int(a6s[i, 0]), int(a6s[i, 1]))}/{len6s[i]}"
            dst = "ANY" if d_any[i] else f"{_ip6_text(int(a6d[i, 0]), int(a6d[i, 1]))}/{len6d[i]}"
        else:
            src = "ANY" if s_any[i] else f"{_ip4_text(int(a4s[i]))}/{len4s[i]}"
            dst = "ANY" if d_any[i] else f"{_ip4_text(int(a4d[i]))}/{len4d[i]}"
        proto = {0: "ANY", 6: "TCP", 17: "UDP"}[int(proto_pick[i])]
        out = {0: "Reject", 1: "Accept"}.get(int(outs[i]), str(int(outs[i])))
        lines.append(f"{src} {dst} {proto} {_port_text(sp[i, 0], sp[i, 1], sk[i])} "
                     f"{_port_text(dp[i, 0], dp[i, 1], dk[i])} {out}")
    text = "\n".join(lines) + "\n"

    v4, v6 = ~is6, is6
    return GenRules(
        text=text,
        v4_src=a4s[v4], v4_src_len=np.where(s_any, -1, len4s)[v4],
        v4_dst=a4d[v4], v4_dst_len=np.where(d_any, -1, len4d)[v4],
        v4_proto=proto_pick[v4], v4_sp=sp[v4], v4_dp=dp[v4],
        v6_src=a6s[v6], v6_src_len=np.where(s_any, -1, len6s)[v6],
        v6_dst=a6d[v6], v6_dst_len=np.where(d_any, -1, len6d)[v6],
        v6_proto=proto_pick[v6], v6_sp=sp[v6], v6_dp=dp[v6],
    )


def firewall_rules(text: str) -> GenRules:
    """GenRules view of a small hand-written rule file (C1: firewall.conf),
    parsed here only to steer packet generation (the engine parses the text)."""
    import ipaddress
    rows4, rows6 = [], []
    for line in text.splitlines():
        if not line or line[0] == "#":
            continue
        f = line.split()
        if len(f) == 5:
            f.append("false")
        src, dst, proto, sport, dport = f[:5]
        pr = {"ANY": 0, "TCP": 6, "tcp": 6, "UDP": 17, "udp": 17, "ICMP": 1, "icmp": 1}.get(proto, 0)

        def port(p):
            if p == "ANY":
                return (0, 65535)
            a, _, b = p.partition(":")
            return (int(a), int(b or a))
        fam = 4
        for a in (src, dst):
            if a != "ANY" and ":" in a:
                fam = 6
        nets = []
        for a in (src, dst):
            if a == "ANY":
                nets.append(None)
            else:
                nets.append(ipaddress.ip_network(a, strict=False))
        row = (nets, pr, port(sport), port(dport))
        if src == "ANY" and dst == "ANY":
            rows4.append(row)
            rows6.append(row)
        elif fam == 4:
            rows4.append(row)
        else:
            rows6.append(row)

    def v4cols(rows):
        s = np.array([int(r[0][0].network_address) if r[0][0] else 0 for r in rows], np.uint32)
        sl = np.array([r[0][0].prefixlen if r[0][0] else -1 for r in rows], np.int64)
        d = np.array([int(r[0][1].network_address) if r[0][1] else 0 for r in rows], np.uint32)
        dl = np.array([r[0][1].prefixlen if r[0][1] else -1 for r in rows], np.int64)
        return s, sl, d, dl

    def v6cols(rows):
        def hl(net):
            x = int(net.network_address) if net else 0
            return [x >> 64, x & 0xFFFFFFFFFFFFFFFF]
        s = np.array([hl(r[0][0]) for r in rows], np.uint64).reshape(-1, 2)
        sl = np.array([r[0][0].prefixlen if r[0][0] else -1 for r in rows], np.int64)
        d = np.array([hl(r[0][1]) for r in rows], np.uint64).reshape(-1, 2)
        dl = np.array([r[0][1].prefixlen if r[0][1] else -1 for r in rows], np.int64)
        return s, sl, d, dl

    s4, s4l, d4, d4l = v4cols(rows4)
    s6, s6l, d6, d6l = v6cols(rows6)
    return GenRules(
        text=text, v4_src=s4, v4_src_len=s4l, v4_dst=d4, v4_dst_len=d4l,
        v4_proto=np.array([r[1] for r in rows4], np.int64),
        v4_sp=np.array([r[2] for r in rows4], np.int64).reshape(-1, 2),
        v4_dp=np.array([r[3] for r in rows4], np.int64).reshape(-1, 2),
        v6_src=s6, v6_src_len=s6l, v6_dst=d6, v6_dst_len=d6l,
        v6_proto=np.array([r[1] for r in rows6], np.int64),
        v6_sp=np.array([r[2] for r in rows6], np.int64).reshape(-1, 2),
        v6_dp=np.array([r[3] for r in rows6], np.int64).reshape(-1, 2),
    )


def _inside(rng, base, length, bits_rand):
    """addr drawn inside prefix (base, length) — 32-bit; length -1 = ANY."""
    m = _mask32(np.where(length < 0, 0, length))
    return (base & m) | (bits_rand & ~m)


def _inside64(base_hi, base_lo, length, r_hi, r_lo):
    ln = np.where(length < 0, 0, length)
    mh, ml = _mask64(ln), _mask64(ln - 64)
    return (base_hi & mh) | (r_hi & ~mh), (base_lo & ml) | (r_lo & ~ml)


def _draw_ports(rng, rngs, n):
    """uniform port in [min, max] per row of rngs (n, 2)"""
    width = (rngs[:, 1] - rngs[:, 0] + 1).astype(np.int64)
    return (rngs[:, 0] + (rng.integers(0, 1 << 62, n) % width)).astype(np.int64)


def gen_headers(rules: GenRules, n: int, seed: int, match_frac: float = 0.5):
    """Header fields for n packets -> dict of column arrays."""
    rng = np.random.default_rng(seed)
    u = rng.random(n)
    kind = np.where(u < 0.85, 4, np.where(u < 0.97, 6, 0))  # 4 / 6 / non-IP
    if len(rules.v4_src) == 0:
        kind[kind == 4] = 0
    if len(rules.v6_src) == 0:
        kind[kind == 6] = 0
    pm = rng.random(n)
    proto = np.where(pm < 0.45, 6, np.where(pm < 0.9, 17, 1))
    proto[kind == 6] = np.where(rng.random(int((kind == 6).sum())) < 0.5, 6, 17)
    ihl = np.full(n, 5, np.int64)
    opt = (kind == 4) & (rng.random(n) < 0.02)
    ihl[opt] = rng.integers(6, 16, int(opt.sum()))
    sport = rng.integers(0, 65536, n)
    dport = rng.integers(0, 65536, n)
    src4 = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    dst4 = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    s6 = rng.integers(0, np.iinfo(np.uint64).max, (n, 2), dtype=np.uint64, endpoint=True)
    d6 = rng.integers(0, np.iinfo(np.uint64).max, (n, 2), dtype=np.uint64, endpoint=True)
    build = rng.random(n) < match_frac

    sel = np.nonzero(build & (kind == 4))[0]
    if len(sel):
        r = rng.integers(0, len(rules.v4_src), len(sel))
        src4[sel] = _inside(rng, rules.v4_src[r], rules.v4_src_len[r], src4[sel])
        dst4[sel] = _inside(rng, rules.v4_dst[r], rules.v4_dst_len[r], dst4[sel])
        rp = rules.v4_proto[r]
        proto[sel] = np.where(rp > 0, rp, proto[sel])
        sport[sel] = _draw_ports(rng, rules.v4_sp[r], len(sel))
        dport[sel] = _draw_ports(rng, rules.v4_dp[r], len(sel))
    sel = np.nonzero(build & (kind == 6))[0]
    if len(sel):
        r = rng.integers(0, len(rules.v6_src), len(sel))
        s6[sel, 0], s6[sel, 1] = _inside64(rules.v6_src[r, 0], rules.v6_src[r, 1], rules.v6_src_len[r],
                                           s6[sel, 0], s6[sel, 1])
        d6[sel, 0], d6[sel, 1] = _inside64(rules.v6_dst[r, 0], rules.v6_dst[r, 1], rules.v6_dst_len[r],
                                           d6[sel, 0], d6[sel, 1])
        rp = rules.v6_proto[r]
        proto[sel] = np.where(rp > 0, rp, proto[sel])
        sport[sel] = _draw_ports(rng, rules.v6_sp[r], len(sel))
        dport[sel] = _draw_ports(rng, rules.v6_dp[r], len(sel))
    nonip = np.where(rng.random(n) < 0.5, 0x0806, 0x8100)
    return dict(kind=kind, proto=proto, ihl=ihl, sport=sport, dport=dport, src4=src4, dst4=dst4,
                s6=s6, d6=d6, nonip=nonip, noise=rng)


def _put_be(buf, col, value, nbytes):
    v = np.asarray(value).astype(np.uint64)
    for k in range(nbytes):
        buf[:, col + k] = ((v >> np.uint64(8 * (nbytes - 1 - k))) & np.uint64(0xFF)).astype(np.uint8)


def write_frames(h, lengths: np.ndarray, width: int) -> np.ndarray:
    """Render headers into a (n, width) uint8 image of each frame's first
    `width` bytes (zero past the frame length)."""
    n = len(h["kind"])
    rng = h["noise"]
    buf = np.zeros((n, width), np.uint8)
    buf[:, 0:12] = rng.integers(0, 256, (n, 12), dtype=np.uint8)  # MACs
    kind = h["kind"]
    et = np.where(kind == 4, 0x0800, np.where(kind == 6, 0x86DD, h["nonip"]))
    _put_be(buf, 12, et, 2)
    m4 = kind == 4
    if m4.any():
        b = buf[m4]
        ihl = h["ihl"][m4]
        b[:, 14] = (0x40 | ihl).astype(np.uint8)
        _put_be(b, 16, np.maximum(lengths[m4] - 14, 20), 2)
        b[:, 22] = 64
        b[:, 23] = h["proto"][m4].astype(np.uint8)
        _put_be(b, 26, h["src4"][m4], 4)
        _put_be(b, 30, h["dst4"][m4], 4)
        # L4 ports at 14 + 4*IHL, only where they fall inside the rendered width
        l4 = 14 + 4 * ihl
        sp, dp = h["sport"][m4], h["dport"][m4]
        rows = np.arange(len(b))
        for off, val in ((0, sp >> 8), (1, sp & 255), (2, dp >> 8), (3, dp & 255)):
            col = l4 + off
            ok = col < width
            b[rows[ok], col[ok]] = val[ok].astype(np.uint8)
        buf[m4] = b
    m6 = kind == 6
    if m6.any():
        b = buf[m6]
        b[:, 14] = 0x60
        _put_be(b, 18, np.maximum(lengths[m6] - 54, 0), 2)
        b[:, 20] = h["proto"][m6].astype(np.uint8)
        b[:, 21] = 64
        _put_be(b, 22, h["s6"][m6, 0], 8)
        _put_be(b, 30, h["s6"][m6, 1], 8)
        _put_be(b, 38, h["d6"][m6, 0], 8)
        _put_be(b, 46, h["d6"][m6, 1], 8)
        if width >= 58:
            _put_be(b, 54, h["sport"][m6], 2)
            _put_be(b, 56, h["dport"][m6], 2)
        buf[m6] = b
    mo = kind == 0
    if mo.any():
        buf[mo, 14:width] = rng.integers(0, 256, (int(mo.sum()), width - 14), dtype=np.uint8)
    # zero everything at or past each frame's length
    cols = np.arange(width)[None, :]
    buf[cols >= lengths[:, None]] = 0
    return buf


def _parallel(fn, starts, workers):
    """Run fn(c0) for every chunk start; chunks are independent (seeded by
    their start), so the output does not depend on the worker count."""
    if workers <= 1 or len(starts) <= 1:
        for c0 in starts:
            fn(c0)
        return
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(min(workers, len(starts))) as ex:
        for f in [ex.submit(fn, c0) for c0 in starts]:
            f.result()


def _workers() -> int:
    try:
        import os
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except (AttributeError, OSError):
        return 1


def gen_slots(rules: GenRules, n: int, seed: int, stride: int = 64, chunk: int = 1 << 22,
              workers: int | None = None) -> np.ndarray:
    """n packets of 64 B frames in dense slots (n*stride bytes, zero padded)."""
    out = np.zeros((n, stride), np.uint8)
    w = min(stride, 64)

    def one(c0):
        c1 = min(n, c0 + chunk)
        h = gen_headers(rules, c1 - c0, seed + c0)
        out[c0:c1, :w] = write_frames(h, np.full(c1 - c0, 64), 64)[:, :w]

    _parallel(one, range(0, n, chunk), _workers() if workers is None else workers)
    return out.reshape(-1)


IMIX = ((64, 7), (570, 4), (1518, 1))


def gen_imix(rules: GenRules, n: int, seed: int, align: int = 64, chunk: int = 1 << 21,
             workers: int | None = None):
    """Packed IMIX frames: returns (frames uint8, desc uint64 = offset<<16 | len).

    Frames start on `align`-byte boundaries like mbuf data rooms; the first
    128 bytes of each frame carry the headers, the rest is zero payload."""
    assert align == 64
    rng = np.random.default_rng(seed ^ 0x1111)
    sizes = np.array([s for s, _ in IMIX])
    weights = np.array([w for _, w in IMIX], float)
    lengths = sizes[rng.choice(len(sizes), n, p=weights / weights.sum())]
    room = (lengths + align - 1) // align * align
    offs = np.zeros(n, np.int64)
    offs[1:] = np.cumsum(room)[:-1]
    total = int(offs[-1] + room[-1]) + 128  # slack so 80-byte reads stay in bounds
    frames = np.zeros(total, np.uint8)
    rows = frames.reshape(-1, 64)  # 64-byte lines; frame i starts at line offs[i] / 64

    def one(c0):
        c1 = min(n, c0 + chunk)
        h = gen_headers(rules, c1 - c0, seed + c0)
        img = write_frames(h, lengths[c0:c1], 128)
        line = offs[c0:c1] // 64
        rows[line] = img[:, :64]
        two = room[c0:c1] > 64  # never touch the next frame's room
        rows[line[two] + 1] = img[two, 64:]

    _parallel(one, range(0, n, chunk), _workers() if workers is None else workers)
    desc = (offs.astype(np.uint64) << np.uint64(16)) | lengths.astype(np.uint64)
    return frames, desc


# ---- L2 ACL workload (§8f: GetL2ACLFromTextTable rules, Ethernet headers) ----------

L2_RULE_SEED = 0x5EED0020
L2_PACKET_SEED = 0x9AC70020
_L2_IDS = [("ANY", 0), ("ipv4", 0x0800), ("IPv6", 0x86DD), ("arp", 0x0806)]


@dataclass
class GenL2Rules:
    text: str
    macs: np.ndarray  # (k, 6) uint8 pool the rules draw from


def _mac_text(m, style: int) -> str:
    h = [f"{b:02x}" for b in m]
    if style == 0:
        return ":".join(h)
    if style == 1:
        return "-".join(h).upper()
    return ".".join(h[i] + h[i + 1] for i in range(0, 6, 2))


def gen_l2_rules(n: int, seed: int = L2_RULE_SEED) -> GenL2Rules:
    """n L2 rules "Source Destination ID Rule": each MAC a pool address with
    p=0.6 else ANY (never both ANY unless ID is set, so rules stay live), MAC
    notations colon / dash / dotted, outputs Accept/Reject/numeric."""
    rng = np.random.default_rng(seed)
    pool = rng.integers(0, 256, (max(8, n // 2), 6), dtype=np.uint8)
    lines = ["# Source MAC, Destination MAC, L3 ID, Output port"]
    for _ in range(n):
        src = _mac_text(pool[rng.integers(len(pool))], int(rng.integers(3))) if rng.random() < 0.6 else "ANY"
        dst = _mac_text(pool[rng.integers(len(pool))], int(rng.integers(3))) if rng.random() < 0.6 else "ANY"
        ident = _L2_IDS[int(rng.integers(len(_L2_IDS)))][0]
        if src == "ANY" and dst == "ANY" and ident == "ANY":
            ident = "ipv6"
        r = rng.random()
        out = "Accept" if r < 0.6 else "Reject" if r < 0.9 else str(int(rng.integers(2, 16)))
        lines.append(f"{src} {dst} {ident} {out}")
    return GenL2Rules("\n".join(lines) + "\n", pool)


def gen_l2_slots(rules: GenL2Rules, n: int, seed: int = L2_PACKET_SEED, stride: int = 64) -> np.ndarray:
    """Dense slots whose Ethernet headers draw MACs from the rule pool (p=0.7)
    and EtherTypes from IPv4/IPv6/ARP/VLAN/random; bytes 14.. random."""
    rng = np.random.default_rng(seed)
    buf = rng.integers(0, 256, (n, stride), dtype=np.uint8)
    pool = rules.macs
    for off in (0, 6):
        take = rng.random(n) < 0.7
        buf[take, off:off + 6] = pool[rng.integers(0, len(pool), int(take.sum()))]
    et = np.array([0x0800, 0x86DD, 0x0806, 0x8100], np.uint16)[rng.integers(0, 4, n)]
    rnd = rng.random(n) < 0.1
    et[rnd] = rng.integers(0, 1 << 16, int(rnd.sum()), dtype=np.uint16)
    buf[:, 12] = et >> 8
    buf[:, 13] = et & 0xFF
    return buf.reshape(-1)
