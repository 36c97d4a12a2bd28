"""HIP path vs the CPU oracle — bit-exact verdicts (run on an MI355X: -m gpu).

Every verdict here comes from libnffacl's HIP kernels through the C-ABI
(nffacl.Engine -> nffacl_classify_*).  The oracle (oracle/acl_oracle.c, pinned
by tests/test_oracle.py against the reference's KATs) is only the checker.
"""
import json

import numpy as np
import pytest

import nffacl
from nffacl import synth
from oracle import oracle, rules_oracle as ro

pytestmark = pytest.mark.gpu

ALGOS = [nffacl.ALGO_LINEAR, nffacl.ALGO_INDEXED, nffacl.ALGO_HYBRID]
THREADS = 16


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.init()
    return torch


def to_dev(torch, arr: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(arr)).to("cuda")


def classify(torch, eng, slots: np.ndarray, stride: int, n: int):
    d_slots = to_dev(torch, slots.view(np.uint8))
    port = torch.zeros(max(n, 1), dtype=torch.int32, device="cuda")
    permit = torch.zeros(max((n + 63) // 64, 1), dtype=torch.int64, device="cuda")
    eng.classify_device(d_slots, stride, n, port, permit)
    torch.cuda.synchronize()
    p = port.cpu().numpy().view(np.uint32)[:n]
    b = permit.cpu().numpy().view(np.uint64)[:(n + 63) // 64]
    return p, b


def permit_bits(port: np.ndarray) -> np.ndarray:
    n = len(port)
    bits = np.zeros((n + 63) // 64 * 64, np.uint64)
    bits[:n] = (port != 0).astype(np.uint64)
    bits = bits.reshape(-1, 64) << np.arange(64, dtype=np.uint64)[None, :]
    return np.bitwise_or.reduce(bits, axis=1)


def slot_buffer(frames, stride):
    buf = np.zeros((len(frames), stride), np.uint8)
    for i, f in enumerate(frames):
        f = f[:stride]
        buf[i, :len(f)] = np.frombuffer(f, np.uint8)
    return buf.reshape(-1)


# ---- reference known answers on the GPU -------------------------------------------

@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("stride", [64, 256])
def test_match_kats_gpu(torch_cuda, golden, algo, stride):
    """All 7369 cases of acl_internal_test.go:501-1141 through the HIP path."""
    torch = torch_cuda
    z = np.load(golden / "acl_match_kats.npz", allow_pickle=False)
    pk = json.loads((golden / "kat_packets.json").read_text())
    frames = [bytes.fromhex(pk[name]) for name in z["packet_names"]]
    slots = slot_buffer(frames, stride)
    d_slots = to_dev(torch, slots)
    total = len(z["c4_want"]) + len(z["c6_want"])
    out = torch.zeros((total, 8), dtype=torch.int32, device="cuda")
    engines, wants, pkts = [], [], []
    row = 0
    for fam in (4, 6):
        rules = z[f"c{fam}_rule"]
        for i in range(len(rules)):
            rs = nffacl.L3Rules.from_arrays(rules[i:i + 1], None) if fam == 4 else \
                nffacl.L3Rules.from_arrays(None, rules[i:i + 1])
            eng = nffacl.Engine(rs, algo=algo)
            eng.classify_device(d_slots, stride, len(frames), out[row])
            engines.append(eng)
            wants.append(int(z[f"c{fam}_want"][i]))
            pkts.append(int(z[f"c{fam}_packet"][i]))
            row += 1
            if len(engines) >= 256:  # keep device tables bounded
                torch.cuda.synchronize()
                for e in engines:
                    e.close()
                engines.clear()
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    verdict = got[np.arange(total), np.array(pkts)]
    bad = np.nonzero(verdict != np.array(wants, np.uint32))[0]
    assert len(bad) == 0, [(int(i), int(verdict[i]), wants[i]) for i in bad[:10]]


@pytest.mark.parametrize("algo", ALGOS)
def test_header_parse_kat_gpu(torch_cuda, golden, algo):
    """packet_test.go:22-338 frames: exact-match rule hits, each perturbed field misses."""
    torch = torch_cuda
    cases = json.loads((golden / "parse_l3_kat.json").read_text())
    frames = [bytes.fromhex(c["hex"]) for c in cases]
    slots = slot_buffer(frames, 64)
    for k, c in enumerate(cases):
        sp = ((c["src_port_le"] & 0xFF) << 8) | (c["src_port_le"] >> 8)
        dp = ((c["dst_port_le"] & 0xFF) << 8) | (c["dst_port_le"] >> 8)
        base = dict(output_number=7, src_addr=c["src_addr"], dst_addr=c["dst_addr"], src_mask=0xFFFFFFFF,
                    dst_mask=0xFFFFFFFF, id=c["proto"], id_mask=0xFF, valid=1, src_port_min=sp,
                    src_port_max=sp, dst_port_min=dp, dst_port_max=dp)
        variants = [({}, 7), ({"src_addr": c["src_addr"] ^ 0x01000000}, 0),
                    ({"dst_addr": c["dst_addr"] ^ 0x100}, 0), ({"id": c["proto"] ^ 0x10}, 0),
                    ({"src_port_min": (sp + 1) & 0xFFFF, "src_port_max": (sp + 1) & 0xFFFF}, 0),
                    ({"dst_port_min": (dp + 1) & 0xFFFF, "dst_port_max": (dp + 1) & 0xFFFF}, 0)]
        for over, want in variants:
            r = np.zeros(1, nffacl.RULE4)
            for key, v in {**base, **over}.items():
                r[key] = v
            with nffacl.Engine(nffacl.L3Rules.from_arrays(r), algo=algo) as eng:
                p, _ = classify(torch, eng, slots, 64, len(frames))
            assert p[k] == want, (k, over)


# ---- synthetic batches vs the oracle ---------------------------------------------

def _rules_and_arrays(text: str):
    return nffacl.L3Rules.parse_text(text), ro.parse_text_table(text.encode()).arrays()


@pytest.mark.parametrize("algo", ALGOS)
def test_firewall_conf_c1(torch_cuda, golden, algo):
    text = (golden / "rules" / "firewall.conf").read_text()
    rules, (a4, a6) = _rules_and_arrays(text)
    g = synth.firewall_rules(text)
    n = 1 << 18
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS["c1"])
    with nffacl.Engine(rules, algo=algo) as eng:
        p, b = classify(torch_cuda, eng, slots, 64, n)
    want = oracle.classify_slots(slots, 64, n, a4, a6, threads=THREADS)
    np.testing.assert_array_equal(p, want)
    np.testing.assert_array_equal(b, permit_bits(want))
    assert 0 < (want != 0).mean() < 1


@pytest.mark.parametrize("algo", ALGOS)
def test_c2_1k_rules(torch_cuda, algo):
    g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = (1 << 20) + 37  # ragged tail
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS["c2"])
    with nffacl.Engine(rules, algo=algo) as eng:
        p, b = classify(torch_cuda, eng, slots, 64, n)
    want = oracle.classify_slots(slots, 64, n, a4, a6, threads=THREADS)
    np.testing.assert_array_equal(p, want)
    np.testing.assert_array_equal(b, permit_bits(want))


@pytest.mark.parametrize("algo", ALGOS)
def test_c5_port_ranges(torch_cuda, algo):
    spec = synth.RuleSpec(20000, sport=(0.0, 0.7, 0.3), dport=(0.5, 0.4, 0.1))
    g = synth.gen_rules(spec, synth.RULE_SEEDS["c5"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = 1 << 16
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS["c5"])
    with nffacl.Engine(rules, algo=algo) as eng:
        p, _ = classify(torch_cuda, eng, slots, 64, n)
    np.testing.assert_array_equal(p, oracle.classify_slots(slots, 64, n, a4, a6, threads=THREADS))


@pytest.mark.parametrize("algo", ALGOS)
def test_c3_imix_frames(torch_cuda, algo):
    torch = torch_cuda
    spec = synth.RuleSpec(10000, sport=(0.0, 0.2, 0.8), dport=(0.5, 0.3, 0.2))
    g = synth.gen_rules(spec, synth.RULE_SEEDS["c3"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = 1 << 16
    frames, desc = synth.gen_imix(g, n, synth.PACKET_SEEDS["c3"])
    with nffacl.Engine(rules, algo=algo) as eng:
        port = torch.zeros(n, dtype=torch.int32, device="cuda")
        permit = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")
        eng.classify_frames_device(to_dev(torch, frames), to_dev(torch, desc.view(np.int64)), n, port, permit)
        torch.cuda.synchronize()
    want = oracle.classify_frames(frames, desc, a4, a6, threads=THREADS)
    got = port.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(permit.cpu().numpy().view(np.uint64), permit_bits(want))


@pytest.mark.parametrize("algo", ALGOS)
def test_ip_options_and_wide_slots(torch_cuda, algo):
    """IHL 0..15 with 128-byte slots: ports at bytes up to 77 are real bytes;
    with 64-byte slots the same frames read zeros past byte 63."""
    rng = np.random.default_rng(3)
    n = 4096
    frames = []
    for i in range(n):
        ihl = i % 16
        f = bytearray(rng.integers(0, 256, 128, dtype=np.uint8).tobytes())
        f[12:14] = b"\x08\x00"
        f[14] = 0x40 | ihl
        f[23] = [6, 17, 1][i % 3]
        frames.append(bytes(f))
    text = "\n".join(f"ANY ANY {p} {a}:{b} {c}:{d} {o}" for p, a, b, c, d, o in [
        ("TCP", 0, 30000, 0, 65535, 2), ("UDP", 20000, 65535, 100, 40000, 3), ("ANY", 0, 0, 0, 65535, 4),
        ("ANY", 0, 65535, 0, 0, 5), ("ANY", 1000, 50000, 1000, 50000, 6)]) + "\n"
    rules, (a4, a6) = _rules_and_arrays(text)
    for stride in (64, 128):
        slots = slot_buffer(frames, stride)
        with nffacl.Engine(rules, algo=algo) as eng:
            p, _ = classify(torch_cuda, eng, slots, stride, n)
        np.testing.assert_array_equal(p, oracle.classify_slots(slots, stride, n, a4, a6))


@pytest.mark.parametrize("algo", ALGOS)
def test_ip_options_frames_vlan(torch_cuda, algo):
    """IHL 0..15 on packed frames (the frames kernels take ports inside the
    first 64 bytes from registers and read memory only past them), untagged
    and 802.1Q-tagged, frame lengths 128 / 80 / 64 / 61 / 40 (bytes past the
    length read as 0), with and without NFFACL_PARSE_VLAN."""
    torch = torch_cuda
    rng = np.random.default_rng(13)
    n = 4099
    lens = [128, 80, 64, 61, 40]
    buf, desc, off = [], [], 0
    for i in range(n):
        ihl = i % 16
        f = bytearray(rng.integers(0, 256, 132, dtype=np.uint8).tobytes())
        f[12:14] = b"\x08\x00"
        f[14] = 0x40 | ihl
        f[23] = [6, 17, 1][i % 3]
        if (i // 16) % 2:  # tagged: TPID 0x8100 + TCI, the header 4 bytes later
            f = f[:12] + bytearray(b"\x81\x00\x00\x05") + f[12:128]
        ln = lens[(i // 32) % len(lens)]
        room = (ln + 63) // 64 * 64
        buf.append(bytes(f[:ln]) + bytes(room - ln))
        desc.append(off << 16 | ln)
        off += room
    frames = np.frombuffer(b"".join(buf), np.uint8).copy()
    desc = np.array(desc, np.uint64)
    text = "\n".join(f"ANY ANY {p} {a}:{b} {c}:{d} {o}" for p, a, b, c, d, o in [
        ("TCP", 0, 30000, 0, 65535, 2), ("UDP", 20000, 65535, 100, 40000, 3), ("ANY", 0, 0, 0, 65535, 4),
        ("ANY", 0, 65535, 0, 0, 5), ("ANY", 1000, 50000, 1000, 50000, 6)]) + "\n"
    rules, (a4, a6) = _rules_and_arrays(text)
    d_frames, d_desc = to_dev(torch, frames), to_dev(torch, desc.view(np.int64))
    with nffacl.Engine(rules, algo=algo) as eng:
        for flags in (0, nffacl.PARSE_VLAN):
            port = torch.zeros(n, dtype=torch.int32, device="cuda")
            eng.classify_frames_device(d_frames, d_desc, n, port, None, None, flags)
            torch.cuda.synchronize()
            want = oracle.classify_frames(frames, desc, a4, a6, flags=flags)
            np.testing.assert_array_equal(port.cpu().numpy().view(np.uint32), want)
            assert len(set(want.tolist())) > 3


@pytest.mark.parametrize("algo", ALGOS)
def test_port_free_rules_options_vlan(torch_cuda, algo):
    """Rules that constrain no port (C2's shape) compile INDEXED tables that
    take the no-port kernel (kTabLdsNP: no option-port reads, no port tests):
    IHL 0..15, tagged and untagged, 64/128-byte slots and packed frames, with
    and without NFFACL_PARSE_VLAN, against the oracle."""
    torch = torch_cuda
    rng = np.random.default_rng(29)
    n = 4099
    raw = []
    for i in range(n):
        f = bytearray(rng.integers(0, 256, 132, dtype=np.uint8).tobytes())
        f[12:14] = b"\x08\x00"
        f[14] = 0x40 | (i % 16)
        f[23] = [6, 17, 1][i % 3]
        if (i // 16) % 2:
            f = f[:12] + bytearray(b"\x81\x00\x00\x05") + f[12:128]
        raw.append(bytes(f[:128]))
    text = "\n".join([
        "ANY 128.0.0.0/1 TCP ANY ANY 2", "0.0.0.0/1 ANY UDP ANY ANY 3", "ANY ANY ICMP ANY ANY 4",
        "64.0.0.0/2 192.0.0.0/2 ANY ANY ANY 5", "10.0.0.0/8 ANY ANY ANY ANY 6", "ANY 0.0.0.0/3 TCP ANY ANY 7"]) + "\n"
    rules, (a4, a6) = _rules_and_arrays(text)
    for stride in (64, 128):
        slots = slot_buffer(raw, stride)
        with nffacl.Engine(rules, algo=algo) as eng:
            p, _ = classify(torch, eng, slots, stride, n)
        want = oracle.classify_slots(slots, stride, n, a4, a6)
        np.testing.assert_array_equal(p, want)
        assert len(set(want.tolist())) > 3
    frames = np.frombuffer(b"".join(raw), np.uint8).copy()
    desc = (np.arange(n, dtype=np.uint64) * np.uint64(128)) << np.uint64(16) | np.uint64(128)
    d_frames, d_desc = to_dev(torch, frames), to_dev(torch, desc.view(np.int64))
    with nffacl.Engine(rules, algo=algo) as eng:
        for flags in (0, nffacl.PARSE_VLAN):
            port = torch.zeros(n, dtype=torch.int32, device="cuda")
            eng.classify_frames_device(d_frames, d_desc, n, port, None, None, flags)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(port.cpu().numpy().view(np.uint32),
                                          oracle.classify_frames(frames, desc, a4, a6, flags=flags))


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000])
def test_ragged_sizes(torch_cuda, algo, n):
    g = synth.gen_rules(synth.RuleSpec(300), 11)
    rules, (a4, a6) = _rules_and_arrays(g.text)
    slots = synth.gen_slots(g, n, 12)
    with nffacl.Engine(rules, algo=algo) as eng:
        p, b = classify(torch_cuda, eng, slots, 64, n)
    want = oracle.classify_slots(slots, 64, n, a4, a6)
    np.testing.assert_array_equal(p, want)
    np.testing.assert_array_equal(b, permit_bits(want))


def test_empty_batch_and_empty_rules(torch_cuda):
    torch = torch_cuda
    empty = nffacl.L3Rules.from_arrays(None, None)
    g = synth.gen_rules(synth.RuleSpec(10), 1)
    slots = synth.gen_slots(g, 256, 2)
    with nffacl.Engine(empty) as eng:
        p, b = classify(torch, eng, slots, 64, 256)
        assert not p.any() and not b.any()
        eng.classify_device(to_dev(torch, slots), 64, 0, None, None)  # n == 0 is a no-op
    only6 = nffacl.L3Rules.parse_text(b"::/0 ANY ANY ANY ANY 9\n")
    with nffacl.Engine(only6) as eng:
        p, _ = classify(torch, eng, slots, 64, 256)
    want = oracle.classify_slots(slots, 64, 256, *ro.parse_text_table(b"::/0 ANY ANY ANY ANY 9\n").arrays())
    np.testing.assert_array_equal(p, want)


def test_invalid_arguments(torch_cuda):
    torch = torch_cuda
    rules = nffacl.L3Rules.parse_text(b"ANY ANY ANY ANY ANY Accept\n")
    with nffacl.Engine(rules) as eng:
        buf = torch.zeros(4096, dtype=torch.uint8, device="cuda")
        out = torch.zeros(64, dtype=torch.int32, device="cuda")
        for stride in (0, 48, 72):
            with pytest.raises(nffacl.NFError):
                eng.classify_device(buf, stride, 16, out)
        with pytest.raises(nffacl.NFError):
            eng.classify_device(buf.data_ptr() + 4, 64, 16, out)  # misaligned slots


def test_swap_rules_between_batches(torch_cuda):
    torch = torch_cuda
    g = synth.gen_rules(synth.RuleSpec(500), 21)
    n = 1 << 14
    slots = synth.gen_slots(g, n, 22)
    r1, (a4, a6) = _rules_and_arrays(g.text)
    r2, (b4, b6) = _rules_and_arrays(synth.gen_rules(synth.RuleSpec(700), 23).text)
    with nffacl.Engine(r1) as eng:
        p1, _ = classify(torch, eng, slots, 64, n)
        eng.swap_rules(r2)
        p2, _ = classify(torch, eng, slots, 64, n)
        eng.swap_rules(r1)
        p3, _ = classify(torch, eng, slots, 64, n)
    np.testing.assert_array_equal(p1, oracle.classify_slots(slots, 64, n, a4, a6))
    np.testing.assert_array_equal(p2, oracle.classify_slots(slots, 64, n, b4, b6))
    np.testing.assert_array_equal(p3, p1)


def test_classify_host_matches_device(torch_cuda):
    g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = (1 << 21) + 5  # > one pipeline chunk, ragged
    slots = synth.gen_slots(g, n, 99)
    with nffacl.Engine(rules) as eng:
        port, permit = eng.classify_host(slots, 64, n)
    want = oracle.classify_slots(slots, 64, n, a4, a6, threads=THREADS)
    np.testing.assert_array_equal(port, want)
    np.testing.assert_array_equal(permit, (want != 0).astype(np.uint8))


@pytest.mark.parametrize("stride", [64, 80])
def test_classify_host_pinned_zero_copy(torch_cuda, stride):
    """Pinned input: the kernel reads the host slots over PCIe itself (no
    copies) and writes the verdicts into mapped memory; ragged n, > one chunk,
    pinned and pageable verdict buffers."""
    torch = torch_cuda
    g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = (1 << 21) + 37
    slots = synth.gen_slots(g, n, 123, stride=stride)
    pinned = torch.from_numpy(slots).pin_memory()
    want = oracle.classify_slots(slots, stride, n, a4, a6, threads=THREADS)
    with nffacl.Engine(rules) as eng:
        port, permit = eng.classify_host(pinned.numpy(), stride, n)
        np.testing.assert_array_equal(port, want)
        np.testing.assert_array_equal(permit, (want != 0).astype(np.uint8))
        out = torch.zeros(n, dtype=torch.int32).pin_memory()  # pinned verdicts: written in place
        st = nffacl._classify_host(eng._h, pinned.data_ptr(), stride, n, out.data_ptr(), None, 0)
        assert st == nffacl.OK
        np.testing.assert_array_equal(out.numpy().view(np.uint32), want)


@pytest.mark.parametrize("dma,bufs,chunk", [(0, 2, 12), (0, 4, 14), (1, 2, 12), (1, 3, 13), (1, 4, 20)])
def test_classify_host_pipeline_variants(torch_cuda, monkeypatch, dma, bufs, chunk):
    """nffacl_classify_host's forms (NFFACL_TUNE_HOST_*): zero-copy or DMA'd
    pinned input, pageable input (staged), 2-4 buffers in flight, chunks of
    2^12-2^20 packets (many chunks: the buffers wrap), verdicts into pinned or
    pageable memory — all bit-exact vs the oracle."""
    torch = torch_cuda
    monkeypatch.setenv("NFFACL_TUNE_HOST_DMA", str(dma))
    monkeypatch.setenv("NFFACL_TUNE_HOST_BUFS", str(bufs))
    monkeypatch.setenv("NFFACL_TUNE_HOST_CHUNK", str(chunk))
    g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = 11 * (1 << chunk) // 2 + 29 if chunk < 20 else (1 << 20) + 29
    slots = synth.gen_slots(g, n, 7 + chunk, stride=80)
    want = oracle.classify_slots(slots, 80, n, a4, a6, threads=THREADS)
    pinned = torch.from_numpy(slots).pin_memory()
    out = torch.zeros(n, dtype=torch.int32).pin_memory().numpy().view(np.uint32)
    with nffacl.Engine(rules) as eng:
        port, permit = eng.classify_host(slots, 80, n)  # pageable in and out
        np.testing.assert_array_equal(port, want)
        np.testing.assert_array_equal(permit, (want != 0).astype(np.uint8))
        port, _ = eng.classify_host(pinned.numpy(), 80, n, out=out, permit=False)  # pinned in and out
        np.testing.assert_array_equal(out, want)
        port, permit = eng.classify_host(pinned.numpy(), 80, n)  # pinned in, pageable out
        np.testing.assert_array_equal(port, want)
        np.testing.assert_array_equal(permit, (want != 0).astype(np.uint8))


def test_stability_separate_split_proportions(torch_cuda, golden):
    """testSingleWorkingFF.go: separate -> exactly the dst-port-111 third is
    permitted; split -> outputs 1/2 by dst port (test-*.conf)."""
    n = 3 * 4000
    frames = []
    for i in range(n):
        f = bytearray(bytes.fromhex(json.loads((golden / "kat_packets.json").read_text())["ipv4_udp"]))
        dport = (111, 222, 333)[i % 3]
        f[36:38] = dport.to_bytes(2, "big")
        frames.append(bytes(f))
    slots = slot_buffer(frames, 64)
    sep = nffacl.L3Rules.from_text_file(golden / "rules" / "test-separate-l3rules.conf")
    with nffacl.Engine(sep) as eng:
        p, _ = classify(torch_cuda, eng, slots, 64, n)
    assert (p != 0).sum() == n // 3 and (p[0::3] == 1).all() and not p[1::3].any() and not p[2::3].any()
    split = nffacl.L3Rules.from_text_file(golden / "rules" / "test-split.conf")
    with nffacl.Engine(split) as eng:
        p, _ = classify(torch_cuda, eng, slots, 64, n)
    assert (p[0::3] == 1).all() and (p[1::3] == 2).all() and (p[2::3] == 3).all()
    # dhandle (test-handle-l3rules.conf): the kept third
    handle = nffacl.L3Rules.from_text_file(golden / "rules" / "test-handle-l3rules.conf")
    with nffacl.Engine(handle) as eng:
        p, _ = classify(torch_cuda, eng, slots, 64, n)
    assert (p != 0).sum() == n // 3 and (p[0::3] == 1).all()
    # split scenario generator (generatePacket, :425-431): every 5th packet to
    # dst port 111, the rest to 222 -> outputs 1 / 2 at exactly 20 / 80 %
    frames5 = []
    for i in range(n):
        f = bytearray(frames[i])
        f[36:38] = (111 if i % 5 == 0 else 222).to_bytes(2, "big")
        frames5.append(bytes(f))
    with nffacl.Engine(split) as eng:
        p, _ = classify(torch_cuda, eng, slot_buffer(frames5, 64), 64, n)
    assert (p == 1).sum() * 5 == n and (p == 2).sum() * 5 == 4 * n


# ---- BASELINE-size properties (2^24 packets, C2) ------------------------------------

def test_full_size_c2_properties(torch_cuda):
    """At the bench size: linear == indexed on every packet, a 2^16 random
    sample equals the oracle, and classifying two halves separately equals
    classifying the whole batch (size independence)."""
    torch = torch_cuda
    g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = 1 << 24
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS["c2"])
    d_slots = to_dev(torch, slots)
    del slots
    outs = {}
    for algo in ALGOS:
        with nffacl.Engine(rules, algo=algo) as eng:
            port = torch.zeros(n, dtype=torch.int32, device="cuda")
            eng.classify_device(d_slots, 64, n, port)
            half = torch.zeros(n, dtype=torch.int32, device="cuda")
            h = n // 2 + 64 * 3 + 17
            eng.classify_device(d_slots, 64, h, half)
            eng.classify_device(d_slots.data_ptr() + h * 64, 64, n - h, half.data_ptr() + h * 4)
            torch.cuda.synchronize()
            assert torch.equal(port, half)
            outs[algo] = port
    assert torch.equal(outs[nffacl.ALGO_LINEAR], outs[nffacl.ALGO_INDEXED])
    assert torch.equal(outs[nffacl.ALGO_LINEAR], outs[nffacl.ALGO_HYBRID])
    rng = np.random.default_rng(5)
    idx = np.sort(rng.choice(n, 1 << 16, replace=False))
    sample = d_slots.view(n, 64)[torch.from_numpy(idx).to("cuda")].cpu().numpy().reshape(-1)
    want = oracle.classify_slots(sample, 64, len(idx), a4, a6, threads=THREADS)
    got = outs[nffacl.ALGO_LINEAR].cpu().numpy().view(np.uint32)[idx]
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("flat", [0, 1, 2])
def test_full_size_c5_hybrid(torch_cuda, monkeypatch, flat):
    """C5 (100k rules with port ranges) at 2^22 packets: HYBRID (AUTO's choice)
    == INDEXED read from global memory on every packet, and a 2^14 random
    sample equals the oracle."""
    torch = torch_cuda
    monkeypatch.setenv("NFFACL_TUNE_FLAT", str(flat))
    g = synth.gen_rules(synth.SPECS["c5"], synth.RULE_SEEDS["c5"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = 1 << 22
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS["c5"])
    d_slots = to_dev(torch, slots)
    del slots
    outs = {}
    for algo in (nffacl.ALGO_AUTO, nffacl.ALGO_INDEXED):
        with nffacl.Engine(rules, algo=algo) as eng:
            assert eng.algo == (nffacl.ALGO_HYBRID if algo == nffacl.ALGO_AUTO else nffacl.ALGO_INDEXED)
            port = torch.zeros(n, dtype=torch.int32, device="cuda")
            eng.classify_device(d_slots, 64, n, port)
            torch.cuda.synchronize()
            outs[algo] = port
    assert torch.equal(outs[nffacl.ALGO_AUTO], outs[nffacl.ALGO_INDEXED])
    rng = np.random.default_rng(7)
    idx = np.sort(rng.choice(n, 1 << 14, replace=False))
    sample = d_slots.view(n, 64)[torch.from_numpy(idx).to("cuda")].cpu().numpy().reshape(-1)
    want = oracle.classify_slots(sample, 64, len(idx), a4, a6, threads=THREADS)
    np.testing.assert_array_equal(outs[nffacl.ALGO_AUTO].cpu().numpy().view(np.uint32)[idx], want)


def test_full_size_c3_hybrid(torch_cuda):
    """C3 at the bench size: 2^24 IMIX (64/570/1518 at 7:4:1) packed frames,
    10 k L3+L4 rules — HYBRID (AUTO's choice) == INDEXED read from global
    memory on every frame, classifying two halves separately == the whole
    batch, and a 2^14 random sample equals the oracle."""
    torch = torch_cuda
    g = synth.gen_rules(synth.SPECS["c3"], synth.RULE_SEEDS["c3"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = 1 << 24
    frames, desc = synth.gen_imix(g, n, synth.PACKET_SEEDS["c3"])
    d_frames = to_dev(torch, frames)
    d_desc = torch.from_numpy(desc.view(np.int64)).to("cuda")
    outs = {}
    for algo in (nffacl.ALGO_AUTO, nffacl.ALGO_INDEXED):
        with nffacl.Engine(rules, algo=algo) as eng:
            assert eng.algo == (nffacl.ALGO_HYBRID if algo == nffacl.ALGO_AUTO else nffacl.ALGO_INDEXED)
            port = torch.zeros(n, dtype=torch.int32, device="cuda")
            eng.classify_frames_device(d_frames, d_desc, n, port)
            if algo == nffacl.ALGO_AUTO:
                half = torch.zeros(n, dtype=torch.int32, device="cuda")
                h = n // 2 + 64 * 5 + 29
                eng.classify_frames_device(d_frames, d_desc, h, half)
                eng.classify_frames_device(d_frames, d_desc.data_ptr() + h * 8, n - h, half.data_ptr() + h * 4)
                torch.cuda.synchronize()
                assert torch.equal(port, half)
            torch.cuda.synchronize()
            outs[algo] = port
    assert torch.equal(outs[nffacl.ALGO_AUTO], outs[nffacl.ALGO_INDEXED])
    rng = np.random.default_rng(11)
    idx = np.sort(rng.choice(n, 1 << 14, replace=False))
    want = oracle.classify_frames(frames, desc[idx], a4, a6, threads=THREADS)
    np.testing.assert_array_equal(outs[nffacl.ALGO_AUTO].cpu().numpy().view(np.uint32)[idx], want)


@pytest.mark.parametrize("coarse,dir8,rounds", [("1", "1", None), ("0", "0", None), ("1", "1", "2")])
def test_c5_flat_lds_layout_options(torch_cuda, monkeypatch, coarse, dir8, rounds):
    """The flat-LDS layout options besides the default (u8 directories, no
    coarse slots): coarse address slots (five generalized slots: the NS = 5
    kernels) and u16 directories, on 64-byte slots and IMIX frames, against
    the oracle.  rounds "2" (ADVICE round 4, medium): generalized slots with
    NFFACL_TUNE_ROUNDS=2 still launch their 4-round kernel with its scratch."""
    torch = torch_cuda
    monkeypatch.setenv("NFFACL_TUNE_COARSE", coarse)
    monkeypatch.setenv("NFFACL_TUNE_DIR8", dir8)
    if rounds:
        monkeypatch.setenv("NFFACL_TUNE_ROUNDS", rounds)
    g = synth.gen_rules(synth.SPECS["c5"], synth.RULE_SEEDS["c5"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = (1 << 16) + 3
    slots = synth.gen_slots(g, n, 31)
    with nffacl.Engine(rules, algo=nffacl.ALGO_HYBRID) as eng:
        p, b = classify(torch, eng, slots, 64, n)
        want = oracle.classify_slots(slots, 64, n, a4, a6, threads=THREADS)
        np.testing.assert_array_equal(p, want)
        np.testing.assert_array_equal(b, permit_bits(want))
        frames, desc = synth.gen_imix(g, 1 << 14, 32)
        port = torch.zeros(1 << 14, dtype=torch.int32, device="cuda")
        eng.classify_frames_device(to_dev(torch, frames), to_dev(torch, desc.view(np.int64)), 1 << 14, port)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(port.cpu().numpy().view(np.uint32),
                                      oracle.classify_frames(frames, desc, a4, a6, threads=THREADS))


@pytest.mark.parametrize("case", ["grid_overflow", "dir_overflow"])
def test_c5_fine_grids_when_offsets_overflow_gpu(torch_cuda, case):
    """ADVICE round 4 (high), on the GPU: C5 plus 300 rules that overflow a
    fine grid's / a 1-D slot's u8 offsets (tests/test_index_compile.py
    test_hybrid_fine_grids_when_offsets_overflow) compile to a table that
    fits the LDS and classify exactly as the oracle, packets aimed at the
    added rules included."""
    torch = torch_cuda
    g = synth.gen_rules(synth.SPECS["c5"], synth.RULE_SEEDS["c5"])
    line = ("ANY 33.128.0.0/9 TCP ANY 8192:9000 Accept" if case == "grid_overflow"
            else "ANY 44.55.66.77/32 UDP 1000:2000 ANY Reject")
    text = g.text + (line + "\n") * 300
    rules, (a4, a6) = _rules_and_arrays(text)
    n = (1 << 16) + 9
    slots = synth.gen_slots(g, n, 41)
    for i in range(0, n, 37):
        pk = slots[i * 64:(i + 1) * 64]
        pk[12:14] = (0x08, 0x00)
        pk[14] = 0x45
        pk[23] = 6 if case == "grid_overflow" else 17
        pk[30:34] = (33, 200, 1, 2) if case == "grid_overflow" else (44, 55, 66, 77)
        pk[34:38] = (0x05, 0xDC, 0x21, 0x98)
    with nffacl.Engine(rules, algo=nffacl.ALGO_HYBRID) as eng:
        p, b = classify(torch, eng, slots, 64, n)
        want = oracle.classify_slots(slots, 64, n, a4, a6, threads=THREADS)
        np.testing.assert_array_equal(p, want)
        np.testing.assert_array_equal(b, permit_bits(want))
        assert (want[::37] != 0).any()


@pytest.mark.parametrize("flat", [0, 1, 2])
@pytest.mark.parametrize("dir_kb", [1, 16, 1024])
def test_hybrid_directory_budgets(torch_cuda, monkeypatch, dir_kb, flat):
    """Narrow directories (long candidate lists) and wide ones stay exact,
    walked per lane or flattened per wave: C3-style rules on slots and on
    IMIX frames."""
    torch = torch_cuda
    monkeypatch.setenv("NFFACL_TUNE_DIR_KB", str(dir_kb))
    monkeypatch.setenv("NFFACL_TUNE_FLAT", str(flat))
    g = synth.gen_rules(synth.SPECS["c3"], synth.RULE_SEEDS["c3"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = (1 << 15) + 5
    slots = synth.gen_slots(g, n, 21)
    with nffacl.Engine(rules, algo=nffacl.ALGO_HYBRID) as eng:
        assert eng.algo == nffacl.ALGO_HYBRID
        p, b = classify(torch, eng, slots, 64, n)
        want = oracle.classify_slots(slots, 64, n, a4, a6, threads=THREADS)
        np.testing.assert_array_equal(p, want)
        np.testing.assert_array_equal(b, permit_bits(want))
        frames, desc = synth.gen_imix(g, 1 << 14, 22)
        port = torch.zeros(1 << 14, dtype=torch.int32, device="cuda")
        eng.classify_frames_device(to_dev(torch, frames), to_dev(torch, desc.view(np.int64)), 1 << 14, port)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(port.cpu().numpy().view(np.uint32),
                                      oracle.classify_frames(frames, desc, a4, a6, threads=THREADS))


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("n", [1, 63, 65, 4097, (1 << 20) + 3])
def test_frames_ragged_and_short(torch_cuda, algo, n):
    """Packed frames (the cooperative 64-lane frame-line loads): ragged batch
    counts, and frames of 0..80 bytes whose bytes past the length hold
    garbage that must read as 0 — against the oracle on the same buffer."""
    torch = torch_cuda
    g = synth.gen_rules(synth.SPECS["c3"], synth.RULE_SEEDS["c3"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    rng = np.random.default_rng(n)
    m = min(n, 4096)
    short = synth.gen_slots(g, m, 41, stride=96).reshape(m, 96)
    lens = rng.integers(0, 81, m)
    frames = np.full(m * 96 + 64, 0xEE, np.uint8)
    for i in range(m):
        frames[i * 96:i * 96 + lens[i]] = short[i, :lens[i]]
    desc = (np.arange(m, dtype=np.uint64) * np.uint64(96) << np.uint64(16)) | lens.astype(np.uint64)
    if n > m:  # the bulk: IMIX frames after the short ones
        big, bdesc = synth.gen_imix(g, n - m, 42)
        bdesc = bdesc + (np.uint64(len(frames)) << np.uint64(16))
        frames = np.concatenate([frames, big])
        desc = np.concatenate([desc, bdesc])
    with nffacl.Engine(rules, algo=algo) as eng:
        port = torch.zeros(n, dtype=torch.int32, device="cuda")
        permit = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")
        eng.classify_frames_device(to_dev(torch, frames), to_dev(torch, desc.view(np.int64)), n, port, permit)
        torch.cuda.synchronize()
    want = oracle.classify_frames(frames, desc, a4, a6, threads=THREADS)
    np.testing.assert_array_equal(port.cpu().numpy().view(np.uint32), want)
    np.testing.assert_array_equal(permit.cpu().numpy().view(np.uint64), permit_bits(want))


@pytest.mark.parametrize("cfg", ["c2", "c3", "c5"])
def test_pulled_batches_gpu(torch_cuda, monkeypatch, cfg):
    """Batches pulled from the per-stream heads (NFFACL_TUNE_DYN=2) ==
    the fixed grid stride (DYN=0) == the oracle: ragged sizes back to back on
    one stream (each launch must leave its heads zeroed for the next), on 64-B
    slots and IMIX frames, and launches alternating over two streams."""
    torch = torch_cuda
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    sizes = [1, 63, 64 * 7 + 5, (1 << 16) + 3, (1 << 20) + 17, 200]
    nmax = max(sizes)
    slots = synth.gen_slots(g, nmax, 41)
    frames, desc = synth.gen_imix(g, nmax, 42)
    d_slots, d_frames = to_dev(torch, slots), to_dev(torch, frames)
    d_desc = to_dev(torch, desc.view(np.int64))
    outs = {}
    for dyn in ("0", "2"):  # (2: every indexed batch kernel pulls, the default 1 only the flat-LDS walks)
        monkeypatch.setenv("NFFACL_TUNE_DYN", dyn)
        with nffacl.Engine(rules) as eng:
            s2 = torch.cuda.Stream()
            res = []
            for k, n in enumerate(sizes):
                st = torch.cuda.current_stream() if k % 3 != 2 else s2
                port = torch.empty(n, dtype=torch.int32, device="cuda")  # (every word is written)
                fport = torch.empty(n, dtype=torch.int32, device="cuda")
                bits = torch.empty((n + 63) // 64, dtype=torch.int64, device="cuda")
                with torch.cuda.stream(st):
                    eng.classify_device(d_slots, 64, n, port, bits, st)
                    eng.classify_frames_device(d_frames, d_desc, n, fport, None, st)
                res.append((port, bits, fport))
            torch.cuda.synchronize()
            outs[dyn] = [[t.cpu().numpy() for t in r] for r in res]
    for k, n in enumerate(sizes):
        for a, b in zip(outs["0"][k], outs["2"][k]):
            np.testing.assert_array_equal(a, b)
    m = (1 << 16) + 3
    k = sizes.index(m)
    want = oracle.classify_slots(slots[:m * 64], 64, m, a4, a6, threads=THREADS)
    np.testing.assert_array_equal(outs["2"][k][0].view(np.uint32), want)
    np.testing.assert_array_equal(outs["2"][k][1].view(np.uint64), permit_bits(want))
    want_f = oracle.classify_frames(frames, desc[:m], a4, a6, threads=THREADS)
    np.testing.assert_array_equal(outs["2"][k][2].view(np.uint32), want_f)


def test_pulled_batches_many_streams_gpu(torch_cuda, monkeypatch):
    """More streams than an engine has blocks of pull heads (64): launches on
    the streams past them take the grid stride; every verdict equals the
    oracle, and a stream that launched before keeps its heads."""
    torch = torch_cuda
    monkeypatch.setenv("NFFACL_TUNE_DYN", "2")
    g = synth.gen_rules(synth.SPECS["c5"], synth.RULE_SEEDS["c5"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = 64 * 37 + 11
    slots = synth.gen_slots(g, n, 43)
    want = oracle.classify_slots(slots, 64, n, a4, a6, threads=THREADS)
    d_slots = to_dev(torch, slots)
    with nffacl.Engine(rules) as eng:
        streams = [torch.cuda.Stream() for _ in range(70)]
        outs = []
        for rep in range(2):
            for st in streams:
                port = torch.empty(n, dtype=torch.int32, device="cuda")
                with torch.cuda.stream(st):
                    eng.classify_device(d_slots, 64, n, port, None, st)
                outs.append(port)
        torch.cuda.synchronize()
        for port in outs:
            np.testing.assert_array_equal(port.cpu().numpy().view(np.uint32), want)


@pytest.mark.parametrize("cfg", ["c2", "c5"])
def test_graph_capture_replay_gpu(torch_cuda, cfg):
    """A classify launch captured into a HIP graph (torch.cuda.CUDAGraph) and
    replayed back to back: every replay equals the oracle (C5's pulled-batch
    heads are left zeroed by each replay for the next)."""
    torch = torch_cuda
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = (1 << 16) + 3
    slots = synth.gen_slots(g, n, 47)
    want = oracle.classify_slots(slots, 64, n, a4, a6, threads=THREADS)
    d_slots = to_dev(torch, slots)
    port = torch.zeros(n, dtype=torch.int32, device="cuda")
    bits = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")
    with nffacl.Engine(rules) as eng:
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):  # warm-up launch outside the capture
            eng.classify_device(d_slots, 64, n, port, bits, s)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            eng.classify_device(d_slots, 64, n, port, bits, torch.cuda.current_stream())
        for _ in range(3):
            port.zero_()
            bits.zero_()
            graph.replay()
            torch.cuda.synchronize()
            np.testing.assert_array_equal(port.cpu().numpy().view(np.uint32), want)
            np.testing.assert_array_equal(bits.cpu().numpy().view(np.uint64), permit_bits(want))
        del graph


def test_per_thread_stream_launches_gpu(torch_cuda):
    """hipStreamPerThread is ONE handle value for a
    different stream on every thread, so launches on it from two threads may
    run at once; they must not share one block of pull heads (the engine
    takes the grid stride for that handle).  Two threads x 6 launches of C5
    (a pulled-batch walk by default) on hipStreamPerThread, every launch
    equal to the oracle."""
    import threading
    torch = torch_cuda
    g = synth.gen_rules(synth.SPECS["c5"], synth.RULE_SEEDS["c5"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = (1 << 18) + 11
    slots = synth.gen_slots(g, n, 43)
    want = oracle.classify_slots(slots, 64, n, a4, a6, threads=THREADS)
    d_slots = to_dev(torch, slots)
    per_thread = 2  # hipStreamPerThread ((hipStream_t)2, hip_runtime_api.h)
    errors, outs = [], {}
    with nffacl.Engine(rules) as eng:
        assert eng.kernel_info().pulled == 1  # the walk pulls its batches on ordinary streams

        def worker(t):
            try:
                ports = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(6)]
                for p in ports:
                    eng.classify_device(d_slots, 64, n, p, None, per_thread)
                torch.cuda.synchronize()
                outs[t] = [p.cpu().numpy().view(np.uint32) for p in ports]
            except Exception as e:  # surfaced below
                errors.append(e)
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
    assert not errors, errors
    for t in range(2):
        for p in outs[t]:
            np.testing.assert_array_equal(p, want)


@pytest.mark.parametrize("fine_slots,ns", [(None, 6), ("7", 7), ("11", 8), ("15", 8)])
def test_c5_more_fine_grids_gpu(torch_cuda, monkeypatch, fine_slots, ns):
    """Fine grids on two (default) / three / all four positional grid slots
    (NFFACL_TUNE_FINE_SLOTS): the PIPELINED walk at NS = 6 / 7 / 8 slots
    (asserted through nffacl_engine_kernel_info), slots over 8 launches and
    IMIX frames equal the oracle.  VERDICT round 5 item 1: the NS = 7
    pipelined kernel lost 1-7 IPv6 matches of 2^16 per launch (76 in 20
    launches, gpurun_out/r6_hunt) — a 64-bit shift reading its amount from
    the allocation's last VGPR; the shift is gone and every
    build is checked for the pattern (tests/test_isa_guard.py)."""
    torch = torch_cuda
    if fine_slots:
        monkeypatch.setenv("NFFACL_TUNE_FINE_SLOTS", fine_slots)
    g = synth.gen_rules(synth.SPECS["c5"], synth.RULE_SEEDS["c5"])
    rules, (a4, a6) = _rules_and_arrays(g.text)
    n = (1 << 16) + 5
    slots = synth.gen_slots(g, n, 61)
    with nffacl.Engine(rules, algo=nffacl.ALGO_HYBRID) as eng:
        k = eng.kernel_info()
        assert k.walk == nffacl.WALK_FLAT_LDS_PIPELINED and k.slots == ns, (k.walk, k.slots)
        want = oracle.classify_slots(slots, 64, n, a4, a6, threads=THREADS)
        for _ in range(8):  # the round-5 failure varied from launch to launch
            p, b = classify(torch, eng, slots, 64, n)
            np.testing.assert_array_equal(p, want)
            np.testing.assert_array_equal(b, permit_bits(want))
        frames, desc = synth.gen_imix(g, 1 << 14, 62)
        port = torch.zeros(1 << 14, dtype=torch.int32, device="cuda")
        eng.classify_frames_device(to_dev(torch, frames), to_dev(torch, desc.view(np.int64)), 1 << 14, port)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(port.cpu().numpy().view(np.uint32),
                                      oracle.classify_frames(frames, desc, a4, a6, threads=THREADS))
