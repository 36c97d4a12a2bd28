"""NFFACL_PARSE_VLAN: L3 ACL over ParseAllKnownL3CheckVLAN (packet/vlan.go:104-117)
instead of ParseAllKnownL3 ("VLAN-aware L3 parse").

The oracle's VLAN parse is pinned by the tagged frame of vlan_test.go:23 and
the headers TestParseAllKnownL3CheckVLAN (:239-269) expects in it, probed
through verdicts; the GPU is then checked against the oracle.
"""
import json

import numpy as np
import pytest

import nffacl
from nffacl import synth
from oracle import oracle, rules_oracle as ro

V = oracle.PARSE_VLAN


@pytest.fixture(scope="module")
def kat(golden):
    k = json.loads((golden / "vlan_kat.json").read_text())
    k["frame"] = bytes.fromhex(k["hex"])
    return k


def _rule(src, dst, proto, sport, dport, out="Accept"):
    return f"{src} {dst} {proto} {sport} {dport} {out}\n".encode()


def _oracle_port(frame: bytes, rule_text: bytes, flags: int) -> int:
    a4, a6 = ro.parse_text_table(rule_text).arrays()
    buf = np.zeros(128, np.uint8)
    buf[:len(frame)] = np.frombuffer(frame, np.uint8)
    return int(oracle.classify_slots(buf, 128, 1, a4, a6, flags=flags)[0])


def test_vlan_frame_fields_pinned(kat):
    """The 5-tuple ParseAllKnownL3CheckVLAN finds in gtLineIPv4TCPVLAN."""
    f = kat["frame"]
    s = ".".join(map(str, kat["src"])) + "/32"
    d = ".".join(map(str, kat["dst"])) + "/32"
    exact = _rule(s, d, "TCP", kat["sport"], kat["dport"])
    assert _oracle_port(f, exact, V) == 1
    assert _oracle_port(f, exact, 0) == 0  # the reference's ParseAllKnownL3: tag -> no verdict
    for bad in (_rule(s, d, "UDP", kat["sport"], kat["dport"]),
                _rule(s, d, "TCP", kat["sport"] + 1, kat["dport"]),
                _rule(s, d, "TCP", kat["sport"], kat["dport"] - 1),
                _rule("131.151.32.22/32", d, "TCP", "ANY", "ANY"),
                _rule(s, "131.151.32.128/32", "TCP", "ANY", "ANY")):
        assert _oracle_port(f, bad, V) == 0, bad
    # untagged frame (tag removed) parses identically with or without the flag
    untagged = f[:12] + f[16:]
    assert _oracle_port(untagged, exact, V) == 1 and _oracle_port(untagged, exact, 0) == 1


def tag_slots(slots: np.ndarray, n: int, stride: int, frac: float, seed: int) -> np.ndarray:
    """Insert an 802.1Q tag (TPID 0x8100, random TCI) after the MACs of a random
    subset of packets — the wire form AddVLANTag (vlan.go:119-135) produces."""
    rng = np.random.default_rng(seed)
    s = slots.reshape(n, stride).copy()
    pick = rng.random(n) < frac
    body = s[pick, 12:stride - 4].copy()
    s[pick, 12] = 0x81
    s[pick, 13] = 0x00
    tci = rng.integers(0, 1 << 16, int(pick.sum()))
    s[pick, 14] = tci >> 8
    s[pick, 15] = tci & 0xFF
    s[pick, 16:stride] = body
    return s.reshape(-1)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("algo", [nffacl.ALGO_LINEAR, nffacl.ALGO_INDEXED])
@pytest.mark.parametrize("stride", [64, 128])
def test_gpu_vlan_flag(torch_cuda, algo, stride):
    torch = torch_cuda
    g = synth.gen_rules(synth.SPECS["c3"], synth.RULE_SEEDS["c3"])  # L3+L4 rules: ports matter
    a4, a6 = ro.parse_text_table(g.text.encode()).arrays()
    n = (1 << 16) + 11
    slots = tag_slots(synth.gen_slots(g, n, 0x71A9, stride=stride), n, stride, 0.5, 3)
    d = torch.from_numpy(slots).to("cuda")
    with nffacl.Engine(nffacl.L3Rules.parse_text(g.text), algo=algo) as eng:
        for flags in (0, nffacl.PARSE_VLAN):
            port = torch.zeros(n, dtype=torch.int32, device="cuda")
            eng.classify_device(d, stride, n, port, None, None, flags)
            torch.cuda.synchronize()
            want = oracle.classify_slots(slots, stride, n, a4, a6, threads=16, flags=flags)
            np.testing.assert_array_equal(port.cpu().numpy().view(np.uint32), want)
        assert (want != 0).sum() > n // 10
        with pytest.raises(nffacl.NFError):
            eng.classify_device(d, stride, n, port, None, None, 2)  # unknown flag


@pytest.mark.gpu
def test_gpu_vlan_frames_and_kat(torch_cuda, kat):
    torch = torch_cuda
    f = kat["frame"]
    s = ".".join(map(str, kat["src"])) + "/32"
    d = ".".join(map(str, kat["dst"])) + "/32"
    text = _rule(s, d, "TCP", kat["sport"], kat["dport"], "7")
    frames = np.zeros(256, np.uint8)
    frames[:len(f)] = np.frombuffer(f, np.uint8)
    frames[128:128 + len(f) - 4] = np.frombuffer(f[:12] + f[16:], np.uint8)
    desc = np.array([len(f), (128 << 16) | (len(f) - 4), (0 << 16) | 20], np.uint64)  # + a truncated copy
    with nffacl.Engine(nffacl.L3Rules.parse_text(text)) as eng:
        for flags, want in ((0, [0, 7, 0]), (nffacl.PARSE_VLAN, [7, 7, 0])):
            port = torch.zeros(3, dtype=torch.int32, device="cuda")
            eng.classify_frames_device(torch.from_numpy(frames).to("cuda"),
                                       torch.from_numpy(desc.view(np.int64)).to("cuda"), 3, port, None, None, flags)
            torch.cuda.synchronize()
            assert list(port.cpu().numpy()) == want
