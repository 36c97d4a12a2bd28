"""Pin the CPU oracle against the reference's own known answers (CPU only).

Mirrors packet/acl_internal_test.go (match + parse KATs) and
packet/packet_test.go (header-parse KAT); the expected values come from the
reference's test tables, transcribed by tests/golden/make_kats.py.
"""
import json

import numpy as np
import pytest

from oracle import oracle, rules_oracle as ro


def _kats(golden):
    z = np.load(golden / "acl_match_kats.npz", allow_pickle=False)
    pk = json.loads((golden / "kat_packets.json").read_text())
    packets = [bytes.fromhex(pk[name]) for name in z["packet_names"]]
    return z, packets


def test_match_kat_counts(golden):
    z, _ = _kats(golden)
    groups = list(z["groups"])
    n = {g: 0 for g in groups}
    for arr in (z["c4_group"], z["c6_group"]):
        for gi in arr:
            n[groups[gi]] += 1
    # acl_internal_test.go:501-1141
    assert n == {"l4ACL_ipv4_tcp": 15, "l3ACL_ipv4_tcp": 64, "l3l4_ipv4_tcp": 2160,
                 "l3l4_ipv6_tcp": 1215, "l3l4_ipv6_udp": 1215, "l3l4_ipv4_icmp": 1728,
                 "l3l4_ipv6_icmp": 972}


def test_oracle_match_kats(golden):
    """TestInternal_l4ACL / l3ACL / l3ACL_l4ACL_* (every case)."""
    z, packets = _kats(golden)
    bad = []
    for fam in (4, 6):
        rules = z[f"c{fam}_rule"]
        for i in range(len(rules)):
            pkt = packets[z[f"c{fam}_packet"][i]]
            r = rules[i:i + 1]
            got = oracle.l3acl(pkt, r, None) if fam == 4 else oracle.l3acl(pkt, None, r)
            if got != z[f"c{fam}_want"][i]:
                bad.append((fam, i, got, int(z[f"c{fam}_want"][i])))
    assert not bad, bad[:10]


def test_oracle_cross_family_is_zero(golden):
    """An IPv4 packet never consults ip6 rules and vice versa (acl.go:524-563)."""
    z, packets = _kats(golden)
    match_all4 = np.zeros(1, ro.RULE4_DTYPE)
    match_all4["output_number"] = 9
    match_all6 = np.zeros(1, ro.RULE6_DTYPE)
    match_all6["output_number"] = 9
    match_all6["src_port_max"] = 65535
    match_all6["dst_port_max"] = 65535
    for name, pkt in zip(z["packet_names"], packets):
        v4 = oracle.l3acl(pkt, match_all4, None)
        v6 = oracle.l3acl(pkt, None, match_all6)
        assert (v4, v6) == ((9, 0) if name.startswith("ipv4") else (0, 9)), name


def test_oracle_non_ip_is_zero():
    arp = bytes(12) + b"\x08\x06" + bytes(50)
    vlan = bytes(12) + b"\x81\x00" + bytes(50)
    r4 = np.zeros(1, ro.RULE4_DTYPE)
    r4["output_number"] = 3
    assert oracle.l3acl(arp, r4) == 0
    assert oracle.l3acl(vlan, r4) == 0
    assert oracle.l3acl(b"", r4) == 0


def test_oracle_v6_always_checks_ports():
    """acl.go:555-558: IPv6 runs l4ACL whatever L4.valid says."""
    pkt = bytes.fromhex(json.loads(_golden_text("kat_packets.json"))["ipv6_tcp"])
    r6 = np.zeros(1, ro.RULE6_DTYPE)
    r6["output_number"] = 5  # valid=0, ranges 0..0 -> ports 1234/5678 fail
    assert oracle.l3acl(pkt, None, r6) == 0
    r6["src_port_max"] = 65535
    r6["dst_port_max"] = 65535
    assert oracle.l3acl(pkt, None, r6) == 5


def _golden_text(name):
    from pathlib import Path
    return (Path(__file__).resolve().parent / "golden" / name).read_text()


@pytest.mark.parametrize("case", json.loads(_golden_text("parse_l3_kat.json")), ids=lambda c: c["hex"][:20])
def test_oracle_header_parse_kat(case):
    """packet_test.go TestParseL3/TestParseL4: the oracle's field offsets give
    exactly the header values the reference expects (probed through verdicts)."""
    pkt = bytes.fromhex(case["hex"])
    sp = ((case["src_port_le"] & 0xFF) << 8) | (case["src_port_le"] >> 8)  # SwapBytesUint16
    dp = ((case["dst_port_le"] & 0xFF) << 8) | (case["dst_port_le"] >> 8)

    def rule(**over):
        r = np.zeros(1, ro.RULE4_DTYPE)
        vals = dict(output_number=7, src_addr=case["src_addr"], dst_addr=case["dst_addr"],
                    src_mask=0xFFFFFFFF, dst_mask=0xFFFFFFFF, id=case["proto"], id_mask=0xFF, valid=1,
                    src_port_min=sp, src_port_max=sp, dst_port_min=dp, dst_port_max=dp)
        vals.update(over)
        for k, v in vals.items():
            r[k] = v
        return r

    assert oracle.l3acl(pkt, rule()) == 7
    assert oracle.l3acl(pkt, rule(src_addr=case["src_addr"] ^ 0x01000000)) == 0
    assert oracle.l3acl(pkt, rule(dst_addr=case["dst_addr"] ^ 0x00000100)) == 0
    assert oracle.l3acl(pkt, rule(id=case["proto"] ^ 0x10)) == 0
    assert oracle.l3acl(pkt, rule(src_port_min=(sp + 1) & 0xFFFF, src_port_max=(sp + 1) & 0xFFFF)) == 0
    assert oracle.l3acl(pkt, rule(dst_port_min=(dp + 1) & 0xFFFF, dst_port_max=(dp + 1) & 0xFFFF)) == 0


# ---- parser oracle ----------------------------------------------------------------

def _want_record(case):
    w = case["want"]
    if case["family"] == 4:
        return (w["output_number"], w["src_addr"], w["dst_addr"], w["src_mask"], w["dst_mask"],
                w["id"], w["id_mask"], int(w["valid"]), w["src_port_min"], w["src_port_max"],
                w["dst_port_min"], w["dst_port_max"])
    return (w["output_number"], bytes.fromhex(w["src_addr"]), bytes.fromhex(w["dst_addr"]),
            bytes.fromhex(w["src_mask"]), bytes.fromhex(w["dst_mask"]), w["id"], w["id_mask"],
            int(w["valid"]), w["src_port_min"], w["src_port_max"], w["dst_port_min"], w["dst_port_max"])


def _got_record(r):
    l4 = r.l4
    return (r.output_number, r.src_addr, r.dst_addr, r.src_mask, r.dst_mask, l4.id, l4.id_mask,
            int(l4.valid), l4.src_port_min, l4.src_port_max, l4.dst_port_min, l4.dst_port_max)


HEADER = b"# Source address, Destination address, L4 protocol ID, Source port, Destination port, Output port\n"


def test_oracle_parse_kats_text_and_json(golden):
    """TestGetL3ACLFromJSON (:377-431) and the text-table variant of the same
    table (:435-497, which the reference generates vacuously)."""
    cases = json.loads((golden / "parse_kats.json").read_text())
    assert len(cases) == 494
    for c in cases:
        line = " ".join(c["raw"]).encode()
        got_t = ro.parse_text_table(HEADER + line)
        doc = {"L3Rules": [dict(zip(("SrcAddr", "DstAddr", "ID", "SrcPort", "DstPort", "OutputNumber"), c["raw"]))]}
        got_j = ro.parse_json(json.dumps(doc).encode())
        for got in (got_t, got_j):
            lst = got.ip4 if c["family"] == 4 else got.ip6
            assert _got_record(lst[0]) == _want_record(c), c


def test_oracle_firewall_conf(golden):
    """examples/firewall/firewall.conf: 4 text rules -> 4 ip4 + 1 ip6."""
    r = ro.load_text_table(golden / "rules" / "firewall.conf")
    assert len(r.ip4) == 4 and len(r.ip6) == 1
    assert r.ip4[0].src_addr == int.from_bytes(bytes([10, 10, 0, 0]), "little")
    assert r.ip4[0].src_mask == 0x00FFFFFF
    assert (r.ip4[1].l4.src_port_min, r.ip4[1].l4.src_port_max) == (49, 122)
    assert r.ip4[2].dst_addr == int.from_bytes(bytes([21, 23, 45, 10]), "little")
    assert r.ip6[0].l4.dst_port_min == 4080 and r.ip6[0].l4.valid


def test_oracle_text_json_stash_parity(golden):
    """test/stash: the same rules as text and JSON parse identically."""
    t = ro.load_text_table(golden / "rules" / "forwardingTestL3_ACL.conf")
    j = ro.load_json(golden / "rules" / "forwardingTestL3_ACL.json")
    assert [_got_record(x) for x in t.ip4] == [_got_record(x) for x in j.ip4]
    assert [_got_record(x) for x in t.ip6] == [_got_record(x) for x in j.ip6]


@pytest.mark.parametrize("line,code", [
    (b"ANY ANY TCP", ro.PARSE_RULE_ERR),                    # too few fields
    (b"ANY ANY TCP ANY ANY Accept extra", ro.PARSE_RULE_ERR),
    (b"   ", ro.PARSE_RULE_ERR),                            # whitespace-only line is not skipped
    (b"  # indented comment", ro.PARSE_RULE_ERR),
    (b"ANY ANY SCTP ANY ANY Accept", ro.INCORRECT_ARG_IN_RULES),
    (b"ANY ANY ICMP 80 ANY Accept", ro.INCORRECT_ARG_IN_RULES),
    (b"ANY ANY ICMP 0:65535 ANY Accept", ro.INCORRECT_ARG_IN_RULES),  # literal "ANY" required
    (b"ANY ANY TCP 10:5 ANY Accept", ro.INCORRECT_ARG_IN_RULES),
    (b"ANY ANY TCP 65536 ANY Accept", ro.INCORRECT_ARG_IN_RULES),
    (b"ANY ANY TCP 1:2:3 ANY Accept", ro.INCORRECT_ARG_IN_RULES),
    (b"ANY ANY TCP -1 ANY Accept", ro.INCORRECT_ARG_IN_RULES),
    (b"1.2.3.4/8 ::/0 TCP ANY ANY Accept", ro.INCORRECT_ARG_IN_RULES),
    (b"::/0 1.2.3.4/8 TCP ANY ANY Accept", ro.INCORRECT_ARG_IN_RULES),
    (b"1.2.3.4 ANY TCP ANY ANY Accept", ro.INCORRECT_ARG_IN_RULES),  # no prefix: reference panics
    (b"ANY ANY TCP ANY ANY Maybe", ro.INCORRECT_RULE),
    (b"ANY ANY TCP ANY ANY 4294967296", ro.INCORRECT_RULE),
])
def test_oracle_parse_errors(line, code):
    with pytest.raises(ro.OracleParseError) as e:
        ro.parse_text_table(line + b"\n")
    assert e.value.code == code


def test_oracle_parse_go_quirks():
    # go1.13 accepts leading zeros in dotted quads (decimal, not octal)
    r = ro.parse_text_table(b"010.001.0.0/16 ANY ANY ANY ANY 4\n")
    assert r.ip4[0].src_addr == int.from_bytes(bytes([10, 1, 0, 0]), "little")
    # "0:65535" is ANY (valid=false); a 5-field line is Reject; CR is dropped
    r = ro.parse_text_table(b"ANY 1.2.3.0/24 UDP 0:65535 ANY\r\n")
    assert r.ip4[0].l4.valid is False and r.ip4[0].output_number == 0
    # tab / NBSP / ideographic space separate fields (strings.Fields)
    r = ro.parse_text_table("ANY\tANY TCP　ANY ANY 7\n".encode())
    assert r.ip4[0].output_number == 7 and r.ip6[0].output_number == 7
    # IPv4-mapped IPv6 stays an IPv6 rule; network address is masked
    r = ro.parse_text_table(b"::ffff:1.2.3.4/120 ANY ANY ANY ANY 1\n")
    assert len(r.ip6) == 1 and r.ip6[0].src_addr[-1] == 0 and r.ip6[0].src_addr[-2] == 3
