"""libnffacl's C++ rule parser (the product) against the reference's parse KATs
and the independent oracle parser (CPU only; no device work)."""
import json

import numpy as np
import pytest

import nffacl
from nffacl import synth
from oracle import rules_oracle as ro

HEADER = b"# Source address, Destination address, L4 protocol ID, Source port, Destination port, Output port\n"
FIELDS = ("SrcAddr", "DstAddr", "ID", "SrcPort", "DstPort", "OutputNumber")


def _same(product: nffacl.L3Rules, orc: ro.L3Rules):
    a4, a6 = orc.arrays()
    p4, p6 = product.ip4(), product.ip6()
    assert p4.tobytes() == a4.tobytes()
    assert p6.tobytes() == a6.tobytes()


def test_parse_kats_text(golden):
    """TestGetL3ACLFromTextTable restated over the (non-vacuous) KAT table."""
    cases = json.loads((golden / "parse_kats.json").read_text())
    for c in cases:
        text = HEADER + " ".join(c["raw"]).encode()
        p = nffacl.L3Rules.parse_text(text)
        o = ro.parse_text_table(text)
        _same(p, o)
        w = c["want"]
        rec = p.ip4()[0] if c["family"] == 4 else p.ip6()[0]
        assert rec["output_number"] == w["output_number"]
        assert rec["id"] == w["id"] and rec["id_mask"] == w["id_mask"] and bool(rec["valid"]) == w["valid"]
        assert (rec["src_port_min"], rec["src_port_max"]) == (w["src_port_min"], w["src_port_max"])
        if c["family"] == 4:
            assert (rec["src_addr"], rec["src_mask"], rec["dst_addr"], rec["dst_mask"]) == \
                (w["src_addr"], w["src_mask"], w["dst_addr"], w["dst_mask"])
        else:
            assert bytes(rec["src_addr"]) == bytes.fromhex(w["src_addr"])
            assert bytes(rec["dst_mask"]) == bytes.fromhex(w["dst_mask"])


def test_parse_kats_json(golden):
    """TestGetL3ACLFromJSON (acl_internal_test.go:377-431)."""
    cases = json.loads((golden / "parse_kats.json").read_text())
    for c in cases:
        doc = json.dumps({"L3Rules": [dict(zip(FIELDS, c["raw"]))]}).encode()
        _same(nffacl.L3Rules.parse_json(doc), ro.parse_json(doc))


@pytest.mark.parametrize("name", ["firewall.conf", "forwarding.conf", "tutorial_rules1.conf",
                                  "tutorial_rules2.conf", "forwardingTestL3_ACL.conf",
                                  "test-separate-l3rules.conf", "test-split.conf",
                                  "test-handle-l3rules.conf"])
def test_reference_rule_files_text(golden, name):
    path = golden / "rules" / name
    rules, err = nffacl.GetL3ACLFromTextTable(path)
    assert err is None, err
    _same(rules, ro.load_text_table(path))


@pytest.mark.parametrize("name", ["forwardingTestL3_ACL.json", "demoL3_ACL.json"])
def test_reference_rule_files_json(golden, name):
    path = golden / "rules" / name
    rules, err = nffacl.GetL3ACLFromJSON(path)
    assert err is None, err
    _same(rules, ro.load_json(path))


def test_firewall_counts(golden):
    rules, _ = nffacl.GetL3ACLFromTextTable(golden / "rules" / "firewall.conf")
    assert rules.counts() == (4, 1)


@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_synthetic_rule_files(cfg):
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    _same(nffacl.L3Rules.parse_text(g.text), ro.parse_text_table(g.text.encode()))


def test_missing_file():
    rules, err = nffacl.GetL3ACLFromTextTable("/nonexistent/rules.conf")
    assert rules is None and err.code == 12  # FileErr


ERROR_LINES = [
    b"ANY ANY TCP", b"ANY ANY TCP ANY ANY Accept extra", b"   ", b"  # indented comment",
    b"ANY ANY SCTP ANY ANY Accept", b"ANY ANY ICMP 80 ANY Accept", b"ANY ANY ICMP 0:65535 ANY Accept",
    b"ANY ANY TCP 10:5 ANY Accept", b"ANY ANY TCP 65536 ANY Accept", b"ANY ANY TCP 1:2:3 ANY Accept",
    b"ANY ANY TCP -1 ANY Accept", b"ANY ANY TCP +1 ANY Accept", b"ANY ANY TCP :5 ANY Accept",
    b"1.2.3.4/8 ::/0 TCP ANY ANY Accept", b"::/0 1.2.3.4/8 TCP ANY ANY Accept",
    b"1.2.3.4 ANY TCP ANY ANY Accept", b"1.2.3.4/33 ANY TCP ANY ANY Accept",
    b"1.2.3/8 ANY TCP ANY ANY Accept", b"256.1.1.1/8 ANY TCP ANY ANY Accept",
    b"::1::2/64 ANY ANY ANY ANY 1", b"1:2:3:4:5:6:7:8:9/64 ANY ANY ANY ANY 1", b"any ANY TCP ANY ANY 1",
    b"ANY ANY TCP ANY ANY Maybe", b"ANY ANY TCP ANY ANY 4294967296", b"ANY ANY TCP ANY ANY -3",
    b"ANY ANY tcP ANY ANY 1", b"fe80::1%eth0/64 ANY ANY ANY ANY 1",
]


@pytest.mark.parametrize("line", ERROR_LINES)
def test_error_codes_match_oracle(line):
    with pytest.raises(ro.OracleParseError) as oe:
        ro.parse_text_table(line + b"\n")
    with pytest.raises(nffacl.NFError) as pe:
        nffacl.L3Rules.parse_text(line + b"\n")
    assert pe.value.code == oe.value.code, (line, pe.value, oe.value)


QUIRK_LINES = [
    b"010.001.0.0/16 ANY ANY ANY ANY 4", b"ANY 1.2.3.0/24 UDP 0:65535 ANY\r",
    "ANY\tANY TCP　ANY ANY 7".encode(), "ANY ANY TCP ANY ANY 7".encode(),
    b"::ffff:1.2.3.4/120 ANY ANY ANY ANY 1", b"::/0 ANY ANY ANY ANY 1", b"::1.2.3.4/128 ANY ANY ANY ANY 1",
    b"1:2:3:4:5:6:1.2.3.4/96 ANY ANY ANY ANY 1", b"ABCD:00001::/32 ANY ANY ANY ANY 1",
    b"1.2.3.4/032 ANY TCP 0080 00443:00444 0017", b"ANY ANY 0x06 5 5 true", b"ANY ANY 17 5 5 false",
    b"0.0.0.0/0 0.0.0.0/0 ICMP ANY ANY 2", b"255.255.255.255/32 ANY Icmp ANY ANY 4294967295",
    b"ANY ::/0 Udp 1:65535 0:0 3", b"#comment only", b"", b"\r",
]


@pytest.mark.parametrize("line", QUIRK_LINES)
def test_quirks_match_oracle(line):
    text = line + b"\n"
    _same(nffacl.L3Rules.parse_text(text), ro.parse_text_table(text))


def test_fuzz_lines_match_oracle():
    """Random token soups: identical accept/reject decisions and records."""
    rng = np.random.default_rng(7)
    toks = [b"ANY", b"TCP", b"udp", b"ICMP", b"6", b"0x11", b"1", b"Accept", b"Reject", b"true", b"0",
            b"65535", b"80", b"1:1024", b"5:4", b"0:65535", b"10.0.0.0/8", b"10.1.2.3/32", b"1.2.3.4/0",
            b"::/0", b"dead::beef/64", b"2001:db8::/32", b"fe80::/10", b"1.2.3.4", b"x", b"4294967295",
            b"\t", b" ", " ".encode(), b"#"]
    for _ in range(3000):
        k = int(rng.integers(0, 8))
        line = b" ".join(toks[int(i)] for i in rng.integers(0, len(toks), k))
        text = line + b"\n"
        try:
            o = ro.parse_text_table(text)
        except ro.OracleParseError as e:
            with pytest.raises(nffacl.NFError) as pe:
                nffacl.L3Rules.parse_text(text)
            assert pe.value.code == e.code, line
            continue
        _same(nffacl.L3Rules.parse_text(text), o)


JSON_CASES = [
    b'{"L3Rules":[{"SrcAddr":"ANY","DstAddr":"ANY","ID":"TCP","SrcPort":"ANY","DstPort":"80","OutputNumber":"2"}]}',
    b'{"l3rules":[{"srcaddr":"10.0.0.0/8","dstaddr":"ANY","id":"ANY","srcport":"ANY","dstport":"ANY","outputnumber":"Accept"}]}',
    b'{"L3Rules":null}', b'null', b'{}', b'{"Other": 5, "L3Rules": []}',
    b'{"L3Rules":[{"SrcAddr":"ANY","DstAddr":"ANY","ID":"ANY","SrcPort":"ANY","DstPort":"ANY","OutputNumber":null}]}',
    b'{"L3Rules":[{"SrcAddr":"ANY","DstAddr":"ANY","ID":"ANY","SrcPort":"ANY","DstPort":"ANY","OutputNumber":"1"}],'
    b' "L3Rules":[{"SrcAddr":"ANY","DstAddr":"ANY","ID":"UDP","SrcPort":"ANY","DstPort":"ANY","OutputNumber":"3"}]}',
    b'{"L3Rules":[{"SrcAddr":"ANY","DstAddr":"ANY","ID":"ANY","SrcPort":"ANY","DstPort":"ANY","OutputNumber":1}]}',
    b'{"L3Rules":{}}', b'[1,2]', b'{"L3Rules":[', b'{"L3Rules":[]} x',
    b'{"L3Rules":[{"SrcAddr":"ANY","DstAddr":"ANY","ID":"ANY","SrcPort":"ANY","DstPort":"ANY"}]}',
    b'{"L3Rules":[{"SrcAddr":"\\u0041NY","DstAddr":"ANY","ID":"ANY","SrcPort":"ANY","DstPort":"ANY","OutputNumber":"1"}]}',
    b'  {"L3Rules" : [ ] }  ',
]


@pytest.mark.parametrize("doc", JSON_CASES)
def test_json_matches_oracle(doc):
    try:
        o = ro.parse_json(doc)
    except ro.OracleParseError as e:
        with pytest.raises(nffacl.NFError) as pe:
            nffacl.L3Rules.parse_json(doc)
        assert pe.value.code == e.code, doc
        return
    _same(nffacl.L3Rules.parse_json(doc), o)


def test_from_arrays_roundtrip():
    a4 = np.zeros(3, nffacl.RULE4)
    a4["output_number"] = [1, 2, 3]
    a4["src_mask"] = [0, 0xFFFFFFFF, 0x00FF00FF]
    a6 = np.zeros(2, nffacl.RULE6)
    a6["src_addr"][1, 0] = 0xDE
    r = nffacl.L3Rules.from_arrays(a4, a6)
    assert r.counts() == (3, 2)
    assert r.ip4().tobytes() == a4.tobytes() and r.ip6().tobytes() == a6.tobytes()
