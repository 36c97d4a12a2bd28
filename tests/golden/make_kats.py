#!/usr/bin/env python3
"""Generate the golden known-answer fixtures of tests/golden/ from the
reference's own test tables (transcribed as data, not executed).

Sources (aregm/nff-go, read as text):
  packet/utils_for_test.go:33-126   the six test packets (payload 100 B)
  packet/packet.go:509-705          InitEmpty*Packet field defaults they rely on
  types/const.go:22-83              EtherType / protocol / length constants
  packet/acl_internal_test.go:91-161    parse KAT table (rulesL3Ctxt)
  packet/acl_internal_test.go:266-370   generateTestL3Rules cartesian product
  packet/acl_internal_test.go:501-1141  match KATs (l4ACL + six l3ACL tables)
  packet/packet_test.go:22-267          header-parse KAT (8 hex frames)
  packet/acl_internal_test.go:66-89, 174-243   L2 parse KAT (rulesL2Ctxt, generateTestL2Rules)
  packet/acl_internal_test.go:1144-1273 L2 match KATs (IPv4 UDP and ARP request packets)
  packet/utils_for_test.go:95-104, packet/arp.go:60-93   ARP request test packet,
  packet/arp_test.go:22                 its layout pinned by gtLineARPRequest
  packet/vlan_test.go:23-67,239-269     VLAN-tagged IPv4/TCP frame + the headers
                                        ParseAllKnownL3CheckVLAN must find in it

Outputs:
  kat_packets.json    the test packets as hex
  acl_match_kats.npz  7369 (packet, single-rule table, expected port) cases
  parse_kats.json     (rule-file line, expected ip4/ip6 record) cases
  parse_l3_kat.json   8 frames + the header fields packet_test.go expects
  l2_kats.json        L2 parse cases (JSON + text) and the 216 L2 match cases
  vlan_kat.json       the tagged frame and its expected L3/L4 fields

Run:  python tests/golden/make_kats.py   (deterministic; no inputs)
"""
from __future__ import annotations

import json
import struct
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent

L4 = [("id", "u1"), ("id_mask", "u1"), ("valid", "u1"), ("reserved", "u1"),
      ("src_port_min", "<u2"), ("src_port_max", "<u2"), ("dst_port_min", "<u2"), ("dst_port_max", "<u2")]
RULE4 = np.dtype([("output_number", "<u4"), ("src_addr", "<u4"), ("dst_addr", "<u4"),
                  ("src_mask", "<u4"), ("dst_mask", "<u4")] + L4)
RULE6 = np.dtype([("output_number", "<u4"), ("src_addr", "u1", 16), ("dst_addr", "u1", 16),
                  ("src_mask", "u1", 16), ("dst_mask", "u1", 16)] + L4)

# ---- test packets (utils_for_test.go + packet.go InitEmpty*) ------------------
PAYLOAD = 100
DMAC = bytes([0x00, 0x11, 0x22, 0x33, 0x44, 0x55])
SMAC = bytes([0x01, 0x11, 0x21, 0x31, 0x41, 0x51])
V4_SRC, V4_DST = bytes([127, 0, 0, 1]), bytes([128, 9, 9, 5])
V6_ADDR = bytes.fromhex("dead000000000000000000000000beaf")  # net.ParseIP("dead::beaf")


def ipv4_packet(proto: int, l4len: int, l4: bytes) -> bytes:
    eth = DMAC + SMAC + b"\x08\x00"
    total = 20 + l4len + PAYLOAD
    # VersionIhl 0x45, TotalLength BE, TTL 64, NextProtoID; other fields 0 (fresh mbuf)
    ip = bytes([0x45, 0]) + struct.pack(">H", total) + b"\0\0\0\0" + bytes([64, proto]) + b"\0\0" + V4_SRC + V4_DST
    body = l4 + bytes(l4len - len(l4))
    return eth + ip + body + bytes(PAYLOAD)


def ipv6_packet(proto: int, l4len: int, l4: bytes) -> bytes:
    eth = DMAC + SMAC + b"\x86\xdd"
    # VtcFlow = 0x60 stored as a little-endian uint32 field, PayloadLen BE, Proto, HopLimits 255
    ip = struct.pack("<I", 0x60) + struct.pack(">H", l4len + PAYLOAD) + bytes([proto, 255]) + V6_ADDR + V6_ADDR
    body = l4 + bytes(l4len - len(l4))
    return eth + ip + body + bytes(PAYLOAD)


PORTS = struct.pack(">HH", 1234, 5678)  # initPorts
TCP = PORTS + bytes(8) + bytes([0x50])  # DataOff = TCPMinDataOffset
UDP = PORTS + struct.pack(">H", 8 + PAYLOAD)  # DgramLen

PACKETS = {
    "ipv4_tcp": ipv4_packet(6, 20, TCP),
    "ipv4_udp": ipv4_packet(17, 8, UDP),
    "ipv4_icmp": ipv4_packet(1, 8, b""),
    "ipv6_tcp": ipv6_packet(6, 20, TCP),
    "ipv6_udp": ipv6_packet(17, 8, UDP),
    "ipv6_icmp": ipv6_packet(58, 8, b""),
}
PKT_NAMES = list(PACKETS)

# ---- match KAT tables (acl_internal_test.go) ----------------------------------
# Addr4Mask {addr, msk, ok} — types.IPv4Address values as written in the test
SRC4 = [(0x0100007f, 0xffffffff, True), (0, 0, True), (0x0200007f, 0x00ffffff, True), (0x0200007f, 0xffffffff, False)]
DST4 = [(0x05090980, 0xffffffff, True), (0, 0, True), (0x0200007f, 0x00ffffff, False), (0x05050980, 0x0000ffff, True)]


def a6(*b):
    return bytes(b)


Z16 = bytes(16)
BB = a6(0xde, 0xad, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xbb, 0xbb)
BBM = a6(0xff, 0xff, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff)
DD = a6(0xde, 0xad, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xdd, 0xdd)
DDM = a6(0xff, 0xff, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)
ADDR6 = [(Z16, Z16, True), (BB, BBM, False), (DD, DDM, True)]  # same list for src and dst

# portRange {min, max, valid, ok}
SRC_TCPUDP = [(0, 65535, False, True), (13, 17, True, False), (1234, 1234, True, True),
              (1233, 1299, True, True), (0, 0, True, False)]
DST_TCPUDP = [(0, 65535, False, True), (9999, 9999, True, False), (5678, 5678, True, True)]
SRC_ICMP = [(0, 65535, False, True), (13, 17, True, False), (1234, 1234, True, False)]
DST_ICMP = [(0, 65535, False, True), (9999, 9999, True, False), (5678, 5678, True, False)]


def rec4(out, src, dst, idm=(0, 0), sp=(0, 0), dp=(0, 0), valid=False):
    return (out, src[0], dst[0], src[1], dst[1], idm[0], idm[1], int(valid), 0, sp[0], sp[1], dp[0], dp[1])


def rec6(out, src, dst, idm=(0, 0), sp=(0, 0), dp=(0, 0), valid=False):
    return (out, np.frombuffer(src[0], "u1"), np.frombuffer(dst[0], "u1"), np.frombuffer(src[1], "u1"),
            np.frombuffer(dst[1], "u1"), idm[0], idm[1], int(valid), 0, sp[0], sp[1], dp[0], dp[1])


def match_cases():
    c4, c6 = [], []  # (group, packet, record, want)
    # TestInternal_l4ACL_packetIPv4_TCP (:501-537): l4ACL alone, routed through l3ACL
    # with an otherwise-ANY IPv4 rule, valid=true, OutputNumber 1.
    src_r = [(0, 65535, True), (1234, 1234, True), (1233, 1299, True), (0, 0, False), (2000, 2000, False)]
    dst_r = [(0, 65535, True), (5678, 5678, True), (9999, 9999, False)]
    for s in src_r:
        for d in dst_r:
            c4.append(("l4ACL_ipv4_tcp", "ipv4_tcp",
                       rec4(1, (0, 0), (0, 0), (0, 0), s[:2], d[:2], True), 1 if s[2] and d[2] else 0))
    # TestInternal_l3ACL_packetIPv4_TCP (:540-610): zero l4Rules
    for out in (0, 1, 10, 65535):
        for s in SRC4:
            for d in DST4:
                c4.append(("l3ACL_ipv4_tcp", "ipv4_tcp", rec4(out, s, d), out if s[2] and d[2] else 0))

    def l3l4(group, pkt, ids, srcs, dsts, outs, addr_s, addr_d, fam):
        for idm in ids:
            for sp in srcs:
                for dp in dsts:
                    valid = sp[2] or dp[2]
                    for out in outs:
                        for s in addr_s:
                            for d in addr_d:
                                ok = idm[2] and sp[3] and dp[3] and s[2] and d[2]
                                mk = rec4 if fam == 4 else rec6
                                r = mk(out, s, d, idm[:2], sp[:2], dp[:2], valid)
                                (c4 if fam == 4 else c6).append((group, pkt, r, out if ok else 0))

    ids_tcp = [(0, 0, True), (6, 0xff, True), (17, 0xff, False)]
    ids_udp = [(0, 0, True), (6, 0xff, False), (17, 0xff, True)]
    l3l4("l3l4_ipv4_tcp", "ipv4_tcp", ids_tcp, SRC_TCPUDP, DST_TCPUDP, (0, 1, 65535), SRC4, DST4, 4)
    l3l4("l3l4_ipv6_tcp", "ipv6_tcp", ids_tcp, SRC_TCPUDP, DST_TCPUDP, (0, 1, 65535), ADDR6, ADDR6, 6)
    l3l4("l3l4_ipv6_udp", "ipv6_udp", ids_udp, SRC_TCPUDP, DST_TCPUDP, (0, 1, 65535), ADDR6, ADDR6, 6)
    l3l4("l3l4_ipv4_icmp", "ipv4_icmp", [(0, 0, True), (6, 0xff, False), (17, 0xff, False), (1, 0xff, True)],
         SRC_ICMP, DST_ICMP, (0, 1, 65535), SRC4, DST4, 4)
    l3l4("l3l4_ipv6_icmp", "ipv6_icmp", [(0, 0, True), (6, 0xff, False), (17, 0xff, False), (58, 0xff, True)],
         SRC_ICMP, DST_ICMP, (0, 1, 65535), ADDR6, ADDR6, 6)
    return c4, c6


# ---- parse KAT (rulesL3Ctxt, :91-161; generateTestL3Rules :266-370) -------------
P_SRC4 = [("ANY", 0, 0), ("127.0.0.1/31", 0x0000007f, 0xfeffffff)]
P_DST4 = [("ANY", 0, 0), ("128.9.9.5/24", 0x00090980, 0x00ffffff)]
P_SRC6 = [("ANY", Z16, Z16), ("::/0", Z16, Z16),
          ("dead::beef/16", a6(0xde, 0xad, *[0] * 14), a6(0xff, 0xff, *[0] * 14))]
P_DST6 = [("ANY", Z16, Z16), ("::/0", Z16, Z16),
          ("dead::beef/128", a6(0xde, 0xad, *[0] * 12, 0xbe, 0xef), bytes([0xff] * 16))]
P_IDS = [("ANY", 0, 0), ("TCP", 6, 0xff), ("UDP", 0x11, 0xff), ("ICMP", 1, 0xff)]
P_SPORTS = [("ANY", 0, 65535, False), ("1222", 1222, 1222, True), ("0:222", 0, 222, True)]
P_DPORTS = [("ANY", 0, 65535, False), ("1222", 1222, 1222, True)]
P_RULES = [("Accept", 1), ("Reject", 0)]  # decisions = rules[:2]


def parse_cases():
    cases = []
    for rr, gout in P_RULES:
        for rid, gid, gmask in P_IDS:
            for sp in P_SPORTS:
                for dp in P_DPORTS:
                    if rid == "ICMP" and (sp[0] != "ANY" or dp[0] != "ANY"):
                        continue
                    l4 = dict(id=gid, id_mask=gmask, valid=sp[3] or dp[3], src_port_min=sp[1],
                              src_port_max=sp[2], dst_port_min=dp[1], dst_port_max=dp[2])
                    for s in P_SRC4:
                        for d in P_DST4:
                            cases.append(dict(
                                family=4, raw=[s[0], d[0], rid, sp[0], dp[0], rr],
                                want=dict(output_number=gout, src_addr=s[1], dst_addr=d[1],
                                          src_mask=s[2], dst_mask=d[2], **l4)))
                    for s in P_SRC6:
                        for d in P_DST6:
                            cases.append(dict(
                                family=6, raw=[s[0], d[0], rid, sp[0], dp[0], rr],
                                want=dict(output_number=gout, src_addr=s[1].hex(), dst_addr=d[1].hex(),
                                          src_mask=s[2].hex(), dst_mask=d[2].hex(), **l4)))
    return cases


# ---- header-parse KAT (packet_test.go:22-267) ------------------------------------
PARSE_LINES = [
    "00112233445501112131415108004500002ebffd00000406747a7f0000018009090504d2162e123456781234569050102000ffe60000",
    "00112233445501112131415108004500002ebffd00000406747a7f000000800909ff04d2162f123456781234569050102000ffe60000",
    "00112233445501112131415208004500002ebffd00000411747a7f000000800909ff04d3162f00400000",
    "00112233445501112131415208004500002ebffd00000406747a7f0000ff800909051234162f123456781234569050102000ffe60000",
    "00112233445501112131415208004500002ebffd00000406747a123456788009090f12345678123456781234569050102000ffe60000",
    "00122233445501112131415208004500002ebffd00000411747a123456788009091404d2000000400000",
    "10112233445501112131415108004500002ebffd00000406747a123456788009091412345678123456781234569050102000ffe60000",
    "00112233445501112131415108004500002ebffd00000411747a123456788009091404d2000000400000",
]
# (VersionIhl, NextProtoID, SrcAddr, DstAddr) of IPHeader[0..6]; L4 (SrcPort, DstPort) as stored
IPH = [(0x45, 0x06, 0x0100007f, 0x05090980), (0x45, 0x06, 0x0000007f, 0xff090980),
       (0x45, 0x11, 0x0000007f, 0xff090980), (0x45, 0x06, 0xff00007f, 0x05090980),
       (0x45, 0x06, 0x78563412, 0x0f090980), (0x45, 0x11, 0x78563412, 0x14090980),
       (0x45, 0x06, 0x78563412, 0x14090980)]
TCPH = [(0xd204, 0x2e16), (0xd204, 0x2f16), (0x3412, 0x2f16), (0x3412, 0x7856)]
UDPH = [(0xd304, 0x2f16), (0xd204, 0x0000)]
PKTS = [(0, TCPH[0]), (1, TCPH[1]), (2, UDPH[0]), (3, TCPH[2]), (4, TCPH[3]), (5, UDPH[1]), (6, TCPH[3]), (5, UDPH[1])]


def parse_l3_kat():
    out = []
    for line, (ipi, l4) in zip(PARSE_LINES, PKTS):
        vihl, proto, src, dst = IPH[ipi]
        out.append(dict(hex=line, version_ihl=vihl, proto=proto, src_addr=src, dst_addr=dst,
                        src_port_le=l4[0], dst_port_le=l4[1]))
    return out


# ---- L2 (acl_internal_test.go:66-89, 174-243, 1144-1273) -------------------------
BCAST = bytes([0xff] * 6)


def arp_request(sha: bytes, spa: bytes, tpa: bytes) -> bytes:
    """InitARPRequestPacket (arp.go:79-93 over initARPCommonData :60-73 and
    InitEmptyARPPacket packet.go:563-573): Ether + 28-byte ARP, fresh mbuf zeros."""
    eth = BCAST + sha + b"\x08\x06"
    arp = struct.pack(">HHBBH", 1, 0x0800, 6, 4, 1) + sha + spa + BCAST + tpa
    return eth + arp


# arp_test.go:22 (gtLineARPRequest, made with gopacket) for the parameters of
# TestInitARPCommonDataPacket / TestInitARPRequestPacket: pins arp_request().
GT_ARP_REQUEST = "ffffffffffff00070daff4540806000108000604000100070daff45418a6ac01ffffffffffff18a6ad9f"
assert arp_request(bytes.fromhex("00070daff454"), bytes([24, 166, 172, 1]),
                   bytes([24, 166, 173, 159])).hex() == GT_ARP_REQUEST

# getARPRequestTestPacket (utils_for_test.go:95-104)
PACKETS["arp_request"] = arp_request(SMAC, V4_SRC, V4_DST)

L2_RULES = [("Accept", 1), ("Reject", 0), ("3", 3), ("", 0)]  # "" only in the text format
L2_SRCS = [("ANY", bytes(6), False), ("00:11:22:33:44:55", DMAC, True)]
L2_DSTS = [("ANY", bytes(6), False), ("01:11:21:31:41:51", SMAC, True)]
L2_IDS = [("ANY", 0, 0), ("IPv4", 0x0800, 0xffff), ("IPv6", 0x86dd, 0xffff), ("arp", 0x0806, 0xffff)]


def l2_parse_cases():
    """generateTestL2Rules: JSON over decisions = rules[:2] (the reference's
    text-format test iterates an empty decision list, :180-182, so the text
    cases here reuse all four decisions — an extension, not a transcription)."""
    cases = []
    for fmt, decisions in (("json", L2_RULES[:2]), ("text", L2_RULES)):
        for rr, gout in decisions:
            for s in L2_SRCS:
                for d in L2_DSTS:
                    for rid, gid, gmask in L2_IDS:
                        cases.append(dict(
                            format=fmt, raw=dict(Rule=rr, Source=s[0], Destination=d[0], ID=rid),
                            want=dict(output_number=gout, daddr_not_any=d[2], saddr_not_any=s[2],
                                      daddr=d[1].hex(), saddr=s[1].hex(), id_mask=gmask, id=gid)))
    return cases


def l2_match_cases():
    """TestInternal_l2ACL_packetIPv4 / _packetARP (:1144-1273): one single-rule
    table per (output, id, src, dst) combination; want = output iff all ok."""
    outs = [0, 1, 65535]
    tables = {
        "ipv4_udp": (
            [(0, 0, True), (0x0800, 0xffff, True), (0x86dd, 0xffff, False), (0x0806, 0xffff, False)],
            [(bytes(6), False, True), (SMAC, True, True), (bytes([0, 0x55, 0x55, 0x55, 0x55, 0]), True, False)],
            [(bytes(6), False, True), (DMAC, True, True), (SMAC, True, False)]),
        "arp_request": (
            [(0, 0, True), (0x0800, 0xffff, False), (0x86dd, 0xffff, False), (0x0806, 0xffff, True)],
            [(bytes(6), False, True), (SMAC, True, True), (DMAC, True, False)],
            [(bytes(6), False, True), (BCAST, True, True), (SMAC, True, False)]),
    }
    cases = []
    for pkt, (ids, srcs, dsts) in tables.items():
        for out in outs:
            for idv, idm, idok in ids:
                for sa, sna, sok in srcs:
                    for da, dna, dok in dsts:
                        cases.append(dict(
                            packet=pkt,
                            rule=dict(output_number=out, daddr_not_any=dna, saddr_not_any=sna,
                                      daddr=da.hex(), saddr=sa.hex(), id_mask=idm, id=idv),
                            want=out if (idok and sok and dok) else 0))
    return cases


# ---- VLAN parse KAT (vlan_test.go:23-67, TestParseAllKnownL3CheckVLAN :239-269) ----
VLAN_KAT = dict(
    hex="00400540ef240060089fb1f3810000200800450000288a1b00004006000083972015839720811770048a"
        "0000000100000d9550107c7000000000",
    tci=32, inner_ethertype=0x0800,
    src=[131, 151, 32, 21], dst=[131, 151, 32, 129], proto=6,  # IPv4HeaderVLAN
    sport=6000, dport=1162,                                   # TCPHeaderVLAN
)


def main():
    (HERE / "kat_packets.json").write_text(json.dumps({k: v.hex() for k, v in PACKETS.items()}, indent=1) + "\n")
    c4, c6 = match_cases()
    groups = sorted({c[0] for c in c4 + c6})
    np.savez_compressed(
        HERE / "acl_match_kats.npz",
        packet_names=np.array(PKT_NAMES), groups=np.array(groups),
        c4_group=np.array([groups.index(c[0]) for c in c4], np.uint8),
        c4_packet=np.array([PKT_NAMES.index(c[1]) for c in c4], np.uint8),
        c4_rule=np.array([c[2] for c in c4], RULE4),
        c4_want=np.array([c[3] for c in c4], np.uint32),
        c6_group=np.array([groups.index(c[0]) for c in c6], np.uint8),
        c6_packet=np.array([PKT_NAMES.index(c[1]) for c in c6], np.uint8),
        c6_rule=np.array([c[2] for c in c6], RULE6),
        c6_want=np.array([c[3] for c in c6], np.uint32),
    )
    (HERE / "parse_kats.json").write_text(
        "[\n" + ",\n".join(json.dumps(c, separators=(",", ":")) for c in parse_cases()) + "\n]\n")
    (HERE / "parse_l3_kat.json").write_text(json.dumps(parse_l3_kat(), indent=1) + "\n")
    (HERE / "vlan_kat.json").write_text(json.dumps(VLAN_KAT, indent=1) + "\n")
    l2 = dict(parse=l2_parse_cases(), match=l2_match_cases())
    (HERE / "l2_kats.json").write_text(
        "{\"parse\": [\n" + ",\n".join(json.dumps(c, separators=(",", ":")) for c in l2["parse"]) +
        "\n], \"match\": [\n" + ",\n".join(json.dumps(c, separators=(",", ":")) for c in l2["match"]) + "\n]}\n")
    print(f"match KATs: {len(c4)} ipv4 + {len(c6)} ipv6 = {len(c4) + len(c6)}; "
          f"parse KATs: {len(parse_cases())}; parse-L3 frames: {len(PARSE_LINES)}; "
          f"L2 parse: {len(l2['parse'])}, L2 match: {len(l2['match'])}")


if __name__ == "__main__":
    main()
