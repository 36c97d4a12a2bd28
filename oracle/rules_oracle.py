"""TEST INFRASTRUCTURE ONLY — independent restatement of nff-go's rule loader.

This module is the parity oracle for libnffacl's rule parser (the product's
parser is C++, nff-go_amd/csrc/rules.cpp; this one shares no code with it).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
it.  It follows, with go1.13 standard-library semantics (Dockerfile:25 pins
go1.13.1):

  GetL3ACLFromTextTable  packet/acl.go:148-178   bufio.ScanLines + strings.Fields
  GetL3ACLFromJSON       packet/acl.go:121-134   encoding/json into rawL3Rules
  rawL3Parse             packet/acl.go:226-355
  parseL4Port            packet/acl.go:357-383   strconv.ParseUint(s, 10, 16)
  parseRuleResult        packet/acl.go:385-398   strconv.ParseUint(s, 10, 32)
  parseAddr4/6           packet/acl.go:400-411   net.ParseCIDR -> LE uint32 / 16 bytes
  GetL2ACLFromTextTable  packet/acl.go:88-117    (L2 rules, §8f next row)
  GetL2ACLFromJSON       packet/acl.go:70-84
  rawL2Parse             packet/acl.go:356-383   net.ParseMAC

Pinning: the expected records of the reference's parse KATs
(packet/acl_internal_test.go:91-161, via tests/golden/make_kats.py) and the
rule files the reference ships (tests/golden/rules/).

Divergence (shared with the product, documented in DESIGN.md): a malformed
CIDR makes the reference dereference a nil *IPNet (acl.go:275-282); here it is
IncorrectArgInRules (14).
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field

import numpy as np

# common.ErrorCode values (common/error.go:18-50)
PARSE_RULE_JSON_ERR = 11
FILE_ERR = 12
PARSE_RULE_ERR = 13
INCORRECT_ARG_IN_RULES = 14
INCORRECT_RULE = 15

# numpy views of the records (same byte layout as nffacl_rule4/6 and orc_rule4/6)
L4_FIELDS = [("id", "u1"), ("id_mask", "u1"), ("valid", "u1"), ("reserved", "u1"),
             ("src_port_min", "<u2"), ("src_port_max", "<u2"),
             ("dst_port_min", "<u2"), ("dst_port_max", "<u2")]
RULE4_DTYPE = np.dtype([("output_number", "<u4"), ("src_addr", "<u4"), ("dst_addr", "<u4"),
                        ("src_mask", "<u4"), ("dst_mask", "<u4")] + L4_FIELDS)
RULE6_DTYPE = np.dtype([("output_number", "<u4"), ("src_addr", "u1", 16), ("dst_addr", "u1", 16),
                        ("src_mask", "u1", 16), ("dst_mask", "u1", 16)] + L4_FIELDS)
assert RULE4_DTYPE.itemsize == 32 and RULE6_DTYPE.itemsize == 80
L2RULE_DTYPE = np.dtype([("output_number", "<u4"), ("daddr_not_any", "u1"), ("saddr_not_any", "u1"),
                         ("daddr", "u1", 6), ("saddr", "u1", 6), ("id_mask", "<u2"), ("id", "<u2"),
                         ("reserved", "<u2")])
assert L2RULE_DTYPE.itemsize == 24


class OracleParseError(Exception):
    def __init__(self, code: int, message: str):
        super().__init__(f"{message} ({code})")
        self.code = code
        self.message = message


@dataclass
class L4:
    id: int = 0
    id_mask: int = 0
    valid: bool = False
    src_port_min: int = 0
    src_port_max: int = 0
    dst_port_min: int = 0
    dst_port_max: int = 0


@dataclass
class Rule4:
    output_number: int
    src_addr: int
    dst_addr: int
    src_mask: int
    dst_mask: int
    l4: L4


@dataclass
class Rule6:
    output_number: int
    src_addr: bytes
    dst_addr: bytes
    src_mask: bytes
    dst_mask: bytes
    l4: L4


@dataclass
class L3Rules:
    ip4: list = field(default_factory=list)
    ip6: list = field(default_factory=list)

    def arrays(self):
        """(ip4, ip6) as numpy record arrays (RULE4_DTYPE / RULE6_DTYPE)."""
        a4 = np.zeros(len(self.ip4), RULE4_DTYPE)
        for i, r in enumerate(self.ip4):
            a4[i] = (r.output_number, r.src_addr, r.dst_addr, r.src_mask, r.dst_mask,
                     r.l4.id, r.l4.id_mask, int(r.l4.valid), 0, r.l4.src_port_min,
                     r.l4.src_port_max, r.l4.dst_port_min, r.l4.dst_port_max)
        a6 = np.zeros(len(self.ip6), RULE6_DTYPE)
        for i, r in enumerate(self.ip6):
            a6[i] = (r.output_number, np.frombuffer(r.src_addr, "u1"), np.frombuffer(r.dst_addr, "u1"),
                     np.frombuffer(r.src_mask, "u1"), np.frombuffer(r.dst_mask, "u1"),
                     r.l4.id, r.l4.id_mask, int(r.l4.valid), 0, r.l4.src_port_min,
                     r.l4.src_port_max, r.l4.dst_port_min, r.l4.dst_port_max)
        return a4, a6


# --------------------------------------------------------------------------
# go1.13 stdlib pieces
# --------------------------------------------------------------------------

_GO_SPACE = {0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x20, 0x85, 0xA0, 0x1680, 0x2028, 0x2029, 0x202F,
             0x205F, 0x3000} | set(range(0x2000, 0x200B))


def go_fields(line: bytes) -> list[bytes]:
    """strings.Fields: split on unicode.IsSpace runes of the UTF-8 text."""
    out, cur, i = [], bytearray(), 0
    n = len(line)
    while i < n:
        r, w = _decode_rune(line, i)
        if r in _GO_SPACE:
            if cur:
                out.append(bytes(cur))
                cur = bytearray()
        else:
            cur += line[i:i + w]
        i += w
    if cur:
        out.append(bytes(cur))
    return out


def _decode_rune(b: bytes, i: int):
    """utf8.DecodeRune: (rune, width); invalid -> (0xFFFD, 1)."""
    for w in (1, 2, 3, 4):
        chunk = b[i:i + w]
        if len(chunk) < w:
            break
        try:
            s = chunk.decode("utf-8", errors="strict")
        except UnicodeDecodeError:
            continue
        if len(s) == 1:
            return ord(s), w
    return 0xFFFD, 1


def go_parse_uint(s: bytes, bits: int):
    """strconv.ParseUint(s, 10, bits) -> int or None on error."""
    if not s or any(c < 0x30 or c > 0x39 for c in s):
        return None
    v = int(s.decode("ascii"))
    return v if v <= (1 << bits) - 1 else None


_BIG = 0xFFFFFF


def _dtoi(s: str):
    n, i = 0, 0
    while i < len(s) and "0" <= s[i] <= "9":
        n = n * 10 + ord(s[i]) - 48
        if n >= _BIG:
            return _BIG, i, False
        i += 1
    if i == 0:
        return 0, 0, False
    return n, i, True


def _xtoi(s: str):
    n, i = 0, 0
    while i < len(s):
        c = s[i]
        if "0" <= c <= "9":
            d = ord(c) - 48
        elif "a" <= c <= "f":
            d = ord(c) - 87
        elif "A" <= c <= "F":
            d = ord(c) - 55
        else:
            break
        n = n * 16 + d
        if n >= _BIG:
            return 0, i, False
        i += 1
    if i == 0:
        return 0, i, False
    return n, i, True


def _parse_ipv4(s: str):
    out = []
    for i in range(4):
        if not s:
            return None
        if i > 0:
            if s[0] != ".":
                return None
            s = s[1:]
        n, c, ok = _dtoi(s)
        if not ok or n > 0xFF:
            return None
        s = s[c:]
        out.append(n)
    if s:
        return None
    return bytes(out)


def _parse_ipv6(s: str):
    ip = bytearray(16)
    ellipsis = -1
    if len(s) >= 2 and s[0] == ":" and s[1] == ":":
        ellipsis = 0
        s = s[2:]
        if not s:
            return bytes(ip)
    i = 0
    while i < 16:
        n, c, ok = _xtoi(s)
        if not ok or n > 0xFFFF:
            return None
        if c < len(s) and s[c] == ".":
            if ellipsis < 0 and i != 12:
                return None
            if i + 4 > 16:
                return None
            v4 = _parse_ipv4(s)
            if v4 is None:
                return None
            ip[i:i + 4] = v4
            s = ""
            i += 4
            break
        ip[i] = n >> 8
        ip[i + 1] = n & 0xFF
        i += 2
        s = s[c:]
        if not s:
            break
        if s[0] != ":" or len(s) == 1:
            return None
        s = s[1:]
        if s[0] == ":":
            if ellipsis >= 0:
                return None
            ellipsis = i
            s = s[1:]
            if not s:
                break
    if s:
        return None
    if i < 16:
        if ellipsis < 0:
            return None
        n = 16 - i
        ip[ellipsis + n:16] = ip[ellipsis:i]
        ip[ellipsis:ellipsis + n] = bytes(n)
    elif ellipsis >= 0:
        return None
    return bytes(ip)


def go_parse_cidr(text: bytes):
    """net.ParseCIDR -> (network ip bytes, mask bytes) or None.

    Dotted quads come back as 4 bytes (IP.Mask trims the v4-in-v6 form
    against the 4-byte mask), IPv6 syntax as 16."""
    try:
        s = text.decode("utf-8")
    except UnicodeDecodeError:
        s = text.decode("latin-1")  # cannot parse either way
    if "/" not in s:
        return None
    addr, m = s.split("/", 1)
    ip = _parse_ipv4(addr)
    iplen = 4
    if ip is None:
        iplen = 16
        ip = _parse_ipv6(addr)
    n, used, ok = _dtoi(m)
    if ip is None or not ok or used != len(m) or n < 0 or n > 8 * iplen:
        return None
    ones = (1 << (8 * iplen)) - 1
    mask_int = (ones << (8 * iplen - n)) & ones
    mask = mask_int.to_bytes(iplen, "big")
    net = bytes(a & b for a, b in zip(ip, mask))
    return net, mask


# --------------------------------------------------------------------------
# acl.go restatement
# --------------------------------------------------------------------------

_IDS = {
    b"ANY": (0, 0),
    **{k: (6, 0xFF) for k in (b"tcp", b"TCP", b"Tcp", b"0x06", b"6")},
    **{k: (17, 0xFF) for k in (b"udp", b"UDP", b"Udp", b"0x11", b"17")},
    **{k: (1, 0xFF) for k in (b"icmp", b"ICMP", b"Icmp", b"0x01", b"1")},
}


def parse_l4_port(port: bytes):
    """parseL4Port, acl.go:357-383 -> (min, max, valid)."""
    if port in (b"ANY", b"0:65535"):
        return 0, 65535, False
    if b":" not in port:
        port = port + b":" + port
    lo_s, hi_s = port.split(b":", 1)
    lo, hi = go_parse_uint(lo_s, 16), go_parse_uint(hi_s, 16)
    if lo is None or hi is None:
        raise OracleParseError(INCORRECT_ARG_IN_RULES,
                               f"Incorrect request: cannot parse Min and Max port values in {port!r}")
    if lo > hi:
        raise OracleParseError(INCORRECT_ARG_IN_RULES, f"Incorrect request: minPort > maxPort, port: {port!r}")
    return lo, hi, True


def parse_rule_result(rule: bytes) -> int:
    """parseRuleResult, acl.go:385-398."""
    if rule in (b"Accept", b"true"):
        return 1
    if rule in (b"Reject", b"false"):
        return 0
    v = go_parse_uint(rule, 32)
    if v is None:
        raise OracleParseError(INCORRECT_RULE, f"Incorrect rule: {rule!r}")
    return v


def raw_l3_parse(raw: list) -> L3Rules:
    """rawL3Parse, acl.go:226-355.  raw: list of 6-tuples of bytes
    (SrcAddr, DstAddr, ID, SrcPort, DstPort, OutputNumber)."""
    rules = L3Rules()
    for src, dst, ident, sport, dport, outnum in raw:
        if ident not in _IDS:
            raise OracleParseError(INCORRECT_ARG_IN_RULES, f"Incorrect  L4 protocol ID: {ident!r}")
        pid, pmask = _IDS[ident]
        if pid == 1 and (sport != b"ANY" or dport != b"ANY"):
            raise OracleParseError(INCORRECT_ARG_IN_RULES,
                                   "Incorrect request: for ICMP rule Source port and Destination port should be ANY")
        smin, smax, svalid = parse_l4_port(sport)
        dmin, dmax, dvalid = parse_l4_port(dport)
        l4 = L4(pid, pmask, svalid or dvalid, smin, smax, dmin, dmax)

        def addr(text):
            if text == b"ANY":
                return None
            parsed = go_parse_cidr(text)
            if parsed is None:  # reference: nil dereference panic
                raise OracleParseError(INCORRECT_ARG_IN_RULES, f"Incorrect address (invalid CIDR): {text!r}")
            return parsed

        sa, da = addr(src), addr(dst)
        slen = 0 if sa is None else len(sa[0])
        dlen = 0 if da is None else len(da[0])
        if {slen, dlen} == {4, 16}:
            raise OracleParseError(INCORRECT_ARG_IN_RULES, "Incorrect request: IPv4 + IPv6 in one rule")

        def v4(a):
            return (0, 0) if a is None else (int.from_bytes(a[0], "little"), int.from_bytes(a[1], "little"))

        def v6(a):
            return (bytes(16), bytes(16)) if a is None else a

        if slen == 0 and dlen == 0:
            out = parse_rule_result(outnum)
            rules.ip4.append(Rule4(out, 0, 0, 0, 0, l4))
            out = parse_rule_result(outnum)
            rules.ip6.append(Rule6(out, bytes(16), bytes(16), bytes(16), bytes(16), l4))
        elif 4 in (slen, dlen):
            out = parse_rule_result(outnum)
            (s_a, s_m), (d_a, d_m) = v4(sa), v4(da)
            rules.ip4.append(Rule4(out, s_a, d_a, s_m, d_m, l4))
        else:
            out = parse_rule_result(outnum)
            (s_a, s_m), (d_a, d_m) = v6(sa), v6(da)
            rules.ip6.append(Rule6(out, s_a, d_a, s_m, d_m, l4))
    return rules


def _scan_table(data: bytes, nfields: int, incomplete: str) -> list:
    """bufio.ScanLines + strings.Fields loop shared by both text loaders
    (acl.go:97-112, 156-173)."""
    rows = []
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()  # ScanLines yields no empty final token
    for line in lines:
        if len(line) >= 64 * 1024:
            raise OracleParseError(FILE_ERR, "file error during rules parsing: token too long")
        if line.endswith(b"\r"):
            line = line[:-1]
        if len(line) == 0 or line[0:1] == b"#":
            continue
        f = go_fields(line)
        if len(f) == nfields - 1:
            f.append(b"false")
        elif len(f) != nfields:
            raise OracleParseError(PARSE_RULE_ERR, incomplete)
        rows.append(tuple(f))
    return rows


def parse_text_table(data: bytes) -> L3Rules:
    """GetL3ACLFromTextTable body over a file image (acl.go:156-177)."""
    return raw_l3_parse(_scan_table(data, 6, "Incomplete 5-tuple for rule parsing"))


def load_text_table(path) -> L3Rules:
    try:
        with open(path, "rb") as fh:
            data = fh.read()
    except OSError as e:
        raise OracleParseError(FILE_ERR, f"file error during rules parsing: {e}") from None
    return parse_text_table(data)


_JSON_FIELDS = ("SrcAddr", "DstAddr", "ID", "SrcPort", "DstPort", "OutputNumber")


def _reject_constant(name):
    raise ValueError(f"invalid JSON literal {name}")


def json_key_matches(key: str, field_name: str) -> bool:
    """encoding/json field lookup (go1.13 fold.go): ASCII case folding, plus
    U+017F (long s) for s and U+212A (Kelvin) for k."""
    key = key.replace("\u017f", "s").replace("\u212a", "k")
    return key.isascii() and key.lower() == field_name.lower()


def _json_records(data: bytes, top: str, fields: tuple) -> list:
    """json.Unmarshal of {top: [{field: string}]} (the last matching key wins,
    null leaves the field as is, a non-string value is an UnmarshalTypeError)."""
    try:
        doc = json.loads(data.decode("utf-8", errors="replace"), parse_constant=_reject_constant,
                         object_pairs_hook=lambda pairs: ("obj", pairs))
    except ValueError as e:
        raise OracleParseError(PARSE_RULE_JSON_ERR, f"JSON error during rules parsing: {e}") from None
    if doc is None:
        return []
    if not (isinstance(doc, tuple) and doc[0] == "obj"):
        raise OracleParseError(PARSE_RULE_JSON_ERR, "JSON error during rules parsing: not an object")
    type_error = False
    arr = None
    for k, v in doc[1]:
        if json_key_matches(k, top):
            if v is None:
                continue
            if not isinstance(v, list):
                type_error = True
                continue
            arr = v
    raw = []
    for elem in arr or []:
        rec = {f: b"" for f in fields}
        if elem is not None and not (isinstance(elem, tuple) and elem[0] == "obj"):
            type_error = True
        elif elem is not None:
            for k, v in elem[1]:
                for f in fields:
                    if json_key_matches(k, f):
                        if isinstance(v, str):
                            # lone surrogates from \u escapes -> U+FFFD, as Go does
                            rec[f] = v.encode("utf-16", "surrogatepass").decode("utf-16", "replace").encode("utf-8")
                        elif v is not None:
                            type_error = True
                        break
        raw.append(tuple(rec[f] for f in fields))
    if type_error:
        raise OracleParseError(PARSE_RULE_JSON_ERR, "JSON error during rules parsing: type mismatch")
    return raw


def parse_json(data: bytes) -> L3Rules:
    """GetL3ACLFromJSON body (acl.go:129-133): json.Unmarshal into rawL3Rules,
    then rawL3Parse."""
    return raw_l3_parse(_json_records(data, "L3Rules", _JSON_FIELDS))


def load_json(path) -> L3Rules:
    try:
        with open(path, "rb") as fh:
            data = fh.read()
    except OSError as e:
        raise OracleParseError(FILE_ERR, f"file error during rules parsing: {e}") from None
    return parse_json(data)


# --------------------------------------------------------------------------
# L2 rules (acl.go:68-117, 356-383)
# --------------------------------------------------------------------------

@dataclass
class Rule2:
    output_number: int = 0
    daddr_not_any: bool = False
    saddr_not_any: bool = False
    daddr: bytes = bytes(6)
    saddr: bytes = bytes(6)
    id_mask: int = 0
    id: int = 0


@dataclass
class L2Rules:
    eth: list = field(default_factory=list)

    def array(self) -> np.ndarray:
        a = np.zeros(len(self.eth), L2RULE_DTYPE)
        for i, r in enumerate(self.eth):
            a[i] = (r.output_number, int(r.daddr_not_any), int(r.saddr_not_any),
                    np.frombuffer(r.daddr, "u1"), np.frombuffer(r.saddr, "u1"), r.id_mask, r.id, 0)
        return a


_HEX = "0123456789abcdefABCDEF"


def go_parse_mac(s: bytes):
    """go1.13 net.ParseMAC: bytes of a 6/8/20-byte address, or None."""
    s = s.decode("latin-1")  # byte-wise, as Go indexes the string

    def two_hex(x: str):
        if len(x) != 2 or x[0] not in _HEX or x[1] not in _HEX:
            return None
        return int(x, 16)

    if len(s) < 14:
        return None
    out = []
    if s[2] in ":-":
        sep = s[2]
        if (len(s) + 1) % 3:
            return None
        n = (len(s) + 1) // 3
        if n not in (6, 8, 20):
            return None
        for i in range(n):
            grp = s[3 * i:3 * i + 2]
            if 3 * i + 2 < len(s) and s[3 * i + 2] != sep:
                return None
            b = two_hex(grp)
            if b is None:
                return None
            out.append(b)
    elif s[4] == ".":
        if (len(s) + 1) % 5:
            return None
        n = 2 * (len(s) + 1) // 5
        if n not in (6, 8, 20):
            return None
        for g in range(n // 2):
            x = 5 * g
            if x + 4 < len(s) and s[x + 4] != ".":
                return None
            hi, lo = two_hex(s[x:x + 2]), two_hex(s[x + 2:x + 4])
            if hi is None or lo is None:
                return None
            out += [hi, lo]
    else:
        return None
    return bytes(out)


_L2_IDS = {
    b"ANY": (0, 0),
    **{k: (0x0800, 0xFFFF) for k in (b"ipv4", b"Ipv4", b"IPv4", b"IPV4", b"0x0800")},
    **{k: (0x86DD, 0xFFFF) for k in (b"ipv6", b"Ipv6", b"IPv6", b"IPV6", b"0x86dd")},
    **{k: (0x0806, 0xFFFF) for k in (b"arp", b"Arp", b"ARP", b"0x0806")},
}


def raw_l2_parse(raw: list) -> L2Rules:
    """rawL2Parse (acl.go:356-383); raw items are (Rule, Source, Destination, ID)."""
    rules = L2Rules()
    for rule, src, dst, ident in raw:
        r = Rule2(output_number=parse_rule_result(rule))
        if src != b"ANY":
            r.saddr_not_any = True
            hw = go_parse_mac(src)
            if hw is None:
                raise OracleParseError(INCORRECT_ARG_IN_RULES, f"Incorrect source MAC: {src!r}")
            r.saddr = hw[:6]
        if dst != b"ANY":
            r.daddr_not_any = True
            hw = go_parse_mac(dst)
            if hw is None:
                raise OracleParseError(INCORRECT_ARG_IN_RULES, f"Incorrect destination MAC: {dst!r}")
            r.daddr = hw[:6]
        if ident not in _L2_IDS:
            raise OracleParseError(INCORRECT_ARG_IN_RULES, f"Incorrect  L3 protocol ID: {ident!r}")
        r.id, r.id_mask = _L2_IDS[ident]
        rules.eth.append(r)
    return rules


def parse_l2_text_table(data: bytes) -> L2Rules:
    """GetL2ACLFromTextTable body (acl.go:97-117): Source Destination ID [Rule]."""
    rows = _scan_table(data, 4, "Incomplete 3-tuple for rule parsing")
    return raw_l2_parse([(f[3], f[0], f[1], f[2]) for f in rows])


_L2_JSON_FIELDS = ("Rule", "Source", "Destination", "ID")


def parse_l2_json(data: bytes) -> L2Rules:
    """GetL2ACLFromJSON body (acl.go:78-83)."""
    return raw_l2_parse(_json_records(data, "L2Rules", _L2_JSON_FIELDS))
