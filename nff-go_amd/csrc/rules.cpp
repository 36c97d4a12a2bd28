// rules.cpp — rule-file parsing for libnffacl.
//
// Restates, for the C-ABI, nff-go's rule loader:
//   GetL3ACLFromTextTable  packet/acl.go:148-178
//   rawL3Parse             packet/acl.go:226-355
//   parseL4Port            packet/acl.go:357-383
//   parseRuleResult        packet/acl.go:385-398
//   parseAddr4/parseAddr6  packet/acl.go:400-411
// with the go1.13 standard-library behaviour those functions lean on
// (Dockerfile:25 pins go1.13.1): bufio.ScanLines, strings.Fields,
// strconv.ParseUint, net.ParseCIDR.
//
// Documented divergence: where the reference dereferences the nil *IPNet that
// net.ParseCIDR returns for a malformed address (acl.go:275-282, a panic), this
// parser reports NFFACL_ERR_INCORRECT_ARG_IN_RULES instead.
#include "rules.hpp"

#include <cstdio>
#include <cstring>

namespace nffacl {

namespace {

// ---- go1.13 unicode.IsSpace over UTF-8 (strings.Fields) -------------------

// Decode one rune starting at s[i]; returns its byte width (>=1).  Invalid
// encodings decode as U+FFFD with width 1, as Go's utf8.DecodeRuneInString.
int decode_rune(const std::string &s, size_t i, uint32_t &r) {
    const unsigned char c0 = static_cast<unsigned char>(s[i]);
    if (c0 < 0x80) { r = c0; return 1; }
    auto cont = [&](size_t k) -> int {
        if (k >= s.size()) return -1;
        unsigned char c = static_cast<unsigned char>(s[k]);
        return (c & 0xC0) == 0x80 ? (c & 0x3F) : -1;
    };
    if (c0 >= 0xC2 && c0 <= 0xDF) {
        int c1 = cont(i + 1);
        if (c1 >= 0) { r = ((c0 & 0x1F) << 6) | c1; return 2; }
    } else if (c0 >= 0xE0 && c0 <= 0xEF) {
        int c1 = cont(i + 1), c2 = cont(i + 2);
        if (c1 >= 0 && c2 >= 0) {
            uint32_t v = ((c0 & 0x0F) << 12) | (c1 << 6) | c2;
            if (v >= 0x800 && !(v >= 0xD800 && v <= 0xDFFF)) { r = v; return 3; }
        }
    } else if (c0 >= 0xF0 && c0 <= 0xF4) {
        int c1 = cont(i + 1), c2 = cont(i + 2), c3 = cont(i + 3);
        if (c1 >= 0 && c2 >= 0 && c3 >= 0) {
            uint32_t v = ((c0 & 0x07) << 18) | (c1 << 12) | (c2 << 6) | c3;
            if (v >= 0x10000 && v <= 0x10FFFF) { r = v; return 4; }
        }
    }
    r = 0xFFFD;
    return 1;
}

bool go_is_space(uint32_t r) {
    switch (r) {
    case '\t': case '\n': case '\v': case '\f': case '\r': case ' ':
    case 0x85: case 0xA0: case 0x1680: case 0x2028: case 0x2029:
    case 0x202F: case 0x205F: case 0x3000:
        return true;
    default:
        return r >= 0x2000 && r <= 0x200A;
    }
}

// ---- go1.13 net package pieces -------------------------------------------

constexpr int kBig = 0xFFFFFF;  // net.big

// net.dtoi: decimal prefix of s.
void go_dtoi(const std::string &s, size_t start, int &n, size_t &used, bool &ok) {
    n = 0;
    size_t i = start;
    for (; i < s.size() && s[i] >= '0' && s[i] <= '9'; ++i) {
        n = n * 10 + (s[i] - '0');
        if (n >= kBig) { n = kBig; used = i - start; ok = false; return; }
    }
    used = i - start;
    ok = used != 0;
    if (!ok) n = 0;
}

// net.xtoi: hexadecimal prefix of s.
void go_xtoi(const std::string &s, size_t start, int &n, size_t &used, bool &ok) {
    n = 0;
    size_t i = start;
    for (; i < s.size(); ++i) {
        char c = s[i];
        int d;
        if (c >= '0' && c <= '9') d = c - '0';
        else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
        else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
        else break;
        n = n * 16 + d;
        if (n >= kBig) { n = 0; used = i - start; ok = false; return; }
    }
    used = i - start;
    ok = used != 0;
    if (!ok) n = 0;
}

// net.parseIPv4 (go1.13: leading zeros accepted, decimal).
bool go_parse_ipv4(const std::string &s, uint8_t out[4]) {
    size_t p = 0;
    for (int i = 0; i < 4; ++i) {
        if (p >= s.size()) return false;
        if (i > 0) {
            if (s[p] != '.') return false;
            ++p;
        }
        int n; size_t c; bool ok;
        go_dtoi(s, p, n, c, ok);
        if (!ok || n > 0xFF) return false;
        p += c;
        out[i] = static_cast<uint8_t>(n);
    }
    return p == s.size();
}

// net.parseIPv6(s, zoneAllowed=false).
bool go_parse_ipv6(const std::string &str, uint8_t ip[16]) {
    std::memset(ip, 0, 16);
    std::string s = str;
    int ellipsis = -1;
    if (s.size() >= 2 && s[0] == ':' && s[1] == ':') {
        ellipsis = 0;
        s = s.substr(2);
        if (s.empty()) return true;
    }
    int i = 0;
    while (i < 16) {
        int n; size_t c; bool ok;
        go_xtoi(s, 0, n, c, ok);
        if (!ok || n > 0xFFFF) return false;
        if (c < s.size() && s[c] == '.') {
            if (ellipsis < 0 && i != 16 - 4) return false;
            if (i + 4 > 16) return false;
            uint8_t v4[4];
            if (!go_parse_ipv4(s, v4)) return false;
            std::memcpy(ip + i, v4, 4);
            s.clear();
            i += 4;
            break;
        }
        ip[i] = static_cast<uint8_t>(n >> 8);
        ip[i + 1] = static_cast<uint8_t>(n);
        i += 2;
        s = s.substr(c);
        if (s.empty()) break;
        if (s[0] != ':' || s.size() == 1) return false;
        s = s.substr(1);
        if (s[0] == ':') {
            if (ellipsis >= 0) return false;
            ellipsis = i;
            s = s.substr(1);
            if (s.empty()) break;
        }
    }
    if (!s.empty()) return false;
    if (i < 16) {
        if (ellipsis < 0) return false;
        int n = 16 - i;
        for (int j = i - 1; j >= ellipsis; --j) ip[j + n] = ip[j];
        for (int j = ellipsis + n - 1; j >= ellipsis; --j) ip[j] = 0;
    } else if (ellipsis >= 0) {
        return false;
    }
    return true;
}

// ---- acl.go helpers -------------------------------------------------------

void wrap(ParseError &err, int code, const std::string &msg) {
    err.code = code;
    err.message = msg;
}

// parseL4Port, acl.go:357-383.
bool parse_l4_port(std::string port, uint16_t &mn, uint16_t &mx, bool &valid, ParseError &err) {
    valid = true;
    if (port == "ANY" || port == "0:65535") {
        mn = 0; mx = 65535; valid = false;
        return true;
    }
    if (port.find(':') == std::string::npos) port = port + ":" + port;
    size_t colon = port.find(':');
    std::string a = port.substr(0, colon), b = port.substr(colon + 1);  // SplitN(..., 2)
    uint64_t lo = 0, hi = 0;
    bool okLo = go_parse_uint10(a, 16, lo), okHi = go_parse_uint10(b, 16, hi);
    if (!okLo || !okHi) {
        wrap(err, NFFACL_ERR_INCORRECT_ARG_IN_RULES,
             "Incorrect request: cannot parse Min and Max port values in " + port);
        return false;
    }
    if (lo > hi) {
        wrap(err, NFFACL_ERR_INCORRECT_ARG_IN_RULES,
             "Incorrect request: minPort > maxPort, port: " + port);
        return false;
    }
    mn = static_cast<uint16_t>(lo);
    mx = static_cast<uint16_t>(hi);
    return true;
}

// parseRuleResult, acl.go:385-398.
bool parse_rule_result(const std::string &rule, uint32_t &out, ParseError &err) {
    if (rule == "Accept" || rule == "true") { out = 1; return true; }
    if (rule == "Reject" || rule == "false") { out = 0; return true; }
    uint64_t v = 0;
    if (!go_parse_uint10(rule, 32, v)) {
        wrap(err, NFFACL_ERR_INCORRECT_RULE, "Incorrect rule: " + rule);
        return false;
    }
    out = static_cast<uint32_t>(v);
    return true;
}

// Parsed address field: len 0 (ANY), 4 or 16, network address + mask.
struct Addr {
    int len = 0;
    uint8_t ip[16] = {0};
    uint8_t mask[16] = {0};
};

bool parse_addr_field(const std::string &s, Addr &a, ParseError &err) {
    if (s == "ANY") { a.len = 0; return true; }
    std::vector<uint8_t> ip, mask;
    if (!go_parse_cidr(s, ip, mask)) {
        // Reference: nil *IPNet dereference (acl.go:275-282).
        wrap(err, NFFACL_ERR_INCORRECT_ARG_IN_RULES, "Incorrect address (invalid CIDR): " + s);
        return false;
    }
    a.len = static_cast<int>(ip.size());
    std::memcpy(a.ip, ip.data(), ip.size());
    std::memcpy(a.mask, mask.data(), mask.size());
    return true;
}

uint32_t le32(const uint8_t *b) {  // binary.LittleEndian.Uint32, acl.go:401
    return uint32_t(b[0]) | uint32_t(b[1]) << 8 | uint32_t(b[2]) << 16 | uint32_t(b[3]) << 24;
}

}  // namespace

// ---- exported helpers -------------------------------------------------------

std::vector<std::string> go_fields(const std::string &line) {
    std::vector<std::string> out;
    size_t i = 0, start = 0;
    bool in_field = false;
    while (i < line.size()) {
        uint32_t r;
        int w = decode_rune(line, i, r);
        if (go_is_space(r)) {
            if (in_field) { out.push_back(line.substr(start, i - start)); in_field = false; }
        } else if (!in_field) {
            in_field = true;
            start = i;
        }
        i += static_cast<size_t>(w);
    }
    if (in_field) out.push_back(line.substr(start));
    return out;
}

bool go_parse_uint10(const std::string &s, int bits, uint64_t &out) {
    if (s.empty()) return false;
    const uint64_t max_val = (bits >= 64) ? ~0ull : ((1ull << bits) - 1);
    uint64_t n = 0;
    for (char ch : s) {
        if (ch < '0' || ch > '9') return false;  // letters are digits >= base 10 -> syntax error
        uint64_t d = static_cast<uint64_t>(ch - '0');
        if (n > (max_val - d) / 10) return false;  // range error
        n = n * 10 + d;
    }
    out = n;
    return true;
}

bool go_parse_cidr(const std::string &s, std::vector<uint8_t> &ip, std::vector<uint8_t> &mask) {
    size_t slash = s.find('/');
    if (slash == std::string::npos) return false;
    std::string addr = s.substr(0, slash), m = s.substr(slash + 1);
    int iplen = 4;
    uint8_t full[16];
    uint8_t v4[4];
    bool is4 = go_parse_ipv4(addr, v4);
    if (!is4) {
        iplen = 16;
        if (!go_parse_ipv6(addr, full)) return false;
    }
    int n; size_t used; bool ok;
    go_dtoi(m, 0, n, used, ok);
    if (!ok || used != m.size() || n < 0 || n > 8 * iplen) return false;
    mask.assign(static_cast<size_t>(iplen), 0);
    for (int b = 0; b < n; ++b) mask[static_cast<size_t>(b / 8)] |= static_cast<uint8_t>(0x80u >> (b % 8));
    ip.assign(static_cast<size_t>(iplen), 0);
    // IP.Mask: a dotted-quad parses to a v4-in-v6 16-byte IP that Mask() cuts
    // back to 4 bytes against the 4-byte mask; IPv6 syntax stays 16 bytes.
    const uint8_t *src = is4 ? v4 : full;
    for (int k = 0; k < iplen; ++k) ip[static_cast<size_t>(k)] = src[k] & mask[static_cast<size_t>(k)];
    return true;
}

bool raw_l3_parse(const std::vector<RawL3Rule> &raw, nffacl_rules &out, ParseError &err) {
    out.ip4.reserve(out.ip4.size() + raw.size());
    for (const RawL3Rule &r : raw) {
        nffacl_l4 l4{};
        // L4 ID, acl.go:240-258
        const std::string &id = r.id;
        if (id == "ANY") {
            l4.id = 0; l4.id_mask = 0;
        } else if (id == "tcp" || id == "TCP" || id == "Tcp" || id == "0x06" || id == "6") {
            l4.id = 6; l4.id_mask = 0xff;
        } else if (id == "udp" || id == "UDP" || id == "Udp" || id == "0x11" || id == "17") {
            l4.id = 17; l4.id_mask = 0xff;
        } else if (id == "icmp" || id == "ICMP" || id == "Icmp" || id == "0x01" || id == "1") {
            l4.id = 1; l4.id_mask = 0xff;
            if (r.src_port != "ANY" || r.dst_port != "ANY") {
                wrap(err, NFFACL_ERR_INCORRECT_ARG_IN_RULES,
                     "Incorrect request: for ICMP rule Source port and Destination port should be ANY");
                return false;
            }
        } else {
            wrap(err, NFFACL_ERR_INCORRECT_ARG_IN_RULES, "Incorrect  L4 protocol ID: " + id);
            return false;
        }
        // ports, acl.go:261-269
        bool vs = false, vd = false;
        if (!parse_l4_port(r.src_port, l4.src_port_min, l4.src_port_max, vs, err)) return false;
        if (!parse_l4_port(r.dst_port, l4.dst_port_min, l4.dst_port_max, vd, err)) return false;
        l4.valid = (vs || vd) ? 1 : 0;

        // addresses, acl.go:272-283
        Addr src, dst;
        if (!parse_addr_field(r.src_addr, src, err)) return false;
        if (!parse_addr_field(r.dst_addr, dst, err)) return false;

        uint32_t outnum = 0;
        auto push4 = [&](const Addr *s, const Addr *d) {
            nffacl_rule4 x{};
            x.output_number = outnum;
            if (s) { x.src_addr = le32(s->ip); x.src_mask = le32(s->mask); }
            if (d) { x.dst_addr = le32(d->ip); x.dst_mask = le32(d->mask); }
            x.l4 = l4;
            out.ip4.push_back(x);
        };
        auto push6 = [&](const Addr *s, const Addr *d) {
            nffacl_rule6 x{};
            x.output_number = outnum;
            if (s) { std::memcpy(x.src_addr, s->ip, 16); std::memcpy(x.src_mask, s->mask, 16); }
            if (d) { std::memcpy(x.dst_addr, d->ip, 16); std::memcpy(x.dst_mask, d->mask, 16); }
            x.l4 = l4;
            out.ip6.push_back(x);
        };
        static const char *kMix = "Incorrect request: IPv4 + IPv6 in one rule";
        // family dispatch, acl.go:285-352
        if (src.len == 0) {
            if (dst.len == 0) {
                if (!parse_rule_result(r.output_number, outnum, err)) return false;
                push4(nullptr, nullptr);
                if (!parse_rule_result(r.output_number, outnum, err)) return false;
                push6(nullptr, nullptr);
            } else if (dst.len == 4) {
                if (!parse_rule_result(r.output_number, outnum, err)) return false;
                push4(nullptr, &dst);
            } else {
                if (!parse_rule_result(r.output_number, outnum, err)) return false;
                push6(nullptr, &dst);
            }
        } else if (src.len == 4) {
            if (dst.len == 16) { wrap(err, NFFACL_ERR_INCORRECT_ARG_IN_RULES, kMix); return false; }
            if (!parse_rule_result(r.output_number, outnum, err)) return false;
            push4(&src, dst.len == 4 ? &dst : nullptr);
        } else {
            if (dst.len == 4) { wrap(err, NFFACL_ERR_INCORRECT_ARG_IN_RULES, kMix); return false; }
            if (!parse_rule_result(r.output_number, outnum, err)) return false;
            push6(&src, dst.len == 16 ? &dst : nullptr);
        }
    }
    return true;
}

namespace {

// bufio.Scanner + ScanLines (64 KiB max token) + strings.Fields, the loop both
// text loaders share (acl.go:97-112 for L2, 156-173 for L3): comment and empty
// lines skipped, a missing last field defaults to "false", any other field
// count is ParseRuleErr.
bool scan_table(const char *data, size_t len, size_t nfields, const char *incomplete,
                std::vector<std::vector<std::string>> &rows, ParseError &err) {
    constexpr size_t kMaxToken = 64 * 1024;
    size_t pos = 0;
    while (pos < len) {
        const void *nl = std::memchr(data + pos, '\n', len - pos);
        size_t end = nl ? static_cast<size_t>(static_cast<const char *>(nl) - data) : len;
        // A line (CR included) of >= 64 KiB never fits the scanner buffer
        // together with its terminator / the EOF probe -> bufio.ErrTooLong.
        if (end - pos >= kMaxToken) {
            wrap(err, NFFACL_ERR_FILE, "file error during rules parsing: bufio.Scanner: token too long");
            return false;
        }
        std::string line(data + pos, end - pos);
        if (!line.empty() && line.back() == '\r') line.pop_back();  // dropCR
        pos = nl ? end + 1 : len;
        if (line.empty() || line[0] == '#') continue;
        std::vector<std::string> f = go_fields(line);
        if (f.size() == nfields - 1) {
            f.push_back("false");
        } else if (f.size() != nfields) {
            wrap(err, NFFACL_ERR_PARSE_RULE, incomplete);
            return false;
        }
        rows.push_back(std::move(f));
    }
    return true;
}

}  // namespace

bool parse_text_table(const char *data, size_t len, nffacl_rules &out, ParseError &err) {
    std::vector<std::vector<std::string>> rows;
    if (!scan_table(data, len, 6, "Incomplete 5-tuple for rule parsing", rows, err)) return false;
    std::vector<RawL3Rule> raw;
    raw.reserve(rows.size());
    for (auto &f : rows) raw.push_back(RawL3Rule{f[0], f[1], f[2], f[3], f[4], f[5]});
    return raw_l3_parse(raw, out, err);
}

// ---- L2 (acl.go:88-117, 356-383) ----------------------------------------------

// go1.13 net.ParseMAC: 6-, 8- or 20-byte addresses in colon, dash or dotted
// (Cisco) notation.
bool go_parse_mac(const std::string &s, std::vector<uint8_t> &hw) {
    auto xtoi2 = [&](size_t x, size_t lim, char e, uint8_t &b) -> bool {
        // xtoi2(s[x:lim], e): two hex digits, then (if more bytes follow) e.
        if (lim - x > 2 && s[x + 2] != e) return false;
        const std::string two = s.substr(x, 2);
        int n; size_t used; bool ok;
        go_xtoi(two, 0, n, used, ok);
        b = static_cast<uint8_t>(n);
        return ok && used == 2;
    };
    hw.clear();
    const size_t L = s.size();
    if (L < 14) return false;
    if (s[2] == ':' || s[2] == '-') {
        if ((L + 1) % 3 != 0) return false;
        const size_t n = (L + 1) / 3;
        if (n != 6 && n != 8 && n != 20) return false;
        hw.resize(n);
        for (size_t i = 0, x = 0; i < n; ++i, x += 3)
            if (!xtoi2(x, L, s[2], hw[i])) return false;
    } else if (s[4] == '.') {
        if ((L + 1) % 5 != 0) return false;
        const size_t n = 2 * (L + 1) / 5;
        if (n != 6 && n != 8 && n != 20) return false;
        hw.resize(n);
        for (size_t i = 0, x = 0; i < n; i += 2, x += 5) {
            if (!xtoi2(x, x + 2, 0, hw[i])) return false;
            if (!xtoi2(x + 2, L, s[4], hw[i + 1])) return false;
        }
    } else {
        return false;
    }
    return true;
}

bool raw_l2_parse(const std::vector<RawL2Rule> &raw, nffacl_l2rules &out, ParseError &err) {
    std::vector<nffacl_l2_rule> eth(raw.size());
    for (size_t i = 0; i < raw.size(); ++i) {
        const RawL2Rule &r = raw[i];
        nffacl_l2_rule &e = eth[i];
        e = nffacl_l2_rule{};
        if (!parse_rule_result(r.rule, e.output_number, err)) return false;
        std::vector<uint8_t> hw;
        if (r.source != "ANY") {
            e.saddr_not_any = 1;
            if (!go_parse_mac(r.source, hw)) {
                wrap(err, NFFACL_ERR_INCORRECT_ARG_IN_RULES, "Incorrect source MAC: " + r.source);
                return false;
            }
            std::memcpy(e.saddr, hw.data(), 6);  // copy(SAddr[:], t): first 6 bytes
        }
        if (r.destination != "ANY") {
            e.daddr_not_any = 1;
            if (!go_parse_mac(r.destination, hw)) {
                wrap(err, NFFACL_ERR_INCORRECT_ARG_IN_RULES, "Incorrect destination MAC: " + r.destination);
                return false;
            }
            std::memcpy(e.daddr, hw.data(), 6);
        }
        const std::string &id = r.id;
        if (id == "ANY") {
            e.id = 0; e.id_mask = 0;
        } else if (id == "ipv4" || id == "Ipv4" || id == "IPv4" || id == "IPV4" || id == "0x0800") {
            e.id = 0x0800; e.id_mask = 0xffff;
        } else if (id == "ipv6" || id == "Ipv6" || id == "IPv6" || id == "IPV6" || id == "0x86dd") {
            e.id = 0x86dd; e.id_mask = 0xffff;
        } else if (id == "arp" || id == "Arp" || id == "ARP" || id == "0x0806") {
            e.id = 0x0806; e.id_mask = 0xffff;
        } else {
            wrap(err, NFFACL_ERR_INCORRECT_ARG_IN_RULES, "Incorrect  L3 protocol ID: " + id);
            return false;
        }
    }
    out.eth.insert(out.eth.end(), eth.begin(), eth.end());
    return true;
}

bool parse_l2_text_table(const char *data, size_t len, nffacl_l2rules &out, ParseError &err) {
    std::vector<std::vector<std::string>> rows;
    if (!scan_table(data, len, 4, "Incomplete 3-tuple for rule parsing", rows, err)) return false;
    std::vector<RawL2Rule> raw;
    raw.reserve(rows.size());
    // text column order Source Destination ID Rule (acl.go:108-109)
    for (auto &f : rows) raw.push_back(RawL2Rule{f[3], f[0], f[1], f[2]});
    return raw_l2_parse(raw, out, err);
}

}  // namespace nffacl

// ---- GetL3ACLFromJSON (acl.go:121-134) ------------------------------------
//
// encoding/json semantics for `json.Unmarshal(f, &rawL3Rules{})`:
//  * RFC 8259 syntax, one top-level value, surrounding whitespace only;
//  * object keys match the exported fields case-insensitively; the last
//    matching key wins; unknown keys are ignored;
//  * null leaves the destination untouched (a null array element appends a
//    zero rawL3Rule); a value of the wrong JSON type is an UnmarshalTypeError,
//    reported once decoding has finished;
//  * strings: standard escapes, surrogate pairs, lone surrogates and invalid
//    UTF-8 become U+FFFD.
namespace nffacl {
namespace {

struct JsonCursor {
    const char *p, *end;
    bool type_error = false;
    std::string syntax;  // first syntax error

    bool fail(const char *why) {
        if (syntax.empty()) syntax = why;
        return false;
    }
    void ws() {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
    }
    static void put_utf8(std::string &o, uint32_t r) {
        if (r < 0x80) o += static_cast<char>(r);
        else if (r < 0x800) { o += static_cast<char>(0xC0 | (r >> 6)); o += static_cast<char>(0x80 | (r & 0x3F)); }
        else if (r < 0x10000) {
            o += static_cast<char>(0xE0 | (r >> 12)); o += static_cast<char>(0x80 | ((r >> 6) & 0x3F));
            o += static_cast<char>(0x80 | (r & 0x3F));
        } else {
            o += static_cast<char>(0xF0 | (r >> 18)); o += static_cast<char>(0x80 | ((r >> 12) & 0x3F));
            o += static_cast<char>(0x80 | ((r >> 6) & 0x3F)); o += static_cast<char>(0x80 | (r & 0x3F));
        }
    }
    int hex4(const char *q) {
        int v = 0;
        for (int i = 0; i < 4; ++i) {
            char c = q[i];
            int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10
                  : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
            if (d < 0) return -1;
            v = v * 16 + d;
        }
        return v;
    }
    bool string(std::string *out) {  // at '"'
        ++p;
        std::string raw;
        while (true) {
            if (p >= end) return fail("unexpected end of JSON input");
            unsigned char c = static_cast<unsigned char>(*p);
            if (c == '"') { ++p; break; }
            if (c < 0x20) return fail("invalid character in string literal");
            if (c != '\\') { raw += static_cast<char>(c); ++p; continue; }
            ++p;
            if (p >= end) return fail("unexpected end of JSON input");
            char e = *p++;
            switch (e) {
            case '"': raw += '"'; break;
            case '\\': raw += '\\'; break;
            case '/': raw += '/'; break;
            case 'b': raw += '\b'; break;
            case 'f': raw += '\f'; break;
            case 'n': raw += '\n'; break;
            case 'r': raw += '\r'; break;
            case 't': raw += '\t'; break;
            case 'u': {
                if (end - p < 4) return fail("invalid \\u escape");
                int v = hex4(p);
                if (v < 0) return fail("invalid \\u escape");
                p += 4;
                uint32_t r = static_cast<uint32_t>(v);
                if (r >= 0xD800 && r < 0xDC00) {
                    // high surrogate: combine with a following \uDC00-\uDFFF
                    if (end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                        int lo = hex4(p + 2);
                        if (lo >= 0xDC00 && lo < 0xE000) {
                            r = 0x10000 + ((r - 0xD800) << 10) + (static_cast<uint32_t>(lo) - 0xDC00);
                            p += 6;
                        } else {
                            r = 0xFFFD;
                        }
                    } else {
                        r = 0xFFFD;
                    }
                } else if (r >= 0xDC00 && r < 0xE000) {
                    r = 0xFFFD;
                }
                put_utf8(raw, r);
                break;
            }
            default: return fail("invalid escape in string literal");
            }
        }
        if (out) {
            // invalid UTF-8 -> U+FFFD per byte (utf8.DecodeRune)
            out->clear();
            size_t i = 0;
            while (i < raw.size()) {
                uint32_t r;
                int w = decode_rune(raw, i, r);
                if (r == 0xFFFD && w == 1 && static_cast<unsigned char>(raw[i]) >= 0x80) put_utf8(*out, 0xFFFD);
                else out->append(raw, i, static_cast<size_t>(w));
                i += static_cast<size_t>(w);
            }
        }
        return true;
    }
    bool literal(const char *lit) {
        size_t n = std::strlen(lit);
        if (static_cast<size_t>(end - p) < n || std::memcmp(p, lit, n) != 0) return fail("invalid literal");
        p += n;
        return true;
    }
    bool number() {
        const char *q = p;
        if (q < end && *q == '-') ++q;
        if (q >= end) return fail("invalid number");
        if (*q == '0') ++q;
        else if (*q >= '1' && *q <= '9') { while (q < end && *q >= '0' && *q <= '9') ++q; }
        else return fail("invalid number");
        if (q < end && *q == '.') {
            ++q;
            if (q >= end || *q < '0' || *q > '9') return fail("invalid number");
            while (q < end && *q >= '0' && *q <= '9') ++q;
        }
        if (q < end && (*q == 'e' || *q == 'E')) {
            ++q;
            if (q < end && (*q == '+' || *q == '-')) ++q;
            if (q >= end || *q < '0' || *q > '9') return fail("invalid number");
            while (q < end && *q >= '0' && *q <= '9') ++q;
        }
        p = q;
        return true;
    }
    // Skip any value (type already known to be unwanted by the caller).
    bool skip() {
        ws();
        if (p >= end) return fail("unexpected end of JSON input");
        char c = *p;
        if (c == '"') return string(nullptr);
        if (c == '{') return object([&](const std::string &) { return skip(); });
        if (c == '[') return array([&]() { return skip(); });
        if (c == 't') return literal("true");
        if (c == 'f') return literal("false");
        if (c == 'n') return literal("null");
        return number();
    }
    template <class OnKey>
    bool object(OnKey on_key) {  // at '{'
        ++p;
        ws();
        if (p < end && *p == '}') { ++p; return true; }
        while (true) {
            ws();
            if (p >= end || *p != '"') return fail("expected object key");
            std::string key;
            if (!string(&key)) return false;
            ws();
            if (p >= end || *p != ':') return fail("expected ':'");
            ++p;
            if (!on_key(key)) return false;
            ws();
            if (p < end && *p == ',') { ++p; continue; }
            if (p < end && *p == '}') { ++p; return true; }
            return fail("expected ',' or '}'");
        }
    }
    template <class OnElem>
    bool array(OnElem on_elem) {  // at '['
        ++p;
        ws();
        if (p < end && *p == ']') { ++p; return true; }
        while (true) {
            if (!on_elem()) return false;
            ws();
            if (p < end && *p == ',') { ++p; continue; }
            if (p < end && *p == ']') { ++p; return true; }
            return fail("expected ',' or ']'");
        }
    }
    // Decode a value into a string field: string sets, null keeps, else type error.
    bool string_field(std::string &dst) {
        ws();
        if (p >= end) return fail("unexpected end of JSON input");
        if (*p == '"') return string(&dst);
        if (*p == 'n') return literal("null");
        type_error = true;
        return skip();
    }
};

// encoding/json's key matching for a struct field name (go1.13 fold.go):
// ASCII case folding, plus — for names containing s/S or k/K, which select
// equalFoldRight — U+017F (long s) matching s and U+212A (Kelvin) matching k.
bool json_key_eq(const std::string &key, const char *field) {
    size_t t = 0;
    for (const char *f = field; *f; ++f) {
        if (t >= key.size()) return false;
        const unsigned char tb = static_cast<unsigned char>(key[t]);
        const char lf = (*f >= 'A' && *f <= 'Z') ? static_cast<char>(*f - 'A' + 'a') : *f;
        if (tb < 0x80) {
            const char lt = (tb >= 'A' && tb <= 'Z') ? static_cast<char>(tb - 'A' + 'a') : static_cast<char>(tb);
            const bool letter = lf >= 'a' && lf <= 'z';
            if (letter ? lt != lf : static_cast<char>(tb) != *f) return false;
            ++t;
            continue;
        }
        if (lf == 's' && key.compare(t, 2, "\xC5\xBF") == 0) { t += 2; continue; }
        if (lf == 'k' && key.compare(t, 3, "\xE2\x84\xAA") == 0) { t += 3; continue; }
        return false;
    }
    return t == key.size();
}

// json.Unmarshal of {"<top>": [ {<fields>: string, ...}, ... ]} into a slice
// of records of string fields (rawL2Rules acl.go:44-53, rawL3Rules :55-66).
bool parse_json_records(const char *data, size_t len, const char *top, const char *const *fields, size_t nf,
                        const char *type_name, std::vector<std::vector<std::string>> &rows, ParseError &err) {
    JsonCursor c{data, data + len, false, std::string()};
    bool ok = true;
    c.ws();
    if (c.p >= c.end) {
        ok = c.fail("unexpected end of JSON input");
    } else if (*c.p == 'n') {
        ok = c.literal("null");
    } else if (*c.p == '{') {
        ok = c.object([&](const std::string &key) -> bool {
            if (!json_key_eq(key, top)) return c.skip();
            c.ws();
            if (c.p < c.end && *c.p == 'n') return c.literal("null");
            if (c.p >= c.end || *c.p != '[') {
                c.type_error = true;
                return c.skip();
            }
            rows.clear();  // a later matching key replaces the slice
            return c.array([&]() -> bool {
                std::vector<std::string> r(nf);
                c.ws();
                bool elem_ok;
                if (c.p < c.end && *c.p == '{') {
                    elem_ok = c.object([&](const std::string &k) -> bool {
                        for (size_t i = 0; i < nf; ++i)
                            if (json_key_eq(k, fields[i])) return c.string_field(r[i]);
                        return c.skip();
                    });
                } else if (c.p < c.end && *c.p == 'n') {
                    elem_ok = c.literal("null");
                } else {
                    c.type_error = true;
                    elem_ok = c.skip();
                }
                rows.push_back(std::move(r));
                return elem_ok;
            });
        });
    } else {
        c.type_error = true;
        ok = c.skip();
    }
    if (ok) {
        c.ws();
        if (c.p != c.end) ok = c.fail("invalid character after top-level value");
    }
    if (!ok) {
        err.code = NFFACL_ERR_PARSE_RULE_JSON;
        err.message = "JSON error during rules parsing: " + c.syntax;
        return false;
    }
    if (c.type_error) {
        err.code = NFFACL_ERR_PARSE_RULE_JSON;
        err.message = std::string("JSON error during rules parsing: json: cannot unmarshal value into ") + type_name;
        return false;
    }
    return true;
}

}  // namespace

bool parse_json(const char *data, size_t len, nffacl_rules &out, ParseError &err) {
    static const char *const kFields[] = {"SrcAddr", "DstAddr", "ID", "SrcPort", "DstPort", "OutputNumber"};
    std::vector<std::vector<std::string>> rows;
    if (!parse_json_records(data, len, "L3Rules", kFields, 6, "rawL3Rules", rows, err)) return false;
    std::vector<RawL3Rule> raw;
    raw.reserve(rows.size());
    for (auto &f : rows) raw.push_back(RawL3Rule{f[0], f[1], f[2], f[3], f[4], f[5]});
    return raw_l3_parse(raw, out, err);
}

bool parse_l2_json(const char *data, size_t len, nffacl_l2rules &out, ParseError &err) {
    static const char *const kFields[] = {"Rule", "Source", "Destination", "ID"};
    std::vector<std::vector<std::string>> rows;
    if (!parse_json_records(data, len, "L2Rules", kFields, 4, "rawL2Rules", rows, err)) return false;
    std::vector<RawL2Rule> raw;
    raw.reserve(rows.size());
    for (auto &f : rows) raw.push_back(RawL2Rule{f[0], f[1], f[2], f[3]});
    return raw_l2_parse(raw, out, err);
}

}  // namespace nffacl
