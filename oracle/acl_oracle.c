/*
 * acl_oracle.c — TEST INFRASTRUCTURE ONLY.  Not part of libnffacl.
 *
 * A deliberately literal CPU restatement of nff-go's per-packet ACL verdict,
 * used as the parity checker for the HIP path (tests/, __graft_entry__.smoke)
 * and, timed, as the CPU baseline of bench.py ("port" of the reference
 * algorithm — the Go reference itself cannot be built here: no Go toolchain,
 * DPDK un-vendored).  Nothing in the product links this.
 *
 * Followed line by line:
 *   (*Packet).l3ACL        packet/acl.go:522-565   (first match, per family)
 *   (*Packet).l4ACL        packet/acl.go:508-520   (no protocol check)
 *   ParseAllKnownL3        packet/packet.go:353-363
 *   ParseL3                packet/packet.go:233-235   (L3 = Ether + 14)
 *   GetIPv4 / GetIPv6      packet/packet.go:238-243, 264-269
 *   ParseL4ForIPv4         packet/packet.go:278-280   (L4 = L3 + IHL*4)
 *   ParseL4ForIPv6         packet/packet.go:283-285   (L4 = L3 + 40)
 *   SwapBytesUint16        packet/packet.go:713-715
 *   IPv4Hdr / IPv6Hdr / UDPHdr layouts packet/packet.go:107-170
 *   types.IPv4Address = LE uint32 of wire bytes   types/ipv4.go:13-28
 *   (*Packet).l2ACL        packet/acl.go:478-491   (L2 ACL, §8f next row)
 *   ParseAllKnownL3CheckVLAN packet/vlan.go:104-117 (+ GetEtherType :53-62,
 *                          ParseL3CheckVLAN :66-75) — the VLAN-aware parse the
 *                          NFFACL_PARSE_VLAN flag substitutes for ParseAllKnownL3
 *   EtherHdr layout        packet/packet.go:96-100 (DAddr, SAddr, EtherType)
 *
 * Packet memory convention: the reference reads raw mbuf memory; here a packet
 * is `len` bytes and any byte at index >= len reads as 0.
 *
 * Parity pinning: checked against every match KAT of
 * packet/acl_internal_test.go (:501-1141, transcribed by
 * tests/golden/make_kats.py) and the header-parse KAT frames of
 * packet/packet_test.go:22-267 (tests/test_oracle.py).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Same field meaning as the reference's l4Rules / l3Rules4 / l3Rules6
 * (acl.go:423-449); byte layout shared with tests/ via numpy dtypes. */
typedef struct {
    uint8_t ID, IDMask, valid, pad;
    uint16_t SrcPortMin, SrcPortMax, DstPortMin, DstPortMax;
} orc_l4;

typedef struct {
    uint32_t OutputNumber;
    uint32_t SrcAddr, DstAddr, SrcMask, DstMask; /* types.IPv4Address */
    orc_l4 L4;
} orc_rule4;

typedef struct {
    uint32_t OutputNumber;
    uint8_t SrcAddr[16], DstAddr[16], SrcMask[16], DstMask[16];
    orc_l4 L4;
} orc_rule6;

/* l2Rules, acl.go:413-421 (byte layout shared with tests/ via numpy). */
typedef struct {
    uint32_t OutputNumber;
    uint8_t DAddrNotAny, SAddrNotAny;
    uint8_t DAddr[6], SAddr[6];
    uint16_t IDMask, ID;
    uint16_t pad;
} orc_l2rule;

/* A packet: its bytes and the parse "pointers" (offsets) of packet.Packet. */
typedef struct {
    const uint8_t *data;
    uint32_t len;
    uint32_t L3, L4; /* offsets from Ether */
} orc_packet;

static uint8_t at(const orc_packet *p, uint32_t i) { return i < p->len ? p->data[i] : 0; }

/* Little-endian load of a Go uint16/uint32 header field at byte offset. */
static uint16_t u16le(const orc_packet *p, uint32_t off) {
    return (uint16_t)(at(p, off) | (uint16_t)at(p, off + 1) << 8);
}
static uint32_t u32le(const orc_packet *p, uint32_t off) {
    return (uint32_t)at(p, off) | (uint32_t)at(p, off + 1) << 8 | (uint32_t)at(p, off + 2) << 16 |
           (uint32_t)at(p, off + 3) << 24;
}

static uint16_t SwapBytesUint16(uint16_t x) { return (uint16_t)(x << 8 | x >> 8); }

enum { EtherLen = 14, VLANLen = 4, IPv6Len = 40, SwapIPV4Number = 0x0008, SwapIPV6Number = 0xdd86,
       SwapVLANNumber = 0x0081 };

/* ParseAllKnownL3: returns 4, 6 or 0 */
static int ParseAllKnownL3(orc_packet *p) {
    p->L3 = EtherLen;                          /* ParseL3 */
    uint16_t et = u16le(p, 12);                /* Ether.EtherType */
    if (et == SwapIPV4Number) return 4;        /* GetIPv4 */
    if (et == SwapIPV6Number) return 6;        /* GetIPv6 */
    return 0;                                  /* ARP or unknown: no ACL verdict */
}

/* ParseAllKnownL3CheckVLAN: one 802.1Q tag moves L3 by VLANLen and the
 * EtherType compared is the tag's (GetEtherType). */
static int ParseAllKnownL3CheckVLAN(orc_packet *p) {
    uint16_t et = u16le(p, 12);
    if (et == SwapVLANNumber) {               /* ParseL3CheckVLAN */
        p->L3 = EtherLen + VLANLen;
        et = u16le(p, EtherLen + 2);          /* VLANHdr.EtherType */
    } else {
        p->L3 = EtherLen;
    }
    if (et == SwapIPV4Number) return 4;
    if (et == SwapIPV6Number) return 6;
    return 0;
}

static void ParseL4ForIPv4(orc_packet *p) {
    uint8_t VersionIhl = at(p, p->L3 + 0);
    p->L4 = p->L3 + (uint32_t)((VersionIhl & 0x0f) << 2);
}

static void ParseL4ForIPv6(orc_packet *p) { p->L4 = p->L3 + IPv6Len; }

static int l4ACL(const orc_packet *p, const orc_l4 *L4) {
    uint16_t srcPort = SwapBytesUint16(u16le(p, p->L4 + 0)); /* UDPHdr.SrcPort */
    if (srcPort < L4->SrcPortMin || srcPort > L4->SrcPortMax) return 0;
    uint16_t dstPort = SwapBytesUint16(u16le(p, p->L4 + 2)); /* UDPHdr.DstPort */
    if (dstPort < L4->DstPortMin || dstPort > L4->DstPortMax) return 0;
    return 1;
}

/* l3ACL.  *which (if non-NULL) receives the index of the matching rule in its
 * family slice, or -1 when no rule matches. */
enum { ORC_PARSE_VLAN = 1 };

uint32_t oracle_l3acl_flags(const uint8_t *data, uint32_t len, const orc_rule4 *ip4, size_t n4,
                            const orc_rule6 *ip6, size_t n6, int64_t *which, uint32_t flags) {
    orc_packet pkt = {data, len, 0, 0};
    if (which) *which = -1;
    int fam = (flags & ORC_PARSE_VLAN) ? ParseAllKnownL3CheckVLAN(&pkt) : ParseAllKnownL3(&pkt);
    if (fam == 4) {
        uint32_t SrcAddr = u32le(&pkt, pkt.L3 + 12);
        uint32_t DstAddr = u32le(&pkt, pkt.L3 + 16);
        uint8_t NextProtoID = at(&pkt, pkt.L3 + 9);
        for (size_t i = 0; i < n4; i++) {
            const orc_rule4 *rule = &ip4[i];
            if (((rule->SrcAddr ^ SrcAddr) & rule->SrcMask) != 0) continue;
            if (((rule->DstAddr ^ DstAddr) & rule->DstMask) != 0) continue;
            if (((rule->L4.ID ^ NextProtoID) & rule->L4.IDMask) != 0) continue;
            if (rule->L4.valid) {
                ParseL4ForIPv4(&pkt);
                if (!l4ACL(&pkt, &rule->L4)) continue;
            }
            if (which) *which = (int64_t)i;
            return rule->OutputNumber;
        }
    } else if (fam == 6) {
        uint8_t Proto = at(&pkt, pkt.L3 + 6);
        for (size_t i = 0; i < n6; i++) {
            const orc_rule6 *rule = &ip6[i];
            int skip = 0;
            for (int b = 0; b < 16; b++) {
                if (((rule->SrcAddr[b] ^ at(&pkt, pkt.L3 + 8 + b)) & rule->SrcMask[b]) != 0 ||
                    ((rule->DstAddr[b] ^ at(&pkt, pkt.L3 + 24 + b)) & rule->DstMask[b]) != 0) {
                    skip = 1;
                    break;
                }
            }
            if (skip) continue;
            if (((rule->L4.ID ^ Proto) & rule->L4.IDMask) != 0) continue;
            ParseL4ForIPv6(&pkt);
            if (!l4ACL(&pkt, &rule->L4)) continue;
            if (which) *which = (int64_t)i;
            return rule->OutputNumber;
        }
    } else {
        return 0;
    }
    return 0;
}

uint32_t oracle_l3acl_which(const uint8_t *data, uint32_t len, const orc_rule4 *ip4, size_t n4,
                            const orc_rule6 *ip6, size_t n6, int64_t *which) {
    return oracle_l3acl_flags(data, len, ip4, n4, ip6, n6, which, 0);
}

uint32_t oracle_l3acl(const uint8_t *data, uint32_t len, const orc_rule4 *ip4, size_t n4,
                      const orc_rule6 *ip6, size_t n6) {
    return oracle_l3acl_which(data, len, ip4, n4, ip6, n6, NULL);
}

/* ---- batch drivers (std::thread-like shards over pthreads) ---------------- */

/* (*Packet).l2ACL, acl.go:478-491: Ether.DAddr = bytes 0..5, SAddr = 6..11,
 * EtherType = LE u16 of bytes 12..13 (compared after SwapBytesUint16). */
uint32_t oracle_l2acl(const uint8_t *data, uint32_t len, const orc_l2rule *eth, size_t n) {
    orc_packet p = {data, len, 0, 0};
    uint8_t DAddr[6], SAddr[6];
    for (int i = 0; i < 6; i++) {
        DAddr[i] = at(&p, (uint32_t)i);
        SAddr[i] = at(&p, (uint32_t)(6 + i));
    }
    const uint16_t EtherType = u16le(&p, 12);
    for (size_t r = 0; r < n; r++) {
        const orc_l2rule *rule = &eth[r];
        if (rule->SAddrNotAny && memcmp(rule->SAddr, SAddr, 6) != 0) continue;
        if (rule->DAddrNotAny && memcmp(rule->DAddr, DAddr, 6) != 0) continue;
        if (((rule->ID ^ SwapBytesUint16(EtherType)) & rule->IDMask) != 0) continue;
        return rule->OutputNumber;
    }
    return 0;
}

typedef struct {
    const uint8_t *base;
    const uint64_t *desc; /* NULL: dense slots */
    uint32_t stride;
    uint64_t first, count;
    const orc_rule4 *ip4;
    size_t n4;
    const orc_rule6 *ip6;
    size_t n6;
    uint32_t *out;
    int64_t *which; /* optional */
    const orc_l2rule *eth; /* non-NULL: L2 ACL instead of L3 */
    size_t neth;
    uint32_t flags;        /* ORC_PARSE_VLAN */
} orc_job;

static void *orc_worker(void *arg) {
    orc_job *j = (orc_job *)arg;
    for (uint64_t i = j->first; i < j->first + j->count; i++) {
        const uint8_t *pkt;
        uint32_t len;
        if (j->desc) {
            pkt = j->base + (j->desc[i] >> 16);
            len = (uint32_t)(j->desc[i] & 0xffff);
        } else {
            pkt = j->base + i * (uint64_t)j->stride;
            len = j->stride;
        }
        j->out[i] = j->eth ? oracle_l2acl(pkt, len, j->eth, j->neth)
                           : oracle_l3acl_flags(pkt, len, j->ip4, j->n4, j->ip6, j->n6,
                                                j->which ? &j->which[i] : NULL, j->flags);
    }
    return NULL;
}

static int orc_run_any(const uint8_t *base, const uint64_t *desc, uint32_t stride, uint64_t n,
                       const orc_rule4 *ip4, size_t n4, const orc_rule6 *ip6, size_t n6,
                       const orc_l2rule *eth, size_t neth, uint32_t *out, int64_t *which, int threads,
                       uint32_t flags) {
    if (threads < 1) threads = 1;
    if ((uint64_t)threads > n) threads = n ? (int)n : 1;
    pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    orc_job *jobs = (orc_job *)calloc((size_t)threads, sizeof(orc_job));
    if (!tid || !jobs) {
        free(tid);
        free(jobs);
        return -1;
    }
    uint64_t per = n / (uint64_t)threads, rem = n % (uint64_t)threads, first = 0;
    for (int t = 0; t < threads; t++) {
        uint64_t cnt = per + ((uint64_t)t < rem ? 1 : 0);
        orc_job j = {base, desc, stride, first, cnt, ip4, n4, ip6, n6, out, which, eth, neth, flags};
        jobs[t] = j;
        first += cnt;
    }
    for (int t = 1; t < threads; t++) pthread_create(&tid[t], NULL, orc_worker, &jobs[t]);
    orc_worker(&jobs[0]);
    for (int t = 1; t < threads; t++) pthread_join(tid[t], NULL);
    free(tid);
    free(jobs);
    return 0;
}

static int orc_run(const uint8_t *base, const uint64_t *desc, uint32_t stride, uint64_t n,
                   const orc_rule4 *ip4, size_t n4, const orc_rule6 *ip6, size_t n6,
                   uint32_t *out, int64_t *which, int threads) {
    return orc_run_any(base, desc, stride, n, ip4, n4, ip6, n6, NULL, 0, out, which, threads, 0);
}

/* Dense slots / packed frames with parse flags (ORC_PARSE_VLAN). */
int oracle_classify_slots_flags(const uint8_t *slots, uint32_t stride, uint64_t n, const orc_rule4 *ip4,
                                size_t n4, const orc_rule6 *ip6, size_t n6, uint32_t *out, int threads,
                                uint32_t flags) {
    return orc_run_any(slots, NULL, stride, n, ip4, n4, ip6, n6, NULL, 0, out, NULL, threads, flags);
}

int oracle_classify_frames_flags(const uint8_t *frames, const uint64_t *desc, uint64_t n, const orc_rule4 *ip4,
                                 size_t n4, const orc_rule6 *ip6, size_t n6, uint32_t *out, int threads,
                                 uint32_t flags) {
    return orc_run_any(frames, desc, 0, n, ip4, n4, ip6, n6, NULL, 0, out, NULL, threads, flags);
}

/* Dense slots: packet i is slots[i*stride .. (i+1)*stride). */
int oracle_classify_slots(const uint8_t *slots, uint32_t stride, uint64_t n, const orc_rule4 *ip4,
                          size_t n4, const orc_rule6 *ip6, size_t n6, uint32_t *out, int threads) {
    return orc_run(slots, NULL, stride, n, ip4, n4, ip6, n6, out, NULL, threads);
}

/* Same, also reporting the matching rule index per packet (-1 = none). */
int oracle_classify_slots_which(const uint8_t *slots, uint32_t stride, uint64_t n,
                                const orc_rule4 *ip4, size_t n4, const orc_rule6 *ip6, size_t n6,
                                uint32_t *out, int64_t *which, int threads) {
    return orc_run(slots, NULL, stride, n, ip4, n4, ip6, n6, out, which, threads);
}

/* Packed frames: frame i at frames + (desc[i] >> 16), length desc[i] & 0xffff. */
int oracle_classify_frames(const uint8_t *frames, const uint64_t *desc, uint64_t n,
                           const orc_rule4 *ip4, size_t n4, const orc_rule6 *ip6, size_t n6,
                           uint32_t *out, int threads) {
    return orc_run(frames, desc, 0, n, ip4, n4, ip6, n6, out, NULL, threads);
}

/* L2 ACL over dense slots / packed frames. */
int oracle_l2_classify_slots(const uint8_t *slots, uint32_t stride, uint64_t n, const orc_l2rule *eth,
                             size_t neth, uint32_t *out, int threads) {
    static const orc_l2rule none;
    return orc_run_any(slots, NULL, stride, n, NULL, 0, NULL, 0, neth ? eth : &none, neth, out, NULL, threads, 0);
}

int oracle_l2_classify_frames(const uint8_t *frames, const uint64_t *desc, uint64_t n, const orc_l2rule *eth,
                              size_t neth, uint32_t *out, int threads) {
    static const orc_l2rule none;
    return orc_run_any(frames, desc, 0, n, NULL, 0, NULL, 0, neth ? eth : &none, neth, out, NULL, threads, 0);
}

int oracle_l2rule_size(void) { return (int)sizeof(orc_l2rule); }
int oracle_rule4_size(void) { return (int)sizeof(orc_rule4); }
int oracle_rule6_size(void) { return (int)sizeof(orc_rule6); }
