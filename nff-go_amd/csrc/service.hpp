// service.hpp — the persistent scalar-call consumer behind nffacl_service_*
// (internal).  See service.hip.
//
// The reference's primary call shape is one packet per call: a
// SetSeparator / SetSplitter user function calling pkt.L3ACLPermit(rules) or
// pkt.L3ACLPort(rules) (flow/flow.go:128, 1795-1797;
// examples/firewall/firewall.go:54-57; examples/tutorial/step08.go:33-35),
// from one OS thread per flow-function clone.  A kernel launch per call costs
// ~20 µs of launch + completion round trip, so this path keeps ONE small
// kernel resident instead: every calling thread owns a 128-byte mailbox in
// mapped pinned host memory, the kernel's waves poll the mailboxes over PCIe,
// classify whatever is complete and write {sequence, port} back to host
// memory, where the caller spins on it.  The kernel exits by itself after an
// idle period, a lifetime cap or a host stop word, and the host re-arms it on
// the next call.
#pragma once

#include <cstdint>

#include "table.hpp"

namespace nffacl {

// ---- mailbox (host memory, one per calling thread) ---------------------------
//
// Eight 16-byte chunks, each written by ONE aligned 16-byte host store and read
// by ONE 16-byte device load, each carrying the request's sequence tag in its
// last dword:
//   chunk c < 7: packet bytes [12c, 12c + 12) (84 bytes; bytes at or past
//                min(len, 80) are 0 — the batcher's 80-byte slot convention)
//   chunk 7:     {desc address lo, desc address hi, table generation << 1 | vlan flag, tag}
// A request is complete when all eight tags are equal and differ from the
// last tag the kernel answered; a read that raced the host's stores sees
// mixed tags and is simply retried on the next poll.
constexpr uint32_t kSvcChunks = 8;
constexpr uint32_t kSvcPktChunks = 7;
constexpr uint32_t kSvcSlot = 80;          // packet bytes handed to the GPU (as nffgo.hpp kSlot)
constexpr uint32_t kSvcBoxBytes = kSvcChunks * 16;
constexpr uint32_t kSvcRespStride = 8;     // u64 words per response (64 B: one line per mailbox)
constexpr uint32_t kSvcStatWords = 8;      // per-wave counters: polls, poll ticks, groups, group ticks, requests
constexpr uint32_t kSvcLdsDwords = 16384;  // INDEXED tables up to 64 KiB are walked from LDS
constexpr uint32_t kSvcMbPerWave = 8;      // mailboxes per consumer wave (a multiple of 8: 1 KiB per poll load)

// A request withdrawn by a caller that gave up (service.hip, the timeout
// policy): the chunk-7 key the consumer answers with port 0 without reading
// any table (the caller may free its rules as soon as it returns).
constexpr uint32_t kSvcWithdrawn = 0xFFFFFFFEu;

// ---- burst mailbox (host memory, one per calling thread of a burst service) --
//
// The VectorSeparateFunction shape (flow/flow.go:131, 1487-1520): a clone's
// whole burst of up to kSvcBurstMax packets in one request, one answer per
// packet.  16-byte chunks as above, each carrying the tag in its last dword:
//   chunk 0:          {desc address lo, desc address hi, generation << 1 | vlan, tag}
//   chunk 1:          {packets n (1..kSvcBurstMax), 0, 0, tag}
//   chunk 2 + 6i + j: packet i bytes [12 + 12j, 24 + 12j) — the scalar
//                     mailbox's chunks without the MAC addresses (bytes 0-11,
//                     which no L3/L4 verdict reads): 14 % fewer bytes to poll
// One consumer wave per mailbox: lane i < n classifies packet i and writes
// {tag, port} to its own 8-byte response word (kSvcBurstRespWords per
// mailbox); the caller waits until all n words carry its tag.
constexpr uint32_t kSvcBurstMax = 32;
constexpr uint32_t kSvcBurstHdrChunks = 2;
constexpr uint32_t kSvcBurstPktChunks = kSvcPktChunks - 1;  // 6
constexpr uint32_t kSvcBurstChunks = kSvcBurstHdrChunks + kSvcBurstMax * kSvcBurstPktChunks;  // 194
constexpr uint32_t kSvcBurstBoxBytes = 4096;  // 4 coalesced poll loads (3 104 bytes used)
constexpr uint32_t kSvcBurstLoads = (kSvcBurstChunks * 16 + 1023) / 1024;
constexpr uint32_t kSvcBurstTailLanes = kSvcBurstChunks - (kSvcBurstLoads - 1) * 64;  // lanes of the last load
constexpr uint32_t kSvcBurstRespWords = kSvcBurstMax;  // 256 B: four lines per mailbox
static_assert(kSvcBurstChunks * 16 <= kSvcBurstBoxBytes, "burst mailbox");

// ---- table descriptor (device memory, after each table's blob) ---------------
//
// What the consumer needs to walk a table, read once per table generation.
// A consumer launch only walks tables uploaded before it started (service.hip:
// table generations), so none of its caches can hold an older copy.
enum SvcKind : uint32_t {
    kSvcNone = 0,     // layout the consumer does not walk (tuning-only forms)
    kSvcLinear = 1,   // LINEAR records
    kSvcIndexed = 2,  // INDEXED inline entries (read from global memory)
    kSvcFlat = 3,     // HYBRID flat-LDS layout, directory image read from global memory
};

struct SvcFamily {
    uint32_t off_resid, n_resid, off_cold, off_ent_base;
    // per positional slot: shift | shift2 << 8 | bits2 << 16, off_dir, off_ent, off_dir16
    // (slots 4..7: the flat form's fine 2-D grids, compile.cpp build_hybrid)
    uint32_t slot[kMaxSlots][4];
};

struct SvcDesc {
    uint32_t kind;        // SvcKind
    uint32_t ns;          // slots walked (2..8; INDEXED 2..4)
    uint32_t back;        // dwords from the blob start to this descriptor
    uint32_t dir8;        // two-level directories with u8 offsets
    uint32_t off_rec4, n4, off_rec6, n6;  // LINEAR records
    SvcFamily fam[2];     // [0] IPv4, [1] IPv6
};
constexpr uint32_t kSvcDescDwords = sizeof(SvcDesc) / 4;
static_assert(sizeof(SvcDesc) % 16 == 0, "descriptor is loaded in 16-byte pieces");

}  // namespace nffacl
