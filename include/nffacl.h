/*
 * nffacl.h — C-ABI of libnffacl, the MI355X-native replacement for nff-go's
 * L3/L4 ACL hot path (packet/acl.go + the header parsing of packet/packet.go).
 *
 * Every entry point is plain C: pointers, sizes and integer status codes; no
 * HIP, torch or C++ types cross this boundary (a HIP stream is passed as
 * `void*`).  A Go cgo package, a Python ctypes binding and the C++ host mirror
 * (nff-go_amd/host/nffgo.hpp) all bind exactly these symbols.
 *
 * Reference interfaces replaced (paths relative to aregm/nff-go):
 *   nffacl_rules_load_text      <- packet.GetL3ACLFromTextTable   packet/acl.go:148-178
 *   nffacl_rules_parse_text     <- same parser, from a memory buffer (acl.go:156-177)
 *   nffacl_rules_load_json      <- packet.GetL3ACLFromJSON        packet/acl.go:121-134
 *   nffacl_rules_from_arrays    <- L3Rules{ip4: ..., ip6: ...} literals the reference
 *                                  tests build directly (acl_internal_test.go:588-593)
 *   nffacl_rules_get4/get6      <- the unexported ip4/ip6 slices read by the reference
 *                                  parse tests (acl_internal_test.go:392, 420)
 *   nffacl_classify_device      <- (*Packet).L3ACLPort / L3ACLPermit  acl.go:495-506,
 *                                  l3ACL acl.go:522-565, l4ACL acl.go:508-520,
 *                                  ParseAllKnownL3 packet.go:353-363,
 *                                  ParseL4ForIPv4/6 packet.go:278-285 — over a batch of
 *                                  packets resident in HBM
 *   nffacl_classify_frames_device  same, over packed variable-length frames (IMIX)
 *   nffacl_classify_host        <- the VectorSeparateFunction body the reference runs per
 *                                  burst (flow/flow.go:131, 1487-1520;
 *                                  test/stability/testSingleWorkingFF/testSingleWorkingFF.go:538-546)
 *                                  — host slots in, verdicts out, PCIe staging inside
 *   nffacl_engine_swap_rules    <- the atomic *L3Rules pointer swap user code performs
 *                                  on rule reload (examples/tutorial/step08.go:33-44)
 *   nffacl_batcher_*            <- the per-burst VectorSeparateFunction calls of every
 *                                  flow-function clone (flow/flow.go:131, 1487-1520),
 *                                  aggregated across threads into shared GPU batches
 *   nffacl_l2rules_load_text    <- packet.GetL2ACLFromTextTable   packet/acl.go:88-117
 *   nffacl_l2rules_load_json    <- packet.GetL2ACLFromJSON        packet/acl.go:70-84
 *   nffacl_l2_classify_device   <- (*Packet).L2ACLPort / L2ACLPermit  acl.go:462-491
 *                                  (l2ACL acl.go:478-491) over a batch in HBM
 *
 * Verdict semantics (bit-exact with acl.go):
 *   port  = OutputNumber of the FIRST rule (file order, per address family) that
 *           matches, 0 if none or the packet is neither IPv4 nor IPv6;
 *   permit = port > 0.
 * Packet bytes past the end of the slot/frame read as 0 (the reference reads
 * whatever mbuf memory follows; the slot convention pins that to zero).
 *
 * Status codes: 0 on success, negative on error.  The rule-parser codes are the
 * negated nff-go common.ErrorCode values (common/error.go:18-50) so a cgo shim
 * can rebuild the exact NFError{Code} the reference returns.
 *
 * Threading: rules objects are immutable after creation and may be shared by
 * any number of threads.  An engine may be used concurrently from several host
 * threads (each on its own stream); nffacl_engine_swap_rules may run
 * concurrently with classification and takes effect for launches issued after
 * it returns.
 */
#ifndef NFFACL_H
#define NFFACL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NFFACL_ABI_VERSION 7

/* Only the entry points below are exported from libnffacl.so (built with
 * -fvisibility=hidden). */
#if defined(__GNUC__)
#define NFFACL_API __attribute__((visibility("default")))
#else
#define NFFACL_API
#endif

/* ---- status codes ------------------------------------------------------ */
enum nffacl_status {
    NFFACL_OK = 0,
    /* negated common.ErrorCode (common/error.go:18-50) */
    NFFACL_ERR_PARSE_RULE_JSON = -11,      /* ParseRuleJSONErr */
    NFFACL_ERR_FILE = -12,                 /* FileErr */
    NFFACL_ERR_PARSE_RULE = -13,           /* ParseRuleErr ("Incomplete 5-tuple") */
    NFFACL_ERR_INCORRECT_ARG_IN_RULES = -14, /* IncorrectArgInRules */
    NFFACL_ERR_INCORRECT_RULE = -15,       /* IncorrectRule (bad OutputNumber) */
    /* engine / device errors (no reference counterpart) */
    NFFACL_ERR_INVALID_ARG = -100,
    NFFACL_ERR_NOMEM = -101,
    NFFACL_ERR_HIP = -102,
    NFFACL_ERR_NO_DEVICE = -103,
    NFFACL_ERR_UNSUPPORTED = -104,
    NFFACL_ERR_TIMEOUT = -105    /* a bounded wait ran out (the work may still complete) */
};

/* ---- rule records (internal representation of acl.go:423-449) --------- */

/* l4Rules, acl.go:423-431 */
typedef struct nffacl_l4 {
    uint8_t id;            /* L4 protocol number (types.TCPNumber ...) */
    uint8_t id_mask;       /* 0 = ANY, 0xff = exact */
    uint8_t valid;         /* ports constrained (IPv4 rules skip the port test when 0) */
    uint8_t reserved;      /* must be 0 */
    uint16_t src_port_min; /* host-order port numbers */
    uint16_t src_port_max;
    uint16_t dst_port_min;
    uint16_t dst_port_max;
} nffacl_l4; /* 12 bytes */

/* l3Rules4, acl.go:433-440.  Addresses and masks are types.IPv4Address values:
 * the little-endian uint32 of the four wire bytes (types/ipv4.go:13-28), so
 * 127.0.0.1 is 0x0100007f exactly as in the reference. */
typedef struct nffacl_rule4 {
    uint32_t output_number; /* Go `uint`; the parsers bound it to 32 bits */
    uint32_t src_addr;
    uint32_t dst_addr;
    uint32_t src_mask;
    uint32_t dst_mask;
    nffacl_l4 l4;
} nffacl_rule4; /* 32 bytes */

/* l3Rules6, acl.go:442-449.  Wire byte order. */
typedef struct nffacl_rule6 {
    uint32_t output_number;
    uint8_t src_addr[16];
    uint8_t dst_addr[16];
    uint8_t src_mask[16];
    uint8_t dst_mask[16];
    nffacl_l4 l4;
} nffacl_rule6; /* 80 bytes */

typedef struct nffacl_rules nffacl_rules;
typedef struct nffacl_engine nffacl_engine;

/* ---- rules ------------------------------------------------------------- */

/* GetL3ACLFromTextTable (acl.go:148).  On error *out is NULL and `err`
 * (if non-NULL) receives the message.  The reference additionally hands back a
 * partially filled *L3Rules next to the error (acl.go:177); no caller uses it. */
NFFACL_API int nffacl_rules_load_text(const char *path, nffacl_rules **out, char *err, size_t errlen);
/* Same grammar, parsing `len` bytes of an in-memory file image. */
NFFACL_API int nffacl_rules_parse_text(const char *text, size_t len, nffacl_rules **out, char *err,
                            size_t errlen);
/* GetL3ACLFromJSON (acl.go:121). */
NFFACL_API int nffacl_rules_load_json(const char *path, nffacl_rules **out, char *err, size_t errlen);
NFFACL_API int nffacl_rules_parse_json(const char *text, size_t len, nffacl_rules **out, char *err,
                            size_t errlen);
/* Build a rule set from already-parsed records, as the reference tests build
 * L3Rules literals (arrays are copied; either pointer may be NULL when its
 * count is 0). */
NFFACL_API int nffacl_rules_from_arrays(const nffacl_rule4 *r4, size_t n4, const nffacl_rule6 *r6,
                             size_t n6, nffacl_rules **out);
NFFACL_API void nffacl_rules_free(nffacl_rules *rules);
NFFACL_API int nffacl_rules_counts(const nffacl_rules *rules, size_t *n4, size_t *n6);
NFFACL_API int nffacl_rules_get4(const nffacl_rules *rules, size_t i, nffacl_rule4 *out);
NFFACL_API int nffacl_rules_get6(const nffacl_rules *rules, size_t i, nffacl_rule6 *out);

/* Compile `rules` for HIP device `hip_device` and upload the table now; the
 * calls that take a rule set per call (nffacl_service_classify,
 * nffacl_batcher_submit_rules) otherwise do this on first use.  The table
 * belongs to the rule set: nffacl_rules_free retires it (stream-ordered
 * behind the work that used it).  This is what makes the reference's rule
 * reload — build a new *L3Rules, swap the pointer (examples/tutorial/
 * step08.go:38-44) — work unchanged: every call classifies against exactly
 * the rule set it was given.  A rule set must outlive the calls using it. */
NFFACL_API int nffacl_rules_prepare(const nffacl_rules *rules, int hip_device);

/* The HIP device the calling thread (a flow-function clone) should use, or
 * NFFACL_ERR_NO_DEVICE: ABI 6 spreads the clones of a NUMA node over ALL of
 * that node's GPUs — the device is nffacl_pick_device() of the thread's CPU
 * (its rank among its node's CPUs, modulo the node's device count; every
 * device when none is on the node).  Stable per thread: its first call
 * decides.  nff-go pins every clone to a core (flow/scheduler.go:283-289,
 * internal/low/low.go:654-666), so the clones of a 2-socket, 8-GPU node land
 * on all 8 GPUs (ABI 5 gave every clone the node's first GPU).  Replaces the
 * binding's former hard-wired GPU 0. */
NFFACL_API int nffacl_local_device(void);

/* The device map behind nffacl_local_device, on any topology: CPU `cpu`
 * (cpu_node[c] = NUMA node of CPU c, -1 unknown; n_cpus entries) gets device
 * local[rank % |local|], where local = the devices d with dev_node[d] equal
 * to the CPU's node (all devices when none) and rank = the number of CPUs
 * below `cpu` on its node.  NFFACL_ERR_INVALID_ARG on bad arguments. */
NFFACL_API int nffacl_pick_device(int cpu, const int *cpu_node, int n_cpus, const int *dev_node, int n_devs);

/* The NUMA node of a HIP device's PCIe attachment (>= 0), or a negative
 * status (NFFACL_ERR_INVALID_ARG, NFFACL_ERR_NO_DEVICE; NFFACL_ERR_HIP when
 * the platform does not report one).  One-packet calls through
 * nffacl_service_classify are fastest from threads on this node (the
 * mailboxes are allocated there): pin the flow-function clones (DPDK lcores)
 * to it.  32 callers on the device's node: 5.8-5.9 Mpps; on the other
 * socket: 3.9-4.4. */
NFFACL_API int nffacl_device_numa_node(int hip_device);

/* ---- engine ------------------------------------------------------------ */

/* Matching strategy compiled into the device table. */
enum nffacl_algo {
    NFFACL_ALGO_AUTO = 0,   /* library picks (indexed when the rule set allows) */
    NFFACL_ALGO_LINEAR = 1, /* wave-uniform first-match scan (acl.go's loop order) */
    NFFACL_ALGO_INDEXED = 2, /* host-compiled interval index + ordered candidate lists */
    NFFACL_ALGO_HYBRID = 3   /* the same index for tables larger than LDS: bucket
                                directories in LDS, compact 16-byte candidates and
                                per-rule records in HBM (CIDR rule sets; AUTO picks
                                it when the INDEXED table outgrows LDS) */
};

/* Compile `rules` for HIP device `hip_device` and upload the table. */
NFFACL_API int nffacl_engine_create(int hip_device, const nffacl_rules *rules, nffacl_engine **out);
NFFACL_API int nffacl_engine_create_ex(int hip_device, const nffacl_rules *rules, int algo,
                            nffacl_engine **out);
/* Compile + upload a new table, then atomically make it the active one.
 * Launches issued before the call keep using the previous table. */
NFFACL_API int nffacl_engine_swap_rules(nffacl_engine *eng, const nffacl_rules *rules);
NFFACL_API void nffacl_engine_destroy(nffacl_engine *eng);
/* Algorithm actually compiled into the active table (NFFACL_ALGO_LINEAR/INDEXED/HYBRID). */
NFFACL_API int nffacl_engine_algo(const nffacl_engine *eng);
/* Bytes of the active device table (rule records + index), for reporting. */
NFFACL_API int nffacl_engine_table_bytes(const nffacl_engine *eng, uint64_t *bytes);

/* The kernel the active table's launches over dense 64-byte slots take
 * (inspection and tests; ABI 7). */
enum nffacl_walk {
    NFFACL_WALK_LINEAR = 0,          /* wave-uniform rule scan (k_linear_slots) */
    NFFACL_WALK_INDEXED_GLOBAL = 1,  /* per-lane candidate lists, table in global memory */
    NFFACL_WALK_INDEXED_LDS = 2,     /* per-lane candidate lists, table staged in LDS */
    NFFACL_WALK_HYBRID_LANE = 3,     /* LDS directories, per-lane walks of HBM entries */
    NFFACL_WALK_FLAT = 4,            /* flat candidate walk, directories in global memory */
    NFFACL_WALK_FLAT_LDS = 5,        /* flat candidate walk, directories in LDS (classify_flat) */
    NFFACL_WALK_FLAT_LDS_GENERIC = 6,/* the same over generalized (compacted) slots */
    NFFACL_WALK_FLAT_LDS_PIPELINED = 7 /* pipelined family-split walk (classify_flat_pipe) */
};
typedef struct nffacl_kernel_info {
    int32_t walk;        /* enum nffacl_walk */
    uint32_t slots;      /* key slots the kernel walks (its NS) */
    uint32_t rounds;     /* flat walks: entry-load rounds per window (2 or 4); else 0 */
    uint32_t block;      /* threads per workgroup */
    uint32_t per_cu;     /* workgroups launched per CU */
    int32_t load_mode;   /* packet load mode at stride 64 (engine.hip) */
    uint32_t pulled;     /* 1: waves pull their batches at run time (BatchSource) */
    uint32_t reserved;
    uint64_t lds_bytes;  /* dynamic LDS per workgroup */
} nffacl_kernel_info;
NFFACL_API int nffacl_engine_kernel_info(nffacl_engine *eng, nffacl_kernel_info *out);

/* Host-side compilation of a rule set into the device table blob, without a
 * device (tooling / inspection; the engine runs the same compiler).  Call with
 * blob == NULL to learn info->blob_dwords, then again with a buffer of at
 * least that many dwords. */
typedef struct nffacl_dim_info {
    uint32_t kind;       /* key: 0 src4, 1 dst4, 2 src6 (top 32 bits), 3 dst6, 4 sport, 5 dport */
    uint32_t shift;      /* bucket = key >> shift (1-D); see kind2 */
    uint32_t n_buckets;  /* radix buckets */
    uint32_t off_dir;    /* dword offset of dir[n_buckets + 1] (bucket bounds, in entries) */
    uint32_t off_entries;/* dword offset of the bucket entries (inline rules, ascending per bucket) */
    uint32_t n_rules;    /* rules indexed by this key */
    uint32_t max_list;   /* longest bucket list */
    uint32_t off_dir16;  /* 0, or (two-level directory) dword offset of u16 offsets dir16[n_buckets + 1];
                            then off_dir holds u32 group bases and dir[t] = base[t >> 6] + dir16[t] */
    uint64_t n_entries;  /* bucket entries (with replication) */
    uint32_t kind2;      /* 6 = none (1-D slot); else a second key (kinds as above): the slot is a
                            2-D grid, bucket = (key >> shift) << bits2 | key2 >> shift2 */
    uint32_t shift2, bits2;
    uint32_t dir8;       /* 1: off_dir16 holds u8 offsets dir8[n_buckets + 1] and off_dir the u32 bases
                            of 16-bucket groups: dir[t] = base[t >> 4] + dir8[t] */
} nffacl_dim_info;

#define NFFACL_MAX_SLOTS 8

typedef struct nffacl_family_info {
    uint32_t n_rec;        /* live rules of the family */
    uint32_t off_rec;      /* LINEAR: dword offset of the rule records (8 dwords IPv4, 20 IPv6);
                              HYBRID flat forms: of the output array (one u32 per rule) */
    uint32_t entry_dwords; /* INDEXED / lane form: dwords per entry (8 IPv4, 20 IPv6);
                              HYBRID flat forms: 6 IPv4, 12 IPv6 (exact entries) */
    uint32_t off_resid, n_resid; /* INDEXED: entries scanned linearly (no selective key) */
    nffacl_dim_info dims[NFFACL_MAX_SLOTS]; /* INDEXED: [dst addr, src addr, dst port, src port];
                                               HYBRID global-directory form: any 1-D / 2-D keys */
    uint32_t n_slots;            /* slots in use (dims[0, n_slots)) */
    uint32_t off_ent_base;       /* HYBRID flat forms: dword offset of the family's first entry
                                    (directory values are entry numbers counted from it) */
} nffacl_family_info;

typedef struct nffacl_table_info {
    int32_t algo;        /* NFFACL_ALGO_LINEAR, _INDEXED or _HYBRID */
    uint32_t lds_dwords; /* HYBRID: blob[0, lds_dwords) = the directories staged in LDS */
    uint64_t blob_dwords;
    nffacl_family_info fam[2]; /* [0] IPv4, [1] IPv6 */
    uint32_t off_params; /* HYBRID flat-LDS positional forms: the slot parameter block in the LDS image (0: none) */
    uint32_t reserved;
} nffacl_table_info;

NFFACL_API int nffacl_table_compile(const nffacl_rules *rules, int algo, uint32_t *blob,
                                    uint64_t cap_dwords, nffacl_table_info *info);

/* ---- classification ------------------------------------------------------ */

/* Parse flags (the *_ex entry points).  0 = the reference's l3ACL exactly. */
enum nffacl_parse_flags {
    /* Parse L3 with ParseAllKnownL3CheckVLAN (packet/vlan.go:104-117) instead
     * of ParseAllKnownL3: one 802.1Q tag (EtherType 0x8100) moves the L3
     * header 4 bytes and the tag's EtherType selects IPv4/IPv6.  The
     * reference's L3ACLPermit never does this (a tagged frame gets 0); the
     * flag serves pipelines that composed the VLAN-aware parse themselves. */
    NFFACL_PARSE_VLAN = 1u
};

/* Device-resident dense slots: packet i occupies d_slots[i*stride, (i+1)*stride)
 * with its frame starting at byte 0 (the Ether header) and zero padding after
 * the frame.  stride % 16 == 0, stride >= 64, d_slots 16-byte aligned.
 * d_port[i]  <- L3ACLPort (may be NULL)
 * d_permit_bits[i/64] bit i%64 <- L3ACLPermit (may be NULL; ceil(n/64) words;
 *   bits past n in the last word are 0).
 * Asynchronous on `stream` (hipStream_t, NULL = default stream).  Launches
 * of one engine on one stream run in stream order; the large-table kernels
 * hand out their batches through per-stream counters of the engine, so a
 * launch captured into a graph must not be replayed concurrently with
 * launches of the same engine on the stream it was captured from (or set
 * NFFACL_TUNE_DYN=0 before creating the engine). */
NFFACL_API int nffacl_classify_device(nffacl_engine *eng, const uint8_t *d_slots, uint32_t stride,
                           uint64_t n, uint32_t *d_port, uint64_t *d_permit_bits,
                           void *stream);

/* Device-resident packed frames (IMIX): frame i starts at d_frames + (desc[i] >> 16)
 * and is (desc[i] & 0xffff) bytes long; bytes past its length read as 0.
 * Frame starts must be 16-byte aligned (mbuf data rooms are cache-line aligned). */
NFFACL_API int nffacl_classify_frames_device(nffacl_engine *eng, const uint8_t *d_frames,
                                  const uint64_t *d_desc, uint64_t n, uint32_t *d_port,
                                  uint64_t *d_permit_bits, void *stream);

/* The same with parse flags (enum nffacl_parse_flags). */
NFFACL_API int nffacl_classify_device_ex(nffacl_engine *eng, const uint8_t *d_slots, uint32_t stride,
                                         uint64_t n, uint32_t *d_port, uint64_t *d_permit_bits,
                                         void *stream, uint32_t flags);
NFFACL_API int nffacl_classify_frames_device_ex(nffacl_engine *eng, const uint8_t *d_frames,
                                                const uint64_t *d_desc, uint64_t n, uint32_t *d_port,
                                                uint64_t *d_permit_bits, void *stream, uint32_t flags);

/* Host slots in, host verdicts out: pinned staging + async H2D / kernel / D2H,
 * double-buffered across chunks.  Synchronous.  h_port / h_permit may be NULL
 * (h_permit gets one byte per packet, 0 or 1). */
NFFACL_API int nffacl_classify_host(nffacl_engine *eng, const uint8_t *h_slots, uint32_t stride,
                         uint64_t n, uint32_t *h_port, uint8_t *h_permit);
NFFACL_API int nffacl_classify_host_ex(nffacl_engine *eng, const uint8_t *h_slots, uint32_t stride,
                                       uint64_t n, uint32_t *h_port, uint8_t *h_permit, uint32_t flags);

/* ---- burst aggregator (host ingest) ----------------
 *
 * Many threads (the reference's flow-function clones, each with a burst of
 * <= 32 packets) submit bursts; the library copies each packet's first
 * `stride` bytes into a shared pinned slot ring and ships the open batch as
 * soon as fewer than two batches are on the GPU — so batches grow while the
 * GPU is busy, up to `max_batch` packets — and every submitter of that batch
 * sleeps until its verdicts are back.  A batch whose first burst has waited
 * `max_delay_us` ships whatever else is in flight.  Thread-safe: any number of
 * concurrent submitters per batcher.  Every ticket must be waited for exactly
 * once (its batch buffer is reused only then).  Tickets not yet waited for
 * keep their batches' buffers busy: a batch ships at the latest when its first
 * burst is max_delay_us old, so a caller that submits without waiting can hold
 * as few as one burst per buffer.  When every buffer is busy, submit waits for
 * one to free (back-pressure) at most 1 s and then returns NFFACL_ERR_TIMEOUT
 * without a ticket (the bursts held are the caller's own to collect).
 * Each batch carries its own status: a failed launch fails the bursts of that
 * batch only.  A batch classifies against one table — the engine's active
 * table, or the rule set a burst was submitted with (nffacl_batcher_*_rules):
 * bursts for different rule sets never share a batch.
 */
typedef struct nffacl_batcher nffacl_batcher;

typedef struct nffacl_ticket {
    uint64_t seq;
    uint32_t buf, off, n, reserved;  /* reserved: the burst's number in its batch */
} nffacl_ticket;

typedef struct nffacl_batcher_stats {
    uint64_t batches;  /* GPU launches */
    uint64_t packets;  /* packets classified */
    uint64_t bursts;   /* submit calls */
    uint64_t timeouts; /* batches shipped before max_batch filled */
} nffacl_batcher_stats;

/* stride: slot bytes per packet (multiple of 16, >= 64; 80 keeps IPv4 with IHL
 * 15 exact); max_batch: packets per GPU launch (>= 64); nbuf: batch buffers in
 * rotation (>= 2).  The engine must outlive the batcher. */
NFFACL_API int nffacl_batcher_create(nffacl_engine *eng, uint32_t stride, uint32_t max_batch,
                                     uint32_t max_delay_us, uint32_t nbuf, nffacl_batcher **out);
/* A batcher of HIP device `hip_device` with no engine: every burst names its
 * rule set (nffacl_batcher_submit_rules / _classify_rules), the binding's
 * shape for the reference's per-call *L3Rules (examples/tutorial/step08.go:
 * 33-44: clones load the current pointer, a reload goroutine stores a new
 * one). */
NFFACL_API int nffacl_batcher_create_device(int hip_device, uint32_t stride, uint32_t max_batch,
                                            uint32_t max_delay_us, uint32_t nbuf, nffacl_batcher **out);
/* Queue a burst: frames[i] points at packet i's Ether header, lens[i] its
 * bytes (NULL lens: `stride` bytes each; bytes past a length read as 0).
 * n <= max_batch.  Returns without waiting; *ticket identifies the burst.
 * Engine batchers only (the engine's active table at launch). */
NFFACL_API int nffacl_batcher_submit(nffacl_batcher *b, const uint8_t *const *frames, const uint32_t *lens,
                                     uint32_t n, nffacl_ticket *ticket);
/* The same against `rules` (its own table on the batcher's device, compiled
 * on first use; nffacl_rules_prepare).  `rules` must outlive the wait. */
NFFACL_API int nffacl_batcher_submit_rules(nffacl_batcher *b, const nffacl_rules *rules,
                                           const uint8_t *const *frames, const uint32_t *lens, uint32_t n,
                                           nffacl_ticket *ticket);
/* Block until the burst's batch is classified; ports[i] <- L3ACLPort of packet
 * i.  Returns the batch's status; a second wait on a ticket is rejected. */
NFFACL_API int nffacl_batcher_wait(nffacl_batcher *b, const nffacl_ticket *ticket, uint32_t *ports);
/* The same, giving up after timeout_us: NFFACL_ERR_TIMEOUT means the batch is
 * not done yet (shipped or not) — no verdict, and the ticket stays valid: wait
 * on it again. */
NFFACL_API int nffacl_batcher_wait_timeout(nffacl_batcher *b, const nffacl_ticket *ticket, uint32_t *ports,
                                           uint64_t timeout_us);
/* submit + wait: the body of a VectorSeparateFunction. */
NFFACL_API int nffacl_batcher_classify(nffacl_batcher *b, const uint8_t *const *frames, const uint32_t *lens,
                                       uint32_t n, uint32_t *ports);
NFFACL_API int nffacl_batcher_classify_rules(nffacl_batcher *b, const nffacl_rules *rules,
                                             const uint8_t *const *frames, const uint32_t *lens, uint32_t n,
                                             uint32_t *ports);
/* Ship the currently open batch now (do not wait for max_batch / max_delay_us). */
NFFACL_API int nffacl_batcher_flush(nffacl_batcher *b);
NFFACL_API int nffacl_batcher_get_stats(nffacl_batcher *b, nffacl_batcher_stats *out);
/* Ships queued bursts, waits for the batches in flight, then frees; no
 * submit/wait may be running. */
NFFACL_API void nffacl_batcher_destroy(nffacl_batcher *b);

/* ---- scalar calls: persistent GPU consumer ------------------------------
 *
 * (*Packet).L3ACLPort / L3ACLPermit (acl.go:495-506) called ONE packet at a
 * time, the shape of every SetSeparator / SetSplitter user function
 * (flow/flow.go:128, 1795-1797; examples/firewall/firewall.go:54-57;
 * examples/tutorial/step08.go:33-35).  A service keeps one small kernel
 * resident on its GPU that polls per-thread mailboxes in pinned host memory:
 * a call writes its packet's first 80 bytes into the calling thread's
 * mailbox and waits until the kernel has written the verdict back — no
 * kernel launch, no driver call per packet.  A caller spins; once the callers
 * outnumber the CPUs the process may use (affinity, cgroup quota) it first
 * sleeps through most of the round trip (a nap adapted per mailbox), so that
 * waiting callers leave the CPUs to posting ones.  The kernel exits after
 * `idle_us` without calls (and every 100 ms) and is re-armed by the next
 * call.  Thread-safe; one service per GPU serves every thread.
 */
typedef struct nffacl_service nffacl_service;

typedef struct nffacl_service_stats {
    uint64_t launches;  /* consumer kernel launches (re-arms) */
    uint64_t requests;  /* calls answered */
    uint64_t timeouts;  /* calls that returned NFFACL_ERR_TIMEOUT */
    uint64_t running;   /* 1 while the consumer kernel is resident */
    uint64_t table_oob; /* 1 if a table walk ever indexed outside its table (read as 0 instead
                           of faulting; a compiler/upload bug — the tests require 0) */
    /* where the time goes, summed over the consumer's completed launches: */
    uint64_t polls;     /* mailbox polls (one PCIe read of every hot mailbox each) */
    double poll_ns;     /* mean poll duration, load issue to data */
    uint64_t groups;    /* request groups classified (one table per group) */
    double group_ns;    /* mean time to classify + answer a group */
    uint64_t answered;  /* requests answered by the consumer (packets) */
    uint64_t retries;   /* requests re-posted after a first timeout (see the failure policy below) */
    uint64_t torn;      /* polls that read a request while its caller was still writing it (re-read) */
} nffacl_service_stats;

/* mailboxes: a multiple of 64 (one consumer wave per 8; 0 = 128), one per
 * calling thread (threads beyond that share mailboxes under a lock);
 * idle_us: consumer lifetime without calls (0 = 2000). */
NFFACL_API int nffacl_service_create(int hip_device, uint32_t mailboxes, uint32_t idle_us, nffacl_service **out);
/* A burst service (ABI 5): the VectorSeparateFunction shape — every call
 * carries a clone's whole burst of up to 32 packets (flow/flow.go:131,
 * 1487-1520: segmentProcess hands the separator one burst at a time and
 * waits for its answers).  One mailbox per calling thread (mailboxes 1..1024,
 * 0 = 64), one consumer wave per mailbox; a request is one rule set. */
NFFACL_API int nffacl_service_create_burst(int hip_device, uint32_t mailboxes, uint32_t idle_us,
                                           nffacl_service **out);
/* L3ACLPort of one packet: frame = its Ether header, len its bytes (bytes past
 * len, and past 80, read as 0 — the batcher's 80-byte slot); flags:
 * enum nffacl_parse_flags.  *port <- the verdict (permit = port > 0).  Blocks
 * about one PCIe round trip.  On a burst service: a burst of one.
 *
 * Failure policy (the reference's verdict path never errors, acl.go:522-565;
 * a caller must not crash the flow function it runs in): a call with no answer
 * after 1 s (NFFACL_TUNE_SVC_TIMEOUT_US) re-posts its request once and re-arms
 * the consumer (stats.retries); with no answer after another 1 s it withdraws
 * the request (the consumer answers a withdrawn request without reading any
 * table, so the rules may be freed at once), sets the verdict(s) to 0 —
 * reject, the value l3ACL gives a packet that matches no rule — and returns
 * NFFACL_ERR_TIMEOUT (stats.timeouts).  Bindings use the verdict and count the
 * event instead of failing the flow function.  Later calls
 * are served normally once the consumer runs again. */
NFFACL_API int nffacl_service_classify(nffacl_service *svc, const nffacl_rules *rules, const uint8_t *frame,
                                       uint32_t len, uint32_t flags, uint32_t *port);
/* L3ACLPort of a burst (burst services only): frames[i] / lens[i] as above
 * (lens NULL: 80 bytes each), n <= 32; ports[i] <- the verdict of packet i.
 * One PCIe round trip for the whole burst; failure policy as above. */
NFFACL_API int nffacl_service_classify_burst(nffacl_service *svc, const nffacl_rules *rules,
                                             const uint8_t *const *frames, const uint32_t *lens, uint32_t n,
                                             uint32_t flags, uint32_t *ports);
/* paused != 0: stop the resident consumer and launch none until resumed (GPU
 * maintenance; calls meanwhile follow the failure policy); 0: resume. */
NFFACL_API int nffacl_service_pause(nffacl_service *svc, int paused);
NFFACL_API int nffacl_service_get_stats(nffacl_service *svc, nffacl_service_stats *out);
/* Stops the consumer and frees; no call may be running. */
NFFACL_API void nffacl_service_destroy(nffacl_service *svc);

/* ---- L2 ACL (packet/acl.go:68-117, 356-383, 413-421, 457-491) ----------- */

/* l2Rules, acl.go:413-421.  MAC addresses in wire order; `id` is the EtherType
 * as a host-order number (types.IPV4Number = 0x0800 ...), compared with the
 * frame's big-endian EtherType under `id_mask` (0 = ANY, 0xffff = exact). */
typedef struct nffacl_l2_rule {
    uint32_t output_number;
    uint8_t daddr_not_any; /* 1: daddr must equal Ether.DAddr (frame bytes 0..5) */
    uint8_t saddr_not_any; /* 1: saddr must equal Ether.SAddr (frame bytes 6..11) */
    uint8_t daddr[6];
    uint8_t saddr[6];
    uint16_t id_mask;
    uint16_t id;
    uint16_t reserved; /* must be 0 */
} nffacl_l2_rule; /* 24 bytes */

typedef struct nffacl_l2rules nffacl_l2rules;
typedef struct nffacl_l2engine nffacl_l2engine;

/* GetL2ACLFromTextTable (acl.go:88): "SrcMAC DstMAC ID [Rule]" per line. */
NFFACL_API int nffacl_l2rules_load_text(const char *path, nffacl_l2rules **out, char *err, size_t errlen);
NFFACL_API int nffacl_l2rules_parse_text(const char *text, size_t len, nffacl_l2rules **out, char *err,
                                         size_t errlen);
/* GetL2ACLFromJSON (acl.go:70): {"L2Rules": [{"Source", "Destination", "ID", "Rule"}]}. */
NFFACL_API int nffacl_l2rules_load_json(const char *path, nffacl_l2rules **out, char *err, size_t errlen);
NFFACL_API int nffacl_l2rules_parse_json(const char *text, size_t len, nffacl_l2rules **out, char *err,
                                         size_t errlen);
/* L2Rules{eth: ...} literal (acl_internal_test.go:1186-1193); copied. */
NFFACL_API int nffacl_l2rules_from_array(const nffacl_l2_rule *r, size_t n, nffacl_l2rules **out);
NFFACL_API void nffacl_l2rules_free(nffacl_l2rules *rules);
NFFACL_API int nffacl_l2rules_count(const nffacl_l2rules *rules, size_t *n);
NFFACL_API int nffacl_l2rules_get(const nffacl_l2rules *rules, size_t i, nffacl_l2_rule *out);

/* algo: NFFACL_ALGO_LINEAR (file-order scan) or NFFACL_ALGO_INDEXED (one hashed
 * probe per rule shape; AUTO picks it when the rules use <= 8 distinct
 * MAC/EtherType mask shapes, which every parsed rule file does). */
NFFACL_API int nffacl_l2_engine_create(int hip_device, const nffacl_l2rules *rules, nffacl_l2engine **out);
NFFACL_API int nffacl_l2_engine_create_ex(int hip_device, const nffacl_l2rules *rules, int algo,
                                          nffacl_l2engine **out);
NFFACL_API int nffacl_l2_engine_algo(const nffacl_l2engine *eng);
NFFACL_API int nffacl_l2_engine_swap_rules(nffacl_l2engine *eng, const nffacl_l2rules *rules);
NFFACL_API void nffacl_l2_engine_destroy(nffacl_l2engine *eng);

/* L2ACLPort / L2ACLPermit over device-resident slots / packed frames; same
 * buffer conventions as nffacl_classify_device / _frames_device (only frame
 * bytes 0..13 are read; bytes past a frame's length read as 0). */
NFFACL_API int nffacl_l2_classify_device(nffacl_l2engine *eng, const uint8_t *d_slots, uint32_t stride,
                                         uint64_t n, uint32_t *d_port, uint64_t *d_permit_bits,
                                         void *stream);
NFFACL_API int nffacl_l2_classify_frames_device(nffacl_l2engine *eng, const uint8_t *d_frames,
                                                const uint64_t *d_desc, uint64_t n, uint32_t *d_port,
                                                uint64_t *d_permit_bits, void *stream);
/* Host slots in, host verdicts out (synchronous; staging inside, sized to the
 * request).  h_port / h_permit (one byte per packet) may be NULL. */
NFFACL_API int nffacl_l2_classify_host(nffacl_l2engine *eng, const uint8_t *h_slots, uint32_t stride,
                                       uint64_t n, uint32_t *h_port, uint8_t *h_permit);

/* ---- device group: one process, several GPUs (ABI 6) -------------------
 * The reference's multi-core deployment is ONE process whose core-pinned
 * clones share one *L3Rules (flow/scheduler.go:283-289, packet/acl.go:
 * 495-506); a group lets such a host spread one batch over several GPUs
 * without a process per GPU.  nffacl_group_create opens one RCCL
 * communicator per device (ncclCommInitAll), compiles `rules` once on the
 * host, uploads the table to hip_devices[0] (the root) and ncclBroadcasts
 * it to the others over xGMI.  The group owns its tables (the rule set may
 * be freed afterwards); a rule reload is a new group.  Devices must be
 * distinct.  NFFACL_ERR_NO_DEVICE without HIP devices; NFFACL_ERR_HIP with
 * the last error "RCCL not available: ..." when librccl cannot be loaded —
 * RCCL is opened here (dlopen), so nothing else in the library needs it.
 * Every RCCL call and device switch is checked; a failure inside a group
 * call closes the group and returns NFFACL_ERR_HIP.  (Groups of more than
 * one device have run on no multi-GPU node yet: their scatter / gather
 * parity is unverified on hardware) */
typedef struct nffacl_group nffacl_group;
NFFACL_API int nffacl_group_create(const int *hip_devices, int n, const nffacl_rules *rules, nffacl_group **out);
NFFACL_API int nffacl_group_size(const nffacl_group *g);
/* L3ACLPort / L3ACLPermit of n packets resident on the ROOT device (slots as
 * nffacl_classify_device; d_port / d_permit_bits on the root too, either may
 * be NULL but not both): 64-aligned shards go to the group's devices by
 * ncclSend/ncclRecv (the root keeps the first), every device classifies its
 * shard, and the verdicts (ports, permit words) come back by ncclSend/
 * ncclRecv into the root's arrays.  Enqueued on `stream` (a root-device
 * hipStream_t; NULL = default) and the group's own per-device streams:
 * returns at once; the verdicts are complete when `stream` is.  Calls on one
 * group are serialised (they share its communicators). */
NFFACL_API int nffacl_group_classify_device(nffacl_group *g, const uint8_t *d_slots, uint32_t stride, uint64_t n,
                                            uint32_t *d_port, uint64_t *d_permit_bits, void *stream);
NFFACL_API void nffacl_group_destroy(nffacl_group *g);
/* The group's shard plan (pure; ABI 7): shard i of n packets over n_devices
 * devices is [*off, *off + *len) — shards of ceil(ceil(n / N) / 64) * 64
 * packets in device order, the last ones shorter or empty, *off always a
 * multiple of 64 (so the shard's permit words start at *off / 64 and no
 * word straddles two devices).  NFFACL_ERR_INVALID_ARG for N outside 1..64,
 * i outside 0..N-1, n > 2^48 or NULL outputs. */
NFFACL_API int nffacl_group_shard(uint64_t n, int n_devices, int i, uint64_t *off, uint64_t *len);

/* ---- misc ------------------------------------------------------------- */
NFFACL_API const char *nffacl_strerror(int status);
NFFACL_API int nffacl_abi_version(void);
/* Last HIP / engine error message recorded on this thread ("" if none). */
NFFACL_API const char *nffacl_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* NFFACL_H */
