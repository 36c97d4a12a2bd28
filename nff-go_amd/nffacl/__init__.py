"""nffacl — Python binding of libnffacl (ctypes over include/nffacl.h).

Used by the parity tests, bench.py and __graft_entry__.  Names mirror the
reference API this path replaces (packet/acl.go):

  GetL3ACLFromTextTable(filename) -> (L3Rules, NFError|None)   acl.go:148
  GetL3ACLFromJSON(filename)      -> (L3Rules, NFError|None)   acl.go:121
  Engine(rules).L3ACLPort / L3ACLPermit over whole packet batches
                                   (acl.go:495-506, run on the GPU)
  GetL2ACLFromTextTable / GetL2ACLFromJSON -> (L2Rules, NFError|None)  acl.go:88, 70
  L2Engine(rules).L2ACLPort / L2ACLPermit                        acl.go:462-491

There is no CPU fallback: every verdict comes from the HIP kernels in
libnffacl.so.  Importing this module fails loudly if the library is missing.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("NFFACL_LIB", _HERE.parent / "libnffacl.so"))

if not LIB_PATH.exists():
    raise ImportError(
        f"libnffacl.so not found at {LIB_PATH}; build it with `make -C nff-go_amd` "
        "(or __graft_entry__.build()).  There is no CPU fallback.")

# PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64 (same SONAME
# libamdhip64.so.7 as /opt/rocm's).  If libnffacl were loaded first, torch
# would later bring in a second HIP/HSA runtime and the two fight over the
# device ("no HIP device").  Loading torch first makes libnffacl bind to the
# runtime already in the process, so device pointers and streams are shared.
try:  # pragma: no cover - import side effect only
    import torch as _torch  # noqa: F401
except ImportError:
    _torch = None

_lib = ctypes.CDLL(str(LIB_PATH))

# ---- status codes (include/nffacl.h) -----------------------------------------
OK = 0
ERR_PARSE_RULE_JSON = -11
ERR_FILE = -12
ERR_PARSE_RULE = -13
ERR_INCORRECT_ARG_IN_RULES = -14
ERR_INCORRECT_RULE = -15
ERR_INVALID_ARG = -100
ERR_NOMEM = -101
ERR_HIP = -102
ERR_NO_DEVICE = -103
ERR_UNSUPPORTED = -104
ERR_TIMEOUT = -105

ALGO_AUTO, ALGO_LINEAR, ALGO_INDEXED, ALGO_HYBRID = 0, 1, 2, 3
PARSE_VLAN = 1  # ParseAllKnownL3CheckVLAN (packet/vlan.go:104-117) instead of ParseAllKnownL3

# ---- record layouts ------------------------------------------------------------
_L4 = [("id", "u1"), ("id_mask", "u1"), ("valid", "u1"), ("reserved", "u1"),
       ("src_port_min", "<u2"), ("src_port_max", "<u2"),
       ("dst_port_min", "<u2"), ("dst_port_max", "<u2")]
RULE4 = np.dtype([("output_number", "<u4"), ("src_addr", "<u4"), ("dst_addr", "<u4"),
                  ("src_mask", "<u4"), ("dst_mask", "<u4")] + _L4)
RULE6 = np.dtype([("output_number", "<u4"), ("src_addr", "u1", 16), ("dst_addr", "u1", 16),
                  ("src_mask", "u1", 16), ("dst_mask", "u1", 16)] + _L4)
assert RULE4.itemsize == 32 and RULE6.itemsize == 80
L2RULE = np.dtype([("output_number", "<u4"), ("daddr_not_any", "u1"), ("saddr_not_any", "u1"),
                   ("daddr", "u1", 6), ("saddr", "u1", 6), ("id_mask", "<u2"), ("id", "<u2"),
                   ("reserved", "<u2")])
assert L2RULE.itemsize == 24

_vp, _sz, _u32, _u64, _i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
_pp = ctypes.POINTER(ctypes.c_void_p)


def _sig(name, res, *args):
    f = getattr(_lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_rules_load_text = _sig("nffacl_rules_load_text", _i, ctypes.c_char_p, _pp, ctypes.c_char_p, _sz)
_rules_parse_text = _sig("nffacl_rules_parse_text", _i, ctypes.c_char_p, _sz, _pp, ctypes.c_char_p, _sz)
_rules_load_json = _sig("nffacl_rules_load_json", _i, ctypes.c_char_p, _pp, ctypes.c_char_p, _sz)
_rules_parse_json = _sig("nffacl_rules_parse_json", _i, ctypes.c_char_p, _sz, _pp, ctypes.c_char_p, _sz)
_rules_from_arrays = _sig("nffacl_rules_from_arrays", _i, _vp, _sz, _vp, _sz, _pp)
_rules_free = _sig("nffacl_rules_free", None, _vp)
_rules_counts = _sig("nffacl_rules_counts", _i, _vp, ctypes.POINTER(_sz), ctypes.POINTER(_sz))
_rules_get4 = _sig("nffacl_rules_get4", _i, _vp, _sz, _vp)
_rules_get6 = _sig("nffacl_rules_get6", _i, _vp, _sz, _vp)
_engine_create_ex = _sig("nffacl_engine_create_ex", _i, _i, _vp, _i, _pp)
_engine_swap = _sig("nffacl_engine_swap_rules", _i, _vp, _vp)
_engine_destroy = _sig("nffacl_engine_destroy", None, _vp)
_engine_algo = _sig("nffacl_engine_algo", _i, _vp)
_engine_table_bytes = _sig("nffacl_engine_table_bytes", _i, _vp, ctypes.POINTER(_u64))
_classify_device = _sig("nffacl_classify_device_ex", _i, _vp, _vp, _u32, _u64, _vp, _vp, _vp, _u32)
_classify_frames = _sig("nffacl_classify_frames_device_ex", _i, _vp, _vp, _vp, _u64, _vp, _vp, _vp, _u32)
_classify_host = _sig("nffacl_classify_host_ex", _i, _vp, _vp, _u32, _u64, _vp, _vp, _u32)
_l2_load_text = _sig("nffacl_l2rules_load_text", _i, ctypes.c_char_p, _pp, ctypes.c_char_p, _sz)
_l2_parse_text = _sig("nffacl_l2rules_parse_text", _i, ctypes.c_char_p, _sz, _pp, ctypes.c_char_p, _sz)
_l2_load_json = _sig("nffacl_l2rules_load_json", _i, ctypes.c_char_p, _pp, ctypes.c_char_p, _sz)
_l2_parse_json = _sig("nffacl_l2rules_parse_json", _i, ctypes.c_char_p, _sz, _pp, ctypes.c_char_p, _sz)
_l2_from_array = _sig("nffacl_l2rules_from_array", _i, _vp, _sz, _pp)
_l2_free = _sig("nffacl_l2rules_free", None, _vp)
_l2_count = _sig("nffacl_l2rules_count", _i, _vp, ctypes.POINTER(_sz))
_l2_get = _sig("nffacl_l2rules_get", _i, _vp, _sz, _vp)
_l2_engine_create = _sig("nffacl_l2_engine_create", _i, _i, _vp, _pp)
_l2_engine_create_ex = _sig("nffacl_l2_engine_create_ex", _i, _i, _vp, _i, _pp)
_l2_engine_algo = _sig("nffacl_l2_engine_algo", _i, _vp)
_l2_engine_swap = _sig("nffacl_l2_engine_swap_rules", _i, _vp, _vp)
_l2_engine_destroy = _sig("nffacl_l2_engine_destroy", None, _vp)
_l2_classify_device = _sig("nffacl_l2_classify_device", _i, _vp, _vp, _u32, _u64, _vp, _vp, _vp)
_l2_classify_frames = _sig("nffacl_l2_classify_frames_device", _i, _vp, _vp, _vp, _u64, _vp, _vp, _vp)
_l2_classify_host = _sig("nffacl_l2_classify_host", _i, _vp, _vp, _u32, _u64, _vp, _vp)
class Ticket(ctypes.Structure):
    """nffacl_ticket.  `rules` (Python side only) holds the burst's L3Rules
    until the ticket is waited for: the header requires the rule set to
    outlive the wait, and an L3Rules collected before it would free the
    table its batch reads."""
    _fields_ = [("seq", ctypes.c_uint64), ("buf", ctypes.c_uint32), ("off", ctypes.c_uint32),
                ("n", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]
    rules = None


class BatcherStats(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_uint64), ("packets", ctypes.c_uint64), ("bursts", ctypes.c_uint64),
                ("timeouts", ctypes.c_uint64)]


_batcher_create = _sig("nffacl_batcher_create", _i, _vp, _u32, _u32, _u32, _u32, _pp)
_batcher_create_device = _sig("nffacl_batcher_create_device", _i, _i, _u32, _u32, _u32, _u32, _pp)
_batcher_submit_rules = _sig("nffacl_batcher_submit_rules", _i, _vp, _vp, _vp, _vp, _u32, ctypes.POINTER(Ticket))
_batcher_classify_rules = _sig("nffacl_batcher_classify_rules", _i, _vp, _vp, _vp, _vp, _u32, _vp)
_batcher_wait_timeout = _sig("nffacl_batcher_wait_timeout", _i, _vp, ctypes.POINTER(Ticket), _vp, _u64)
_batcher_submit = _sig("nffacl_batcher_submit", _i, _vp, _vp, _vp, _u32, ctypes.POINTER(Ticket))
_batcher_wait = _sig("nffacl_batcher_wait", _i, _vp, ctypes.POINTER(Ticket), _vp)
_batcher_classify = _sig("nffacl_batcher_classify", _i, _vp, _vp, _vp, _u32, _vp)
_batcher_flush = _sig("nffacl_batcher_flush", _i, _vp)
_batcher_stats = _sig("nffacl_batcher_get_stats", _i, _vp, ctypes.POINTER(BatcherStats))
_batcher_destroy = _sig("nffacl_batcher_destroy", None, _vp)
class ServiceStats(ctypes.Structure):
    _fields_ = [("launches", ctypes.c_uint64), ("requests", ctypes.c_uint64), ("timeouts", ctypes.c_uint64),
                ("running", ctypes.c_uint64), ("table_oob", ctypes.c_uint64), ("polls", ctypes.c_uint64),
                ("poll_ns", ctypes.c_double), ("groups", ctypes.c_uint64), ("group_ns", ctypes.c_double),
                ("answered", ctypes.c_uint64), ("retries", ctypes.c_uint64), ("torn", ctypes.c_uint64)]


_rules_prepare = _sig("nffacl_rules_prepare", _i, _vp, _i)
_local_device = _sig("nffacl_local_device", _i)
_pick_device = _sig("nffacl_pick_device", _i, _i, _vp, _i, _vp, _i)
_group_create = _sig("nffacl_group_create", _i, _vp, _i, _vp, _pp)
_group_size = _sig("nffacl_group_size", _i, _vp)
_group_classify = _sig("nffacl_group_classify_device", _i, _vp, _vp, _u32, ctypes.c_uint64, _vp, _vp, _vp)
_group_destroy = _sig("nffacl_group_destroy", None, _vp)
_group_shard = _sig("nffacl_group_shard", _i, _u64, _i, _i, ctypes.POINTER(_u64), ctypes.POINTER(_u64))


class KernelInfo(ctypes.Structure):
    """nffacl_kernel_info (ABI 7): the kernel an engine's slot launches take."""
    _fields_ = [("walk", ctypes.c_int32), ("slots", ctypes.c_uint32), ("rounds", ctypes.c_uint32),
                ("block", ctypes.c_uint32), ("per_cu", ctypes.c_uint32), ("load_mode", ctypes.c_int32),
                ("pulled", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("lds_bytes", ctypes.c_uint64)]


WALK_LINEAR, WALK_INDEXED_GLOBAL, WALK_INDEXED_LDS, WALK_HYBRID_LANE = 0, 1, 2, 3
WALK_FLAT, WALK_FLAT_LDS, WALK_FLAT_LDS_GENERIC, WALK_FLAT_LDS_PIPELINED = 4, 5, 6, 7
_kernel_info = _sig("nffacl_engine_kernel_info", _i, _vp, ctypes.POINTER(KernelInfo))
_device_numa_node = _sig("nffacl_device_numa_node", _i, _i)
_service_create = _sig("nffacl_service_create", _i, _i, _u32, _u32, _pp)
_service_classify = _sig("nffacl_service_classify", _i, _vp, _vp, _vp, _u32, _u32, ctypes.POINTER(_u32))
_service_create_burst = _sig("nffacl_service_create_burst", _i, _i, _u32, _u32, _pp)
_service_classify_burst = _sig("nffacl_service_classify_burst", _i, _vp, _vp, _vp, _vp, _u32, _u32, _vp)
_service_pause = _sig("nffacl_service_pause", _i, _vp, _i)
_service_stats = _sig("nffacl_service_get_stats", _i, _vp, ctypes.POINTER(ServiceStats))
_service_destroy = _sig("nffacl_service_destroy", None, _vp)
_strerror = _sig("nffacl_strerror", ctypes.c_char_p, _i)
_last_error = _sig("nffacl_last_error", ctypes.c_char_p)
_abi_version = _sig("nffacl_abi_version", _i)

EXPORTED_SYMBOLS = [
    "nffacl_rules_load_text", "nffacl_rules_parse_text", "nffacl_rules_load_json",
    "nffacl_rules_parse_json", "nffacl_rules_from_arrays", "nffacl_rules_free",
    "nffacl_rules_counts", "nffacl_rules_get4", "nffacl_rules_get6",
    "nffacl_engine_create", "nffacl_engine_create_ex", "nffacl_engine_swap_rules",
    "nffacl_engine_destroy", "nffacl_engine_algo", "nffacl_engine_table_bytes",
    "nffacl_classify_device", "nffacl_classify_frames_device", "nffacl_classify_host",
    "nffacl_classify_device_ex", "nffacl_classify_frames_device_ex", "nffacl_classify_host_ex",
    "nffacl_table_compile", "nffacl_strerror", "nffacl_abi_version", "nffacl_last_error",
    "nffacl_l2rules_load_text", "nffacl_l2rules_parse_text", "nffacl_l2rules_load_json",
    "nffacl_l2rules_parse_json", "nffacl_l2rules_from_array", "nffacl_l2rules_free",
    "nffacl_l2rules_count", "nffacl_l2rules_get", "nffacl_l2_engine_create",
    "nffacl_l2_engine_create_ex", "nffacl_l2_engine_algo",
    "nffacl_l2_engine_swap_rules", "nffacl_l2_engine_destroy", "nffacl_l2_classify_device",
    "nffacl_l2_classify_frames_device", "nffacl_l2_classify_host",
    "nffacl_batcher_create", "nffacl_batcher_submit", "nffacl_batcher_wait", "nffacl_batcher_classify",
    "nffacl_batcher_flush", "nffacl_batcher_get_stats", "nffacl_batcher_destroy",
    "nffacl_batcher_create_device", "nffacl_batcher_submit_rules", "nffacl_batcher_classify_rules",
    "nffacl_batcher_wait_timeout", "nffacl_local_device", "nffacl_device_numa_node",
    "nffacl_rules_prepare", "nffacl_service_create", "nffacl_service_classify", "nffacl_service_get_stats",
    "nffacl_service_destroy", "nffacl_service_create_burst", "nffacl_service_classify_burst",
    "nffacl_service_pause", "nffacl_pick_device", "nffacl_group_create", "nffacl_group_size",
    "nffacl_group_classify_device", "nffacl_group_destroy", "nffacl_group_shard", "nffacl_engine_kernel_info",
]


def abi_version() -> int:
    return _abi_version()


def local_device() -> int:
    """nffacl_local_device: the HIP device of the calling thread (its CPU's
    rank on its NUMA node modulo the node's GPUs; stable per thread)."""
    return _local_device()


def pick_device(cpu: int, cpu_node, dev_node) -> int:
    """nffacl_pick_device: the device map behind local_device() on any
    topology (cpu_node[c] / dev_node[d] = NUMA nodes, -1 unknown)."""
    cn = np.ascontiguousarray(cpu_node, np.int32)
    dn = np.ascontiguousarray(dev_node, np.int32)
    return _pick_device(cpu, cn.ctypes.data if len(cn) else None, len(cn), dn.ctypes.data if len(dn) else None,
                        len(dn))


def group_shard(n: int, n_devices: int, i: int):
    """nffacl_group_shard: (offset, length) of device i's shard of n packets."""
    off, ln = _u64(), _u64()
    st = _group_shard(n, n_devices, i, ctypes.byref(off), ctypes.byref(ln))
    if st != OK:
        _raise(st, "nffacl_group_shard")
    return off.value, ln.value


class Group:
    """nffacl_group: one rule set on several GPUs of this process (RCCL
    broadcast of the table; scatter of a root-resident batch, gather of the
    verdicts).  The reference's clones-in-one-process deployment
    (flow/scheduler.go:283-289) on a multi-GPU node."""

    def __init__(self, devices, rules: L3Rules):
        devs = np.ascontiguousarray(devices, np.int32)
        h = ctypes.c_void_p()
        st = _group_create(devs.ctypes.data if len(devs) else None, len(devs), rules.handle, ctypes.byref(h))
        if st != OK:
            _raise(st, "nffacl_group_create")
        self._h = h

    def size(self) -> int:
        return _group_size(self._h)

    def classify_device(self, d_slots, stride: int, n: int, port=None, permit=None, stream=None):
        """Root-device tensors (torch) or raw device addresses."""
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        st = _group_classify(self._h, _ptr(d_slots), stride, n, _ptr(port), _ptr(permit), s)
        if st != OK:
            _raise(st, "nffacl_group_classify_device")

    def close(self):
        if getattr(self, "_h", None):
            _group_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def device_numa_node(device: int) -> int:
    """nffacl_device_numa_node: the NUMA node of a device's PCIe attachment
    (negative status if unknown) — where one-packet callers should run."""
    return _device_numa_node(device)


class NFError(Exception):
    """Mirror of common.NFError (common/error.go:54-66): Code is the positive
    common.ErrorCode for parser errors; engine errors keep the negative status."""

    def __init__(self, status: int, message: str):
        self.status = status
        self.code = -status if -15 <= status <= -11 else status
        self.message = message
        super().__init__(message)


def _raise(status: int, what: str = ""):
    detail = (_last_error() or b"").decode(errors="replace")
    msg = f"{what}: {_strerror(status).decode()}" + (f" [{detail}]" if detail else "")
    raise NFError(status, msg)


def _ptr(x) -> int | None:
    """Raw pointer of a torch tensor / numpy array / int / None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(f"cannot take a pointer of {type(x)}")


class L3Rules:
    """Owner of an nffacl_rules handle (the reference's *packet.L3Rules)."""

    def __init__(self, handle):
        self._h = handle

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and _rules_free is not None:
            try:
                _rules_free(h)
            except Exception:  # interpreter teardown
                pass

    @property
    def handle(self):
        return self._h

    @staticmethod
    def _parse(fn, *args):
        out = ctypes.c_void_p()
        err = ctypes.create_string_buffer(512)
        st = fn(*args, ctypes.byref(out), err, len(err))
        if st != OK:
            raise NFError(st, err.value.decode(errors="replace"))
        return L3Rules(out.value)

    @classmethod
    def from_text_file(cls, path) -> "L3Rules":
        return cls._parse(_rules_load_text, str(path).encode())

    @classmethod
    def parse_text(cls, text: bytes | str) -> "L3Rules":
        b = text.encode() if isinstance(text, str) else bytes(text)
        return cls._parse(_rules_parse_text, b, len(b))

    @classmethod
    def from_json_file(cls, path) -> "L3Rules":
        return cls._parse(_rules_load_json, str(path).encode())

    @classmethod
    def parse_json(cls, text: bytes | str) -> "L3Rules":
        b = text.encode() if isinstance(text, str) else bytes(text)
        return cls._parse(_rules_parse_json, b, len(b))

    @classmethod
    def from_arrays(cls, ip4=None, ip6=None) -> "L3Rules":
        a4 = np.ascontiguousarray(ip4 if ip4 is not None else np.zeros(0, RULE4), RULE4)
        a6 = np.ascontiguousarray(ip6 if ip6 is not None else np.zeros(0, RULE6), RULE6)
        out = ctypes.c_void_p()
        st = _rules_from_arrays(a4.ctypes.data if len(a4) else None, len(a4),
                                a6.ctypes.data if len(a6) else None, len(a6), ctypes.byref(out))
        if st != OK:
            _raise(st, "nffacl_rules_from_arrays")
        return L3Rules(out.value)

    def counts(self):
        n4, n6 = _sz(), _sz()
        st = _rules_counts(self._h, ctypes.byref(n4), ctypes.byref(n6))
        if st != OK:
            _raise(st, "nffacl_rules_counts")
        return n4.value, n6.value

    def ip4(self) -> np.ndarray:
        n4, _ = self.counts()
        a = np.zeros(n4, RULE4)
        for i in range(n4):
            _rules_get4(self._h, i, a[i:i + 1].ctypes.data)
        return a

    def ip6(self) -> np.ndarray:
        _, n6 = self.counts()
        a = np.zeros(n6, RULE6)
        for i in range(n6):
            _rules_get6(self._h, i, a[i:i + 1].ctypes.data)
        return a

    def prepare(self, device: int = 0):
        """Compile + upload this rule set's own device table now (else on first use)."""
        st = _rules_prepare(self._h, device)
        if st != OK:
            _raise(st, "nffacl_rules_prepare")


def GetL3ACLFromTextTable(filename):
    """(rules, err) like the Go API; rules is None on error."""
    try:
        return L3Rules.from_text_file(filename), None
    except NFError as e:
        return None, e


def GetL3ACLFromJSON(filename):
    try:
        return L3Rules.from_json_file(filename), None
    except NFError as e:
        return None, e


class Engine:
    """A compiled rule table resident on one HIP device."""

    def __init__(self, rules: L3Rules, device: int = 0, algo: int = ALGO_AUTO):
        out = ctypes.c_void_p()
        st = _engine_create_ex(device, rules.handle, algo, ctypes.byref(out))
        if st != OK:
            _raise(st, "nffacl_engine_create")
        self._h = out.value
        self.device = device

    def close(self):
        h, self._h = getattr(self, "_h", None), None
        if h and _engine_destroy is not None:
            try:
                _engine_destroy(h)
            except Exception:  # interpreter teardown
                pass

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def algo(self) -> int:
        return _engine_algo(self._h)

    @property
    def table_bytes(self) -> int:
        b = _u64()
        st = _engine_table_bytes(self._h, ctypes.byref(b))
        if st != OK:
            _raise(st, "nffacl_engine_table_bytes")
        return b.value

    def kernel_info(self) -> KernelInfo:
        """nffacl_engine_kernel_info: the kernel the active table's slot launches take."""
        k = KernelInfo()
        st = _kernel_info(self._h, ctypes.byref(k))
        if st != OK:
            _raise(st, "nffacl_engine_kernel_info")
        return k

    def swap_rules(self, rules: L3Rules):
        st = _engine_swap(self._h, rules.handle)
        if st != OK:
            _raise(st, "nffacl_engine_swap_rules")

    def classify_device(self, slots, stride: int, n: int, port=None, permit_bits=None, stream=None, flags: int = 0):
        """Asynchronous on `stream` (a torch.cuda.Stream, raw handle or None)."""
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        st = _classify_device(self._h, _ptr(slots), stride, n, _ptr(port), _ptr(permit_bits), s, flags)
        if st != OK:
            _raise(st, "nffacl_classify_device")

    def classify_frames_device(self, frames, desc, n: int, port=None, permit_bits=None, stream=None,
                               flags: int = 0):
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        st = _classify_frames(self._h, _ptr(frames), _ptr(desc), n, _ptr(port), _ptr(permit_bits), s, flags)
        if st != OK:
            _raise(st, "nffacl_classify_frames_device")

    def classify_host(self, slots: np.ndarray, stride: int, n: int | None = None, flags: int = 0,
                      out: np.ndarray | None = None, permit: bool = True):
        """Host slots (uint8, n*stride bytes) -> (port uint32[n], permit uint8[n] or None).
        `out`: the port array to fill (e.g. pinned memory, which the kernel
        writes directly); permit=False skips the per-packet permit bytes."""
        slots = np.ascontiguousarray(slots, np.uint8)
        if n is None:
            n = slots.size // stride
        if slots.size < n * stride:
            raise ValueError("slot buffer too small")
        if out is None:
            port = np.zeros(n, np.uint32)
        else:
            if out.dtype != np.uint32 or out.size < n or not out.flags.c_contiguous:
                raise ValueError("out: contiguous uint32[n] expected")
            port = out
        perm = np.zeros(n, np.uint8) if permit else None
        st = _classify_host(self._h, slots.ctypes.data, stride, n, port.ctypes.data,
                            perm.ctypes.data if permit else None, flags)
        if st != OK:
            _raise(st, "nffacl_classify_host")
        return port, perm

    # Batch forms of the reference's per-packet API (acl.go:495-506)
    def L3ACLPort(self, slots: np.ndarray, stride: int):
        return self.classify_host(slots, stride)[0]

    def L3ACLPermit(self, slots: np.ndarray, stride: int):
        return self.classify_host(slots, stride)[1].astype(bool)


class Batcher:
    """Multi-producer burst aggregator (nffacl_batcher_*): the body of the
    reference's VectorSeparateFunction (flow.go:131) shared by many threads.
    ctypes drops the GIL during the calls, so Python threads really overlap."""

    def __init__(self, engine: "Engine | None", stride: int = 80, max_batch: int = 1 << 16,
                 max_delay_us: int = 100, nbuf: int = 4, device: int | None = None):
        """An engine batcher (`engine`), or with engine=None and `device` a
        device batcher whose bursts name their rule set (classify(..., rules=))."""
        out = ctypes.c_void_p()
        if engine is None and device is not None:
            st = _batcher_create_device(device, stride, max_batch, max_delay_us, nbuf, ctypes.byref(out))
        else:
            st = _batcher_create(engine._h if engine is not None else None, stride, max_batch, max_delay_us, nbuf,
                                 ctypes.byref(out))
        if st != OK:
            _raise(st, "nffacl_batcher_create")
        self._h = out.value
        self._engine = engine  # keep the engine alive
        self.stride = stride

    def close(self):
        h, self._h = getattr(self, "_h", None), None
        if h and _batcher_destroy is not None:
            try:
                _batcher_destroy(h)
            except Exception:  # interpreter teardown
                pass

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @staticmethod
    def frame_pointers(buf: np.ndarray, offsets, lens):
        """(uint64 pointer array, uint32 length array) for frames inside `buf`."""
        base = buf.ctypes.data
        ptrs = (base + np.asarray(offsets, np.uint64)).astype(np.uint64)
        return ptrs, np.ascontiguousarray(lens, np.uint32)

    @staticmethod
    def _burst_arrays(ptrs, lens):
        """uint64 pointers and uint32 lengths as contiguous arrays the caller
        keeps bound for the C call (a converted temporary's .ctypes.data
        would point at freed memory)."""
        pa = np.ascontiguousarray(ptrs, np.uint64)
        la = None if lens is None else np.ascontiguousarray(lens, np.uint32)
        if la is not None and len(la) != len(pa):
            raise ValueError(f"{len(la)} lengths for {len(pa)} frames")
        return pa, la

    def classify(self, ptrs: np.ndarray, lens: np.ndarray | None, rules: "L3Rules | None" = None) -> np.ndarray:
        ptrs, lens = self._burst_arrays(ptrs, lens)
        n = len(ptrs)
        ports = np.zeros(n, np.uint32)
        lp = None if lens is None else lens.ctypes.data
        if rules is None:
            st = _batcher_classify(self._h, ptrs.ctypes.data, lp, n, ports.ctypes.data)
        else:
            st = _batcher_classify_rules(self._h, rules.handle, ptrs.ctypes.data, lp, n, ports.ctypes.data)
        if st != OK:
            _raise(st, "nffacl_batcher_classify")
        return ports

    def submit(self, ptrs: np.ndarray, lens: np.ndarray | None, rules: "L3Rules | None" = None) -> Ticket:
        t = Ticket()
        ptrs, lens = self._burst_arrays(ptrs, lens)
        lp = None if lens is None else lens.ctypes.data
        if rules is None:
            st = _batcher_submit(self._h, ptrs.ctypes.data, lp, len(ptrs), ctypes.byref(t))
        else:
            st = _batcher_submit_rules(self._h, rules.handle, ptrs.ctypes.data, lp, len(ptrs), ctypes.byref(t))
        if st != OK:
            _raise(st, "nffacl_batcher_submit")
        t.rules = rules  # alive until wait() has collected the burst
        return t

    def wait(self, t: Ticket, timeout_us: int | None = None) -> np.ndarray:
        """Verdicts of a submitted burst; with timeout_us, NFError(ERR_TIMEOUT)
        if its batch is not done by then (the ticket stays valid)."""
        ports = np.zeros(t.n, np.uint32)
        if timeout_us is None:
            st = _batcher_wait(self._h, ctypes.byref(t), ports.ctypes.data)
        else:
            st = _batcher_wait_timeout(self._h, ctypes.byref(t), ports.ctypes.data, timeout_us)
        if st == ERR_TIMEOUT:  # not collected: the ticket (and its rules) stay valid
            _raise(st, "nffacl_batcher_wait")
        t.rules = None
        if st != OK:
            _raise(st, "nffacl_batcher_wait")
        return ports

    def flush(self):
        st = _batcher_flush(self._h)
        if st != OK:
            _raise(st, "nffacl_batcher_flush")

    def stats(self) -> dict:
        s = BatcherStats()
        _batcher_stats(self._h, ctypes.byref(s))
        return {k: getattr(s, k) for k, _ in BatcherStats._fields_}


class Service:
    """Persistent GPU consumer (nffacl_service_*).  Scalar services: one
    packet per call — the reference's (*Packet).L3ACLPort / L3ACLPermit
    called from a SetSeparator / SetSplitter function (acl.go:495-506,
    flow.go:128).  Burst services (burst=True): a clone's whole burst of up
    to 32 packets per call — the VectorSeparateFunction shape (flow.go:131,
    1487-1520).  The rule set is passed per call.  ctypes drops the GIL
    during the calls.

    Failure policy (nffacl.h): `classify` / `classify_burst` raise
    NFError(ERR_TIMEOUT) when the consumer did not answer (twice); the
    reference-shaped `L3ACLPort` / `L3ACLPermit` never raise for that — like
    l3ACL (acl.go:522-565) they return the verdict the library set, 0
    (reject), and the event is counted in stats()["timeouts"]."""

    def __init__(self, device: int = 0, mailboxes: int = 0, idle_us: int = 2000, burst: bool = False):
        out = ctypes.c_void_p()
        create = _service_create_burst if burst else _service_create
        st = create(device, mailboxes, idle_us, ctypes.byref(out))
        if st != OK:
            _raise(st, "nffacl_service_create")
        self._h = out.value
        self.device = device
        self.burst = burst

    def close(self):
        h, self._h = getattr(self, "_h", None), None
        if h and _service_destroy is not None:
            try:
                _service_destroy(h)
            except Exception:  # interpreter teardown
                pass

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _classify(self, rules: L3Rules, frame, flags: int = 0):
        buf = np.frombuffer(bytes(frame), np.uint8) if not isinstance(frame, np.ndarray) else \
            np.ascontiguousarray(frame, np.uint8)
        port = _u32()
        st = _service_classify(self._h, rules.handle, buf.ctypes.data if len(buf) else None, len(buf), flags,
                               ctypes.byref(port))
        return st, port.value

    def classify(self, rules: L3Rules, frame, flags: int = 0) -> int:
        """L3ACLPort of one frame (bytes / uint8 array starting at the Ether header)."""
        st, port = self._classify(rules, frame, flags)
        if st != OK:
            _raise(st, "nffacl_service_classify")
        return port

    def classify_burst(self, rules: L3Rules, ptrs: np.ndarray, lens: np.ndarray | None = None,
                       flags: int = 0, _raise_timeout: bool = True) -> np.ndarray:
        """L3ACLPort of a burst (<= 32 frames; pointers and lengths as
        Batcher.frame_pointers gives them)."""
        ptrs = np.ascontiguousarray(ptrs, np.uint64)
        n = len(ptrs)
        ports = np.zeros(n, np.uint32)
        # the converted lengths stay bound to a local for the call (a
        # temporary's .ctypes.data would point at freed memory)
        la = None if lens is None else np.ascontiguousarray(lens, np.uint32)
        if la is not None and len(la) != n:
            raise ValueError(f"classify_burst: {len(la)} lengths for {n} frames")
        lp = None if la is None or n == 0 else la.ctypes.data
        st = _service_classify_burst(self._h, rules.handle, ptrs.ctypes.data if n else None, lp, n, flags,
                                     ports.ctypes.data if n else None)
        del la
        if st != OK and (st != ERR_TIMEOUT or _raise_timeout):
            _raise(st, "nffacl_service_classify_burst")
        return ports

    def L3ACLPort(self, rules: L3Rules, frame) -> int:
        st, port = self._classify(rules, frame)
        if st not in (OK, ERR_TIMEOUT):  # timeout: the policy's verdict (0), counted by the library
            _raise(st, "nffacl_service_classify")
        return port

    def L3ACLPermit(self, rules: L3Rules, frame) -> bool:
        return self.L3ACLPort(rules, frame) > 0

    def L3ACLPortBurst(self, rules: L3Rules, ptrs: np.ndarray, lens: np.ndarray | None = None) -> np.ndarray:
        """The VectorSeparateFunction body: verdicts of a burst (timeouts: 0s, counted)."""
        return self.classify_burst(rules, ptrs, lens, _raise_timeout=False)

    def pause(self, paused: bool = True):
        """nffacl_service_pause: stop the resident consumer (calls then follow
        the failure policy) / resume it."""
        st = _service_pause(self._h, 1 if paused else 0)
        if st != OK:
            _raise(st, "nffacl_service_pause")

    def stats(self) -> dict:
        s = ServiceStats()
        _service_stats(self._h, ctypes.byref(s))
        return {k: getattr(s, k) for k, _ in ServiceStats._fields_}


# ---- L2 ACL (acl.go:68-117, 356-383, 457-491) ---------------------------------

class L2Rules:
    """Owner of an nffacl_l2rules handle (the reference's *packet.L2Rules)."""

    def __init__(self, handle):
        self._h = handle

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and _l2_free is not None:
            try:
                _l2_free(h)
            except Exception:  # interpreter teardown
                pass

    @property
    def handle(self):
        return self._h

    @staticmethod
    def _parse(fn, *args):
        out = ctypes.c_void_p()
        err = ctypes.create_string_buffer(512)
        st = fn(*args, ctypes.byref(out), err, len(err))
        if st != OK:
            raise NFError(st, err.value.decode(errors="replace"))
        return L2Rules(out.value)

    @classmethod
    def from_text_file(cls, path) -> "L2Rules":
        return cls._parse(_l2_load_text, str(path).encode())

    @classmethod
    def parse_text(cls, text: bytes | str) -> "L2Rules":
        b = text.encode() if isinstance(text, str) else bytes(text)
        return cls._parse(_l2_parse_text, b, len(b))

    @classmethod
    def from_json_file(cls, path) -> "L2Rules":
        return cls._parse(_l2_load_json, str(path).encode())

    @classmethod
    def parse_json(cls, text: bytes | str) -> "L2Rules":
        b = text.encode() if isinstance(text, str) else bytes(text)
        return cls._parse(_l2_parse_json, b, len(b))

    @classmethod
    def from_array(cls, eth) -> "L2Rules":
        a = np.ascontiguousarray(eth if eth is not None else np.zeros(0, L2RULE), L2RULE)
        out = ctypes.c_void_p()
        st = _l2_from_array(a.ctypes.data if len(a) else None, len(a), ctypes.byref(out))
        if st != OK:
            _raise(st, "nffacl_l2rules_from_array")
        return L2Rules(out.value)

    def count(self) -> int:
        n = _sz()
        st = _l2_count(self._h, ctypes.byref(n))
        if st != OK:
            _raise(st, "nffacl_l2rules_count")
        return n.value

    def eth(self) -> np.ndarray:
        n = self.count()
        a = np.zeros(n, L2RULE)
        for i in range(n):
            _l2_get(self._h, i, a[i:i + 1].ctypes.data)
        return a


def GetL2ACLFromTextTable(filename):
    """(rules, err) like the Go API; rules is None on error."""
    try:
        return L2Rules.from_text_file(filename), None
    except NFError as e:
        return None, e


def GetL2ACLFromJSON(filename):
    try:
        return L2Rules.from_json_file(filename), None
    except NFError as e:
        return None, e


class L2Engine:
    """A compiled L2 rule table resident on one HIP device."""

    def __init__(self, rules: L2Rules, device: int = 0, algo: int = ALGO_AUTO):
        out = ctypes.c_void_p()
        st = _l2_engine_create_ex(device, rules.handle, algo, ctypes.byref(out))
        if st != OK:
            _raise(st, "nffacl_l2_engine_create")
        self._h = out.value
        self.device = device

    def close(self):
        h, self._h = getattr(self, "_h", None), None
        if h and _l2_engine_destroy is not None:
            try:
                _l2_engine_destroy(h)
            except Exception:  # interpreter teardown
                pass

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def algo(self) -> int:
        return _l2_engine_algo(self._h)

    def swap_rules(self, rules: L2Rules):
        st = _l2_engine_swap(self._h, rules.handle)
        if st != OK:
            _raise(st, "nffacl_l2_engine_swap_rules")

    def classify_device(self, slots, stride: int, n: int, port=None, permit_bits=None, stream=None):
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        st = _l2_classify_device(self._h, _ptr(slots), stride, n, _ptr(port), _ptr(permit_bits), s)
        if st != OK:
            _raise(st, "nffacl_l2_classify_device")

    def classify_frames_device(self, frames, desc, n: int, port=None, permit_bits=None, stream=None):
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        st = _l2_classify_frames(self._h, _ptr(frames), _ptr(desc), n, _ptr(port), _ptr(permit_bits), s)
        if st != OK:
            _raise(st, "nffacl_l2_classify_frames_device")

    def classify_host(self, slots: np.ndarray, stride: int, n: int | None = None):
        """Host slots -> (port uint32[n], permit uint8[n])."""
        slots = np.ascontiguousarray(slots, np.uint8)
        if n is None:
            n = slots.size // stride
        if slots.size < n * stride:
            raise ValueError("slot buffer too small")
        port = np.zeros(n, np.uint32)
        permit = np.zeros(n, np.uint8)
        st = _l2_classify_host(self._h, slots.ctypes.data, stride, n, port.ctypes.data, permit.ctypes.data)
        if st != OK:
            _raise(st, "nffacl_l2_classify_host")
        return port, permit

    # Batch forms of the reference's per-packet API (acl.go:462-476)
    def L2ACLPort(self, slots: np.ndarray, stride: int):
        return self.classify_host(slots, stride)[0]

    def L2ACLPermit(self, slots: np.ndarray, stride: int):
        return self.classify_host(slots, stride)[1].astype(bool)
