"""TEST INFRASTRUCTURE ONLY — ctypes front of the C oracle (acl_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / the timed CPU baseline — never as the
thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

from .rules_oracle import L2RULE_DTYPE, RULE4_DTYPE, RULE6_DTYPE

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "liboracle.so"
_lib = None


def build():
    """Compile liboracle.so (gcc, seconds)."""
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)


def _load():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            build()
        lib = ctypes.CDLL(str(_LIB_PATH))
        vp, sz, u32, u64, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        lib.oracle_l3acl.restype = u32
        lib.oracle_l3acl.argtypes = [vp, u32, vp, sz, vp, sz]
        lib.oracle_classify_slots.restype = i
        lib.oracle_classify_slots.argtypes = [vp, u32, u64, vp, sz, vp, sz, vp, i]
        lib.oracle_classify_slots_which.restype = i
        lib.oracle_classify_slots_which.argtypes = [vp, u32, u64, vp, sz, vp, sz, vp, vp, i]
        lib.oracle_classify_frames.restype = i
        lib.oracle_classify_frames.argtypes = [vp, vp, u64, vp, sz, vp, sz, vp, i]
        lib.oracle_classify_slots_flags.restype = i
        lib.oracle_classify_slots_flags.argtypes = [vp, u32, u64, vp, sz, vp, sz, vp, i, u32]
        lib.oracle_classify_frames_flags.restype = i
        lib.oracle_classify_frames_flags.argtypes = [vp, vp, u64, vp, sz, vp, sz, vp, i, u32]
        lib.oracle_l2acl.restype = u32
        lib.oracle_l2acl.argtypes = [vp, u32, vp, sz]
        lib.oracle_l2_classify_slots.restype = i
        lib.oracle_l2_classify_slots.argtypes = [vp, u32, u64, vp, sz, vp, i]
        lib.oracle_l2_classify_frames.restype = i
        lib.oracle_l2_classify_frames.argtypes = [vp, vp, u64, vp, sz, vp, i]
        assert lib.oracle_l2rule_size() == L2RULE_DTYPE.itemsize
        assert lib.oracle_rule4_size() == RULE4_DTYPE.itemsize
        assert lib.oracle_rule6_size() == RULE6_DTYPE.itemsize
        _lib = lib
    return _lib


def _rules(a4, a6):
    a4 = np.ascontiguousarray(a4 if a4 is not None else np.zeros(0, RULE4_DTYPE)).view(RULE4_DTYPE)
    a6 = np.ascontiguousarray(a6 if a6 is not None else np.zeros(0, RULE6_DTYPE)).view(RULE6_DTYPE)
    return a4, a6


def l3acl(packet: bytes, a4=None, a6=None) -> int:
    """L3ACLPort of one packet (bytes past len(packet) read as 0)."""
    lib = _load()
    a4, a6 = _rules(a4, a6)
    buf = np.frombuffer(bytes(packet) or b"\0", np.uint8)
    return lib.oracle_l3acl(buf.ctypes.data, len(packet), a4.ctypes.data, len(a4), a6.ctypes.data, len(a6))


PARSE_VLAN = 1  # ParseAllKnownL3CheckVLAN instead of ParseAllKnownL3


def classify_slots(slots: np.ndarray, stride: int, n: int, a4=None, a6=None, threads: int = 1,
                   flags: int = 0) -> np.ndarray:
    lib = _load()
    a4, a6 = _rules(a4, a6)
    slots = np.ascontiguousarray(slots, np.uint8)
    assert slots.size >= n * stride
    out = np.zeros(n, np.uint32)
    st = lib.oracle_classify_slots_flags(slots.ctypes.data, stride, n, a4.ctypes.data, len(a4),
                                         a6.ctypes.data, len(a6), out.ctypes.data, threads, flags)
    if st != 0:
        raise RuntimeError("oracle_classify_slots failed")
    return out


def classify_slots_which(slots: np.ndarray, stride: int, n: int, a4=None, a6=None, threads: int = 1):
    """(ports, index of the first-matching rule in its family slice or -1)."""
    lib = _load()
    a4, a6 = _rules(a4, a6)
    slots = np.ascontiguousarray(slots, np.uint8)
    assert slots.size >= n * stride
    out = np.zeros(n, np.uint32)
    which = np.zeros(n, np.int64)
    st = lib.oracle_classify_slots_which(slots.ctypes.data, stride, n, a4.ctypes.data, len(a4),
                                         a6.ctypes.data, len(a6), out.ctypes.data, which.ctypes.data, threads)
    if st != 0:
        raise RuntimeError("oracle_classify_slots_which failed")
    return out, which


def classify_frames(frames: np.ndarray, desc: np.ndarray, a4=None, a6=None, threads: int = 1,
                    flags: int = 0) -> np.ndarray:
    lib = _load()
    a4, a6 = _rules(a4, a6)
    frames = np.ascontiguousarray(frames, np.uint8)
    desc = np.ascontiguousarray(desc, np.uint64)
    out = np.zeros(len(desc), np.uint32)
    st = lib.oracle_classify_frames_flags(frames.ctypes.data, desc.ctypes.data, len(desc), a4.ctypes.data,
                                          len(a4), a6.ctypes.data, len(a6), out.ctypes.data, threads, flags)
    if st != 0:
        raise RuntimeError("oracle_classify_frames failed")
    return out


def _l2(eth):
    return np.ascontiguousarray(eth if eth is not None else np.zeros(0, L2RULE_DTYPE)).view(L2RULE_DTYPE)


def l2acl(packet: bytes, eth=None) -> int:
    """L2ACLPort of one packet (bytes past len(packet) read as 0)."""
    lib = _load()
    eth = _l2(eth)
    buf = np.frombuffer(bytes(packet) or b"\0", np.uint8)
    return lib.oracle_l2acl(buf.ctypes.data, len(packet), eth.ctypes.data, len(eth))


def l2_classify_slots(slots: np.ndarray, stride: int, n: int, eth=None, threads: int = 1) -> np.ndarray:
    lib = _load()
    eth = _l2(eth)
    slots = np.ascontiguousarray(slots, np.uint8)
    assert slots.size >= n * stride
    out = np.zeros(n, np.uint32)
    if lib.oracle_l2_classify_slots(slots.ctypes.data, stride, n, eth.ctypes.data, len(eth),
                                    out.ctypes.data, threads) != 0:
        raise RuntimeError("oracle_l2_classify_slots failed")
    return out


def l2_classify_frames(frames: np.ndarray, desc: np.ndarray, eth=None, threads: int = 1) -> np.ndarray:
    lib = _load()
    eth = _l2(eth)
    frames = np.ascontiguousarray(frames, np.uint8)
    desc = np.ascontiguousarray(desc, np.uint64)
    out = np.zeros(len(desc), np.uint32)
    if lib.oracle_l2_classify_frames(frames.ctypes.data, desc.ctypes.data, len(desc), eth.ctypes.data,
                                     len(eth), out.ctypes.data, threads) != 0:
        raise RuntimeError("oracle_l2_classify_frames failed")
    return out
