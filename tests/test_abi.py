"""The C-ABI library loads and exports every symbol include/nffacl.h declares
(CPU only: no compute calls without a GPU)."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest

import nffacl

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "nffacl.h"


def declared_symbols():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nffacl_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for must in ("nffacl_rules_load_text", "nffacl_engine_create", "nffacl_engine_swap_rules",
                 "nffacl_classify_device", "nffacl_classify_host", "nffacl_classify_frames_device"):
        assert must in syms


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", str(nffacl.LIB_PATH)], check=True,
                         capture_output=True, text=True).stdout
    exported = set(re.findall(r"\b(nffacl_[a-z0-9_]+)\b", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    lib = ctypes.CDLL(str(nffacl.LIB_PATH))
    for s in declared_symbols():
        assert getattr(lib, s) is not None
    assert set(nffacl.EXPORTED_SYMBOLS) <= set(declared_symbols())


def test_abi_version():
    assert nffacl.abi_version() == 5  # 3: generalized slots in nffacl_table_info; 5: burst service


def test_exports_are_c_linkage_only():
    """No C++-mangled or torch symbols leak through the public boundary."""
    out = subprocess.run(["nm", "-D", "--defined-only", str(nffacl.LIB_PATH)], check=True,
                         capture_output=True, text=True).stdout
    public = [l.split()[-1] for l in out.splitlines() if " T " in l]
    assert all(not s.startswith("_Z") or "nffacl" not in s for s in public)
    assert "torch" not in out


def test_rule_structs_match_header_sizes():
    assert nffacl.RULE4.itemsize == 32 and nffacl.RULE6.itemsize == 80


def test_strerror_codes_mirror_nferror():
    for st, word in ((-11, "JSON"), (-12, "file"), (-13, "5-tuple"), (-14, "argument"), (-15, "rule")):
        assert word.lower() in nffacl._strerror(st).decode().lower()


def test_engine_without_device_fails_loudly(gpu_available):
    if gpu_available:
        pytest.skip("device present")
    rules = nffacl.L3Rules.parse_text(b"ANY ANY ANY ANY ANY Accept\n")
    with pytest.raises(nffacl.NFError) as e:
        nffacl.Engine(rules)
    assert e.value.status in (nffacl.ERR_NO_DEVICE, nffacl.ERR_HIP)


def test_device_numa_node(gpu_available):
    """nffacl_device_numa_node: NO_DEVICE without a GPU; with one, device 0's
    node (or ERR_HIP where the platform reports none) and INVALID_ARG for a
    device that does not exist."""
    if not gpu_available:
        assert nffacl.device_numa_node(0) == nffacl.ERR_NO_DEVICE
        return
    assert nffacl.device_numa_node(0) >= 0 or nffacl.device_numa_node(0) == nffacl.ERR_HIP
    assert nffacl.device_numa_node(-1) == nffacl.ERR_INVALID_ARG
    assert nffacl.device_numa_node(4096) == nffacl.ERR_INVALID_ARG
