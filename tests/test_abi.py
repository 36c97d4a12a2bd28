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
    # 3: generalized slots in nffacl_table_info; 5: burst service; 6: device groups, nffacl_pick_device;
    # 7: nffacl_group_shard, nffacl_engine_kernel_info
    assert nffacl.abi_version() == 7


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


def test_pick_device_spreads_a_node_over_its_gpus():
    """a synthetic 2-socket host (256 CPUs, SMT
    siblings numbered +128, node 0 = CPUs 0-63 and 128-191) with 8 GPUs, 4 on
    each node: every node's clones spread evenly over that node's 4 GPUs, by
    the CPU's rank among the node's CPUs (nffacl_local_device's map)."""
    cpu_node = [0] * 64 + [1] * 64 + [0] * 64 + [1] * 64
    dev_node = [0, 0, 0, 0, 1, 1, 1, 1]
    got = [nffacl.pick_device(c, cpu_node, dev_node) for c in range(256)]
    assert got[:8] == [0, 1, 2, 3, 0, 1, 2, 3]
    assert got[64:72] == [4, 5, 6, 7, 4, 5, 6, 7]
    assert got[128] == 0 and got[129] == 1 and got[192] == 4  # SMT siblings continue the node's rank
    for node, devs in ((0, {0, 1, 2, 3}), (1, {4, 5, 6, 7})):
        mine = [got[c] for c in range(256) if cpu_node[c] == node]
        assert set(mine) == devs
        counts = [mine.count(d) for d in sorted(devs)]
        assert max(counts) - min(counts) <= 1  # even spread: 32 clones per GPU
    # GPUs interleaved over the nodes (dev_node 0,1,0,1,...)
    inter = [0, 1] * 4
    assert [nffacl.pick_device(c, cpu_node, inter) for c in range(4)] == [0, 2, 4, 6]
    assert [nffacl.pick_device(c, cpu_node, inter) for c in range(64, 68)] == [1, 3, 5, 7]
    # no device on the CPU's node, or unknown nodes: every device, by CPU number
    assert [nffacl.pick_device(c, cpu_node, [-1] * 8) for c in range(10)] == [c % 8 for c in range(10)]
    assert nffacl.pick_device(3, [], [0, 0]) == 1  # unknown CPU map
    assert nffacl.pick_device(0, cpu_node, []) < 0  # no devices: NFFACL_ERR_INVALID_ARG


def test_group_without_device_reports_no_device():
    """nffacl_group_create without a HIP device: NFFACL_ERR_NO_DEVICE (the
    group itself runs in tests/test_group.py on the GPU); bad arguments are
    rejected before any device is touched."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is visible")
    rules = nffacl.L3Rules.parse_text("ANY ANY TCP ANY 80 Accept\n")
    with pytest.raises(nffacl.NFError) as e:
        nffacl.Group([0], rules)
    assert e.value.status == nffacl.ERR_NO_DEVICE
    with pytest.raises(nffacl.NFError) as e:
        nffacl.Group([], rules)
    assert e.value.status == nffacl.ERR_INVALID_ARG


@pytest.mark.parametrize("ndev", range(1, 9))
def test_group_shard_plan(ndev):
    """the device group's shard plan (group.cpp, the
    pure nffacl_group_shard) for N = 1..8 devices — empty batches, batches
    smaller than 64 N (trailing devices get nothing), ragged tails, and the
    permit words each shard's verdicts go back to: the shards tile [0, n) in
    device order, every offset is a multiple of 64, every shard is at most
    ceil(ceil(n / N) / 64) * 64 packets, and the shards' permit words
    [off / 64, off / 64 + ceil(len / 64)) tile the batch's ceil(n / 64) words
    with no word shared by two devices."""
    sizes = {0, 1, 37, 63, 64, 65, 64 * ndev - 1, 64 * ndev, 64 * ndev + 1, 64 * ndev * 3 + 17, 1000003,
             (1 << 20) + 37, 1 << 24}
    for n in sorted(sizes):
        per = ((n + ndev - 1) // ndev + 63) // 64 * 64
        pos, words = 0, 0
        for i in range(ndev):
            off, ln = nffacl.group_shard(n, ndev, i)
            assert off == min(n, pos) and off % 64 == 0 or (ln == 0 and off == n), (n, i, off, ln)
            assert ln <= per
            if ln:
                assert off == pos
                assert off // 64 == words  # the shard's first permit word follows the previous shard's last
                words += (ln + 63) // 64
                assert ln == per or off + ln == n  # only the last non-empty shard is short
            pos += ln
        assert pos == n and words == (n + 63) // 64
        # the root keeps the first (largest) shard: the staging on devices 1.. never needs more
        assert nffacl.group_shard(n, ndev, 0)[1] == min(n, per)


def test_group_shard_rejects_bad_arguments():
    for args in ((10, 0, 0), (10, 65, 0), (10, 2, 2), (10, 2, -1), ((1 << 48) + 1, 2, 0)):
        with pytest.raises(nffacl.NFError) as e:
            nffacl.group_shard(*args)
        assert e.value.status == nffacl.ERR_INVALID_ARG


def test_library_needs_no_rccl():
    """RCCL is dlopen'ed by nffacl_group_create only, so
    single-GPU users need no RCCL: the library has no link dependency on it."""
    out = subprocess.run(["readelf", "-d", str(nffacl.LIB_PATH)], check=True, capture_output=True, text=True).stdout
    needed = re.findall(r"\(NEEDED\).*\[(.*)\]", out)
    assert needed and not any("rccl" in x for x in needed), needed
