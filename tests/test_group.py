"""Device groups (nffacl_group_*, ABI 6) on the GPU (-m gpu): one rule set
compiled once, its table broadcast over RCCL, a root-resident batch
scattered in 64-aligned shards and the verdicts gathered back — bit-exact
against the oracle.  The driver's GPU box has one device, so the group here
has one member (the RCCL communicator, table upload and launch path); with
two or more devices visible the multi-device test runs the scatter and
gather themselves."""
import numpy as np
import pytest

import nffacl
from nffacl import synth
from oracle import oracle, rules_oracle as ro

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def _c2(n, seed=51):
    g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    slots = synth.gen_slots(g, n, seed)
    a4, a6 = ro.parse_text_table(g.text.encode()).arrays()
    want = oracle.classify_slots(slots, 64, n, a4, a6, threads=16)
    return g, slots, want


def _bits(want):
    n = len(want)
    b = np.zeros((n + 63) // 64 * 64, np.uint64)
    b[:n] = want != 0
    return np.bitwise_or.reduce(b.reshape(-1, 64) << np.arange(64, dtype=np.uint64), axis=1)


def _run(torch, grp, slots, n, dev=0, port=True, permit=True):
    d = torch.from_numpy(slots).to(f"cuda:{dev}")
    p = torch.full((max(n, 1),), -1, dtype=torch.int32, device=f"cuda:{dev}") if port else None
    b = torch.zeros(((n + 63) // 64,), dtype=torch.int64, device=f"cuda:{dev}") if permit else None
    grp.classify_device(d, 64, n, p, b, torch.cuda.current_stream(dev))
    torch.cuda.synchronize(dev)
    return (p.cpu().numpy().view(np.uint32)[:n] if port else None,
            b.cpu().numpy().view(np.uint64) if permit else None)


@pytest.mark.parametrize("n", [1, 63, 64, (1 << 20) + 37])
def test_one_device_group_c2_vs_oracle(torch_cuda, n):
    torch = torch_cuda
    g, slots, want = _c2(n)
    rules = nffacl.L3Rules.parse_text(g.text)
    with nffacl.Group([0], rules) as grp:
        del rules  # the group owns its tables
        assert grp.size() == 1
        p, b = _run(torch, grp, slots, n)
        np.testing.assert_array_equal(p, want)
        np.testing.assert_array_equal(b, _bits(want))
        p, _ = _run(torch, grp, slots, n, permit=False)
        np.testing.assert_array_equal(p, want)
        _, b = _run(torch, grp, slots, n, port=False)
        np.testing.assert_array_equal(b, _bits(want))


def test_one_device_group_c5_vs_engine_and_oracle(torch_cuda):
    """The large-table path (HYBRID flat-LDS, ~5 MB of entries broadcast from
    the root): the group's verdicts equal an Engine's on the same rules and
    the oracle."""
    torch = torch_cuda
    g = synth.gen_rules(synth.SPECS["c5"], synth.RULE_SEEDS["c5"])
    n = (1 << 16) + 3
    slots = synth.gen_slots(g, n, 53)
    a4, a6 = ro.parse_text_table(g.text.encode()).arrays()
    want = oracle.classify_slots(slots, 64, n, a4, a6, threads=16)
    rules = nffacl.L3Rules.parse_text(g.text)
    with nffacl.Group([0], rules) as grp:
        p, b = _run(torch, grp, slots, n)
    np.testing.assert_array_equal(p, want)
    np.testing.assert_array_equal(b, _bits(want))
    with nffacl.Engine(rules) as eng:
        d = torch.from_numpy(slots).to("cuda")
        port = torch.empty(n, dtype=torch.int32, device="cuda")
        eng.classify_device(d, 64, n, port)
        torch.cuda.synchronize()
    np.testing.assert_array_equal(port.cpu().numpy().view(np.uint32), p)


def test_group_arguments_and_local_device(torch_cuda):
    g, _, _ = _c2(64)
    rules = nffacl.L3Rules.parse_text(g.text)
    with pytest.raises(nffacl.NFError):
        nffacl.Group([0, 0], rules)  # one member per device
    with pytest.raises(nffacl.NFError):
        nffacl.Group([torch_cuda.cuda.device_count()], rules)
    d = nffacl.local_device()
    assert 0 <= d < torch_cuda.cuda.device_count()
    assert nffacl.local_device() == d  # stable per thread


def test_multi_device_group_scatter_gather(torch_cuda):
    torch = torch_cuda
    nd = torch.cuda.device_count()
    if nd < 2:
        pytest.skip("one HIP device: the scatter / gather need two")
    n = (1 << 20) + 37
    g, slots, want = _c2(n, 52)
    with nffacl.Group(list(range(nd)), nffacl.L3Rules.parse_text(g.text)) as grp:
        p, b = _run(torch, grp, slots, n)
        np.testing.assert_array_equal(p, want)
        np.testing.assert_array_equal(b, _bits(want))
        p, b = _run(torch, grp, slots, 100)  # fewer packets than devices x 64
        np.testing.assert_array_equal(p, want[:100])
