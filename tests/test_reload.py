"""examples/tutorial/step08.go's rule reload, end to end (-m gpu).

step08.go keeps `rulesp unsafe.Pointer` to the current *L3Rules; a goroutine
loads a fresh rule file every 5 s and swaps the pointer (atomic.StorePointer,
:38-44) while every flow-function clone classifies against whatever pointer
it loaded (atomic.LoadPointer, :33-35).  With the binding's design — each rule
set owns its compiled device table (nffacl_rules_prepare), calls take the
rule set (nffacl_service_classify / nffacl_batcher_classify_rules) — that
pattern needs nothing else.  Here a reload thread re-parses one of three C2
rule texts every few ms while 16 threads classify bursts through one device
batcher and single packets through the persistent consumer; every answer
must equal the oracle's for the rule set that call named, and old rule sets
are freed (their tables retired) while the others keep running.
"""
import threading
import time

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
    torch.cuda.init()
    return torch


def test_step08_reload_while_classifying(torch_cuda):
    texts = [synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"] + k).text for k in range(3)]
    g0 = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    n = 8192
    slots = synth.gen_slots(g0, n, 0x5708, stride=80)
    wants = []
    for t in texts:
        a4, a6 = ro.parse_text_table(t.encode()).arrays()
        wants.append(oracle.classify_slots(slots, 80, n, a4, a6, threads=16))
    ptrs, lens = nffacl.Batcher.frame_pointers(slots, np.arange(n, dtype=np.uint64) * 80, np.full(n, 80, np.uint32))
    frames = slots.reshape(n, 80)

    class Gen:  # what rulesp points at: a rule set + which text it came from
        def __init__(self, k):
            self.k = k
            self.rules = nffacl.L3Rules.parse_text(texts[k])
            self.rules.prepare(0)  # compiled in the reload thread, as the loader would

    cur = [Gen(0)]  # a Python list store / load is atomic under the GIL
    svc = nffacl.Service(0, mailboxes=64)
    bat = nffacl.Batcher(None, stride=80, max_batch=4096, max_delay_us=50, nbuf=4, device=0)
    halt = threading.Event()
    errors, seen = [], set()
    calls = [0] * 16

    def clone(c):
        try:
            it = 0
            while not halt.is_set():
                local = cur[0]  # atomic.LoadPointer
                s = (it * 16 + c) * 32 % (n - 32)
                got = bat.classify(ptrs[s:s + 32], lens[s:s + 32], rules=local.rules)
                if not np.array_equal(got, wants[local.k][s:s + 32]):
                    errors.append(("burst", c, s, local.k))
                i = (s + 7) % n
                p = svc.classify(local.rules, frames[i])
                if p != wants[local.k][i]:
                    errors.append(("scalar", c, i, local.k, p, int(wants[local.k][i])))
                seen.add(local.k)
                calls[c] += 1
                it += 1
        except Exception as ex:  # surfaced below
            errors.append(ex)

    ths = [threading.Thread(target=clone, args=(c,)) for c in range(16)]
    for t in ths:
        t.start()
    reloads = 0
    t_end = time.time() + 3.0
    while time.time() < t_end:  # updateSeparateRules with the 5 s sleep shortened
        time.sleep(0.005)
        cur[0] = Gen((reloads + 1) % 3)  # atomic.StorePointer; the old set is freed with its last user
        reloads += 1
    halt.set()
    for t in ths:
        t.join()
    st = svc.stats()
    svc.close()
    bat.close()
    assert not errors, errors[:10]
    assert reloads > 50 and seen == {0, 1, 2}
    assert min(calls) > 0
    assert st["table_oob"] == 0 and st["timeouts"] == 0
