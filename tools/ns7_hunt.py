#!/usr/bin/env python3
"""Where does the pipelined walk go wrong at 7 slots?  Runs the NS = 7
pipelined kernel (an experiment build: make EXTRA=-DNFFACL_PIPE_MAX_NS=8,
loaded through NFFACL_LIB) on test_c5_more_fine_grids_gpu[7]'s input many
times under several launch shapes, and places every wrong verdict in the walk
with the CPU model (tests/pipe_emu.py): batch, lane, family, stream totals,
and the pass / window / round / candidate lane of the winning candidate.
usage: NFFACL_LIB=... [HUNT_FINE_SLOTS=7] [HUNT_VARIANTS=default,...] python tools/ns7_hunt.py OUT.json [LAUNCHES]"""
import json
import os
import sys

os.environ["NFFACL_TUNE_FINE_SLOTS"] = os.environ.get("HUNT_FINE_SLOTS", "7")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "nff-go_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nffacl  # noqa: E402
import pipe_emu  # noqa: E402
from nffacl import synth  # noqa: E402
from oracle import oracle, rules_oracle as ro  # noqa: E402
from test_index_compile import compile_table  # noqa: E402

VARIANTS = {
    "default": {},
    "stride": {"NFFACL_TUNE_DYN": "0"},
    "blk256": {"NFFACL_TUNE_BLOCK": "256"},
    "blk512": {"NFFACL_TUNE_BLOCK": "512"},
    "pipe_off": {"NFFACL_TUNE_PIPE": "0"},
}


def main():
    out_path = sys.argv[1]
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    g = synth.gen_rules(synth.SPECS["c5"], synth.RULE_SEEDS["c5"])
    rules = nffacl.L3Rules.parse_text(g.text)
    a4, a6 = ro.parse_text_table(g.text.encode()).arrays()
    blob, info = compile_table(rules, nffacl.ALGO_HYBRID)
    ns = max(info.fam[0].n_slots, info.fam[1].n_slots)
    n = (1 << 16) + 5
    slots = synth.gen_slots(g, n, 61)
    want, which = oracle.classify_slots_which(slots, 64, n, a4, a6, threads=16)
    trace, where = [], {}
    emu = pipe_emu.emulate_pipe(blob, info, ns, slots, n, trace=trace, where=where)
    F = pipe_emu.slot_fields(slots, n)
    res = {"ns": ns, "emulator_wrong": int((emu != want).sum()), "variants": {}}
    print(json.dumps({"ns": ns, "emulator_wrong": res["emulator_wrong"]}), flush=True)
    d_slots = torch.from_numpy(slots.view(np.uint8)).cuda()
    only = os.environ.get("HUNT_VARIANTS")
    for name, env in VARIANTS.items():
        if only and name not in only.split(","):
            continue
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            eng = nffacl.Engine(rules, algo=nffacl.ALGO_HYBRID)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        bad = []
        for it in range(launches):
            port = torch.zeros(n, dtype=torch.int32, device="cuda")
            eng.classify_device(d_slots, 64, n, port, None)
            torch.cuda.synchronize()
            p = port.cpu().numpy().view(np.uint32)
            for i in np.nonzero(p != want)[0]:
                i = int(i)
                b = i // 64
                tr = trace[b]
                bad.append(dict(launch=it, idx=i, batch=b, lane=i % 64, v6=bool(F["is6"][i]), got=int(p[i]),
                                want=int(want[i]), rule=int(which[i]), T4=tr["T4"], T6=tr["T6"],
                                passes=len(tr["passes"]), at=where.get(i)))
        eng.close()
        res["variants"][name] = {"launches": launches, "wrong": len(bad),
                                 "launches_with_errors": len({x["launch"] for x in bad}), "cases": bad[:200]}
        print(name, len(bad), flush=True)
        for x in bad[:12]:
            print("  ", x, flush=True)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
