#!/usr/bin/env python3
"""Write the service_bench inputs: a rule file, 2^16 slots of 80 bytes and the
oracle's verdict for each (expect.bin, u32).  usage: service_bench.py OUTDIR [c2|c3|c5]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "nff-go_amd"))
from nffacl import synth  # noqa: E402
from oracle import oracle, rules_oracle as ro  # noqa: E402  (checker only)

out = Path(sys.argv[1])
cfg = sys.argv[2] if len(sys.argv) > 2 else "c2"
out.mkdir(parents=True, exist_ok=True)
g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
(out / "rules.conf").write_text(g.text)
n = 1 << 16
slots = synth.gen_slots(g, n, synth.PACKET_SEEDS[cfg], stride=80)
slots.tofile(out / "slots.bin")
a4, a6 = ro.parse_text_table(g.text.encode()).arrays()
oracle.classify_slots(slots, 80, n, a4, a6, threads=16).astype("<u4").tofile(out / "expect.bin")
