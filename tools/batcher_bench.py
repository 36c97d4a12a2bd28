#!/usr/bin/env python3
"""Write the batcher_bench inputs: C2 rule file + 2^20 slots of 80 bytes."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "nff-go_amd"))
from nffacl import synth  # noqa: E402

out = Path(sys.argv[1])
out.mkdir(parents=True, exist_ok=True)
g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
(out / "rules.conf").write_text(g.text)
synth.gen_slots(g, 1 << 20, synth.PACKET_SEEDS["c2"], stride=80).tofile(out / "slots.bin")
