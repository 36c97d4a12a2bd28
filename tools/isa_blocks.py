#!/usr/bin/env python3
"""Per-basic-block instruction classes of one kernel in a hipcc -S listing
(static counts: VALU / SALU / DS / VMEM / waits / branches), to see where a
kernel's instructions sit (batch loop, windows, rounds).
usage: python tools/isa_blocks.py engine.s KERNEL_SUBSTRING [--dump]"""
import collections
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    s = open(path).read()
    m = re.search(r"^(_Z\S*" + re.escape(key) + r"\S*):", s, re.M)
    if not m:
        sys.exit(f"no kernel matching {key}")
    i = m.start()
    j = s.index(".Lfunc_end", i)
    body = s[i:j].splitlines()
    print(m.group(1))
    blocks = []
    cur = ["entry", collections.Counter(), []]
    for ln in body:
        t = ln.strip()
        if re.match(r"^\.LBB\d+_\d+:", t):
            blocks.append(cur)
            cur = [t.rstrip(":"), collections.Counter(), []]
            continue
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        cls = ("VALU" if op.startswith("v_") else "WAIT" if op.startswith("s_waitcnt") else
               "BR" if op.startswith(("s_cbranch", "s_branch")) else "SALU" if op.startswith("s_") else
               "DS" if op.startswith("ds_") else "VMEM" if op.startswith(("global_", "buffer_", "flat_")) else op)
        cur[1][cls] += 1
        cur[2].append(t)
    blocks.append(cur)
    tot = collections.Counter()
    for name, c, ins in blocks:
        tot.update(c)
        tgt = [x.split()[-1] for x in ins if x.startswith(("s_cbranch", "s_branch"))]
        print(f"{name:14s} VALU {c['VALU']:4d} SALU {c['SALU']:4d} DS {c['DS']:3d} VMEM {c['VMEM']:3d} "
              f"WAIT {c['WAIT']:3d}  -> {' '.join(tgt)}")
    print("total", dict(tot))
    if "--dump" in sys.argv:
        for name, c, ins in blocks:
            print("==", name)
            print("\n".join(ins))


if __name__ == "__main__":
    main()
