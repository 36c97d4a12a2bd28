#!/usr/bin/env python3
"""Static check of one kernel's memory waits in a hipcc -S listing: a
dataflow pass over the kernel's control-flow graph that tracks which memory
operations may still be in flight (vmcnt: VMEM loads and stores, completing
in order; lgkmcnt: LDS / bpermute in order among themselves, SMEM out of
order) and reports every instruction that reads or overwrites a register a
possibly-incomplete load is still to write.  A hit means the listing uses a
value before its load is known to have returned: timing-dependent results.

State per program point: for each possibly-outstanding op, the fewest ops of
its counter class issued after it on any path reaching the point (the join
takes the minimum, so the check is conservative).  s_waitcnt vmcnt(N)
retires every VMEM op with >= N later VMEM ops; lgkmcnt(N) every LDS op with
>= N later LDS ops (SMEM only at lgkmcnt(0)).

usage: python tools/waitcnt_check.py engine.s KERNEL_SUBSTRING"""
import re
import sys

REG = re.compile(r"\b([vsa])(\d+)\b|\b([vsa])\[(\d+):(\d+)\]")
CAP = 64


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            k, lo, hi = m.group(3), int(m.group(4)), int(m.group(5))
            out.update((k, r) for r in range(lo, hi + 1))
    return out


def split_ops(rest):
    ops, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            ops.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        ops.append(cur.strip())
    return ops


def classify(op, t):
    """(class, has_dest) of a memory op, or None.  class: vm / lds / smem."""
    if op.startswith(("global_load", "buffer_load", "scratch_load", "flat_load")):
        return "vm", "lds" not in t.split()[-1]
    if op.startswith(("global_atomic", "buffer_atomic", "flat_atomic")):
        return "vm", bool(re.search(r"\b(glc|sc0)\b", t))
    if op.startswith(("global_store", "buffer_store", "scratch_store", "flat_store", "buffer_wbl2", "buffer_inv")):
        return "vm", False
    if op.startswith("ds_"):
        if op.startswith(("ds_write", "ds_store")):
            return "lds", False
        if op.startswith(("ds_read", "ds_load", "ds_bpermute", "ds_permute", "ds_swizzle")) or "_rtn" in op:
            return "lds", True
        return "lds", False
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem", True
    return None


def parse(path, key):
    s = open(path).read()
    m = re.search(r"^(_Z\S*" + re.escape(key) + r"\S*):", s, re.M)
    if not m:
        sys.exit(f"no kernel matching {key}")
    i = m.start()
    j = s.index(".Lfunc_end", i)
    insts, labels = [], {}
    for ln in s[i:j].splitlines()[1:]:
        t = ln.split(";")[0].strip()
        if re.match(r"^\.LBB\d+_\d+:", t):
            labels[t[:-1]] = len(insts)
            continue
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        insts.append(t)
    return m.group(1), insts, labels


def succ(insts, labels, k):
    t = insts[k]
    op = t.split()[0]
    if op == "s_endpgm":
        return []
    if op == "s_branch":
        return [labels[t.split()[1]]]
    if op.startswith("s_cbranch"):
        return [labels[t.split()[1]], k + 1]
    return [k + 1]


def step(state, k, t):
    """Transfer function: state = {op index: (class, later count)}."""
    op = t.split()[0]
    st = dict(state)
    if op == "s_waitcnt":
        mv = re.search(r"vmcnt\((\d+)\)", t)
        ml = re.search(r"lgkmcnt\((\d+)\)", t)
        for i, (c, later) in list(st.items()):
            if c == "vm" and mv and later >= int(mv.group(1)):
                del st[i]
            elif c == "lds" and ml and later >= int(ml.group(1)):
                del st[i]
            elif c == "smem" and ml and int(ml.group(1)) == 0:
                del st[i]
        return st
    c = classify(op, t)
    if c:
        cls = c[0]
        same = ("lds",) if cls == "lds" else (cls,)
        for i, (c2, later) in list(st.items()):
            if c2 in same:
                st[i] = (c2, min(CAP, later + 1))
        st[k] = (cls, 0)
    return st


def join(a, b):
    if a is None:
        return dict(b)
    out = dict(a)
    for i, (c, later) in b.items():
        out[i] = (c, min(later, out[i][1])) if i in out else (c, later)
    return out


def main():
    name, insts, labels = parse(sys.argv[1], sys.argv[2])
    print(name, len(insts), "instructions")
    dests = {}
    for k, t in enumerate(insts):
        op = t.split()[0]
        c = classify(op, t)
        if c and c[1]:
            ops = split_ops(t[len(op):])
            dests[k] = regs(ops[0]) if ops else set()
    IN = [None] * len(insts)
    IN[0] = {}
    work = [0]
    while work:
        k = work.pop()
        out = step(IN[k], k, insts[k])
        for s2 in succ(insts, labels, k):
            if s2 >= len(insts):
                continue
            m = join(IN[s2], out)
            if m != IN[s2]:
                IN[s2] = m
                work.append(s2)
    bad = 0
    for k, t in enumerate(insts):
        if IN[k] is None or t.startswith("s_waitcnt"):
            continue
        op = t.split()[0]
        used = set()
        for o in split_ops(t[len(op):]):
            used |= regs(o)
        hits = []
        for i, (c, later) in IN[k].items():
            if i == k:
                continue
            h = used & dests.get(i, set())
            if h:
                hits.append((i, c, later, sorted(h)))
        if hits:
            bad += 1
            print(f"{k:5d}: {t}")
            for i, c, later, h in hits:
                print(f"        {c} op [{i}] (>= {later} later) {insts[i]}  regs {h[:6]}")
    print(bad, "instructions touch registers of possibly-incomplete loads")


if __name__ == "__main__":
    main()
