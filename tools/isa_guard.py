#!/usr/bin/env python3
"""Static guard over the gfx950 code objects inside a built library (or a
hipcc -S listing): no kernel may feed the LAST register of its VGPR
allocation to a 64-bit VALU instruction as a 32-bit operand.

Why (tools/v127_probe.hip): on MI355X, a 64-bit
instruction whose 32-bit operand sits in the allocation's top register —
`v_lshrrev_b64 v[116:117], v127, s[58:59]` in a 128-VGPR kernel — reads the
register past it as well, which belongs to the next wave on the SIMD (its
v0); the result then depends on that wave.  Probe: with every wave's v0 =
-1, 2.8 G of 34 G such shifts were wrong; the same shift reading v125, or a
32-bit shift reading v127, 0 of 34 G.  This is what made the NS = 7
pipelined walk lose IPv6 matches.  The compiler does not know the rule, so
every build is checked (tests/test_isa_guard.py).

usage: python tools/isa_guard.py LIB.so | LISTING.s"""
import os
import re
import struct
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
REG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
# 64-bit-class VALU opcodes (not the _e64 encoding suffix): *_b64, *_u64, *_i64, *_f64, *_u64_u32 ...
OP64 = re.compile(r"^v_\w*?_(?:[biuf]64)(?:_|$)")


def code_objects(lib: str):
    """The amdgcn code objects (ELF bytes) of every offload bundle in the
    library's .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat], check=True)
        data = open(fat, "rb").read()
    out = []
    p = data.find(MAGIC)
    while p >= 0:
        n = struct.unpack_from("<Q", data, p + 24)[0]
        q = p + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, q)
            q += 24
            triple = data[q:q + tl].decode()
            q += tl
            if "amdgcn" in triple and size:
                out.append((triple, data[p + off:p + off + size]))
        p = data.find(MAGIC, p + 1)
    return out


def disassemble(blob: bytes) -> str:
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(blob)
        f.flush()
        return subprocess.run([OBJDUMP, "-d", f.name], check=True, capture_output=True, text=True).stdout


def kernels_from_objdump(text: str):
    """name -> instruction lines (mnemonic + operands) of each function."""
    ks, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
        if m:
            cur = m.group(1)
            ks[cur] = []
            continue
        if cur is None:
            continue
        t = line.strip()
        if not t or t.startswith(";"):
            continue
        t = t.split("//")[0].strip()
        if t.startswith(("v_", "s_", "ds_", "global_", "buffer_", "flat_", "scratch_")):
            ks[cur].append(t)
    return ks


def kernels_from_listing(text: str):
    ks, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            ks[cur] = []
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
            continue
        t = line.split(";")[0].strip()
        if t.startswith(("v_", "s_", "ds_", "global_", "buffer_", "flat_", "scratch_")):
            ks[cur].append(t)
    return ks


def hazards(insts):
    """Instructions of one kernel that give a 64-bit VALU op a 32-bit
    operand in the allocation's last register (granule of 8)."""
    top = -1
    for t in insts:
        for m in REG.finditer(t):
            top = max(top, int(m.group(1) if m.group(1) else m.group(3)))
    if top < 0 or top % 8 != 7:
        return top, []  # the allocation's last register is never referenced
    bad = []
    for t in insts:
        op = t.split()[0]
        if not OP64.match(op):
            continue
        ops = [o.strip() for o in t[len(op):].split(",")]
        if any(o == f"v{top}" for o in ops):
            bad.append(t)
    return top, bad


def scan(path: str):
    """{kernel: (top register, offending instructions)} with hazards only."""
    if path.endswith(".s"):
        ks = kernels_from_listing(open(path).read())
    else:
        ks = {}
        for _, blob in code_objects(path):
            ks.update(kernels_from_objdump(disassemble(blob)))
    out = {}
    for name, insts in ks.items():
        top, bad = hazards(insts)
        if bad:
            out[name] = (top, bad)
    return out, len(ks)


def main():
    res, n = scan(sys.argv[1])
    for name, (top, bad) in res.items():
        print(f"{name}: top v{top}: {bad[:3]}")
    print(f"{len(res)} of {n} kernels feed their last VGPR to a 64-bit op")
    return 1 if res else 0


if __name__ == "__main__":
    sys.exit(main())
