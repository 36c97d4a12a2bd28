"""Index statistics of a compiled table for a synthetic config: per key slot
(rules, buckets, entries, longest list) and the per-packet / per-wave walk
lengths the INDEXED kernel pays (loop trips = max over slots of entries walked;
a wave pays the max over its 64 lanes).  CPU only (nffacl_table_compile).
usage: python tools/index_stats.py c5 [n_packets]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "nff-go_amd"), str(ROOT / "tests")]

import numpy as np  # noqa: E402

import nffacl  # noqa: E402
from nffacl import synth  # noqa: E402
from test_index_compile import compile_table, fields, match, KEYS  # noqa: E402


def walk(blob, info, F, n):
    trips = np.zeros(n, np.int64)
    reads = np.zeros(n, np.int64)
    best = np.full(n, 0xFFFFFFFF, np.uint64)
    for fam, v6 in ((0, False), (1, True)):
        fi = info.fam[fam]
        ew = fi.entry_dwords
        mine = F["is6"] if v6 else F["is4"]
        for d in range(4):
            di = fi.dims[d]
            if di.n_rules == 0:
                continue
            key = KEYS[di.kind](F).astype(np.uint64)
            dirv = blob[di.off_dir:di.off_dir + di.n_buckets + 1].astype(np.int64)
            t = (key >> np.uint64(di.shift)).astype(np.int64)
            start, end = dirv[t], dirv[t + 1]
            start0 = start.copy()
            for k in range(di.max_list):
                live = mine & (start < end)
                if not live.any():
                    break
                sel = np.nonzero(live)[0]
                ok, idx, out = match(blob, di.off_entries + start[sel] * ew, v6, F, sel)
                keep = idx < best[sel]
                ok &= keep
                best[sel[ok]] = idx[ok]
                stop = ok | ~keep
                start[sel] += 1
                start[sel[stop]] = end[sel[stop]] + 0
                reads[sel] += 1
            # note: trips approximated by max walked per slot (order-dependent)
            walked = np.where(mine, np.minimum(end - start0, 1 << 30), 0)
    return best, reads


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 14
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    rules = nffacl.L3Rules.parse_text(g.text)
    blob, info = compile_table(rules)
    print(f"{cfg}: blob {blob.nbytes/1e6:.2f} MB")
    for fam in range(2):
        fi = info.fam[fam]
        print(f" fam {fam}: n_rec {fi.n_rec} resid {fi.n_resid}")
        for d in range(4):
            di = fi.dims[d]
            dirv = blob[di.off_dir:di.off_dir + di.n_buckets + 1].astype(np.int64)
            ln = np.diff(dirv)
            print(f"  dim {d} kind {di.kind} rules {di.n_rules} buckets {di.n_buckets} shift {di.shift} "
                  f"entries {di.n_entries} max_list {di.max_list} mean_list {ln.mean():.2f} "
                  f"bytes {(di.n_entries*fi.entry_dwords*4 + 4*len(dirv))/1e6:.2f} MB")
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS[cfg]) if cfg != "c3" else synth.gen_slots(g, n, 3)
    F = fields(slots, n)
    best, reads = walk(blob, info, F, n)
    w = reads[: n // 64 * 64].reshape(-1, 64)
    print(f" entries read per packet: mean {reads.mean():.2f} p50 {np.median(reads)} p99 {np.percentile(reads, 99)} "
          f"max {reads.max()}; per-wave max mean {w.max(1).mean():.2f}")


if __name__ == "__main__":
    main()
