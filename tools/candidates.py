#!/usr/bin/env python3
"""Candidates per packet of the HYBRID table (CPU, no device): compiles a
synthetic config's rules with nffacl_table_compile, looks every packet of a
2^16 sample up in each slot's directory (the kernel's lookup, restated by the
tests/test_index_compile.py helpers) and prints per-slot list lengths, the
candidates per packet, how many pass the full rule test, and the flat walk's
rounds per 64-packet batch.  Layout knobs (NFFACL_TUNE_*) apply.
usage: python tools/candidates.py c3|c5"""
import sys, numpy as np
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / 'nff-go_amd'), str(ROOT / 'tests')]
import nffacl
from nffacl import synth
from test_index_compile import compile_table, fields, dir_values, bucket_of, hyb_test
cfg=sys.argv[1]
g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
n=1<<16
slots = synth.gen_slots(g, n, synth.PACKET_SEEDS[cfg])
rules = nffacl.L3Rules.parse_text(g.text)
blob, info = compile_table(rules, nffacl.ALGO_HYBRID)
F=fields(slots,n)
tot=np.zeros(n,np.int64); passes=np.zeros(n,np.int64)
for fam,v6 in ((0,False),(1,True)):
    fi=info.fam[fam]; mine=F["is6"] if v6 else F["is4"]
    print("fam",fam,"slots",fi.n_slots,"resid",fi.n_resid, "ew",fi.entry_dwords)
    for d in range(fi.n_slots):
        di=fi.dims[d]
        if di.n_rules==0: continue
        dirv=dir_values(blob,di); t=bucket_of(di,F)
        ln=np.where(mine, dirv[t+1]-dirv[t],0)
        tot+=ln
        print(f"  slot {d} kind {di.kind} shift {di.shift} nb {di.n_buckets} rules {di.n_rules} ents {di.n_entries} maxlist {di.max_list} mean cand {ln[mine].mean():.2f}")
        start=dirv[t]
        for k in range(di.max_list):
            live=mine&(k<ln)
            if not live.any(): break
            sel=np.nonzero(live)[0]
            ok,_,_=hyb_test(blob,info,fi.off_ent_base+(start[sel]+k)*fi.entry_dwords,v6,F,sel)
            passes[sel]+=ok
ip=F["is4"]|F["is6"]
print("mean cand/packet (IP)", tot[ip].mean(), " overall", tot.mean(), "pass", passes[ip].mean())
T=tot.reshape(-1,64).sum(1)
rounds=np.ceil(T/64)  # adaptive last window: only the rounds its candidates fill
print("T/batch mean",T.mean(),"p50",np.median(T),"p90",np.percentile(T,90),"max",T.max())
print("rounds executed mean",rounds.mean()," useful",(T/64).mean())
print("hist of cand per packet", np.bincount(np.minimum(tot,40))[:41])
