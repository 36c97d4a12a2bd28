R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/batcher_spin2"; mkdir -p "$OUT"; cd "$R"
python tools/batcher_bench.py "$OUT/in" || exit 1
for sp in 13 4 0; do for tb in 1:1 8:1 32:1 1:32 16:32 32:32 64:32; do
  t=${tb%:*}; b=${tb#*:}
  NFFACL_TUNE_BATCH_SPIN=$sp timeout -k 10 60 ./tools/batcher_bench "$OUT/in/rules.conf" "$OUT/in/slots.bin" 80 $t $b 8192 100 2 > "$OUT/r.json" 2>> "$OUT/sweep.err" || exit 1
  python3 -c "import json,sys;d=json.load(open('$OUT/r.json'));d['spin']=$sp;print(json.dumps(d))" >> "$OUT/sweep.jsonl"
done; done
rm -rf "$OUT/in"
