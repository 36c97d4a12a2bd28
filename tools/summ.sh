#!/bin/bash
# Summarise bench JSON lines in a directory.  usage: summ.sh DIR
for f in "$1"/*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); r=d['roofline']; print(f\"{'$(basename $f)':22s} {d['config']['algo']:8s} {d['value']:9.1f} Mpps frac {r['frac']:.4f} kernel {r['kernel_ms_mean']:.4f} ms\")"; done
