#!/usr/bin/env python3
"""Summarise tools/profile_pmc.sh output: per-kernel averages of every counter (per dispatch)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/pmc'
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r['Kernel_Name'].split('(')[0].replace('void ', '')
        vals[name][r['Counter_Name']].append(float(r['Counter_Value']))
for k, cs in vals.items():
    if 'mpcb' not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f'   {c:32s} {sum(v) / len(v):16.4g}   (n={len(v)})')
