#!/usr/bin/env python3
"""Summarise tools/profile_pmc.sh output: per-kernel averages of every counter (per dispatch).

    tools/pmc_summary.py PMC_DIR [--json OUT.json]

With --json, also writes the per-kernel averages plus the corrected HBM traffic of the Riccati
kernel (bench.py's roofline.traffic): bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 per launch.
FETCH_SIZE/WRITE_SIZE are in KiB (rocprofiler-sdk counter_defs.yaml); on gfx950 FETCH_SIZE
tallies 128-B read requests at 64 B, hence the doubling (MI355X_MICROARCH.md, HBM section).
"""
import collections
import csv
import glob
import json
import os
import sys

args = [a for a in sys.argv[1:] if not a.startswith('--')]
d = args[0] if args else 'gpurun_out/pmc'
out = sys.argv[sys.argv.index('--json') + 1] if '--json' in sys.argv else None
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r['Kernel_Name'].split('(')[0].replace('void ', '')
        vals[name][r['Counter_Name']].append(float(r['Counter_Value']))
summary = {}
for k, cs in vals.items():
    if 'mpcb' not in k:
        continue
    summary[k] = {c: sum(v) / len(v) for c, v in sorted(cs.items())}
    print(k)
    for c, v in sorted(cs.items()):
        print(f'   {c:32s} {sum(v) / len(v):16.4g}   (n={len(v)})')
if out:
    ric = [k for k in summary if 'riccati_kernel' in k]
    res = {'source': d, 'kernels': summary}
    if ric:
        c = summary[ric[0]]
        if 'FETCH_SIZE' in c and 'WRITE_SIZE' in c:
            res['riccati_kernel'] = ric[0]
            res['hbm_bytes_per_riccati_launch'] = (2 * c['FETCH_SIZE'] + c['WRITE_SIZE']) * 1024
        if 'TCC_HIT_sum' in c and c.get('TCC_MISS_sum') is not None:
            res['riccati_l2_hit'] = c['TCC_HIT_sum'] / max(1.0, c['TCC_HIT_sum'] + c['TCC_MISS_sum'])
    json.dump(res, open(out, 'w'), indent=1)
    print('wrote', out)
