#!/usr/bin/env python3
"""Summarise tools/profile_pmc.sh output: per-kernel averages of every counter (per dispatch).

    tools/pmc_summary.py PMC_DIR [--json OUT.json]

With --json, also writes the per-kernel averages plus, per kernel, the corrected HBM traffic
(bench.py's roofline.traffic): bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 per launch, the
counter-executed flops, the L2 hit rate, the LDS bank-conflict share and the waiting share.
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
    res = {'source': d, 'kernels': summary, 'per_kernel': {}}
    for k, c in summary.items():
        e = {}
        if 'FETCH_SIZE' in c and 'WRITE_SIZE' in c:
            e['hbm_bytes_per_launch'] = (2 * c['FETCH_SIZE'] + c['WRITE_SIZE']) * 1024
        if 'SQ_INSTS_VALU_FLOPS_FP64' in c:
            # per-wave flop tallies (FMA = 2) x 64 lanes; MFMA ops in units of 512 flop
            e['executed_flops_per_launch'] = 64 * (c['SQ_INSTS_VALU_FLOPS_FP64'] + c.get('SQ_INSTS_VALU_FLOPS_FP32', 0.0)) \
                + 512 * c.get('SQ_INSTS_VALU_MFMA_MOPS_F32', 0.0)
        if c.get('TCC_HIT_sum') is not None and c.get('TCC_MISS_sum') is not None:
            e['l2_hit'] = c['TCC_HIT_sum'] / max(1.0, c['TCC_HIT_sum'] + c['TCC_MISS_sum'])
        if c.get('SQ_LDS_IDX_ACTIVE'):
            e['lds_bank_conflict_frac'] = c.get('SQ_LDS_BANK_CONFLICT', 0.0) / c['SQ_LDS_IDX_ACTIVE']
        if c.get('SQ_WAVE_CYCLES'):
            e['wait_frac'] = c.get('SQ_WAIT_ANY', 0.0) / c['SQ_WAVE_CYCLES']
        res['per_kernel'][k] = e
    json.dump(res, open(out, 'w'), indent=1)
    print('wrote', out)
