#!/usr/bin/env python3
"""Summarise an A/B directory written by tools/ab_tmp.sh: value and phase ms per log."""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, '*.log'))):
    try:
        line = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    r = line['roofline']
    ph = ' '.join(f'{k}={v * 1000:.1f}' for k, v in r['phase_ms'].items())
    print(f'{os.path.basename(f):24s} {line["value"] / 1e6:8.2f}M/s  {line["ms_per_step"] * 1000:8.1f}us  {ph}  frac={r["frac"]:.3f}')
