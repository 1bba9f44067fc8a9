#!/usr/bin/env python3
"""Summarise gpurun_out/<dir>/bench_*.log lines from tools/ab_p2.sh."""
import glob, json, os, sys
d = sys.argv[1]
for f in sorted(glob.glob(os.path.join('gpurun_out', d, 'bench_*.log'))):
    try:
        r = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, 'unparsable', e); continue
    ro = r['roofline']; sec = r.get('secondary') or {}
    print(f"{os.path.basename(f):24s} {r['value']:.4g} frac {ro['frac']:.3f} phases "
          + ' '.join(f"{k}={v*1e3:.1f}us" for k, v in ro['phase_ms'].items())
          + (f" | c3 {sec['value']:.4g}" if sec else ''))
