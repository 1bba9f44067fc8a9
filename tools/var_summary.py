#!/usr/bin/env python3
"""Print value / per-phase ms of gpurun_out/var_*.log (tools/var_bench.sh output)."""
import glob
import json
import os

for f in sorted(glob.glob('gpurun_out/var_*.log'), key=os.path.getmtime):
    for line in open(f):
        if line.startswith('{'):
            d = json.loads(line)
            ph = d['roofline']['phase_ms']
            out = f"{os.path.basename(f)[4:-4]:10s} {d['value']:.3e}  P1 {ph['nominal']:.4f} P2 {ph['riccati']:.4f} P3 {ph['forward']:.4f}  bad {d['bad_status']}"
            if 'secondary' in d:
                s = d['secondary']
                p3 = s['roofline']['phase_ms']
                out += f"  | c3 {s['value']:.3e}  P1 {p3['nominal']:.4f} P2 {p3['riccati']:.4f} P3 {p3['forward']:.4f}"
            print(out)
