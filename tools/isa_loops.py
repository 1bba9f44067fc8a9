#!/usr/bin/env python3
"""Instructions and SGPR-spill lane moves (v_readlane / v_writelane) of one kernel by loop depth,
from a hipcc -save-temps .s file (host-only diagnostic).

    tools/isa_loops.py FILE.s MANGLED_KERNEL_NAME [-v]
"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
blocks, cur = [], None
for line in s[i:j].split('\n'):
    ls = line.strip()
    if ls.startswith('.LBB') or ls.startswith('; %bb.'):
        cur = {'label': ls.split()[0], 'ins': [], 'depth': 0, 'hdr': None}
        blocks.append(cur)
    if cur is None:
        continue
    m = re.search(r'Header=(\S+) Depth=(\d+)|Loop Header: Depth=(\d+)', ls)
    if m:
        cur['depth'] = int(m.group(2) or m.group(3))
        cur['hdr'] = m.group(1) or cur['label']
    if ls and not ls.startswith((';', '.')):
        cur['ins'].append(ls.split()[0])
tot = collections.defaultdict(lambda: [0, 0, 0])
per_loop = collections.defaultdict(lambda: [0, 0])
for b in blocks:
    lanes = sum(1 for x in b['ins'] if x in ('v_readlane_b32', 'v_writelane_b32'))
    scr = sum(1 for x in b['ins'] if 'scratch' in x or 'buffer_store' in x or 'buffer_load' in x)
    t = tot[b['depth']]
    t[0] += len(b['ins']); t[1] += lanes; t[2] += scr
    if b['hdr']:
        p = per_loop[(b['depth'], b['hdr'])]
        p[0] += len(b['ins']); p[1] += lanes
print('depth: instructions, readlane+writelane, scratch ops')
for d in sorted(tot):
    print(f'  {d}: {tot[d]}')
if '-v' in sys.argv:
    for (d, h), (n, l) in sorted(per_loop.items()):
        print(f'  loop {h} depth {d}: {n} instructions, {l} lane moves')
