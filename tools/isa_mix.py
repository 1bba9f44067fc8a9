#!/usr/bin/env python3
"""Instruction mix of one loop (by its header block) of one kernel in a hipcc -save-temps .s file
(host-only diagnostic; loop headers as tools/isa_loops.py -v prints them).

    tools/isa_mix.py FILE.s MANGLED_KERNEL_NAME LOOP_HEADER [--dump]
"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
i = s.index(sys.argv[2] + ':')
j = s.index('.Lfunc_end', i)
hdr = sys.argv[3].lstrip('.L')
cnt, body, cur, label = collections.Counter(), [], None, ''
for line in s[i:j].split('\n'):
    ls = line.strip()
    if ls.startswith('.LBB') or ls.startswith('; %bb.'):
        cur = None
        label = ls.split()[0].rstrip(':').lstrip('.L')
    m = re.search(r'Header=(\S+) Depth=(\d+)|Loop Header: Depth=(\d+)', ls)
    if m:
        h = (m.group(1) or '').lstrip('.L')
        if h == hdr or (m.group(3) and label == hdr):
            cur = True
    if cur and ls and not ls.startswith((';', '.')):
        cnt[ls.split()[0]] += 1
        body.append(ls)
print(hdr, sum(cnt.values()))
print(sorted(cnt.items(), key=lambda x: -x[1]))
if '--dump' in sys.argv:
    print('\n'.join(body))
