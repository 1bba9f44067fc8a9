#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -save-temps .s file.

    tools/isa_stats.py FILE.s KERNEL_SUBSTRING [--waits]
"""
import collections
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
s = open(path).read()
for m in re.finditer(r'^(\S+):\s+; @', s, re.M):
    name = m.group(1)
    if pat not in name:
        continue
    j = s.index('.Lfunc_end', m.end())
    lines = [l.strip() for l in s[m.end():j].split('\n')]
    ops = collections.Counter(l.split()[0] for l in lines if l and not l.startswith((';', '.')) and not l.endswith(':'))
    print(name, 'instructions', sum(ops.values()))
    for op, n in sorted(ops.items(), key=lambda x: -x[1])[:40]:
        print(f'   {op:32s} {n}')
    if '--waits' in sys.argv:
        for i, l in enumerate(lines):
            if 'vmcnt' in l:
                print('   ', i, l)
