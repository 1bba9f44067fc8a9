#!/usr/bin/env python3
"""Instruction mix of the outermost loop body of one kernel in a hipcc -save-temps .s file,
without the blocks of the ocml sin/cos fallback that holds v_trig_preop / v_ldexp (never taken
on flying attitudes).  Still counted: ocml's medium-range reduction blocks, also not taken.

    tools/isa_loop.py FILE.s MANGLED_KERNEL_NAME
"""
import re,collections,sys
s=open(sys.argv[1]).read(); name=sys.argv[2]
i=s.index(name+':'); j=s.index('.Lfunc_end',i)
L=[l.strip() for l in s[i:j].split('\n')]
hdrs=[l for l in L if 'Loop Header: Depth=1' in l]
bb=hdrs[0].split(':')[0][2:]
blocks=[];cur=None
for k,l in enumerate(L):
    if l.startswith('.LBB') or l.startswith('; %bb.'):
        cur=[k,[]]; blocks.append(cur)
    elif cur is not None: cur[1].append(l)
ins=[]
for k,body in blocks:
    head=L[k]+' '+(body[0] if body else '')
    if ('Header='+bb) in head or L[k].startswith('.L'+bb+':'):
        if any('trig_preop' in x or 'v_ldexp' in x for x in body): continue
        ins+= [x for x in body if x and not x.startswith((';','.'))]
c=collections.Counter(x.split()[0] for x in ins)
print('loop fast-path instrs ~',len(ins))
print(sorted(c.items(),key=lambda x:-x[1])[:34])
