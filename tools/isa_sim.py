#!/usr/bin/env python3
"""In-order issue model of one kernel's outermost loop body (one wave alone on its SIMD, the
situation of the c2 kernels): each instruction issues when the previous one has left the issue
slot and its source registers are ready.  Costs are the tools/micro/issue_check.hip measurements
on MI355X (cycles, s_memtime at the shader clock): every VALU instruction ~4.4 to issue (fp64,
fp32, DPP and v_cndmask alike), a dependent fp64 FMA back to back (4.6), a DPP FMA's result after
7.6, v_rcp_f64 / v_rsq_f64 16 per instruction.  Memory results are taken as ready (the loops
prefetch a stage ahead).  The estimate ranks schedules of one loop against each other; it is not
a cycle-accurate model (PMC: the c2 kernels spend ~25 % of their wave cycles in waits it omits).

    tools/isa_sim.py FILE.s MANGLED_KERNEL [--trace]
"""
import re
import sys

sys.path.insert(0, __import__('os').path.dirname(__file__))

ISSUE64, ISSUE32, LAT, LAT_DPP, LAT_TRANS, ISSUE_S = 4.4, 4.4, 4.6, 7.6, 20.0, 1.0


def loop_body(path, name):
    s = open(path).read()
    i = s.index(name + ':')
    j = s.index('.Lfunc_end', i)
    L = [l.strip() for l in s[i:j].split('\n')]
    hdrs = [l for l in L if 'Loop Header: Depth=1' in l]
    blocks, cur = [], None
    for k, l in enumerate(L):
        if l.startswith('.LBB') or l.startswith('; %bb.'):
            cur = [k, []]
            blocks.append(cur)
        elif cur is not None:
            cur[1].append(l)
    best = []
    for h in hdrs:   # the largest outermost loop
        bb = h.split(':')[0][2:]
        ins = []
        for k, body in blocks:
            head = L[k] + ' ' + (body[0] if body else '')
            if ('Header=' + bb) in head or L[k].startswith('.L' + bb + ':'):
                if any('trig_preop' in x or 'v_ldexp' in x for x in body):
                    continue
                ins += [x.split(';')[0].strip() for x in body if x and not x.startswith((';', '.'))]
        if len(ins) > len(best):
            best = ins
    ins = best
    return [x for x in ins if x]


REG = re.compile(r'\b([vsa])(\d+)\b|\b([vsa])\[(\d+):(\d+)\]|\b(vcc|exec|scc)\b')


def regs(txt):
    out = []
    for m in REG.finditer(txt):
        if m.group(1):
            out.append(m.group(1) + m.group(2))
        elif m.group(3):
            out += [m.group(3) + str(r) for r in range(int(m.group(4)), int(m.group(5)) + 1)]
        else:
            out.append(m.group(6))
    return out


def simulate(ins, trace=False):
    ready = {}
    t = 0.0
    tot_issue = 0.0
    for x in ins:
        op = x.split()[0]
        rest = x[len(op):]
        ops = [o.strip() for o in rest.split(',')] if rest.strip() else []
        store = op.startswith(('global_store', 'buffer_store', 'ds_write', 'scratch_store'))
        if op.startswith('s_') and not op.startswith(('s_load', 's_buffer')):
            if op.startswith(('s_waitcnt', 's_nop', 's_cbranch', 's_branch')):
                if op == 's_nop':
                    t += int(ops[0]) + 1 if ops else 1
                continue
            cost, lat = ISSUE_S, 2.0
        elif op.startswith(('global_load', 'buffer_load', 'ds_read', 'scratch_load', 's_load', 's_buffer')):
            cost, lat = 4.0, 0.0          # prefetched: treated as ready
        elif store:
            cost, lat = 4.0, 0.0
        elif op.startswith('v_'):
            wide = '_f64' in op or '_b64' in op or 'lshl_add_u64' in op or '_u64' in op
            cost = ISSUE64 if wide else ISSUE32
            lat = LAT
            if 'dpp' in op or 'row_newbcast' in x or 'quad_perm' in x or 'row_sh' in x:
                lat = LAT_DPP
            if op.startswith(('v_rcp', 'v_rsq', 'v_sqrt', 'v_sin', 'v_cos', 'v_exp', 'v_log')):
                lat = LAT_TRANS
                cost = 16.0
        else:
            cost, lat = 1.0, 2.0
        if store or op.startswith(('s_cmp', 'v_cmp')) and False:
            dst, src = [], regs(rest)
        else:
            dst = regs(ops[0]) if ops else []
            src = regs(','.join(ops[1:]))
            if op.startswith(('v_fmac', 'v_mac')):
                src += dst
        if store:
            dst, src = [], regs(rest)
        start = max([t] + [ready.get(r, 0.0) for r in src])
        t = start + cost
        tot_issue += cost
        for r in dst:
            ready[r] = start + lat
        if trace:
            print(f'{start:9.1f} {x}')
    return t, tot_issue


if __name__ == '__main__':
    ins = loop_body(sys.argv[1], sys.argv[2])
    t, issue = simulate(ins, '--trace' in sys.argv)
    print(f'{len(ins)} instructions: modelled {t:.0f} cycles per loop iteration (issue alone {issue:.0f}; '
          f'{t / max(len(ins), 1):.2f} per instruction)')
