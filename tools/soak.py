#!/usr/bin/env python3
"""Determinism soak: every BASELINE workload (c2-c5 at its bench batch) and the 17/6 reference OCP
with both boxes solved repeatedly on one handle; every repetition's outputs must equal the first
bit for bit (the active set's work counter, the fallback list and the chunking hand instances to
waves in a different order each time, so this also checks that no result depends on scheduling).

    python tools/soak.py [--seconds 20]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_blaster_amd import BatchedMPC, MPCConfig  # noqa: E402

W = {   # bench.py WORKLOADS
    'c2': dict(batch=4096, N=20, dtype='f64', ref='hover', box=False, wind=False, seed=1002),
    'c3': dict(batch=65536, N=20, dtype='f32', ref='sine', box=False, wind=False, seed=1003),
    'c4': dict(batch=65536, N=30, dtype='f32', ref='hover', box=True, wind=False, seed=1004),
    'c5': dict(batch=131072, N=40, dtype='f32', ref='hover', box=False, wind=True, seed=1005),
}


def outputs(m):
    torch.cuda.synchronize()
    return [t.clone() for t in (m.get_control(), m.get_state_trajectory(), m.get_input_trajectory(),
                                m.get_status())]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--seconds', type=float, default=20.0)
    args = ap.parse_args()
    bad = 0
    for name, w in W.items():
        B, N = w['batch'], w['N']
        m = BatchedMPC(MPCConfig(N=N, dtype=w['dtype'], lbu=np.zeros(4) if w['box'] else None,
                                 ubu=np.full(4, 65.0) if w['box'] else None), max_batch=B)
        d = m.gen_inputs(B, seed=w['seed'], ref=w['ref'], wind=w['wind'])
        m.solve(d['x0'], d['xref'], d['uref'], wind=d['wind'])
        ref = outputs(m)
        t0, n, diff = time.time(), 0, 0
        while time.time() - t0 < args.seconds / (len(W) + 1):
            m.solve(d['x0'], d['xref'], d['uref'], wind=d['wind'])
            got = outputs(m)
            diff += sum(0 if torch.equal(a, b) else 1 for a, b in zip(got, ref))
            n += 1
        bad += diff
        print(f'{name}: {n} repeated solves of {B}, outputs differing from the first: {diff}', flush=True)
    # the hand-over paths: the hard-box draw (sine references, +-5 N wind) sends about a quarter of
    # its instances to the interior-point fallback and, in fp32, to the refinement kernel; both
    # queues are filled by atomics (c4's draws never reach the fallback)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
    from test_oracle_ocp import hard_box_inputs
    hb = hard_box_inputs(8192, 18, 11)
    for dt in ('f64', 'f32'):
        m = BatchedMPC(MPCConfig(N=18, dtype=dt, lbu=np.zeros(4), ubu=np.full(4, 65.0)), max_batch=8192)
        m.solve(hb['x0'], hb['xref'], hb['uref'], wind=hb['wind'])
        ref = outputs(m)
        t0, n, diff = time.time(), 0, 0
        while time.time() - t0 < args.seconds / (len(W) + 1):
            m.solve(hb['x0'], hb['xref'], hb['uref'], wind=hb['wind'])
            diff += sum(0 if torch.equal(a, b) else 1 for a, b in zip(outputs(m), ref))
            n += 1
        bad += diff
        print(f'hard box {dt}: {n} repeated solves of 8192, outputs differing from the first: {diff}', flush=True)
        del m
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from sbox_stall_study import draws   # the 17/6 bench draws (tools/bench_full17.py --bounds all)
    x0, xref, uref, p, lbu, ubu, lbx, ubx = draws(60, 1024)
    m = BatchedMPC(MPCConfig.full(N=60, lbu=lbu, ubu=ubu, lbx=lbx, ubx=ubx), max_batch=1024)
    m.set_params(p)
    args17 = (x0, xref, uref)
    m.solve(*args17)
    ref = outputs(m)
    t0, n, diff = time.time(), 0, 0
    while time.time() - t0 < args.seconds / (len(W) + 1):
        m.solve(*args17)
        got = outputs(m)
        diff += sum(0 if torch.equal(a, b) else 1 for a, b in zip(got, ref))
        n += 1
    bad += diff
    print(f'17/6 both boxes: {n} repeated solves of 1024, outputs differing from the first: {diff}', flush=True)
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()
