"""CPU stand-in for BatchedMPC used ONLY by the bench launcher test (tests/test_bench_launch.py).

``bench.py --backend gloo --solver-stub tests.bench_stub`` runs the same launcher, rank setup,
StepPipeline and timed loop as the GPU bench, with this object in place of the HIP handle: its
solve is the NumPy oracle (test infrastructure), its inputs the oracle's Philox draws for the
rank's global ids, so the gathered u0 can be compared with an unsharded oracle solve.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from oracle.inputs import make_inputs
from oracle.ocp import OcpSpec, mpc_solve


# the stalled-rank case of the launcher test: this rank never reaches the rendezvous (bench.py
# imports the stub before init_process_group), so the others must fail within --init-timeout
if os.environ.get('BENCH_STUB_STALL_RANK') not in (None, '') and \
        os.environ.get('RANK') == os.environ['BENCH_STUB_STALL_RANK']:
    time.sleep(3600)


class _StubSolver:
    path = 'split'
    dtype = torch.float64

    def __init__(self, w, B):
        self.w, self.B = w, B
        box = w['box']
        self.spec = OcpSpec(N=w['N'], lbu=np.zeros(4) if box else None, ubu=np.full(4, 65.0) if box else None)
        self.timing = False
        self.stats = np.zeros((B, 2), dtype=np.int32)

    def gen_inputs(self, B, seed, id_offset=0, ref='hover', wind=False):
        inp = make_inputs(self.w['name'], ids=np.arange(id_offset, id_offset + B, dtype=np.uint64), N=self.w['N'])
        return inp

    def solve(self, x0, xref, uref, wind=None, want_traj=True, out=None):
        r = mpc_solve(x0, xref, uref, self.spec, wind=wind)
        out[0].copy_(torch.from_numpy(r['u0']))
        if want_traj:
            out[1].copy_(torch.from_numpy(r['X']))
            out[2].copy_(torch.from_numpy(r['U']))
        out[3].copy_(torch.from_numpy(r['status']))
        self.stats[:, 0] = r['iters']
        return out[0]

    def histogram(self, u0, lo=0.0, hi=65.0, nbins=64, counts=None):
        v = u0.double().numpy()
        b = np.clip(np.floor((v - lo) * (nbins / (hi - lo))), 0, nbins - 1).astype(np.int64)
        for m in range(v.shape[1]):
            counts[m] += torch.from_numpy(np.bincount(b[:, m], minlength=nbins))
        return counts

    def set_timing(self, on):
        self.timing = bool(on)

    def last_timing(self):
        return dict(nominal=0.01, riccati=0.02, forward=0.01)

    def last_kernels(self):
        return dict(nominal='stub::nominal', riccati='stub::riccati', forward='stub::forward')

    def qp_stats(self, B):
        return torch.from_numpy(self.stats[:B].copy())

    def close(self):
        pass


def make_solver(w, B):
    return _StubSolver(w, B)
