"""Writes tests/golden/sbox_thin_interior.npz: two LP-feasible state-box QPs of
tools/bench_full17.py's distribution (the same generator) on which the interior point's Riccati
recursion loses positive definiteness before mu = 1e-8 (lambda / s ~ 1e16 on strongly active
rows): instance 301 of the B = 1024 draw (361 active state rows, largest interior margin 4.3e-3,
breakdown at mu = 2.5e-8) and instance 304 of the B = 4096 draw (breakdown at mu ~ 1e-6 on the
device, one iteration before the oracle's).  Inputs only; the expected values come from the
oracle in the test.

usage: python tools/make_sbox_fixture.py"""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def draw(B, idx):
    rng = np.random.default_rng(1017)            # tools/bench_full17.py's draw order
    x0 = np.zeros((B, 17))
    x0[:, 0:3] = rng.uniform(-1, 1, (B, 3))
    x0[:, 2] += 3.5
    x0[:, 3:6] = rng.uniform(-0.17, 0.17, (B, 3))
    x0[:, 6:9] = rng.uniform(-0.5, 0.5, (B, 3))
    x0[:, 9:12] = rng.uniform(-0.087, 0.087, (B, 3))
    p = np.zeros((B, 25))
    p[:, :24] = rng.uniform(-0.5, 0.5, (B, 24))
    p[:, 24] = 2.2 * 9.81
    lbx = np.array([-1.5, -1.5, 0, -0.174532925, -0.174532925, -0.349066, -1.0, -1.0, -1.0, -0.0872665,
                    -0.0872665, -0.0872665, -0.174532925, -0.523599, -1.5, -1.5, -2.5])
    ubx = -lbx
    ubx[[2, 12]] = 5.0, 1.22173
    x0 = np.clip(x0, 0.5 * lbx, 0.5 * ubx)
    x0[:, 2] = 3.5 + rng.uniform(-0.5, 0.5, B)
    return x0[idx], p[idx], lbx, ubx


def main():
    N = 60
    cases = [(1024, 301), (4096, 304)]
    d = [draw(B, i) for B, i in cases]
    np.savez(os.path.join(ROOT, 'tests', 'golden', 'sbox_thin_interior.npz'), x0=np.stack([c[0] for c in d]),
             p=np.stack([c[1] for c in d]), lbx=d[0][2], ubx=d[0][3], N=N, draw=np.array(cases))


if __name__ == '__main__':
    main()
