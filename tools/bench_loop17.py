#!/usr/bin/env python3
"""Batched closed loop on the reference's own OCP (simulation_blaster.py:56-107 for B instances at
once): acados_ocp_blasterModel.json (17/6, N = 60, input box + state box, the JSON's parameter
values), per step one SQP_RTI solve from the persistent iterate and the plant step, everything on
the device (mpc_blaster_amd.closed_loop).  Initial states: tools/make_loop17_fixture.py's
distribution (hover at z = 3 with small perturbations).  Prints one JSON line: solves/s over the
whole loop (B * NSIM / wall time), the per-step wall time and the statuses of all steps.

    python tools/bench_loop17.py [--batch 4096] [--nsim 20] [--warmup-steps 2]
"""
import argparse
import json
import os
import sys
import time
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=4096)
    ap.add_argument('--nsim', type=int, default=20)
    ap.add_argument('--warmup-steps', type=int, default=2)
    args = ap.parse_args()
    import torch

    from mpc_blaster_amd import BatchedMPC, load_acados_ocp_json
    from mpc_blaster_amd.closed_loop import closed_loop
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        cfg, info = load_acados_ocp_json(os.path.join(ROOT, 'tests', 'golden', 'ocp_json_pin.json'))
    B, N = args.batch, cfg.N
    rng = np.random.default_rng(2027)
    yref = info['yref']
    x0 = np.tile(yref[:17], (B, 1))
    x0[:, 2] = 3.0
    x0[:, 0:3] += rng.uniform(-0.3, 0.3, (B, 3))
    x0[:, 3:6] += rng.uniform(-0.05, 0.05, (B, 3))
    x0[:, 6:9] += rng.uniform(-0.2, 0.2, (B, 3))
    x0[:, 9:12] += rng.uniform(-0.02, 0.02, (B, 3))
    xref = np.where(np.arange(17) == 2, 3.5, yref[:17])
    xref = np.where(np.arange(17) == 14, 0.2, xref)
    uref = np.r_[np.full(4, 22.0725), yref[21:23]]
    m = BatchedMPC(cfg, max_batch=B)
    dev = f'cuda:{m.device}'
    m.set_params(torch.as_tensor(np.tile(info['p'], (B, 1)), dtype=m.dtype, device=dev))
    x0t = torch.as_tensor(x0, dtype=m.dtype, device=dev)
    xr = torch.as_tensor(np.broadcast_to(xref, (1, N + 1, 17)).copy(), dtype=m.dtype, device=dev)
    ur = torch.as_tensor(np.broadcast_to(uref, (1, N, 6)).copy(), dtype=m.dtype, device=dev)
    if args.warmup_steps:
        closed_loop(m, x0t, xr, ur, args.warmup_steps)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Xs, Us, st = closed_loop(m, x0t, xr, ur, args.nsim)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    sc = np.bincount(st.cpu().numpy(), minlength=5).tolist()
    print(json.dumps({'metric': f'closed-loop MPC solves/sec (reference OCP, 17/6, N={N}, input + state box)',
                      'value': B * args.nsim / el, 'unit': 'solves/s', 'ms_per_step': el / args.nsim * 1e3,
                      'batch': B, 'nsim': args.nsim, 'dtype': 'f64',
                      'worst_status_counts': sc,
                      'final_x_finite': bool(torch.isfinite(Xs[:, -1]).all().item()),
                      'config': 'acados_ocp_blasterModel.json via load_acados_ocp_json; persistent iterate '
                                '(zeros at start), plant = one RK4 step of Tf/N; x0 hover z=3 +- small'}))


if __name__ == '__main__':
    main()
