"""Per-instance device statuses of tools/bench_full17.py's state-box draw (same generator), saved
to gpurun_out/full17_status_<B>.npy for a comparison with oracle.ocp.lp_box_feasible on the CPU.

usage (GPU box): python tools/full17_status.py [B]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from mpc_blaster_amd import BatchedMPC, MPCConfig
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    N = 60
    rng = np.random.default_rng(1017)
    x0 = np.zeros((B, 17))
    x0[:, 0:3] = rng.uniform(-1, 1, (B, 3))
    x0[:, 2] += 3.5
    x0[:, 3:6] = rng.uniform(-0.17, 0.17, (B, 3))
    x0[:, 6:9] = rng.uniform(-0.5, 0.5, (B, 3))
    x0[:, 9:12] = rng.uniform(-0.087, 0.087, (B, 3))
    xref = np.zeros((1, N + 1, 17))
    xref[..., 2], xref[..., 14] = 3.5, 0.2
    uref = np.zeros((1, N, 6))
    uref[..., :4] = 22.0725
    p = np.zeros((B, 25))
    p[:, :24] = rng.uniform(-0.5, 0.5, (B, 24))
    p[:, 24] = 2.2 * 9.81
    lbu = np.array([0.0, 0.0, 0.0, 0.0, -0.0872665, -0.0872665])
    ubu = np.array([65.0, 65.0, 65.0, 65.0, 0.0872665, 0.0872665])
    lbx = np.array([-1.5, -1.5, 0, -0.174532925, -0.174532925, -0.349066, -1.0, -1.0, -1.0, -0.0872665,
                    -0.0872665, -0.0872665, -0.174532925, -0.523599, -1.5, -1.5, -2.5])
    ubx = -lbx
    ubx[[2, 12]] = 5.0, 1.22173
    x0 = np.clip(x0, 0.5 * lbx, 0.5 * ubx)
    x0[:, 2] = 3.5 + rng.uniform(-0.5, 0.5, B)
    m = BatchedMPC(MPCConfig.full(N=N, lbu=lbu, ubu=ubu, lbx=lbx, ubx=ubx), max_batch=B)
    m.set_params(p)
    m.solve(x0, xref, uref)
    torch.cuda.synchronize()
    st = m.get_status().cpu().numpy()
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    np.save(os.path.join(ROOT, 'gpurun_out', f'full17_status_{B}.npy'), st)
    print('statuses', np.bincount(st), 'failed', np.where(st != 0)[0].tolist())


if __name__ == '__main__':
    main()
