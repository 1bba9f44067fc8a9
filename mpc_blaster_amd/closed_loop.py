"""Device-resident closed-loop Monte-Carlo: the receding-horizon loop of
src/scripts/simulation_blaster.py:56-107 for a whole batch, without leaving the GPU.

Per step (one batch launch each): SQP_RTI solve from the persistent iterate (acados keeps the
iterate between ``solve()`` calls and does not shift it; initial iterate = zeros), then the
plant integrator (AcadosSimSolver: one RK4 step of Tsim = Tf/N, JSON ``Tsim``) applies u0*.
"""
from __future__ import annotations

from .api import BatchedMPC


def closed_loop(mpc: BatchedMPC, x0, x_ref, u_ref, nsim: int, wind=None, plant_T=None,
                xbar=None, ubar=None):
    """Returns (X_sim [B, nsim+1, nx], U_sim [B, nsim, nu], status [B] = max over steps)."""
    import torch
    dev = f'cuda:{mpc.device}'
    dt = mpc.dtype
    x = torch.as_tensor(x0, dtype=dt, device=dev).contiguous()
    B, N = x.shape[0], mpc.cfg.N
    NX, NU = mpc.nx, mpc.nu
    xb = torch.zeros((B, N + 1, NX), dtype=dt, device=dev) if xbar is None else \
        torch.as_tensor(xbar, dtype=dt, device=dev).clone()
    ub = torch.zeros((B, N, NU), dtype=dt, device=dev) if ubar is None else \
        torch.as_tensor(ubar, dtype=dt, device=dev).clone()
    u0 = torch.empty((B, NU), dtype=dt, device=dev)
    st = torch.empty((B,), dtype=torch.int32, device=dev)
    worst = torch.zeros((B,), dtype=torch.int32, device=dev)
    Xs = torch.empty((B, nsim + 1, NX), dtype=dt, device=dev)
    Us = torch.empty((B, nsim, NU), dtype=dt, device=dev)
    Xs[:, 0] = x
    for i in range(nsim):
        mpc.solve_iterate(x, xb, ub, x_ref, u_ref, wind=wind, out=(u0, xb, ub, st))
        worst = torch.maximum(worst, st)
        Us[:, i] = u0
        x = mpc.sim_step(x, u0, T=plant_T, wind=wind)
        Xs[:, i + 1] = x
    return Xs, Us, worst
