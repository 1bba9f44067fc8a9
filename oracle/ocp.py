"""One Gauss-Newton SQP_RTI step of the BLASTER LINEAR_LS OCP (oracle; test infrastructure only).

Problem (``blastermodel.py:226-287``; numbers pinned by ``acados_ocp_blasterModel.json``):

    min  sum_{k<N} s_k/2 (|x_k - xr_k|_Q^2 + |u_k - ur_k|_R^2) + 1/2 |x_N - xr_N|_QN^2
    s.t. x_0 = x0                               (lbx_0 = ubx_0 = x, simulation_blaster.py:60-61)
         x_{k+1} = Phi(x_k, u_k)                 (RK4, oracle.rk4)
         lbu <= u_k <= ubu                       (idxbu, blastermodel.py:261-264; optional)

W = blkdiag(Q, R), W_e = QN (``blastermodel.py:244-245``); V are selectors (``:247-254``) so
the Gauss-Newton Hessian is blkdiag(Q, R).  s_k = cost_scale (default dt = Tf/N) for k < N,
1 at the terminal stage: the acados template sets the LS cost "scaling" to ``time_steps[k]``
[acados 0.1.x convention, third-party, unpinned — switchable via ``cost_scale``].

SQP_RTI (``nlp_solver_type='SQP_RTI'``, JSON ``globalization=FIXED_STEP``,
``nlp_solver_step_length=1.0``): linearise at the iterate (xbar, ubar), solve the LQ QP in
(dx, du) with gaps b_k = Phi(xbar_k, ubar_k) - xbar_{k+1}, take the full step.  ``X`` is the
linear prediction xbar + dx (what ``ocp_solver.get(k, 'x')`` returns), ``U = ubar + du``.

Two linearisation modes:

* ``rollout`` (the batch ``solve(x0, x_ref, u_ref)`` surface): ubar = u_ref, xbar = RK4 rollout
  from x0 (gap-free, dx_0 = 0).
* ``iterate`` (the acados facade): xbar, ubar supplied (the persistent SQP_RTI iterate).

QP solvers here:

* ``riccati_solve``: Riccati recursion (HPIPM's OCP-QP structure; the QP is strictly convex so
  its minimiser is unique and method-independent).  Input boxes are handled by an exact
  primal-dual active-set loop (with the Kim-Park block-principal-pivoting safeguard) around a
  masked Riccati — the same algorithm the device
  runs.  HPIPM instead uses an interior-point method; both converge to the same unique
  minimiser, to within HPIPM's tolerance.  [parity unpinned: HPIPM absent]
* ``dense_box_qp`` (tests only): condensed QP solved by SciPy BVLS, an independent exact check.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .model import Params, f12
from .rk4 import rk4_sens, rk4_step

NX, NU = 12, 4
STATUS_OK, STATUS_NAN, STATUS_MAXITER, STATUS_MINSTEP, STATUS_QP_FAIL = 0, 1, 2, 3, 4   # acados' codes


def default_Q() -> np.ndarray:
    # simulation_blaster.py:24 sliced to the 12 rigid-body states (JSON cost.W diag[0:12])
    return np.diag([1e3] * 6 + [5.0] * 3 + [10.0] * 3)


def default_R() -> np.ndarray:
    # simulation_blaster.py:27 sliced to the 4 motor thrusts (JSON cost.W diag[17:21])
    return np.diag([0.05] * 4)


@dataclass
class OcpSpec:
    N: int = 20
    dt: float = 1.0 / 30.0
    Q: np.ndarray = field(default_factory=default_Q)
    R: np.ndarray = field(default_factory=default_R)
    QN: np.ndarray | None = None            # default 10 * Q (simulation_blaster.py:25)
    cost_scale: float | None = None         # default dt (acados time_steps scaling)
    lbu: np.ndarray | None = None           # None -> unconstrained
    ubu: np.ndarray | None = None
    params: Params = field(default_factory=Params)
    max_as_iter: int = 200

    def __post_init__(self):
        if self.QN is None:
            self.QN = 10.0 * np.asarray(self.Q)

    @property
    def s(self) -> float:
        return self.dt if self.cost_scale is None else self.cost_scale

    @property
    def boxed(self) -> bool:
        return self.lbu is not None


def rollout(x0, ubar, spec: OcpSpec, wind=None):
    B = x0.shape[0]
    X = np.empty((B, spec.N + 1, NX))
    X[:, 0] = x0
    for k in range(spec.N):
        X[:, k + 1] = rk4_step(X[:, k], ubar[:, k], spec.dt, spec.params, wind)
    return X


def linearise(xbar, ubar, spec: OcpSpec, wind=None):
    """A_k, B_k, gaps b_k at the iterate."""
    B = xbar.shape[0]
    N = spec.N
    A = np.empty((B, N, NX, NX))
    Bm = np.empty((B, N, NX, NU))
    gap = np.empty((B, N, NX))
    for k in range(N):
        xn, A[:, k], Bm[:, k] = rk4_sens(xbar[:, k], ubar[:, k], spec.dt, spec.params, wind)
        gap[:, k] = xn - xbar[:, k + 1]
    return A, Bm, gap


def _masked_stage(Huu, Hux, hu, fixed, delta):
    """Eliminate fixed input components (value du_m = delta_m) from the stage QP."""
    Ht = Huu.copy()
    Hxt = Hux.copy()
    ht = hu.copy()
    if fixed is not None and fixed.any():
        # free rows: h_F += H_FA delta_A
        ht = ht + np.einsum('bij,bj->bi', Huu, np.where(fixed, delta, 0.0))
        eye = np.eye(Huu.shape[-1])[None]
        fr = fixed[:, :, None] | fixed[:, None, :]
        diag = fixed[:, :, None] & fixed[:, None, :] & (eye > 0)
        Ht = np.where(fr, 0.0, Ht)
        Ht = np.where(diag, 1.0, Ht)
        Hxt = np.where(fixed[:, :, None], 0.0, Hxt)
        ht = np.where(fixed, -delta, ht)
    return Ht, Hxt, ht


def riccati_solve(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec: OcpSpec,
                  fixed=None, delta=None, Rd=None, rd=None, Qd=None, qd=None):
    """Solve the (masked) LQ QP.  Returns dx (B,N+1,nx), du (B,N,nu), mu (B,N,nu), ok (B,).
    Dimensions come from A (nx) and Bm (nu): the 12/4 slice and the 17/6 model share it.
    Rd, rd (B,N,nu) / Qd, qd (B,N,nx): extra diagonal input / state Hessian and gradient per
    stage k < N (the barrier terms of ``ipm_box_solve``)."""
    Bsz, N = xbar.shape[0], spec.N
    NX, NU = A.shape[-1], Bm.shape[-1]
    s = spec.s
    Q, R, QN = (np.asarray(M, dtype=np.float64) for M in (spec.Q, spec.R, spec.QN))
    P = np.broadcast_to(QN, (Bsz, NX, NX)).copy()
    p = np.einsum('ij,bj->bi', QN, xbar[:, N] - xref[:, N])
    K = np.empty((Bsz, N, NU, NX))
    kff = np.empty((Bsz, N, NU))
    Huus = np.empty((Bsz, N, NU, NU))
    Huxs = np.empty((Bsz, N, NU, NX))
    hus = np.empty((Bsz, N, NU))
    ok = np.ones(Bsz, dtype=bool)
    for k in range(N - 1, -1, -1):
        Ak, Bk, bk = A[:, k], Bm[:, k], gap[:, k]
        pt = p + np.einsum('bij,bj->bi', P, bk)
        PA = np.einsum('bij,bjk->bik', P, Ak)
        PB = np.einsum('bij,bjk->bik', P, Bk)
        Hxx = s * Q + np.einsum('bji,bjk->bik', Ak, PA)
        Hux = np.einsum('bji,bjk->bik', Bk, PA)
        Huu = s * R + np.einsum('bji,bjk->bik', Bk, PB)
        hx = s * np.einsum('ij,bj->bi', Q, xbar[:, k] - xref[:, k]) + np.einsum('bji,bj->bi', Ak, pt)
        hu = s * np.einsum('ij,bj->bi', R, ubar[:, k] - uref[:, k]) + np.einsum('bji,bj->bi', Bk, pt)
        if Rd is not None:
            Huu = Huu + Rd[:, k, :, None] * np.eye(NU)[None]
            hu = hu + rd[:, k]
        if Qd is not None:
            Hxx = Hxx + Qd[:, k, :, None] * np.eye(NX)[None]
            hx = hx + qd[:, k]
        fk = None if fixed is None else fixed[:, k]
        dk = None if delta is None else delta[:, k]
        Ht, Hxt, ht = _masked_stage(Huu, Hux, hu, fk, dk)
        try:
            L = np.linalg.cholesky(Ht)
        except np.linalg.LinAlgError:   # rare: find the failing instances one by one
            ev_ok = np.ones(Bsz, dtype=bool)
            for b in range(Bsz):
                try:
                    np.linalg.cholesky(Ht[b])
                except np.linalg.LinAlgError:
                    ev_ok[b] = False
            ok &= ev_ok
            Ht = np.where(ev_ok[:, None, None], Ht, np.eye(NU)[None])
            Hxt = np.where(ev_ok[:, None, None], Hxt, 0.0)
            ht = np.where(ev_ok[:, None], ht, 0.0)
            L = np.linalg.cholesky(Ht)
        Kk = -np.linalg.solve(Ht, Hxt)
        kk = -np.linalg.solve(Ht, ht[..., None])[..., 0]
        K[:, k], kff[:, k] = Kk, kk
        Huus[:, k], Huxs[:, k], hus[:, k] = Huu, Hux, hu
        P = Hxx + np.einsum('bji,bjk->bik', Hux, Kk)
        P = 0.5 * (P + np.swapaxes(P, 1, 2))
        p = hx + np.einsum('bji,bj->bi', Hux, kk)
        del L
    dx = np.empty((Bsz, N + 1, NX))
    du = np.empty((Bsz, N, NU))
    mu = np.empty((Bsz, N, NU))
    dx[:, 0] = dx0
    for k in range(N):
        du[:, k] = np.einsum('bij,bj->bi', K[:, k], dx[:, k]) + kff[:, k]
        mu[:, k] = (np.einsum('bij,bj->bi', Huus[:, k], du[:, k])
                    + np.einsum('bij,bj->bi', Huxs[:, k], dx[:, k]) + hus[:, k])
        dx[:, k + 1] = (np.einsum('bij,bj->bi', A[:, k], dx[:, k])
                        + np.einsum('bij,bj->bi', Bm[:, k], du[:, k]) + gap[:, k])
    return dx, du, mu, ok


# The 12/4 input box's fallback: an instance whose active set has not converged after
# min(max_as_iter, AS_IPM_AFTER) passes is solved again by the interior point (ipm_box_solve with
# the adaptive centring, input rows only, at most AS_IPM_ITERS iterations).  The least-index backup
# rule terminates finitely but can need thousands of passes: with a +-5 N wind and sine references
# (N = 18) 262 of 3000 instances took more than 60, one more than 1500, where the interior point
# needs at most 24 iterations; on the c4 bench draws the active set needs at most 39 passes, so
# the fallback never runs there.
AS_IPM_AFTER, AS_IPM_ITERS = 48, 100
# ... and an instance whose first pass (the unconstrained solution) violates more than 7/20 of the
# horizon's input components is handed over at once: on strongly constrained draws (sine
# references, the iterate perturbed by 0.05 / 1 N, N = 11) 801 of the 803 of 1500 instances that
# need more than 48 passes violate more than 16 of 44 after the first, and the instances there
# that the active set does finish need ~19 passes, as many as the interior point's iterations;
# on the c4 draws no instance violates more than 19 of 120 (tools/box_ipm_direct.py)
AS_IPM_NV_NUM, AS_IPM_NV_DEN = 7, 20


def pdas_solve(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec: OcpSpec, pbar: int = 3):
    """Exact input-box QP: primal-dual active set with the Kim-Park block-principal-pivoting
    safeguard (finite termination for the SPD reduced Hessian, a P-matrix LCP).

    Each iteration solves the equality-constrained LQ problem with the current sets (masked
    Riccati), then collects the infeasible set V = {free u < lb} U {free u > ub} U
    {u at lb with mu < 0} U {u at ub with mu > 0}.  |V| = 0 means the KKT conditions hold.
    Full exchange of V while |V| keeps decreasing (or for ``pbar`` tries); otherwise only the
    element of V with the least index k*nu + m is exchanged (Murty's least-index backup rule,
    finite for a P-matrix LCP).  Measured on 2000 c4 instances: the least index converges in at
    most 28 iterations where the largest index needs up to 132 (mean 3.8 vs 4.0).  Instances not
    converged after min(max_as_iter, AS_IPM_AFTER) passes, or whose first pass violates more than
    AS_IPM_NV_NUM / AS_IPM_NV_DEN of the input components, are handed to the interior point (see
    AS_IPM_AFTER); their status and solution are the interior point's, their iteration count the
    passes plus its iterations.
    Returns dx, du, status, iterations, the mask of the instances handed over.
    """
    Bsz, N = xbar.shape[0], spec.N
    NX, NU = A.shape[-1], Bm.shape[-1]
    lb = np.broadcast_to(np.asarray(spec.lbu, dtype=np.float64), (NU,))
    ub = np.broadcast_to(np.asarray(spec.ubu, dtype=np.float64), (NU,))
    low = np.zeros((Bsz, N, NU), dtype=bool)
    up = np.zeros((Bsz, N, NU), dtype=bool)
    done = np.zeros(Bsz, dtype=bool)
    ok = np.ones(Bsz, dtype=bool)
    iters = np.zeros(Bsz, dtype=np.int32)
    best = np.full(Bsz, np.iinfo(np.int32).max)
    pcount = np.full(Bsz, pbar)
    out_dx = np.zeros((Bsz, N + 1, NX))
    out_du = np.zeros((Bsz, N, NU))
    flat_idx = np.arange(N * NU).reshape(N, NU)
    stopped = np.zeros(Bsz, dtype=bool)   # converged, or handed over after the first pass
    for it in range(min(spec.max_as_iter, AS_IPM_AFTER)):
        fixed = low | up
        delta = np.where(low, lb - ubar, np.where(up, ub - ubar, 0.0))
        dx, du, mu, ok2 = riccati_solve(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec, fixed, delta)
        act = ~stopped
        ok &= ok2 | stopped
        out_dx[act], out_du[act] = dx[act], du[act]
        iters[act] += 1
        u = ubar + du
        v_lo = ~fixed & (u < lb)
        v_hi = ~fixed & (u > ub)
        v_fl = low & (mu < 0)
        v_fu = up & (mu > 0)
        V = v_lo | v_hi | v_fl | v_fu
        nV = V.sum(axis=(1, 2))
        conv = nV == 0
        done |= conv & ~stopped
        if it == 0:
            stopped |= nV * AS_IPM_NV_DEN > AS_IPM_NV_NUM * N * NU
        stopped |= done
        if stopped.all():
            break
        full = (nV < best) | (pcount > 0)
        improve = nV < best
        pcount = np.where(improve, pbar, np.where(full, pcount - 1, pcount))
        best = np.minimum(best, nV)
        # backup: only the least-index infeasible element
        first = np.where(V, flat_idx[None], N * NU).reshape(Bsz, -1).min(axis=1)
        sel = np.where(full[:, None, None], V, flat_idx[None] == first[:, None, None])
        sel &= ~stopped[:, None, None]
        low = np.where(sel & v_lo, True, np.where(sel & v_fl, False, low))
        up = np.where(sel & v_hi, True, np.where(sel & v_fu, False, up))
    status = np.where(done, STATUS_OK, STATUS_MAXITER).astype(np.int32)
    status = np.where(ok, status, STATUS_QP_FAIL).astype(np.int32)
    fb = np.nonzero(~done & ok)[0]
    if len(fb):   # the interior point's fallback
        sub = lambda a: a[fb]
        with np.errstate(all='ignore'):
            fdx, fdu, fst, fit = ipm_box_solve(sub(A), sub(Bm), sub(gap), sub(dx0), sub(xbar), sub(ubar), sub(xref),
                                               sub(uref), spec, max_iter=AS_IPM_ITERS, centring='adaptive')
        out_dx[fb], out_du[fb], status[fb] = fdx, fdu, fst
        iters[fb] += fit
    handed = np.zeros(Bsz, dtype=bool)
    handed[fb] = True
    return out_dx, out_du, status, iters, handed


# IPM_BREAK_TOL: a Newton system that loses positive definiteness, or a collapsed step, once mu is
# below it on a feasible iterate (residual <= 1e-9, so an infeasible QP cannot pass) counts as
# converged.  1e-8 flagged LP-feasible bench instances whose Riccati recursion broke at
# mu = 2.5e-8 (361 active state rows, lambda / s ~ 4e16) and, on the device one iteration before
# the oracle, at mu = 1.3e-6; with 1e-5 device and oracle flag exactly the LP-infeasible
# instances of the bench's 1024 and 4096 draws (68 of 4096).  Kept there, the iterate has a KKT
# certificate of stationarity <= 1.8e-5 and duality gap <= 4.6e-4
# (test_gpu_full17.py::test_solve17_state_box_thin_interior_instance_converges).
IPM_SIGMA_MIN, IPM_SIGMA_MAX, IPM_TAU, IPM_THETA, IPM_TOL, IPM_BREAK_TOL, IPM_STALL = 0.05, 0.9, 0.995, 0.1, 1e-12, 1e-5, 1e-6
IPM_SHORT, IPM_SHORT_RUN = 1e-2, 10   # steps below 1e-2 ten times in a row: a stalled (infeasible) QP
# ... with the state box (the only QPs that can be infeasible): 7 steps in a row below 0.05 while
# not near the solution.  Chosen on the oracle's traces of the 4096 bench draws (tools/bench_full17.py,
# N = 60): no LP-feasible instance takes more than 3 such steps in a row; the 68 LP-infeasible ones
# now stop after at most 69 iterations (was 114; the feasible maximum is 62): the tail of the
# device launch (tools/sbox_stall_study.py)
IPM_SBOX_SHORT, IPM_SBOX_SHORT_RUN = 5e-2, 7


def _ipm_box_mehrotra(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec, max_iter=60, lbx=None, ubx=None, trace=None):
    """ipm_box_solve for the input box alone (no state rows): the same interior point with
    Mehrotra's predictor-corrector instead of the adaptive centring (device:
    riccati17q_kernel<double, true, true>; it also handles state rows, but there its
    infeasibility tail and the degenerate instances measured worse).  Constraint rows: the input box on stages 0..N-1 and, when ``lbx``/``ubx`` are
    given (JSON idxbx), the state box on stages 1..N-1.  Each row y in [lb, ub] carries slacks
    s_l, s_u > 0 with residuals r_l = y - lb - s_l, r_u = ub - y - s_u (an infeasible start: the
    state rows need not be feasible initially) and multipliers lambda_l, lambda_u > 0.  Every
    iteration takes the Newton step of the barrier-perturbed KKT system: the LQ problem in
    (Delta x, Delta u) LINEARISED AT THE CURRENT ITERATE (references shifted by (dx, du), zero
    gaps, Delta x_0 = 0) with Hessian + D and gradient + d per row, for complementarity targets
    t_l, t_u,
        D = lambda_l/s_l + lambda_u/s_u,
        d = -(t_l/s_l - t_u/s_u) + (lambda_l/s_l) r_l - (lambda_u/s_u) r_u,
        Delta lambda_l = (t_l - lambda_l s_l - lambda_l Delta s_l) / s_l   (likewise the upper side),
    by Mehrotra's predictor-corrector (HPIPM's scheme): the predictor takes targets 0 (the affine
    direction); its full step to the boundary alpha_a gives mu_a = mean((s + alpha_a Delta s)
    (lambda + alpha_a Delta lambda)), sigma = clip((mu_a / mu)^3, 0, 1); the corrector takes
    t = sigma mu - Delta s_a Delta lambda_a per row.  The iterate moves along the corrector by a
    common step, a fraction tau of the way to the boundary of (s, lambda).  (On the bench's 17/6
    input-box instances: 11.9 iterations on average against 20.9 with the previous adaptive
    centring sigma = clip(1 - alpha, 0.05, 0.9).)  Start: du =
    clip(0, lb + theta w, ub - theta w) (dx by the dynamics), s = max(distance, theta w),
    lambda = 1.  Stops when mu = mean(lambda s) <= IPM_TOL and max |r| <= 1e-9, or when the
    Newton system stops being positive definite once mu <= IPM_BREAK_TOL (an active row with
    lambda / s ~ 1e18: the current iterate is kept and counts as converged; likewise a step
    alpha < IPM_STALL there), or on a failure: a step alpha < IPM_STALL before that, or
    IPM_SBOX_SHORT_RUN steps in a row shorter than IPM_SBOX_SHORT (an infeasible QP: on the 4096
    bench draws no LP-feasible instance took more than 3 such steps in a row away from the
    solution; without a state box IPM_SHORT_RUN / IPM_SHORT), or a non-finite iterate, or after
    ``max_iter`` iterations.  Returns dx, du, status, iterations."""
    Bsz, N = xbar.shape[0], spec.N
    NX, NU = A.shape[-1], Bm.shape[-1]
    lbu = np.asarray(spec.lbu, dtype=np.float64) - ubar      # input rows, du coordinates
    ubu = np.asarray(spec.ubu, dtype=np.float64) - ubar
    wu = ubu - lbu
    du = np.clip(np.zeros_like(lbu), lbu + IPM_THETA * wu, ubu - IPM_THETA * wu)
    dx = np.empty((Bsz, N + 1, NX))
    dx[:, 0] = dx0
    for k in range(N):
        dx[:, k + 1] = np.einsum('bij,bj->bi', A[:, k], dx[:, k]) + np.einsum('bij,bj->bi', Bm[:, k], du[:, k]) + gap[:, k]
    sx = lbx is not None
    if sx:   # state rows on stages 1..N-1 (dx coordinates; stage 0 is pinned, no terminal box)
        lbx_ = np.asarray(lbx, dtype=np.float64) - xbar[:, 1:N]
        ubx_ = np.asarray(ubx, dtype=np.float64) - xbar[:, 1:N]
        wx = ubx_ - lbx_
    rows = N * NU + (N - 1) * NX * sx

    def slacks_init(y, lb, ub, w):
        return np.maximum(y - lb, IPM_THETA * w), np.maximum(ub - y, IPM_THETA * w)

    sul, suu = du - lbu, ubu - du
    llu, luu = np.ones_like(du), np.ones_like(du)
    if sx:
        sxl, sxu = slacks_init(dx[:, 1:N], lbx_, ubx_, wx)
        llx, lux = np.ones_like(sxl), np.ones_like(sxl)
    it = np.zeros(Bsz, dtype=np.int32)
    ok = np.ones(Bsz, dtype=bool)
    act = np.ones(Bsz, dtype=bool)
    conv = np.zeros(Bsz, dtype=bool)
    nshort = np.zeros(Bsz, dtype=np.int32)
    zgap = np.zeros_like(gap)
    zdx0 = np.zeros_like(dx0)

    def measure():
        tot = (llu * sul + luu * suu).sum(axis=(1, 2))
        res = np.maximum(np.abs(du - lbu - sul).max(axis=(1, 2)), np.abs(ubu - du - suu).max(axis=(1, 2)))
        if sx:
            tot = tot + (llx * sxl + lux * sxu).sum(axis=(1, 2))
            yx = dx[:, 1:N]
            res = np.maximum(res, np.maximum(np.abs(yx - lbx_ - sxl).max(axis=(1, 2)),
                                             np.abs(ubx_ - yx - sxu).max(axis=(1, 2))))
        return tot / (2 * rows), res

    def newton(y, lb, ub, sl, su, ll, lu, tl, tu):
        # barrier-perturbed row terms with the complementarity targets t_l, t_u (s lambda -> t)
        rl, ru = y - lb - sl, ub - y - su
        D = ll / sl + lu / su
        d = -(tl / sl - tu / su) + (ll / sl) * rl - (lu / su) * ru
        return D, d, rl, ru

    def duals(dy, rl, ru, sl, su, ll, lu, tl, tu):
        dsl, dsu = dy + rl, ru - dy
        dll = (tl - ll * sl - ll * dsl) / sl
        dlu = (tu - lu * su - lu * dsu) / su
        return dsl, dsu, dll, dlu

    def maxstep(v, dv):
        with np.errstate(divide='ignore', invalid='ignore'):
            return np.where(dv < 0, -v / dv, np.inf).min(axis=(1, 2))

    def direction(f3, tul, tuu, txl, txu):
        """Newton direction for the targets (t_l, t_u) of the input and state rows."""
        Du, du_lin, rul, ruu = newton(du, lbu, ubu, sul, suu, llu, luu, tul, tuu)
        Qd = qd = None
        rx = None
        if sx:
            Dx, dx_lin, rxl, rxu = newton(dx[:, 1:N], lbx_, ubx_, sxl, sxu, llx, lux, txl, txu)
            Qd = np.zeros((Bsz, N, NX))
            qd = np.zeros((Bsz, N, NX))
            Qd[:, 1:N], qd[:, 1:N] = Dx, dx_lin
            rx = (rxl, rxu)
        fin = np.isfinite(Du).all(axis=(1, 2)) & np.isfinite(du_lin).all(axis=(1, 2)) & np.isfinite(dx).all(axis=(1, 2))
        if sx:
            fin &= np.isfinite(Qd).all(axis=(1, 2)) & np.isfinite(qd).all(axis=(1, 2))
        if f3 is not None:
            fin = fin & f3[:, 0, 0]
        g3 = fin[:, None, None]
        Du, du_lin = np.where(g3, Du, 1.0), np.where(g3, du_lin, 0.0)
        if sx:
            Qd, qd = np.where(g3, Qd, 1.0), np.where(g3, qd, 0.0)
        ddx, dd, _, ok2 = riccati_solve(A, Bm, zgap, zdx0, xbar + np.where(g3, dx, 0.0), ubar + np.where(g3, du, 0.0),
                                        xref, uref, spec, Rd=Du, rd=du_lin, Qd=Qd, qd=qd)
        dul = duals(dd, rul, ruu, sul, suu, llu, luu, tul, tuu)
        dxl = duals(ddx[:, 1:N], rx[0], rx[1], sxl, sxu, llx, lux, txl, txu) if sx else None
        return fin, ok2, ddx, dd, dul, dxl

    def pairs(dul, dxl):
        out = list(zip((sul, suu, llu, luu), dul))
        if sx:
            out += list(zip((sxl, sxu, llx, lux), dxl))
        return out

    zero = np.zeros((Bsz, 1, 1))
    for _ in range(max_iter):
        mu, res = measure()
        act = act & ((mu > IPM_TOL) | (res > 1e-9))
        if not act.any():
            break
        # predictor: the affine-scaling direction (targets 0)
        fin, ok_a, _, _, dul_a, dxl_a = direction(None, zero, zero, zero, zero)
        # an instance whose iterate left the finite range (an infeasible QP drives the multipliers
        # to infinity) is frozen: it keeps a harmless system and fails at the end
        ok &= fin
        act &= fin
        f3 = fin[:, None, None]
        pr = pairs(dul_a, dxl_a)
        alpha_a = np.minimum(1.0, np.min(np.stack([maxstep(v, dv) for v, dv in pr]), axis=0))
        aa = alpha_a[:, None, None]
        mu_a = sum(((v + aa * dv) * (w + aa * dw)).sum(axis=(1, 2))
                   for (v, dv), (w, dw) in zip(pr[0::4] + pr[1::4], pr[2::4] + pr[3::4])) / (2 * rows)
        with np.errstate(divide='ignore', invalid='ignore'):
            sig = np.clip((mu_a / mu) ** 3, 0.0, 1.0)
        sig = np.where(np.isfinite(sig), sig, 1.0)
        smu = (sig * mu)[:, None, None]
        # corrector: targets sigma mu - (Delta s Delta lambda) of the predictor, per row
        tul, tuu = smu - dul_a[0] * dul_a[2], smu - dul_a[1] * dul_a[3]
        txl = txu = None
        if sx:
            txl, txu = smu - dxl_a[0] * dxl_a[2], smu - dxl_a[1] * dxl_a[3]
        _, ok2, ddx, dd, dul, dxl = direction(f3, tul, tuu, txl, txu)
        ok2 = ok2 & ok_a
        # breakdown of the Newton system near the solution (lambda / s ~ 1e18 on an active row
        # costs the Riccati recursion its positive definiteness): keep the current iterate
        brk = ~ok2 & act & (mu <= IPM_BREAK_TOL) & (res <= 1e-9)
        conv |= brk
        act &= ~brk
        ok &= ok2 | ~act
        alpha = np.minimum(1.0, IPM_TAU * np.min(np.stack([maxstep(v, dv) for v, dv in pairs(dul, dxl)]), axis=0))
        # a collapsed step ends the instance: near the solution (mu <= IPM_BREAK_TOL, feasible) the
        # Newton direction has reached the conditioning limit and the iterate counts as converged;
        # earlier it means an infeasible QP (the residual cannot reach zero)
        short, short_run = (IPM_SBOX_SHORT, IPM_SBOX_SHORT_RUN) if sx else (IPM_SHORT, IPM_SHORT_RUN)
        nshort = np.where(alpha < short, nshort + 1, 0)
        stall = act & ((alpha < IPM_STALL) | (nshort >= short_run))
        near = (mu <= IPM_BREAK_TOL) & (res <= 1e-9)
        conv |= stall & near
        ok &= ~(stall & ~near)
        act &= ~stall
        alpha = np.where(act, alpha, 0.0)[:, None, None]
        du = du + alpha * dd
        dx = dx + alpha * ddx
        sul, suu, llu, luu = (v + alpha * dv for v, dv in zip((sul, suu, llu, luu), dul))
        if sx:
            sxl, sxu, llx, lux = (v + alpha * dv for v, dv in zip((sxl, sxu, llx, lux), dxl))
        it += act
        if trace is not None:   # diagnostics: (mu, max |r|, step) per iteration
            trace.append((mu.copy(), res.copy(), alpha[:, 0, 0].copy()))
    mu, res = measure()
    status = np.where(conv | ((mu <= IPM_TOL) & (res <= 1e-9)), STATUS_OK, STATUS_MAXITER).astype(np.int32)
    status = np.where(ok, status, STATUS_QP_FAIL).astype(np.int32)
    # a stop at the conditioning limit (breakdown / collapsed step) is a reduced-accuracy iterate
    status = np.where((status == STATUS_OK) & ~((mu <= IPM_TOL) & (res <= 1e-9)), STATUS_MINSTEP, status).astype(np.int32)
    return dx, du, status, it


def ipm_box_solve(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec, max_iter=60, lbx=None, ubx=None, trace=None,
                  centring=None):
    """Box-constrained QP by a primal-dual interior point over the Riccati recursion (the method
    of acados' HPIPM; the full 17/6 model, where the active set above can need thousands of
    exchanges).  Constraint rows: the input box on stages 0..N-1 and, when ``lbx``/``ubx`` are
    given (JSON idxbx), the state box on stages 1..N-1.  Each row y in [lb, ub] carries slacks
    s_l, s_u > 0 with residuals r_l = y - lb - s_l, r_u = ub - y - s_u (an infeasible start: the
    state rows need not be feasible initially) and multipliers lambda_l, lambda_u > 0.  Every
    iteration takes the Newton step of the barrier-perturbed KKT system: the LQ problem in
    (Delta x, Delta u) LINEARISED AT THE CURRENT ITERATE (references shifted by (dx, du), zero
    gaps, Delta x_0 = 0) with Hessian + D and gradient + d per row,
        D = lambda_l/s_l + lambda_u/s_u,
        d = -sigma mu (1/s_l - 1/s_u) + (lambda_l/s_l) r_l - (lambda_u/s_u) r_u,
    then a common step, a fraction tau of the way to the boundary of (s, lambda).  The centring
    parameter follows the previous step length alpha: sigma = clip(1 - alpha, 0.05, 0.9) (a short
    step means a badly centred iterate; on infeasible starts this cuts the 99th-percentile
    iteration count from ~180 to ~50 against a fixed sigma = 0.1).  Start: du =
    clip(0, lb + theta w, ub - theta w) (dx by the dynamics), s = max(distance, theta w),
    lambda = 1.  Stops when mu = mean(lambda s) <= IPM_TOL and max |r| <= 1e-9, or when the
    Newton system stops being positive definite once mu <= IPM_BREAK_TOL (an active row with
    lambda / s ~ 1e18: the current iterate is kept and counts as converged; likewise a step
    alpha < IPM_STALL there), or on a failure: a step alpha < IPM_STALL before that, or
    IPM_SBOX_SHORT_RUN steps in a row shorter than IPM_SBOX_SHORT (an infeasible QP: on the 4096
    bench draws no LP-feasible instance took more than 3 such steps in a row away from the
    solution; without a state box IPM_SHORT_RUN / IPM_SHORT), or a non-finite iterate, or after
    ``max_iter`` iterations.  Returns dx, du, status, iterations.
    ``centring='adaptive'`` keeps this scheme for the input box alone (the 12/4 active set's
    fallback, pdas_solve); otherwise the input box alone takes Mehrotra's predictor-corrector."""
    if lbx is None and centring != 'adaptive':   # the input box alone: _ipm_box_mehrotra
        return _ipm_box_mehrotra(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec, max_iter=max_iter, trace=trace)
    Bsz, N = xbar.shape[0], spec.N
    NX, NU = A.shape[-1], Bm.shape[-1]
    lbu = np.asarray(spec.lbu, dtype=np.float64) - ubar      # input rows, du coordinates
    ubu = np.asarray(spec.ubu, dtype=np.float64) - ubar
    wu = ubu - lbu
    du = np.clip(np.zeros_like(lbu), lbu + IPM_THETA * wu, ubu - IPM_THETA * wu)
    dx = np.empty((Bsz, N + 1, NX))
    dx[:, 0] = dx0
    for k in range(N):
        dx[:, k + 1] = np.einsum('bij,bj->bi', A[:, k], dx[:, k]) + np.einsum('bij,bj->bi', Bm[:, k], du[:, k]) + gap[:, k]
    sx = lbx is not None
    if sx:   # state rows on stages 1..N-1 (dx coordinates; stage 0 is pinned, no terminal box)
        lbx_ = np.asarray(lbx, dtype=np.float64) - xbar[:, 1:N]
        ubx_ = np.asarray(ubx, dtype=np.float64) - xbar[:, 1:N]
        wx = ubx_ - lbx_
    rows = N * NU + (N - 1) * NX * sx

    def slacks_init(y, lb, ub, w):
        return np.maximum(y - lb, IPM_THETA * w), np.maximum(ub - y, IPM_THETA * w)

    sul, suu = du - lbu, ubu - du
    llu, luu = np.ones_like(du), np.ones_like(du)
    if sx:
        sxl, sxu = slacks_init(dx[:, 1:N], lbx_, ubx_, wx)
        llx, lux = np.ones_like(sxl), np.ones_like(sxl)
    it = np.zeros(Bsz, dtype=np.int32)
    ok = np.ones(Bsz, dtype=bool)
    act = np.ones(Bsz, dtype=bool)
    conv = np.zeros(Bsz, dtype=bool)
    prev_alpha = np.ones(Bsz)
    nshort = np.zeros(Bsz, dtype=np.int32)
    zgap = np.zeros_like(gap)
    zdx0 = np.zeros_like(dx0)

    def measure():
        tot = (llu * sul + luu * suu).sum(axis=(1, 2))
        res = np.maximum(np.abs(du - lbu - sul).max(axis=(1, 2)), np.abs(ubu - du - suu).max(axis=(1, 2)))
        if sx:
            tot = tot + (llx * sxl + lux * sxu).sum(axis=(1, 2))
            yx = dx[:, 1:N]
            res = np.maximum(res, np.maximum(np.abs(yx - lbx_ - sxl).max(axis=(1, 2)),
                                             np.abs(ubx_ - yx - sxu).max(axis=(1, 2))))
        return tot / (2 * rows), res

    def newton(y, lb, ub, sl, su, ll, lu, smu):
        rl, ru = y - lb - sl, ub - y - su
        D = ll / sl + lu / su
        d = -smu * (1.0 / sl - 1.0 / su) + (ll / sl) * rl - (lu / su) * ru
        return D, d, rl, ru

    def duals(dy, rl, ru, sl, su, ll, lu, smu):
        dsl, dsu = dy + rl, ru - dy
        dll = (smu - ll * sl - ll * dsl) / sl
        dlu = (smu - lu * su - lu * dsu) / su
        return dsl, dsu, dll, dlu

    def maxstep(v, dv):
        with np.errstate(divide='ignore', invalid='ignore'):
            return np.where(dv < 0, -v / dv, np.inf).min(axis=(1, 2))

    for _ in range(max_iter):
        mu, res = measure()
        act = act & ((mu > IPM_TOL) | (res > 1e-9))
        if not act.any():
            break
        sig = np.clip(1.0 - prev_alpha, IPM_SIGMA_MIN, IPM_SIGMA_MAX)   # centre harder after a short step
        smu = (sig * mu)[:, None, None]
        Du, du_lin, rul, ruu = newton(du, lbu, ubu, sul, suu, llu, luu, smu)
        Qd = qd = None
        if sx:
            Dx, dx_lin, rxl, rxu = newton(dx[:, 1:N], lbx_, ubx_, sxl, sxu, llx, lux, smu)
            Qd = np.zeros((Bsz, N, NX))
            qd = np.zeros((Bsz, N, NX))
            Qd[:, 1:N], qd[:, 1:N] = Dx, dx_lin
        # an instance whose iterate left the finite range (an infeasible QP drives the multipliers
        # to infinity) is frozen: it keeps a harmless system and fails at the end
        fin = np.isfinite(Du).all(axis=(1, 2)) & np.isfinite(du_lin).all(axis=(1, 2)) & np.isfinite(dx).all(axis=(1, 2))
        if sx:
            fin &= np.isfinite(Qd).all(axis=(1, 2)) & np.isfinite(qd).all(axis=(1, 2))
        ok &= fin
        act &= fin
        f3 = fin[:, None, None]
        Du, du_lin = np.where(f3, Du, 1.0), np.where(f3, du_lin, 0.0)
        if sx:
            Qd, qd = np.where(f3, Qd, 1.0), np.where(f3, qd, 0.0)
        ddx, dd, _, ok2 = riccati_solve(A, Bm, zgap, zdx0, xbar + np.where(f3, dx, 0.0), ubar + np.where(f3, du, 0.0),
                                        xref, uref, spec, Rd=Du, rd=du_lin, Qd=Qd, qd=qd)
        # breakdown of the Newton system near the solution (lambda / s ~ 1e18 on an active row
        # costs the Riccati recursion its positive definiteness): keep the current iterate
        brk = ~ok2 & act & (mu <= IPM_BREAK_TOL) & (res <= 1e-9)
        conv |= brk
        act &= ~brk
        ok &= ok2 | ~act
        steps = []
        dul = duals(dd, rul, ruu, sul, suu, llu, luu, smu)
        steps += [maxstep(v, dv) for v, dv in zip((sul, suu, llu, luu), dul)]
        if sx:
            dxl = duals(ddx[:, 1:N], rxl, rxu, sxl, sxu, llx, lux, smu)
            steps += [maxstep(v, dv) for v, dv in zip((sxl, sxu, llx, lux), dxl)]
        alpha = np.minimum(1.0, IPM_TAU * np.min(np.stack(steps), axis=0))
        prev_alpha = alpha
        # a collapsed step ends the instance: near the solution (mu <= IPM_BREAK_TOL, feasible) the
        # Newton direction has reached the conditioning limit and the iterate counts as converged;
        # earlier it means an infeasible QP (the residual cannot reach zero)
        short, short_run = (IPM_SBOX_SHORT, IPM_SBOX_SHORT_RUN) if sx else (IPM_SHORT, IPM_SHORT_RUN)
        nshort = np.where(alpha < short, nshort + 1, 0)
        stall = act & ((alpha < IPM_STALL) | (nshort >= short_run))
        near = (mu <= IPM_BREAK_TOL) & (res <= 1e-9)
        conv |= stall & near
        ok &= ~(stall & ~near)
        act &= ~stall
        alpha = np.where(act, alpha, 0.0)[:, None, None]
        du = du + alpha * dd
        dx = dx + alpha * ddx
        sul, suu, llu, luu = (v + alpha * dv for v, dv in zip((sul, suu, llu, luu), dul))
        if sx:
            sxl, sxu, llx, lux = (v + alpha * dv for v, dv in zip((sxl, sxu, llx, lux), dxl))
        it += act
        if trace is not None:   # diagnostics: (mu, max |r|, step) per iteration
            trace.append((mu.copy(), res.copy(), alpha[:, 0, 0].copy()))
    mu, res = measure()
    status = np.where(conv | ((mu <= IPM_TOL) & (res <= 1e-9)), STATUS_OK, STATUS_MAXITER).astype(np.int32)
    status = np.where(ok, status, STATUS_QP_FAIL).astype(np.int32)
    acc = np.zeros(Bsz, dtype=bool)
    if sx and POLISH_ITERS > 0:
        rows_u = (du, lbu, ubu, sul, suu, llu, luu)
        rows_x = (dx[:, 1:N], lbx_, ubx_, sxl, sxu, llx, lux)
        pdx, pdu, acc = al_polish(A, Bm, xbar, ubar, xref, uref, spec, dx, du, rows_u, rows_x,
                                  status == STATUS_OK)
        dx = np.where(acc[:, None, None], pdx, dx)
        du = np.where(acc[:, None, None], pdu, du)
    # an early exit (breakdown or stall at the conditioning limit) that no polish certified keeps its
    # reduced-accuracy iterate under acados' MINSTEP status, not OK
    status = np.where((status == STATUS_OK) & ~acc & ~((mu <= IPM_TOL) & (res <= 1e-9)),
                      STATUS_MINSTEP, status).astype(np.int32)
    return dx, du, status, it


# The polish after the state-box interior point (HPIPM's analogue: its final "exact" step on the
# identified active set).  At the interior point's last iterate a row is taken as active on its
# lower side when lambda_l > POLISH_ACT s_l (upper likewise): on a strongly active row lambda / s ~
# 1e4..1e16, on an inactive one ~1e-2 or less; the rows in between (lambda ~ s ~ sqrt(mu): weakly
# active, degenerate) are left free at first.  (With the midpoint ratio 1, 33 of the 4096 bench
# draws took such rows into mutually inconsistent sets, whose multipliers then run off and the
# pass cap ended the polish; with 100 every LP-feasible draw instance is polished in <= 4 passes.)  The equality-constrained QP on that active set is solved by the
# method of multipliers over the same Riccati recursion: each pass is one linear solve, the
# minimiser of the augmented Lagrangian  J + nu'(Cz - b) + rho/2 |Cz - b|^2  (diagonal rho on the
# active rows, gradient nu + rho (y - b): the interior point's D / d slots), linearised at the
# interior point's iterate z0 (the QP is quadratic, so the minimiser does not depend on it), then
# nu <- nu + rho (y - b).  nu starts at lambda_u - lambda_l.  Every pass also corrects the set by
# one primal active-set step: the active row whose multiplier is the most negative once signed is
# released (nu = 0), else the inactive row furthest outside its bound is fixed at it (nu = 0).  An
# instance is done when its set did not change and every active row is within POLISH_EQ of its
# bound; it then keeps the polished point if the Riccati recursion stayed positive definite.  An
# instance not done after POLISH_ITERS passes keeps the interior-point iterate.
POLISH_RHO, POLISH_ITERS, POLISH_EQ, POLISH_FEAS = 1e10, 12, 1e-10, 1e-10
POLISH_ACT = 100.0   # a row is active when lambda > 100 s (ratio 1 takes ambiguous rows: inconsistent sets)


def al_polish(A, Bm, xbar, ubar, xref, uref, spec, dx, du, rows_u, rows_x, ok, rho=None, iters=None, diag=None):
    """Augmented-Lagrangian polish of the box QP on the interior point's active set (see above).
    rows_u / rows_x = (y, lb, ub, s_l, s_u, lambda_l, lambda_u) of the input rows (stages 0..N-1)
    and the state rows (stages 1..N-1).  Returns the polished (dx, du) and the per-instance
    acceptance flag (False where ``ok`` is False)."""
    rho = POLISH_RHO if rho is None else rho
    iters = POLISH_ITERS if iters is None else iters
    Bsz, N = xbar.shape[0], spec.N
    NX = A.shape[-1]

    def classify(y, lb, ub, sl, su, ll, lu):
        side = np.where(ll > POLISH_ACT * sl, -1.0, np.where(lu > POLISH_ACT * su, 1.0, 0.0))
        return side, np.where(side != 0, lu - ll, 0.0)

    su_, nu_u = classify(*rows_u)
    sx_, nu_x = classify(*rows_x)
    yu0, yx0 = rows_u[0], rows_x[0]
    (lbu, ubu), (lbx, ubx) = rows_u[1:3], rows_x[1:3]
    zgap = np.zeros((Bsz, N, NX))
    zdx0 = np.zeros((Bsz, NX))
    Qd = np.zeros((Bsz, N, NX))
    qd = np.zeros((Bsz, N, NX))
    okp = ok.copy()
    done = np.zeros(Bsz, dtype=bool)
    pdx, pdu = np.zeros_like(dx), np.zeros_like(du)
    passes = np.zeros(Bsz, dtype=np.int32)
    g3 = ok[:, None, None]
    for _ in range(iters):
        act3 = (okp & ~done)[:, None, None]
        bu, bx = np.where(su_ < 0, lbu, ubu), np.where(sx_ < 0, lbx, ubx)
        Rd = np.where(g3 & (su_ != 0), rho, 0.0)
        rd = np.where(g3 & (su_ != 0), nu_u + rho * (yu0 - bu), 0.0)
        Qd[:, 1:N] = np.where(g3 & (sx_ != 0), rho, 0.0)
        qd[:, 1:N] = np.where(g3 & (sx_ != 0), nu_x + rho * (yx0 - bx), 0.0)
        ddx, dd, _, ok2 = riccati_solve(A, Bm, zgap, zdx0, xbar + np.where(g3, dx, 0.0),
                                        ubar + np.where(g3, du, 0.0), xref, uref, spec,
                                        Rd=Rd, rd=rd, Qd=Qd, qd=qd)
        fin = np.isfinite(ddx).all(axis=(1, 2)) & np.isfinite(dd).all(axis=(1, 2))
        okp &= (ok2 & fin) | done
        act3 = (okp & ~done)[:, None, None]
        pdx, pdu = np.where(act3, ddx, pdx), np.where(act3, dd, pdu)
        passes += (okp & ~done)
        yu, yx = yu0 + dd, yx0 + ddx[:, 1:N]
        eu, ex = np.where(su_ != 0, yu - bu, 0.0), np.where(sx_ != 0, yx - bx, 0.0)
        nun_u, nun_x = nu_u + rho * eu, nu_x + rho * ex
        eq = np.maximum(np.abs(eu).max(axis=(1, 2)), np.abs(ex).max(axis=(1, 2)))

        # one change per pass (a primal active-set step): release the active row whose multiplier
        # is the most negative once signed, else fix the inactive row furthest outside its bound
        wu, wx = np.where(su_ != 0, su_ * nun_u, np.inf), np.where(sx_ != 0, sx_ * nun_x, np.inf)
        vu = np.where(su_ == 0, np.maximum(lbu - yu, yu - ubu), -np.inf)
        vx = np.where(sx_ == 0, np.maximum(lbx - yx, yx - ubx), -np.inf)
        wmin = np.minimum(wu.min(axis=(1, 2)), wx.min(axis=(1, 2)))
        vmax = np.maximum(vu.max(axis=(1, 2)), vx.max(axis=(1, 2)))
        rel = wmin < 0
        add = ~rel & (vmax > POLISH_FEAS)
        conv = ~rel & ~add & (eq <= POLISH_EQ)
        live = okp & ~done
        if diag is not None:
            diag.setdefault('trace', []).append((eq.copy(), wmin.copy(), vmax.copy()))
        nu_u, nu_x = np.where(live[:, None, None] & (su_ != 0), nun_u, nu_u), np.where(live[:, None, None] & (sx_ != 0), nun_x, nu_x)
        for b in np.nonzero(live & (rel | add))[0]:
            if rel[b]:
                if wu[b].min() <= wx[b].min():
                    j = np.unravel_index(np.argmin(wu[b]), wu[b].shape)
                    su_[b][j], nu_u[b][j] = 0.0, 0.0
                else:
                    j = np.unravel_index(np.argmin(wx[b]), wx[b].shape)
                    sx_[b][j], nu_x[b][j] = 0.0, 0.0
            else:
                if vu[b].max() >= vx[b].max():
                    j = np.unravel_index(np.argmax(vu[b]), vu[b].shape)
                    su_[b][j], nu_u[b][j] = (-1.0 if yu[b][j] < lbu[b][j] else 1.0), 0.0
                else:
                    j = np.unravel_index(np.argmax(vx[b]), vx[b].shape)
                    sx_[b][j], nu_x[b][j] = (-1.0 if yx[b][j] < lbx[b][j] else 1.0), 0.0
        done |= okp & conv
        if not (okp & ~done).any():
            break
    acc = done & okp
    if diag is not None:   # diagnostics (tools, tests)
        diag.update(passes=passes, done=done, okp=okp, n_act=(su_ != 0).sum(axis=(1, 2)) + (sx_ != 0).sum(axis=(1, 2)))
    return dx + pdx, du + pdu, acc


def mpc_solve(x0, xref, uref, spec: OcpSpec, wind=None, mode='rollout', xbar=None, ubar=None,
              return_lin=False):
    """One SQP_RTI step for a batch.  x0 (B,12), xref (B,N+1,12), uref (B,N,4)."""
    x0 = np.asarray(x0, dtype=np.float64)
    Bsz, N = x0.shape[0], spec.N
    xref = np.broadcast_to(np.asarray(xref, dtype=np.float64), (Bsz, N + 1, NX))
    uref = np.broadcast_to(np.asarray(uref, dtype=np.float64), (Bsz, N, NU))
    if mode == 'rollout':
        ubar = uref.copy()
        xbar = rollout(x0, ubar, spec, wind)
    else:
        xbar = np.asarray(xbar, dtype=np.float64)
        ubar = np.asarray(ubar, dtype=np.float64)
    A, Bm, gap = linearise(xbar, ubar, spec, wind)
    dx0 = x0 - xbar[:, 0]
    if spec.boxed:
        dx, du, status, iters, handed = pdas_solve(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec)
    else:
        dx, du, _, ok = riccati_solve(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec)
        status = np.where(ok, STATUS_OK, STATUS_QP_FAIL).astype(np.int32)
        iters = np.zeros(Bsz, dtype=np.int32)
        handed = np.zeros(Bsz, dtype=bool)
    X = xbar + dx
    U = ubar + du
    bad = ~(np.isfinite(X).all(axis=(1, 2)) & np.isfinite(U).all(axis=(1, 2)))
    status = np.where(bad, STATUS_NAN, status).astype(np.int32)
    # (fallback: the instances the input box's active set handed to the interior point)
    out = dict(u0=U[:, 0].copy(), X=X, U=U, status=status, iters=iters, xbar=xbar, ubar=ubar, fallback=handed)
    if return_lin:
        out.update(A=A, B=Bm, gap=gap)
    return out


def stage_cost(X, U, xref, uref, spec: OcpSpec) -> np.ndarray:
    """Objective at (X, U) — what acados ``get_cost()`` reports for the new iterate."""
    s = spec.s
    Q, R, QN = (np.asarray(M, dtype=np.float64) for M in (spec.Q, spec.R, spec.QN))
    ex = X[:, :-1] - xref[:, :-1]
    eu = U - uref
    eN = X[:, -1] - xref[:, -1]
    c = 0.5 * s * (np.einsum('bki,ij,bkj->b', ex, Q, ex) + np.einsum('bki,ij,bkj->b', eu, R, eu))
    return c + 0.5 * np.einsum('bi,ij,bj->b', eN, QN, eN)


def fp32_sensitivity(o, x0, xref, uref, spec: OcpSpec, trials: int = 2, rel: float = 2.0 ** -22, seed: int = 0):
    """How far the exact input-box minimiser moves when the QP data carry fp32-level noise: the
    linearisation [A|B] of ``o`` (mpc_solve(..., return_lin=True)) scaled entrywise by
    (1 + rel * N(0, 1)), i.e. ~2 ulp of fp32, and re-solved exactly by ``pdas_solve``, ``trials``
    times.  Returns per instance the largest normwise move of U and of u0 (the parity metric).

    An fp32 solver's own linearisation carries at least this much error, so an instance that moves
    by more than a parity bound here cannot be held to it by ANY fp32 computation: the sweeps hold
    such instances (counted and printed) to the QP's optimal objective instead
    (tests/test_gpu_fuzz.py).  On c4's draws the move is ~1e-6 (tests/test_oracle_sensitivity.py); on strongly constrained short
    horizons (sweep cases 33 / 67 / 158: N = 2, 6, 4, wind) up to 2e-4."""
    B = x0.shape[0]
    N = spec.N
    xr = np.broadcast_to(np.asarray(xref, dtype=np.float64), (B, N + 1, NX))
    ur = np.broadcast_to(np.asarray(uref, dtype=np.float64), (B, N, NU))
    rs = np.random.default_rng(seed)
    worst = np.zeros(B)
    den = np.maximum(np.abs(o['U']).reshape(B, -1).max(axis=1), 1.0)
    den0 = np.maximum(np.abs(o['u0']).max(axis=1), 1.0)
    for _ in range(trials):
        A = o['A'] * (1.0 + rel * rs.standard_normal(o['A'].shape))
        Bm = o['B'] * (1.0 + rel * rs.standard_normal(o['B'].shape))
        with np.errstate(all='ignore'):
            _, du, _, _, _ = pdas_solve(A, Bm, o['gap'], x0 - o['xbar'][:, 0], o['xbar'], o['ubar'], xr, ur, spec)
        U = o['ubar'] + du
        eU = np.abs(U - o['U']).reshape(B, -1).max(axis=1) / den
        eu = np.abs(U[:, 0] - o['u0']).max(axis=1) / den0
        worst = np.maximum(worst, np.maximum(eU, eu))
    return worst


def dense_box_qp(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec: OcpSpec):
    """Independent check (tests only): condense the QP in du and solve it with SciPy BVLS."""
    from scipy.optimize import lsq_linear

    Bsz, N = xbar.shape[0], spec.N
    NX, NU = A.shape[-1], Bm.shape[-1]
    s = spec.s
    Q, R, QN = (np.asarray(M, dtype=np.float64) for M in (spec.Q, spec.R, spec.QN))
    out_du = np.empty((Bsz, N, NU))
    for b in range(Bsz):
        # dx_k = c_k + G_k du  (G_k: NX x N*NU)
        c = np.zeros((N + 1, NX))
        G = np.zeros((N + 1, NX, N * NU))
        c[0] = dx0[b]
        for k in range(N):
            c[k + 1] = A[b, k] @ c[k] + gap[b, k]
            G[k + 1] = A[b, k] @ G[k]
            G[k + 1][:, k * NU:(k + 1) * NU] += Bm[b, k]
        H = np.zeros((N * NU, N * NU))
        g = np.zeros(N * NU)
        for k in range(N + 1):
            W = QN if k == N else s * Q
            e = c[k] + xbar[b, k] - xref[b, k]
            H += G[k].T @ W @ G[k]
            g += G[k].T @ W @ e
        for k in range(N):
            sl = slice(k * NU, (k + 1) * NU)
            H[sl, sl] += s * R
            g[sl] += s * R @ (ubar[b, k] - uref[b, k])
        L = np.linalg.cholesky(H)            # H = L L^T ; min 1/2|L^T z + L^{-1} g|^2
        Lt = L.T
        rhs = -np.linalg.solve(L, g)
        lb = np.tile(np.asarray(spec.lbu, dtype=np.float64), N) - ubar[b].reshape(-1)
        ub = np.tile(np.asarray(spec.ubu, dtype=np.float64), N) - ubar[b].reshape(-1)
        res = lsq_linear(Lt, rhs, bounds=(lb, ub), method='bvls', tol=1e-14, lsmr_tol='auto',
                         max_iter=10000)
        out_du[b] = res.x.reshape(N, NU)
    return out_du


def dense_kkt_certificate(A, Bm, gap, dx0, xbar, ubar, xref, uref, spec, du, lbx=None, ubx=None, act_tol=1e-6):
    """Independent check (tests only) of a box-QP solution with state rows.  Condenses the QP in
    du (f(z) = z'Hz/2 + g'z, rows C z <= h: the input box, then the state box on stages 1..N-1),
    takes the rows within ``act_tol`` of a bound as the active set A and finds multipliers
    lambda >= 0 by NNLS on H z + g + C_A' lambda = 0 (the rows can be linearly dependent: an input
    at its bound and the state it drives, so lambda is not unique and a plain solve can return a
    negative one).  Returns per instance: stationarity residual relative to |H z + g|, the largest
    row violation, and the duality gap sum lambda (h - C z)_A, which bounds f(z) - f* above."""
    from scipy.optimize import nnls

    Bsz, N = xbar.shape[0], spec.N
    NX, NU = A.shape[-1], Bm.shape[-1]
    s = spec.s
    Q, R, QN = (np.asarray(M, dtype=np.float64) for M in (spec.Q, spec.R, spec.QN))
    nz = N * NU
    stat = np.zeros(Bsz)
    viol = np.zeros(Bsz)
    dgap = np.zeros(Bsz)
    for b in range(Bsz):
        c = np.zeros((N + 1, NX))
        G = np.zeros((N + 1, NX, nz))
        c[0] = dx0[b]
        for k in range(N):
            c[k + 1] = A[b, k] @ c[k] + gap[b, k]
            G[k + 1] = A[b, k] @ G[k]
            G[k + 1][:, k * NU:(k + 1) * NU] += Bm[b, k]
        H = np.zeros((nz, nz))
        g = np.zeros(nz)
        for k in range(N + 1):
            W = QN if k == N else s * Q
            e = c[k] + xbar[b, k] - xref[b, k]
            H += G[k].T @ W @ G[k]
            g += G[k].T @ W @ e
        for k in range(N):
            sl = slice(k * NU, (k + 1) * NU)
            H[sl, sl] += s * R
            g[sl] += s * R @ (ubar[b, k] - uref[b, k])
        C = [np.eye(nz), -np.eye(nz)]
        h = [np.tile(np.asarray(spec.ubu, dtype=np.float64), N) - ubar[b].reshape(-1),
             -(np.tile(np.asarray(spec.lbu, dtype=np.float64), N) - ubar[b].reshape(-1))]
        if lbx is not None:
            Gx = G[1:N].reshape(-1, nz)
            cx = (c[1:N] + xbar[b, 1:N]).reshape(-1)
            C += [Gx, -Gx]
            h += [np.tile(np.asarray(ubx, dtype=np.float64), N - 1) - cx,
                  -(np.tile(np.asarray(lbx, dtype=np.float64), N - 1) - cx)]
        C = np.vstack(C)
        h = np.concatenate(h)
        z = du[b].reshape(-1)
        grad = H @ z + g
        v = C @ z - h
        act = np.nonzero(v > -act_tol)[0]
        lam, res = nnls(C[act].T, -grad) if len(act) else (np.zeros(0), np.linalg.norm(grad))
        stat[b] = res / max(1.0, np.linalg.norm(grad))
        viol[b] = max(0.0, v.max())
        dgap[b] = float(lam @ -v[act]) if len(act) else 0.0
    return stat, viol, dgap


def lp_box_feasible(A, Bm, gap, dx0, xbar, ubar, spec, lbx, ubx):
    """Independent check (tests only): is the box QP of each instance feasible?  The condensed
    rows (input box; state box on stages 1..N-1) as an LP feasibility problem for SciPy's HiGHS.
    Returns a bool per instance."""
    from scipy.optimize import linprog

    Bsz, N = xbar.shape[0], spec.N
    NX, NU = A.shape[-1], Bm.shape[-1]
    out = np.zeros(Bsz, dtype=bool)
    for b in range(Bsz):
        c = np.zeros((N + 1, NX))
        G = np.zeros((N + 1, NX, N * NU))
        c[0] = dx0[b]
        for k in range(N):
            c[k + 1] = A[b, k] @ c[k] + gap[b, k]
            G[k + 1] = A[b, k] @ G[k]
            G[k + 1][:, k * NU:(k + 1) * NU] += Bm[b, k]
        Gx = G[1:N].reshape(-1, N * NU)
        lo = (np.asarray(lbx) - xbar[b, 1:N] - c[1:N]).ravel()
        hi = (np.asarray(ubx) - xbar[b, 1:N] - c[1:N]).ravel()
        bnds = list(zip((np.asarray(spec.lbu) - ubar[b]).ravel(), (np.asarray(spec.ubu) - ubar[b]).ravel()))
        r = linprog(np.zeros(N * NU), A_ub=np.vstack([Gx, -Gx]), b_ub=np.concatenate([hi, -lo]), bounds=bnds,
                    method='highs')
        out[b] = r.status == 0
    return out
