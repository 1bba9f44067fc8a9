/*
 * mpc_oracle.c — plain-C restatement of the CPU oracle (TEST INFRASTRUCTURE ONLY: the timed CPU
 * baseline of bench.py and a cross-check of oracle/ocp.py; never linked by the product).
 *
 * Same algorithm as oracle/ocp.py (unconstrained GN SQP_RTI step, rollout linearisation):
 *   RK4 rollout of u_ref from x0 (acados sim_erk, 4 stages, 1 step; blastermodel.py:277),
 *   exact forward sensitivities A_k, B_k of the RK4 map,
 *   LINEAR_LS cost with stage scaling s = dt (blastermodel.py:228-257),
 *   Riccati recursion with symmetrised P, forward pass -> u0, X, U.
 * Dynamics: 12-state/4-input slice of f_expl_expr (blastermodel.py:95-201).
 * Input box (c4, blastermodel.py:259-264): the primal-dual active set with the Kim-Park safeguard
 * and Murty's least-index backup of oracle/ocp.py pdas_solve, over the masked Riccati recursion.
 * pdas_solve's interior-point fallback (after 48 passes, or after a first pass that violates more
 * than 7/20 of the input components) is not restated: no c4 draw reaches it (at most 39 passes
 * and 19 of 120 violations), so the timed c4 sample does the same work as the device.
 * Parallel over instances with OpenMP (one instance per thread at a time).
 */
#define _POSIX_C_SOURCE 199309L
#include <math.h>
#include <time.h>
#include <string.h>

#define NX 12
#define NU 4
#define NZ 16

typedef struct {
  double minv, g, t_blast, lx, ly, c;
  double J[9], Jinv[9];
  double Q[NX * NX], R[NU * NU], QN[NX * NX];
  double dt, s;
} oracle_params;

static void f_eval(const double* x, const double* u, const oracle_params* P, const double* w, double* f, double* Jf /* NX x NZ or NULL */) {
  const double sf = sin(x[3]), cf = cos(x[3]), st = sin(x[4]), ct = cos(x[4]), sp = sin(x[5]), cp = cos(x[5]);
  const double ict = 1.0 / ct, tt = st * ict;
  const double wx = x[9], wy = x[10], wz = x[11];
  f[0] = x[6]; f[1] = x[7]; f[2] = x[8];
  const double a = sf * wy + cf * wz, b = cf * wy - sf * wz;
  f[3] = wx + tt * a; f[4] = b; f[5] = a * ict;
  const double Tt = u[0] + u[1] + u[2] + u[3] + P->t_blast, s = Tt * P->minv;
  const double r0 = cp * cf * st + sp * sf, r1 = sp * cf * st - cp * sf, r2 = cf * ct;
  f[6] = r0 * s; f[7] = r1 * s; f[8] = r2 * s - P->g;
  if (w) { f[6] += w[0] * P->minv; f[7] += w[1] * P->minv; f[8] += w[2] * P->minv; }   /* c5 wind force */
  const double* J = P->J;
  const double jw0 = J[0] * wx + J[1] * wy + J[2] * wz, jw1 = J[3] * wx + J[4] * wy + J[5] * wz,
               jw2 = J[6] * wx + J[7] * wy + J[8] * wz;
  const double m0 = (u[1] + u[3] - u[0] - u[2]) * P->ly - (wy * jw2 - wz * jw1);
  const double m1 = (u[1] + u[2] - u[0] - u[3]) * P->lx - (wz * jw0 - wx * jw2);
  const double m2 = (u[2] + u[3] - u[0] - u[1]) * P->c - (wx * jw1 - wy * jw0);
  const double* Ji = P->Jinv;
  f[9] = Ji[0] * m0 + Ji[1] * m1 + Ji[2] * m2;
  f[10] = Ji[3] * m0 + Ji[4] * m1 + Ji[5] * m2;
  f[11] = Ji[6] * m0 + Ji[7] * m1 + Ji[8] * m2;
  if (!Jf) return;
  memset(Jf, 0, sizeof(double) * NX * NZ);
#define JF(i, j) Jf[(i) * NZ + (j)]
  JF(0, 6) = 1; JF(1, 7) = 1; JF(2, 8) = 1;
  JF(3, 9) = 1; JF(3, 10) = sf * tt; JF(3, 11) = cf * tt;
  JF(4, 10) = cf; JF(4, 11) = -sf;
  JF(5, 10) = sf * ict; JF(5, 11) = cf * ict;
  JF(3, 3) = tt * b; JF(4, 3) = -sf * wy - cf * wz; JF(5, 3) = b * ict;
  JF(3, 4) = a * ict * ict; JF(5, 4) = a * st * ict * ict;
  JF(6, 3) = (-cp * sf * st + sp * cf) * s; JF(7, 3) = (-sp * sf * st - cp * cf) * s; JF(8, 3) = -sf * ct * s;
  JF(6, 4) = cp * cf * ct * s; JF(7, 4) = sp * cf * ct * s; JF(8, 4) = -cf * st * s;
  JF(6, 5) = (-sp * cf * st + cp * sf) * s; JF(7, 5) = (cp * cf * st + sp * sf) * s;
  for (int m = 0; m < NU; ++m) { JF(6, 12 + m) = r0 * P->minv; JF(7, 12 + m) = r1 * P->minv; JF(8, 12 + m) = r2 * P->minv; }
  /* d(w x Jw)/dw = [w]x J - [Jw]x */
  const double S[9] = {0, -wz, wy, wz, 0, -wx, -wy, wx, 0};
  const double Sj[9] = {0, -jw2, jw1, jw2, 0, -jw0, -jw1, jw0, 0};
  double D[9];
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 3; ++k) {
      double acc = -Sj[i * 3 + k];
      for (int l = 0; l < 3; ++l) acc += S[i * 3 + l] * J[l * 3 + k];
      D[i * 3 + k] = acc;
    }
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 3; ++k) {
      double acc = 0;
      for (int l = 0; l < 3; ++l) acc -= Ji[i * 3 + l] * D[l * 3 + k];
      JF(9 + i, 9 + k) = acc;
    }
  const double dM[12] = {-P->ly, P->ly, -P->ly, P->ly, -P->lx, P->lx, P->lx, -P->lx, -P->c, -P->c, P->c, P->c};
  for (int i = 0; i < 3; ++i)
    for (int m = 0; m < NU; ++m) {
      double acc = 0;
      for (int l = 0; l < 3; ++l) acc += Ji[i * 3 + l] * dM[l * 4 + m];
      JF(9 + i, 12 + m) = acc;
    }
#undef JF
}

/* x_next and S = [A | B] (NX x NZ, row-major) */
static void rk4_sens(const double* x, const double* u, const oracle_params* P, const double* w, double* xn, double* S) {
  const double h = P->dt;
  double k[4][NX], dk[4][NX * NZ], xs[NX], Jf[NX * NZ], Ss[NX * NZ];
  double S0[NX * NZ];
  memset(S0, 0, sizeof S0);
  for (int i = 0; i < NX; ++i) S0[i * NZ + i] = 1.0;
  const double c[4] = {0.0, 0.5, 0.5, 1.0};
  for (int st = 0; st < 4; ++st) {
    for (int i = 0; i < NX; ++i) xs[i] = st ? x[i] + c[st] * h * k[st - 1][i] : x[i];
    for (int i = 0; i < NX * NZ; ++i) Ss[i] = st ? S0[i] + c[st] * h * dk[st - 1][i] : S0[i];
    f_eval(xs, u, P, w, k[st], Jf);
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NZ; ++j) {
        double acc = (j >= NX) ? Jf[i * NZ + j] : 0.0;
        for (int l = 0; l < NX; ++l) acc += Jf[i * NZ + l] * Ss[l * NZ + j];
        dk[st][i * NZ + j] = acc;
      }
  }
  for (int i = 0; i < NX; ++i) xn[i] = x[i] + h / 6.0 * (k[0][i] + 2.0 * k[1][i] + 2.0 * k[2][i] + k[3][i]);
  for (int i = 0; i < NX * NZ; ++i) S[i] = S0[i] + h / 6.0 * (dk[0][i] + 2.0 * dk[1][i] + 2.0 * dk[2][i] + dk[3][i]);
}

static int chol_solve4(const double* H, double* Bm /* NU x ncols, overwritten */, int ncols) {
  double L[16] = {0};
  for (int i = 0; i < NU; ++i)
    for (int j = 0; j <= i; ++j) {
      double acc = H[i * NU + j];
      for (int k = 0; k < j; ++k) acc -= L[i * NU + k] * L[j * NU + k];
      if (i == j) { if (!(acc > 0)) return -1; L[i * NU + i] = sqrt(acc); }
      else L[i * NU + j] = acc / L[j * NU + j];
    }
  for (int c = 0; c < ncols; ++c) {
    double y[NU];
    for (int i = 0; i < NU; ++i) {
      double acc = Bm[i * ncols + c];
      for (int k = 0; k < i; ++k) acc -= L[i * NU + k] * y[k];
      y[i] = acc / L[i * NU + i];
    }
    for (int i = NU - 1; i >= 0; --i) {
      double acc = y[i];
      for (int k = i + 1; k < NU; ++k) acc -= L[k * NU + i] * Bm[k * ncols + c];
      Bm[i * ncols + c] = acc / L[i * NU + i];
    }
  }
  return 0;
}

static int solve_one(int N, const oracle_params* P, const double* x0, const double* xr, const double* ur,
                     const double* w, double* u0, double* X, double* U, double* work) {
  double* xb = work;                     /* (N+1) x NX */
  double* S = xb + (N + 1) * NX;         /* N x NX x NZ */
  double* K = S + N * NX * NZ;           /* N x NU x NX */
  double* kf = K + N * NU * NX;          /* N x NU */
  memcpy(xb, x0, sizeof(double) * NX);
  for (int k = 0; k < N; ++k) rk4_sens(xb + k * NX, ur + k * NU, P, w, xb + (k + 1) * NX, S + k * NX * NZ);
  double Pm[NX * NX], p[NX], e[NX];
  memcpy(Pm, P->QN, sizeof Pm);
  for (int i = 0; i < NX; ++i) e[i] = xb[N * NX + i] - xr[N * NX + i];
  for (int i = 0; i < NX; ++i) { double acc = 0; for (int j = 0; j < NX; ++j) acc += P->QN[i * NX + j] * e[j]; p[i] = acc; }
  for (int k = N - 1; k >= 0; --k) {
    const double* Sk = S + k * NX * NZ;
    double PS[NX * NZ], H[NZ * NZ], h[NZ];
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NZ; ++j) { double acc = 0; for (int l = 0; l < NX; ++l) acc += Pm[i * NX + l] * Sk[l * NZ + j]; PS[i * NZ + j] = acc; }
    for (int i = 0; i < NZ; ++i)
      for (int j = 0; j < NZ; ++j) { double acc = 0; for (int l = 0; l < NX; ++l) acc += Sk[l * NZ + i] * PS[l * NZ + j]; H[i * NZ + j] = acc; }
    for (int j = 0; j < NZ; ++j) { double acc = 0; for (int l = 0; l < NX; ++l) acc += Sk[l * NZ + j] * p[l]; h[j] = acc; }
    for (int i = 0; i < NX; ++i) e[i] = xb[k * NX + i] - xr[k * NX + i];
    for (int i = 0; i < NX; ++i) {
      double acc = 0;
      for (int j = 0; j < NX; ++j) { H[i * NZ + j] += P->s * P->Q[i * NX + j]; acc += P->Q[i * NX + j] * e[j]; }
      h[i] += P->s * acc;
    }
    for (int m = 0; m < NU; ++m) {
      double acc = 0;
      for (int n = 0; n < NU; ++n) { H[(NX + m) * NZ + NX + n] += P->s * P->R[m * NU + n]; acc += P->R[m * NU + n] * (ur[k * NU + n] - ur[k * NU + n]); }
      h[NX + m] += P->s * acc;   /* ubar = uref in rollout mode */
    }
    double Huu[16], rhs[NU * (NX + 1)];
    for (int m = 0; m < NU; ++m) {
      for (int n = 0; n < NU; ++n) Huu[m * NU + n] = H[(NX + m) * NZ + NX + n];
      for (int i = 0; i < NX; ++i) rhs[m * (NX + 1) + i] = -H[(NX + m) * NZ + i];
      rhs[m * (NX + 1) + NX] = -h[NX + m];
    }
    if (chol_solve4(Huu, rhs, NX + 1)) return 4;
    for (int m = 0; m < NU; ++m) {
      for (int i = 0; i < NX; ++i) K[(k * NU + m) * NX + i] = rhs[m * (NX + 1) + i];
      kf[k * NU + m] = rhs[m * (NX + 1) + NX];
    }
    double Pn[NX * NX];
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NX; ++j) {
        double acc = H[i * NZ + j];
        for (int m = 0; m < NU; ++m) acc += H[(NX + m) * NZ + i] * K[(k * NU + m) * NX + j];
        Pn[i * NX + j] = acc;
      }
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NX; ++j) Pm[i * NX + j] = 0.5 * (Pn[i * NX + j] + Pn[j * NX + i]);
    for (int i = 0; i < NX; ++i) {
      double acc = h[i];
      for (int m = 0; m < NU; ++m) acc += H[(NX + m) * NZ + i] * kf[k * NU + m];
      p[i] = acc;
    }
  }
  double dx[NX];
  memset(dx, 0, sizeof dx);
  for (int k = 0; k < N; ++k) {
    double du[NU];
    for (int m = 0; m < NU; ++m) {
      double acc = kf[k * NU + m];
      for (int i = 0; i < NX; ++i) acc += K[(k * NU + m) * NX + i] * dx[i];
      du[m] = acc;
    }
    if (X) for (int i = 0; i < NX; ++i) X[k * NX + i] = xb[k * NX + i] + dx[i];
    if (U) for (int m = 0; m < NU; ++m) U[k * NU + m] = ur[k * NU + m] + du[m];
    if (k == 0) for (int m = 0; m < NU; ++m) u0[m] = ur[m] + du[m];
    const double* Sk = S + k * NX * NZ;
    double dn[NX];
    for (int i = 0; i < NX; ++i) {
      double acc = 0;
      for (int j = 0; j < NX; ++j) acc += Sk[i * NZ + j] * dx[j];
      for (int m = 0; m < NU; ++m) acc += Sk[i * NZ + NX + m] * du[m];
      dn[i] = acc;
    }
    memcpy(dx, dn, sizeof dx);
  }
  if (X) for (int i = 0; i < NX; ++i) X[N * NX + i] = xb[N * NX + i] + dx[i];
  return 0;
}

#include <stdlib.h>

/* ---- input box: oracle/ocp.py pdas_solve (rollout mode: ubar = uref, zero gaps, dx_0 = 0) ---- */
typedef struct { double lbu[NU], ubu[NU]; int max_iter, pbar; } box_params;

/* One masked Riccati pass + forward pass with multipliers (oracle/ocp.py riccati_solve with
 * fixed / delta): fixed inputs du = delta, the others free.  Writes du, dx, mu; returns 0 or 4. */
static int masked_pass(int N, const oracle_params* P, const double* xb, const double* S, const double* xr,
                       const double* ur, const unsigned char* fixed, const double* delta, double* K,
                       double* kf, double* Huus, double* Huxs, double* hus, double* dx, double* du,
                       double* mu) {
  double Pm[NX * NX], p[NX], e[NX];
  memcpy(Pm, P->QN, sizeof Pm);
  for (int i = 0; i < NX; ++i) e[i] = xb[N * NX + i] - xr[N * NX + i];
  for (int i = 0; i < NX; ++i) { double acc = 0; for (int j = 0; j < NX; ++j) acc += P->QN[i * NX + j] * e[j]; p[i] = acc; }
  for (int k = N - 1; k >= 0; --k) {
    const double* Sk = S + k * NX * NZ;
    double PS[NX * NZ], H[NZ * NZ], h[NZ];
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NZ; ++j) { double acc = 0; for (int l = 0; l < NX; ++l) acc += Pm[i * NX + l] * Sk[l * NZ + j]; PS[i * NZ + j] = acc; }
    for (int i = 0; i < NZ; ++i)
      for (int j = 0; j < NZ; ++j) { double acc = 0; for (int l = 0; l < NX; ++l) acc += Sk[l * NZ + i] * PS[l * NZ + j]; H[i * NZ + j] = acc; }
    for (int j = 0; j < NZ; ++j) { double acc = 0; for (int l = 0; l < NX; ++l) acc += Sk[l * NZ + j] * p[l]; h[j] = acc; }
    for (int i = 0; i < NX; ++i) e[i] = xb[k * NX + i] - xr[k * NX + i];
    for (int i = 0; i < NX; ++i) {
      double acc = 0;
      for (int j = 0; j < NX; ++j) { H[i * NZ + j] += P->s * P->Q[i * NX + j]; acc += P->Q[i * NX + j] * e[j]; }
      h[i] += P->s * acc;
    }
    for (int m = 0; m < NU; ++m)
      for (int n = 0; n < NU; ++n) H[(NX + m) * NZ + NX + n] += P->s * P->R[m * NU + n];   /* ubar = uref */
    double* Huu = Huus + k * NU * NU;
    double* Hux = Huxs + k * NU * NX;
    double* hu = hus + k * NU;
    for (int m = 0; m < NU; ++m) {
      for (int n = 0; n < NU; ++n) Huu[m * NU + n] = H[(NX + m) * NZ + NX + n];
      for (int i = 0; i < NX; ++i) Hux[m * NX + i] = H[(NX + m) * NZ + i];
      hu[m] = h[NX + m];
    }
    /* the masked stage (oracle/ocp.py _masked_stage) */
    const unsigned char* fk = fixed + k * NU;
    const double* dk = delta + k * NU;
    double Ht[16], rhs[NU * (NX + 1)];
    for (int m = 0; m < NU; ++m) {
      double ht = hu[m];
      for (int n = 0; n < NU; ++n) ht += fk[n] ? Huu[m * NU + n] * dk[n] : 0.0;
      for (int n = 0; n < NU; ++n) Ht[m * NU + n] = (fk[m] || fk[n]) ? (m == n ? 1.0 : 0.0) : Huu[m * NU + n];
      for (int i = 0; i < NX; ++i) rhs[m * (NX + 1) + i] = fk[m] ? 0.0 : -Hux[m * NX + i];
      rhs[m * (NX + 1) + NX] = fk[m] ? dk[m] : -ht;
    }
    if (chol_solve4(Ht, rhs, NX + 1)) return 4;
    for (int m = 0; m < NU; ++m) {
      for (int i = 0; i < NX; ++i) K[(k * NU + m) * NX + i] = rhs[m * (NX + 1) + i];
      kf[k * NU + m] = rhs[m * (NX + 1) + NX];
    }
    double Pn[NX * NX];
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NX; ++j) {
        double acc = H[i * NZ + j];
        for (int m = 0; m < NU; ++m) acc += Hux[m * NX + i] * K[(k * NU + m) * NX + j];
        Pn[i * NX + j] = acc;
      }
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NX; ++j) Pm[i * NX + j] = 0.5 * (Pn[i * NX + j] + Pn[j * NX + i]);
    for (int i = 0; i < NX; ++i) {
      double acc = h[i];
      for (int m = 0; m < NU; ++m) acc += Hux[m * NX + i] * kf[k * NU + m];
      p[i] = acc;
    }
  }
  memset(dx, 0, sizeof(double) * NX);
  for (int k = 0; k < N; ++k) {
    const double* xk = dx + k * NX;
    double* uk = du + k * NU;
    for (int m = 0; m < NU; ++m) {
      double acc = kf[k * NU + m];
      for (int i = 0; i < NX; ++i) acc += K[(k * NU + m) * NX + i] * xk[i];
      uk[m] = acc;
    }
    for (int m = 0; m < NU; ++m) {
      double acc = hus[k * NU + m];
      for (int n = 0; n < NU; ++n) acc += Huus[k * NU * NU + m * NU + n] * uk[n];
      for (int i = 0; i < NX; ++i) acc += Huxs[k * NU * NX + m * NX + i] * xk[i];
      mu[k * NU + m] = acc;
    }
    const double* Sk = S + k * NX * NZ;
    for (int i = 0; i < NX; ++i) {
      double acc = 0;
      for (int j = 0; j < NX; ++j) acc += Sk[i * NZ + j] * xk[j];
      for (int m = 0; m < NU; ++m) acc += Sk[i * NZ + NX + m] * uk[m];
      dx[(k + 1) * NX + i] = acc;
    }
  }
  return 0;
}

static int solve_one_box(int N, const oracle_params* P, const box_params* bp, const double* x0, const double* xr,
                         const double* ur, double* u0, double* X, double* U, int* iters, double* work,
                         unsigned char* flags) {
  double* xb = work;                     /* (N+1) x NX */
  double* S = xb + (N + 1) * NX;         /* N x NX x NZ */
  double* K = S + N * NX * NZ;           /* N x NU x NX */
  double* kf = K + N * NU * NX;          /* N x NU */
  double* Huus = kf + N * NU;            /* N x NU x NU */
  double* Huxs = Huus + N * NU * NU;     /* N x NU x NX */
  double* hus = Huxs + N * NU * NX;      /* N x NU */
  double* dx = hus + N * NU;             /* (N+1) x NX */
  double* du = dx + (N + 1) * NX;        /* N x NU */
  double* mu = du + N * NU;              /* N x NU */
  double* delta = mu + N * NU;           /* N x NU */
  unsigned char* low = flags;            /* N x NU */
  unsigned char* up = low + N * NU;
  unsigned char* fixed = up + N * NU;
  unsigned char* V = fixed + N * NU;
  memcpy(xb, x0, sizeof(double) * NX);
  for (int k = 0; k < N; ++k) rk4_sens(xb + k * NX, ur + k * NU, P, NULL, xb + (k + 1) * NX, S + k * NX * NZ);
  memset(low, 0, 2 * N * NU);
  int best = 0x7fffffff, pcount = bp->pbar, done = 0, st = 0, it;
  for (it = 0; it < bp->max_iter; ++it) {
    for (int e = 0; e < N * NU; ++e) {
      const int m = e % NU;
      fixed[e] = low[e] | up[e];
      delta[e] = low[e] ? bp->lbu[m] - ur[e] : (up[e] ? bp->ubu[m] - ur[e] : 0.0);
    }
    if (masked_pass(N, P, xb, S, xr, ur, fixed, delta, K, kf, Huus, Huxs, hus, dx, du, mu)) { st = 4; ++it; break; }
    int nV = 0, first = -1;
    for (int e = 0; e < N * NU; ++e) {
      const int m = e % NU;
      const double u = ur[e] + du[e];
      V[e] = 0;
      if (!fixed[e] && u < bp->lbu[m]) V[e] = 1;          /* v_lo */
      else if (!fixed[e] && u > bp->ubu[m]) V[e] = 2;     /* v_hi */
      else if (low[e] && mu[e] < 0) V[e] = 3;             /* v_fl */
      else if (up[e] && mu[e] > 0) V[e] = 4;              /* v_fu */
      if (V[e]) { ++nV; if (first < 0) first = e; }
    }
    if (nV == 0) { done = 1; ++it; break; }
    const int full = (nV < best) || (pcount > 0);
    pcount = (nV < best) ? bp->pbar : (full ? pcount - 1 : pcount);
    if (nV < best) best = nV;
    for (int e = 0; e < N * NU; ++e) {
      if (!V[e] || (!full && e != first)) continue;
      if (V[e] == 1) low[e] = 1;
      else if (V[e] == 2) up[e] = 1;
      else if (V[e] == 3) low[e] = 0;
      else up[e] = 0;
    }
  }
  if (!st && !done) st = 2;
  *iters = it;
  for (int k = 0; k <= N; ++k)
    if (X) for (int i = 0; i < NX; ++i) X[k * NX + i] = xb[k * NX + i] + dx[k * NX + i];
  for (int k = 0; k < N; ++k)
    if (U) for (int m = 0; m < NU; ++m) U[k * NU + m] = ur[k * NU + m] + du[k * NU + m];
  for (int m = 0; m < NU; ++m) u0[m] = ur[m] + du[m];
  return st;
}

/* Input-box rollout-mode solve (BASELINE c4) for B instances; returns the number of non-OK ones. */
int mpc_oracle_solve_box(int B, int N, const oracle_params* P, const double* lbu, const double* ubu,
                         int max_iter, const double* x0, const double* xref, long xref_sb,
                         const double* uref, long uref_sb, double* u0, double* X, double* U,
                         int* status, int* iters, int nthreads) {
  box_params bp;
  memcpy(bp.lbu, lbu, sizeof bp.lbu);
  memcpy(bp.ubu, ubu, sizeof bp.ubu);
  bp.max_iter = max_iter;
  bp.pbar = 3;
  int bad = 0;
  const size_t wsz = (size_t)(N + 1) * NX * 2 + (size_t)N * (NX * NZ + NU * NX * 2 + NU * NU + NU * 5);
#pragma omp parallel num_threads(nthreads) reduction(+ : bad)
  {
    double* work = (double*)malloc(sizeof(double) * wsz);
    unsigned char* flags = (unsigned char*)malloc((size_t)4 * N * NU);
#pragma omp for schedule(dynamic, 16)
    for (int b = 0; b < B; ++b) {
      int it = 0;
      int st = solve_one_box(N, P, &bp, x0 + (size_t)b * NX, xref + (size_t)b * xref_sb, uref + (size_t)b * uref_sb,
                             u0 + (size_t)b * NU, X ? X + (size_t)b * (N + 1) * NX : NULL,
                             U ? U + (size_t)b * N * NU : NULL, &it, work, flags);
      if (status) status[b] = st;
      if (iters) iters[b] = it;
      bad += st != 0;
    }
    free(flags);
    free(work);
  }
  return bad;
}

/* Unconstrained rollout-mode solve for B instances; returns the number of failed instances. */
int mpc_oracle_solve(int B, int N, const oracle_params* P, const double* x0, const double* xref,
                     long xref_sb, const double* uref, long uref_sb, const double* wind, long wind_sb,
                     double* u0, double* X, double* U, int* status, int nthreads) {
  int bad = 0;
  const size_t wsz = (size_t)(N + 1) * NX + (size_t)N * NX * NZ + (size_t)N * NU * NX + (size_t)N * NU;
#pragma omp parallel num_threads(nthreads) reduction(+ : bad)
  {
    double* work = (double*)malloc(sizeof(double) * wsz);
#pragma omp for schedule(static)
    for (int b = 0; b < B; ++b) {
      int st = solve_one(N, P, x0 + (size_t)b * NX, xref + (size_t)b * xref_sb, uref + (size_t)b * uref_sb,
                         wind ? wind + (size_t)b * wind_sb : NULL, u0 + (size_t)b * NU, X ? X + (size_t)b * (N + 1) * NX : NULL,
                         U ? U + (size_t)b * N * NU : NULL, work);
      if (status) status[b] = st;
      bad += st != 0;
    }
    free(work);
  }
  return bad;
}

/* Per-instance latency at the c1 shape (the reference's one-solve-per-control-step
 * loop simulation_blaster.py:56-107): R single-instance solves on the calling thread, each timed
 * with CLOCK_MONOTONIC into ns[r] (instance r % B of x0, so the draws vary).  No Python in the
 * timed region.  Returns the number of failed solves. */
int mpc_oracle_latency_b1(int B, int N, const oracle_params* P, const double* x0, const double* xref,
                          const double* uref, int R, double* ns) {
  const size_t wsz = (size_t)(N + 1) * NX + (size_t)N * NX * NZ + (size_t)N * NU * NX + (size_t)N * NU;
  double* work = (double*)malloc(sizeof(double) * wsz);
  double* X = (double*)malloc(sizeof(double) * (size_t)(N + 1) * NX);
  double* U = (double*)malloc(sizeof(double) * (size_t)N * NU);
  double u0[NU];
  int bad = 0;
  for (int r = 0; r < R; ++r) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    bad += solve_one(N, P, x0 + (size_t)(r % B) * NX, xref, uref, NULL, u0, X, U, work) != 0;
    clock_gettime(CLOCK_MONOTONIC, &t1);
    ns[r] = (double)(t1.tv_sec - t0.tv_sec) * 1e9 + (double)(t1.tv_nsec - t0.tv_nsec);
  }
  free(work); free(X); free(U);
  return bad;
}
