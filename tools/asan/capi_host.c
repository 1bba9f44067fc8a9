/* Host-side validation of the C ABI (include/mpcb.h) under AddressSanitizer / UBSan, on a CPU
 * host with no GPU (tools/asan_cpu.sh).  Every entry point's argument checks and error path run
 * here: null handles and pointers, unsupported shapes, bad horizons / dtypes / boxes, a singular
 * inertia, and mpcb_create's no-device path.  No kernel is launched. */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "../../include/mpcb.h"

static double Q[MPCB_MAX_NX * MPCB_MAX_NX], R[36], QN[MPCB_MAX_NX * MPCB_MAX_NX];
static int fails = 0;

static void expect_err(int rc, const char* what) {
  const char* m = mpcb_last_error();
  if (rc >= 0 || !m || !m[0]) { printf("FAIL %s: rc=%d msg='%s'\n", what, rc, m ? m : "(null)"); ++fails; }
  else printf("ok   %-34s rc=%d  %s\n", what, rc, m);
}

static mpcb_config base(void) {
  mpcb_config c;
  memset(&c, 0, sizeof c);
  c.nx = 12; c.nu = 4; c.N = 20; c.dtype = MPCB_F64;
  c.dt = 1.0 / 30; c.mass = 9.0; c.g = 9.81; c.lx = 0.3434; c.ly = 0.3475; c.c = 0.03;
  c.J[0] = 0.50781; c.J[4] = 0.47314; c.J[8] = 0.72975;
  for (int i = 0; i < 12; ++i) { Q[i * 12 + i] = 1e3; QN[i * 12 + i] = 1e4; }
  for (int i = 0; i < 4; ++i) R[i * 4 + i] = 0.05;
  memcpy(c.Q, Q, sizeof c.Q < sizeof Q ? sizeof c.Q : sizeof Q);
  memcpy(c.R, R, sizeof c.R < sizeof R ? sizeof c.R : sizeof R);
  memcpy(c.QN, QN, sizeof c.QN < sizeof QN ? sizeof c.QN : sizeof QN);
  c.cost_scale = c.dt; c.max_as_iter = 200;
  return c;
}

int main(void) {
  mpcb_handle* h = NULL;
  mpcb_config c = base();
  if (mpcb_abi_version() != MPCB_ABI_VERSION) { printf("FAIL abi\n"); ++fails; }
  expect_err(mpcb_create(NULL, 0, 16, &h), "create(null cfg)");
  expect_err(mpcb_create(&c, 0, 16, NULL), "create(null out)");
  c = base(); c.nx = 13; expect_err(mpcb_create(&c, 0, 16, &h), "create(nx=13)");
  c = base(); c.N = 0; expect_err(mpcb_create(&c, 0, 16, &h), "create(N=0)");
  c = base(); c.N = 5000; expect_err(mpcb_create(&c, 0, 16, &h), "create(N=5000)");
  c = base(); c.dtype = 7; expect_err(mpcb_create(&c, 0, 16, &h), "create(dtype=7)");
  c = base(); c.dt = -1; expect_err(mpcb_create(&c, 0, 16, &h), "create(dt<0)");
  c = base(); c.mass = NAN; expect_err(mpcb_create(&c, 0, 16, &h), "create(mass=nan)");
  c = base(); expect_err(mpcb_create(&c, 0, 0, &h), "create(max_batch=0)");
  c = base(); c.box_u = 1; c.N = 65; for (int m = 0; m < 4; ++m) c.ubu[m] = 65;
  expect_err(mpcb_create(&c, 0, 16, &h), "create(12/4 box N=65)");
  c = base(); c.box_u = 1; c.max_as_iter = 0; for (int m = 0; m < 4; ++m) c.ubu[m] = 65;
  expect_err(mpcb_create(&c, 0, 16, &h), "create(max_as_iter=0)");
  c = base(); c.box_x = 1; expect_err(mpcb_create(&c, 0, 16, &h), "create(12/4 box_x)");
  c = base(); c.nx = 17; c.nu = 6; c.box_u = 1; c.box_x = 1; c.dtype = MPCB_F32;
  for (int m = 0; m < 6; ++m) c.ubu[m] = 1;
  for (int i = 0; i < 17; ++i) c.ubx[i] = 1;
  expect_err(mpcb_create(&c, 0, 16, &h), "create(17/6 box_x f32)");
  c = base(); c.nx = 17; c.nu = 6; c.box_u = 1; expect_err(mpcb_create(&c, 0, 16, &h), "create(17/6 lbu==ubu)");
  c = base(); memset(c.J, 0, sizeof c.J); expect_err(mpcb_create(&c, 0, 16, &h), "create(singular J)");
  c = base(); expect_err(mpcb_create(&c, -1, 16, &h), "create(device -1)");
  c = base(); expect_err(mpcb_create(&c, 0, 16, &h), "create(no GPU on this host)");
  if (h) { printf("FAIL handle set after a failed create\n"); ++fails; }
  /* every handle-taking entry point refuses a null handle */
  double buf[64];
  int32_t st[4];
  float ms[4];
  expect_err(mpcb_solve(NULL, 1, buf, 0, buf, 0, buf, 0, NULL, 0, buf, buf, buf, st, NULL), "solve(null handle)");
  expect_err(mpcb_solve_iterate(NULL, 1, buf, 0, buf, buf, buf, 0, buf, 0, NULL, 0, buf, buf, buf, st, NULL),
             "solve_iterate(null handle)");
  expect_err(mpcb_linearize(NULL, 1, buf, buf, NULL, 0, buf, buf, buf, NULL), "linearize(null handle)");
  expect_err(mpcb_sim_step(NULL, 1, buf, buf, NULL, 0, 1.0 / 30, buf, NULL), "sim_step(null handle)");
  expect_err(mpcb_gen_inputs(NULL, 1, 1, 0, 0, buf, buf, 0, buf, 0, NULL, NULL), "gen_inputs(null handle)");
  expect_err(mpcb_histogram(NULL, 1, buf, 0, 65, 64, NULL, NULL), "histogram(null handle)");
  expect_err(mpcb_qp_stats(NULL, 1, st, NULL), "qp_stats(null handle)");
  expect_err(mpcb_set_timing(NULL, 1), "set_timing(null handle)");
  expect_err(mpcb_last_timing(NULL, ms), "last_timing(null handle)");
  expect_err(mpcb_set_params(NULL, 1, buf, 0, 0), "set_params(null handle)");
  expect_err(mpcb_set_t_blast(NULL, 1.0), "set_t_blast(null handle)");
  expect_err(mpcb_quat_ops(-1, NULL, NULL, NULL, NULL, NULL, NULL), "quat_ops(B=-1)");
  expect_err(mpcb_poc_jacobians(-1, NULL, 0, NULL, 1, 0, NULL, NULL, NULL, NULL, NULL, NULL, NULL), "poc_jacobians(B=-1)");
  if (mpcb_workspace_bytes(NULL) != 0 || mpcb_path(NULL) != -1) { printf("FAIL null getters\n"); ++fails; }
  mpcb_destroy(NULL);
  printf(fails ? "capi_host: %d FAILURES\n" : "capi_host: all checks passed\n", fails);
  return fails != 0;
}
