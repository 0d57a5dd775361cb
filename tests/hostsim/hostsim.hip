// Host-side driver of the per-lane device functions in dat_core.hpp (TEST-ONLY).
//
// Compiled with hipcc into tests/hostsim/libdat_hostsim.so and loaded only by tests/ (never by
// the product package): it runs the exact __host__ __device__ code of one GPU lane on the CPU so
// the reduced-QP algebra, the env rows and the rollout can be checked against the oracle in the
// dev container, which has no GPU.  The product path has no CPU fallback.
#include "../../distributed_aerial_transportation_amd/csrc/dat_core.hpp"

using namespace dat;

#ifndef HS_TOL
#define HS_TOL 1e-10
#endif

extern "C" {

int hs_qp_cadmm(const double* prm, int n, const double* st, const double* acc, const double* env_lhs,
                const double* env_rhs, int nenv, int i, const double* lam, const double* fbar, double rho,
                double* f_out, int* iters) {
  double Rt_all[16 * 9];
  const double* Rl = st + DAT_S_RL(n);
  for (int j = 0; j < n; ++j) make_Rt(prm + DAT_P_RCOM(n) + 3 * j, Rl, Rt_all + 9 * j);
  QP<1> P;
  build_cadmm_static(P, prm, n, st, acc, i, Rt_all);
  add_env_rows(P, nenv, (const double(*)[3])env_lhs, env_rhs);
  build_cadmm_dynamic(P, prm, n, i, Rt_all, lam, fbar, rho);
  double y[1][3], w[6];
  IPMOut o = ipm_solve<MODE_CADMM, 1>(P, y, w, 50, HS_TOL);
  cadmm_materialize(P, n, i, Rt_all, lam, fbar, y[0], o.pi, f_out);
  *iters = o.iters;
  return o.status;
}

int hs_qp_dd(const double* prm, int n, const double* st, const double* acc, const double* env_lhs,
             const double* env_rhs, int nenv, int i, const double* c9, double* x_out, int* iters) {
  double Rt[9];
  make_Rt(prm + DAT_P_RCOM(n) + 3 * i, st + DAT_S_RL(n), Rt);
  QP<1> P;
  build_dd_static(P, prm, n, st, acc, i, Rt);
  set_dd_price(P, prm, n, i, c9);
  add_env_rows(P, nenv, (const double(*)[3])env_lhs, env_rhs);
  double y[1][3], w[6];
  IPMOut o = ipm_solve<MODE_DD, 1>(P, y, w, 50, HS_TOL);
  for (int c = 0; c < 3; ++c) x_out[c] = y[0][c];
  for (int c = 0; c < 6; ++c) x_out[3 + c] = w[c];
  *iters = o.iters;
  return o.status;
}

int hs_qp_cent(const double* prm, int n, const double* st, const double* acc, const double* env_lhs,
               const double* env_rhs, int nenv, double* f_out, int* iters) {
  if (n != 3 && n != 6) return -1;
  int status;
  if (n == 3) {
    QP<3> P;
    build_cent(P, prm, n, st, acc);
    add_env_rows(P, nenv, (const double(*)[3])env_lhs, env_rhs);
    double y[3][3], w[6];
    IPMOut o = ipm_solve<MODE_CENT, 3>(P, y, w, 50, HS_TOL);
    for (int k = 0; k < 3; ++k)
      for (int c = 0; c < 3; ++c) f_out[3 * k + c] = y[k][c];
    *iters = o.iters;
    status = o.status;
  } else {
    QP<6> P;
    build_cent(P, prm, n, st, acc);
    add_env_rows(P, nenv, (const double(*)[3])env_lhs, env_rhs);
    double y[6][3], w[6];
    IPMOut o = ipm_solve<MODE_CENT, 6>(P, y, w, 50, HS_TOL);
    for (int k = 0; k < 6; ++k)
      for (int c = 0; c < 3; ++c) f_out[3 * k + c] = y[k][c];
    *iters = o.iters;
    status = o.status;
  }
  return status;
}

int hs_env_rows(const double* prm, int n, const double* st, const double* trees, int ntree, int agent,
                double alpha, double* lhs, double* rhs, int* collision, double* min_dist) {
  int nrow = 0;
  EnvOut e = env_rows(prm, n, st, trees, ntree, agent, alpha, &nrow, (double(*)[3])lhs, rhs);
  *collision = e.collision;
  *min_dist = e.min_env_dist;
  return nrow;
}

void hs_sim_step(const double* prm, int n, double* st, int* counter, const double* fdes, double dt) {
  sim_step<16>(prm, n, st, counter, fdes, dt);
}

void hs_ll_control(const double* R, const double* w, const double* J, const double* fdes, double* f, double* M) {
  ll_control_agent(R, w, J, fdes, f, M);
}

void hs_desired_accel(const double* st, int n, const double* mountain, double x_offset, double* acc) {
  desired_accel_forest(st, n, mountain, x_offset, acc);
}
}
