// Host-side driver of the per-lane device functions in dat_core.hpp (TEST-ONLY).
//
// Compiled with hipcc into tests/hostsim/libdat_hostsim.so and loaded only by tests/ (never by
// the product package): it runs the exact __host__ __device__ code of one GPU lane on the CPU so
// the reduced-QP algebra, the env rows and the rollout can be checked against the oracle in the
// dev container, which has no GPU.  The product path has no CPU fallback.
#include "../../distributed_aerial_transportation_amd/csrc/dat_qp.hpp"

using namespace dat;

#ifndef HS_TOL
#define HS_TOL 1e-10
#endif

namespace {
// compacted (nenv x 3, nenv) env rows -> slot arrays + mask
void env_slots(const double* env_lhs, const double* env_rhs, int nenv, double lhs[DAT_NENV][3], double rhs[DAT_NENV],
               unsigned* mask) {
  *mask = 0u;
  for (int j = 0; j < DAT_NENV; ++j) {
    lhs[j][0] = lhs[j][1] = lhs[j][2] = 0.0;
    rhs[j] = 0.0;
    if (j < nenv) {
      for (int c = 0; c < 3; ++c) lhs[j][c] = env_lhs[3 * j + c];
      rhs[j] = env_rhs[j];
      *mask |= 1u << j;
    }
  }
}
// diagnostics of the last solve (hs_last_diag)
double g_merit = 0.0;
int g_inband = 0, g_why = 0;
int g_refs = 0, g_corrs = 0;
void diag(const IPMOut& o) {
  g_merit = o.merit;
  g_inband = o.inband;
  g_why = o.why;
  g_refs = o.refs;
  g_corrs = o.corrs;
}

template <int NB>
int cent_nb_(const double* prm, const double* st, const double* acc, const double* env_lhs, const double* env_rhs,
            int nenv, double* f_out, int* iters) {
  QPShared S;
  build_shared(S, prm, NB, st, acc, prm[DAT_P_KFC], prm[DAT_P_KMC], 2, false);
  QPLane<NB> P;
  double Rt[NB][9];
  lane_cent(P, prm, NB, st, Rt);
  double lhs[DAT_NENV][3], rhs[DAT_NENV];
  unsigned mask;
  env_slots(env_lhs, env_rhs, nenv, lhs, rhs, &mask);
  EnvRows E;
  set_env_rows(P, E, S, mask, lhs, rhs);
  double y[NB][3], w[6], best[best_size(NB)];
  IPMOut o = ipm_solve_rows<MODE_CENT, NB>(rows_needed(P.emask), PlainRef<QPShared>{&S}, EnvPlain{&E},
                                           RtPtr{&Rt[0][0]}, P, prm + DAT_P_FEQ(NB), y, w, best, 50, HS_TOL);
  diag(o);
  for (int k = 0; k < NB; ++k)
    for (int c = 0; c < 3; ++c) f_out[3 * k + c] = y[k][c];
  *iters = o.iters;
  return o.status;
}

}  // namespace

extern "C" {

// refinement passes run and corrections applied by the last solve
void hs_last_work(int* refs, int* corrs) {
  *refs = g_refs;
  *corrs = g_corrs;
}
void hs_last_diag(double* merit, int* inband, int* why) {
  *merit = g_merit;
  *inband = g_inband;
  *why = g_why;
}

int hs_qp_cadmm_ex(const double* prm, int n, const double* st, const double* acc, const double* env_lhs,
                   const double* env_rhs, int nenv, int i, const double* lam, const double* fbar, double rho,
                   int tuned, double* f_out, int* iters, int* inband);
// stiff exits of the fast solver since the last call (hs_qp_cadmm_ex: the redo count of IPM_FAST_REDO)
long long g_stiff_redo = 0;
long long hs_stiff_redos() { return g_stiff_redo; }
int g_last_stiff = 0;
// the last solve was redone robustly (IPM_FAST_REDO: its fast attempt was not clean)
int hs_last_stiff() { return g_last_stiff; }
int hs_qp_cadmm(const double* prm, int n, const double* st, const double* acc, const double* env_lhs,
                const double* env_rhs, int nenv, int i, const double* lam, const double* fbar, double rho,
                double* f_out, int* iters) {
  int ib = 0;
  return hs_qp_cadmm_ex(prm, n, st, acc, env_lhs, env_rhs, nenv, i, lam, fbar, rho, 0, f_out, iters, &ib);
}
// as hs_qp_cadmm with k_cadmm's IPM start policy flag (P.tuned) and the in-band exit flag out
int hs_qp_cadmm_ex(const double* prm, int n, const double* st, const double* acc, const double* env_lhs,
                   const double* env_rhs, int nenv, int i, const double* lam, const double* fbar, double rho,
                   int tuned, double* f_out, int* iters, int* inband) {
  if (nenv > DAT_NENV) return -1;
  double Rt_all[16 * 9];
  const double* Rl = st + DAT_S_RL(n);
  for (int j = 0; j < n; ++j) make_Rt(prm + DAT_P_RCOM(n) + 3 * j, Rl, Rt_all + 9 * j);
  QPShared S;
  build_shared(S, prm, n, st, acc, prm[DAT_P_KFD], prm[DAT_P_KMD], 3, true);
  QPLane<1> P;
  lane_cadmm_static(P, prm, i);
  double lhs[DAT_NENV][3], rhs[DAT_NENV];
  unsigned mask;
  env_slots(env_lhs, env_rhs, nenv, lhs, rhs, &mask);
  EnvRows E;
  set_env_rows(P, E, S, mask, lhs, rhs);
  lane_cadmm_dynamic(P, prm, n, i, Rt_all, lam, fbar, rho);
  P.tuned = tuned;
  // the GPU's C-ADMM agent QP (k_cadmm / k_cadmm_tail): rows certified infeasible are held; the fast solver,
  // redone robustly when not clean
  if (dvl_rows_infeasible(PlainRef<QPShared>{&S}, EnvPlain{&E}, P.emask)) P.infeasible = 1;
  double y[1][3], w[6], best[best_size(1)];
  IPMOut o = ipm_solve_rows<MODE_CADMM, 1, IPM_FAST_REDO>(rows_needed(P.emask), PlainRef<QPShared>{&S}, EnvPlain{&E},
                                                          RtPtr{Rt_all + 9 * i}, P, prm + DAT_P_FEQ(n) + 3 * i, y, w,
                                                          best, 50, HS_TOL);
  if (o.stiff) ++g_stiff_redo;
  g_last_stiff = o.stiff;
  *inband = o.inband ? 10 * o.why + 1 : 0;
  diag(o);
  for (int j = 0; j < n; ++j) {
    if (j == i) {
      for (int c = 0; c < 3; ++c) f_out[3 * j + c] = y[0][c];
    } else {
      cadmm_free_block(Rt_all + 9 * j, lam + 3 * j, fbar + 3 * j, o.pi, rho, f_out + 3 * j);
    }
  }
  *iters = o.iters;
  return o.status;
}

// as hs_qp_cadmm_ex with the tail kernel's agent QP: the certificate of infeasible rows, the warm-start record
// (wrec: WREC_SIZE doubles, in / out: the converged iterate is recorded) and, wson != 0, the warm first attempt
// (when wrec[0] = 1) and the stall exit
int hs_qp_cadmm_warm(const double* prm, int n, const double* st, const double* acc, const double* env_lhs,
                     const double* env_rhs, int nenv, int i, const double* lam, const double* fbar, double rho,
                     int tuned, double* wrec, int wson, double* f_out, int* iters, int* inband) {
  if (nenv > DAT_NENV) return -1;
  double Rt_all[16 * 9];
  const double* Rl = st + DAT_S_RL(n);
  for (int j = 0; j < n; ++j) make_Rt(prm + DAT_P_RCOM(n) + 3 * j, Rl, Rt_all + 9 * j);
  QPShared S;
  build_shared(S, prm, n, st, acc, prm[DAT_P_KFD], prm[DAT_P_KMD], 3, true);
  QPLane<1> P;
  lane_cadmm_static(P, prm, i);
  double lhs[DAT_NENV][3], rhs[DAT_NENV];
  unsigned mask;
  env_slots(env_lhs, env_rhs, nenv, lhs, rhs, &mask);
  EnvRows E;
  set_env_rows(P, E, S, mask, lhs, rhs);
  lane_cadmm_dynamic(P, prm, n, i, Rt_all, lam, fbar, rho);
  P.tuned = tuned;
  // the tail kernel's certificate of infeasible rows (k_cadmm_tail, at the scenario's hand-over)
  if (dvl_rows_infeasible(PlainRef<QPShared>{&S}, EnvPlain{&E}, P.emask)) P.infeasible = 1;
  double y[1][3], w[6], best[best_size(1)];
  IPMOut o = ipm_solve_rows<MODE_CADMM, 1, IPM_FAST_REDO, true>(rows_needed(P.emask), PlainRef<QPShared>{&S},
                                                                EnvPlain{&E}, RtPtr{Rt_all + 9 * i}, P,
                                                                prm + DAT_P_FEQ(n) + 3 * i, y, w, best, 50, HS_TOL, wrec,
                                                                wson != 0);
  if (o.stiff) ++g_stiff_redo;
  g_last_stiff = o.stiff;
  *inband = o.inband ? 10 * o.why + 1 : 0;
  diag(o);
  for (int j = 0; j < n; ++j) {
    if (j == i) {
      for (int c = 0; c < 3; ++c) f_out[3 * j + c] = y[0][c];
    } else {
      cadmm_free_block(Rt_all + 9 * j, lam + 3 * j, fbar + 3 * j, o.pi, rho, f_out + 3 * j);
    }
  }
  *iters = o.iters;
  return o.status;
}

// one ipm_attempt of the C-ADMM agent QP (development: tools/loose_probe.py): rob selects the robust
// instantiation, start the initial point (0 conservative, 1 tuned, 2 conservative x 10)
int hs_qp_cadmm_attempt(const double* prm, int n, const double* st, const double* acc, const double* env_lhs,
                        const double* env_rhs, int nenv, int i, const double* lam, const double* fbar, double rho,
                        int rob, int start, double* f_out, int* iters) {
  if (nenv > DAT_NENV) return -1;
  double Rt_all[16 * 9];
  const double* Rl = st + DAT_S_RL(n);
  for (int j = 0; j < n; ++j) make_Rt(prm + DAT_P_RCOM(n) + 3 * j, Rl, Rt_all + 9 * j);
  QPShared S;
  build_shared(S, prm, n, st, acc, prm[DAT_P_KFD], prm[DAT_P_KMD], 3, true);
  QPLane<1> P;
  lane_cadmm_static(P, prm, i);
  double lhs[DAT_NENV][3], rhs[DAT_NENV];
  unsigned mask;
  env_slots(env_lhs, env_rhs, nenv, lhs, rhs, &mask);
  EnvRows E;
  set_env_rows(P, E, S, mask, lhs, rhs);
  lane_cadmm_dynamic(P, prm, n, i, Rt_all, lam, fbar, rho);
  double y[1][3], w[6], best[best_size(1)];
  const PlainRef<QPShared> sh{&S};
  const EnvPlain er{&E};
  const RtPtr rt{Rt_all + 9 * i};
  IPMOut o = rob ? ipm_attempt<MODE_CADMM, 1, DAT_MAXROW, PlainRef<QPShared>, EnvPlain, RtPtr, RowRegs, 0, NoGrp, true>(
                       sh, er, rt, P, prm + DAT_P_FEQ(n) + 3 * i, y, w, best, 50, HS_TOL, RowRegs{}, NoGrp{}, start)
                 : ipm_attempt<MODE_CADMM, 1, DAT_MAXROW, PlainRef<QPShared>, EnvPlain, RtPtr, RowRegs, 0, NoGrp, false>(
                       sh, er, rt, P, prm + DAT_P_FEQ(n) + 3 * i, y, w, best, 50, HS_TOL, RowRegs{}, NoGrp{}, start);
  diag(o);
  for (int j = 0; j < n; ++j) {
    if (j == i) {
      for (int c = 0; c < 3; ++c) f_out[3 * j + c] = y[0][c];
    } else {
      cadmm_free_block(Rt_all + 9 * j, lam + 3 * j, fbar + 3 * j, o.pi, rho, f_out + 3 * j);
    }
  }
  *iters = o.iters;
  return o.status;
}

int hs_qp_dd(const double* prm, int n, const double* st, const double* acc, const double* env_lhs,
             const double* env_rhs, int nenv, int i, const double* c9, double* x_out, int* iters) {
  if (nenv > DAT_NENV) return -1;
  double Rt[9];
  make_Rt(prm + DAT_P_RCOM(n) + 3 * i, st + DAT_S_RL(n), Rt);
  QPShared S;
  build_shared(S, prm, n, st, acc, prm[DAT_P_KFD], prm[DAT_P_KMD], 3, false);
  QPLane<1> P;
  lane_dd_static(P, prm, i);
  set_dd_price(P, prm, n, i, c9);
  double lhs[DAT_NENV][3], rhs[DAT_NENV];
  unsigned mask;
  env_slots(env_lhs, env_rhs, nenv, lhs, rhs, &mask);
  EnvRows E;
  set_env_rows(P, E, S, mask, lhs, rhs);
  double y[1][3], w[6], best[best_size(1)];
  IPMOut o = ipm_solve_rows<MODE_DD, 1>(rows_needed(P.emask), PlainRef<QPShared>{&S}, EnvPlain{&E},
                                        RtPtr{Rt}, P, prm + DAT_P_FEQ(n) + 3 * i, y, w, best, 50, HS_TOL);
  diag(o);
  for (int c = 0; c < 3; ++c) x_out[c] = y[0][c];
  for (int c = 0; c < 6; ++c) x_out[3 + c] = w[c];
  *iters = o.iters;
  return o.status;
}

int hs_qp_cent(const double* prm, int n, const double* st, const double* acc, const double* env_lhs,
               const double* env_rhs, int nenv, double* f_out, int* iters) {
  if (nenv > DAT_NENV) return -1;
  if (n == 3) return cent_nb_<3>(prm, st, acc, env_lhs, env_rhs, nenv, f_out, iters);
  if (n == 6) return cent_nb_<6>(prm, st, acc, env_lhs, env_rhs, nenv, f_out, iters);
  return -1;
}

int hs_env_rows(const double* prm, int n, const double* st, const double* trees, int ntree, int agent,
                double alpha, double* lhs, double* rhs, int* collision, double* min_dist) {
  double L[DAT_NENV][3], R[DAT_NENV];
  unsigned mask;
  EnvOut e = env_rows(prm, n, st, trees, ntree, agent, alpha, &mask, L, R);
  *collision = e.collision;
  *min_dist = e.min_env_dist;
  int k = 0;
  for (int j = 0; j < DAT_NENV; ++j) {
    if (!((mask >> j) & 1u)) continue;
    for (int c = 0; c < 3; ++c) lhs[3 * k + c] = L[j][c];
    rhs[k] = R[j];
    ++k;
  }
  return k;
}

void hs_sim_step(const double* prm, int n, double* st, int* counter, const double* fdes, double dt) {
  sim_step<16>(prm, n, st, counter, fdes, dt);
}

void hs_sim_step_ll(const double* prm, int n, double* st, int* counter, const double* fdes, double dt, int kind) {
  sim_step<16>(prm, n, st, counter, fdes, dt, kind);
}

void hs_rp_step(const double* prm, int n, double* st, int* counter, const double* f, double dt) {
  rp_step(prm, n, st, counter, f, dt);
}

void hs_ll_control(const double* R, const double* w, const double* J, const double* fdes, double* f, double* M) {
  ll_control_agent(R, w, J, fdes, f, M);
}

void hs_ll_control_kind(const double* R, const double* w, const double* J, const double* fdes, double* f, double* M,
                        int kind) {
  ll_control_agent(R, w, J, fdes, f, M, kind);
}

void hs_desired_accel(const double* st, int n, const double* mountain, double x_offset, double* acc) {
  desired_accel_forest(st, n, mountain, x_offset, acc);
}
}
