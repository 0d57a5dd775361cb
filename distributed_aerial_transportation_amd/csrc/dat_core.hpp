// dat_core.hpp -- fp64 per-lane math of the agent-QP hot path (gfx950 device code).
//
// Everything here is __host__ __device__ so the unit tests can also drive single lanes on the CPU
// (tests/hostsim); the product path runs it only inside the HIP kernels of dat_kernels.hip.
//
// Contents
//   * small fixed-size linear algebra (3x3, 6x6, Cholesky, partial-pivot LU)
//   * Lie helpers: skew products, exp3 (Rodrigues + small-angle series), polar projection
//   * build_*: the per-step QP data of one agent (reference _update_cvx_parameters
//     control/rqp_cadmm.py:268-305 and the constraint/cost builders :376-471; DD
//     control/rqp_dd.py:275-460; centralized control/rqp_centralized.py:253-425) in the
//     *reduced* form used by the solver (see DESIGN.md "Reduced agent QP")
//   * env_rows: analytic capsule/tree distance + CBF linearisation (replaces the hppfcl loop,
//     example/env_forest.py:139-212 and control/rqp_cadmm.py:307-373)
//   * ipm_solve: structure-exploiting primal-dual interior-point method (NT scaling,
//     Mehrotra predictor-corrector, iterative refinement) -- the replacement for Clarabel
//   * rollout: SO(3) PD low-level control + forward dynamics + Lie midpoint integration
//     (control/rqp_centralized.py:503-535, system/rigid_quadrotor_payload.py:129-222)
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

#include "dat_layout.h"

#define DAT_HD __host__ __device__ inline

namespace dat {

enum Status { ST_OPTIMAL = 0, ST_INACCURATE = 1, ST_INFEASIBLE = 2, ST_FAILED = 3 };
enum Mode { MODE_CENT = 0, MODE_CADMM = 1, MODE_DD = 2 };

// =====================================================================================
// small linear algebra (row-major)
// =====================================================================================
DAT_HD double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
DAT_HD void cross3(const double* a, const double* b, double* o) {
  double x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}
DAT_HD void mv3(const double* M, const double* v, double* o) {
  double x = M[0] * v[0] + M[1] * v[1] + M[2] * v[2];
  double y = M[3] * v[0] + M[4] * v[1] + M[5] * v[2];
  double z = M[6] * v[0] + M[7] * v[1] + M[8] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}
DAT_HD void mtv3(const double* M, const double* v, double* o) {
  double x = M[0] * v[0] + M[3] * v[1] + M[6] * v[2];
  double y = M[1] * v[0] + M[4] * v[1] + M[7] * v[2];
  double z = M[2] * v[0] + M[5] * v[1] + M[8] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}
DAT_HD void mm3(const double* A, const double* B, double* O) {  // O = A B (O may not alias)
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) O[3 * r + c] = A[3 * r] * B[c] + A[3 * r + 1] * B[3 + c] + A[3 * r + 2] * B[6 + c];
}
DAT_HD void mmt3(const double* A, const double* B, double* O) {  // O = A B'
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) O[3 * r + c] = A[3 * r] * B[3 * c] + A[3 * r + 1] * B[3 * c + 1] + A[3 * r + 2] * B[3 * c + 2];
}
DAT_HD void skew3(const double* v, double* S) {
  S[0] = 0; S[1] = -v[2]; S[2] = v[1];
  S[3] = v[2]; S[4] = 0; S[5] = -v[0];
  S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}

// exp3: Rodrigues with the small-angle series (pinocchio::exp3 semantics).
DAT_HD void exp3(const double* v, double* R) {
  double t2 = dot3(v, v), a, b;
  if (t2 < 1e-8) {
    a = 1.0 - t2 / 6.0 + t2 * t2 / 120.0;
    b = 0.5 - t2 / 24.0 + t2 * t2 / 720.0;
  } else {
    double t = sqrt(t2);
    a = sin(t) / t;
    b = (1.0 - cos(t)) / t2;
  }
  double K[9], K2[9];
  skew3(v, K);
  mm3(K, K, K2);
  for (int i = 0; i < 9; ++i) R[i] = a * K[i] + b * K2[i];
  R[0] += 1.0; R[4] += 1.0; R[8] += 1.0;
}

DAT_HD double det3(const double* M) {
  return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}
// inverse transpose: (M^-1)^T = cofactor(M) / det
DAT_HD void invT3(const double* M, double* O) {
  double id = 1.0 / det3(M);
  O[0] = (M[4] * M[8] - M[5] * M[7]) * id; O[1] = -(M[3] * M[8] - M[5] * M[6]) * id; O[2] = (M[3] * M[7] - M[4] * M[6]) * id;
  O[3] = -(M[1] * M[8] - M[2] * M[7]) * id; O[4] = (M[0] * M[8] - M[2] * M[6]) * id; O[5] = -(M[0] * M[7] - M[1] * M[6]) * id;
  O[6] = (M[1] * M[5] - M[2] * M[4]) * id; O[7] = -(M[0] * M[5] - M[2] * M[3]) * id; O[8] = (M[0] * M[4] - M[1] * M[3]) * id;
}
// Orthogonal polar factor (replaces scipy.linalg.polar, system/rigid_quadrotor_payload.py:121-127):
// Newton iteration X <- (X + X^-T)/2, quadratically convergent for nonsingular X.
DAT_HD void polar3(double* X) {
  for (int it = 0; it < 20; ++it) {
    double Y[9];
    invT3(X, Y);
    double d = 0.0;
    for (int i = 0; i < 9; ++i) {
      double nx = 0.5 * (X[i] + Y[i]);
      d = fmax(d, fabs(nx - X[i]));
      X[i] = nx;
    }
    if (d < 1e-16) break;
  }
}

// symmetric 3x3 inverse of an SPD matrix (full storage)
DAT_HD void inv3sym(const double* D, double* O) {
  double c00 = D[4] * D[8] - D[5] * D[7], c01 = D[5] * D[6] - D[3] * D[8], c02 = D[3] * D[7] - D[4] * D[6];
  double det = D[0] * c00 + D[1] * c01 + D[2] * c02;
  double id = 1.0 / det;
  O[0] = c00 * id; O[1] = c01 * id; O[2] = c02 * id;
  O[4] = (D[0] * D[8] - D[2] * D[6]) * id;
  O[5] = (D[2] * D[3] - D[0] * D[5]) * id;
  O[8] = (D[0] * D[4] - D[1] * D[3]) * id;
  O[3] = O[1]; O[6] = O[2]; O[7] = O[5];
}

// Cholesky-based SPD 3x3 solve (more accurate than the cofactor inverse for graded matrices).
struct Chol3 {
  double l00, l10, l11, l20, l21, l22;
};
DAT_HD bool chol3(const double* D, Chol3& L) {
  if (!(D[0] > 0)) return false;
  L.l00 = sqrt(D[0]);
  L.l10 = D[3] / L.l00;
  L.l20 = D[6] / L.l00;
  double t = D[4] - L.l10 * L.l10;
  if (!(t > 0)) return false;
  L.l11 = sqrt(t);
  L.l21 = (D[7] - L.l20 * L.l10) / L.l11;
  t = D[8] - L.l20 * L.l20 - L.l21 * L.l21;
  if (!(t > 0)) return false;
  L.l22 = sqrt(t);
  return true;
}
DAT_HD void chol3_solve(const Chol3& L, const double* b, double* x) {
  double y0 = b[0] / L.l00;
  double y1 = (b[1] - L.l10 * y0) / L.l11;
  double y2 = (b[2] - L.l20 * y0 - L.l21 * y1) / L.l22;
  x[2] = y2 / L.l22;
  x[1] = (y1 - L.l21 * x[2]) / L.l11;
  x[0] = (y0 - L.l10 * x[1] - L.l20 * x[2]) / L.l00;
}

// 6x6 LU with partial pivoting (in place); returns false when singular.
DAT_HD bool lu6(double A[6][6], int piv[6]) {
  for (int k = 0; k < 6; ++k) {
    int p = k;
    double mx = fabs(A[k][k]);
    for (int r = k + 1; r < 6; ++r)
      if (fabs(A[r][k]) > mx) { mx = fabs(A[r][k]); p = r; }
    piv[k] = p;
    if (!(mx > 0)) return false;
    if (p != k)
      for (int c = 0; c < 6; ++c) { double t = A[k][c]; A[k][c] = A[p][c]; A[p][c] = t; }
    double inv = 1.0 / A[k][k];
    for (int r = k + 1; r < 6; ++r) {
      double f = A[r][k] * inv;
      A[r][k] = f;
      for (int c = k + 1; c < 6; ++c) A[r][c] -= f * A[k][c];
    }
  }
  return true;
}
DAT_HD void lu6_solve(const double A[6][6], const int piv[6], double* b) {
  // PA = LU with the multipliers swapped along with their rows: permute b fully, then solve.
  for (int k = 0; k < 6; ++k) {
    int p = piv[k];
    if (p != k) { double t = b[k]; b[k] = b[p]; b[p] = t; }
  }
  for (int k = 0; k < 6; ++k)
    for (int r = k + 1; r < 6; ++r) b[r] -= A[r][k] * b[k];
  for (int k = 5; k >= 0; --k) {
    double s = b[k];
    for (int c = k + 1; c < 6; ++c) s -= A[k][c] * b[c];
    b[k] = s / A[k][k];
  }
}
// 6x6 Cholesky (lower, in place); returns false if not SPD.
DAT_HD bool chol6(double A[6][6]) {
  for (int j = 0; j < 6; ++j) {
    double s = A[j][j];
    for (int k = 0; k < j; ++k) s -= A[j][k] * A[j][k];
    if (!(s > 0)) return false;
    double d = sqrt(s);
    A[j][j] = d;
    for (int i = j + 1; i < 6; ++i) {
      double t = A[i][j];
      for (int k = 0; k < j; ++k) t -= A[i][k] * A[j][k];
      A[i][j] = t / d;
    }
  }
  return true;
}
DAT_HD void chol6_solve(const double L[6][6], double* b) {
  for (int i = 0; i < 6; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= L[i][k] * b[k];
    b[i] = s / L[i][i];
  }
  for (int i = 5; i >= 0; --i) {
    double s = b[i];
    for (int k = i + 1; k < 6; ++k) s -= L[k][i] * b[k];
    b[i] = s / L[i][i];
  }
}

// =====================================================================================
// the reduced agent QP
// =====================================================================================
// u = (S, Mo) in R^6: aggregate force and moment about the CoM in payload axes,
//   S = sum_j f_j,  Mo = sum_j hat(r_com_j) Rl' f_j      (control/rqp_cadmm.py:376-392)
// Accelerations are affine in u:
//   dwl = JT^-1 Mo + bw,           bw = -JT^-1 (wl x JT wl)
//   dvl = S/mT + Bv Mo + bv,       Bv = Rl hat(x_com) JT^-1,
//                                  bv = -g e3 - Rl hat(wl)^2 x_com + Rl hat(x_com) bw
// Cone block k (an agent's own force f_k in R^3): f_kz >= min_fz, ||f_k|| <= sec f_kz,
// ||f_k|| <= max_f.  u-rows (tilt, |wl|, |vl|, env CBFs) are affine in (dvl, dwl).
struct UMap {
  double inv_mT, Bv[9], JTi[9], bv[3], bw[3];
};

struct Rows {
  int nw;                      // rows [0, nw) act on dwl, rows [nw, n) on dvl
  int n;
  int infeasible;              // an all-zero row with a negative constant
  double a[DAT_MAXROW][3];     // coefficients on dwl or dvl
  double b[DAT_MAXROW];        // constant: a'(acc) + b >= 0 with acc the *linear* part of dvl/dwl in u
};

DAT_HD void rows_add(Rows& R, const UMap& m, bool on_dwl, const double* al, double beta0) {
  if (al[0] == 0.0 && al[1] == 0.0 && al[2] == 0.0) {
    if (beta0 < 0.0) R.infeasible = 1;  // 0 >= -beta0 fails: the QP is infeasible
    return;                             // 0 >= 0 (or a slack constant row) carries no information
  }
  int k = R.n++;
  R.a[k][0] = al[0]; R.a[k][1] = al[1]; R.a[k][2] = al[2];
  R.b[k] = beta0 + (on_dwl ? dot3(al, m.bw) : dot3(al, m.bv));
}

// linear parts of (dvl, dwl) for a u-space vector
DAT_HD void umap_lin(const UMap& m, const double* u, double* dv, double* dw) {
  double t[3];
  mv3(m.Bv, u + 3, t);
  dv[0] = m.inv_mT * u[0] + t[0]; dv[1] = m.inv_mT * u[1] + t[1]; dv[2] = m.inv_mT * u[2] + t[2];
  mv3(m.JTi, u + 3, dw);
}
// u-space vector of A' z for dvl-coefficients gv and dwl-coefficients gw
DAT_HD void umap_adj(const UMap& m, const double* gv, const double* gw, double* o) {
  double t[3], s[3];
  mtv3(m.Bv, gv, t);
  mtv3(m.JTi, gw, s);
  o[0] = m.inv_mT * gv[0]; o[1] = m.inv_mT * gv[1]; o[2] = m.inv_mT * gv[2];
  o[3] = t[0] + s[0]; o[4] = t[1] + s[1]; o[5] = t[2] + s[2];
}

template <int NB>
struct QP {
  UMap m;
  Rows rows;
  double C[6][6], cu[6];     // 1/2 u'Cu + cu'u
  double kappa;              // per-block Hessian kappa I
  double q[NB][3];           // per-block linear term
  double Rt[NB][9];          // U_k = [I; Rt_k],  Rt_k = hat(r_com_k) Rl'
  double y0[NB][3];          // interior initial guess (f_eq)
  double min_fz, max_f, sec;
  double K[6][6], atil[6], rho;  // CADMM free aggregate: sum_{j != i} U_j U_j', sum_{j != i} U_j a_j
  double cw[6];                  // DD: linear cost on w = (F_i, M_i)
};

// ------------------------------------------------------------------ common QP data (u-maps, Phi, rows)
// params: per-scenario block (dat_layout.h); state: per-scenario block.
// k_f, k_m: total force / moment weights; kdv: leader weight for the desired-acceleration costs.
template <int NB>
DAT_HD void build_common(QP<NB>& P, const double* prm, int n, const double* st, const double* acc,
                         double k_f, double k_m, double kdv) {
  const double mT = prm[DAT_P_MT];
  const double* xc = prm + DAT_P_XCOM;
  const double* JT = prm + DAT_P_JT;
  const double* JTi = prm + DAT_P_JTI;
  const double* Rl = st + DAT_S_RL(n);
  const double* wl = st + DAT_S_WL(n);
  const double* vl = st + DAT_S_VL(n);
  UMap& m = P.m;
  m.inv_mT = 1.0 / mT;
  for (int i = 0; i < 9; ++i) m.JTi[i] = JTi[i];
  double Xh[9], RX[9];
  skew3(xc, Xh);
  mm3(Rl, Xh, RX);              // Rl hat(x_com)
  mm3(RX, JTi, m.Bv);           // Rl hat(x_com) JT^-1
  double Jw[3], wJw[3];
  mv3(JT, wl, Jw);
  cross3(wl, Jw, wJw);
  mv3(JTi, wJw, m.bw);          // c_w = JT^-1 (wl x JT wl)
  m.bw[0] = -m.bw[0]; m.bw[1] = -m.bw[1]; m.bw[2] = -m.bw[2];
  // bv = -g e3 - Rl hat(wl)^2 x_com + Rl hat(x_com) bw
  double wx[3], wwx[3], t1[3], t2[3];
  cross3(wl, xc, wx);
  cross3(wl, wx, wwx);          // hat(wl)^2 x_com
  mv3(Rl, wwx, t1);
  mv3(RX, m.bw, t2);
  m.bv[0] = -t1[0] + t2[0];
  m.bv[1] = -t1[1] + t2[1];
  m.bv[2] = -DAT_GRAVITY - t1[2] + t2[2];

  // Phi(u) = k_f ||S - mT g e3||^2 + k_m ||Mo||^2 + kdv (||dvl||^2 - 2 dvl_des'dvl)
  //          + kdv (||dwl||^2 - 2 dwl_des'dwl)          (control/rqp_cadmm.py:436-458)
  for (int r = 0; r < 6; ++r)
    for (int c = 0; c < 6; ++c) P.C[r][c] = 0.0;
  for (int r = 0; r < 3; ++r) { P.C[r][r] = 2.0 * k_f; P.C[3 + r][3 + r] = 2.0 * k_m; }
  for (int r = 0; r < 6; ++r) P.cu[r] = 0.0;
  P.cu[2] = -2.0 * k_f * mT * DAT_GRAVITY;
  if (kdv != 0.0) {
    // Av = [I/mT, Bv], Aw = [0, JTi]: C += 2 kdv (Av'Av + Aw'Aw)
    double im = m.inv_mT;
    for (int r = 0; r < 3; ++r) {
      P.C[r][r] += 2.0 * kdv * im * im;
      for (int c = 0; c < 3; ++c) {
        double v = 2.0 * kdv * im * m.Bv[3 * r + c];  // (I/mT)' Bv
        P.C[r][3 + c] += v;
        P.C[3 + c][r] += v;
      }
    }
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double s = 0.0;
        for (int k = 0; k < 3; ++k) s += m.Bv[3 * k + r] * m.Bv[3 * k + c] + m.JTi[3 * k + r] * m.JTi[3 * k + c];
        P.C[3 + r][3 + c] += 2.0 * kdv * s;
      }
    double ev[3] = {m.bv[0] - acc[0], m.bv[1] - acc[1], m.bv[2] - acc[2]};
    double ew[3] = {m.bw[0] - acc[3], m.bw[1] - acc[4], m.bw[2] - acc[5]};
    double g[6];
    umap_adj(m, ev, ew, g);
    for (int r = 0; r < 6; ++r) P.cu[r] += 2.0 * kdv * g[r];
  }

  // rows (control/rqp_cadmm.py:406-430): dwl rows first
  Rows& R = P.rows;
  R.n = 0;
  R.infeasible = 0;
  double Rw[3], Rww[3];  // third rows of Rl hat(wl) and Rl hat(wl)^2 evaluated at e3
  {
    // (Rl hat(wl))[2,2] = Rl[2,:] . (wl x e3);  (Rl hat(wl)^2)[2,2] = Rl[2,:] . (wl x (wl x e3))
    double e3[3] = {0, 0, 1}, a[3], b[3];
    cross3(wl, e3, a);
    cross3(wl, a, b);
    Rw[0] = dot3(Rl + 6, a);
    Rww[0] = dot3(Rl + 6, b);
    (void)Rw; (void)Rww;
  }
  double tilt_beta = Rww[0] + 2.0 * Rw[0] + (Rl[8] - prm[DAT_P_COSP]);
  double al_t[3] = {-Rl[7], Rl[6], 0.0};  // -(e3' Rl hat(e3)) = -[Rl21, -Rl20, 0]
  rows_add(R, m, true, al_t, tilt_beta);
  double al_w[3] = {-2.0 * wl[0], -2.0 * wl[1], -2.0 * wl[2]};
  rows_add(R, m, true, al_w, prm[DAT_P_MAXWL2] - dot3(wl, wl));
  R.nw = R.n;
  double al_v[3] = {-2.0 * vl[0], -2.0 * vl[1], -2.0 * vl[2]};
  rows_add(R, m, false, al_v, prm[DAT_P_MAXVL2] - dot3(vl, vl));
  P.min_fz = prm[DAT_P_MINFZ];
  P.max_f = prm[DAT_P_MAXF];
  P.sec = prm[DAT_P_SEC];
}

// Rt_j = hat(r_com_j) Rl'
DAT_HD void make_Rt(const double* rcom, const double* Rl, double* Rt) {
  double H[9];
  skew3(rcom, H);
  mmt3(H, Rl, Rt);
}
// U_j x = (x, Rt x)
DAT_HD void U_apply(const double* Rt, const double* x, double* o) {
  o[0] = x[0]; o[1] = x[1]; o[2] = x[2];
  mv3(Rt, x, o + 3);
}
// U_j' v = v[0:3] + Rt' v[3:6]
DAT_HD void Ut_apply(const double* Rt, const double* v, double* o) {
  mtv3(Rt, v + 3, o);
  o[0] += v[0]; o[1] += v[1]; o[2] += v[2];
}
// M += U D U' for U = [I; Rt] and symmetric 3x3 D
DAT_HD void add_UDUt(double M[6][6], const double* Rt, const double* D, double scale) {
  double RD[9], RDR[9];
  mm3(Rt, D, RD);
  mmt3(RD, Rt, RDR);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      M[r][c] += scale * D[3 * r + c];
      M[3 + r][c] += scale * RD[3 * r + c];
      M[r][3 + c] += scale * RD[3 * c + r];
      M[3 + r][3 + c] += scale * RDR[3 * r + c];
    }
}

// =====================================================================================
// environment: capsule vs tree distance and CBF rows (K5)
// =====================================================================================
struct EnvOut {
  int collision;
  double min_env_dist;
};

// Point-to-solid-cylinder (axis z, radius DAT_BARK_RADIUS, half height DAT_BARK_HALF_HEIGHT).
DAT_HD double point_cyl(const double* p, const double* c, double* qn) {
  double dx = p[0] - c[0], dy = p[1] - c[1];
  double rho = sqrt(dx * dx + dy * dy);
  double hz = p[2] - c[2];
  if (rho > DAT_BARK_RADIUS) {
    qn[0] = c[0] + dx / rho * DAT_BARK_RADIUS;
    qn[1] = c[1] + dy / rho * DAT_BARK_RADIUS;
  } else {
    qn[0] = p[0];
    qn[1] = p[1];
  }
  qn[2] = c[2] + fmin(fmax(hz, -DAT_BARK_HALF_HEIGHT), DAT_BARK_HALF_HEIGHT);
  double ex = p[0] - qn[0], ey = p[1] - qn[1], ez = p[2] - qn[2];
  return sqrt(ex * ex + ey * ey + ez * ez);
}

// d/dt of the squared point-cylinder distance along p(t) = x0 + t d (convex in t).
DAT_HD double dist2_slope(const double* x0, const double* d, const double* c, double t) {
  double px = x0[0] + t * d[0] - c[0], py = x0[1] + t * d[1] - c[1], pz = x0[2] + t * d[2] - c[2];
  double rho = sqrt(px * px + py * py);
  double g = 0.0;
  if (rho > DAT_BARK_RADIUS) g += 2.0 * (rho - DAT_BARK_RADIUS) * (px * d[0] + py * d[1]) / rho;
  double az = fabs(pz) - DAT_BARK_HALF_HEIGHT;
  if (az > 0.0) g += 2.0 * az * (pz > 0 ? d[2] : -d[2]);
  return g;
}

// Capsule (segment x0 -> x0 + d, radius rc) vs tree at c: signed distance (hppfcl semantics for
// the separated case) and nearest points p1 (capsule surface) / p2 (tree surface), world frame.
DAT_HD double capsule_tree(const double* x0, const double* d, double rc, const double* c, double* p1, double* p2) {
  double t;
  if (dist2_slope(x0, d, c, 0.0) >= 0.0) {
    t = 0.0;
  } else if (dist2_slope(x0, d, c, 1.0) <= 0.0) {
    t = 1.0;
  } else {
    double lo = 0.0, hi = 1.0;
    for (int it = 0; it < 64; ++it) {  // bisection on the monotone slope: t to machine precision
      double mid = 0.5 * (lo + hi);
      if (mid <= lo || mid >= hi) break;
      if (dist2_slope(x0, d, c, mid) < 0.0) lo = mid; else hi = mid;
    }
    t = 0.5 * (lo + hi);
  }
  double p[3] = {x0[0] + t * d[0], x0[1] + t * d[1], x0[2] + t * d[2]};
  double ds = point_cyl(p, c, p2);
  if (ds > 0.0) {
    double k = rc / ds;
    p1[0] = p[0] + (p2[0] - p[0]) * k;
    p1[1] = p[1] + (p2[1] - p[1]) * k;
    p1[2] = p[2] + (p2[2] - p[2]) * k;
  } else {
    p1[0] = p[0]; p1[1] = p[1]; p1[2] = p[2];
  }
  return ds - rc;
}

// Env CBF rows of one solve: fills lhs (nrow x 3) / rhs (the reference's env_cbf_lhs/rhs, rows with
// zero lhs omitted) and returns collision / min_env_dist (control/rqp_cadmm.py:307-373;
// camera == nullptr selects the centralized query without vision cone, rqp_centralized.py:280-337).
// Tree selection: distance of the capsule centre to tree_pos <= vision_r + bark radius, plus the
// 2-D cone test for distributed agents; the DAT_NENV nearest of the selected trees become rows.
DAT_HD EnvOut env_rows(const double* prm, int n, const double* st, const double* trees, int ntree,
                       int agent /* -1: centralized */, double alpha_env, int* nrow, double lhs[DAT_NENV][3],
                       double rhs[DAT_NENV]) {
  EnvOut out;
  out.collision = 0;
  out.min_env_dist = prm[DAT_P_VISR];
  *nrow = 0;
  if (trees == nullptr || ntree <= 0) return out;
  const double* xl = st + DAT_S_XL(n);
  const double* vl = st + DAT_S_VL(n);
  const double* Rl = st + DAT_S_RL(n);
  const double maxdec = prm[DAT_P_MAXDEC], visr = prm[DAT_P_VISR], rc = prm[DAT_P_COLR];
  double v2 = dot3(vl, vl);
  double h = 0.5 * v2 / maxdec;
  double speed = sqrt(v2);
  double vdir[3] = {0, 0, 0}, seg[3] = {0, 0, 0}, ctr[3] = {xl[0], xl[1], xl[2]};
  if (speed != 0.0) {
    vdir[0] = vl[0] / speed; vdir[1] = vl[1] / speed; vdir[2] = vl[2] / speed;
    seg[0] = h * vdir[0]; seg[1] = h * vdir[1]; seg[2] = h * vdir[2];
    ctr[0] += 0.5 * seg[0]; ctr[1] += 0.5 * seg[1]; ctr[2] += 0.5 * seg[2];
  }
  double cam[2] = {0, 0}, dir[2] = {0, 0}, cosang = prm[DAT_P_COSCONE];
  if (agent >= 0) {
    const double* r = prm + DAT_P_R(n) + 3 * agent;
    double Rr[3];
    mv3(Rl, r, Rr);
    cam[0] = xl[0] + Rr[0];
    cam[1] = xl[1] + Rr[1];
    double dx = cam[0] - xl[0], dy = cam[1] - xl[1];
    double nn = sqrt(dx * dx + dy * dy);
    if (nn == 0.0) {
      out.collision = 1;
      return out;
    }
    dir[0] = dx / nn; dir[1] = dy / nn;
  }
  // keep the DAT_NENV smallest distances (sorted insertion)
  double bd[DAT_NENV], bp1[DAT_NENV][3], bp2[DAT_NENV][3];
  int cnt = 0, kept = 0;
  double dmin = 1e300;
  for (int t = 0; t < ntree; ++t) {
    const double* c = trees + 3 * t;
    double ex = ctr[0] - c[0], ey = ctr[1] - c[1], ez = ctr[2] - c[2];
    if (sqrt(ex * ex + ey * ey + ez * ez) > visr + DAT_BARK_RADIUS) continue;
    if (agent >= 0) {
      double tx = c[0] - cam[0], ty = c[1] - cam[1];
      double nn = sqrt(tx * tx + ty * ty);
      if (nn > 0.0 && (tx / nn * dir[0] + ty / nn * dir[1]) < cosang) continue;
    }
    double p1[3], p2[3];
    double dd = capsule_tree(xl, seg, rc, c, p1, p2);
    if (dd < 1e-4) out.collision = 1;
    dmin = fmin(dmin, dd);
    ++cnt;
    int pos = kept;
    while (pos > 0 && bd[pos - 1] > dd) --pos;
    if (pos < DAT_NENV) {
      int last = kept < DAT_NENV ? kept : DAT_NENV - 1;
      for (int j = last; j > pos; --j) {
        bd[j] = bd[j - 1];
        for (int q = 0; q < 3; ++q) { bp1[j][q] = bp1[j - 1][q]; bp2[j][q] = bp2[j - 1][q]; }
      }
      bd[pos] = dd;
      for (int q = 0; q < 3; ++q) { bp1[pos][q] = p1[q]; bp2[pos][q] = p2[q]; }
      if (kept < DAT_NENV) ++kept;
    }
  }
  if (cnt > 0 && speed > 0.0) {
    out.min_env_dist = dmin;
    for (int j = 0; j < kept; ++j) {
      double di = bd[j];
      if (di <= 1e-4) continue;
      double rel[3] = {bp1[j][0] - xl[0], bp1[j][1] - xl[1], bp1[j][2] - xl[2]};
      double proj = fmax(0.0, fmin(h, dot3(rel, vdir)));
      double mt = sqrt(2.0 * (h - proj) / maxdec);
      mt = fmax(0.0, speed / maxdec - mt);
      // proj = 0 makes the two terms equal in exact arithmetic (the reference gets an exact 0);
      // snap the rounding residue so such rows stay "0 >= rhs" like the reference's.
      if (mt < 1e-12 * speed / maxdec) mt = 0.0;
      double nr[3] = {bp1[j][0] - bp2[j][0], bp1[j][1] - bp2[j][1], bp1[j][2] - bp2[j][2]};
      double nn = sqrt(dot3(nr, nr));
      nr[0] /= nn; nr[1] /= nn; nr[2] /= nn;
      int k = (*nrow)++;
      lhs[k][0] = nr[0] * mt; lhs[k][1] = nr[1] * mt; lhs[k][2] = nr[2] * mt;
      rhs[k] = -alpha_env * (di - prm[DAT_P_DISTEPS]) - dot3(nr, vl);
    }
  }
  return out;
}

template <int NB>
DAT_HD void add_env_rows(QP<NB>& P, int nrow, const double lhs[DAT_NENV][3], const double rhs[DAT_NENV]) {
  for (int k = 0; k < nrow; ++k) rows_add(P.rows, P.m, false, lhs[k], -rhs[k]);
}

// =====================================================================================
// interior-point method on the reduced problem
// =====================================================================================
// Per cone block: slack/dual layout [fz | soc1 (4) | soc2 (4)] (9 entries),
//   s = h - G y,  G y = -(y2, sec y2, y0, y1, y2, 0, y0, y1, y2),  h = (-min_fz, 0,0,0,0, max_f, 0,0,0).
// u-rows: s_l = a_l'(lin(u)) + b_l >= 0.
struct SocScale {
  double w[4];
  double eta;
};

DAT_HD double soc_det(const double* v) {
  double n1 = sqrt(v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
  return (v[0] - n1) * (v[0] + n1);
}
DAT_HD bool soc_scaling(const double* s, const double* z, SocScale& S) {
  double ds = soc_det(s), dz = soc_det(z);
  if (!(ds > 0) || !(dz > 0)) return false;
  double sn = sqrt(ds), zn = sqrt(dz);
  double ss[4], zz[4];
  for (int i = 0; i < 4; ++i) { ss[i] = s[i] / sn; zz[i] = z[i] / zn; }
  double g = sqrt(0.5 * (1.0 + ss[0] * zz[0] + ss[1] * zz[1] + ss[2] * zz[2] + ss[3] * zz[3]));
  S.w[0] = (ss[0] + zz[0]) / (2.0 * g);
  for (int i = 1; i < 4; ++i) S.w[i] = (ss[i] - zz[i]) / (2.0 * g);
  S.eta = sqrt(sn / zn);
  return true;
}
// o = W v (inv = false) or W^-1 v (inv = true); W = eta H(w), W^-1 = H(Jw)/eta
DAT_HD void soc_apply(const SocScale& S, const double* v, double* o, bool inv) {
  double sg = inv ? -1.0 : 1.0;
  double w1 = sg * S.w[1], w2 = sg * S.w[2], w3 = sg * S.w[3];
  double wv = w1 * v[1] + w2 * v[2] + w3 * v[3];
  double k = (v[0] + wv / (1.0 + S.w[0]));
  double sc = inv ? 1.0 / S.eta : S.eta;
  double o0 = S.w[0] * v[0] + wv;
  o[1] = sc * (v[1] + k * w1);
  o[2] = sc * (v[2] + k * w2);
  o[3] = sc * (v[3] + k * w3);
  o[0] = sc * o0;
}
// x = lam \ y (inverse Jordan product) for a 4-dim SOC
DAT_HD void soc_jdiv(const double* l, const double* y, double* x) {
  double det = l[0] * l[0] - (l[1] * l[1] + l[2] * l[2] + l[3] * l[3]);
  double x0 = (l[0] * y[0] - (l[1] * y[1] + l[2] * y[2] + l[3] * y[3])) / det;
  x[0] = x0;
  for (int i = 1; i < 4; ++i) x[i] = (y[i] - x0 * l[i]) / l[0];
}
DAT_HD void soc_jprod(const double* a, const double* b, double* o) {
  double d = a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
  for (int i = 1; i < 4; ++i) o[i] = a[0] * b[i] + b[0] * a[i];
  o[0] = d;
}
DAT_HD double soc_step(const double* x, const double* d) {
  double a = d[0] * d[0] - (d[1] * d[1] + d[2] * d[2] + d[3] * d[3]);
  double b = x[0] * d[0] - (x[1] * d[1] + x[2] * d[2] + x[3] * d[3]);
  double n1 = sqrt(x[1] * x[1] + x[2] * x[2] + x[3] * x[3]);
  double c = (x[0] - n1) * (x[0] + n1);
  double disc = b * b - a * c;
  if (a < 0.0 || (b < 0.0 && disc >= 0.0)) {
    double den = -b + sqrt(fmax(disc, 0.0));
    return den > 0.0 ? c / den : 0.0;
  }
  return 1e300;
}

struct IPMOut {
  int status;
  int iters;
  double pi[6];   // u-space gradient C u + cu - A' z_rows at the solution
  double u[6];
};

// Solve the reduced QP. MODE_CADMM: NB = 1, implicit free blocks through (K, atil, rho);
// MODE_DD: NB = 1, w = (F_i, M_i) free with linear cost cw; MODE_CENT: NB = n, no w.
// y (NB x 3) and w (6) are outputs.
template <int MODE, int NB>
DAT_HD IPMOut ipm_solve(const QP<NB>& P, double y[NB][3], double w[6], int max_iter, double tol) {
  IPMOut out;
  out.status = ST_FAILED;
  out.iters = 0;
  const Rows& R = P.rows;
  const int ml = R.n, nw = R.nw;
  const double sec = P.sec, kap = P.kappa;
  if (R.infeasible) {
    out.status = ST_INFEASIBLE;
    return out;
  }
  double sk[NB][9], zk[NB][9], sl[DAT_MAXROW], zl[DAT_MAXROW];
  double u[6];

  auto Gy = [&](const double* yy, double* o) {
    o[0] = -yy[2]; o[1] = -sec * yy[2]; o[2] = -yy[0]; o[3] = -yy[1]; o[4] = -yy[2];
    o[5] = 0.0; o[6] = -yy[0]; o[7] = -yy[1]; o[8] = -yy[2];
  };
  auto GTz = [&](const double* z, double* o) {
    o[0] = -(z[2] + z[6]);
    o[1] = -(z[3] + z[7]);
    o[2] = -(z[0] + sec * z[1] + z[4] + z[8]);
  };
  const double hk[9] = {-P.min_fz, 0, 0, 0, 0, P.max_f, 0, 0, 0};
  auto compute_u = [&](double* uo) {
    for (int r = 0; r < 6; ++r) uo[r] = (MODE == MODE_CENT) ? 0.0 : w[r];
    for (int k = 0; k < NB; ++k) {
      double t[6];
      U_apply(P.Rt[k], y[k], t);
      for (int r = 0; r < 6; ++r) uo[r] += t[r];
    }
  };
  auto row_vals = [&](const double* uu, double* vals, bool with_const) {
    double dv[3], dw[3];
    umap_lin(P.m, uu, dv, dw);
    for (int l = 0; l < ml; ++l) vals[l] = dot3(R.a[l], l < nw ? dw : dv) + (with_const ? R.b[l] : 0.0);
  };
  auto rows_adj = [&](const double* zz, double* o) {  // o = A' zz (u-space)
    double gv[3] = {0, 0, 0}, gw[3] = {0, 0, 0};
    for (int l = 0; l < ml; ++l) {
      double* g = l < nw ? gw : gv;
      g[0] += zz[l] * R.a[l][0]; g[1] += zz[l] * R.a[l][1]; g[2] += zz[l] * R.a[l][2];
    }
    umap_adj(P.m, gv, gw, o);
  };
  auto Cmul = [&](const double* v, double* o) {
    for (int r = 0; r < 6; ++r) {
      double s = 0.0;
      for (int c = 0; c < 6; ++c) s += P.C[r][c] * v[c];
      o[r] = s;
    }
  };
  auto Kmul = [&](const double* v, double* o) {
    for (int r = 0; r < 6; ++r) {
      double s = 0.0;
      for (int c = 0; c < 6; ++c) s += P.K[r][c] * v[c];
      o[r] = s;
    }
  };

  // ---------------- initial point
  for (int k = 0; k < NB; ++k) {
    for (int c = 0; c < 3; ++c) y[k][c] = P.y0[k][c];
    double g[9];
    Gy(y[k], g);
    for (int j = 0; j < 9; ++j) sk[k][j] = hk[j] - g[j];
    // shift into the interior if the guess is not strictly feasible
    double m1 = sk[k][0], m2 = sk[k][1] - sqrt(sk[k][2] * sk[k][2] + sk[k][3] * sk[k][3] + sk[k][4] * sk[k][4]);
    double m3 = sk[k][5] - sqrt(sk[k][6] * sk[k][6] + sk[k][7] * sk[k][7] + sk[k][8] * sk[k][8]);
    double mn = fmin(m1, fmin(m2, m3));
    if (mn < 1e-3) { sk[k][0] += 1.0 - mn; sk[k][1] += 1.0 - mn; sk[k][5] += 1.0 - mn; }
    for (int j = 0; j < 9; ++j) zk[k][j] = 0.0;
    zk[k][0] = 1.0; zk[k][1] = 1.0; zk[k][5] = 1.0;
  }
  for (int l = 0; l < ml; ++l) zl[l] = 1.0;
  for (int r = 0; r < 6; ++r) w[r] = 0.0;
  if (MODE == MODE_CADMM) {
    // consistent free aggregate: (rho I + K C) w = rho atil - K (C U y + cu - A' zl)
    double uy[6], cuy[6], az[6], rhs[6], Kt[6];
    compute_u(uy);  // w = 0 here
    Cmul(uy, cuy);
    rows_adj(zl, az);
    for (int r = 0; r < 6; ++r) cuy[r] += P.cu[r] - az[r];
    Kmul(cuy, Kt);
    double A[6][6];
    for (int r = 0; r < 6; ++r) {
      rhs[r] = P.rho * P.atil[r] - Kt[r];
      for (int c = 0; c < 6; ++c) {
        double s = 0.0;
        for (int k = 0; k < 6; ++k) s += P.K[r][k] * P.C[k][c];
        A[r][c] = s + (r == c ? P.rho : 0.0);
      }
    }
    int piv[6];
    if (!lu6(A, piv)) return out;
    lu6_solve(A, piv, rhs);
    for (int r = 0; r < 6; ++r) w[r] = rhs[r];
  }
  compute_u(u);
  {
    double rv[DAT_MAXROW];
    row_vals(u, rv, true);
    for (int l = 0; l < ml; ++l) sl[l] = fmax(rv[l], 1.0);
  }

  // scales for the relative stopping rule
  double nh = 1.0 + fmax(P.min_fz, P.max_f), nq = 1.0;
  for (int l = 0; l < ml; ++l) nh = fmax(nh, 1.0 + fabs(R.b[l]));
  for (int k = 0; k < NB; ++k)
    for (int c = 0; c < 3; ++c) nq = fmax(nq, 1.0 + fabs(P.q[k][c]));
  for (int r = 0; r < 6; ++r) nq = fmax(nq, 1.0 + fabs(P.cu[r]));

  double best_merit = 1e300, best_y[NB][3], best_w[6], best_pi[6], best_u[6];
  const int deg = 3 * NB + ml;

  for (int it = 0;; ++it) {
    // ------------- residuals
    compute_u(u);
    double pi[6], az[6];
    Cmul(u, pi);
    rows_adj(zl, az);
    for (int r = 0; r < 6; ++r) pi[r] += P.cu[r] - az[r];
    double rk[NB][3], Rf[6];
    double dres = 0.0, pres = 0.0, gap = 0.0;
    for (int k = 0; k < NB; ++k) {
      double ut[3], gz[3];
      Ut_apply(P.Rt[k], pi, ut);
      GTz(zk[k], gz);
      for (int c = 0; c < 3; ++c) {
        rk[k][c] = kap * y[k][c] + P.q[k][c] + ut[c] + gz[c];
        dres = fmax(dres, fabs(rk[k][c]));
      }
    }
    if (MODE == MODE_CADMM) {
      double kp[6];
      Kmul(pi, kp);
      for (int r = 0; r < 6; ++r) Rf[r] = P.rho * (w[r] - P.atil[r]) + kp[r];
    } else if (MODE == MODE_DD) {
      for (int r = 0; r < 6; ++r) Rf[r] = pi[r] + P.cw[r];
    } else {
      for (int r = 0; r < 6; ++r) Rf[r] = 0.0;
    }
    for (int r = 0; r < 6; ++r) dres = fmax(dres, fabs(Rf[r]));
    double rzk[NB][9], rzl[DAT_MAXROW];
    for (int k = 0; k < NB; ++k) {
      double g[9];
      Gy(y[k], g);
      for (int j = 0; j < 9; ++j) {
        rzk[k][j] = g[j] + sk[k][j] - hk[j];
        pres = fmax(pres, fabs(rzk[k][j]));
        gap += sk[k][j] * zk[k][j];
      }
    }
    {
      double rv[DAT_MAXROW];
      row_vals(u, rv, true);
      for (int l = 0; l < ml; ++l) {
        rzl[l] = -rv[l] + sl[l];
        pres = fmax(pres, fabs(rzl[l]));
        gap += sl[l] * zl[l];
      }
    }
    out.iters = it;
    if (!(dres == dres) || !(pres == pres) || !(gap == gap)) {  // NaN
      out.status = ST_FAILED;
      break;
    }
    double merit = fmax(fmax(pres / nh, dres / nq), gap);
    if (pres < tol * nh && dres < tol * nq && gap < 10.0 * tol) {
      out.status = ST_OPTIMAL;
      for (int r = 0; r < 6; ++r) { out.pi[r] = pi[r]; out.u[r] = u[r]; }
      return out;
    }
    if (merit < best_merit) {
      best_merit = merit;
      for (int k = 0; k < NB; ++k)
        for (int c = 0; c < 3; ++c) best_y[k][c] = y[k][c];
      for (int r = 0; r < 6; ++r) { best_w[r] = w[r]; best_pi[r] = pi[r]; best_u[r] = u[r]; }
    } else if (merit > 1e3 * best_merit || it >= max_iter) {
      break;
    }
    if (it >= max_iter) break;

    // ------------- NT scaling
    SocScale S1[NB], S2[NB];
    double d0[NB], lamk[NB][9], dl[DAT_MAXROW], laml[DAT_MAXROW];
    bool okc = true;
    for (int k = 0; k < NB; ++k) {
      d0[k] = sqrt(sk[k][0] / zk[k][0]);
      lamk[k][0] = sqrt(sk[k][0] * zk[k][0]);
      okc = okc && soc_scaling(sk[k] + 1, zk[k] + 1, S1[k]) && soc_scaling(sk[k] + 5, zk[k] + 5, S2[k]);
      soc_apply(S1[k], zk[k] + 1, lamk[k] + 1, false);
      soc_apply(S2[k], zk[k] + 5, lamk[k] + 5, false);
    }
    if (!okc) break;
    for (int l = 0; l < ml; ++l) {
      dl[l] = sqrt(sl[l] / zl[l]);
      laml[l] = sqrt(sl[l] * zl[l]);
    }
    // scaled block constraint matrix Gs = W^-1 G (9 x 3) and D_k = kappa I + Gs'Gs
    double Gs[NB][9][3], Dinv[NB][9];
    for (int k = 0; k < NB; ++k) {
      for (int c = 0; c < 3; ++c) {
        double e[3] = {0, 0, 0};
        e[c] = 1.0;
        double g[9];
        Gy(e, g);
        Gs[k][0][c] = g[0] / d0[k];
        double t[4];
        soc_apply(S1[k], g + 1, t, true);
        for (int j = 0; j < 4; ++j) Gs[k][1 + j][c] = t[j];
        soc_apply(S2[k], g + 5, t, true);
        for (int j = 0; j < 4; ++j) Gs[k][5 + j][c] = t[j];
      }
      double D[9];
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
          double s = (r == c) ? kap : 0.0;
          for (int j = 0; j < 9; ++j) s += Gs[k][j][r] * Gs[k][j][c];
          D[3 * r + c] = s;
        }
      // explicit inverse through Cholesky (the cofactor formula cancels catastrophically when
      // an active cone makes D_k strongly graded)
      Chol3 Lc;
      if (!chol3(D, Lc)) { okc = false; break; }
      for (int c = 0; c < 3; ++c) {
        double e[3] = {0, 0, 0}, x[3];
        e[c] = 1.0;
        chol3_solve(Lc, e, x);
        Dinv[k][c] = x[0]; Dinv[k][3 + c] = x[1]; Dinv[k][6 + c] = x[2];
      }
    }
    if (!okc) break;
    // M = C + sum_l (z/s) a_l a_l' (u-space), assembled in (dvl, dwl) coordinates
    double Mm[6][6];
    {
      double Xv[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, Xw[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      for (int l = 0; l < ml; ++l) {
        double wgt = zl[l] / sl[l];
        double* X = l < nw ? Xw : Xv;
        for (int r = 0; r < 3; ++r)
          for (int c = 0; c < 3; ++c) X[3 * r + c] += wgt * R.a[l][r] * R.a[l][c];
      }
      // Av = [im I, Bv];  Av' Xv Av = [[im^2 Xv, im Xv Bv], [im Bv' Xv, Bv' Xv Bv]]
      const double im = P.m.inv_mT;
      double XB[9], BXB[9], JXJ[9], XJ[9];
      mm3(Xv, P.m.Bv, XB);
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
          double s = 0.0;
          for (int k2 = 0; k2 < 3; ++k2) s += P.m.Bv[3 * k2 + r] * XB[3 * k2 + c];
          BXB[3 * r + c] = s;
        }
      mm3(Xw, P.m.JTi, XJ);
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
          double s = 0.0;
          for (int k2 = 0; k2 < 3; ++k2) s += P.m.JTi[3 * k2 + r] * XJ[3 * k2 + c];
          JXJ[3 * r + c] = s;
        }
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
          Mm[r][c] = P.C[r][c] + im * im * Xv[3 * r + c];
          Mm[r][3 + c] = P.C[r][3 + c] + im * XB[3 * r + c];
          Mm[3 + r][c] = P.C[3 + r][c] + im * XB[3 * c + r];
          Mm[3 + r][3 + c] = P.C[3 + r][3 + c] + BXB[3 * r + c] + JXJ[3 * r + c];
        }
    }
    // factorisations
    double LU[6][6];
    int piv[6];
    if (MODE == MODE_DD) {
      for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 6; ++c) LU[r][c] = Mm[r][c];
      if (!chol6(LU)) break;
    } else {
      // T = sum_k U_k D_k^-1 U_k' (+ K / rho);  factor (I + M T)
      double T[6][6];
      for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 6; ++c) T[r][c] = (MODE == MODE_CADMM) ? P.K[r][c] / P.rho : 0.0;
      for (int k = 0; k < NB; ++k) add_UDUt(T, P.Rt[k], Dinv[k], 1.0);
      for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 6; ++c) {
          double s = (r == c) ? 1.0 : 0.0;
          for (int k = 0; k < 6; ++k) s += Mm[r][k] * T[k][c];
          LU[r][c] = s;
        }
      if (!lu6(LU, piv)) break;
    }

    // core structured solve of (D + U'MU) dx = b (CADMM/CENT) or its DD analogue
    auto core = [&](double bk[NB][3], const double* Rfr, const double* bu, double dy[NB][3], double* dw,
                    double* du) {
      if (MODE == MODE_DD) {
        double rw[6];
        for (int r = 0; r < 6; ++r) rw[r] = -Rfr[r] + bu[r];
        chol6_solve(LU, rw);
        for (int r = 0; r < 6; ++r) du[r] = rw[r];
        for (int k = 0; k < NB; ++k) {
          double t[3], v[3];
          Ut_apply(P.Rt[k], Rfr, t);
          for (int c = 0; c < 3; ++c) v[c] = bk[k][c] + t[c];
          mv3(Dinv[k], v, dy[k]);
        }
        for (int r = 0; r < 6; ++r) dw[r] = du[r];
        for (int k = 0; k < NB; ++k) {
          double t[6];
          U_apply(P.Rt[k], dy[k], t);
          for (int r = 0; r < 6; ++r) dw[r] -= t[r];
        }
        return;
      }
      double bk2[NB][3], yv[6] = {0, 0, 0, 0, 0, 0};
      for (int k = 0; k < NB; ++k) {
        double t[3], v[3], ut[6];
        Ut_apply(P.Rt[k], bu, t);
        for (int c = 0; c < 3; ++c) bk2[k][c] = bk[k][c] + t[c];
        mv3(Dinv[k], bk2[k], v);
        U_apply(P.Rt[k], v, ut);
        for (int r = 0; r < 6; ++r) yv[r] += ut[r];
      }
      double kb[6] = {0, 0, 0, 0, 0, 0};
      if (MODE == MODE_CADMM) {
        Kmul(bu, kb);
        for (int r = 0; r < 6; ++r) yv[r] += (-Rfr[r] + kb[r]) / P.rho;
      }
      double tau[6];
      for (int r = 0; r < 6; ++r) {
        double s = 0.0;
        for (int c = 0; c < 6; ++c) s += Mm[r][c] * yv[c];
        tau[r] = s;
      }
      lu6_solve(LU, piv, tau);
      for (int k = 0; k < NB; ++k) {
        double t[3], v[3];
        Ut_apply(P.Rt[k], tau, t);
        for (int c = 0; c < 3; ++c) v[c] = bk2[k][c] - t[c];
        mv3(Dinv[k], v, dy[k]);
      }
      if (MODE == MODE_CADMM) {
        double kt[6];
        Kmul(tau, kt);
        for (int r = 0; r < 6; ++r) dw[r] = (-Rfr[r] + kb[r] - kt[r]) / P.rho;
      } else {
        for (int r = 0; r < 6; ++r) dw[r] = 0.0;
      }
      for (int r = 0; r < 6; ++r) du[r] = (MODE == MODE_CADMM) ? dw[r] : 0.0;
      for (int k = 0; k < NB; ++k) {
        double t[6];
        U_apply(P.Rt[k], dy[k], t);
        for (int r = 0; r < 6; ++r) du[r] += t[r];
      }
    };

    // Newton direction for complementarity target rs (scaled). Outputs scaled dz (W dz) and
    // scaled ds (W^-1 ds) for cone blocks and rows, plus dy, dw.
    double dy[NB][3], dw[6], dun[6], dzs_k[NB][9], dss_k[NB][9], dzs_l[DAT_MAXROW], dss_l[DAT_MAXROW];
    auto newton = [&](const double rsk[NB][9], const double* rsl) {
      double tks[NB][9], lrs[NB][9], tls[DAT_MAXROW], bk[NB][3], bu[6];
      for (int k = 0; k < NB; ++k) {
        double wr[9];
        wr[0] = rzk[k][0] / d0[k];
        soc_apply(S1[k], rzk[k] + 1, wr + 1, true);
        soc_apply(S2[k], rzk[k] + 5, wr + 5, true);
        lrs[k][0] = rsk[k][0] / lamk[k][0];
        soc_jdiv(lamk[k] + 1, rsk[k] + 1, lrs[k] + 1);
        soc_jdiv(lamk[k] + 5, rsk[k] + 5, lrs[k] + 5);
        for (int j = 0; j < 9; ++j) tks[k][j] = wr[j] - lrs[k][j];
        for (int c = 0; c < 3; ++c) {
          double s = 0.0;
          for (int j = 0; j < 9; ++j) s += Gs[k][j][c] * tks[k][j];
          bk[k][c] = -rk[k][c] - s;
        }
      }
      double zw[DAT_MAXROW];
      for (int l = 0; l < ml; ++l) {
        tls[l] = rzl[l] / dl[l] - rsl[l] / laml[l];
        zw[l] = tls[l] / dl[l];
      }
      rows_adj(zw, bu);
      double du[6];
      core(bk, Rf, bu, dy, dw, du);
      for (int ref = 0; ref < 3; ++ref) {
        // scaled dual directions implied by (dy, du)
        for (int k = 0; k < NB; ++k)
          for (int j = 0; j < 9; ++j) {
            double s = tks[k][j];
            for (int c = 0; c < 3; ++c) s += Gs[k][j][c] * dy[k][c];
            dzs_k[k][j] = s;
          }
        double ra[DAT_MAXROW];
        row_vals(du, ra, false);
        for (int l = 0; l < ml; ++l) dzs_l[l] = -ra[l] / dl[l] + tls[l];
        if (ref == 2) break;
        // linearised dual residual of the full system; refine
        double dzl[DAT_MAXROW], dpi[6], adz[6];
        for (int l = 0; l < ml; ++l) dzl[l] = dzs_l[l] / dl[l];
        Cmul(du, dpi);
        rows_adj(dzl, adz);
        for (int r = 0; r < 6; ++r) dpi[r] -= adz[r];
        double ek[NB][3], ef[6];
        for (int k = 0; k < NB; ++k) {
          double ut[3];
          Ut_apply(P.Rt[k], dpi, ut);
          for (int c = 0; c < 3; ++c) {
            double s = 0.0;
            for (int j = 0; j < 9; ++j) s += Gs[k][j][c] * dzs_k[k][j];
            ek[k][c] = -(kap * dy[k][c] + ut[c] + s + rk[k][c]);
          }
        }
        if (MODE == MODE_CADMM) {
          double kp[6];
          Kmul(dpi, kp);
          for (int r = 0; r < 6; ++r) ef[r] = P.rho * dw[r] + kp[r] + Rf[r];
        } else if (MODE == MODE_DD) {
          for (int r = 0; r < 6; ++r) ef[r] = dpi[r] + Rf[r];
        } else {
          for (int r = 0; r < 6; ++r) ef[r] = 0.0;
        }
        double zero6[6] = {0, 0, 0, 0, 0, 0}, cy[NB][3], cw6[6], cu6[6];
        core(ek, ef, zero6, cy, cw6, cu6);
        for (int k = 0; k < NB; ++k)
          for (int c = 0; c < 3; ++c) dy[k][c] += cy[k][c];
        for (int r = 0; r < 6; ++r) { dw[r] += cw6[r]; du[r] += cu6[r]; }
      }
      for (int r = 0; r < 6; ++r) dun[r] = du[r];
      for (int k = 0; k < NB; ++k)
        for (int j = 0; j < 9; ++j) dss_k[k][j] = -lrs[k][j] - dzs_k[k][j];
      for (int l = 0; l < ml; ++l) dss_l[l] = -rsl[l] / laml[l] - dzs_l[l];
    };
    auto step_len = [&]() {
      double a = 1e300;
      for (int k = 0; k < NB; ++k) {
        if (dss_k[k][0] < 0) a = fmin(a, -lamk[k][0] / dss_k[k][0]);
        if (dzs_k[k][0] < 0) a = fmin(a, -lamk[k][0] / dzs_k[k][0]);
        a = fmin(a, soc_step(lamk[k] + 1, dss_k[k] + 1));
        a = fmin(a, soc_step(lamk[k] + 1, dzs_k[k] + 1));
        a = fmin(a, soc_step(lamk[k] + 5, dss_k[k] + 5));
        a = fmin(a, soc_step(lamk[k] + 5, dzs_k[k] + 5));
      }
      for (int l = 0; l < ml; ++l) {
        if (dss_l[l] < 0) a = fmin(a, -laml[l] / dss_l[l]);
        if (dzs_l[l] < 0) a = fmin(a, -laml[l] / dzs_l[l]);
      }
      return a;
    };

    // predictor
    double rsk[NB][9], rsl[DAT_MAXROW];
    for (int k = 0; k < NB; ++k) {
      rsk[k][0] = lamk[k][0] * lamk[k][0];
      soc_jprod(lamk[k] + 1, lamk[k] + 1, rsk[k] + 1);
      soc_jprod(lamk[k] + 5, lamk[k] + 5, rsk[k] + 5);
    }
    for (int l = 0; l < ml; ++l) rsl[l] = laml[l] * laml[l];
    newton(rsk, rsl);
    double aaff = fmin(1.0, step_len());
    double gaff = 0.0;
    for (int k = 0; k < NB; ++k)
        for (int j = 0; j < 9; ++j) gaff += (lamk[k][j] + aaff * dss_k[k][j]) * (lamk[k][j] + aaff * dzs_k[k][j]);
    for (int l = 0; l < ml; ++l) gaff += (laml[l] + aaff * dss_l[l]) * (laml[l] + aaff * dzs_l[l]);
    double sig = gaff / gap;
    sig = fmax(0.0, fmin(1.0, sig * sig * sig));
    double mu = gap / deg;
    // corrector: rs = lam o lam + dss_aff o dzs_aff - sig mu e
    for (int k = 0; k < NB; ++k) {
      double c1[4], c2[4];
      soc_jprod(dss_k[k] + 1, dzs_k[k] + 1, c1);
      soc_jprod(dss_k[k] + 5, dzs_k[k] + 5, c2);
      rsk[k][0] += dss_k[k][0] * dzs_k[k][0] - sig * mu;
      for (int j = 0; j < 4; ++j) { rsk[k][1 + j] += c1[j]; rsk[k][5 + j] += c2[j]; }
      rsk[k][1] -= sig * mu;
      rsk[k][5] -= sig * mu;
    }
    for (int l = 0; l < ml; ++l) rsl[l] += dss_l[l] * dzs_l[l] - sig * mu;
    newton(rsk, rsl);
    double alpha = fmin(1.0, 0.99 * step_len());
    // safeguard: Mehrotra's corrector can increase the gap of a feasible iterate (it then cycles);
    // backtrack until the complementarity gap decreases
    const bool feasible = pres < 1e-8 * nh && dres < 1e-8 * nq;
    for (int bt = 0; feasible && bt < 8; ++bt) {
      double g = 0.0;
      for (int k = 0; k < NB; ++k)
        for (int j = 0; j < 9; ++j) g += (lamk[k][j] + alpha * dss_k[k][j]) * (lamk[k][j] + alpha * dzs_k[k][j]);
      for (int l = 0; l < ml; ++l) g += (laml[l] + alpha * dss_l[l]) * (laml[l] + alpha * dzs_l[l]);
      if (g <= gap * (1.0 - 0.01 * alpha)) break;
      alpha *= 0.5;
    }
    // update.  ds from the primal equation (keeps G y + s = h exact), dz = W^-1 dzs.
    for (int k = 0; k < NB; ++k) {
      double g[9], dz[9];
      Gy(dy[k], g);
      dz[0] = dzs_k[k][0] / d0[k];
      soc_apply(S1[k], dzs_k[k] + 1, dz + 1, true);
      soc_apply(S2[k], dzs_k[k] + 5, dz + 5, true);
      for (int j = 0; j < 9; ++j) {
        sk[k][j] += alpha * (-rzk[k][j] - g[j]);
        zk[k][j] += alpha * dz[j];
      }
      for (int c = 0; c < 3; ++c) y[k][c] += alpha * dy[k][c];
    }
    for (int r = 0; r < 6; ++r) w[r] += alpha * dw[r];
    {
      double ra[DAT_MAXROW];
      row_vals(dun, ra, false);
      for (int l = 0; l < ml; ++l) {
        sl[l] += alpha * (-rzl[l] + ra[l]);
        zl[l] += alpha * dzs_l[l] / dl[l];
      }
    }
  }
  // not converged to tol: return the best iterate seen; "optimal" if within 100 tol (Clarabel's
  // reduced-accuracy band), otherwise inaccurate (the reference holds its previous solution).
  if (best_merit < 1e300) {
    for (int k = 0; k < NB; ++k)
      for (int c = 0; c < 3; ++c) y[k][c] = best_y[k][c];
    for (int r = 0; r < 6; ++r) { w[r] = best_w[r]; out.pi[r] = best_pi[r]; out.u[r] = best_u[r]; }
    out.status = best_merit < 1e2 * tol ? ST_OPTIMAL : ST_INACCURATE;
  }
  return out;
}

// =====================================================================================
// per-controller QP builders
// =====================================================================================
// C-ADMM agent i (control/rqp_cadmm.py:26-501): variables f in R^{3 x n} (agent i's full copy).
// Cost: Phi(u) with k = 0.1/n, k_feq ||f_i - f_eq_i||^2, leader terms, <lam, f> + rho/2 ||f||^2
// - <rho fbar, f>  ==  rho/2 ||f - a||^2 + const with a = fbar - lam / rho.
// Only f_i carries cones; f_j (j != i) are free and eliminated through (K, atil).
// lam, fbar: (3n) agent-major.  Rt_all: n x 9 (hat(r_com_j) Rl').
DAT_HD void build_cadmm_static(QP<1>& P, const double* prm, int n, const double* st, const double* acc, int i,
                               const double* Rt_all) {
  build_common(P, prm, n, st, acc, prm[DAT_P_KFD], prm[DAT_P_KMD], i == 0 ? 1.0 : 0.0);
  for (int r = 0; r < 6; ++r)
    for (int c = 0; c < 6; ++c) P.K[r][c] = 0.0;
  double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  for (int j = 0; j < n; ++j)
    if (j != i) add_UDUt(P.K, Rt_all + 9 * j, I3, 1.0);
  for (int c = 0; c < 9; ++c) P.Rt[0][c] = Rt_all[9 * i + c];
  const double* feq = prm + DAT_P_FEQ(n) + 3 * i;
  for (int c = 0; c < 3; ++c) P.y0[0][c] = feq[c];
}
// per-iteration part: penalty rho and a = fbar - lam / rho
DAT_HD void build_cadmm_dynamic(QP<1>& P, const double* prm, int n, int i, const double* Rt_all, const double* lam,
                                const double* fbar, double rho) {
  const double kfeq = prm[DAT_P_KFEQ];
  P.rho = rho;
  P.kappa = 2.0 * kfeq + rho;
  const double* feq = prm + DAT_P_FEQ(n) + 3 * i;
  for (int r = 0; r < 6; ++r) P.atil[r] = 0.0;
  for (int j = 0; j < n; ++j) {
    double a[3] = {fbar[3 * j] - lam[3 * j] / rho, fbar[3 * j + 1] - lam[3 * j + 1] / rho,
                   fbar[3 * j + 2] - lam[3 * j + 2] / rho};
    if (j == i) {
      for (int c = 0; c < 3; ++c) P.q[0][c] = -2.0 * kfeq * feq[c] - rho * a[c];
    } else {
      double t[6];
      U_apply(Rt_all + 9 * j, a, t);
      for (int r = 0; r < 6; ++r) P.atil[r] += t[r];
    }
  }
}
// materialise agent i's copy: f_i = y, f_j = a_j - U_j' pi / rho  (stationarity of the free blocks)
DAT_HD void cadmm_materialize(const QP<1>& P, int n, int i, const double* Rt_all, const double* lam,
                              const double* fbar, const double* y, const double* pi, double* f) {
  for (int j = 0; j < n; ++j) {
    if (j == i) {
      f[3 * j] = y[0]; f[3 * j + 1] = y[1]; f[3 * j + 2] = y[2];
      continue;
    }
    double t[3];
    Ut_apply(Rt_all + 9 * j, pi, t);
    for (int c = 0; c < 3; ++c) f[3 * j + c] = fbar[3 * j + c] - lam[3 * j + c] / P.rho - t[c] / P.rho;
  }
}

// DD agent i (control/rqp_dd.py:27-505): variables (f_i, F_i, M_i); with w = (F_i, M_i),
// u = U_i f_i + w.  Cost Phi(u) + k_feq ||f_i - f_eq_i||^2 + c_fi'f_i + (c_Fi, c_Mi)'w.
DAT_HD void build_dd_static(QP<1>& P, const double* prm, int n, const double* st, const double* acc, int i,
                            const double* Rt_i) {
  build_common(P, prm, n, st, acc, prm[DAT_P_KFD], prm[DAT_P_KMD], i == 0 ? 1.0 : 0.0);
  const double* feq = prm + DAT_P_FEQ(n) + 3 * i;
  for (int c = 0; c < 9; ++c) P.Rt[0][c] = Rt_i[c];
  for (int c = 0; c < 3; ++c) P.y0[0][c] = feq[c];
  P.kappa = 2.0 * prm[DAT_P_KFEQ];
  P.rho = 1.0;
}
// prices c = (c_fi, c_Fi, c_Mi) (control/rqp_dd.py:718-722)
DAT_HD void set_dd_price(QP<1>& P, const double* prm, int n, int i, const double* c9) {
  const double* feq = prm + DAT_P_FEQ(n) + 3 * i;
  const double kfeq = prm[DAT_P_KFEQ];
  for (int c = 0; c < 3; ++c) P.q[0][c] = -2.0 * kfeq * feq[c] + c9[c];
  for (int r = 0; r < 6; ++r) P.cw[r] = c9[3 + r];
}

// Centralized (control/rqp_centralized.py:27-448): all n agents' forces, k = 0.1, leader terms on.
template <int NB>
DAT_HD void build_cent(QP<NB>& P, const double* prm, int n, const double* st, const double* acc) {
  build_common(P, prm, n, st, acc, prm[DAT_P_KFC], prm[DAT_P_KMC], 1.0);
  const double kfeq = prm[DAT_P_KFEQ];
  const double* Rl = st + DAT_S_RL(n);
  for (int k = 0; k < NB; ++k) {
    const double* feq = prm + DAT_P_FEQ(n) + 3 * k;
    make_Rt(prm + DAT_P_RCOM(n) + 3 * k, Rl, P.Rt[k]);
    for (int c = 0; c < 3; ++c) {
      P.y0[k][c] = feq[c];
      P.q[k][c] = -2.0 * kfeq * feq[c];
    }
  }
  P.kappa = 2.0 * kfeq;
  P.rho = 1.0;
}

// =====================================================================================
// low-level control + dynamics rollout (K6)
// =====================================================================================
// RQPLowLevelController._rotation_from_unit_vector (control/rqp_centralized.py:503-516)
DAT_HD void rot_from_unit(const double* q, double* R) {
  double sx = -q[1];
  double cx = sqrt(q[0] * q[0] + q[2] * q[2]);
  double sy = q[0] / cx, cy = q[2] / cx;
  R[0] = cy; R[3] = 0.0; R[6] = -sy;
  R[1] = sx * sy; R[4] = cx; R[7] = cy * sx;
  R[2] = q[0]; R[5] = q[1]; R[8] = q[2];
}

// SO(3) PD law with wd = dwd = 0 (utils/so3_tracking_controllers.py:18-43, gains
// control/rqp_centralized.py:488-489): M = -kR e_R - kW w + w x J w, e_R = vee(Rd'R - R'Rd)/2;
// thrust f = f_des . R e3 (control/rqp_centralized.py:527).
DAT_HD void ll_control_agent(const double* R, const double* w, const double* J, const double* fdes, double* f,
                             double* M) {
  *f = fdes[0] * R[2] + fdes[1] * R[5] + fdes[2] * R[8];
  double nn = sqrt(dot3(fdes, fdes));
  double qd[3] = {fdes[0] / nn, fdes[1] / nn, fdes[2] / nn};
  double Rd[9];
  rot_from_unit(qd, Rd);
  double A[9];  // Rd' R
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) A[3 * r + c] = Rd[r] * R[c] + Rd[3 + r] * R[3 + c] + Rd[6 + r] * R[6 + c];
  // vee(A - A')/2
  double eR[3] = {0.5 * (A[7] - A[5]), 0.5 * (A[2] - A[6]), 0.5 * (A[3] - A[1])};
  double Jw[3], wJw[3];
  mv3(J, w, Jw);
  cross3(w, Jw, wJw);
  const double kR = 0.25, kW = 0.075;
  for (int c = 0; c < 3; ++c) M[c] = -kR * eR[c] - kW * w[c] + wJw[c];
}

// One simulation step of one scenario: LL control from f_des, forward dynamics, integration
// (system/rigid_quadrotor_payload.py:173-222, 129-148).  counter: steps since the last projection.
template <int NMAX>
DAT_HD void sim_step(const double* prm, int n, double* st, int* counter, const double* fdes, double dt) {
  double* R = st + DAT_S_R(n);
  double* W = st + DAT_S_W(n);
  double* xl = st + DAT_S_XL(n);
  double* vl = st + DAT_S_VL(n);
  double* Rl = st + DAT_S_RL(n);
  double* wl = st + DAT_S_WL(n);
  const double mT = prm[DAT_P_MT];
  const double* xc = prm + DAT_P_XCOM;
  const double* JT = prm + DAT_P_JT;
  const double* JTi = prm + DAT_P_JTI;
  const double* rcom = prm + DAT_P_RCOM(n);
  const double* J = prm + DAT_P_J(n);
  const double* Ji = prm + DAT_P_JINV(n);
  double dvc[3] = {0, 0, 0}, mom[3] = {0, 0, 0};
  double dw[NMAX][3];
  for (int i = 0; i < n; ++i) {
    double f, M[3];
    ll_control_agent(R + 9 * i, W + 3 * i, J + 9 * i, fdes + 3 * i, &f, M);
    double Jw[3], wJw[3], t[3];
    mv3(J + 9 * i, W + 3 * i, Jw);
    cross3(W + 3 * i, Jw, wJw);
    for (int c = 0; c < 3; ++c) t[c] = M[c] - wJw[c];
    mv3(Ji + 9 * i, t, dw[i]);
    double u[3] = {R[9 * i + 2] * f, R[9 * i + 5] * f, R[9 * i + 8] * f};  // f R e3
    dvc[0] += u[0]; dvc[1] += u[1]; dvc[2] += u[2];
    double ub[3], m3[3];
    mtv3(Rl, u, ub);
    cross3(rcom + 3 * i, ub, m3);
    mom[0] += m3[0]; mom[1] += m3[1]; mom[2] += m3[2];
  }
  for (int c = 0; c < 3; ++c) dvc[c] /= mT;
  dvc[2] -= DAT_GRAVITY;
  double Jwl[3], wJwl[3], t[3], dwl[3];
  mv3(JT, wl, Jwl);
  cross3(wl, Jwl, wJwl);
  for (int c = 0; c < 3; ++c) t[c] = mom[c] - wJwl[c];
  mv3(JTi, t, dwl);
  // dvl = dv_com - Rl (hat(wl)^2 + hat(dwl)) x_com
  double a1[3], a2[3], a3[3], sum[3], Rs[3], dvl[3];
  cross3(wl, xc, a1);
  cross3(wl, a1, a2);
  cross3(dwl, xc, a3);
  for (int c = 0; c < 3; ++c) sum[c] = a2[c] + a3[c];
  mv3(Rl, sum, Rs);
  for (int c = 0; c < 3; ++c) dvl[c] = dvc[c] - Rs[c];
  // integrate
  for (int i = 0; i < n; ++i) {
    double v[3], E[9], Rn[9];
    for (int c = 0; c < 3; ++c) v[c] = (W[3 * i + c] + dw[i][c] * dt / 2.0) * dt;
    exp3(v, E);
    mm3(R + 9 * i, E, Rn);
    for (int c = 0; c < 9; ++c) R[9 * i + c] = Rn[c];
    for (int c = 0; c < 3; ++c) W[3 * i + c] += dw[i][c] * dt;
  }
  for (int c = 0; c < 3; ++c) {
    xl[c] = xl[c] + vl[c] * dt + dvl[c] * dt * dt / 2.0;
    vl[c] = vl[c] + dvl[c] * dt;
  }
  {
    double v[3], E[9], Rn[9];
    for (int c = 0; c < 3; ++c) v[c] = (wl[c] + dwl[c] * dt / 2.0) * dt;
    exp3(v, E);
    mm3(Rl, E, Rn);
    for (int c = 0; c < 9; ++c) Rl[c] = Rn[c];
    for (int c = 0; c < 3; ++c) wl[c] += dwl[c] * dt;
  }
  *counter += 1;
  if (*counter >= 20) {  // _INTEGRATION_STEPS_PER_ROTATION_PROJECTION
    polar3(Rl);
    for (int i = 0; i < n; ++i) polar3(R + 9 * i);
    *counter = 0;
  }
}

// _desired_acceleration_forest (example/rqp_example.py:33-59); acc = (dvl_des, dwl_des)
DAT_HD void desired_accel_forest(const double* st, int n, const double* mountain, double x_offset, double* acc) {
  const double* xl = st + DAT_S_XL(n);
  const double* vl = st + DAT_S_VL(n);
  double xr[3] = {xl[0] + x_offset, 0.0, 1.5};
  double dx = xl[0] - mountain[DAT_M_CX], dy = xl[1] - mountain[DAT_M_CY];
  double nn = sqrt(dx * dx + dy * dy);
  if (nn < mountain[DAT_M_RADIUS])
    xr[2] = sqrt(mountain[DAT_M_SPHERE_R] * mountain[DAT_M_SPHERE_R] - nn * nn) - mountain[DAT_M_DEPTH] + 1.5;
  double vr[3] = {0.5, 0.0, 0.0};
  double d[3];
  for (int c = 0; c < 3; ++c) d[c] = -(vl[c] - vr[c]) - (xl[c] - xr[c]);
  double dn = sqrt(dot3(d, d));
  if (dn > 0) {
    double s = fmin(dn, 1.0) / dn;
    for (int c = 0; c < 3; ++c) d[c] *= s;
  }
  acc[0] = d[0]; acc[1] = d[1]; acc[2] = d[2];
  acc[3] = 0.0; acc[4] = 0.0; acc[5] = 0.0;
}

}  // namespace dat
