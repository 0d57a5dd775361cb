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
// LDS address space: solver data kept in LDS is read through volatile address_space(3) pointers
// (dat_qp.hpp "How the IPM reads LDS").
#define DAT_LDS __attribute__((address_space(3)))
typedef double dat_d2 __attribute__((ext_vector_type(2)));

// N consecutive doubles into registers.  Plain pointers: element copies.  A volatile LDS pointer to
// a 16-byte aligned record: one ds_read_b128 per pair -- the compiler never merges volatile reads,
// so element reads would be N ds_read_b64 instructions, each with its own wait (every LDS-resident
// record the kernels read this way starts on a 16-byte boundary: QPShared, the RT_STRIDE U-maps).
template <int N, class P>
DAT_HD void ldn(P p, double* o) {
#pragma unroll
  for (int k = 0; k < N; ++k) o[k] = p[k];
}
template <int N>
DAT_HD void ldn(const volatile DAT_LDS double* p, double* o) {
#if defined(__HIP_DEVICE_COMPILE__)
  const volatile DAT_LDS dat_d2* q = (const volatile DAT_LDS dat_d2*)p;
#pragma unroll
  for (int k = 0; k < N / 2; ++k) {
    const dat_d2 v = q[k];
    o[2 * k] = v.x;
    o[2 * k + 1] = v.y;
  }
  if (N & 1) o[N - 1] = p[N - 1];
#else
  for (int k = 0; k < N; ++k) o[k] = p[k];
#endif
}

DAT_HD double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
DAT_HD void cross3(const double* a, const double* b, double* o) {
  double x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}
template <class PM>
DAT_HD void mv3(PM Mp, const double* v, double* o) {
  double M[9];
  ldn<9>(Mp, M);
  double x = M[0] * v[0] + M[1] * v[1] + M[2] * v[2];
  double y = M[3] * v[0] + M[4] * v[1] + M[5] * v[2];
  double z = M[6] * v[0] + M[7] * v[1] + M[8] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}
template <class PM>
DAT_HD void mtv3(PM Mp, const double* v, double* o) {
  double M[9];
  ldn<9>(Mp, M);
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

// fast fp64 reciprocal: hardware estimate + two Newton steps (<= 1 ulp off the correctly
// rounded quotient; the IPM does not need IEEE division)
DAT_HD double frcp(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  return fma(fma(-x, r, 1.0), r, r);
#else
  return 1.0 / x;
#endif
}

// packed symmetric storage (upper triangle, row-major): 6x6 -> 21, 3x3 -> 6
DAT_HD constexpr int sp6(int r, int c) {
  return r <= c ? r * 6 - (r * (r - 1)) / 2 + (c - r) : c * 6 - (c * (c - 1)) / 2 + (r - c);
}
DAT_HD constexpr int sp3(int r, int c) {
  return r <= c ? r * 3 - (r * (r - 1)) / 2 + (c - r) : c * 3 - (c * (c - 1)) / 2 + (r - c);
}
template <class PA>
DAT_HD void spmv6(PA Ap, const double* v, double* o) {
  double A[21];
  ldn<21>(Ap, A);  // one read per entry pair (Ap may be a volatile LDS pointer)
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < 6; ++c) s += A[sp6(r, c)] * v[c];
    o[r] = s;
  }
}
DAT_HD void spmv3(const double* A, const double* v, double* o) {
  double x = A[0] * v[0] + A[1] * v[1] + A[2] * v[2];
  double y = A[1] * v[0] + A[3] * v[1] + A[4] * v[2];
  double z = A[2] * v[0] + A[4] * v[1] + A[5] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}

// inverse of an SPD 3x3 (packed in / packed out) through its Cholesky factor (the cofactor
// formula cancels catastrophically when an active cone makes the matrix strongly graded)
DAT_HD bool inv3_spd(const double* D, double* O) {
  if (!(D[0] > 0)) return false;
  double l00 = sqrt(D[0]), i00 = frcp(l00);
  double l10 = D[1] * i00, l20 = D[2] * i00;
  double d1 = D[3] - l10 * l10;
  if (!(d1 > 0)) return false;
  double l11 = sqrt(d1), i11 = frcp(l11);
  double l21 = (D[4] - l20 * l10) * i11;
  double d2 = D[5] - l20 * l20 - l21 * l21;
  if (!(d2 > 0)) return false;
  double l22 = sqrt(d2), i22 = frcp(l22);
  // L^-1 (lower): m00 = i00, m11 = i11, m22 = i22, m10 = -l10 i00 i11, m21 = -l21 i11 i22,
  // m20 = (l10 l21 - l11 l20) i00 i11 i22 ;  D^-1 = L^-T L^-1
  double m10 = -l10 * i00 * i11, m21 = -l21 * i11 * i22, m20 = (l10 * l21 - l11 * l20) * i00 * i11 * i22;
  O[0] = i00 * i00 + m10 * m10 + m20 * m20;
  O[1] = m10 * i11 + m20 * m21;
  O[2] = m20 * i22;
  O[3] = i11 * i11 + m21 * m21;
  O[4] = m21 * i22;
  O[5] = i22 * i22;
  return true;
}

// Square-root factor of D = kappa I + Gs'Gs for a 9 x 3 block Gs (columns gc[c]): Householder QR of the
// stacked 12 x 3 matrix [sqrt(kappa) I; Gs], D = R'R.  Forming D itself cancels catastrophically once an
// active cone makes Gs stiff: with |Gs| ~ 1e7-1e12 the entries of D carry absolute rounding errors
// eps |Gs|^2 >> kappa, so the compliant directions of D (and of D^-1, kept as an explicit matrix) are lost
// and the corrector's iterative refinement diverges.  QR is column-wise backward stable: the error it makes
// in the compliant directions is ~eps |Gs| instead of eps |Gs|^2.  Packed output (sp3 layout, upper):
// R[sp3(r, c)] = R_rc for r < c, R[sp3(j, j)] = 1 / R_jj.  Returns false on a non-finite or singular factor.
DAT_HD bool qr_cone(double kappa, const double gc[3][9], double* R) {
  const double sk = sqrt(kappa);
  double A[3][12];  // A[c][i]: column c, row i
#pragma unroll
  for (int c = 0; c < 3; ++c) {
#pragma unroll
    for (int i = 0; i < 3; ++i) A[c][i] = (i == c) ? sk : 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) A[c][3 + i] = gc[c][i];
  }
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    double nx = 0.0;
#pragma unroll
    for (int i = j; i < 12; ++i) nx += A[j][i] * A[j][i];
    nx = sqrt(nx);
    const double al = A[j][j] >= 0.0 ? -nx : nx;  // R_jj = al; v = x - al e_j
    const double v0 = A[j][j] - al;
    const double vv = nx * (nx + fabs(A[j][j]));  // v'v / 2
    ok = ok && (vv > 0.0) && (fabs(al) < 1e300);
    const double ivv = frcp(vv);
#pragma unroll
    for (int c = j + 1; c < 3; ++c) {
      double s = v0 * A[c][j];
#pragma unroll
      for (int i = j + 1; i < 12; ++i) s += A[j][i] * A[c][i];
      s *= ivv;
      A[c][j] -= s * v0;
#pragma unroll
      for (int i = j + 1; i < 12; ++i) A[c][i] -= s * A[j][i];
      R[sp3(j, c)] = A[c][j];
    }
    R[sp3(j, j)] = frcp(al);
  }
  return ok;
}
// o = D^-1 v = R^-1 R^-T v for the packed factor of qr_cone (o may alias v)
DAT_HD void dsolve3(const double* R, const double* v, double* o) {
  const double t0 = v[0] * R[0];
  const double t1 = (v[1] - R[1] * t0) * R[3];
  const double t2 = (v[2] - R[2] * t0 - R[4] * t1) * R[5];
  const double o2 = t2 * R[5];
  const double o1 = (t1 - R[4] * o2) * R[3];
  o[0] = (t0 - R[1] * o1 - R[2] * o2) * R[0];
  o[1] = o1;
  o[2] = o2;
}
// explicit D^-1 (packed) from the factor of qr_cone: M = R^-1 (upper), D^-1 = M M'
DAT_HD void dinv_explicit(const double* R, double* Di) {
  const double m00 = R[0], m11 = R[3], m22 = R[5];
  const double m01 = -R[1] * m11 * m00;
  const double m12 = -R[4] * m22 * m11;
  const double m02 = -(R[1] * m12 + R[2] * m22) * m00;
  Di[0] = m00 * m00 + m01 * m01 + m02 * m02;
  Di[1] = m01 * m11 + m02 * m12;
  Di[2] = m02 * m22;
  Di[3] = m11 * m11 + m12 * m12;
  Di[4] = m12 * m22;
  Di[5] = m22 * m22;
}

// 6x6 Cholesky of a packed SPD matrix into a packed lower factor (L[sp6(i,j)] = L_ij, i >= j);
// diagonal entries hold 1 / L_jj.  Returns false if not SPD.
DAT_HD bool chol6(const double* A, double* L) {
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double s = A[sp6(j, j)];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= L[sp6(j, k)] * L[sp6(j, k)];
    if (!(s > 0)) return false;
    double id = frcp(sqrt(s));
    L[sp6(j, j)] = id;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double t = A[sp6(i, j)];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= L[sp6(i, k)] * L[sp6(j, k)];
      L[sp6(i, j)] = t * id;
    }
  }
  return true;
}
// Same factorization with the true diagonal kept (L[sp6(j,j)] = L_jj): the factor is used as a
// multiplier (L v, L' v), not for substitution.
DAT_HD bool chol6_lower(const double* A, double* L) {
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double s = A[sp6(j, j)];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= L[sp6(j, k)] * L[sp6(j, k)];
    if (!(s > 0)) return false;
    const double d = sqrt(s);
    const double id = frcp(d);
    L[sp6(j, j)] = d;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double t = A[sp6(i, j)];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= L[sp6(i, k)] * L[sp6(j, k)];
      L[sp6(i, j)] = t * id;
    }
  }
  return true;
}
// N = I + L' T L (packed) for a packed lower factor L with true diagonal and a packed symmetric T:
// column c of T L, then the upper triangle of column c of L' (T L).
DAT_HD void ltl_plus_identity(const double* L, const double* T, double* N) {
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    double col[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      double s = 0.0;
#pragma unroll
      for (int j = c; j < 6; ++j) s += T[sp6(k, j)] * L[sp6(j, c)];
      col[k] = s;
    }
#pragma unroll
    for (int r = 0; r <= c; ++r) {
      double s = (r == c) ? 1.0 : 0.0;
#pragma unroll
      for (int k = r; k < 6; ++k) s += L[sp6(k, r)] * col[k];
      N[sp6(r, c)] = s;
    }
  }
}
DAT_HD void chol6_solve(const double* L, double* b) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s -= L[sp6(i, k)] * b[k];
    b[i] = s * L[sp6(i, i)];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    double s = b[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) s -= L[sp6(k, i)] * b[k];
    b[i] = s * L[sp6(i, i)];
  }
}

// P = Lm N^-1 Lm' (packed) from the packed lower factor Lm (true diagonal) of M and the Cholesky
// factor Ln of N (reciprocal diagonal, chol6): with X = Lm Ln^-T (row r: Ln x = Lm[r, :]'), P = X X'.
// The IPM keeps P (21 doubles) instead of Lm and Ln (42) through the Newton solves of an iteration;
// the corrector's iterative refinement absorbs the accuracy of the explicit product.
DAT_HD void schur_P(const double* Lm, const double* Ln, double* P) {
  double X[6][6];
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      double s = (i <= r) ? Lm[sp6(r, i)] : 0.0;
#pragma unroll
      for (int k = 0; k < i; ++k) s -= Ln[sp6(i, k)] * X[r][k];
      X[r][i] = s * Ln[sp6(i, i)];
    }
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int c = r; c < 6; ++c) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) s += X[r][k] * X[c][k];
      P[sp6(r, c)] = s;
    }
}

// Rt_j = hat(r_com_j) Rl' ;  U_j = [I; Rt_j] maps an agent force to its (force, CoM moment) pair
DAT_HD void make_Rt(const double* rcom, const double* Rl, double* Rt) {
  double H[9];
  skew3(rcom, H);
  mmt3(H, Rl, Rt);
}
// U_j x = (x, Rt x)
template <class PR>
DAT_HD void U_apply(PR Rt, const double* x, double* o) {
  o[0] = x[0]; o[1] = x[1]; o[2] = x[2];
  mv3(Rt, x, o + 3);
}
// U_j' v = v[0:3] + Rt' v[3:6]
template <class PR>
DAT_HD void Ut_apply(PR Rt, const double* v, double* o) {
  mtv3(Rt, v + 3, o);
  o[0] += v[0]; o[1] += v[1]; o[2] += v[2];
}
// packed 6x6 M += scale * U D U' for U = [I; Rt] and packed symmetric 3x3 D
template <class PR>
DAT_HD void add_UDUt(double* M, PR Rtp, const double* D, double scale) {
  double Df[9] = {D[0], D[1], D[2], D[1], D[3], D[4], D[2], D[4], D[5]};
  double Rt[9], RD[9], RDR[9];
  ldn<9>(Rtp, Rt);  // one read per entry pair (Rtp may be a volatile LDS pointer)
  mm3(Rt, Df, RD);
  mmt3(RD, Rt, RDR);
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      if (c >= r) {
        M[sp6(r, c)] += scale * Df[3 * r + c];
        M[sp6(3 + r, 3 + c)] += scale * RDR[3 * r + c];
      }
      M[sp6(r, 3 + c)] += scale * RD[3 * c + r];
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
    // Safeguarded Newton on the monotone slope g(t) = f'(t) inside the bracket [lo, hi] (g(lo) < 0 <
    // g(hi)): Newton steps where f is smooth, bisection whenever a step leaves the bracket or f''
    // vanishes.  Converges to the bracket's machine precision in a handful of steps where the
    // previous plain bisection took ~52.
    double lo = 0.0, hi = 1.0;
    t = 0.5;
    const double dxy2 = d[0] * d[0] + d[1] * d[1];
    for (int it = 0; it < 64; ++it) {
      double px = x0[0] + t * d[0] - c[0], py = x0[1] + t * d[1] - c[1], pz = x0[2] + t * d[2] - c[2];
      double rho = sqrt(px * px + py * py);
      double g = 0.0, hs = 0.0;
      if (rho > DAT_BARK_RADIUS) {
        double rp = (px * d[0] + py * d[1]) / rho;  // d rho / dt
        g += 2.0 * (rho - DAT_BARK_RADIUS) * rp;
        hs += 2.0 * rp * rp + 2.0 * (rho - DAT_BARK_RADIUS) * (dxy2 - rp * rp) / rho;
      }
      double az = fabs(pz) - DAT_BARK_HALF_HEIGHT;
      if (az > 0.0) {
        g += 2.0 * az * (pz > 0 ? d[2] : -d[2]);
        hs += 2.0 * d[2] * d[2];
      }
      if (g == 0.0) break;
      if (g < 0.0) lo = t; else hi = t;
      double tn = (hs > 0.0) ? t - g / hs : 0.5 * (lo + hi);
      if (!(tn > lo && tn < hi)) tn = 0.5 * (lo + hi);
      if (tn == t || tn <= lo || tn >= hi) break;
      t = tn;
    }
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

// Env CBF rows of one solve (control/rqp_cadmm.py:307-373; camera == none selects the centralized
// query without vision cone, rqp_centralized.py:280-337).  Tree selection: distance of the capsule
// centre to tree_pos <= vision_r + bark radius, plus the 2-D cone test for distributed agents; the
// DAT_NENV nearest selected trees fill the slots in order of distance.  Slot j carries the row
// lhs[j] . dvl >= rhs[j]; bit j of *mask is set when the reference emits that row (a tree closer
// than 1e-4 leaves it zero).  All slot indices are compile-time so the rows stay in registers.
DAT_HD EnvOut env_rows(const double* prm, int n, const double* st, const double* trees, int ntree,
                       int agent /* -1: centralized */, double alpha_env, unsigned* mask, double lhs[DAT_NENV][3],
                       double rhs[DAT_NENV]) {
  EnvOut out;
  out.collision = 0;
  out.min_env_dist = prm[DAT_P_VISR];
  *mask = 0u;
#pragma unroll
  for (int j = 0; j < DAT_NENV; ++j) { lhs[j][0] = lhs[j][1] = lhs[j][2] = 0.0; rhs[j] = 0.0; }
  if (trees == nullptr || ntree <= 0) return out;
  const double* xl = st + DAT_S_XL(n);
  const double* vl = st + DAT_S_VL(n);
  const double* Rl = st + DAT_S_RL(n);
  const double maxdec = prm[DAT_P_MAXDEC], visr = prm[DAT_P_VISR], rc = prm[DAT_P_COLR];
  const double deps = prm[DAT_P_DISTEPS];
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
  // sorted insertion of (distance, row) into the DAT_NENV slots
  double bd[DAT_NENV];
#pragma unroll
  for (int j = 0; j < DAT_NENV; ++j) bd[j] = 1e300;
  int cnt = 0;
  double dmin = 1e300;
  // trees are sorted by x (dat_set_forests): only the window |c.x - ctr.x| <= visr + bark radius
  // can pass the range test below; lower bound by binary search, stop past the upper edge
  const double reach = visr + DAT_BARK_RADIUS;
  int t0 = 0;
  for (int len = ntree; len > 0;) {
    int half = len >> 1;
    if (trees[3 * (t0 + half)] < ctr[0] - reach) { t0 += half + 1; len -= half + 1; } else { len = half; }
  }
  for (int t = t0; t < ntree; ++t) {
    const double* c = trees + 3 * t;
    if (c[0] > ctr[0] + reach) break;
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
    // the row this tree produces (zero when dd <= 1e-4 or the payload is at rest)
    double l3[3] = {0, 0, 0}, r1 = 0.0;
    if (dd > 1e-4 && speed > 0.0) {
      double rel[3] = {p1[0] - xl[0], p1[1] - xl[1], p1[2] - xl[2]};
      double proj = fmax(0.0, fmin(h, dot3(rel, vdir)));
      double mt = sqrt(2.0 * (h - proj) / maxdec);
      mt = fmax(0.0, speed / maxdec - mt);
      // proj = 0 makes the two terms equal in exact arithmetic (the reference gets an exact 0);
      // snap the rounding residue so such rows stay "0 >= rhs" like the reference's.
      if (mt < 1e-12 * speed / maxdec) mt = 0.0;
      double nr[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
      double nn = sqrt(dot3(nr, nr));
      nr[0] /= nn; nr[1] /= nn; nr[2] /= nn;
      l3[0] = nr[0] * mt; l3[1] = nr[1] * mt; l3[2] = nr[2] * mt;
      r1 = -alpha_env * (dd - deps) - dot3(nr, vl);
    }
    // position = number of kept entries with distance <= dd (ties keep arrival order)
    int pos = 0;
#pragma unroll
    for (int j = 0; j < DAT_NENV; ++j) pos += (bd[j] <= dd) ? 1 : 0;
    if (pos >= DAT_NENV) continue;
#pragma unroll
    for (int j = DAT_NENV - 1; j >= 1; --j) {
      if (j > pos) {
        bd[j] = bd[j - 1];
        lhs[j][0] = lhs[j - 1][0]; lhs[j][1] = lhs[j - 1][1]; lhs[j][2] = lhs[j - 1][2];
        rhs[j] = rhs[j - 1];
      }
    }
#pragma unroll
    for (int j = 0; j < DAT_NENV; ++j) {
      if (j == pos) {
        bd[j] = dd;
        lhs[j][0] = l3[0]; lhs[j][1] = l3[1]; lhs[j][2] = l3[2];
        rhs[j] = r1;
      }
    }
  }
  if (cnt > 0 && speed > 0.0) {
    out.min_env_dist = dmin;
    unsigned m = 0u;
#pragma unroll
    for (int j = 0; j < DAT_NENV; ++j)
      if (bd[j] < 1e299 && bd[j] > 1e-4) m |= 1u << j;
    *mask = m;
  }
  return out;
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

// Low-level SO(3) attitude laws of RQPLowLevelController (control/rqp_centralized.py:457-535), both
// with wd = dwd = 0 (:530-532); thrust f = f_des . R e3 (:525), Rd from f_des / |f_des| (:527-528).
constexpr int LL_PD = 0;  // so3_pd_tracking_control (utils/so3_tracking_controllers.py:18-43)
constexpr int LL_SM = 1;  // so3_sm_tracking_control (utils/so3_tracking_controllers.py:52-95)

// sign(y) |y|^r with sign(0) = 0 (np.power(np.abs(y), r) * np.sign(y))
DAT_HD double spow(double y, double r) { return y > 0.0 ? pow(y, r) : (y < 0.0 ? -pow(-y, r) : 0.0); }

// PD (gains control/rqp_centralized.py:488-489): M = -kR e_R - kW w + w x J w, e_R = vee(Rd'R - R'Rd)/2.
// SM (gains :491-496: r 0.5, k_R 1.415, l_R 0.707, k_s 0.113, l_s 0.057), Lee 2018 eqs. (34)-(36):
//   s = e_W + k_R e_R + l_R S(r, e_R),  E = (tr(R'Rd) I - R'Rd) / 2,  e_W = w,
//   M = -k_s s - l_s S(r, s) + w x J w - (k_R J + l_s r J T) E e_W,
// with T exactly as the reference evaluates it: the call T(e_R, r) (:92) swaps the arguments of
// T = lambda r, y: diag((|y| + 1e-6)^(r - 1)) (:88), so T = diag((0.5 + 1e-6)^(e_R,k - 1)).
DAT_HD void ll_control_agent(const double* R, const double* w, const double* J, const double* fdes, double* f,
                             double* M, int kind = LL_PD) {
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
  if (kind == LL_SM) {
    const double r = 0.5, kR = 1.415, lR = 0.707, ks = 0.113, ls = 0.057, eps = 1e-6;
    double sv[3];
    for (int c = 0; c < 3; ++c) sv[c] = w[c] + kR * eR[c] + lR * spow(eR[c], r);
    // E e_W with R'Rd = A'
    const double tr = A[0] + A[4] + A[8];
    double Ew[3];
    for (int c = 0; c < 3; ++c) Ew[c] = 0.5 * (tr * w[c] - (A[c] * w[0] + A[3 + c] * w[1] + A[6 + c] * w[2]));
    // (k_R J + l_s r J T) Ew = J (k_R Ew + l_s r T Ew)
    double v[3], Jv[3];
    for (int c = 0; c < 3; ++c) v[c] = kR * Ew[c] + ls * r * pow(r + eps, eR[c] - 1.0) * Ew[c];
    mv3(J, v, Jv);
    for (int c = 0; c < 3; ++c) M[c] = -ks * sv[c] - ls * spow(sv[c], r) + wJw[c] - Jv[c];
    return;
  }
  const double kR = 0.25, kW = 0.075;
  for (int c = 0; c < 3; ++c) M[c] = -kR * eR[c] - kW * w[c] + wJw[c];
}

// One simulation step of one scenario: LL control from f_des, forward dynamics, integration
// (system/rigid_quadrotor_payload.py:173-222, 129-148).  counter: steps since the last projection.
template <int NMAX>
DAT_HD void sim_step(const double* prm, int n, double* st, int* counter, const double* fdes, double dt,
                     int ll_kind = LL_PD) {
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
    ll_control_agent(R + 9 * i, W + 3 * i, J + 9 * i, fdes + 3 * i, &f, M, ll_kind);
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

// One step of the rigid payload driven by actuator forces f (3n, agent-major, ground frame) --
// RPDynamics.forward_dynamics + RPState.integrate (system/rigid_payload.py:76-90, 109-130), on the
// payload part of a dat state block with the rigid-payload parameter block (mT = ml, JT = Jl,
// r_com = r): ml dvl = sum f - ml g e3, Jl dwl + wl x Jl wl = sum hat(r_i) Rl' f_i.
DAT_HD void rp_step(const double* prm, int n, double* st, int* counter, const double* f, double dt) {
  double* xl = st + DAT_S_XL(n);
  double* vl = st + DAT_S_VL(n);
  double* Rl = st + DAT_S_RL(n);
  double* wl = st + DAT_S_WL(n);
  const double ml = prm[DAT_P_MT];
  const double* Jl = prm + DAT_P_JT;
  const double* Jli = prm + DAT_P_JTI;
  const double* r = prm + DAT_P_RCOM(n);
  double F[3] = {0, 0, 0}, Mo[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i) {
    double fb[3], m3[3];
    mtv3(Rl, f + 3 * i, fb);
    cross3(r + 3 * i, fb, m3);
    for (int c = 0; c < 3; ++c) { F[c] += f[3 * i + c]; Mo[c] += m3[c]; }
  }
  double dvl[3] = {F[0] / ml, F[1] / ml, F[2] / ml - DAT_GRAVITY};
  double Jw[3], wJw[3], t[3], dwl[3];
  mv3(Jl, wl, Jw);
  cross3(wl, Jw, wJw);
  for (int c = 0; c < 3; ++c) t[c] = Mo[c] - wJw[c];
  mv3(Jli, t, dwl);
  for (int c = 0; c < 3; ++c) {
    xl[c] = xl[c] + vl[c] * dt + dvl[c] * dt * dt / 2.0;
    vl[c] = vl[c] + dvl[c] * dt;
  }
  double v[3], E[9], Rn[9];
  for (int c = 0; c < 3; ++c) v[c] = (wl[c] + dwl[c] * dt / 2.0) * dt;
  exp3(v, E);
  mm3(Rl, E, Rn);
  for (int c = 0; c < 9; ++c) Rl[c] = Rn[c];
  for (int c = 0; c < 3; ++c) wl[c] += dwl[c] * dt;
  *counter += 1;
  if (*counter >= 20) {  // _INTEGRATION_STEPS_PER_ROTATION_PROJECTION (system/rigid_payload.py:11)
    polar3(Rl);
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
