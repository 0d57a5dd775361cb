// dat_qp.hpp -- the reduced agent QP and its interior-point solver (per-lane fp64 device code).
//
// Data placement (DESIGN.md "Register and LDS budget"):
//   QPShared   everything that is the same for all agents of one scenario (u-maps, the packed
//              u-space Hessians, the base rows, the C-ADMM aggregate K).  The C-ADMM / DD kernels
//              keep one copy per scenario in LDS; the centralized kernel keeps it in registers.
//   EnvRows    the agent's env CBF rows (LDS in the C-ADMM / DD kernels).
//   Rt         the agent's U-map hat(r_com) Rl' (LDS in the C-ADMM / DD kernels), read through an
//              accessor at each use.
//   QPLane     the agent's per-solve scalars and linear terms (registers).
//   best       the best iterate seen (lane-private global memory: written, read only on failure).
// Every array the solver keeps in registers is indexed with compile-time indices only (rows are
// fixed slots with an activity mask, loops are unrolled, the LU row exchange is a predicated
// swap), so nothing is demoted to scratch memory.
//
// u = (S, Mo) in R^6: aggregate force and moment about the CoM in payload axes,
//   S = sum_j f_j,  Mo = sum_j hat(r_com_j) Rl' f_j      (control/rqp_cadmm.py:376-392)
// Accelerations are affine in u:
//   dwl = JT^-1 Mo + bw,           bw = -JT^-1 (wl x JT wl)
//   dvl = S/mT + Bv Mo + bv,       Bv = Rl hat(x_com) JT^-1,
//                                  bv = -g e3 - Rl hat(wl)^2 x_com + Rl hat(x_com) bw
// Cone block k (an agent's own force f_k in R^3): f_kz >= min_fz, ||f_k|| <= sec f_kz,
// ||f_k|| <= max_f.  Row slots (affine in (dvl, dwl)):  0 tilt (dwl), 1 |wl| (dwl), 2 |vl| (dvl),
// 3 .. 3+DAT_NENV-1 env CBFs (dvl).  Active env rows are compacted to the front of the env
// slots, so a solve whose rows all fit in NR slots runs the NR-slot instantiation.
#pragma once

#include "dat_core.hpp"

namespace dat {

constexpr int NWROW = 2;          // slots [0, NWROW) act on dwl
constexpr int NBASE = 3;          // base slots shared by all agents of a scenario
// iterative-refinement passes per corrector solve (at most; a pass stops the loop once the linearised
// system is solved to rounding, so well-scaled QPs run one).  Badly scaled agent QPs -- consensus
// multipliers ~1e3-1e4 in a stalled ADMM loop, active rows with barrier weights z/s ~1e15 -- need up to
// six to keep the dual residual below the stopping tolerance (tools/hard_qp_probe.py: 2 passes left
// 281 of 798 such solves at in-band exits, 6 passes 69, all within 1.5e-6 of the oracle)
constexpr int NREF = 6;
// The robust instantiation (stiff rows in augmented form) at most one: on the C4 stall stretches (host build,
// tools/stall_warm_hostsim.py) its warm-started solves ran 4.75 refinement passes and 4.43 corrections per IPM
// iteration with six -- most stop at the cap, the residual of the augmented system does not reach the rounding
// test -- 1.9 / 1.7 with two and 1.0 / 0.9 with one, at about the same IPM iterations per solve (8.5, 8.2) and
// f_des within 1.5e-6 of the oracle.  GPU A/B (tools/r06_ab.sh): the stall stretches alone 48.1 / 36.5 -> 41.6 /
// 33.2 ms per step, the 10 s loop 36.0 -> 33.0 ms per step on average, 0 accepts beyond 1e-8 either way.
constexpr int NREF_ROB = 1;
// Initial point: cone / row slacks shifted to at least IPM_S0 inside, duals IPM_Z0 e.  The agent QPs'
// multipliers are O(1e-2) at the solution; starting the duals and the slack margins there instead of at 1
// takes 7.00 -> 5.23 IPM iterations per C-ADMM agent QP on the C4 closed loop (CPU sweep over
// {0.01, 0.03, 0.1, 0.3, 1, 3, 10}^2, tools/ipm_init_sweep.py; same solutions to the solver tolerance).
constexpr double IPM_S0 = 0.03, IPM_Z0 = 0.03;
constexpr double IPM_ETA = 0.999;  // fraction of the step to the cone boundary (7.00 -> 5.23 -> 4.28 it/QP)
// DD agent QPs: the conservative start.  Round-3 A/B on C3 (IPM it/QP, ms per step against 9.46,
// 20.3 / 20.7): S0 = Z0 = 0.3 -> 9.00, 21.4; 0.1 -> 8.89, 22.0; ETA 0.995 -> 9.29, 20.9; 0.1 and 0.995 ->
// 8.71, 21.8 -- fewer iterations on average, a wider spread across a wavefront.
constexpr double DD_S0 = 1.0, DD_Z0 = 1.0, DD_ETA = 0.99;
// divergence stop (from the 5th iteration): merit above IPM_DIVERGE x the best seen.  A start close to
// the boundary can raise the residuals by 1e3 in its first steps on a well-posed DD QP.
constexpr double IPM_DIVERGE = 1e6;

// Every array starts on a 16-byte boundary and the kernels place the record 16-byte aligned in LDS,
// so the solver reads entry pairs (ldn: one ds_read_b128 per pair).
struct alignas(16) QPShared {
  double C[2][22];       // packed u-space Hessian (21 + pad): [0] without, [1] with the leader's desired-acc terms
  double K[22];          // C-ADMM: sum over ALL agents of U_j U_j' (agent i subtracts its own term)
  double cu[2][6];       // matching linear terms
  double Bv[10], JTi[10];  // 3x3 row-major + pad
  double rows[NBASE][4]; // base rows (a0, a1, a2, b): coefficients on dwl (slots 0, 1) or dvl (slot 2) and
                         // the constant (the affine offsets bw / bv folded in)
  double bv[4], bw[4];
  double inv_mT, pad_;
  int bmask;             // active base slots
  int infeasible;        // a dropped all-zero row had a negative constant
  int pad2_[2];
};
// LDS stride (doubles) of the U-maps Rt_j the C-ADMM / DD kernels keep per agent: 9 + pad, so each
// map starts on a 16-byte boundary (ldn pair reads)
constexpr int RT_STRIDE = 10;

// env CBF rows of one agent (dvl): a . lin_v(u) + b >= 0 (kept in LDS by the kernels)
struct EnvRows {
  double a[DAT_NENV][3], b[DAT_NENV];
};

// Access to solver data kept outside the register file.  get() re-derives the reference through
// an index the compiler cannot see through, so loads are issued where the data is consumed and
// never hoisted out of the IPM loop or merged across uses (hoisting would pin ~150 doubles of
// loop-invariant data in registers and spill the iterates).
template <class T>
struct PlainRef {
  const T* p;
  DAT_HD const T& get() const { return *p; }
};
// LDS records are read through volatile address_space(3) pointers computed once, outside the
// solver loops: every use is a ds_read with an immediate offset at the point of use (the compiler
// may not hoist, merge or cache a volatile load), costing no register between uses and no address
// arithmetic.
template <class T>
__device__ inline const DAT_LDS T* lds_opaque(const DAT_LDS T* p) {
  __asm__ volatile("" : "+v"(p));
  return p;
}
template <class T>
struct LdsRef {
  const volatile DAT_LDS T* p;
  __device__ LdsRef(const T* b, int idx) : p((const volatile DAT_LDS T*)(b + idx)) {}
  __device__ const volatile DAT_LDS T& get() const { return *p; }
};
// env-row accessors: a(j, c), b(j) of env slot j
struct EnvPlain {
  const EnvRows* p;
  DAT_HD double a(int j, int c) const { return p->a[j][c]; }
  DAT_HD double b(int j) const { return p->b[j]; }
  DAT_HD void a3(int j, double* o) const { o[0] = p->a[j][0]; o[1] = p->a[j][1]; o[2] = p->a[j][2]; }
  DAT_HD void ab(int j, double* o, double& bb) const { a3(j, o); bb = p->b[j]; }
};
// LDS image of the env rows of a 64-lane wavefront, pairs structure of arrays: env slot j is two
// pair fields, (a_j0, a_j1) and (a_j2, b_j), each 64 lanes x 16 bytes, so a lane reads a row with two
// ds_read_b128 and a wavefront reading one field touches 1 KB of consecutive LDS (conflict free):
//   field 2 j + h of lane l at doubles [(2 j + h) * 128 + 2 l, +1].
__host__ __device__ constexpr int env_lds_doubles(int NE) { return 4 * NE * 64; }
constexpr int ENV_LDS_DOUBLES = env_lds_doubles(DAT_NENV);
DAT_HD constexpr int env_lds_index(int j, int c, int lane) { return (2 * j + (c >> 1)) * 128 + 2 * lane + (c & 1); }
template <int NE>
struct EnvLdsN {
  const DAT_LDS double* p;  // the lane's pair column
  __device__ EnvLdsN(const double* b, int lane) : p((const DAT_LDS double*)(b + 2 * lane)) {}
  __device__ dat_d2 field(int f) const { return ((const volatile DAT_LDS dat_d2*)p)[f * 64]; }
  __device__ double a(int j, int c) const { return ((const volatile DAT_LDS double*)p)[env_lds_index(j, c, 0)]; }
  __device__ double b(int j) const { return ((const volatile DAT_LDS double*)p)[env_lds_index(j, 3, 0)]; }
  __device__ void a3(int j, double* o) const {
    const dat_d2 f0 = field(2 * j), f1 = field(2 * j + 1);
    o[0] = f0.x; o[1] = f0.y; o[2] = f1.x;
  }
  __device__ void ab(int j, double* o, double& bb) const {
    const dat_d2 f0 = field(2 * j), f1 = field(2 * j + 1);
    o[0] = f0.x; o[1] = f0.y; o[2] = f1.x;
    bb = f1.y;
  }
};
using EnvLds = EnvLdsN<DAT_NENV>;
// the first NE slots of E (set_env_rows compacts the active rows to the front)
template <int NE = DAT_NENV>
DAT_HD void env_to_lds(double* base, int lane, const EnvRows& E) {
#pragma unroll
  for (int j = 0; j < NE; ++j) {
#pragma unroll
    for (int c = 0; c < 3; ++c) base[env_lds_index(j, c, lane)] = E.a[j][c];
    base[env_lds_index(j, 3, lane)] = E.b[j];
  }
}

// U-map accessors: get(k) -> Rt_k (9 doubles, row-major) of cone block k
struct RtPtr {
  const double* p;  // NB x 9
  DAT_HD const double* get(int k) const { return p + 9 * k; }
};
struct RtLds {
  const volatile DAT_LDS double* p;  // block 0
  __device__ RtLds(const double* b, int off) : p((const volatile DAT_LDS double*)(b + off)) {}
  __device__ const volatile DAT_LDS double* get(int k) const { return p + RT_STRIDE * k; }
};

template <int NB>
struct QPLane {
  int var;                       // C / cu variant
  unsigned emask;                // active env slots (compacted: bits 0 .. k-1)
  int infeasible;
  int tuned;                     // C-ADMM: first ADMM pass of the step (tuned IPM start, see ipm_solve)
  double kappa, rho, min_fz, max_f, sec;
  double a2;                     // C-ADMM: sum_{j != i} ||a_j||^2 (objective constant of the free blocks)
  double q[NB][3];               // per-block linear term
  double atil[6];                // C-ADMM: sum_{j != i} U_j a_j
  double cw[6];                  // DD: linear cost on w = (F_i, M_i)
};

// row slots an IPM instantiation must cover for a lane whose env mask is emask
DAT_HD int rows_needed(unsigned emask) { return NBASE + (emask ? 32 - __builtin_clz(emask) : 0); }

// Stiff rows: a row slot whose barrier weight z/s exceeds IPM_STIFF_W is kept out of the normal-equation
// matrix M and solved in augmented (quasi-definite) form, at most IPM_NSTIFF per solve (see ipm_attempt)
constexpr double IPM_STIFF_W = 1e12;
constexpr int IPM_NSTIFF = 8;

// size (doubles) of the lane-private best-iterate record: y (3 NB), w (6), pi (6), u (6) (best_rec: all a
// non-robust instantiation touches, the stride k_cadmm, DD and centralized index with) plus, behind it, the
// robust instantiation's stiff-row scratch of an iteration (ipm_attempt): per stiff row j a column
// H abar_j = (dy (3 NB), dw (6), du (6)), the row (a (3), on-dwl flag, s / z), its right-hand side g and
// dual direction dz (and a temporary); the Cholesky factor of the Schur complement (packed lower, reciprocal diagonal)
DAT_HD constexpr int best_rec(int NB) { return 3 * NB + 18; }
DAT_HD constexpr int stiff_col(int NB) { return 3 * NB + 12; }
constexpr int STIFF_ROW = 8;  // a0 a1 a2 on_dwl e g dz tmp
// (and, last, FM_DOUBLES for the warm-start instantiation's u-space factor P: ipm_attempt WS)
constexpr int FM_DOUBLES = 21;
DAT_HD constexpr int best_size(int NB) {
  return best_rec(NB) + IPM_NSTIFF * (stiff_col(NB) + STIFF_ROW) + IPM_NSTIFF * (IPM_NSTIFF + 1) / 2 + FM_DOUBLES;
}
// Clarabel's own tolerance: an in-band exit whose merit is above it is one Clarabel would not certify
constexpr double IPM_CLARABEL_TOL = 1e-8;

// Warm start (start 3, ipm_solve WS): the previous ADMM pass's last iterate of the same agent QP (of a converged,
// stall-exited or in-band OPTIMAL solve), in a lane record of WREC_SIZE doubles -- [0] valid flag, y (3), w (6),
// cone slacks (9) and duals (9), the row slacks and duals (DAT_MAXROW each) -- pushed back into the interior so
// that every complementarity pair's product is at least WS_MU (a pair (s, z) below it moves to (s + d, z + d); a
// second-order cone pair by its margins s0 - |s1:3|, z0 - |z1:3|), and solved by the robust instantiation (the
// stall's active rows carry barrier weights of 1e10 and more from the first iteration).  The attempt is capped at
// WS_MAXIT iterations; one that does not end cleanly goes on to the cold starts.  Host build, C4 stall stretches
// (2 x 20 HL steps of 101-pass stalls, tools/stall_warm_hostsim.py): the critical path (the slowest agent QP of
// every pass) 25-32 IPM iterations per pass cold, ~10 warm; f_des within 2.2e-6 of the oracle where it is
// reproducible.  WS_MU in 1e-2 .. 1e3 measured alike (42-49 k critical iterations over the stretches); 1e2 has
// the smallest f_des difference.
constexpr double WS_MU = 1e2;
constexpr int WS_MAXIT = 30;
// the DD agent QPs' warm-start floor (dat.hip DD_WARM_PASS): better scaled than a stalled C-ADMM loop's, they take
// a far smaller push (C3: 1e2 19.0, 1e0 14.0, 1e-2 11.2, 1e-3 10.7, 1e-4 11.0 ms per step warm from pass 1)
constexpr double DD_WS_MU = 1e-3;
// stall exit of the tail kernel's solves (ipm_attempt WS): best in-band merit <= WS_STALL_TOL and not halved
// in WS_STALL_ITS iterations
constexpr double WS_STALL_TOL = 1e-9;
// (WS_STALL_ITS 3 -> 2: stall fixture 39.7 / 30.1 -> 37.7 / 29.5 ms per stalled step, same-call A/B, f_des and ADMM
// counts against the oracle unchanged.  1 measured 35.4 / 29.1 but left the host build of the second stall stretch
// 3.2e-5 off the oracle at step 5, beyond its 1.8e-5 bound (test_hostsim); WS_STALL_TOL 3e-9 and WS_MAXIT 15 measured
// no faster)
constexpr int WS_STALL_ITS = 2;
constexpr int WREC_SIZE = 28 + 2 * DAT_MAXROW;
// The tail rule of the C-ADMM closed loop with a forest: ADMM pass p of a scenario's control step solves its
// agent QPs with the warm start and the stall exit exactly when p >= 1 and (the scenario's previous step took more
// than TAIL_PREV passes -- it is wedged in a stall, where every step is the reference loop's 101-pass max_iter
// stall, control/rqp_cadmm.py:661 -- or p >= TAIL_PASS).  The GPU runs those passes in k_cadmm_tail (dat.hip).
// The rule depends on the scenario's own history only, so its results do not depend on the scenarios it is
// batched with.  Normal C4 steps take 1-14 passes: the warm closed loop never meets it.
// (TAIL_PASS = 8 measured worse: the warm window's 9-14-pass scenarios then finish after k_cadmm, C4 3.87 -> 4.58
// ms per step, and the 10 s loop did not gain, 33.0 -> 34.0 ms per step; tools/r06_ab.sh)
constexpr int TAIL_PREV = 20, TAIL_PASS = 16;

// ------------------------------------------------------------------ shared data
// k_f, k_m: total force / moment weights; variants: bit 0 build C[0] (kdv = 0), bit 1 build C[1]
// (kdv = 1).  with_K: C-ADMM aggregate over all agents.
// Not inlined: the drains call it from two sites (a slot's new scenario, and a fused next step,
// dat_control_steps), and one compiled body keeps the two bitwise identical (inlined copies may contract
// multiply-adds differently).  Once per scenario and step: the call costs nothing measurable.
__host__ __device__ inline __attribute__((noinline)) void build_shared(QPShared& S, const double* prm, int n,
                                                                        const double* st, const double* acc,
                                                                        double k_f, double k_m, int variants,
                                                                        bool with_K) {
  const double mT = prm[DAT_P_MT];
  const double* xc = prm + DAT_P_XCOM;
  const double* JT = prm + DAT_P_JT;
  const double* JTi = prm + DAT_P_JTI;
  const double* Rl = st + DAT_S_RL(n);
  const double* wl = st + DAT_S_WL(n);
  const double* vl = st + DAT_S_VL(n);
  S.inv_mT = 1.0 / mT;
  for (int i = 0; i < 9; ++i) S.JTi[i] = JTi[i];
  double Xh[9], RX[9];
  skew3(xc, Xh);
  mm3(Rl, Xh, RX);              // Rl hat(x_com)
  mm3(RX, JTi, S.Bv);           // Rl hat(x_com) JT^-1
  double Jw[3], wJw[3], bw[3], bv[3];
  mv3(JT, wl, Jw);
  cross3(wl, Jw, wJw);
  mv3(JTi, wJw, bw);            // c_w = JT^-1 (wl x JT wl)
  bw[0] = -bw[0]; bw[1] = -bw[1]; bw[2] = -bw[2];
  // bv = -g e3 - Rl hat(wl)^2 x_com + Rl hat(x_com) bw
  double wx[3], wwx[3], t1[3], t2[3];
  cross3(wl, xc, wx);
  cross3(wl, wx, wwx);
  mv3(Rl, wwx, t1);
  mv3(RX, bw, t2);
  bv[0] = -t1[0] + t2[0];
  bv[1] = -t1[1] + t2[1];
  bv[2] = -DAT_GRAVITY - t1[2] + t2[2];
  for (int c = 0; c < 3; ++c) { S.bw[c] = bw[c]; S.bv[c] = bv[c]; }
  S.bw[3] = S.bv[3] = 0.0;
  S.Bv[9] = S.JTi[9] = 0.0;
  S.pad_ = 0.0;

  // Phi(u) = k_f ||S - mT g e3||^2 + k_m ||Mo||^2 + kdv (||dvl||^2 - 2 dvl_des'dvl)
  //          + kdv (||dwl||^2 - 2 dwl_des'dwl)          (control/rqp_cadmm.py:436-458)
  for (int v = 0; v < 2; ++v) {
    if (!((variants >> v) & 1)) continue;
    double* C = S.C[v];
    double* cu = S.cu[v];
    for (int k = 0; k < 22; ++k) C[k] = 0.0;
    for (int r = 0; r < 3; ++r) { C[sp6(r, r)] = 2.0 * k_f; C[sp6(3 + r, 3 + r)] = 2.0 * k_m; }
    for (int r = 0; r < 6; ++r) cu[r] = 0.0;
    cu[2] = -2.0 * k_f * mT * DAT_GRAVITY;
    if (v == 1) {
      // Av = [I/mT, Bv], Aw = [0, JTi]: C += 2 (Av'Av + Aw'Aw)
      const double im = S.inv_mT;
      for (int r = 0; r < 3; ++r) {
        C[sp6(r, r)] += 2.0 * im * im;
        for (int c = 0; c < 3; ++c) C[sp6(r, 3 + c)] += 2.0 * im * S.Bv[3 * r + c];
      }
      for (int r = 0; r < 3; ++r)
        for (int c = r; c < 3; ++c) {
          double s = 0.0;
          for (int k = 0; k < 3; ++k) s += S.Bv[3 * k + r] * S.Bv[3 * k + c] + JTi[3 * k + r] * JTi[3 * k + c];
          C[sp6(3 + r, 3 + c)] += 2.0 * s;
        }
      double ev[3] = {bv[0] - acc[0], bv[1] - acc[1], bv[2] - acc[2]};
      double ew[3] = {bw[0] - acc[3], bw[1] - acc[4], bw[2] - acc[5]};
      double t[3], s3[3];
      mtv3(S.Bv, ev, t);
      mtv3(JTi, ew, s3);
      for (int r = 0; r < 3; ++r) {
        cu[r] += 2.0 * im * ev[r];
        cu[3 + r] += 2.0 * (t[r] + s3[r]);
      }
    }
  }
  if (with_K) {
    for (int k = 0; k < 22; ++k) S.K[k] = 0.0;
    const double I3[6] = {1, 0, 0, 1, 0, 1};
    for (int j = 0; j < n; ++j) {
      double Rt[9];
      make_Rt(prm + DAT_P_RCOM(n) + 3 * j, Rl, Rt);
      add_UDUt(S.K, Rt, I3, 1.0);
    }
  }

  // base rows (control/rqp_cadmm.py:406-430).  Tilt: (Rl hat(wl))[2,2] = Rl[2,:].(wl x e3),
  // (Rl hat(wl)^2)[2,2] = Rl[2,:].(wl x (wl x e3)).
  S.bmask = 0;
  S.infeasible = 0;
  double e3[3] = {0, 0, 1}, a[3], b[3];
  cross3(wl, e3, a);
  cross3(wl, a, b);
  double al[NBASE][3] = {{-Rl[7], Rl[6], 0.0},
                         {-2.0 * wl[0], -2.0 * wl[1], -2.0 * wl[2]},
                         {-2.0 * vl[0], -2.0 * vl[1], -2.0 * vl[2]}};
  double beta[NBASE] = {dot3(Rl + 6, b) + 2.0 * dot3(Rl + 6, a) + (Rl[8] - prm[DAT_P_COSP]),
                        prm[DAT_P_MAXWL2] - dot3(wl, wl), prm[DAT_P_MAXVL2] - dot3(vl, vl)};
  for (int l = 0; l < NBASE; ++l) {
    for (int c = 0; c < 3; ++c) S.rows[l][c] = al[l][c];
    if (al[l][0] == 0.0 && al[l][1] == 0.0 && al[l][2] == 0.0) {
      if (beta[l] < 0.0) S.infeasible = 1;  // 0 >= -beta fails: the QP is infeasible
      S.rows[l][3] = 1.0;                   // 0 >= 0 carries no information: padding row
      continue;
    }
    S.rows[l][3] = beta[l] + dot3(al[l], l < NWROW ? bw : bv);
    S.bmask |= 1 << l;
  }
}

// env rows (dvl): lhs . dvl >= rhs  <=>  lhs . lin_v(u) + (lhs . bv - rhs) >= 0.  Rows the
// reference would emit are compacted to the front of the slots (P.emask = bits 0 .. k-1); a row
// with lhs = 0 carries no information and is dropped (infeasible if its constant is negative).
// Slot writes are predicated on compile-time indices so a register-resident E stays in registers.
template <int NB>
DAT_HD void set_env_rows(QPLane<NB>& P, EnvRows& E, const QPShared& S, unsigned mask, const double lhs[DAT_NENV][3],
                         const double rhs[DAT_NENV]) {
  P.infeasible = 0;
#pragma unroll
  for (int j = 0; j < DAT_NENV; ++j) {
    // inactive slots hold the padding row 0 . x + 1 >= 0
    E.a[j][0] = 0.0; E.a[j][1] = 0.0; E.a[j][2] = 0.0;
    E.b[j] = 1.0;
  }
  int k = 0;
#pragma unroll
  for (int j = 0; j < DAT_NENV; ++j) {
    const bool on = (mask >> j) & 1u;
    // a row whose coefficients vanish against its constant (|lhs| <= 1e-12 |rhs|: a rounding remnant, it would
    // need accelerations beyond 1e12 to bind) is a zero row
    const bool zero = lhs[j][0] * lhs[j][0] + lhs[j][1] * lhs[j][1] + lhs[j][2] * lhs[j][2] <= 1e-24 * rhs[j] * rhs[j];
    if (on && zero && -rhs[j] < 0.0) P.infeasible = 1;
    if (!on || zero) continue;
    const double bj = -rhs[j] + dot3(lhs[j], S.bv);
#pragma unroll
    for (int s = 0; s <= j; ++s) {
      if (s == k) {
        E.a[s][0] = lhs[j][0]; E.a[s][1] = lhs[j][1]; E.a[s][2] = lhs[j][2];
        E.b[s] = bj;
      }
    }
    ++k;
  }
  P.emask = (1u << k) - 1u;
}

// Certified infeasibility of an agent QP's dvl rows (the |vl| base row, slot 2, and the env rows): a . x + b >= 0
// with x = lin_v(u) in R^3.  In the C-ADMM (and DD) agent QP the aggregate w is free, so u is free and the QP is
// infeasible exactly when its row system is (the cone block alone is feasible; the two dwl rows act on another
// coordinate of u).  By Helly's theorem an empty intersection of half-spaces in R^3 has an empty subsystem of at
// most 4 rows, and one of at most 3 when their normals lie in a plane (the env rows of vertical trees are
// horizontal): a Farkas certificate lambda >= 0, sum_m lambda_m a_m = 0, sum_m lambda_m b_m < 0, with lambda the
// signed cofactors of the subsystem -- two antiparallel normals, three coplanar ones (scalar cross products in
// their plane) or four that positively span R^3 (3 x 3 determinants).  Only strict certificates count: lambda of
// one sign with every entry above 1e-9 of their sum, and a violation beyond 1e-6 of the rows' scale; anything
// closer is left to the IPM, so a certified QP is one whose residuals the IPM cannot bring into band either, and
// one Clarabel reports infeasible (the reference then holds the previous solution, control/rqp_cadmm.py:496-499).
// At most C(11, 2) + C(11, 3) + C(11, 4) = 550 subsystems: the tail kernel runs it once per scenario and step
// (an infeasible agent QP otherwise runs 2 x 50 IPM iterations in every ADMM pass of a stall).
template <class SH, class ER>
DAT_HD bool dvl_rows_infeasible(const SH& sh, const ER& er, unsigned emask) {
  const int ne = __builtin_popcount(emask);  // active env rows: slots 0 .. ne - 1 (set_env_rows compacts them)
  const bool vrow = (sh.get().bmask >> 2) & 1;
  const int m = ne + (vrow ? 1 : 0);
  auto row = [&](int k, double* a, double& b) {
    if (vrow && k == ne) {
      double r4[4];
      ldn<4>(sh.get().rows[2], r4);
      a[0] = r4[0]; a[1] = r4[1]; a[2] = r4[2];
      b = r4[3];
    } else {
      er.ab(k, a, b);
    }
  };
  auto nrm = [](const double* a) { return sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); };
  // lambda (of one sign, normalised positive) certifies infeasibility
  auto cert = [](int q, const double* lam, const double* bb, const double* na) -> bool {
    double sg = lam[0] < 0.0 ? -1.0 : 1.0, tot = 0.0;
    for (int t = 0; t < q; ++t) tot += fabs(lam[t]);
    double lb = 0.0, sc = 0.0;
    for (int t = 0; t < q; ++t) {
      const double l = sg * lam[t];
      if (!(l > 1e-9 * tot)) return false;
      lb += l * bb[t];
      sc += l * (fabs(bb[t]) + na[t]);
    }
    return lb < -1e-6 * sc;
  };
  bool inf = false;
#pragma unroll 1
  for (int i = 0; i < m - 1; ++i) {
    double a1[3], b1;
    row(i, a1, b1);
    const double n1 = nrm(a1);
#pragma unroll 1
    for (int j = i + 1; j < m; ++j) {
      double a2[3], b2, c12[3];
      row(j, a2, b2);
      const double n2 = nrm(a2);
      cross3(a1, a2, c12);
      const double nc12 = nrm(c12);
      if (nc12 <= 1e-9 * n1 * n2 && dot3(a1, a2) < 0.0) {  // antiparallel pair
        const double lam[2] = {n2, n1}, bb[2] = {b1, b2}, na[2] = {n1, n2};
        inf = inf || cert(2, lam, bb, na);
      }
#pragma unroll 1
      for (int k = j + 1; k < m; ++k) {
        double a3[3], b3, c23[3], c31[3];
        row(k, a3, b3);
        const double n3 = nrm(a3);
        cross3(a2, a3, c23);
        cross3(a3, a1, c31);
        const double l4 = -dot3(c12, a3);  // -det(a1, a2, a3)
        if (fabs(l4) <= 1e-9 * n1 * n2 * n3) {  // coplanar triple: scalar cross products in the plane
          const double* nv = c12;
          if (nrm(c23) > nrm(nv)) nv = c23;
          if (nrm(c31) > nrm(nv)) nv = c31;
          const double lam[3] = {dot3(nv, c23), dot3(nv, c31), dot3(nv, c12)}, bb[3] = {b1, b2, b3},
                       na[3] = {n1, n2, n3};
          inf = inf || cert(3, lam, bb, na);
        }
#pragma unroll 1
        for (int l = k + 1; l < m; ++l) {
          double a4[3], b4, c34[3];
          row(l, a4, b4);
          cross3(a3, a4, c34);
          const double lam[4] = {dot3(a2, c34), -dot3(a1, c34), dot3(c12, a4), l4}, bb[4] = {b1, b2, b3, b4},
                       na[4] = {n1, n2, n3, nrm(a4)};
          inf = inf || cert(4, lam, bb, na);
        }
      }
    }
  }
  return inf;
}

// ------------------------------------------------------------------ per-agent data
template <int NB>
DAT_HD void lane_common(QPLane<NB>& P, const double* prm) {
  P.min_fz = prm[DAT_P_MINFZ];
  P.max_f = prm[DAT_P_MAXF];
  P.sec = prm[DAT_P_SEC];
  P.emask = 0u;
  P.infeasible = 0;
  P.tuned = 0;
#pragma unroll
  for (int r = 0; r < 6; ++r) { P.atil[r] = 0.0; P.cw[r] = 0.0; }
  P.rho = 1.0;
  P.a2 = 0.0;
}

// C-ADMM agent i (control/rqp_cadmm.py:26-501): variables f in R^{3 x n} (agent i's full copy).
// Cost: Phi(u) with k = 0.1/n, k_feq ||f_i - f_eq_i||^2, leader terms, <lam, f> + rho/2 ||f||^2
// - <rho fbar, f>  ==  rho/2 ||f - a||^2 + const with a = fbar - lam / rho.
// Only f_i carries cones; f_j (j != i) are free and eliminated through (K, atil).
DAT_HD void lane_cadmm_static(QPLane<1>& P, const double* prm, int i) {
  lane_common(P, prm);
  P.var = (i == 0) ? 1 : 0;
}
// per-iteration part: penalty rho and a = fbar - lam / rho.  lam, fbar: (3n) agent-major;
// Rt_all: n x 9.
DAT_HD void lane_cadmm_dynamic(QPLane<1>& P, const double* prm, int n, int i, const double* Rt_all,
                               const double* lam, const double* fbar, double rho, int rt_stride = 9) {
  const double kfeq = prm[DAT_P_KFEQ];
  const double irho = 1.0 / rho;
  P.rho = rho;
  P.kappa = 2.0 * kfeq + rho;
  const double* feq = prm + DAT_P_FEQ(n) + 3 * i;
#pragma unroll
  for (int r = 0; r < 6; ++r) P.atil[r] = 0.0;
  double a2 = 0.0;
  for (int j = 0; j < n; ++j) {
    double a[3] = {fbar[3 * j] - lam[3 * j] * irho, fbar[3 * j + 1] - lam[3 * j + 1] * irho,
                   fbar[3 * j + 2] - lam[3 * j + 2] * irho};
    if (j == i) {
#pragma unroll
      for (int c = 0; c < 3; ++c) P.q[0][c] = -2.0 * kfeq * feq[c] - rho * a[c];
    } else {
      double t[6];
      U_apply(Rt_all + rt_stride * j, a, t);
#pragma unroll
      for (int r = 0; r < 6; ++r) P.atil[r] += t[r];
      a2 += a[0] * a[0] + a[1] * a[1] + a[2] * a[2];
    }
  }
  P.a2 = a2;
}
// agent i's copy of agent j != i: f_j = a_j - U_j' pi / rho  (stationarity of the free blocks)
DAT_HD void cadmm_free_block(const double* Rt_j, const double* lam_j, const double* fbar_j, const double* pi,
                             double rho, double* f_j) {
  double t[3];
  Ut_apply(Rt_j, pi, t);
  const double irho = 1.0 / rho;
#pragma unroll
  for (int c = 0; c < 3; ++c) f_j[c] = fbar_j[c] - (lam_j[c] + t[c]) * irho;
}

// DD agent i (control/rqp_dd.py:27-505): variables (f_i, F_i, M_i); with w = (F_i, M_i),
// u = U_i f_i + w.  Cost Phi(u) + k_feq ||f_i - f_eq_i||^2 + c_fi'f_i + (c_Fi, c_Mi)'w.
DAT_HD void lane_dd_static(QPLane<1>& P, const double* prm, int i) {
  lane_common(P, prm);
  P.var = (i == 0) ? 1 : 0;
  P.kappa = 2.0 * prm[DAT_P_KFEQ];
}
// prices c = (c_fi, c_Fi, c_Mi) (control/rqp_dd.py:718-722)
DAT_HD void set_dd_price(QPLane<1>& P, const double* prm, int n, int i, const double* c9) {
  const double* feq = prm + DAT_P_FEQ(n) + 3 * i;
  const double kfeq = prm[DAT_P_KFEQ];
#pragma unroll
  for (int c = 0; c < 3; ++c) P.q[0][c] = -2.0 * kfeq * feq[c] + c9[c];
#pragma unroll
  for (int r = 0; r < 6; ++r) P.cw[r] = c9[3 + r];
}

// Centralized (control/rqp_centralized.py:27-448): all n agents' forces, k = 0.1, leader terms on.
// Rt (NB x 9) receives the U-maps of every block.
template <int NB>
DAT_HD void lane_cent(QPLane<NB>& P, const double* prm, int n, const double* st, double Rt[NB][9]) {
  lane_common(P, prm);
  P.var = 1;
  const double kfeq = prm[DAT_P_KFEQ];
  const double* Rl = st + DAT_S_RL(n);
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const double* feq = prm + DAT_P_FEQ(n) + 3 * k;
    make_Rt(prm + DAT_P_RCOM(n) + 3 * k, Rl, Rt[k]);
#pragma unroll
    for (int c = 0; c < 3; ++c) P.q[k][c] = -2.0 * kfeq * feq[c];
  }
  P.kappa = 2.0 * kfeq;
}

// =====================================================================================
// interior-point method on the reduced problem
// =====================================================================================
// Per cone block: slack/dual layout [fz | soc1 (4) | soc2 (4)] (9 entries),
//   s = h - G y,  G y = -(y2, sec y2, y0, y1, y2, 0, y0, y1, y2),  h = (-min_fz, 0,0,0,0, max_f, 0,0,0).
// Cone blocks use Nesterov-Todd scaling; the LP rows (u-slots) are carried unscaled (for the
// nonnegative orthant NT scaling is diagonal and the two forms are algebraically identical).
struct SocScale {
  double w0, w1, w2, w3, eta, ieta, k1;  // k1 = 1 / (1 + w0)
};

DAT_HD double soc_det(const double* v) {
  double n1 = sqrt(v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
  return (v[0] - n1) * (v[0] + n1);
}
DAT_HD bool soc_scaling(const double* s, const double* z, SocScale& S) {
  double ds = soc_det(s), dz = soc_det(z);
  if (!(ds > 0) || !(dz > 0)) return false;
  double sn = sqrt(ds), zn = sqrt(dz);
  double isn = frcp(sn), izn = frcp(zn);
  double s0 = s[0] * isn, s1 = s[1] * isn, s2 = s[2] * isn, s3 = s[3] * isn;
  double z0 = z[0] * izn, z1 = z[1] * izn, z2 = z[2] * izn, z3 = z[3] * izn;
  double g = sqrt(0.5 * (1.0 + s0 * z0 + s1 * z1 + s2 * z2 + s3 * z3));
  double ig = 0.5 * frcp(g);
  S.w0 = (s0 + z0) * ig;
  S.w1 = (s1 - z1) * ig;
  S.w2 = (s2 - z2) * ig;
  S.w3 = (s3 - z3) * ig;
  S.eta = sqrt(sn * izn);
  S.ieta = frcp(S.eta);
  S.k1 = frcp(1.0 + S.w0);
  return true;
}
// o = W v (inv = false) or W^-1 v (inv = true); W = eta H(w), W^-1 = H(Jw)/eta
DAT_HD void soc_apply(const SocScale& S, const double* v, double* o, bool inv) {
  const double sg = inv ? -1.0 : 1.0;
  const double w1 = sg * S.w1, w2 = sg * S.w2, w3 = sg * S.w3;
  const double wv = w1 * v[1] + w2 * v[2] + w3 * v[3];
  const double k = v[0] + wv * S.k1;
  const double sc = inv ? S.ieta : S.eta;
  const double o0 = S.w0 * v[0] + wv;
  o[1] = sc * (v[1] + k * w1);
  o[2] = sc * (v[2] + k * w2);
  o[3] = sc * (v[3] + k * w3);
  o[0] = sc * o0;
}
// x = lam \ y (inverse Jordan product) for a 4-dim SOC
DAT_HD void soc_jdiv(const double* l, const double* y, double* x) {
  double det = l[0] * l[0] - (l[1] * l[1] + l[2] * l[2] + l[3] * l[3]);
  double x0 = (l[0] * y[0] - (l[1] * y[1] + l[2] * y[2] + l[3] * y[3])) * frcp(det);
  double il0 = frcp(l[0]);
  x[0] = x0;
  x[1] = (y[1] - x0 * l[1]) * il0;
  x[2] = (y[2] - x0 * l[2]) * il0;
  x[3] = (y[3] - x0 * l[3]) * il0;
}
DAT_HD void soc_jprod(const double* a, const double* b, double* o) {
  double d = a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
  o[1] = a[0] * b[1] + b[0] * a[1];
  o[2] = a[0] * b[2] + b[0] * a[2];
  o[3] = a[0] * b[3] + b[0] * a[3];
  o[0] = d;
}
// largest step a with x + a d in the SOC (1e300 if unbounded)
DAT_HD double soc_step(const double* x, const double* d) {
  double a = d[0] * d[0] - (d[1] * d[1] + d[2] * d[2] + d[3] * d[3]);
  double b = x[0] * d[0] - (x[1] * d[1] + x[2] * d[2] + x[3] * d[3]);
  double n1 = sqrt(x[1] * x[1] + x[2] * x[2] + x[3] * x[3]);
  double c = (x[0] - n1) * (x[0] + n1);
  double disc = b * b - a * c;
  if (a < 0.0 || (b < 0.0 && disc >= 0.0)) {
    double den = -b + sqrt(fmax(disc, 0.0));
    return den > 0.0 ? c * frcp(den) : 0.0;
  }
  return 1e300;
}

// Per-row IPM state (slack s_l, dual z_l, Newton row term zw_l of each row slot).  RowRegs keeps
// it in registers; RowLds in an LDS image over the 64 lanes of a wavefront: the (s_l, z_l) pair of
// slot l of lane j at doubles [l 128 + 2 j, +1] (one ds_read_b128 / ds_write_b128 per pair; a
// wavefront touches 1 KB of consecutive LDS), zw_l at [2 NR 64 + l 64 + j]; read and written through
// volatile pointers, so the rows cost no registers between uses.  Besides the rows, a store may hold
// NX auxiliary per-lane doubles at [(3 NR + k) 64 + j] (aux slots: the per-iteration quantities
// ipm_solve's AUXM mask moves out of the register file, see ipm_aux_doubles).
struct RowRegs {
  template <int NR, int NX = 0>
  struct Store {
    double s_[NR], z_[NR], w_[NR], x_[NX > 0 ? NX : 1];
    DAT_HD explicit Store(const RowRegs&) {}
    DAT_HD double& s(int l) { return s_[l]; }
    DAT_HD double& z(int l) { return z_[l]; }
    DAT_HD double& w(int l) { return w_[l]; }
    DAT_HD double& x(int k) { return x_[k]; }
    DAT_HD void sz(int l, double& sv, double& zv) { sv = s_[l]; zv = z_[l]; }
    DAT_HD void set_sz(int l, double sv, double zv) { s_[l] = sv; z_[l] = zv; }
  };
};
struct RowLds {
  double* base;
  int lane;
  template <int NR, int NX = 0>
  struct Store {
    DAT_LDS double* p;   // the lane's zw / aux column
    DAT_LDS double* pz;  // the lane's (s, z) pair column
    __device__ explicit Store(const RowLds& r)
        : p((DAT_LDS double*)(r.base + r.lane)), pz((DAT_LDS double*)(r.base + 2 * r.lane)) {}
    __device__ volatile DAT_LDS double& at(int k) { return ((volatile DAT_LDS double*)p)[k * 64]; }
    __device__ volatile DAT_LDS double& s(int l) { return ((volatile DAT_LDS double*)pz)[l * 128]; }
    __device__ volatile DAT_LDS double& z(int l) { return ((volatile DAT_LDS double*)pz)[l * 128 + 1]; }
    __device__ volatile DAT_LDS double& w(int l) { return at(2 * NR + l); }
    __device__ volatile DAT_LDS double& x(int k) { return at(3 * NR + k); }
    __device__ void sz(int l, double& sv, double& zv) {
      const dat_d2 v = ((volatile DAT_LDS dat_d2*)pz)[l * 64];
      sv = v.x;
      zv = v.y;
    }
    __device__ void set_sz(int l, double sv, double zv) {
      dat_d2 v;
      v.x = sv;
      v.y = zv;
      ((volatile DAT_LDS dat_d2*)pz)[l * 64] = v;
    }
  };
};
// Host model of RowLds (the same strided columns in ordinary memory): exercises the aux / row store
// code paths of ipm_solve in the host build (tests/hostsim).
struct RowMem {
  double* base;
  int lane;
  template <int NR, int NX = 0>
  struct Store {
    double* p;
    double* pz;
    DAT_HD explicit Store(const RowMem& r) : p(r.base + r.lane), pz(r.base + 2 * r.lane) {}
    DAT_HD double& at(int k) { return p[k * 64]; }
    DAT_HD double& s(int l) { return pz[l * 128]; }
    DAT_HD double& z(int l) { return pz[l * 128 + 1]; }
    DAT_HD double& w(int l) { return at(2 * NR + l); }
    DAT_HD double& x(int k) { return at(3 * NR + k); }
    DAT_HD void sz(int l, double& sv, double& zv) { sv = s(l); zv = z(l); }
    DAT_HD void set_sz(int l, double sv, double zv) { s(l) = sv; z(l) = zv; }
  };
};
// aux slots of ipm_solve (AUXM bits): SCAL the stopping-rule scales and best merits (4), RES the
// iteration's residuals r_y and R_f (3 NB + 6), LAM the scaled point lambda = W z (9 NB), DINV the
// cone blocks' QR factor of D (qr_cone) and 1 / d0 (7 NB)
constexpr unsigned AUX_SCAL = 1, AUX_RES = 2, AUX_LAM = 4, AUX_DINV = 8;
__host__ __device__ constexpr int ipm_aux_doubles(int NB, unsigned AUXM) {
  return ((AUXM & AUX_SCAL) ? 4 : 0) + ((AUXM & AUX_RES) ? 3 * NB + 6 : 0) + ((AUXM & AUX_LAM) ? 9 * NB : 0) +
         ((AUXM & AUX_DINV) ? 7 * NB : 0);
}
__host__ __device__ constexpr int row_lds_doubles(int NR, int NX = 0) { return (3 * NR + NX) * 64; }  // (s, z) pairs, zw, aux

// Phase profile (development builds only, -DDAT_PHASE_PROF): shader-clock cycles per phase of the
// IPM iteration, summed over wavefronts by the first active lane (tools/phase_prof.py).
#if defined(DAT_PHASE_PROF)
__device__ unsigned long long g_phase[16];
#endif
#if defined(DAT_ITER_HIST)
// IPM iteration histogram of the agent QPs (development builds, tools/iter_hist.py): [iters] solves
__device__ unsigned long long g_iter_hist[64];
#endif
#if defined(DAT_PHASE_PROF) && defined(__HIP_DEVICE_COMPILE__)
struct PhaseClock {
  unsigned long long t0;
  int cur;
  __device__ PhaseClock(int c) : t0(clock64()), cur(c) {}
  __device__ void to(int next) {
    const unsigned long long t = clock64();
    const unsigned long long act = __ballot(1);
    if ((int)__lane_id() == __ffsll((long long)act) - 1) atomicAdd(&g_phase[cur], t - t0);
    t0 = t;
    cur = next;
  }
};
#define DAT_PHASE_INIT(c) PhaseClock pclk_(c)
#define DAT_PHASE(c) pclk_.to(c)
#else
#define DAT_PHASE_INIT(c)
#define DAT_PHASE(c)
#endif

// Refinement statistics (host builds with -DDAT_IPM_STATS only, tools/ipm_stats.py): corrector solves,
// refinement passes run, passes skipped by the rounding-level test.
#if defined(DAT_IPM_STATS) && !defined(__HIP_DEVICE_COMPILE__)
inline long long g_ipm_stats[16];  // [0..2] refinement, [3 + why] non-converged exits, [10] in-band, [11] solves
inline long long g_ipm_hist[3][24];  // [first pass stopped at rounding | correction applied | 2nd pass][log10 max row z/s + 12]
inline double g_maxw;
#define DAT_STAT(k) (++g_ipm_stats[k])
#define DAT_STAT_W(w) (g_maxw = (w) > g_maxw ? (w) : g_maxw)
#define DAT_STAT_H(k)                                                                   \
  do {                                                                                  \
    int b_ = g_maxw > 0 ? (int)floor(log10(g_maxw)) + 12 : 0;                           \
    ++g_ipm_hist[k][b_ < 0 ? 0 : b_ > 23 ? 23 : b_];                                    \
  } while (0)
#else
#define DAT_STAT(k) ((void)0)
#define DAT_STAT_W(w) ((void)0)
#define DAT_STAT_H(k) ((void)0)
#endif

// Cone-block groups.  ipm_solve sums (max, min) its per-block quantities over the blocks a lane
// holds; a group policy extends those reductions over the W lanes of a lane group, so one QP's cone
// blocks can live on W lanes (the centralized QP: one agent's force per lane, dat_cent.hip).  The
// u-space algebra and the row slots are replicated on the group's lanes, so every lane must see
// bit-identical reduced values: the reductions are xor butterflies, whose pairwise sums are computed
// in both orders and IEEE addition / fmax / fmin are commutative.
struct NoGrp {  // one lane holds all blocks of its QP
  static constexpr bool on = false;
  DAT_HD bool act() const { return true; }
  DAT_HD int nblk(int NB) const { return NB; }
  DAT_HD double sum(double x) const { return x; }
  DAT_HD double max(double x) const { return x; }
  DAT_HD double min(double x) const { return x; }
};
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
// x of the lane selected by DPP control CTRL (row-local: a group never reads another group's lanes)
template <int CTRL>
__device__ inline double dpp_d(double x) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(v & 0xffffffffll), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(v >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
// W (4, 8 or 16) lanes, aligned to W: quad_perm xor 1, quad_perm xor 2, row_half_mirror (lane i <-> 7 - i),
// row_mirror (i <-> 15 - i).  Each step combines the lane's partial with its partner group's.
template <int W>
struct GrpDpp {
  static_assert(W == 4 || W == 8 || W == 16, "group width");
  static constexpr bool on = true;
  bool active;  // the lane holds a real block (phantom lanes k >= n contribute nothing)
  int n;        // blocks of the QP
  template <class F>
  __device__ double red(double x, F f) const {
    x = f(x, dpp_d<0xB1>(x));    // quad_perm [1, 0, 3, 2]
    x = f(x, dpp_d<0x4E>(x));    // quad_perm [2, 3, 0, 1]
    if (W >= 8) x = f(x, dpp_d<0x141>(x));   // row_half_mirror
    if (W >= 16) x = f(x, dpp_d<0x140>(x));  // row_mirror
    return x;
  }
  __device__ bool act() const { return active; }
  __device__ int nblk(int) const { return n; }
  __device__ double sum(double x) const { return red(active ? x : 0.0, [](double a, double b) { return a + b; }); }
  __device__ double max(double x) const { return red(active ? x : 0.0, [](double a, double b) { return fmax(a, b); }); }
  __device__ double min(double x) const { return red(active ? x : 1e300, [](double a, double b) { return fmin(a, b); }); }
};
#endif

struct IPMOut {
  int status;
  int iters;
  int inband;     // OPTIMAL through the best in-band iterate of a stalled solve (not converged to tol)
  double merit;   // scaled max(primal residual, dual residual, gap) of the returned iterate
  int why;        // exit: 0 converged, 1 non-finite residuals, 2 divergence / max_iter, 3 cone scaling,
                  // 4 cone block D, 5 Cholesky of M, 6 Cholesky of N
  int refs;       // refinement passes run (residual evaluations of the linearised system)
  int corrs;      // refinement corrections applied (core solves)
  int stiff;      // IPM_ROBUST: stiff rows solved in augmented form in some iteration; IPM_FAST_REDO: redone robustly
  double pi[6];   // u-space gradient C u + cu - A' z_rows at the solution
  double u[6];
};

// Solve the reduced QP. MODE_CADMM: NB = 1, implicit free blocks through (K, atil, rho);
// MODE_DD: NB = 1, w = (F_i, M_i) free with linear cost cw; MODE_CENT: NB = n, no w.
// NR: row slots processed (NBASE .. DAT_MAXROW); every active env row must sit in a slot < NR.
// sh / er / rt: accessors of the scenario data, the env rows and the U-maps; y0: interior initial
// guess (NB x 3, f_eq); best: lane-private record of best_size(NB) doubles.  y (NB x 3) and w (6)
// are outputs.
//
// Register economy (DESIGN.md "Register and LDS budget"): only the iterates (y, w, s, z), the
// per-iteration factors (NT scalings, D^-1, M, LU) and the current Newton direction live in
// registers.  The row loops are branch-free over all NR slots (an inactive slot is the padding
// row 0 . x + 1 >= 0 with z = 0, whose complementarity target is zeroed, so it never moves and
// adds exactly nothing); row reciprocals, primal residuals and the corrector's second-order row
// terms are recomputed where consumed instead of being kept live.
// ROB: the robust instantiation (stiff rows in augmented form, below).
template <int MODE, int NB, int NR, class SH, class ER, class RT, class RW, unsigned AUXM, class GRP, bool ROB,
          bool WS = false>
DAT_HD __attribute__((always_inline)) IPMOut ipm_attempt(const SH& sh, const ER& er, const RT& rt, const QPLane<NB>& P,
                                                          const double* y0,
                          double y[NB][3], double w[6], double* best, int max_iter, double tol, RW rw, GRP grp,
                          int start, double* wrec = nullptr, bool wson = false, int clone = 0, int nclone = 1) {
  static_assert(NR >= NBASE && NR <= DAT_MAXROW, "row slots");
  // aux slot offsets (only the AUXM groups are allocated)
  constexpr int O_SC = 0;
  constexpr int O_RK = O_SC + ((AUXM & AUX_SCAL) ? 4 : 0);
  constexpr int O_RF = O_RK + 3 * NB;
  constexpr int O_LAM = O_RK + ((AUXM & AUX_RES) ? 3 * NB + 6 : 0);
  constexpr int O_DI = O_LAM + ((AUXM & AUX_LAM) ? 9 * NB : 0);
  constexpr int O_ID0 = O_DI + 6 * NB;
  constexpr int NX = ipm_aux_doubles(NB, AUXM);
  IPMOut out;
  out.status = ST_FAILED;
  out.iters = 0;
  out.inband = 0;
  out.why = 0;
  out.refs = 0;
  out.corrs = 0;
  out.stiff = 0;
  out.merit = 1e300;
#pragma unroll
  for (int r = 0; r < 6; ++r) { out.pi[r] = 0.0; out.u[r] = 0.0; }
  if (sh.get().infeasible || P.infeasible) {
    out.status = ST_INFEASIBLE;
    return out;
  }
  const unsigned emask = P.emask << NBASE;
  if (emask >> NR) return out;  // an active row outside the instantiated slots: caller error
  const unsigned mask = (unsigned)sh.get().bmask | emask;
  const int var = P.var;
  const double sec = P.sec, kap = P.kappa;
  const double irho = 1.0 / P.rho;
  const double im = sh.get().inv_mT;
  auto act = [&](int l) -> double { return ((mask >> l) & 1u) ? 1.0 : 0.0; };
  auto Cp = [&]() { return &sh.get().C[var][0]; };
  auto cup = [&]() { return &sh.get().cu[var][0]; };
  auto rb = [&](int l) -> double { return l < NBASE ? sh.get().rows[l < NBASE ? l : 0][3] : er.b(l >= NBASE ? l - NBASE : 0); };
  // row coefficients a_l (base rows: two pair reads of the (a, b) record)
  auto ra3 = [&](int l, double* a) {
    if (l < NBASE) {
      double r4[4];
      ldn<4>(sh.get().rows[l < NBASE ? l : 0], r4);
      a[0] = r4[0]; a[1] = r4[1]; a[2] = r4[2];
    } else {
      er.a3(l >= NBASE ? l - NBASE : 0, a);
    }
  };
  // row value a_l . (dvl or dwl) of the linear map of u
  auto rowdot = [&](int l, const double* dv, const double* dw) -> double {
    const double* x = l < NWROW ? dw : dv;
    double a[3];
    ra3(l, a);
    return a[0] * x[0] + a[1] * x[1] + a[2] * x[2];
  };
  // coefficients and constant of row l in one visit (base rows: two pair reads of the (a, b) record;
  // env rows: two pair fields)
  auto rowld = [&](int l, double* a, double& b) {
    if (l < NBASE) {
      double r4[4];
      ldn<4>(sh.get().rows[l < NBASE ? l : 0], r4);
      a[0] = r4[0]; a[1] = r4[1]; a[2] = r4[2];
      b = r4[3];
    } else {
      er.ab(l >= NBASE ? l - NBASE : 0, a, b);
    }
  };
  auto dot3x = [&](int l, const double* a, const double* v, const double* w) -> double {
    const double* x = l < NWROW ? w : v;
    return a[0] * x[0] + a[1] * x[1] + a[2] * x[2];
  };
  // a_l . (dvl or dwl) + b_l
  auto rowval = [&](int l, const double* dv, const double* dw) -> double {
    const double* x = l < NWROW ? dw : dv;
    double a[3], b;
    if (l < NBASE) {
      double r4[4];
      ldn<4>(sh.get().rows[l < NBASE ? l : 0], r4);
      a[0] = r4[0]; a[1] = r4[1]; a[2] = r4[2];
      b = r4[3];
    } else {
      er.ab(l >= NBASE ? l - NBASE : 0, a, b);
    }
    return (a[0] * x[0] + a[1] * x[1] + a[2] * x[2]) + b;
  };
  auto lin = [&](const double* u, double* dv, double* dw) {
    const auto& S = sh.get();
    double t[3];
    mv3(S.Bv, u + 3, t);
    dv[0] = im * u[0] + t[0]; dv[1] = im * u[1] + t[1]; dv[2] = im * u[2] + t[2];
    mv3(S.JTi, u + 3, dw);
  };
  auto adj = [&](const double* gv, const double* gw, double* o) {
    const auto& S = sh.get();
    double t[3], s[3];
    mtv3(S.Bv, gv, t);
    mtv3(S.JTi, gw, s);
    o[0] = im * gv[0]; o[1] = im * gv[1]; o[2] = im * gv[2];
    o[3] = t[0] + s[0]; o[4] = t[1] + s[1]; o[5] = t[2] + s[2];
  };
  auto rows_adj = [&](auto zz, double* o) {  // o = A' zz (u-space); zz(l): row multiplier
    double gv[3] = {0, 0, 0}, gw[3] = {0, 0, 0};
#pragma unroll
    for (int l = 0; l < NR; ++l) {
      double* g = l < NWROW ? gw : gv;
      const double zv = zz(l);
      double a[3];
      ra3(l, a);
      g[0] += zv * a[0]; g[1] += zv * a[1]; g[2] += zv * a[2];
    }
    adj(gv, gw, o);
  };
  // K_{-i} v = K v - U_i (U_i' v)
  auto Kmul = [&](const double* v, double* o) {
    spmv6(sh.get().K, v, o);
    double t[3], t6[6];
    Ut_apply(rt.get(0), v, t);
    U_apply(rt.get(0), t, t6);
#pragma unroll
    for (int r = 0; r < 6; ++r) o[r] -= t6[r];
  };
  auto Gy = [&](const double* yy, double* o) {
    o[0] = -yy[2]; o[1] = -sec * yy[2]; o[2] = -yy[0]; o[3] = -yy[1]; o[4] = -yy[2];
    o[5] = 0.0; o[6] = -yy[0]; o[7] = -yy[1]; o[8] = -yy[2];
  };
  auto GTz = [&](const double* z, double* o) {
    o[0] = -(z[2] + z[6]);
    o[1] = -(z[3] + z[7]);
    o[2] = -(z[0] + sec * z[1] + z[4] + z[8]);
  };
  const double mfz = P.min_fz, mxf = P.max_f;
  // primal residual of cone block k at the current iterate: G y + s - h
  double sk[NB][9], zk[NB][9];
  typename RW::template Store<NR, NX> rst(rw);  // row slacks / duals / Newton row terms (registers or LDS)
  auto SL = [&](int l) -> decltype(auto) { return rst.s(l); };
  auto ZL = [&](int l) -> decltype(auto) { return rst.z(l); };
  // per-iteration quantities: registers, or the store's aux slots (AUXM)
  double nh_r = 0.0, nq_r = 0.0, bm_r = 0.0, bk_r = 0.0;
  double rk_r[(AUXM & AUX_RES) ? 1 : 3 * NB], rf_r[(AUXM & AUX_RES) ? 1 : 6];
  double lam_r[(AUXM & AUX_LAM) ? 1 : 9 * NB];
  double di_r[(AUXM & AUX_DINV) ? 1 : 6 * NB], id0_r[(AUXM & AUX_DINV) ? 1 : NB];
  auto NH = [&]() -> decltype(auto) {
    if constexpr ((AUXM & AUX_SCAL) != 0) return rst.x(O_SC + 0); else return (nh_r);
  };
  auto NQ = [&]() -> decltype(auto) {
    if constexpr ((AUXM & AUX_SCAL) != 0) return rst.x(O_SC + 1); else return (nq_r);
  };
  auto BM = [&]() -> decltype(auto) {  // best merit seen (divergence stop)
    if constexpr ((AUXM & AUX_SCAL) != 0) return rst.x(O_SC + 2); else return (bm_r);
  };
  auto BK = [&]() -> decltype(auto) {  // merit of the recorded in-band iterate
    if constexpr ((AUXM & AUX_SCAL) != 0) return rst.x(O_SC + 3); else return (bk_r);
  };
  auto RK = [&](int k, int c) -> decltype(auto) {
    if constexpr ((AUXM & AUX_RES) != 0) return rst.x(O_RK + 3 * k + c); else return (rk_r[3 * k + c]);
  };
  auto RF = [&](int r) -> decltype(auto) {
    if constexpr ((AUXM & AUX_RES) != 0) return rst.x(O_RF + r); else return (rf_r[r]);
  };
  auto LAM = [&](int k, int j) -> decltype(auto) {
    if constexpr ((AUXM & AUX_LAM) != 0) return rst.x(O_LAM + 9 * k + j); else return (lam_r[9 * k + j]);
  };
  auto DI = [&](int k, int j) -> decltype(auto) {
    if constexpr ((AUXM & AUX_DINV) != 0) return rst.x(O_DI + 6 * k + j); else return (di_r[6 * k + j]);
  };
  auto ID0 = [&](int k) -> decltype(auto) {
    if constexpr ((AUXM & AUX_DINV) != 0) return rst.x(O_ID0 + k); else return (id0_r[k]);
  };
  auto lam4 = [&](int k, int j0, double* o) {  // lambda_k[j0 .. j0 + 3]
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = LAM(k, j0 + j);
  };
  auto dinv = [&](int k, double* o) {
#pragma unroll
    for (int j = 0; j < 6; ++j) o[j] = DI(k, j);
  };
  auto rzk_of = [&](int k, double* o) {
    Gy(y[k], o);
#pragma unroll
    for (int j = 0; j < 9; ++j) o[j] += sk[k][j];
    o[0] += mfz;
    o[5] -= mxf;
  };
  auto compute_u = [&](double* uo) {
#pragma unroll
    for (int r = 0; r < 6; ++r) uo[r] = (MODE == MODE_CENT) ? 0.0 : w[r];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      double t[6];
      U_apply(rt.get(k), y[k], t);
#pragma unroll
      for (int r = 0; r < 6; ++r) uo[r] += t[r];
    }
    if constexpr (GRP::on) {
#pragma unroll
      for (int r = 0; r < 6; ++r) uo[r] = grp.sum(uo[r]);  // (MODE_CENT: no w)
    }
  };

  // ---------------- initial point
  // The tuned start and step fraction for the C-ADMM agent QPs of a step's first ADMM pass and of
  // scenarios whose previous step took <= 3 passes (P.tuned: the warm closed loop, whose multipliers
  // are O(1e-2)); the conservative ones for the later passes of long ADMM runs (C2 / C5, cold random
  // inputs and 17-28 passes: the tuned start everywhere took C2 13 -> 20 ms and C5 81 -> 118 ms per
  // step), DD agent QPs (C3 29 -> 39 ms) and the centralized QP (also the rigid payload on the same
  // kernel, whose Jl^-1 ~ 50 grades the Newton systems)
  // start 0: conservative (as above), 1: tuned (C-ADMM), 2: the conservative start scaled by 10 (the
  // second start of a DD / centralized solve that ended outside Clarabel's tolerance, see ipm_solve)
  const bool TUNED = MODE == MODE_CADMM && start == 1;
  const double SCL = start == 2 ? 10.0 : 1.0;
  const double S0 = SCL * (TUNED ? IPM_S0 : MODE == MODE_DD ? DD_S0 : 1.0);
  const double Z0 = SCL * (TUNED ? IPM_Z0 : MODE == MODE_DD ? DD_Z0 : 1.0);
  const double ETA = TUNED ? IPM_ETA : MODE == MODE_DD ? DD_ETA : 0.99;
#pragma unroll
  for (int k = 0; k < NB; ++k) {
#pragma unroll
    for (int c = 0; c < 3; ++c) y[k][c] = y0[3 * k + c];
    double g[9];
    Gy(y[k], g);
#pragma unroll
    for (int j = 0; j < 9; ++j) sk[k][j] = -g[j];
    sk[k][0] -= mfz;
    sk[k][5] += mxf;
    // shift into the interior if the guess is not strictly feasible
    double m1 = sk[k][0], m2 = sk[k][1] - sqrt(sk[k][2] * sk[k][2] + sk[k][3] * sk[k][3] + sk[k][4] * sk[k][4]);
    double m3 = sk[k][5] - sqrt(sk[k][6] * sk[k][6] + sk[k][7] * sk[k][7] + sk[k][8] * sk[k][8]);
    double mn = fmin(m1, fmin(m2, m3));
    if (mn < 1e-3) { sk[k][0] += S0 - mn; sk[k][1] += S0 - mn; sk[k][5] += S0 - mn; }
#pragma unroll
    for (int j = 0; j < 9; ++j) zk[k][j] = 0.0;
    zk[k][0] = Z0; zk[k][1] = Z0; zk[k][5] = Z0;
  }
#pragma unroll
  for (int l = 0; l < NR; ++l) ZL(l) = Z0 * act(l);  // (the slack half of the pair is written below)
#pragma unroll
  for (int r = 0; r < 6; ++r) w[r] = 0.0;
  // C-ADMM: the free aggregate starts at its unconstrained minimiser without the u-coupling,
  // w = atil (the infeasible start lets the Newton steps restore rho (w - atil) + K_{-i} pi = 0).
  // A consistent start through a 6x6 LU of (rho I + K C) took the same iteration count and held
  // ~1 KB/lane more spill frame (C4 A/B: k_cadmm 8.9 -> 7.7 ms without it).
  if (MODE == MODE_CADMM) {
#pragma unroll
    for (int r = 0; r < 6; ++r) w[r] = P.atil[r];
  }
  {
    double u[6], dv[3], dw[3];
    compute_u(u);
    lin(u, dv, dw);
#pragma unroll
    for (int l = 0; l < NR; ++l) SL(l) = fmax(rowval(l, dv, dw), S0);
  }
  if constexpr (WS) {
    static_assert(NB == 1 && NR <= DAT_MAXROW, "warm start: C-ADMM agent QP");
    if (start == 3) {
      // (s, z) -> (s + d, z + d) with (s + d)(z + d) >= mu (WS_MU; DD_WS_MU for the DD agent QPs)
      constexpr double mu = MODE == MODE_DD ? DD_WS_MU : WS_MU;
      auto push = [](double s, double z) -> double {
        const double p = s * z;
        if (!(p < mu)) return 0.0;
        const double t = s + z;
        return 0.5 * (sqrt(t * t + 4.0 * (mu - p)) - t);
      };
#pragma unroll
      for (int c = 0; c < 3; ++c) y[0][c] = wrec[1 + c];
#pragma unroll
      for (int r = 0; r < 6; ++r) w[r] = wrec[4 + r];
      double g[9];
      Gy(y[0], g);
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        sk[0][j] = -g[j];
        zk[0][j] = wrec[19 + j];
      }
      sk[0][0] -= mfz;
      sk[0][5] += mxf;
      {
        const double d = push(fmax(sk[0][0], 0.0), fmax(zk[0][0], 0.0));
        sk[0][0] = fmax(sk[0][0], 0.0) + d;
        zk[0][0] = fmax(zk[0][0], 0.0) + d;
      }
#pragma unroll
      for (int b = 1; b <= 5; b += 4) {
        const double ms = sk[0][b] - sqrt(sk[0][b + 1] * sk[0][b + 1] + sk[0][b + 2] * sk[0][b + 2] + sk[0][b + 3] * sk[0][b + 3]);
        const double mz = zk[0][b] - sqrt(zk[0][b + 1] * zk[0][b + 1] + zk[0][b + 2] * zk[0][b + 2] + zk[0][b + 3] * zk[0][b + 3]);
        const double d = push(fmax(ms, 0.0), fmax(mz, 0.0));
        sk[0][b] += d - fmin(ms, 0.0);
        zk[0][b] += d - fmin(mz, 0.0);
      }
      double u[6], dv[3], dw[3];
      compute_u(u);
      lin(u, dv, dw);
#pragma unroll
      for (int l = 0; l < NR; ++l) {
        const double sl = fmax(rowval(l, dv, dw), 0.0), zl = fmax(wrec[28 + DAT_MAXROW + l], 0.0);
        const double d = act(l) * push(sl, zl);
        rst.set_sz(l, act(l) > 0.0 ? sl + d : fmax(rowval(l, dv, dw), S0), act(l) * (zl + d));
      }
    }
  }

  // scales for the relative stopping rule
  {
    double nh = 1.0 + fmax(mfz, mxf), nq = 1.0;
#pragma unroll
    for (int l = 0; l < NR; ++l) nh = fmax(nh, 1.0 + act(l) * fabs(rb(l)));
    {
      double nb = 1.0;
#pragma unroll
      for (int k = 0; k < NB; ++k)
#pragma unroll
        for (int c = 0; c < 3; ++c) nb = fmax(nb, 1.0 + fabs(P.q[k][c]));
      nq = fmax(nq, grp.max(nb));
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) nq = fmax(nq, 1.0 + fabs(cup()[r]));
    NH() = nh;
    NQ() = nq;
  }

  // best in-band iterate (merit of the recorded one) and the best merit seen (divergence stop)
  BM() = 1e300;
  BK() = 1e300;
  out.status = ST_INACCURATE;  // until converged (or failed on non-finite data)
  const double ideg = 1.0 / (double)(3 * grp.nblk(NB) + __builtin_popcount(mask));
  int bk_it = 0;  // WS: the iteration of the last halving of the best in-band merit (stall exit)
  // WS: the current iterate into the warm-start record (the next ADMM pass's start)
  auto record = [&]() {
    if constexpr (WS) {
      if (wrec) {
#pragma unroll
        for (int c = 0; c < 3; ++c) wrec[1 + c] = y[0][c];
#pragma unroll
        for (int r = 0; r < 6; ++r) wrec[4 + r] = w[r];
#pragma unroll
        for (int j = 0; j < 9; ++j) { wrec[10 + j] = sk[0][j]; wrec[19 + j] = zk[0][j]; }
#pragma unroll
        for (int l = 0; l < NR; ++l) {
          double sl, zl;
          rst.sz(l, sl, zl);
          wrec[28 + l] = sl;
          wrec[28 + DAT_MAXROW + l] = zl;
        }
        wrec[0] = 1.0;
      }
    }
  };

  DAT_PHASE_INIT(0);
  for (int it = 0;; ++it) {
    DAT_PHASE(1);
    // ------------- residuals
    double dv[3], dw[3];
    double dres = 0.0, pres = 0.0, gap = 0.0;
    double chk = 0.0;  // plain sum of every residual entry: NaN / Inf propagate (fmax drops NaN)
    // primal objective of the iterate (constants dropped, as cvxpy hands it to the solver): the scale
    // of the relative gap test
    double pobj = 0.0;
    {
      double u[6], pi[6], az[6];
      compute_u(u);
      lin(u, dv, dw);
      spmv6(Cp(), u, pi);
      rows_adj(ZL, az);
      {
        double cu6[6];
        ldn<6>(cup(), cu6);
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          pobj += u[r] * (0.5 * pi[r] + cu6[r]);
          pi[r] += cu6[r] - az[r];
        }
      }
      // the cone blocks' parts (reduced over a lane group, GRP) before the replicated ones
      double pobj_b = 0.0;
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        double ut[3], gz[3];
        Ut_apply(rt.get(k), pi, ut);
        GTz(zk[k], gz);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const double r = kap * y[k][c] + P.q[k][c] + ut[c] + gz[c];
          pobj_b += y[k][c] * (0.5 * kap * y[k][c] + P.q[k][c]);
          RK(k, c) = r;
          dres = fmax(dres, fabs(r));
          chk += r;
        }
      }
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        double rz[9];
        rzk_of(k, rz);
#pragma unroll
        for (int j = 0; j < 9; ++j) {
          pres = fmax(pres, fabs(rz[j]));
          chk += rz[j];
          gap += sk[k][j] * zk[k][j];
        }
      }
      if constexpr (GRP::on) {
        dres = grp.max(dres);
        pres = grp.max(pres);
        chk = grp.sum(chk);
        gap = grp.sum(gap);
        pobj_b = grp.sum(pobj_b);
      }
      pobj += pobj_b;
      {
        double Rf[6];
        if (MODE == MODE_CADMM) {
          // free blocks f_j = a_j - U_j' pi / rho: sum_j rho/2 ||f_j||^2 - rho a_j . f_j
          //   = pi' K_{-i} pi / (2 rho) - rho/2 sum_j ||a_j||^2
          double kp[6];
          Kmul(pi, kp);
          double pkp = 0.0;
#pragma unroll
          for (int r = 0; r < 6; ++r) {
            Rf[r] = P.rho * (w[r] - P.atil[r]) + kp[r];
            pkp += pi[r] * kp[r];
          }
          pobj += 0.5 * (pkp * irho - P.rho * P.a2);
        } else if (MODE == MODE_DD) {
#pragma unroll
          for (int r = 0; r < 6; ++r) {
            Rf[r] = pi[r] + P.cw[r];
            pobj += P.cw[r] * w[r];
          }
        } else {
#pragma unroll
          for (int r = 0; r < 6; ++r) Rf[r] = 0.0;
        }
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          RF(r) = Rf[r];
          dres = fmax(dres, fabs(Rf[r]));
          chk += Rf[r];
        }
      }
#pragma unroll
      for (int l = 0; l < NR; ++l) {
        double sl, zl;
        rst.sz(l, sl, zl);
        const double rl = sl - (rowval(l, dv, dw));
        pres = fmax(pres, fabs(rl));
        chk += rl;
        gap += sl * zl;
      }
      out.iters = it;
      if (!(fabs(chk + gap) < 1e300)) {  // NaN or Inf anywhere in the residuals
        // at the initial point: the problem data itself is not finite (the solver-exception
        // branch); later: a numerical breakdown of a finite problem (not solved)
        out.status = it == 0 ? ST_FAILED : ST_INACCURATE;
        out.why = 1;
        break;
      }
      const double nh = NH(), nq = NQ();
      // complementarity gap, absolute or relative to the objective as Clarabel tests it (gap_abs or
      // gap_rel): converged when gap < 10 tol or gap < tol / 10 |pobj| (at the default tol = 1e-10: 1e-9
      // absolute, or the oracle's own 1e-11 relative rule), i.e. the scaled gap gap / max(1, |pobj| / 100)
      // below 10 tol.  With multipliers ~1e3-1e4 (a stalled ADMM loop, |pobj| ~1e4-1e5) an absolute gap
      // of 1e-9 lies below what the Newton systems resolve; well-scaled QPs (|pobj| <= 100) keep the
      // absolute rule.
      const double grel = gap * frcp(fmax(1.0, 0.01 * fabs(pobj)));
      double merit = fmax(fmax(pres / nh, dres / nq), grel);
#ifdef DAT_IPM_TRACE
      printf("ipm it %2d pres %.3e dres %.3e gap %.3e merit %.3e pobj %.3e\n", it, pres / nh, dres / nq, grel, merit,
             pobj);
#endif
      if (pres < tol * nh && dres < tol * nq && grel < 10.0 * tol) {
        out.status = ST_OPTIMAL;
        out.merit = merit;
#pragma unroll
        for (int r = 0; r < 6; ++r) { out.pi[r] = pi[r]; out.u[r] = u[r]; }
        record();  // the converged iterate: the next pass's warm start
        DAT_PHASE(8);
        return out;
      }
      // Only an in-band iterate (scaled residuals < 1e-7, relative gap < 1e-6) can be returned: a solve
      // that ends out of band is INACCURATE and the callers hold their previous solution instead, so
      // out-of-band iterates are never recorded (the record is written in the last one or two
      // iterations of a stalling solve, not at every iteration).  Its merit is measured as Clarabel
      // measures convergence (residuals, and the gap absolute or relative to the objective, whichever
      // is smaller: max(1, |pobj|) scaling), so inband_loose counts exactly the accepts outside
      // Clarabel's own tolerance.
      const double mclr = fmax(fmax(pres / nh, dres / nq), gap * frcp(fmax(1.0, fabs(pobj))));
      const bool band = fmax(pres / nh, dres / nq) < 1e-7 && mclr < 1e-6;
      const bool prog = band && mclr < 0.5 * BK();  // (WS: the stall exit below)
      if (band && mclr < BK()) {
        BK() = mclr;
#pragma unroll
        for (int k = 0; k < NB; ++k)
#pragma unroll
          for (int c = 0; c < 3; ++c) best[3 * k + c] = y[k][c];
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          best[3 * NB + r] = w[r];
          best[3 * NB + 6 + r] = pi[r];
          best[3 * NB + 12 + r] = u[r];
        }
      }
      if (WS && wson) {
        // stall exit (the tail kernel): an in-band iterate WS_STALL_TOL (ten times inside Clarabel's tolerance)
        // is recorded and the merit has not halved in WS_STALL_ITS iterations -- the Newton systems of a stalled
        // ADMM loop's agent QP resolve no further; its best in-band iterate is returned (OPTIMAL, in band)
        if (prog) bk_it = it;
        if (BK() <= WS_STALL_TOL && it - bk_it >= WS_STALL_ITS) {
          out.why = 7;
          record();  // the current iterate (in band): the next pass's warm start
          break;
        }
      }
      BM() = fmin(BM(), merit);
      if ((it >= 4 && merit > IPM_DIVERGE * BM()) || it >= max_iter) {
        out.why = 2;
        break;
      }
      if (it >= max_iter) break;
    }

    // ------------- NT scaling of the cone blocks
    DAT_PHASE(2);
#if defined(DAT_IPM_STATS) && !defined(__HIP_DEVICE_COMPILE__)
    g_maxw = 0.0;
#endif
    SocScale S1[NB], S2[NB];
    bool okc = true;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      if (ROB) {
        // a second-order cone iterate that rounding put on (or past) the boundary: back inside by a few ulps of
        // its axis (the step rule keeps it strictly inside in exact arithmetic).  Without it the robust solver
        // stopped at the NT scaling (why 3) on the stall QPs the 10 s C4 loop accepted beyond Clarabel's 1e-8 (20
        // of 20 captured, tests/golden/ref_loose_caps.npz); with it all 20 converge to 1e-11.
#pragma unroll
        for (int b0 = 1; b0 <= 5; b0 += 4) {
          double* vv[2] = {sk[k] + b0, zk[k] + b0};
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            double* v = vv[q];
            const double n1 = sqrt(v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
            if (!(v[0] - n1 > 1e-14 * n1)) v[0] = n1 * (1.0 + 1e-14) + 1e-300;
          }
        }
      }
      ID0(k) = sqrt(zk[k][0] * frcp(sk[k][0]));  // 1 / d0, d0 = sqrt(s0 / z0)
      LAM(k, 0) = sqrt(sk[k][0] * zk[k][0]);
      okc = okc && soc_scaling(sk[k] + 1, zk[k] + 1, S1[k]) && soc_scaling(sk[k] + 5, zk[k] + 5, S2[k]);
      double l1[4], l2[4];
      soc_apply(S1[k], zk[k] + 1, l1, false);
      soc_apply(S2[k], zk[k] + 5, l2, false);
#pragma unroll
      for (int j = 0; j < 4; ++j) { LAM(k, 1 + j) = l1[j]; LAM(k, 5 + j) = l2[j]; }
    }
#ifdef DAT_IPM_TRACE
    for (int k = 0; k < NB; ++k)
      printf("    cone s %.2e %.2e %.2e z %.2e %.2e %.2e | eta1 %.2e eta2 %.2e | rows z/s %.2e %.2e %.2e\n", sk[k][0],
             sk[k][1] - sqrt(sk[k][2] * sk[k][2] + sk[k][3] * sk[k][3] + sk[k][4] * sk[k][4]),
             sk[k][5] - sqrt(sk[k][6] * sk[k][6] + sk[k][7] * sk[k][7] + sk[k][8] * sk[k][8]), zk[k][0],
             zk[k][1] - sqrt(zk[k][2] * zk[k][2] + zk[k][3] * zk[k][3] + zk[k][4] * zk[k][4]),
             zk[k][5] - sqrt(zk[k][6] * zk[k][6] + zk[k][7] * zk[k][7] + zk[k][8] * zk[k][8]), S1[k].eta, S2[k].eta,
             (double)ZL(0) / (double)SL(0), (double)ZL(1) / (double)SL(1), (double)ZL(2) / (double)SL(2));
#endif
    if constexpr (GRP::on) okc = grp.min(okc ? 1.0 : 0.0) > 0.5;
    if (!okc) {
      out.why = 3;
      break;
    }
    auto winv = [&](int k, const double* v, double* o) {  // W_k^-1 v
      o[0] = v[0] * ID0(k);
      soc_apply(S1[k], v + 1, o + 1, true);
      soc_apply(S2[k], v + 5, o + 5, true);
    };
    // Gs = W^-1 G applied to a 3-vector / its transpose applied to a 9-vector
    auto gs_mul = [&](int k, const double* v, double* o) {
      double g[9];
      Gy(v, g);
      winv(k, g, o);
    };
    auto gs_tmul = [&](int k, const double* t, double* o) {
      double g[9];
      winv(k, t, g);
      GTz(g, o);
    };
    // D_k = kappa I + Gs'Gs through its QR square-root factor (qr_cone: forming D cancels once an active
    // cone makes Gs stiff); DI holds the factor, applied by dsolve3
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      double gc[3][9];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        double e[3] = {c == 0 ? 1.0 : 0.0, c == 1 ? 1.0 : 0.0, c == 2 ? 1.0 : 0.0};
        gs_mul(k, e, gc[c]);
      }
      double Rd[6];
      okc = okc && qr_cone(kap, gc, Rd);
#pragma unroll
      for (int j = 0; j < 6; ++j) DI(k, j) = Rd[j];
    }
    if constexpr (GRP::on) okc = grp.min(okc ? 1.0 : 0.0) > 0.5;
    if (!okc) {
      out.why = 4;
      break;
    }
    DAT_PHASE(3);
    // M = Lm Lm' (Cholesky; M is SPD: C carries k_f, k_m > 0) and, for CADMM / CENT, the Cholesky
    // factor Ln of the SPD matrix N = I + Lm' T Lm, so that (I + M T)^-1 M = Lm N^-1 Lm' =: P.  N has
    // every eigenvalue >= 1 however large active rows make M, so the factorisation stays well
    // conditioned without a pivoted nonsymmetric LU; only P (21 doubles) is kept for the solves.
    // DD: Lm alone (reciprocal diagonal, for chol6_solve).
    // Stiff rows.  Near the solution an active row's barrier weight z/s grows without bound; inside a
    // stalled ADMM loop (multipliers ~1e3-1e4, rows with tiny coefficients) it reaches 1e10-1e22.  Folded
    // into M = C + A'(Z/S)A it wipes out C's digits, and the row's dual direction dz = zw - (z/s) a.du is
    // a difference of huge terms.  So the first IPM_NSTIFF rows (slot order) whose weight exceeds
    // IPM_STIFF_W stay out of M; their dual directions are unknowns of a small augmented system
    //   a_l . lin(du) + (s_l / z_l) dz_l = g_l      (row primal + complementarity, no 1/s anywhere)
    // solved by a Schur complement on the stiff rows: du = du0 + sum_l dz_l H abar_l, where du0 is the
    // core solve without them and H abar_l a core solve with the row's u-space coefficient as bu (the
    // columns, once per iteration, kept in the lane's scratch record behind `best`).  Without stiff rows
    // (every well-scaled QP) nothing changes.
    unsigned smask = 0u;  // stiff row slots (the rows' data: the scratch record behind `best`)
    double* const hcol = best + best_rec(NB);                    // [j][dy (3 NB), dw (6), du (6)]
    double* const srec = hcol + IPM_NSTIFF * stiff_col(NB);      // [j][a0 a1 a2 on_dwl e g dz tmp]
    double* const sfac = srec + IPM_NSTIFF * STIFF_ROW;          // Cholesky factor of S
    // DD: Cholesky factor of M;  CADMM / CENT: P = Lm N^-1 Lm' (schur_P).  WS (the tail kernel, one scenario
    // per workgroup, latency-bound): kept in the lane's scratch record (LDS there) across the iteration's solves
    // instead of 42 registers of a frame that spills (stall fixture, same-call A/B: 41.8 / 33.7 -> 39.1 / 30.6 ms per
    // stalled step; the cones' s, z and the Newton step's cone terms there as well measured no better, or worse)
    double LmR[21];
    double* const Lm = WS && MODE == MODE_CADMM ? best + best_size(NB) - FM_DOUBLES : LmR;  // (DD: HBM records)
    {
      double Mm[21];
      // M = C + sum_l (z/s) a_l a_l' (u-space, packed), assembled in (dvl, dwl) coordinates
      {
        double Xv[6] = {0, 0, 0, 0, 0, 0}, Xw[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int l = 0; l < NR; ++l) {
          double sl, zl;
          rst.sz(l, sl, zl);
          double wgt = zl * frcp(sl);
          DAT_STAT_W(act(l) * wgt);
          double a3v[3];
          ra3(l, a3v);
          if (ROB && act(l) > 0.0 && wgt > IPM_STIFF_W && __builtin_popcount(smask) < IPM_NSTIFF) {
            double* r = srec + __builtin_popcount(smask) * STIFF_ROW;
            r[0] = a3v[0]; r[1] = a3v[1]; r[2] = a3v[2];
            r[3] = l < NWROW ? 1.0 : 0.0;
            r[4] = sl * frcp(zl);
            smask |= 1u << l;
            wgt = 0.0;
          }
          double* X = l < NWROW ? Xw : Xv;
          const double a0 = a3v[0], a1 = a3v[1], a2 = a3v[2];
          X[0] += wgt * a0 * a0; X[1] += wgt * a0 * a1; X[2] += wgt * a0 * a2;
          X[3] += wgt * a1 * a1; X[4] += wgt * a1 * a2; X[5] += wgt * a2 * a2;
        }
        // Av = [im I, Bv];  Av' Xv Av = [[im^2 Xv, im Xv Bv], [., Bv' Xv Bv]];  Aw = [0, JTi]
        const auto& S = sh.get();
        double XB[9], XJ[9], Bv[10], JTi[10];
        ldn<10>(S.Bv, Bv);
        ldn<10>(S.JTi, JTi);
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            XB[3 * r + c] = Xv[sp3(r, 0)] * Bv[c] + Xv[sp3(r, 1)] * Bv[3 + c] + Xv[sp3(r, 2)] * Bv[6 + c];
            XJ[3 * r + c] = Xw[sp3(r, 0)] * JTi[c] + Xw[sp3(r, 1)] * JTi[3 + c] + Xw[sp3(r, 2)] * JTi[6 + c];
          }
        double C[22];
        ldn<22>(&S.C[var][0], C);
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            if (c >= r) {
              Mm[sp6(r, c)] = C[sp6(r, c)] + im * im * Xv[sp3(r, c)];
              double s = C[sp6(3 + r, 3 + c)];
#pragma unroll
              for (int k2 = 0; k2 < 3; ++k2) s += Bv[3 * k2 + r] * XB[3 * k2 + c] + JTi[3 * k2 + r] * XJ[3 * k2 + c];
              Mm[sp6(3 + r, 3 + c)] = s;
            }
            Mm[sp6(r, 3 + c)] = C[sp6(r, 3 + c)] + im * XB[3 * r + c];
          }
      }
      if (MODE == MODE_DD) {
        if (!chol6(Mm, Lm)) {
          out.why = 5;
          break;
        }
      } else {
        if (!chol6_lower(Mm, Lm)) {
          out.why = 5;
          break;
        }
        // T = sum_k U_k D_k^-1 U_k' (+ K_{-i} / rho)
        double T[21];
        if (MODE == MODE_CADMM) {
          double K[22];
          ldn<22>(&sh.get().K[0], K);
#pragma unroll
          for (int k = 0; k < 21; ++k) T[k] = K[k] * irho;
          // K_{-i}/rho + U_i Dinv U_i' = K/rho + U_i (Dinv - I/rho) U_i'
          double Rd[6], Dm[6];
          dinv(0, Rd);
          dinv_explicit(Rd, Dm);
          Dm[0] -= irho;
          Dm[3] -= irho;
          Dm[5] -= irho;
          add_UDUt(T, rt.get(0), Dm, 1.0);
        } else {
#pragma unroll
          for (int k = 0; k < 21; ++k) T[k] = 0.0;
#pragma unroll
          for (int k = 0; k < NB; ++k) {
            double Rd[6], Di[6];
            dinv(k, Rd);
            dinv_explicit(Rd, Di);
            add_UDUt(T, rt.get(k), Di, 1.0);
          }
          if constexpr (GRP::on) {
#pragma unroll
            for (int k = 0; k < 21; ++k) T[k] = grp.sum(T[k]);
          }
        }
        double Nn[21], Ln[21];
        ltl_plus_identity(Lm, T, Nn);
        if (!chol6(Nn, Ln)) {
          out.why = 6;
          break;
        }
        double Pm[21];
        schur_P(Lm, Ln, Pm);
#pragma unroll
        for (int k = 0; k < 21; ++k) Lm[k] = Pm[k];
      }
    }

    // core structured solve of (D + U'MU) dx = b (CADMM/CENT) or its DD analogue.  bu: u-space
    // part of the right-hand side (has_bu = false: zero); acc: add the solution to the outputs.
    auto core = [&](const double bk[NB][3], const double* Rfr, const double* bu, bool has_bu, bool acc,
                    double dyo[NB][3], double* dwo, double* duo) {
      double dyn[NB][3], dwn[6], dun[6];
      if (MODE == MODE_DD) {
#pragma unroll
        for (int r = 0; r < 6; ++r) dun[r] = -Rfr[r] + (has_bu ? bu[r] : 0.0);
        chol6_solve(Lm, dun);
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          double t[3], v[3];
          Ut_apply(rt.get(k), Rfr, t);
#pragma unroll
          for (int c = 0; c < 3; ++c) v[c] = bk[k][c] + t[c];
          double Rd[6];
          dinv(k, Rd);
          dsolve3(Rd, v, dyn[k]);
        }
#pragma unroll
        for (int r = 0; r < 6; ++r) dwn[r] = dun[r];
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          double t[6];
          U_apply(rt.get(k), dyn[k], t);
#pragma unroll
          for (int r = 0; r < 6; ++r) dwn[r] -= t[r];
        }
      } else {
        double bk2[NB][3], yv[6] = {0, 0, 0, 0, 0, 0}, g6[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          double t[3] = {0, 0, 0}, v[3], ut[6];
          if (has_bu) Ut_apply(rt.get(k), bu, t);
#pragma unroll
          for (int c = 0; c < 3; ++c) bk2[k][c] = bk[k][c] + t[c];
          double Rd[6];
          dinv(k, Rd);
          dsolve3(Rd, bk2[k], v);
          U_apply(rt.get(k), v, ut);
#pragma unroll
          for (int r = 0; r < 6; ++r) yv[r] += ut[r];
        }
        if constexpr (GRP::on) {
#pragma unroll
          for (int r = 0; r < 6; ++r) yv[r] = grp.sum(yv[r]);
        }
        if (MODE == MODE_CADMM) {
          if (has_bu) Kmul(bu, g6);
#pragma unroll
          for (int r = 0; r < 6; ++r) {
            g6[r] -= Rfr[r];  // g6 = -Rf + K_{-i} bu
            yv[r] += g6[r] * irho;
          }
        }
        // tau = (I + M T)^-1 M yv = Lm N^-1 Lm' yv = P yv
        double tau[6];
        spmv6(Lm, yv, tau);
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          double t[3], v[3];
          Ut_apply(rt.get(k), tau, t);
#pragma unroll
          for (int c = 0; c < 3; ++c) v[c] = bk2[k][c] - t[c];
          double Rd[6];
          dinv(k, Rd);
          dsolve3(Rd, v, dyn[k]);
        }
        if (MODE == MODE_CADMM) {
          double kt[6];
          Kmul(tau, kt);
#pragma unroll
          for (int r = 0; r < 6; ++r) dwn[r] = (g6[r] - kt[r]) * irho;
        } else {
#pragma unroll
          for (int r = 0; r < 6; ++r) dwn[r] = 0.0;
        }
#pragma unroll
        for (int r = 0; r < 6; ++r) dun[r] = (MODE == MODE_CADMM) ? dwn[r] : 0.0;
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          double t[6];
          U_apply(rt.get(k), dyn[k], t);
#pragma unroll
          for (int r = 0; r < 6; ++r) dun[r] += t[r];
        }
        if constexpr (GRP::on) {  // (MODE_CENT: no w)
#pragma unroll
          for (int r = 0; r < 6; ++r) dun[r] = grp.sum(dun[r]);
        }
      }
#pragma unroll
      for (int k = 0; k < NB; ++k)
#pragma unroll
        for (int c = 0; c < 3; ++c) dyo[k][c] = (acc ? dyo[k][c] : 0.0) + dyn[k][c];
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        dwo[r] = (acc ? dwo[r] : 0.0) + dwn[r];
        duo[r] = (acc ? duo[r] : 0.0) + dun[r];
      }
    };

    // Newton direction for complementarity targets rsk (cones, scaled) and, for the rows,
    // rc_l = s_l z_l + cadd_l (cadd = 0 for the predictor; the corrector's second-order term is
    // formed in place from the predictor's row direction ddva/ddwa and its zw).  Outputs: dy, dw,
    // du, scaled dz of the cones (dzs_k), lam \ rsk (lrs_k, so dss_k = -lrs_k - dzs_k) and zw
    // (row dz is zw - (z/s) a.lin(du); a stiff row's zw is its dz).
    double dy[NB][3], dwv[6], du[6], dzs_k[NB][9], lrs_k[NB][9];
    auto ZW = [&](int l) -> decltype(auto) { return rst.w(l); };
    // tks_k = W^-1 rz_k - lam \ rsk
    auto tks_of = [&](int k, double* t) {
      double rz[9];
      rzk_of(k, rz);
      winv(k, rz, t);
#pragma unroll
      for (int j = 0; j < 9; ++j) t[j] -= lrs_k[k][j];
    };
    // stiff rows (see the M assembly): the columns H abar_j (core solves with the row's u-space
    // coefficient as bu) and the Cholesky factor of S_ij = a_i . lin(H abar_j) + (s_i / z_i) delta_ij,
    // formed by the predictor's newton call; everything through the lane's scratch record, in run-time
    // loops over the stiff rows (well-scaled QPs never enter)
    const int nst = __builtin_popcount(smask);
    if (nst > 0) out.stiff = 1;
    // a_j . lin(v) of stiff row j
    auto srow = [&](int j, const double* v) -> double {
      const double* r = srec + j * STIFF_ROW;
      double dv2[3], dw2[3];
      lin(v, dv2, dw2);
      const double* x = r[3] != 0.0 ? dw2 : dv2;
      return r[0] * x[0] + r[1] * x[1] + r[2] * x[2];
    };
    // stiff-row step: residuals r_j (in scratch at offset `ro` of each row record) of the stiff rows'
    // equations are turned into dz = S^-1 r (in place), and (yy, ww, uu) += sum_j dz_j H abar_j
    auto stiff_update = [&](int ro, double yy[NB][3], double* ww, double* uu) {
#pragma unroll 1
      for (int i = 0; i < nst; ++i) {
        double t = srec[i * STIFF_ROW + ro];
#pragma unroll 1
        for (int k = 0; k < i; ++k) t -= sfac[i * (i + 1) / 2 + k] * srec[k * STIFF_ROW + ro];
        srec[i * STIFF_ROW + ro] = t * sfac[i * (i + 1) / 2 + i];
      }
#pragma unroll 1
      for (int i = nst - 1; i >= 0; --i) {
        double t = srec[i * STIFF_ROW + ro];
#pragma unroll 1
        for (int k = i + 1; k < nst; ++k) t -= sfac[k * (k + 1) / 2 + i] * srec[k * STIFF_ROW + ro];
        srec[i * STIFF_ROW + ro] = t * sfac[i * (i + 1) / 2 + i];
      }
#pragma unroll 1
      for (int j = 0; j < nst; ++j) {
        const double f = srec[j * STIFF_ROW + ro];
        const double* h = hcol + j * stiff_col(NB);
#pragma unroll
        for (int k = 0; k < NB; ++k)
#pragma unroll
          for (int c = 0; c < 3; ++c) yy[k][c] += f * h[3 * k + c];
#pragma unroll
        for (int q = 0; q < 6; ++q) { ww[q] += f * h[3 * NB + q]; uu[q] += f * h[3 * NB + 6 + q]; }
      }
    };
    // stiff row slot l <-> scratch index j (position among the stiff slots)
    auto spos = [&](int l) -> int { return __builtin_popcount(smask & ((1u << l) - 1u)); };
    auto newton = [&](const double rsk[NB][9], bool corr, const double* ddva, const double* ddwa, double sigmu) {
      double bk[NB][3], bu[6];
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        lrs_k[k][0] = rsk[k][0] * frcp(LAM(k, 0));
        {
          double l4[4];
          lam4(k, 1, l4);
          soc_jdiv(l4, rsk[k] + 1, lrs_k[k] + 1);
          lam4(k, 5, l4);
          soc_jdiv(l4, rsk[k] + 5, lrs_k[k] + 5);
        }
        double tks[9], g3[3];
        tks_of(k, tks);
        gs_tmul(k, tks, g3);
#pragma unroll
        for (int c = 0; c < 3; ++c) bk[k][c] = -RK(k, c) - g3[c];
      }
      // stiff rows: right-hand sides g of their equations go to the scratch record (their zw is 0 in bu)
#pragma unroll
      for (int l = 0; l < NR; ++l) {
        double sl, zl, al3[3], bl;
        rst.sz(l, sl, zl);
        rowld(l, al3, bl);
        const double is = frcp(sl);
        const double rzl = sl - (dot3x(l, al3, dv, dw) + bl);
        const bool stf = (smask >> l) & 1u;
        double cadd = 0.0;
        if (corr) {
          const double a = dot3x(l, al3, ddva, ddwa);
          cadd = act(l) * ((-rzl + a) * (stf ? (double)ZW(l) : ZW(l) - zl * is * a) - sigmu);
        }
        if (__builtin_expect(stf, 0)) {
          srec[spos(l) * STIFF_ROW + 5] = rzl - sl - cadd * frcp(zl);
          ZW(l) = 0.0;
        } else {
          ZW(l) = (zl * rzl - (sl * zl + cadd)) * is;
        }
      }
      rows_adj(ZW, bu);
      if (__builtin_expect(!corr && nst > 0, 0)) {
        // the predictor's call first solves for the iteration's stiff-row columns H abar_j (bk = 0,
        // Rf = 0, bu = abar_j) and factors their Schur complement
        // (k_cadmm_tail: the agent lane's nclone bit-identical clones take every nclone-th column, into the
        // agent's shared scratch record in LDS; the Schur factorisation below reads all of them)
#pragma unroll 1
        for (int j = clone; j < nst; j += nclone) {
          double ab[6];
          {
            const double* r = srec + j * STIFF_ROW;
            double gv[3] = {0, 0, 0}, gw[3] = {0, 0, 0};
            double* g = r[3] != 0.0 ? gw : gv;
            g[0] = r[0]; g[1] = r[1]; g[2] = r[2];
            adj(gv, gw, ab);
          }
          double zb[NB][3], z6[6] = {0, 0, 0, 0, 0, 0}, cy[NB][3], cw[6], cu[6];
#pragma unroll
          for (int k = 0; k < NB; ++k) zb[k][0] = zb[k][1] = zb[k][2] = 0.0;
          core(zb, z6, ab, true, false, cy, cw, cu);
          double* h = hcol + j * stiff_col(NB);
#pragma unroll
          for (int k = 0; k < NB; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) h[3 * k + c] = cy[k][c];
#pragma unroll
          for (int q = 0; q < 6; ++q) { h[3 * NB + q] = cw[q]; h[3 * NB + 6 + q] = cu[q]; }
        }
#if defined(__HIP_DEVICE_COMPILE__)
        if (nclone > 1) {  // the other clones' columns: stores complete before the reads below (one wavefront)
          __builtin_amdgcn_s_waitcnt(0);
          __atomic_signal_fence(__ATOMIC_SEQ_CST);
        }
#endif
        // Cholesky of the symmetrised Schur complement S, column by column
#pragma unroll 1
        for (int j = 0; j < nst; ++j) {
          double d = srow(j, hcol + j * stiff_col(NB) + 3 * NB + 6) + srec[j * STIFF_ROW + 4];
#pragma unroll 1
          for (int k = 0; k < j; ++k) d -= sfac[j * (j + 1) / 2 + k] * sfac[j * (j + 1) / 2 + k];
          const double id = frcp(sqrt(fmax(d, 1e-300)));
          sfac[j * (j + 1) / 2 + j] = id;
#pragma unroll 1
          for (int i = j + 1; i < nst; ++i) {
            double t = 0.5 * (srow(i, hcol + j * stiff_col(NB) + 3 * NB + 6) +
                              srow(j, hcol + i * stiff_col(NB) + 3 * NB + 6));
#pragma unroll 1
            for (int k = 0; k < j; ++k) t -= sfac[i * (i + 1) / 2 + k] * sfac[j * (j + 1) / 2 + k];
            sfac[i * (i + 1) / 2 + j] = t * id;
          }
        }
    }
      {
        double rfv[6];
#pragma unroll
        for (int r = 0; r < 6; ++r) rfv[r] = RF(r);
        core(bk, rfv, bu, true, false, dy, dwv, du);
      }
      // stiff rows' dual directions dz (scratch, and their zw slots)
      auto stiff_store = [&]() {
#pragma unroll
        for (int l = 0; l < NR; ++l)
          if (__builtin_expect((smask >> l) & 1u, 0)) ZW(l) = srec[spos(l) * STIFF_ROW + 6];
      };
      if (__builtin_expect(nst > 0, 0)) {
#pragma unroll 1
        for (int j = 0; j < nst; ++j) srec[j * STIFF_ROW + 6] = srec[j * STIFF_ROW + 5] - srow(j, du);
        stiff_update(6, dy, dwv, du);
        stiff_store();
      }
      // the affine (predictor) direction only sets the step length, sigma and the corrector's
      // second-order term: it is used unrefined; the corrector -- the step actually taken -- is refined
      // (a gate skipping the pass when every row's barrier weight z/s < 1 -- tools/ipm_stats.py: no
      // correction was ever applied below z/s = 10 on the C4 loop -- measured slower: C4 k_cadmm 3.74 ->
      // 4.00 ms, the extra live value costs more than the skipped residual)
      const int nref = corr ? (ROB ? NREF_ROB : NREF) : 0;
      if (corr) DAT_STAT(0);
#pragma unroll 1
      for (int ref = 0; ref < nref; ++ref) {
        DAT_STAT(1);
        ++out.refs;
        if (ref == 1) DAT_STAT_H(2);
        // linearised dual residual of the full system at (dy, dw); refine
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          double tks[9], g9[9];
          tks_of(k, tks);
          gs_mul(k, dy[k], g9);
#pragma unroll
          for (int j = 0; j < 9; ++j) dzs_k[k][j] = tks[j] + g9[j];
        }
        double ddv[3], ddw[3], dpi[6];
        lin(du, ddv, ddw);
        spmv6(Cp(), du, dpi);
        {
          double gv[3] = {0, 0, 0}, gw[3] = {0, 0, 0}, adz[6];
#pragma unroll
          for (int l = 0; l < NR; ++l) {
            double sl, zl, a[3];
            rst.sz(l, sl, zl);
            ra3(l, a);
            const bool stf = (smask >> l) & 1u;
            const double dzl = stf ? (double)ZW(l) : ZW(l) - zl * frcp(sl) * dot3x(l, a, ddv, ddw);
            double* g = l < NWROW ? gw : gv;
            g[0] += dzl * a[0]; g[1] += dzl * a[1]; g[2] += dzl * a[2];
          }
          adj(gv, gw, adz);
#pragma unroll
          for (int r = 0; r < 6; ++r) dpi[r] -= adz[r];
        }
        double ek[NB][3], ef[6];
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          double ut[3], g3[3];
          Ut_apply(rt.get(k), dpi, ut);
          gs_tmul(k, dzs_k[k], g3);
#pragma unroll
          for (int c = 0; c < 3; ++c) ek[k][c] = -(kap * dy[k][c] + ut[c] + g3[c] + RK(k, c));
        }
        if (MODE == MODE_CADMM) {
          double kp[6];
          Kmul(dpi, kp);
#pragma unroll
          for (int r = 0; r < 6; ++r) ef[r] = P.rho * dwv[r] + kp[r] + RF(r);
        } else if (MODE == MODE_DD) {
#pragma unroll
          for (int r = 0; r < 6; ++r) ef[r] = dpi[r] + RF(r);
        } else {
#pragma unroll
          for (int r = 0; r < 6; ++r) ef[r] = 0.0;
        }
        // stiff rows' equations a_l . lin(du) + (s_l / z_l) dz_l = g_l: their residuals
        double eq = 0.0;
#pragma unroll 1
        for (int j = 0; j < nst; ++j) {
          double* r = srec + j * STIFF_ROW;
          const double q = r[5] - srow(j, du) - r[4] * r[6];
          eq = fmax(eq, fabs(q));
        }
        {  // the linearised system is already solved to rounding: the correction would be noise
           // (stopping here: C4 A/B k_cadmm 11.0 ms with two passes per solve -> 8.9 ms, round 2)
          double en = 0.0, sc = 1.0;
#pragma unroll
          for (int k = 0; k < NB; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) { en = fmax(en, fabs(ek[k][c])); sc = fmax(sc, fabs(RK(k, c))); }
          if constexpr (GRP::on) {
            en = grp.max(en);
            sc = grp.max(sc);
          }
#pragma unroll
          for (int r = 0; r < 6; ++r) { en = fmax(en, fabs(ef[r])); sc = fmax(sc, fabs(RF(r))); }
          en = fmax(en, eq);
#ifdef DAT_IPM_TRACE
          printf("    ref %d en %.3e sc %.3e stiff %d\n", ref, en, sc, nst);
#endif
          if (en <= 1e-12 * sc) {
            DAT_STAT(2);
            if (ref == 0) DAT_STAT_H(0);
            break;
          }

          if (ref == 0) DAT_STAT_H(1);
        }
        ++out.corrs;
        core(ek, ef, nullptr, false, true, dy, dwv, du);
        if (__builtin_expect(nst > 0, 0)) {
          // the stiff-row residuals of the corrected (du, dz), solved into a dz correction (tmp)
#pragma unroll 1
          for (int j = 0; j < nst; ++j) {
            double* r = srec + j * STIFF_ROW;
            r[7] = r[5] - srow(j, du) - r[4] * r[6];
          }
          stiff_update(7, dy, dwv, du);
#pragma unroll 1
          for (int j = 0; j < nst; ++j) srec[j * STIFF_ROW + 6] += srec[j * STIFF_ROW + 7];
          stiff_store();
        }
      }
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        double tks[9], g9[9];
        tks_of(k, tks);
        gs_mul(k, dy[k], g9);
#pragma unroll
        for (int j = 0; j < 9; ++j) dzs_k[k][j] = tks[j] + g9[j];
      }
    };
    // row directions of the current Newton solution
    // (s_l, z_l) of the row: sl, zl (one pair read by the caller)
    auto row_dirs = [&](int l, const double* ddv, const double* ddw, double sl, double zl, double& ds, double& dz) {
      double al3[3], bl;
      rowld(l, al3, bl);
      const double a = dot3x(l, al3, ddv, ddw);
      ds = -(sl - (dot3x(l, al3, dv, dw) + bl)) + a;
      dz = ((smask >> l) & 1u) ? (double)ZW(l) : ZW(l) - zl * frcp(sl) * a;
    };
    // step_len / gap_at / the update take the row-space image (ddv, ddw) = lin(du) of the current
    // direction, computed once per direction by the caller
    auto step_len = [&](const double* ddv, const double* ddw) {
      double a = 1e300;
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        double dss[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) dss[j] = -lrs_k[k][j] - dzs_k[k][j];
        const double l0 = LAM(k, 0);
        if (dss[0] < 0) a = fmin(a, -l0 * frcp(dss[0]));
        if (dzs_k[k][0] < 0) a = fmin(a, -l0 * frcp(dzs_k[k][0]));
        double l4[4];
        lam4(k, 1, l4);
        a = fmin(a, soc_step(l4, dss + 1));
        a = fmin(a, soc_step(l4, dzs_k[k] + 1));
        lam4(k, 5, l4);
        a = fmin(a, soc_step(l4, dss + 5));
        a = fmin(a, soc_step(l4, dzs_k[k] + 5));
      }
      if constexpr (GRP::on) a = grp.min(a);
#pragma unroll
      for (int l = 0; l < NR; ++l) {
        double ds, dz;
        double sl, zl;
        rst.sz(l, sl, zl);
        row_dirs(l, ddv, ddw, sl, zl, ds, dz);
        if (ds < 0) a = fmin(a, -sl * frcp(ds));
        if (dz < 0) a = fmin(a, -zl * frcp(dz));
      }
      return a;
    };
    auto gap_at = [&](double al, const double* ddv, const double* ddw) {
      double g = 0.0;
#pragma unroll
      for (int k = 0; k < NB; ++k)
#pragma unroll
        for (int j = 0; j < 9; ++j) {
          double dss = -lrs_k[k][j] - dzs_k[k][j];
          const double lj = LAM(k, j);
          g += (lj + al * dss) * (lj + al * dzs_k[k][j]);
        }
      if constexpr (GRP::on) g = grp.sum(g);
#pragma unroll
      for (int l = 0; l < NR; ++l) {
        double ds, dz;
        double sl, zl;
        rst.sz(l, sl, zl);
        row_dirs(l, ddv, ddw, sl, zl, ds, dz);
        g += (sl + al * ds) * (zl + al * dz);
      }
      return g;
    };

    // predictor
    DAT_PHASE(4);
    {
      double rsk[NB][9];
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        const double l0 = LAM(k, 0);
        rsk[k][0] = l0 * l0;
        double l4[4];
        lam4(k, 1, l4);
        soc_jprod(l4, l4, rsk[k] + 1);
        lam4(k, 5, l4);
        soc_jprod(l4, l4, rsk[k] + 5);
      }
      newton(rsk, false, nullptr, nullptr, 0.0);
    }
    {
      DAT_PHASE(5);
      double ddva[3], ddwa[3];  // lin(du) of the affine direction: its step, gap and the corrector's term
      lin(du, ddva, ddwa);
      const double aaff = fmin(1.0, step_len(ddva, ddwa));
      const double gaff = gap_at(aaff, ddva, ddwa);
      double sig = gaff / gap;
      sig = fmax(0.0, fmin(1.0, sig * sig * sig));
      const double sigmu = sig * gap * ideg;
      // corrector: rs = lam o lam + dss_aff o dzs_aff - sig mu e
      double rsk[NB][9];
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        double dss[9], c1[4], c2[4];
#pragma unroll
        for (int j = 0; j < 9; ++j) dss[j] = -lrs_k[k][j] - dzs_k[k][j];
        const double l0 = LAM(k, 0);
        rsk[k][0] = l0 * l0 + dss[0] * dzs_k[k][0] - sigmu;
        double l4[4];
        lam4(k, 1, l4);
        soc_jprod(l4, l4, rsk[k] + 1);
        lam4(k, 5, l4);
        soc_jprod(l4, l4, rsk[k] + 5);
        soc_jprod(dss + 1, dzs_k[k] + 1, c1);
        soc_jprod(dss + 5, dzs_k[k] + 5, c2);
#pragma unroll
        for (int j = 0; j < 4; ++j) { rsk[k][1 + j] += c1[j]; rsk[k][5 + j] += c2[j]; }
        rsk[k][1] -= sigmu;
        rsk[k][5] -= sigmu;
      }
      DAT_PHASE(6);
      newton(rsk, true, ddva, ddwa, sigmu);
    }
    DAT_PHASE(7);
    double ddv[3], ddw[3];  // lin(du) of the corrector direction
    lin(du, ddv, ddw);
    double alpha = fmin(1.0, ETA * step_len(ddv, ddw));
    // safeguard: Mehrotra's corrector can increase the gap of a feasible iterate (it then cycles);
    // backtrack until the complementarity gap decreases
    const bool feasible = pres < 1e-8 * NH() && dres < 1e-8 * NQ();
    for (int bt = 0; feasible && bt < 8; ++bt) {
      if (gap_at(alpha, ddv, ddw) <= gap * (1.0 - 0.01 * alpha)) break;
      alpha *= 0.5;
    }
    // update.  ds from the primal equation (keeps G y + s = h exact), dz = W^-1 dzs.
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      double g[9], dz[9], rz[9];
      Gy(dy[k], g);
      winv(k, dzs_k[k], dz);
      rzk_of(k, rz);
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        sk[k][j] = sk[k][j] + alpha * (-rz[j] - g[j]);
        zk[k][j] = zk[k][j] + alpha * dz[j];
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) y[k][c] = y[k][c] + alpha * dy[k][c];
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) w[r] = w[r] + alpha * dwv[r];
    {
#pragma unroll
      for (int l = 0; l < NR; ++l) {
        double ds, dz;
        double sl, zl;
        rst.sz(l, sl, zl);
        row_dirs(l, ddv, ddw, sl, zl, ds, dz);
        rst.set_sz(l, sl + alpha * ds, zl + alpha * dz);
      }
    }
  }
  DAT_PHASE(8);
  DAT_STAT(3 + (out.why < 7 ? out.why : 6));
  // not converged to tol: return the best iterate seen; "optimal" if its scaled primal / dual
  // residuals are within north_star's 1e-7 and its complementarity gap within 1e-6 (strongly graded
  // problems -- the rigid payload's Jl^-1 ~ 50 -- can stall at a 1e-7 gap while the structured Newton
  // solve loses accuracy; the minimiser is then still within ~1e-7 of the oracle's), otherwise
  // inaccurate (the reference holds its previous solution).
  if (BK() < 1e300) {
    record();  // the last iterate of an in-band exit: a start for the next pass all the same
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int c = 0; c < 3; ++c) y[k][c] = best[3 * k + c];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      w[r] = best[3 * NB + r];
      out.pi[r] = best[3 * NB + 6 + r];
      out.u[r] = best[3 * NB + 12 + r];
    }
    out.status = ST_OPTIMAL;
    out.inband = 1;
    out.merit = BK();
  }
  return out;
}

// The reduced QP solve (ipm_attempt).  A C-ADMM agent QP on the tuned start (P.tuned: the warm closed
// loop) that does not converge to tolerance -- diverged, hit max_iter or stalled -- is solved again from
// the conservative start: with consensus multipliers ~1e2-1e3 (the first, cold steps of C5 / C2, a
// stalled ADMM loop) the tuned start's small duals and 0.999 step fraction can stall (full-size C5 on the
// CPU replica, diag/c5_cpu.py: 153 of 29.2 M agent QPs, 2 of them beyond 1e-8; every one of them
// converges from the conservative start in 7-16 iterations).
//
// ROBUST selects the instantiation.  The robust one carries the stiff-row machinery, which cost k_cadmm's fast
// path 36-60 % when compiled into the same kernel (register allocation, C4 A/B), and so does any test for stiff
// rows inside the fast one (7-14 %): a solve is judged by its outcome instead.  A fast solve that does not
// end cleanly -- not converged to tolerance (INACCURATE), or accepted through an in-band iterate -- is the
// symptom of stiff rows (a stalled ADMM loop's agent QPs, barrier weights 1e10-1e19, whose Newton systems
// lose the digits convergence needs) and is redone by the robust instantiation from scratch; the better of
// the two outcomes is kept (ipm_rank).  A clean fast solve meets the tolerance on residuals evaluated from
// the iterate itself, however its Newton systems were solved.
//   IPM_FAST        fast (k_cadmm, which hands a scenario with an unclean solve to k_cadmm_rob; DD, centralized)
//   IPM_ROBUST      robust
//   IPM_FAST_REDO   the C-ADMM agent QP's definition: fast, redone robustly when not clean (k_cadmm_rob, the
//                   single-QP surfaces, host builds)
//   IPM_FAST_R      IPM_FAST as IPM_FAST_REDO's first attempt: the same arithmetic as a template instance of
//                   its own, so that k_cadmm's IPM_FAST instance has one call site per class and is inlined
//                   (shared with k_cadmm_rob's redo it was called, and k_cadmm took 7 % longer)
enum { IPM_FAST = 0, IPM_FAST_R = 1, IPM_ROBUST = 2, IPM_FAST_REDO = 3 };
// 0 converged, 1 in-band OPTIMAL, 2 not OPTIMAL
DAT_HD int ipm_rank(const IPMOut& r) { return r.status != ST_OPTIMAL ? 2 : r.inband ? 1 : 0; }
// a fast solve k_cadmm hands over (IPM_FAST_REDO redoes it): INACCURATE (not the solver-exception branch,
// ST_FAILED: non-finite data), or accepted through an in-band iterate outside Clarabel's own tolerance (an
// in-band accept within it is one Clarabel would return as well)
DAT_HD bool ipm_unclean(const IPMOut& r) {
  return r.status == ST_INACCURATE || (r.status == ST_OPTIMAL && r.inband && r.merit > IPM_CLARABEL_TOL);
}
template <int MODE, int NB, int NR, class SH, class ER, class RT, class RW = RowRegs, unsigned AUXM = 0,
          class GRP = NoGrp, int ROBUST = IPM_FAST, bool WS = false>
DAT_HD IPMOut ipm_solve(const SH& sh, const ER& er, const RT& rt, const QPLane<NB>& P, const double* y0,
                        double y[NB][3], double w[6], double* best, int max_iter, double tol, RW rw = RW{},
                        GRP grp = GRP{}, double* wrec = nullptr, bool wson = false, int clone = 0, int nclone = 1) {
  if constexpr (ROBUST == IPM_FAST_REDO) {
    // trip 0 fast; trip 1 robust (the fast outcome not clean); trip 2 fast once more when the robust outcome
    // is worse (deterministic: it reproduces the first; keeping the first iterate instead would hold another
    // y, w, pi, u live across the robust solve).  One call site per instantiation (ipm_attempt is inlined
    // into each: an instance called from two sites is compiled out of line, which cost k_cadmm 7 %).
    // WS: trip 0 may start warm (the record's flag); trip 2 restores the flag so that it reproduces trip 0.
    IPMOut o, f;
    int done = 0, done_refs = 0, done_corrs = 0;
    const double wflag = (WS && wrec) ? wrec[0] : 0.0;
#pragma unroll 1
    for (int trip = 0;; ++trip) {
      if (WS && wrec && trip == 2) wrec[0] = wflag;
      if (trip == 1 || (wson && wflag == 1.0))  // a warm first trip (and its rerun, trip 2) runs the robust solver
        o = ipm_solve<MODE, NB, NR, SH, ER, RT, RW, AUXM, GRP, IPM_ROBUST, WS>(sh, er, rt, P, y0, y, w, best, max_iter,
                                                                               tol, rw, grp, wrec, wson, clone, nclone);
      else
        o = ipm_solve<MODE, NB, NR, SH, ER, RT, RW, AUXM, GRP, IPM_FAST_R, WS>(sh, er, rt, P, y0, y, w, best, max_iter,
                                                                               tol, rw, grp, wrec, wson, clone, nclone);
      o.iters += done;
      o.refs += done_refs;
      o.corrs += done_corrs;
      if (trip == 2) break;
      if (trip == 0) {
        if (!ipm_unclean(o)) return o;
        f = o;
      } else {
        const int rf = ipm_rank(f), rr = ipm_rank(o);
        if (!(rr > rf || (rr == rf && rr == 1 && o.merit > f.merit))) break;
      }
      done = o.iters;
      done_refs = o.refs;
      done_corrs = o.corrs;
    }
    o.stiff = 1;  // redone robustly
    return o;
  } else {
    constexpr bool ROB = ROBUST == IPM_ROBUST;
    // First start: tuned for the C-ADMM agent QPs of the warm closed loop (P.tuned), conservative otherwise.
    // A tuned attempt that does not converge cleanly is redone from the conservative start (a tuned attempt
    // that has not converged in 20 iterations is not converging: C4's tuned solves take 4.3 on average and
    // at most ~10).  A conservative attempt accepted through an in-band iterate outside Clarabel's 1e-8
    // (rounding-path accidents, ~1 agent QP in 10^7 on C5 and C1: the same QPs on the host build converge
    // from either start) is redone from another start (C-ADMM: tuned; DD / centralized: the conservative
    // start scaled by 10), whose result is taken unless it is worse than the first: then the first start
    // is run once more (the attempts are deterministic, so that reproduces the first result; keeping it in
    // registers instead cost k_cadmm 4 % and k_cent 50 % in register pressure, round 4).  (Not the attempts
    // that end with no in-band iterate: they already ran to max_iter, and a second 50 iterations lengthened
    // C1's slowest wavefront by 45 %.)  One code instance runs every attempt (unroll 1).
    const int first = MODE == MODE_CADMM && P.tuned ? 1 : 0;
    int start = first, trip = 0, done = 0, done_refs = 0, done_corrs = 0;
    int rank0 = 0;  // first attempt: 0 converged, 1 in-band OPTIMAL, 2 not OPTIMAL
    double merit0 = 0.0;
    IPMOut o;
    if constexpr (WS) {
      if (wson && wrec && wrec[0] == 1.0) start = 3;  // the warm attempt first (a converged previous pass)
    }
#pragma unroll 1
    for (;;) {
      // (the tuned start as the first attempt is capped at 20 iterations: see above; the warm one at WS_MAXIT)
      o = ipm_attempt<MODE, NB, NR, SH, ER, RT, RW, AUXM, GRP, ROB, WS>(
          sh, er, rt, P, y0, y, w, best,
          start == 3 ? (max_iter > WS_MAXIT ? WS_MAXIT : max_iter)
                     : start == 1 && trip != 1 && max_iter > 20 ? 20 : max_iter,
          tol, rw, grp, start, wrec, wson, clone, nclone);
      o.iters += done;
      o.refs += done_refs;
      o.corrs += done_corrs;
      if (WS && start == 3) {
        // the warm attempt: converged cleanly, stalled in band within WS_STALL_TOL (or certified), else the cold
        // sequence from its first start
        if ((o.why == 0 && !o.inband) || o.why == 7 || o.status == ST_FAILED || o.status == ST_INFEASIBLE) break;
        start = first;
        done = o.iters;
        done_refs = o.refs;
        done_corrs = o.corrs;
        continue;
      }
      if (trip == 2) break;
      if (trip == 1) {
        const int r1 = ipm_rank(o);
        if (r1 < rank0 || (r1 == rank0 && (r1 != 1 || o.merit <= merit0))) break;
        start = first;  // the second attempt is worse: redo the first
      } else {
        if (o.status == ST_FAILED || o.status == ST_INFEASIBLE) break;
        if (start == 1) {
          if ((o.why == 0 && !o.inband) || (WS && o.why == 7)) break;
          start = 0;
        } else {
          if (!(o.status == ST_OPTIMAL && o.inband && o.merit > IPM_CLARABEL_TOL)) break;
          start = MODE == MODE_CADMM ? 1 : 2;
        }
        rank0 = ipm_rank(o);
        merit0 = o.merit;
      }
      ++trip;
      done = o.iters;
      done_refs = o.refs;
      done_corrs = o.corrs;
    }
    if constexpr (WS) {  // only an OPTIMAL solve (converged or in band) leaves a warm start for the next pass
      if (wrec && o.status != ST_OPTIMAL) wrec[0] = 0.0;
    }
    return o;
  }
}

// Solve with the smallest row-slot instantiation that covers every lane of the wavefront
// (nr_wave: wave-uniform maximum of rows_needed over the lanes taking part).
template <int MODE, int NB, int ROBUST = IPM_FAST, bool WS = false, class SH, class ER, class RT>
DAT_HD IPMOut ipm_solve_rows(int nr_wave, const SH& sh, const ER& er, const RT& rt, const QPLane<NB>& P,
                             const double* y0, double y[NB][3], double w[6], double* best, int max_iter, double tol,
                             double* wrec = nullptr, bool wson = false) {
  if (nr_wave <= NBASE)
    return ipm_solve<MODE, NB, NBASE, SH, ER, RT, RowRegs, 0, NoGrp, ROBUST, WS>(sh, er, rt, P, y0, y, w, best,
                                                                                 max_iter, tol, RowRegs{}, NoGrp{}, wrec, wson);
  return ipm_solve<MODE, NB, DAT_MAXROW, SH, ER, RT, RowRegs, 0, NoGrp, ROBUST, WS>(sh, er, rt, P, y0, y, w, best,
                                                                                    max_iter, tol, RowRegs{}, NoGrp{},
                                                                                    wrec, wson);
}

}  // namespace dat
