// dat_kargs.hpp -- kernel arguments and launch-wide constants shared by the translation units of
// libdat.so (dat.hip: C-ADMM, DD, rollout, C-ABI; dat_cent.hip: the centralized kernel).
#pragma once

#include "dat_qp.hpp"

namespace dat {

constexpr int NMAX = 16;        // largest team the kernels are compiled for
constexpr int NMAX_DD = 16;     // DD: k_dd_setup<0> keeps [H | I] (2 (6n)^2 doubles) in LDS: 144 KB at n = 16
constexpr int IPM_MAX_ITER = 50;
constexpr double IPM_TOL = 1e-10;  // default IPM stopping tolerance (dat_set_qp_tolerance)
// C-ADMM env classes (cadmm_block<C>): 0 no env row, then the largest per-agent env-row count of the
// scenario's QPs <= 2, <= 5, <= DAT_NENV.  Row slots of class C: NBASE + CLASS_ENV[C].
constexpr int NCLS = 4;
__host__ __device__ constexpr int class_env_rows(int c) { return c == 0 ? 0 : c == 1 ? 2 : c == 2 ? 5 : DAT_NENV; }
// k_bucket sort key: class x bin of the scenario's previous ADMM iteration count (1, 2, 3, 4-5,
// 6-9, 10-17, 18-33, >= 34), so that scenarios sharing a wavefront tend to need the same number of
// ADMM passes and the longest ones are claimed first (a 101-iteration scenario claimed last is the
// tail of the whole launch)
constexpr int NAB = 8;   // ADMM / DD iteration bins
constexpr int NPB = 4;  // IPM iteration bins (C-ADMM: the slowest agent QP of the scenario's step)
constexpr int NIB = NAB * NPB;
__host__ __device__ inline int iter_bin(int it) {
  if (it <= 3) return it < 1 ? 0 : it - 1;
  const int lg = 31 - __builtin_clz((unsigned)(it - 2));  // floor(log2(it - 2)) >= 1
  return 2 + lg < NAB - 1 ? 2 + lg : NAB - 1;
}
// IPM iterations of a scenario's slowest agent QP: <= 4, 5, 6-7, >= 8 (six bins measured no gain, round 3)
__host__ __device__ inline int ipm_bin(int it) { return it <= 4 ? 0 : it == 5 ? 1 : it <= 7 ? 2 : 3; }
constexpr int NKEY = NCLS * NIB;
// C-ADMM with a forest, the tail rule (TAIL_PREV, TAIL_PASS: dat_qp.hpp).  k_env_class routes the scenarios
// whose previous step took more than TAIL_PREV passes before the step (sort keys NKEY + class: the tail list
// drained concurrently with k_cadmm); k_cadmm hands a scenario over at the end of the pass after which the rule
// holds (resume record, the hand-over list drained after k_cadmm).
constexpr int NKEY_ALL = NKEY + NCLS;
constexpr int CNT_STRIDE = 5;  // per class: QP solves, IPM iterations, x rows, slot iterations, wave passes
// QPs accepted through the best in-band iterate of a stalled IPM (all kernels), and those of them whose
// scaled residual / gap exceeds Clarabel's own tolerance (INBAND_CLARABEL)
constexpr int CNT_INBAND = NCLS * CNT_STRIDE;
// IPM refinement passes run and corrections applied (all kernels; the executed-flop model)
constexpr int CNT_REF = CNT_INBAND + 2;
// C-ADMM control steps of a scenario finished by k_cadmm_tail (handed over by k_cadmm: an agent QP not clean,
// ipm_unclean, or the tail rule; or routed there before the step)
constexpr int CNT_ROB = CNT_REF + 2;
// tail kernel: [0] ADMM passes (wavefront), [1] sum over passes of the slowest agent QP's IPM iterations,
// [2] scenario-steps routed before the step, [3] agent QPs whose rows were certified infeasible
// (dvl_rows_infeasible, per scenario-step), [4] stall exits, [5] warm-started solves
constexpr int CNT_TAIL = CNT_ROB + 1;
// k_env_class: [0] scenario-steps with a collision flag (example/env_forest.py:158-159), [1] the smallest
// min env distance of the counted steps (fp64 bits: atomicMin orders positive doubles)
constexpr int CNT_COLL = CNT_TAIL + 6;
constexpr int DAT_NCOUNTERS = CNT_COLL + 2;
// class table of the C-ADMM / DD queues (k_bucket), per sub-batch: [0, NCLS) class sizes, [NCLS, 2 NCLS) class
// starts in slist, [2 NCLS, 3 NCLS) queue heads; C-ADMM robust redo: [3 NCLS, 4 NCLS) sizes of the classes'
// robust lists (rlist, same class starts), [4 NCLS, 5 NCLS) their queue heads
// [5 NCLS, 6 NCLS) sizes of the classes' tail-routed stretches of slist (keys NKEY + class), [6 NCLS, 7 NCLS)
// their starts, [7 NCLS, 8 NCLS) their heads
constexpr int SCOUNT_INTS = 8 * NCLS;
// Resume record of a scenario k_cadmm hands to k_cadmm_rob: the fused control step and the ADMM pass it
// stopped in, the IPM-iteration maximum so far, and the mask of its agent lanes whose solve of that pass
// was not clean (the others' results of the pass stand; -1: all, a hand-over between passes by the tail rule)
constexpr int RRES_KSTEP = 0, RRES_PASS = 1, RRES_WMX = 2, RRES_LANES = 3, RRES_INTS = 4;
constexpr double INBAND_CLARABEL = IPM_CLARABEL_TOL;
__device__ inline int inband_loose(const IPMOut& o) { return o.inband && o.merit > INBAND_CLARABEL; }

struct KArgs {
  int B, n, P, S, ppp;  // ppp: params per scenario (1) or broadcast (0)
  const double* params;
  double* state;
  int* counter;
  const double* acc;
  double* fdes;
  const double* trees;
  const int* tree_off;
  const int* scen_forest;
  int nforest;
  const double* mountain;
  int max_iter;
  double res_tol;
  int use_total_res;
  double rho0, tau, rho_max;
  int record_err;
  double *cf, *cfbar, *clam;                 // C-ADMM warm state
  double *dlamF, *dlamM, *dprev, *dHinv;      // DD state
  double* pf;                                 // centralized previous solution
  double* best;                               // lane-private best-iterate records of the IPM
  int* iters;
  int* qstatus;
  double* mind;
  unsigned char* col;
  double* err;
  unsigned long long* counters;  // [0] agent-QP solves, [1] IPM iterations, [2] IPM iterations x active rows
                                 // (C-ADMM: [CNT_STRIDE k + .] per env class k, cadmm_block<k>)
  int G;                         // C-ADMM: scenario slots per k_cadmm wavefront (cadmm_slots)
  int* need;                     // C-ADMM: per-scenario sort key of the step (k_env_class)
  int* ipmx;                     // C-ADMM: IPM iterations of the scenario's slowest agent QP, previous step
  int* slist;                    // C-ADMM: scenario ids grouped by class, then by key (k_bucket)
  int* scount;                   // C-ADMM: [0, NCLS) class sizes, [NCLS, 2 NCLS) class start offsets
  int* qhead;                    // C-ADMM: [NCLS] queue heads of the classes (reset by k_bucket)
  int* rlist;                    // C-ADMM: scenarios whose step k_cadmm_rob redoes, by class (class starts as slist)
  int* rres;                     // C-ADMM: per listed scenario, where k_cadmm_rob resumes it (RRES_* fields)
  double* erows;                 // C-ADMM: env rows of the step per agent (k_env_class -> k_cadmm), SoA:
                                 //   [(4 j + c) B n + sc n + i], c < 3: lhs, c = 3: rhs
  unsigned* emask;               // C-ADMM: [B n] env row mask of the step
  int ll_kind;                   // low-level SO(3) law: LL_PD or LL_SM (dat_set_low_level)
  double qp_tol;                 // IPM stopping tolerance of every QP (dat_set_qp_tolerance)
  int ksteps;                    // C-ADMM / DD without a forest: control steps fused into one drain
                                 // (dat_control_steps; acc then holds ksteps x B x 6 values)
  double* wrec;                  // C-ADMM tail: per agent lane the warm-start record (WREC_SIZE doubles)
  int tail_prev, tail_pass;      // C-ADMM: the tail rule (TAIL_PREV / TAIL_PASS with a forest, INT_MAX without)
  int route;                     // C-ADMM, one sub-batch: wedged scenarios go to the tail before the step (k_env_class)
  int tmode;                     // k_cadmm_tail: 0 the hand-over lists (rlist), 1 the tail-routed stretch of slist
};

// wave-uniform maximum (every lane of the wavefront must execute it)
__device__ inline int wave_max(int v) {
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off));
  return v;
}

__device__ inline const double* prm_of(const KArgs& a, int sc) { return a.params + (a.ppp ? (size_t)sc * a.P : 0); }

__device__ inline void forest_of(const KArgs& a, int sc, const double** trees, int* nt) {
  *trees = nullptr;
  *nt = 0;
  if (a.nforest <= 0) return;
  int f = a.scen_forest ? a.scen_forest[sc] : 0;
  if (f < 0 || f >= a.nforest) return;
  *trees = a.trees + 3 * (size_t)a.tree_off[f];
  *nt = a.tree_off[f + 1] - a.tree_off[f];
}

// centralized control step of every scenario (dat_cent.hip): k_cent<W>, one group of W = 4 / 8 / 16
// lanes per scenario (one agent's force per lane), 3 <= n <= NMAX_CENT
constexpr int NMAX_CENT = 16;
int cent_group_width(int n);
hipError_t launch_cent(int n, int B, hipStream_t stream, const KArgs& a);

}  // namespace dat
