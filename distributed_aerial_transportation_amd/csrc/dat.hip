// dat.hip -- gfx950 kernels and the C-ABI (include/dat.h) of the batched agent-QP solver.
//
// Kernels (all fp64, no MFMA -- every contraction is <= 6 wide):
//   k_cadmm    C-ADMM control step: one 64-lane wavefront holds floor(64/n) scenarios x n agents,
//              one lane per agent QP; the whole ADMM loop (reference control/rqp_cadmm.py:631-675)
//              runs on chip: agent QPs (ipm_solve), consensus mean / residual through LDS, dual
//              update; per-scenario convergence masks.
//   k_dd_setup DD quasi-Newton matrix H = A Q^-1 A' and its inverse per scenario, in LDS
//              (control/rqp_dd.py:513-555, 634-657).
//   k_dd       DD control step: prices, agent QPs, consensus error, dual ascent through H^-1
//              (control/rqp_dd.py:659-752).
//   k_cent     centralized QP, one lane group per scenario and one lane per agent's force
//              (control/rqp_centralized.py:436-448): dat_cent.hip.
//   k_rollout_agents  low-level SO(3) law + dynamics + Lie integration, one lane per agent.
//   k_desired  forest desired-acceleration law (example/rqp_example.py:33-59).
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>
#include <vector>
#include <algorithm>
#include <chrono>

#include "../../include/dat.h"
#include "dat_kargs.hpp"

using namespace dat;

#ifdef DAT_CAPTURE_LOOSE
// development builds only (tools/capture_loose.py): the inputs of the tail's agent QPs accepted in band beyond
// Clarabel's 1e-8 -- [0] scenario, [1] agent, [2] ADMM pass, [3] rho, [4] previous step's passes, [5] forest,
// [6] merit, [7] fused step, [8, 14) acc_des, then the state (S), the agent's multipliers (3n) and the mean (3n)
namespace dat {
constexpr int CAP_MAX = 64, CAP_DOUBLES = 320;
__device__ double g_cap[CAP_MAX][CAP_DOUBLES];
__device__ unsigned int g_ncap;
}  // namespace dat
#endif

namespace {

thread_local std::string g_err;

int fail(const std::string& m) {
  g_err = m;
  return -1;
}

#define HIPCHK(x)                                                                 \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) return fail(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

// ------------------------------------------------------------------------------------------------
// C-ADMM
// ------------------------------------------------------------------------------------------------
// A control step runs as three launches:
//   k_env_class   one lane per agent: env CBF rows of the step (they depend on the state only, so
//                 they are fixed for the whole ADMM loop, control/rqp_cadmm.py:305), per-scenario
//                 env class (the largest env-row count among its agents' QPs: 0, <= 2, <= 5,
//                 <= 10), collision, min env distance, and a sort key (class, previous step's
//                 ADMM iteration count); the rows go to HBM (erows / emask, SoA over agents) and
//                 k_cadmm loads them when a slot takes the scenario instead of re-running the query;
//   k_bucket      counting sort of the scenario ids by key (one queue per class; the order within a
//                 key is not fixed, see k_bucket);
//   k_cadmm       persistent blocks (CUs x 4) drain the class queues, classes 3, 2, 1, 0 in turn,
//                 each with its own row-slot instantiation of the IPM (3 + {10, 5, 2, 0} slots:
//                 the register footprint follows the rows the class needs); a scenario slot that
//                 stops is refilled from the queue (cadmm_drain).
// Each scenario's arithmetic does not depend on the scenarios it shares a wavefront with (padding
// rows add exact zeros), so the regrouping does not change any result.
//
// LDS layout of one 64-lane block (G = floor(64/n) scenarios).  Per-lane records use an odd
// stride in doubles so that the 32 lanes of a ds_read_b64 group fall on distinct bank pairs.
//   fbar G x 3n    consensus mean
//   Rt   G x 9n    hat(r_com_j) Rl'
//   sh   G x QPShared (u-maps, packed Hessians, base rows, K)            done / sid / wmx: G ints each
//   area, laid out per env class:
//     rows  the IPM's row state (RowLds: s, z, zw of NR slots x 64 lanes, 3 NR x 64 doubles); the
//           consensus exchange slots red (64 x RDS) alias it: they are used only between solves
//     env   EnvLdsN image of the class's env slots (structure of arrays over the 64 lanes)
// The row state goes to LDS for classes 1 and 2 when their image fits the 40 KB a wavefront may
// hold at four wavefronts per CU (cadmm_rows_lds); class 0 (3 slots) and class 3 (13 slots) keep it
// in registers.  n = 6: class 0 34.8 KB (rows + aux slots), 1 27.3 KB, 2 37.8 KB, 3 39.3 KB (C4 A/B,
// k_cadmm ms: rows of classes 0-2 in LDS 5.53, classes 1-2 5.45, class 2 only 5.51).  Round 4 trimmed
// the exchange slots (RDS 9 -> 7) and the per-slot ints (3 x 64 -> 3 G): class 3's carve was 41.9 KB,
// which with the 256 B of static LDS left room for three workgroups per CU (one SIMD idle); four fit after
// the trim (C4 A/B 3.83 / 3.80 -> 3.72 / 3.77 ms per step), and the budget then went to classes 1 and 2's
// aux groups at three per CU instead (LDS_WAVE_BUDGET).
// DD warm start: from DD pass DD_WARM_PASS of a step on, the agent QPs start from the previous pass's iterate (a
// long DD chain -- C3's slowest scenario runs the reference's cap of 100 passes at every step, the step's
// critical path; ordinary steps take ~4 passes and never reach it).  Its agent QP differs from the previous pass's
// only in the prices.  From pass 1 on it cut C3 further but left the n = 3 golden DD error sequence (25 fixed
// passes) 3e-4 off (bound 1e-4): a warm start lands elsewhere in a weakly convex QP's near-flat minimiser set than
// the reference's cold solve.  Same-call A/B (C3, ms per step): 21.7 -> 13.4 with DD_WS_MU 1e-3 (1e-2: 14.3);
// every DD parity test green (golden sequences, the DD hard stretch, the 100 s loop to the same horizon).
// (DAT_DD_WARM=0: the round-5 cold DD, A/B builds.)
#ifndef DAT_DD_WARM
#define DAT_DD_WARM 1
#endif
constexpr int DD_WARM_PASS = 30;
constexpr int RDS = 7;  // consensus exchange slots per lane: mean (3) or F / M totals (6), total residual at [6]
// LDS budget of one k_cadmm workgroup: 53 KB = three per CU.  Four per CU (40 KB) bought ~2 % (§5 of
// DESIGN.md, round 4); the 13 KB more per workgroup hold classes 1 and 2's IPM aux groups in LDS
// instead (C4 A/B 3.79 / 3.80 -> 3.75 / 3.74 ms per step).
constexpr size_t LDS_WAVE_BUDGET = 53 * 1024;
__host__ __device__ constexpr int cadmm_nr(int cls) { return NBASE + class_env_rows(cls); }
// G: scenario slots per wavefront (cadmm_slots)
// doubles rounded up to a 16-byte multiple: every LDS region starts 16-byte aligned (pair reads)
__host__ __device__ constexpr size_t al2(size_t d) { return (d + 1) & ~(size_t)1; }
// per-slot ints done / sid / wmx (G each), rounded to 16 bytes
__host__ __device__ constexpr int slot_ints(int G) { return (3 * G + 3) & ~3; }
__host__ __device__ inline size_t cadmm_fixed_bytes(int n, int G) {
  return sizeof(double) * (al2((size_t)G * 3 * n) + (size_t)G * RT_STRIDE * n) + sizeof(QPShared) * (size_t)G +
         sizeof(int) * (size_t)slot_ints(G);
}
// IPM per-iteration quantities moved to LDS aux slots (ipm_solve AUXM) per env class, when the class's
// carve still fits the budget: class 0 all groups (its 3 row slots leave room; class-0 probe scratch
// traffic 145 -> 23 ops per IPM pass; A/B on MI355X: C2 12.1 -> 11.0 ms, C5 80.7 -> 73.2 ms per step);
// classes 1 and 2 all groups since round 4, at three workgroups per CU (LDS_WAVE_BUDGET; class 3's 13
// row slots do not fit).
// C-ADMM consensus mean and residual read agent-major, the three components of a block together
// (bitwise equal to the component-major loops; C4 A/B: k_cadmm 3.68 / 3.63 -> 3.57 / 3.54 ms)
__host__ __device__ constexpr unsigned cadmm_auxm(int cls) { return cls < NCLS - 1 ? 15u : 0u; }
// row-state placement of a class: 0 registers, 1 LDS rows, 2 LDS rows + the class's aux slots, 3 LDS rows + all
// aux slots (k_cadmm_tail: one scenario per wavefront, latency-bound, every class in LDS)
constexpr unsigned TAIL_AUXM = 15u;
__host__ __device__ constexpr int cadmm_aux_doubles(int cls, int rmode) {
  return rmode == 2 ? ipm_aux_doubles(1, cadmm_auxm(cls)) : rmode == 3 ? ipm_aux_doubles(1, TAIL_AUXM) : 0;
}
__host__ __device__ inline size_t cadmm_area_doubles(int cls, int rmode) {
  const size_t rows = rmode ? (size_t)row_lds_doubles(cadmm_nr(cls), cadmm_aux_doubles(cls, rmode)) : 0;
  return (rows > 64 * RDS ? rows : 64 * RDS) + (size_t)env_lds_doubles(class_env_rows(cls));
}
// row state of class cls in LDS: with the class's aux slots when that carve fits the budget, else rows
// alone for classes ROWLDS_MIN_CLS .. 2; class 3 (13 slots) never.  Few row slots without aux slots
// are cheaper in registers: an LDS row access costs an LDS round trip, which pays only once the rows
// would otherwise spill.
constexpr int ROWLDS_MIN_CLS = 1;
__host__ __device__ inline int cadmm_row_mode(int n, int G, int cls) {
  if (cls >= NCLS - 1) return 0;
  if (cadmm_auxm(cls) && cadmm_fixed_bytes(n, G) + sizeof(double) * cadmm_area_doubles(cls, 2) <= LDS_WAVE_BUDGET)
    return 2;
  if (cls >= ROWLDS_MIN_CLS && cadmm_fixed_bytes(n, G) + sizeof(double) * cadmm_area_doubles(cls, 1) <= LDS_WAVE_BUDGET)
    return 1;
  return 0;
}
// dynamic LDS of a k_cadmm workgroup: the largest carve of the env classes that can occur (without a
// forest every scenario is class 0, so the launch needs only that carve and more workgroups fit a CU)
__host__ __device__ inline size_t cadmm_lds_bytes(int n, int G, int max_cls = NCLS - 1) {
  size_t m = 0;
  for (int c = 0; c <= max_cls; ++c) {
    const size_t b = cadmm_fixed_bytes(n, G) + sizeof(double) * cadmm_area_doubles(c, cadmm_row_mode(n, G, c));
    m = b > m ? b : m;
  }
  return m;
}
// dynamic LDS of a k_cadmm_tail workgroup (one scenario slot, rmode 3), with the n lanes' IPM scratch records
// (best iterate, stiff-row columns and Schur factor: best_size(1) doubles each) behind the class's area: the
// robust solver's stiff-row loops read and write them at every iteration, an LDS round trip instead of L2 / HBM
// k_cadmm_tail: bit-identical clones per agent lane (the lanes a one-scenario wavefront leaves idle), one per
// stiff-row column of the robust solver at most
__host__ __device__ inline int tail_clones(int n) {
  const int v = 64 / (n > 0 ? n : 1);
  return v < 1 ? 1 : v < IPM_NSTIFF ? v : IPM_NSTIFF;
}
__host__ __device__ inline size_t cadmm_tail_lds_bytes(int n, int max_cls = NCLS - 1) {
  size_t m = 0;
  for (int c = 0; c <= max_cls; ++c) {
    const size_t b = cadmm_fixed_bytes(n, 1) + sizeof(double) * (cadmm_area_doubles(c, 3) + al2((size_t)n * best_size(1)));
    m = b > m ? b : m;
  }
  return m;
}
struct CadmmLds {
  double *fbar, *Rt, *red, *rows;
  QPShared* sh;
  double* env;
  int* done;  // per slot: the scenario stopped in this pass
  int* sid;   // per slot: scenario id, -1 empty, -2 retired (queue drained)
  int* wmx;   // per slot: IPM iterations of the scenario's slowest agent QP so far this step
};
__device__ inline CadmmLds cadmm_carve(double* smem, int n, int G, int cls, int rmode) {
  CadmmLds L;
  L.fbar = smem;
  L.Rt = L.fbar + al2(G * 3 * n);
  L.sh = (QPShared*)(L.Rt + G * RT_STRIDE * n);
  L.done = (int*)(L.sh + G);
  L.sid = L.done + G;
  L.wmx = L.sid + G;
  L.rows = (double*)(L.done + slot_ints(G));
  L.red = L.rows;
  const int ra = rmode ? row_lds_doubles(cadmm_nr(cls), cadmm_aux_doubles(cls, rmode)) : 0;
  L.env = L.rows + (ra > 64 * RDS ? ra : 64 * RDS);
  return L;
}

// order-preserving unsigned key of a double (negative values included) for the running minimum of the env
// distance (atomicMin on the key): the sign bit flipped for x >= 0, every bit for x < 0
__host__ __device__ inline unsigned long long dist_key(double x) {
  unsigned long long b;
  memcpy(&b, &x, sizeof(b));
  return (b >> 63) ? ~b : (b | (1ull << 63));
}
__host__ __device__ inline double dist_of_key(unsigned long long k) {
  const unsigned long long b = (k >> 63) ? (k & ~(1ull << 63)) : ~k;
  double x;
  memcpy(&x, &b, sizeof(x));
  return x;
}

// env class of one agent QP: 0 if it carries no env row, otherwise the smallest class whose slots
// hold the rows set_env_rows keeps (nonzero rows, compacted).  An all-zero row with a positive
// right-hand side (0 >= rhs > 0: the reference's QP is infeasible, set_env_rows flags it) also
// needs an env class.
__device__ inline int env_class_of(unsigned emask, const double lhs[DAT_NENV][3], const double rhs[DAT_NENV]) {
  bool need = false;
  int k = 0;
#pragma unroll
  for (int j = 0; j < DAT_NENV; ++j) {
    const bool on = (emask >> j) & 1u;
    const bool zero = lhs[j][0] == 0.0 && lhs[j][1] == 0.0 && lhs[j][2] == 0.0;
    need = need || (on && (!zero || rhs[j] > 0.0));
    k += (on && !zero) ? 1 : 0;
  }
  if (!need) return 0;
  int c = 1;
  while (c < NCLS - 1 && k > class_env_rows(c)) ++c;
  return c;
}

// Env rows of the n agents of each scenario of a 64-lane block, computed cooperatively
// (control/rqp_cadmm.py:307-373 via env_rows' arithmetic).  The payload capsule and the x-window of
// candidate trees are the same for every agent of a scenario; only the camera-cone filter differs
// (cos 100 deg: most agents see most trees).  Lane i of a scenario evaluates trees base + i of each
// chunk of n candidates -- range test, capsule_tree distance and the CBF row, once per tree instead
// of once per agent that sees it -- and publishes them in LDS; then every lane runs its own cone
// filter and sorted insertion over the chunk in tree order.  Same per-tree arithmetic and insertion
// order as env_rows (the rows are bitwise identical; test_gpu_env_rows / test_gpu_c4).
// Must be called by every lane of the block (barriers inside).
constexpr int ENV_CE = 8;  // published entry: in range, c.x, c.y, dd, l3[3], r1
// LDS stride of a published entry: 9 doubles (18 dwords), so the 32 lanes of a ds_*_b64 half-wave
// start on 32 distinct even banks (a stride of 8 doubles put 64 lanes on 4 bank pairs: 16-way conflicts)
constexpr int ENV_CS = ENV_CE + 1;
__device__ EnvOut env_rows_coop(const double* prm, int n, const double* st, const double* trees, int ntree, int i,
                                int ls, bool valid, double alpha_env, unsigned* mask, double lhs[DAT_NENV][3],
                                double rhs[DAT_NENV], double* ent /* LDS: 64 x ENV_CS */) {
  EnvOut out;
  out.collision = 0;
  out.min_env_dist = valid ? prm[DAT_P_VISR] : 0.0;
  *mask = 0u;
#pragma unroll
  for (int j = 0; j < DAT_NENV; ++j) { lhs[j][0] = lhs[j][1] = lhs[j][2] = 0.0; rhs[j] = 0.0; }
  const bool any = valid && trees != nullptr && ntree > 0;
  bool dead = !any;  // this agent keeps no row (it still evaluates its share of the trees)
  double xl[3] = {0, 0, 0}, vl[3] = {0, 0, 0}, vdir[3] = {0, 0, 0}, seg[3] = {0, 0, 0}, ctr[3] = {0, 0, 0};
  double h = 0.0, speed = 0.0, maxdec = 1.0, reach = 0.0, rc = 0.0, deps = 0.0, cosang = 0.0;
  double cam[2] = {0, 0}, dir[2] = {0, 0};
  int t0 = 0;
  if (any) {
    const double* xlp = st + DAT_S_XL(n);
    const double* vlp = st + DAT_S_VL(n);
    const double* Rl = st + DAT_S_RL(n);
    for (int c = 0; c < 3; ++c) { xl[c] = xlp[c]; vl[c] = vlp[c]; }
    maxdec = prm[DAT_P_MAXDEC];
    rc = prm[DAT_P_COLR];
    deps = prm[DAT_P_DISTEPS];
    cosang = prm[DAT_P_COSCONE];
    const double v2 = dot3(vl, vl);
    h = 0.5 * v2 / maxdec;
    speed = sqrt(v2);
    ctr[0] = xl[0]; ctr[1] = xl[1]; ctr[2] = xl[2];
    if (speed != 0.0) {
      vdir[0] = vl[0] / speed; vdir[1] = vl[1] / speed; vdir[2] = vl[2] / speed;
      seg[0] = h * vdir[0]; seg[1] = h * vdir[1]; seg[2] = h * vdir[2];
      ctr[0] += 0.5 * seg[0]; ctr[1] += 0.5 * seg[1]; ctr[2] += 0.5 * seg[2];
    }
    const double* r = prm + DAT_P_R(n) + 3 * i;
    double Rr[3];
    mv3(Rl, r, Rr);
    cam[0] = xl[0] + Rr[0];
    cam[1] = xl[1] + Rr[1];
    const double dx = cam[0] - xl[0], dy = cam[1] - xl[1];
    const double nn = sqrt(dx * dx + dy * dy);
    if (nn == 0.0) {
      out.collision = 1;
      dead = true;
    } else {
      dir[0] = dx / nn; dir[1] = dy / nn;
    }
    reach = prm[DAT_P_VISR] + DAT_BARK_RADIUS;
    for (int len = ntree; len > 0;) {
      int half = len >> 1;
      if (trees[3 * (t0 + half)] < ctr[0] - reach) { t0 += half + 1; len -= half + 1; } else { len = half; }
    }
  }
  double bd[DAT_NENV];
#pragma unroll
  for (int j = 0; j < DAT_NENV; ++j) bd[j] = 1e300;
  int cnt = 0;
  double dmin = 1e300;
  double* mine = ent + (size_t)threadIdx.x * ENV_CS;
  const double* grp = ent + (size_t)(ls * n) * ENV_CS;
  for (int base = t0;; base += n) {
    // this lane's tree of the chunk
    const int t = base + i;
    const bool cand = any && t < ntree && trees[3 * t] <= ctr[0] + reach;
    double e[ENV_CE] = {0, 0, 0, 1e300, 0, 0, 0, 0};
    if (cand) {
      const double* c = trees + 3 * t;
      const double ex = ctr[0] - c[0], ey = ctr[1] - c[1], ez = ctr[2] - c[2];
      if (!(sqrt(ex * ex + ey * ey + ez * ez) > prm[DAT_P_VISR] + DAT_BARK_RADIUS)) {
        double p1[3], p2[3];
        const double dd = capsule_tree(xl, seg, rc, c, p1, p2);
        double l3[3] = {0, 0, 0}, r1 = 0.0;
        if (dd > 1e-4 && speed > 0.0) {
          double rel[3] = {p1[0] - xl[0], p1[1] - xl[1], p1[2] - xl[2]};
          double proj = fmax(0.0, fmin(h, dot3(rel, vdir)));
          double mt = sqrt(2.0 * (h - proj) / maxdec);
          mt = fmax(0.0, speed / maxdec - mt);
          if (mt < 1e-12 * speed / maxdec) mt = 0.0;
          double nr[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
          double nn = sqrt(dot3(nr, nr));
          nr[0] /= nn; nr[1] /= nn; nr[2] /= nn;
          l3[0] = nr[0] * mt; l3[1] = nr[1] * mt; l3[2] = nr[2] * mt;
          r1 = -alpha_env * (dd - deps) - dot3(nr, vl);
        }
        e[0] = 1.0; e[1] = c[0]; e[2] = c[1]; e[3] = dd;
        e[4] = l3[0]; e[5] = l3[1]; e[6] = l3[2]; e[7] = r1;
      }
    }
    // every lane of the block takes part in the barriers; the loop ends when no lane had a candidate
    if (!__syncthreads_or(cand)) break;
#pragma unroll
    for (int k = 0; k < ENV_CE; ++k) mine[k] = e[k];
    __syncthreads();
    if (!dead) {
      for (int j = 0; j < n; ++j) {  // the chunk in tree order
        const double* q = grp + (size_t)j * ENV_CS;
        if (q[0] == 0.0) continue;
        const double tx = q[1] - cam[0], ty = q[2] - cam[1];
        const double nn = sqrt(tx * tx + ty * ty);
        if (nn > 0.0 && (tx / nn * dir[0] + ty / nn * dir[1]) < cosang) continue;
        const double dd = q[3];
        if (dd < 1e-4) out.collision = 1;
        dmin = fmin(dmin, dd);
        ++cnt;
        int pos = 0;
#pragma unroll
        for (int jj = 0; jj < DAT_NENV; ++jj) pos += (bd[jj] <= dd) ? 1 : 0;
        if (pos >= DAT_NENV) continue;
#pragma unroll
        for (int jj = DAT_NENV - 1; jj >= 1; --jj) {
          if (jj > pos) {
            bd[jj] = bd[jj - 1];
            lhs[jj][0] = lhs[jj - 1][0]; lhs[jj][1] = lhs[jj - 1][1]; lhs[jj][2] = lhs[jj - 1][2];
            rhs[jj] = rhs[jj - 1];
          }
        }
#pragma unroll
        for (int jj = 0; jj < DAT_NENV; ++jj) {
          if (jj == pos) {
            bd[jj] = dd;
            lhs[jj][0] = q[4]; lhs[jj][1] = q[5]; lhs[jj][2] = q[6];
            rhs[jj] = q[7];
          }
        }
      }
    }
    __syncthreads();  // the chunk is consumed before the next one is published
  }
  if (!dead && cnt > 0 && speed > 0.0) {
    out.min_env_dist = dmin;
    unsigned m = 0u;
#pragma unroll
    for (int j = 0; j < DAT_NENV; ++j)
      if (bd[j] < 1e299 && bd[j] > 1e-4) m |= 1u << j;
    *mask = m;
  }
  return out;
}

// Two wavefronts per SIMD (256 VGPRs, 104 B/lane of scratch for the sorted row slots): the build without
// the bound (290 registers, no scratch, one wavefront per SIMD) measured slower, C4 A/B 3.58 / 3.61 ->
// 3.70 / 3.80 ms per step (round 4).  Three or four wavefronts per SIMD (168 / 128 VGPRs, the sorted row
// slots spilled) measured 3.2-3.6x slower by kernel trace: 0.24 -> 0.77 / 0.87 ms (round 4).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_env_class(KArgs a) {
  __shared__ int nd[64], cl[64];
  __shared__ double md[64];
  __shared__ double ent[64 * ENV_CS];
  const int n = a.n, G = 64 / n, NT = G * n;
  const int lane = threadIdx.x;
  const int ls = lane / n, i = lane - ls * n;
  const int sc = blockIdx.x * G + ls;
  const bool valid = (lane < NT) && (sc < a.B);
  int need = 0, col = 0;
  double dist = 1e300;
  const double* prm = valid ? prm_of(a, sc) : a.params;
  const double* trees = nullptr;
  int nt = 0;
  if (valid) forest_of(a, sc, &trees, &nt);
  unsigned emask;
  double lhs[DAT_NENV][3], rhs[DAT_NENV];
  EnvOut e = env_rows_coop(prm, n, valid ? a.state + (size_t)sc * a.S : nullptr, trees, nt, i, ls, valid,
                           prm[DAT_P_AENVD], &emask, lhs, rhs, ent);
  if (valid) {
    need = env_class_of(emask, lhs, rhs);
    col = e.collision;
    dist = e.min_env_dist;
    // hand the rows to k_cadmm (lanes hold consecutive agents: every store is coalesced)
    const size_t NA = (size_t)a.B * n, g = (size_t)sc * n + i;
    a.emask[g] = emask;
#pragma unroll
    for (int j = 0; j < DAT_NENV; ++j) {
      if (!((emask >> j) & 1u)) continue;  // only the slots the mask marks are read back
      a.erows[(4 * j + 0) * NA + g] = lhs[j][0];
      a.erows[(4 * j + 1) * NA + g] = lhs[j][1];
      a.erows[(4 * j + 2) * NA + g] = lhs[j][2];
      a.erows[(4 * j + 3) * NA + g] = rhs[j];
    }
  }
  nd[lane] = need;
  cl[lane] = col;
  md[lane] = dist;
  __syncthreads();
  int cnum = 0;
  double cmin = 1e300;
  if (valid && i == 0) {
    int cls = 0, c = 0;
    double m = prm_of(a, sc)[DAT_P_VISR];
    for (int k = 0; k < n; ++k) {
      cls = max(cls, nd[ls * n + k]);
      c |= cl[ls * n + k];
      m = fmin(m, md[ls * n + k]);
    }
    // previous step's ADMM iterations, then its slowest agent QP's IPM iterations: within a class the
    // longest scenarios are claimed first and scenarios sharing a wavefront tend to need similar
    // numbers of ADMM passes and of IPM iterations per pass (a pass lasts as long as its slowest lane)
    const int bin = NPB * iter_bin(a.iters[sc]) + ipm_bin(a.ipmx[sc]);
    // a scenario wedged in a stall (previous step > TAIL_PREV passes) goes to the tail (key NKEY + class); with
    // sub-batches it stays in k_cadmm's queue, which hands it over after its first pass (the tail rule), the
    // same arithmetic
    a.need[sc] = a.route && a.iters[sc] > a.tail_prev ? NKEY + cls : cls * NIB + (NIB - 1 - bin);
    a.col[sc] = (unsigned char)c;
    a.mind[sc] = m;
    cnum = c;
    cmin = m;
  }
  // collisions and the smallest env distance of the step (bench stats; one atomic per wavefront, the minimum only
  // when it undercuts the running one)
  for (int off = 32; off > 0; off >>= 1) {
    cnum += __shfl_xor(cnum, off);
    cmin = fmin(cmin, __shfl_xor(cmin, off));
  }
  if (lane == 0) {
    if (cnum) atomicAdd(a.counters + CNT_COLL, (unsigned long long)cnum);
    // (an order-preserving key of the signed distance: a collided payload's distance is negative)
    unsigned long long* pm = a.counters + CNT_COLL + 1;
    const unsigned long long key = dist_key(cmin);
    if (cmin == cmin && key < *(volatile unsigned long long*)pm) atomicMin(pm, key);
  }
}

// Counting sort of the scenario ids by key (need[] in [0, NKEY)): list holds the ids of key 0, then
// key 1, ...; count[c] / count[NCLS + c] = size / start of env class c (keys c NIB .. c NIB + NIB -
// 1), count[2 NCLS + c] = 0 (queue head).  Within a class the key is the previous step's (ADMM
// iterations, slowest agent's IPM iterations) bin, in decreasing order, so the longest scenarios are
// claimed first.  One BUCKET_T-thread workgroup, coalesced strided reads, LDS atomics for the
// histogram and the scatter cursors: the order within a key is not fixed, which only changes which
// scenarios share a wavefront, never a scenario's arithmetic (the capped-grid test compares two
// different groupings bitwise).
constexpr int BUCKET_T = 1024;
static_assert(NKEY_ALL <= BUCKET_T, "k_bucket initialises one key per thread");
__global__ __launch_bounds__(BUCKET_T) void k_bucket(int B, const int* need, int* list, int* count) {
  __shared__ int hist[NKEY_ALL], kstart[NKEY_ALL], cursor[NKEY_ALL], tot[NKEY_ALL];
  const int t = threadIdx.x;
  if (t < NKEY_ALL) { hist[t] = 0; cursor[t] = 0; }
  __syncthreads();
  for (int q = t; q < B; q += BUCKET_T) atomicAdd(&hist[min(max(need[q], 0), NKEY_ALL - 1)], 1);
  __syncthreads();
  if (t == 0) {
    int st = 0;
    for (int k = 0; k < NKEY_ALL; ++k) { kstart[k] = st; tot[k] = hist[k]; st += hist[k]; }
  }
  __syncthreads();
  for (int q = t; q < B; q += BUCKET_T) {
    const int key = min(max(need[q], 0), NKEY_ALL - 1);
    list[kstart[key] + atomicAdd(&cursor[key], 1)] = q;
  }
  if (t == 0) {
    int st = 0;
    for (int cl = 0; cl < NCLS; ++cl) {
      int sz = 0;
      for (int b = 0; b < NIB; ++b) sz += tot[cl * NIB + b];
      count[cl] = sz;
      count[NCLS + cl] = st;
      count[2 * NCLS + cl] = 0;  // queue head of the class (k_cadmm)
      count[3 * NCLS + cl] = 0;  // hand-over list of the class (k_cadmm -> k_cadmm_tail) and its head
      count[4 * NCLS + cl] = 0;
      st += sz;
    }
    for (int cl = 0; cl < NCLS; ++cl) {  // the tail-routed stretches (keys NKEY + class) behind them
      count[5 * NCLS + cl] = tot[NKEY + cl];
      count[6 * NCLS + cl] = kstart[NKEY + cl];
      count[7 * NCLS + cl] = 0;
    }
  }
}

// Work counters of one wavefront, flushed once per class it drained.
struct WaveCounters {
  long long qp = 0, ipm = 0, rowit = 0;  // lane-level: agent-QP solves, IPM iterations, x active rows
  long long inband = 0, loose = 0;      // lane-level: solves accepted through the best in-band iterate
  long long refs = 0, corrs = 0;        // lane-level: IPM refinement passes, corrections applied
  long long slot = 0, pass = 0;         // wave-level: sum of (max lane IPM iterations) per pass, passes
  long long cert = 0, stall = 0, warm = 0;  // k_cadmm_tail, lane-level: certified infeasible, stall exits, warm starts
};

// A persistent 64-lane block drains the queue of env class CLS (the class's stretch of the sorted
// scenario list, claimed one scenario at a time through a.qhead[CLS]).  The block holds G scenario
// slots of n lanes; a slot whose scenario stops is refilled with the next scenario of the queue at
// the start of the next ADMM pass, so a wavefront no longer idles until its slowest scenario of a
// fixed group stops (SIMD occupancy: dat_get_class_occupancy).  A scenario's arithmetic does not
// depend on which slot or wavefront runs it.
// Every agent QP is solved as ipm_solve IPM_FAST_REDO defines it: the fast solver, redone by the robust one
// when it does not end cleanly (ipm_unclean).  RB = false (k_cadmm) carries only the fast solver (IPM_FAST): a
// scenario one of whose agent QPs does not end cleanly leaves at the end of that pass's solves with a resume
// record (rres) and goes to its class's hand-over list; so does a scenario whose next pass falls under the tail
// rule (TAIL_PREV / TAIL_PASS, dat_kargs.hpp), at the end of the pass before it.  RB = true (k_cadmm_tail: one
// scenario slot per wavefront) drains the hand-over lists after k_cadmm (tmode 0), resuming each scenario in
// the pass it left (re-solving there only the agent QPs handed over), or the scenarios k_env_class routed to the
// tail before the step, concurrently with k_cadmm (tmode 1), and finishes their steps (and later fused steps).
// The tail's solves: IPM_FAST_REDO with the certificate of infeasible rows (dvl_rows_infeasible, once per
// scenario-step) and, in the passes the tail rule names, the warm start from the agent QP's converged iterate of
// the previous pass and the stall exit (ipm_solve WS).  Built with -ffp-contract=on (multiply-adds fused within
// an expression only), the inlined fast solver computes the same bits in either kernel, and the tail rule
// depends on the scenario's own history: a scenario's results do not depend on which kernel ran which pass.
template <int CLS, bool RB>
__device__ __forceinline__ void cadmm_drain(const KArgs& a) {
  constexpr bool ENV = CLS > 0;
  constexpr int NR = cadmm_nr(CLS);
  constexpr int NE = class_env_rows(CLS);
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int n = a.n, N3 = 3 * n;
  const int G = a.G;  // G <= 64 / n scenario slots (cadmm_slots); the tail: G = 1
  // the tail: V bit-identical clones of each agent lane (clone vi = lane / n) run the agent QP's solve in lockstep
  // and share out its stiff-row columns (ipm_attempt); only clone 0 writes the scenario's outputs
  const int V = RB ? tail_clones(n) : 1;
  const int NT = (RB ? V : G) * n;
  const int lane = threadIdx.x;
  const int vi = RB ? lane / n : 0;
  const int ls = RB ? 0 : lane / n, i = lane - (RB ? vi : ls) * n;
  const int al = RB ? i : lane;  // the lane's column in the row / env / aux images (a clone's: its agent's)
  const int lsc = ls < G ? ls : 0;
  const bool TM = RB && a.tmode == 1;  // the tail-routed stretch of slist (k_env_class), not the hand-over list
  const int first = TM ? a.scount[6 * NCLS + CLS] : a.scount[NCLS + CLS];
  const int cnt = TM ? a.scount[5 * NCLS + CLS] : RB ? a.scount[3 * NCLS + CLS] : a.scount[CLS];
  if (cnt == 0) return;
  int* const qh = TM ? a.scount + 7 * NCLS + CLS : RB ? a.scount + 4 * NCLS + CLS : a.qhead + CLS;
  const int* const ql = (RB && !TM ? a.rlist : a.slist) + first;
  const int rmode = RB ? 3 : cadmm_row_mode(n, G, CLS);  // wave-uniform
  CadmmLds L = cadmm_carve(smem, n, G, CLS, rmode);
  double* fb = L.fbar + lsc * N3;
  double* rts = L.Rt + lsc * RT_STRIDE * n;
  double* myred = L.red + lane * RDS;
  QPShared& S = L.sh[lsc];
  const LdsRef<QPShared> shr{L.sh, lsc};
  const EnvLdsN<NE> err{L.env, al};
  const RtLds rtr{L.Rt, (lsc * n + i) * RT_STRIDE};
  if (lane < G) L.sid[lane] = -1;
  __syncthreads();

  // per-lane state of the slot's current scenario
  DAT_PHASE_INIT(9);
  QPLane<1> P;
  int sc = -1;  // scenario of this lane's slot (-1: empty)
  const double* prm = nullptr;
  double* lam = nullptr;
  double* cfs = nullptr;  // the scenario's n agent copies f^(j), in the warm-state array (HBM / L2)
  double* myf = nullptr;
  double* bst = nullptr;
  double* wrl = nullptr;  // k_cadmm_tail: the lane's warm-start record
  int iter = 0, prev_iter = 0, qstat = ST_OPTIMAL;
  int kstep = 0;  // fused control steps (dat_control_steps): the slot scenario's current step
  int rmask = -1;  // k_cadmm_tail: the lanes that solve in the current pass (a resumed pass: those handed over)
  double rho = a.rho0;
  WaveCounters wc;
  for (;;) {
    // ---- refill empty slots from the queue
    DAT_PHASE(11);
    if (lane < NT && i == 0 && vi == 0 && L.sid[ls] == -1) {
      const int q = atomicAdd(qh, 1);
      const int s2 = q < cnt ? ql[q] : -2;  // -2: queue drained, slot retires
      L.sid[ls] = s2;
      L.done[ls] = 0;
      L.wmx[ls] = RB && !TM && s2 >= 0 ? a.rres[(size_t)s2 * RRES_INTS + RRES_WMX] : 0;
    }
    __syncthreads();
    const int slot_sc = lane < NT ? L.sid[ls] : -2;
    const bool fresh = slot_sc >= 0 && slot_sc != sc;
    if (fresh) {
      sc = slot_sc;
      prm = prm_of(a, sc);
      const double* st = a.state + (size_t)sc * a.S;
      if (vi == 0) make_Rt(prm + DAT_P_RCOM(n) + 3 * i, st + DAT_S_RL(n), rts + RT_STRIDE * i);
      lam = a.clam + ((size_t)sc * n + i) * N3;
      cfs = a.cf + (size_t)sc * n * N3;
      myf = cfs + i * N3;
      if (vi == 0)
        for (int c = 0; c < 3; ++c) fb[3 * i + c] = a.cfbar[(size_t)sc * N3 + 3 * i + c];
      // (the tail: the lane's record in LDS, behind the env image -- a generic pointer, flat loads go to LDS)
      bst = RB ? L.env + env_lds_doubles(NE) + i * best_size(1) : a.best + ((size_t)sc * n + i) * best_rec(1);
      iter = 0;
      prev_iter = a.iters[sc];  // the previous step's ADMM iterations (rewritten when the scenario stops)
      qstat = ST_OPTIMAL;
      rho = a.rho0;
      kstep = 0;
      rmask = -1;
      if (RB) {
        wrl = a.wrec + ((size_t)sc * n + i) * WREC_SIZE;
        wrl[0] = 0.0;  // no recorded iterate yet
      }
      if (RB && !TM) {
        // where k_cadmm left the scenario (its warm state -- multipliers, copies, the mean -- is in place)
        const int* const rr = a.rres + (size_t)sc * RRES_INTS;
        kstep = rr[RRES_KSTEP];
        iter = rr[RRES_PASS];
        rmask = rr[RRES_LANES];
        for (int q = 0; q < iter; ++q) rho = fmin(rho * a.tau, a.rho_max);  // the pass's rho, as k_cadmm had it
        qstat = a.qstatus[(size_t)sc * n + i];  // the pass's status of a lane not solved again
      }
      if (i == 0 && vi == 0)
        build_shared(S, prm, n, st, a.acc + ((size_t)kstep * a.B + sc) * 6, prm[DAT_P_KFD], prm[DAT_P_KMD], 3, true);
    }
    if (!__syncthreads_or(slot_sc >= 0)) break;  // every slot retired
    DAT_PHASE(12);
    if (fresh) {
      lane_cadmm_static(P, prm, i);
      if (ENV) {
        // the rows k_env_class computed from the same state this step
        const size_t NA = (size_t)a.B * n, g = (size_t)sc * n + i;
        const unsigned emask = a.emask[g];
        double lhs[DAT_NENV][3], rhs[DAT_NENV];
#pragma unroll
        for (int j = 0; j < DAT_NENV; ++j) {
          const bool on = (emask >> j) & 1u;  // unmarked slots are never written (set_env_rows skips them)
          lhs[j][0] = on ? a.erows[(4 * j + 0) * NA + g] : 0.0;
          lhs[j][1] = on ? a.erows[(4 * j + 1) * NA + g] : 0.0;
          lhs[j][2] = on ? a.erows[(4 * j + 2) * NA + g] : 0.0;
          rhs[j] = on ? a.erows[(4 * j + 3) * NA + g] : 0.0;
        }
        EnvRows E;
        set_env_rows(P, E, S, emask, lhs, rhs);
        env_to_lds<NE>(L.env, al, E);  // (clones: the same values to the same column)
        // the tail certifies infeasible rows once per scenario-step (such an agent QP would run 2 x 50 IPM
        // iterations in every pass and end INACCURATE: the previous solution is held either way)
        if (RB && !P.infeasible && dvl_rows_infeasible(shr, err, P.emask)) {
          P.infeasible = 1;
          wc.cert += vi == 0;
        }
      }
    }
    // ---- one ADMM pass of every occupied slot
    DAT_PHASE(14);
    bool active = slot_sc >= 0;
    int it_lane = 0;
    bool hand = false;  // k_cadmm: this lane's solve was not clean (ipm_unclean)
    // k_cadmm with sub-batches (no tail routing, KArgs::route): a wedged scenario leaves before its first pass, and
    // the tail runs its step from there, as it runs a routed one
    const bool wedged = !RB && iter == 0 && prev_iter > a.tail_prev;
    if (active && wedged) hand = true;
    if (active && !wedged && ((rmask >> i) & 1)) {
      lane_cadmm_dynamic(P, prm, n, i, rts, lam, fb, rho, RT_STRIDE);
      DAT_PHASE(15);
      P.tuned = iter == 0 || prev_iter <= 3;  // see ipm_solve: first pass, or the warm closed-loop regime
      double y[1][3], w[6];
      IPMOut o;
      DAT_PHASE(10);
      constexpr unsigned AUXM = cadmm_auxm(CLS);
      constexpr int RM = RB ? IPM_FAST_REDO : IPM_FAST;
      using SHT = LdsRef<QPShared>;
      using ERT = EnvLdsN<NE>;
      if constexpr (RB) {
        // the tail rule: warm start and stall exit in pass iter (the record is kept in every pass)
        const bool wson = iter >= 1 && (prev_iter > a.tail_prev || iter >= a.tail_pass);
        wc.warm += vi == 0 && wson && wrl[0] == 1.0;
        o = ipm_solve<MODE_CADMM, 1, NR, SHT, ERT, RtLds, RowLds, TAIL_AUXM, NoGrp, RM, true>(
            shr, err, rtr, P, prm + DAT_P_FEQ(n) + 3 * i, y, w, bst, IPM_MAX_ITER, a.qp_tol, RowLds{L.rows, al},
            NoGrp{}, wrl, wson, vi, V);
        wc.stall += vi == 0 && o.why == 7;
#ifdef DAT_CAPTURE_LOOSE
        if (vi == 0 && inband_loose(o)) {
          const unsigned k = atomicAdd(&g_ncap, 1u);
          if (k < (unsigned)CAP_MAX && 14 + a.S + 6 * n <= CAP_DOUBLES) {
            double* c = g_cap[k];
            c[0] = sc; c[1] = i; c[2] = iter; c[3] = rho; c[4] = prev_iter;
            c[5] = a.scen_forest ? a.scen_forest[sc] : -1; c[6] = o.merit; c[7] = kstep;
            for (int q = 0; q < 6; ++q) c[8 + q] = a.acc[((size_t)kstep * a.B + sc) * 6 + q];
            for (int q = 0; q < a.S; ++q) c[14 + q] = a.state[(size_t)sc * a.S + q];
            for (int q = 0; q < N3; ++q) { c[14 + a.S + q] = lam[q]; c[14 + a.S + N3 + q] = fb[q]; }
          }
        }
#endif
      } else if constexpr (CLS < NCLS - 1 && (CLS >= ROWLDS_MIN_CLS || AUXM != 0)) {
        if (AUXM != 0 && rmode == 2)
          o = ipm_solve<MODE_CADMM, 1, NR, SHT, ERT, RtLds, RowLds, AUXM, NoGrp, RM>(
              shr, err, rtr, P, prm + DAT_P_FEQ(n) + 3 * i, y, w, bst, IPM_MAX_ITER, a.qp_tol, RowLds{L.rows, lane});
        else if (CLS >= ROWLDS_MIN_CLS && rmode == 1)
          o = ipm_solve<MODE_CADMM, 1, NR, SHT, ERT, RtLds, RowLds, 0, NoGrp, RM>(
              shr, err, rtr, P, prm + DAT_P_FEQ(n) + 3 * i, y, w, bst, IPM_MAX_ITER, a.qp_tol, RowLds{L.rows, lane});
        else
          o = ipm_solve<MODE_CADMM, 1, NR, SHT, ERT, RtLds, RowRegs, 0, NoGrp, RM>(
              shr, err, rtr, P, prm + DAT_P_FEQ(n) + 3 * i, y, w, bst, IPM_MAX_ITER, a.qp_tol);
      } else {
        o = ipm_solve<MODE_CADMM, 1, NR, SHT, ERT, RtLds, RowRegs, 0, NoGrp, RM>(
            shr, err, rtr, P, prm + DAT_P_FEQ(n) + 3 * i, y, w, bst, IPM_MAX_ITER, a.qp_tol);
      }
      hand = !RB && ipm_unclean(o);
      DAT_PHASE(9);
      // a solve k_cadmm hands over is counted once, by k_cadmm_tail (its IPM_FAST_REDO runs the fast attempt
      // again): its discarded outcome here is neither an agent-QP solve nor an in-band accept
      const int keep = hand || vi > 0 ? 0 : 1;  // (nor do its iterations enter the pass's slot counts; nor a clone's)
      wc.ipm += keep * o.iters;
      wc.inband += keep * o.inband;
#ifdef DAT_ITER_HIST
      atomicAdd(&g_iter_hist[o.iters < 63 ? o.iters : 63], 1ull);
#endif
      wc.loose += keep * inband_loose(o);
      wc.refs += keep * o.refs;
      wc.corrs += keep * o.corrs;
      it_lane = keep * o.iters;
      wc.rowit += (long long)(keep * o.iters) * (__builtin_popcount(S.bmask) + __builtin_popcount(P.emask));
      wc.qp += keep;
      qstat = o.status;
      if (vi > 0) {
      } else if (o.status == ST_OPTIMAL) {
        for (int j = 0; j < n; ++j) {
          if (j == i) {
            myf[3 * j] = y[0][0]; myf[3 * j + 1] = y[0][1]; myf[3 * j + 2] = y[0][2];
          } else {
            cadmm_free_block(rts + RT_STRIDE * j, lam + 3 * j, fb + 3 * j, o.pi, rho, myf + 3 * j);
          }
        }
      } else if (o.status == ST_FAILED) {  // solver exception -> f_eq (control/rqp_cadmm.py:491-494)
        for (int c = 0; c < N3; ++c) myf[c] = prm[DAT_P_FEQ(n) + c];
      }  // otherwise hold the previous solution (control/rqp_cadmm.py:496-499)
    }
    DAT_PHASE(13);
    wc.slot += wave_max(it_lane);  // (the tail's passes: counted apart, CNT_TAIL)
    ++wc.pass;
    if (active) atomicMax(&L.wmx[ls], it_lane);
    rmask = -1;
    // the slot's lanes whose solve k_cadmm hands over (a ballot: the block is one wavefront)
    const unsigned long long hb = __ballot(hand);
    const int hmask = lane < NT ? (int)((hb >> (ls * n)) & ((1ull << n) - 1ull)) : 0;
    __syncthreads();
    if (!RB && active && hmask) {
      // an agent QP of the pass was not clean: k_cadmm_tail resumes the scenario here (the mean of the pass's
      // start, the statuses of the pass's other solves; multipliers and copies are in place)
      for (int c = 0; c < 3; ++c) a.cfbar[(size_t)sc * N3 + 3 * i + c] = fb[3 * i + c];
      a.qstatus[(size_t)sc * n + i] = qstat;
      if (i == 0) {
        int* const rr = a.rres + (size_t)sc * RRES_INTS;
        rr[RRES_KSTEP] = kstep;
        rr[RRES_PASS] = iter;
        rr[RRES_WMX] = L.wmx[ls];
        rr[RRES_LANES] = hmask;
        a.rlist[first + atomicAdd(a.scount + 3 * NCLS + CLS, 1)] = sc;
        L.sid[ls] = -1;
      }
      active = false;
    }
    if (active) {
      ++iter;
      rho = fmin(rho * a.tau, a.rho_max);
      // consensus mean, summed in agent order like the reference (control/rqp_cadmm.py:591-600)
      // agent-major: the three components of copy k read together (same per-component order)
      double s3[3] = {0.0, 0.0, 0.0};
      for (int k = 0; k < n; ++k) {
        const double* ck = cfs + k * N3 + 3 * i;
        const double c0 = ck[0], c1 = ck[1], c2 = ck[2];
        s3[0] += c0; s3[1] += c1; s3[2] += c2;
      }
      for (int c = 0; c < 3; ++c) myred[c] = s3[c] / n;
    }
    __syncthreads();
    if (active && vi == 0) {
      for (int c = 0; c < 3; ++c) fb[3 * i + c] = myred[c];
    }
    __syncthreads();
    if (active) {
      if (a.use_total_res) {
        double rmax = 0.0;
        double s3[3] = {0.0, 0.0, 0.0};
        for (int j = 0; j < n; ++j) {
          const double m0 = myf[3 * j], m1 = myf[3 * j + 1], m2 = myf[3 * j + 2];
          s3[0] += fabs(m0 - fb[3 * j]);
          s3[1] += fabs(m1 - fb[3 * j + 1]);
          s3[2] += fabs(m2 - fb[3 * j + 2]);
        }
        for (int r = 0; r < 3; ++r) rmax = fmax(rmax, s3[r]);
        myred[6] = rmax;
      } else {
        // aggregate residual (control/rqp_cadmm.py:602-621): own copy's totals of the others
        double F[3] = {0, 0, 0}, M[3] = {0, 0, 0};
        for (int j = 0; j < n; ++j) {
          if (j == i) continue;
          double m3[3];
          mv3(rts + RT_STRIDE * j, myf + 3 * j, m3);
          for (int c = 0; c < 3; ++c) { F[c] += myf[3 * j + c]; M[c] += m3[c]; }
        }
        // E_F,i = F_i - (sum_k f_app_k - f_app_i), E_M,i likewise with moments of f_app
        for (int k = 0; k < n; ++k) {
          if (k == i) continue;
          const double* fk = cfs + k * N3 + 3 * k;  // f_app_k = agent k's own block
          double m3[3];
          mv3(rts + RT_STRIDE * k, fk, m3);
          for (int c = 0; c < 3; ++c) { F[c] -= fk[c]; M[c] -= m3[c]; }
        }
        for (int c = 0; c < 3; ++c) { myred[c] = F[c]; myred[3 + c] = M[c]; }
      }
    }
    __syncthreads();
    if (active && i == 0 && vi == 0) {
      double res = 0.0;
      const double* rg = L.red + (ls * n) * RDS;
      if (a.use_total_res) {
        for (int k = 0; k < n; ++k) res = fmax(res, rg[RDS * k + 6]);
      } else {
        for (int r = 0; r < 3; ++r) {
          double sF = 0.0, sM = 0.0;
          for (int k = 0; k < n; ++k) {
            sF += fabs(rg[RDS * k + r]);
            sM += fabs(rg[RDS * k + 3 + r]);
          }
          res = fmax(res, fmax(sF, sM));
        }
      }
      bool stop = (res < a.res_tol) || (iter > a.max_iter);
      if (!stop && a.record_err && a.err) a.err[(size_t)sc * (a.max_iter + 1) + iter - 1] = res;
      L.done[ls] = stop ? 1 : 0;
    }
    __syncthreads();
    if (active) {
      if (!L.done[ls]) {
        if (vi == 0)
          for (int c = 0; c < N3; ++c) lam[c] += rho * (myf[c] - fb[c]);  // control/rqp_cadmm.py:627-629
        if (!RB && iter >= 1 && (prev_iter > a.tail_prev || iter >= a.tail_pass)) {
          // the tail rule holds from the next pass on: k_cadmm_tail resumes the scenario there (all lanes solve;
          // the mean of this pass goes with it, multipliers and copies are in place)
          for (int c = 0; c < 3; ++c) a.cfbar[(size_t)sc * N3 + 3 * i + c] = fb[3 * i + c];
          a.qstatus[(size_t)sc * n + i] = qstat;
          if (i == 0) {
            int* const rr = a.rres + (size_t)sc * RRES_INTS;
            rr[RRES_KSTEP] = kstep;
            rr[RRES_PASS] = iter;
            rr[RRES_WMX] = L.wmx[ls];
            rr[RRES_LANES] = -1;
            a.rlist[first + atomicAdd(a.scount + 3 * NCLS + CLS, 1)] = sc;
            L.sid[ls] = -1;
          }
        }
      } else {
        // the scenario stopped: write its outputs and free the slot
        if (RB && i == 0 && vi == 0) {  // a scenario-step the tail finished (and, routed before the step, apart)
          atomicAdd(a.counters + CNT_ROB, 1ull);
          if (TM && kstep == 0) atomicAdd(a.counters + CNT_TAIL + 2, 1ull);
        }
        if (vi == 0) {
          for (int c = 0; c < 3; ++c) {
            a.cfbar[(size_t)sc * N3 + 3 * i + c] = fb[3 * i + c];
            a.fdes[(size_t)sc * N3 + 3 * i + c] = myf[3 * i + c];  // f_app = diag copies (:669-671)
          }
          a.qstatus[(size_t)sc * n + i] = qstat;
          if (i == 0) {
            a.iters[sc] = iter;
            a.ipmx[sc] = L.wmx[ls];
          }
        }
        if (kstep + 1 < a.ksteps) {
          // fused steps: the scenario's next control step in the same slot (warm f, f_mean, lambda kept;
          // rho and the iteration count restart as in a new control call, control/rqp_cadmm.py:631-640)
          ++kstep;
          prev_iter = iter;
          iter = 0;
          qstat = ST_OPTIMAL;
          rho = a.rho0;
          if (RB) wrl[0] = 0.0;
          if (i == 0 && vi == 0) {
            build_shared(S, prm, n, a.state + (size_t)sc * a.S, a.acc + ((size_t)kstep * a.B + sc) * 6,
                         prm[DAT_P_KFD], prm[DAT_P_KMD], 3, true);
            L.wmx[ls] = 0;
          }
        } else if (i == 0) {
          L.sid[ls] = -1;
        }
      }
    }
    __syncthreads();
  }
  // work counters of this class: one atomic per wavefront
  unsigned long long q = (unsigned long long)wc.qp, ip = (unsigned long long)wc.ipm, rw = (unsigned long long)wc.rowit;
  unsigned long long ib = (unsigned long long)wc.inband, lo = (unsigned long long)wc.loose;
  unsigned long long rf = (unsigned long long)wc.refs, co = (unsigned long long)wc.corrs;
  unsigned long long ce = (unsigned long long)wc.cert, sx = (unsigned long long)wc.stall, wm = (unsigned long long)wc.warm;
  for (int off = 32; off > 0; off >>= 1) {
    q += __shfl_xor(q, off);
    ip += __shfl_xor(ip, off);
    rw += __shfl_xor(rw, off);
    ib += __shfl_xor(ib, off);
    lo += __shfl_xor(lo, off);
    rf += __shfl_xor(rf, off);
    co += __shfl_xor(co, off);
    if (RB) {
      ce += __shfl_xor(ce, off);
      sx += __shfl_xor(sx, off);
      wm += __shfl_xor(wm, off);
    }
  }
  if (lane == 0) {
    unsigned long long* cc = a.counters + CNT_STRIDE * CLS;
    atomicAdd(cc, q);
    atomicAdd(cc + 1, ip);
    atomicAdd(cc + 2, rw);
    if (RB) {  // the tail's occupancy apart from k_cadmm's class counters
      unsigned long long* ct = a.counters + CNT_TAIL;
      atomicAdd(ct, (unsigned long long)wc.pass);
      atomicAdd(ct + 1, (unsigned long long)wc.slot);
      if (ce) atomicAdd(ct + 3, ce);
      if (sx) atomicAdd(ct + 4, sx);
      if (wm) atomicAdd(ct + 5, wm);
    } else {
      atomicAdd(cc + 3, (unsigned long long)(wc.slot * NT));
      atomicAdd(cc + 4, (unsigned long long)(wc.pass * G));
    }
    if (ib) atomicAdd(a.counters + CNT_INBAND, ib);
    if (lo) atomicAdd(a.counters + CNT_INBAND + 1, lo);
    atomicAdd(a.counters + CNT_REF, rf);
    atomicAdd(a.counters + CNT_REF + 1, co);
  }
  __syncthreads();
}

// The C-ADMM control step of every scenario: persistent blocks drain the env classes in order of
// decreasing row count (the longest-running scenarios first), each class with its own row-slot
// instantiation of the IPM.  All wavefronts work on the same class at (nearly) the same time: the
// unrolled IPM of one class is ~80-130 KB of code, and wavefronts of different classes sharing a
// CU's instruction cache measured 16 % slower (proportional class starts: 12.9 vs 11.1 ms, C4 path).
__global__ __launch_bounds__(64) void k_cadmm(KArgs a) {
  cadmm_drain<3, false>(a);
  cadmm_drain<2, false>(a);
  cadmm_drain<1, false>(a);
  cadmm_drain<0, false>(a);
}
// The tail: the scenario-steps k_cadmm handed over (an agent QP not clean, or the tail rule) and, launched
// concurrently with k_cadmm, those k_env_class routed here (wedged in a stall), one scenario per wavefront,
// every class's row state and IPM aux slots in LDS: the robust redo, the certificate of infeasible rows, the warm
// start and stall exit of the tail rule's passes.  A kernel of its own: the robust solver compiled into k_cadmm
// cost the fast path 36-60 % (register allocation, C4 A/B).  Without a listed scenario its blocks return at once.
__global__ __launch_bounds__(64) void k_cadmm_tail(KArgs a) {
  cadmm_drain<3, true>(a);
  cadmm_drain<2, true>(a);
  cadmm_drain<1, true>(a);
  cadmm_drain<0, true>(a);
}
// Without a forest every scenario is in env class 0 (k_env_class finds no tree): the class-0 drain in a
// kernel of its own, with a 960 B/lane scratch frame instead of k_cadmm's 1,728 (same arithmetic).  C5
// 84.2 / 84.1 -> 80.3 / 79.9 ms per step, C2 12.7 / 12.9 -> 12.0 / 12.1 (round 4, kernel-trace A/B).
// With a forest one launch per class measured 2x slower on C4 (each class launch drains to its own
// tail): k_cadmm keeps the four drains in one launch there.
__global__ __launch_bounds__(64) void k_cadmm0(KArgs a) { cadmm_drain<0, false>(a); }
__global__ __launch_bounds__(64) void k_cadmm0_tail(KArgs a) { cadmm_drain<0, true>(a); }

// ------------------------------------------------------------------------------------------------
// DD: quasi-Newton matrix inverse per scenario (one 64-lane block per scenario)
// ------------------------------------------------------------------------------------------------
// Q_i: strong_convexity_matrix (control/rqp_dd.py:513-555), 9x9 in (f_i, F_i, M_i)
__device__ void dd_strong_convexity(const double* prm, int n, const double* st, int i, double* Q) {
  const double kf = prm[DAT_P_KFD], km = prm[DAT_P_KMD], kfeq = prm[DAT_P_KFEQ];
  const double leader = (i == 0) ? 1.0 : 0.0;
  const double mT = prm[DAT_P_MT];
  const double* Rl = st + DAT_S_RL(n);
  double Rt[9], Xh[9], RX[9], Bv[9];
  make_Rt(prm + DAT_P_RCOM(n) + 3 * i, Rl, Rt);
  skew3(prm + DAT_P_XCOM, Xh);
  mm3(Rl, Xh, RX);
  mm3(RX, prm + DAT_P_JTI, Bv);  // Rl hat(x_com) JT^-1
  for (int k = 0; k < 81; ++k) Q[k] = 0.0;
  for (int k = 0; k < 9; ++k) Q[10 * k] = 1e-6;
  auto acc = [&](const double* T /*3x9*/, double wgt) {
    for (int r = 0; r < 9; ++r)
      for (int c = 0; c < 9; ++c) Q[9 * r + c] += 2.0 * wgt * (T[r] * T[c] + T[9 + r] * T[9 + c] + T[18 + r] * T[18 + c]);
  };
  double T[27];
  for (int k = 0; k < 27; ++k) T[k] = 0.0;
  for (int r = 0; r < 3; ++r) T[9 * r + r] = 1.0;          // [I 0 0]
  acc(T, kfeq);
  for (int r = 0; r < 3; ++r) T[9 * r + 3 + r] = 1.0;      // [I I 0]
  acc(T, kf);
  for (int k = 0; k < 27; ++k) T[k] = 0.0;                 // [Rt 0 I]
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) T[9 * r + c] = Rt[3 * r + c];
    T[9 * r + 6 + r] = 1.0;
  }
  acc(T, km);
  if (leader != 0.0) {
    const double* JTi = prm + DAT_P_JTI;
    double JR[9], BR[9];
    mm3(JTi, Rt, JR);
    mm3(Bv, Rt, BR);
    for (int k = 0; k < 27; ++k) T[k] = 0.0;               // [JT^-1 Rt, 0, JT^-1]
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) { T[9 * r + c] = JR[3 * r + c]; T[9 * r + 6 + c] = JTi[3 * r + c]; }
    acc(T, leader);
    for (int k = 0; k < 27; ++k) T[k] = 0.0;               // [I/mT + Bv Rt, I/mT, Bv]
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        T[9 * r + c] = BR[3 * r + c] + (r == c ? 1.0 / mT : 0.0);
        T[9 * r + 3 + c] = (r == c ? 1.0 / mT : 0.0);
        T[9 * r + 6 + c] = Bv[3 * r + c];
      }
    acc(T, leader);
  }
}

// k_dd_setup keeps the columns of [H | I] in registers for n <= DD_REG_NMAX (dd_setup_h_regs), in LDS
// beyond
constexpr int DD_REG_NMAX = 8;
// doubles of the [H | I] area of k_dd_setup; it first holds the per-agent [Q_i | I] (162 n), their
// pivot columns (9 n) and pivot rows (n ints).  Register path: the Q_i area and two N-double pivot
// column buffers only.
__host__ __device__ inline int dd_setup_hs(int n) {
  const int N = 6 * n;
  if (n <= DD_REG_NMAX) return 171 * n + 1 + 2 * N;  // k_dd_setup<n>
  return 2 * N * N > 171 * n + 1 ? 2 * N * N : 171 * n + 1;
}

// H = A blkdiag(Q_j^-1) A' (control/rqp_dd.py:642-655) and H^-1 by Gauss-Jordan on [H | I], n = NB,
// with the columns of [H | I] in registers: lane c owns column c and, when 2N > 64, column c + 64 (an
// identity column: N <= 48).  Same per-element arithmetic and order as the LDS path, so the result is
// bitwise equal: H_rc summed over blocks j, then over the support p of row r's block in increasing
// order, of A_rp (Q_j A_c)_p with (Q_j A_c)_p summed over q in increasing order; Gauss-Jordan without
// pivoting (H is SPD), per element hk = h_kc / piv, h_rc -= f_r hk.  The column is kept rotated so
// that step k's pivot row is element 0 (no runtime register index): the owner of column k publishes it
// in LDS (double buffered), every lane updates its columns and rotates them by one.
template <int NB>
__device__ void dd_setup_h_regs(const KArgs& a, int sc, const double* Qi, const double* Rts, double* fac) {
  constexpr int N = 6 * NB;
  constexpr bool TWO = 2 * N > 64;
  const int lane = threadIdx.x;
  double h[N], g[TWO ? N : 1];
  // ---- assembly of column lane (H columns for lane < N, identity columns e_{lane - N} beyond)
#pragma unroll
  for (int r = 0; r < N; ++r) {
    h[r] = (lane >= N && r == lane - N) ? 1.0 : 0.0;
    if (TWO) g[r] = (r == lane + 64 - N) ? 1.0 : 0.0;
  }
  if (lane < N) {
    const int ag = lane / 6, comp = lane - 6 * ag;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const double* Q = Qi + 81 * j;
      // w = Q_j a_{c,j}: a_{c,j} = e_{3+comp} (j == ag), -e_comp (comp < 3), -Rt_j[comp-3, :] on f_j
      double w[9];
      if (j == ag) {
#pragma unroll
        for (int p = 0; p < 9; ++p) { double t = 0.0; t += Q[9 * p + 3 + comp] * 1.0; w[p] = t; }
      } else if (comp < 3) {
#pragma unroll
        for (int p = 0; p < 9; ++p) { double t = 0.0; t += Q[9 * p + comp] * -1.0; w[p] = t; }
      } else {
        const double* rt = Rts + 9 * j + 3 * (comp - 3);
        const double v0 = -rt[0], v1 = -rt[1], v2 = -rt[2];
#pragma unroll
        for (int p = 0; p < 9; ++p) {
          double t = 0.0;
          t += Q[9 * p] * v0;
          t += Q[9 * p + 1] * v1;
          t += Q[9 * p + 2] * v2;
          w[p] = t;
        }
      }
#pragma unroll
      for (int r = 0; r < N; ++r) {
        const int agr = r / 6, cr = r % 6;
        if (j == agr) {
          h[r] += 1.0 * w[3 + cr];
        } else if (cr < 3) {
          h[r] += -1.0 * w[cr];
        } else {
          const double* rt = Rts + 9 * j + 3 * (cr - 3);
          h[r] += -rt[0] * w[0];
          h[r] += -rt[1] * w[1];
          h[r] += -rt[2] * w[2];
        }
      }
    }
  }
  // ---- Gauss-Jordan, columns rotated (h[i] = [H | I]_{(k + i) mod N, c} at step k)
  for (int k = 0; k < N; ++k) {
    double* f = fac + (k & 1) * N;
    if (lane == k) {
#pragma unroll
      for (int i = 0; i < N; ++i) f[i] = h[i];
    }
    __syncthreads();
    const double piv = f[0];
    {
      const double hk = h[0] / piv;
#pragma unroll
      for (int i = 1; i < N; ++i) h[i] -= f[i] * hk;
#pragma unroll
      for (int i = 0; i < N - 1; ++i) h[i] = h[i + 1];
      h[N - 1] = hk;
    }
    if (TWO) {
      const double hk = g[0] / piv;
#pragma unroll
      for (int i = 1; i < N; ++i) g[i] -= f[i] * hk;
#pragma unroll
      for (int i = 0; i < N - 1; ++i) g[i] = g[i + 1];
      g[N - 1] = hk;
    }
  }
  // ---- H^-1 = the right half: column N + c' of [H | I] is column c' of H^-1 (row-major output)
  double* out = a.dHinv + (size_t)sc * N * N;
  if (lane >= N && lane < 2 * N) {
#pragma unroll
    for (int r = 0; r < N; ++r) out[(size_t)r * N + (lane - N)] = h[r];
  }
  if (TWO && lane + 64 < 2 * N) {
#pragma unroll
    for (int r = 0; r < N; ++r) out[(size_t)r * N + (lane + 64 - N)] = g[r];
  }
}

// NB = n (<= DD_REG_NMAX: H columns in registers, one instantiation per team size so each has its own
// register footprint) or 0 (any n: H in LDS)
template <int NB>
__global__ __launch_bounds__(64) void k_dd_setup(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int n = a.n, N = 6 * n;
  const int sc = blockIdx.x;
  const int lane = threadIdx.x;
  if (sc >= a.B) return;
  double* Qi = smem;              // n x 81   sym(Q_i^-1)
  double* Rts = Qi + 81 * n;      // n x 9
  double* H = Rts + 9 * n;        // N x 2N   [H | I]
  double* fac = H + dd_setup_hs(n);  // N
  const double* prm = prm_of(a, sc);
  const double* st = a.state + (size_t)sc * a.S;
  // Q_i^-1 by Gauss-Jordan with partial pivoting (np.linalg.inv) on [Q_i | I] in LDS, spread over
  // the wavefront: lane pairs (agent j, column c) update one column each, with the per-element
  // arithmetic of the serial elimination (pivot column copied before the update).
  double* Aug = H;                         // n x 9 x 18, in the [H | I] area (built afterwards)
  double* colk = Aug + 162 * n;            // n x 9: column k before step k's update
  int* pivr = (int*)(colk + 9 * n);        // n
  if (lane < n) {
    double Q[81];
    dd_strong_convexity(prm, n, st, lane, Q);
    for (int r = 0; r < 9; ++r)
      for (int c = 0; c < 18; ++c) Aug[162 * lane + 18 * r + c] = c < 9 ? Q[9 * r + c] : (c - 9 == r ? 1.0 : 0.0);
    make_Rt(prm + DAT_P_RCOM(n) + 3 * lane, st + DAT_S_RL(n), Rts + 9 * lane);
  }
  __syncthreads();
  for (int k = 0; k < 9; ++k) {
    if (lane < n) {
      const double* A = Aug + 162 * lane;
      int p = k;
      for (int r = k + 1; r < 9; ++r)
        if (fabs(A[18 * r + k]) > fabs(A[18 * p + k])) p = r;
      pivr[lane] = p;
    }
    __syncthreads();
    for (int e = lane; e < 18 * n; e += 64) {  // row exchange k <-> p, column by column
      const int j = e / 18, c = e - 18 * j, p = pivr[j];
      double* A = Aug + 162 * j;
      if (p != k) { double t = A[18 * k + c]; A[18 * k + c] = A[18 * p + c]; A[18 * p + c] = t; }
    }
    __syncthreads();
    for (int e = lane; e < 9 * n; e += 64) {
      const int j = e / 9, r = e - 9 * j;
      colk[e] = Aug[162 * j + 18 * r + k];
    }
    __syncthreads();
    for (int e = lane; e < 18 * n; e += 64) {
      const int j = e / 18, c = e - 18 * j;
      double* A = Aug + 162 * j;
      const double inv = 1.0 / colk[9 * j + k];
      const double hk = A[18 * k + c] * inv;
      A[18 * k + c] = hk;
      for (int r = 0; r < 9; ++r)
        if (r != k) A[18 * r + c] -= colk[9 * j + r] * hk;
    }
    __syncthreads();
  }
  for (int e = lane; e < 81 * n; e += 64) {
    const int j = e / 81, rc = e - 81 * j, r = rc / 9, c = rc - 9 * r;
    const double* A = Aug + 162 * j;
    Qi[e] = 0.5 * (A[18 * r + 9 + c] + A[18 * c + 9 + r]);
  }
  __syncthreads();
  if constexpr (NB > 0) {
    dd_setup_h_regs<NB>(a, sc, Qi, Rts, H + 171 * n + 1);  // pivot columns past the Q_i elimination area
    return;
  }
  // H = A blkdiag(Q_j^-1) A'  (control/rqp_dd.py:642-655); row r of A restricted to block j:
  //   j == agent(r): unit vector e_{3 + comp};  j != agent(r): -e_comp (comp < 3) or -Rt_j[comp-3, :] on f_j
  // every index below is compile-time after unrolling, so v stays in registers (no scratch)
  auto arow = [&](int r, int j, double* v) {
    const int ag = r / 6, comp = r % 6;
    const double* rt = Rts + 9 * j + 3 * (comp >= 3 ? comp - 3 : 0);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      double x = 0.0;
      if (j == ag) x = (k == 3 + comp) ? 1.0 : 0.0;
      else if (comp < 3) x = (k == comp) ? -1.0 : 0.0;
      else if (k < 3) x = -rt[k];
      v[k] = x;
    }
  };
  for (int e = lane; e < N * N; e += 64) {
    int r = e / N, c = e % N;
    double s = 0.0;
    for (int j = 0; j < n; ++j) {
      double vr[9], vc[9];
      arow(r, j, vr);
      arow(c, j, vc);
      const double* Q = Qi + 81 * j;
#pragma unroll
      for (int p = 0; p < 9; ++p) {
        if (vr[p] == 0.0) continue;
        double t = 0.0;
#pragma unroll
        for (int q = 0; q < 9; ++q) t += Q[9 * p + q] * vc[q];
        s += vr[p] * t;
      }
    }
    H[2 * N * r + c] = s;
    H[2 * N * r + N + c] = (r == c) ? 1.0 : 0.0;
  }
  __syncthreads();
  // Gauss-Jordan on [H | I] (H is SPD: no pivoting needed)
  // Each lane owns whole columns of [H | I] (no index division; a row of the tile is contiguous
  // across lanes, so the LDS accesses are conflict-free); per-element operation order as before.
  for (int k = 0; k < N; ++k) {
    double piv = H[2 * N * k + k];
    for (int r = lane; r < N; r += 64) fac[r] = H[2 * N * r + k];
    __syncthreads();
    for (int c = lane; c < 2 * N; c += 64) {
      const double hk = H[2 * N * k + c] / piv;
      H[2 * N * k + c] = hk;
      for (int r = 0; r < N; ++r)
        if (r != k) H[2 * N * r + c] -= fac[r] * hk;
    }
    __syncthreads();
  }
  double* out = a.dHinv + (size_t)sc * N * N;
  for (int e = lane; e < N * N; e += 64) out[e] = H[2 * N * (e / N) + N + (e % N)];
}

// ------------------------------------------------------------------------------------------------
// DD step
// ------------------------------------------------------------------------------------------------
constexpr int DD_ES = 7, DD_RS = 5;
// k_dd per-wavefront area: with a forest the env rows' LDS image; without one nothing (n = 6:
// 27.0 KB, four wavefronts per CU -- the unused 20 KB image used to hold k_dd at three, C3 A/B
// 23.8 -> 22.7 ms).  The 3 base rows' IPM state stays in registers: RowLds measured 26.2 ms, and rows
// (+ aux slots) in LDS without a forest measured no gain on C3 in round 3 (git history).
__host__ __device__ constexpr int dd_area_doubles(bool env) { return env ? ENV_LDS_DOUBLES : 0; }
// k_dd_key: drain-order key of every scenario -- the previous step's (DD iteration count, slowest agent
// QP's IPM iterations), longest first, as k_cadmm's key -- sorted by k_bucket into one queue (class 0).
// DD agent QPs run the conservative IPM start (9-10 iterations on average): bins <= 8, 9-10, 11-13, >= 14.
__host__ __device__ inline int dd_ipm_bin(int it) { return it <= 8 ? 0 : it <= 10 ? 1 : it <= 13 ? 2 : 3; }
__global__ void k_dd_key(KArgs a) {
  const int sc = blockIdx.x * blockDim.x + threadIdx.x;
  if (sc < a.B) a.need[sc] = NIB - 1 - (NPB * iter_bin(a.iters[sc]) + dd_ipm_bin(a.ipmx[sc]));
}

// DD control step (control/rqp_dd.py:695-752), persistent: each 64-lane block holds G = floor(64/n)
// scenario slots of n lanes (one lane per agent QP) and drains the sorted scenario queue; a slot whose
// scenario stops is refilled at the next dual-ascent pass.  A scenario's arithmetic does not depend
// on the slot or block that runs it.  ENV = false (no forest on the handle): every QP has the three
// base rows only, and the IPM is instantiated for them alone (the register footprint of the 13-slot
// instantiation is not paid).
template <bool ENV>
__global__ __launch_bounds__(64) void k_dd(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int n = a.n, N3 = 3 * n, N6 = 6 * n;
  const int G = 64 / n, NT = G * n;
  const int lane = threadIdx.x;
  const int ls = lane / n, i = lane - ls * n;
  const int lsc = ls < G ? ls : 0;
  double* X = smem;                     // NT x 9   (f_i, F_i, M_i)
  double* lamF = X + al2(NT * 9);       // G x 3n
  double* lamM = lamF + al2(G * N3);    // G x 3n
  double* E = lamM + al2(G * N3);       // NT x ES  consensus error (ES = 7: odd stride, no bank conflicts)
  double* Rts = E + al2(NT * DD_ES);    // G x n x RT_STRIDE
  double* red = Rts + G * RT_STRIDE * n;  // 64 x DD_RS
  QPShared* shs = (QPShared*)(red + 64 * DD_RS);  // G
  double* envs = (double*)(shs + G);              // EnvLds image (ENV only)
  int* sid = (int*)(envs + dd_area_doubles(ENV));  // G: scenario of the slot (-1 empty, -2 retired)
  int* done = sid + 64;                           // G: the slot's scenario stopped in this pass
  int* wmx = done + 64;                           // G: IPM iterations of the slot's slowest agent QP this step
  QPShared& S = shs[lsc];
  double* myX = X + lane * 9;
  double* lF = lamF + lsc * N3;
  double* lM = lamM + lsc * N3;
  double* rts = Rts + lsc * RT_STRIDE * n;
  const int cnt = a.scount[0], first = a.scount[NCLS];
  const LdsRef<QPShared> shr{shs, lsc};
  const EnvLds err{envs, lane};
  const RtLds rtr{Rts, (lsc * n + i) * RT_STRIDE};
  if (lane < G) sid[lane] = -1;
  __syncthreads();

  QPLane<1> P;
  const double* prm = nullptr;
  const double* Rl = nullptr;
  double* bst = nullptr;
  double* wrl = nullptr;  // DAT_DD_WARM: the agent QP's warm-start record (HBM)
  double prev[9];
  int sc = -1, iter = 0, qstat = ST_OPTIMAL, col = 0;
  int kstep = 0;  // fused control steps (dat_control_steps): the slot scenario's current step
  double mdist = 0.0;
  long long my_ipm = 0, my_qp = 0, my_rowit = 0, my_inband = 0, my_loose = 0, my_refs = 0, my_corrs = 0;
  // phase marks (DAT_PHASE_PROF builds, tools/phase_prof.py): 11 refill + fresh slot setup, 14 prices,
  // 10 ipm_solve, 9 result bookkeeping, 13 consensus error, stop test, dual ascent, outputs
  DAT_PHASE_INIT(11);
  for (;;) {
    DAT_PHASE(11);
    // ---- refill empty slots from the queue
    if (lane < NT && i == 0 && sid[ls] == -1) {
      const int q = atomicAdd(a.qhead, 1);
      sid[ls] = q < cnt ? a.slist[first + q] : -2;
      done[ls] = 0;
      wmx[ls] = 0;
    }
    __syncthreads();
    const int slot_sc = lane < NT ? sid[ls] : -2;
    const bool fresh = slot_sc >= 0 && slot_sc != sc;
    if (fresh) {
      sc = slot_sc;
      prm = prm_of(a, sc);
      const double* st = a.state + (size_t)sc * a.S;
      Rl = st + DAT_S_RL(n);
      make_Rt(prm + DAT_P_RCOM(n) + 3 * i, Rl, rts + RT_STRIDE * i);
      for (int c = 0; c < 3; ++c) {
        lF[3 * i + c] = a.dlamF[(size_t)sc * N3 + 3 * i + c];
        lM[3 * i + c] = a.dlamM[(size_t)sc * N3 + 3 * i + c];
      }
      for (int c = 0; c < 9; ++c) prev[c] = a.dprev[((size_t)sc * n + i) * 9 + c];
      for (int c = 0; c < 9; ++c) myX[c] = prev[c];  // the controller's current (f, F, M)
      bst = a.best + ((size_t)sc * n + i) * best_rec(1);
#if DAT_DD_WARM
      wrl = a.wrec + ((size_t)sc * n + i) * WREC_SIZE;
      wrl[0] = 0.0;
#endif
      iter = 0;
      qstat = ST_OPTIMAL;
      kstep = 0;
      if (i == 0) build_shared(S, prm, n, st, a.acc + (size_t)sc * 6, prm[DAT_P_KFD], prm[DAT_P_KMD], 3, false);
    }
    if (!__syncthreads_or(slot_sc >= 0)) break;  // every slot retired
    if (fresh) {
      lane_dd_static(P, prm, i);
      col = 0;
      mdist = prm[DAT_P_VISR];
      if (ENV) {
        const double* trees;
        int nt;
        unsigned emask;
        forest_of(a, sc, &trees, &nt);
        double lhs[DAT_NENV][3], rhs[DAT_NENV];
        EnvOut env = env_rows(prm, n, a.state + (size_t)sc * a.S, trees, nt, i, prm[DAT_P_AENVD], &emask, lhs, rhs);
        col = env.collision;
        mdist = env.min_env_dist;
        EnvRows Ev;
        set_env_rows(P, Ev, S, emask, lhs, rhs);
        env_to_lds(envs, lane, Ev);
      }
    }
    const bool active = slot_sc >= 0;
    const int nr = wave_max(active ? rows_needed(P.emask) : NBASE);
    DAT_PHASE(14);
    if (active) {
      // prices (control/rqp_dd.py:718-722)
      double sF[3] = {0, 0, 0}, sM[3] = {0, 0, 0};
      for (int k = 0; k < n; ++k)
        for (int c = 0; c < 3; ++c) { sF[c] += lF[3 * k + c]; sM[c] += lM[3 * k + c]; }
      double c9[9], dm[3], rxd[3], Rr[3];
      for (int c = 0; c < 3; ++c) dm[c] = sM[c] - lM[3 * i + c];
      cross3(prm + DAT_P_RCOM(n) + 3 * i, dm, rxd);
      mv3(Rl, rxd, Rr);
      for (int c = 0; c < 3; ++c) {
        c9[c] = -(sF[c] - lF[3 * i + c]) + Rr[c];
        c9[3 + c] = lF[3 * i + c];
        c9[6 + c] = lM[3 * i + c];
      }
      set_dd_price(P, prm, n, i, c9);
      double y[1][3], w[6];
      IPMOut o;
      const double* y0 = prm + DAT_P_FEQ(n) + 3 * i;
      DAT_PHASE(10);
#if DAT_DD_WARM
      // a DD pass after the first: the agent QP differs from the previous pass's only in its prices, so it starts
      // from that pass's last iterate (ipm_solve WS, the tail kernel's warm start)
      const bool wson = iter >= DD_WARM_PASS;
      if constexpr (ENV)
        o = ipm_solve_rows<MODE_DD, 1, IPM_FAST, true>(nr, shr, err, rtr, P, y0, y, w, bst, IPM_MAX_ITER, a.qp_tol,
                                                       wrl, wson);
      else
        o = ipm_solve<MODE_DD, 1, NBASE, LdsRef<QPShared>, EnvLds, RtLds, RowRegs, 0, NoGrp, IPM_FAST, true>(
            shr, err, rtr, P, y0, y, w, bst, IPM_MAX_ITER, a.qp_tol, RowRegs{}, NoGrp{}, wrl, wson);
#else
      if constexpr (ENV)
        o = ipm_solve_rows<MODE_DD, 1>(nr, shr, err, rtr, P, y0, y, w, bst, IPM_MAX_ITER,
                                       a.qp_tol);
      else
        o = ipm_solve<MODE_DD, 1, NBASE>(shr, err, rtr, P, y0, y, w, bst, IPM_MAX_ITER,
                                         a.qp_tol);
#endif
      DAT_PHASE(9);
      my_ipm += o.iters;
      my_inband += o.inband;
      my_loose += inband_loose(o);
      my_refs += o.refs;
      my_corrs += o.corrs;
      atomicMax(&wmx[ls], o.iters);
#ifdef DAT_ITER_HIST
      atomicAdd(&g_iter_hist[o.iters < 63 ? o.iters : 63], 1ull);
#endif
      my_rowit += (long long)o.iters * (__builtin_popcount(S.bmask) + __builtin_popcount(P.emask));
      ++my_qp;
      qstat = o.status;
      if (o.status == ST_OPTIMAL) {
        for (int c = 0; c < 3; ++c) prev[c] = y[0][c];
        for (int c = 0; c < 6; ++c) prev[3 + c] = w[c];
      } else if (o.status == ST_FAILED) {  // control/rqp_dd.py:484-489
        // Quirk a15: the controller's f aliases solver 0's f_eq (control/rqp_dd.py:629, written in
        // place at :725), so agent 0's fallback sums the controller's current forces (every agent's
        // f before this iteration's writes); the other agents sum their own f_eq.
        const double* feq = prm + DAT_P_FEQ(n);
        double s3[3] = {0, 0, 0}, jr[3], rf[3];
        for (int k = 0; k < n; ++k)
          for (int c = 0; c < 3; ++c) s3[c] += (i == 0) ? X[(ls * n + k) * 9 + c] : feq[3 * k + c];
        for (int c = 0; c < 3; ++c) { prev[c] = feq[3 * i + c]; prev[3 + c] = s3[c] - feq[3 * i + c]; }
        cross3(prm + DAT_P_RCOM(n) + 3 * i, prev, rf);
        mv3(prm + DAT_P_JTI, rf, jr);
        for (int c = 0; c < 3; ++c) prev[6 + c] = -jr[c];
      }
    }
    DAT_PHASE(13);
    __syncthreads();  // agent 0's fallback above reads X before this pass's writes
    if (active) {
      for (int c = 0; c < 9; ++c) myX[c] = prev[c];
    }
    __syncthreads();
    if (active) {
      ++iter;
      // consensus error (control/rqp_dd.py:659-676)
      double sf[3] = {0, 0, 0}, sm[3] = {0, 0, 0};
      for (int k = 0; k < n; ++k) {
        if (k == i) continue;
        const double* fk = X + (ls * n + k) * 9;
        double m3[3];
        mv3(rts + RT_STRIDE * k, fk, m3);
        for (int c = 0; c < 3; ++c) { sf[c] += fk[c]; sm[c] += m3[c]; }
      }
      for (int c = 0; c < 3; ++c) {
        E[lane * DD_ES + c] = myX[3 + c] - sf[c];
        E[lane * DD_ES + 3 + c] = myX[6 + c] - sm[c];
      }
      red[lane * DD_RS + 0] = col ? 1.0 : 0.0;
      red[lane * DD_RS + 1] = mdist;
    }
    __syncthreads();
    if (active && i == 0) {
      double res = 0.0;
      for (int r = 0; r < 6; ++r) {
        double s = 0.0;
        for (int k = 0; k < n; ++k) s += fabs(E[(ls * n + k) * DD_ES + r]);
        res = fmax(res, s);
      }
      const bool stop = (res < a.res_tol) || (iter > a.max_iter);
      if (!stop && a.record_err && a.err) a.err[(size_t)sc * (a.max_iter + 1) + iter - 1] = res;
      done[ls] = stop ? 1 : 0;
    }
    __syncthreads();
    if (active) {
      if (!done[ls]) {
        // dual ascent: lambda += H^-1 (A x)   (control/rqp_dd.py:678-693); rows 6i..6i+5
        // The six rows are read agent block by agent block (18 16-byte loads in flight per block, rows
        // and blocks 48-byte aligned), each row's sum kept in the original order c = 0 .. 6n-1.
        const double* Hi = a.dHinv + (size_t)sc * N6 * N6 + (size_t)(6 * i) * N6;
        double stp[6] = {0, 0, 0, 0, 0, 0};
        for (int k = 0; k < n; ++k) {
          dat_d2 h[6][3];
#pragma unroll
          for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int j = 0; j < 3; ++j) h[r][j] = *(const dat_d2*)(Hi + (size_t)r * N6 + 6 * k + 2 * j);
          const double* e = E + (ls * n + k) * DD_ES;
          double ev[6];
#pragma unroll
          for (int j = 0; j < 6; ++j) ev[j] = e[j];
#pragma unroll
          for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              stp[r] += h[r][j].x * ev[2 * j];
              stp[r] += h[r][j].y * ev[2 * j + 1];
            }
        }
        for (int c = 0; c < 3; ++c) {
          lF[3 * i + c] += stp[c];
          lM[3 * i + c] += stp[3 + c];
        }
      } else {
        // the scenario stopped: write its outputs and free the slot
        for (int c = 0; c < 3; ++c) {
          a.dlamF[(size_t)sc * N3 + 3 * i + c] = lF[3 * i + c];
          a.dlamM[(size_t)sc * N3 + 3 * i + c] = lM[3 * i + c];
          a.fdes[(size_t)sc * N3 + 3 * i + c] = myX[c];
        }
        for (int c = 0; c < 9; ++c) a.dprev[((size_t)sc * n + i) * 9 + c] = prev[c];
        a.qstatus[(size_t)sc * n + i] = qstat;
        if (i == 0) {
          a.iters[sc] = iter;
          a.ipmx[sc] = wmx[ls];
          int coll = 0;
          double md = prm[DAT_P_VISR];
          for (int k = 0; k < n; ++k) {
            coll |= red[(ls * n + k) * DD_RS] != 0.0;
            md = fmin(md, red[(ls * n + k) * DD_RS + 1]);
          }
          a.col[sc] = (unsigned char)coll;
          a.mind[sc] = md;
        }
        if (kstep + 1 < a.ksteps) {
          // fused steps (no forest): the scenario's next control step in the same slot, from the warm
          // lambda_F, lambda_M and previous solutions it leaves (control/rqp_dd.py:695-700)
          ++kstep;
          iter = 0;
#if DAT_DD_WARM
          wrl[0] = 0.0;
#endif
          qstat = ST_OPTIMAL;
          if (i == 0) {
            build_shared(S, prm, n, a.state + (size_t)sc * a.S, a.acc + ((size_t)kstep * a.B + sc) * 6,
                         prm[DAT_P_KFD], prm[DAT_P_KMD], 3, false);
            wmx[ls] = 0;
          }
        } else if (i == 0) {
          sid[ls] = -1;
        }
      }
    }
    __syncthreads();
  }
  unsigned long long q = (unsigned long long)my_qp, ip = (unsigned long long)my_ipm, rw = (unsigned long long)my_rowit;
  unsigned long long ib = (unsigned long long)my_inband, lo = (unsigned long long)my_loose;
  unsigned long long rf = (unsigned long long)my_refs, co = (unsigned long long)my_corrs;
  for (int off = 32; off > 0; off >>= 1) {
    q += __shfl_xor(q, off);
    ip += __shfl_xor(ip, off);
    rw += __shfl_xor(rw, off);
    ib += __shfl_xor(ib, off);
    lo += __shfl_xor(lo, off);
    rf += __shfl_xor(rf, off);
    co += __shfl_xor(co, off);
  }
  if (lane == 0) {
    atomicAdd(a.counters, q);
    atomicAdd(a.counters + 1, ip);
    atomicAdd(a.counters + 2, rw);
    if (ib) atomicAdd(a.counters + CNT_INBAND, ib);
    if (lo) atomicAdd(a.counters + CNT_INBAND + 1, lo);
    atomicAdd(a.counters + CNT_REF, rf);
    atomicAdd(a.counters + CNT_REF + 1, co);
  }
}

// ------------------------------------------------------------------------------------------------
// rollout / desired acceleration / warm start
// ------------------------------------------------------------------------------------------------
// `steps` simulation steps (sim_step, system/rigid_quadrotor_payload.py:129-222) with one lane per (scenario, agent): G = floor(64/n) scenarios
// per 64-lane block.  Lane i runs agent i's low-level law, rotational dynamics and attitude
// integration; the payload's force / moment sums go through LDS and every lane of the scenario
// integrates the payload identically (sums in agent order, the arithmetic of sim_step: bitwise the
// same trajectory).  Per-lane state is one quadrotor plus the payload (~40 doubles), so nothing
// spills and the kernel runs many wavefronts per SIMD, for any n (k_rollout<0> kept the whole state
// of a large team in scratch).
constexpr int RO_X = 6;  // per lane in LDS: u = f R e3 (3), hat(r_com) Rl' u (3)
__global__ __launch_bounds__(64) void k_rollout_agents(KArgs a, int steps, double dt, const double* fdes) {
  __shared__ double xs[64 * RO_X];
  const int n = a.n, G = 64 / n, NT = G * n;
  const int lane = threadIdx.x, ls = lane / n, i = lane - ls * n;
  const int sc = blockIdx.x * G + ls;
  const bool valid = lane < NT && sc < a.B;
  const double* prm = valid ? prm_of(a, sc) : a.params;
  double* g = valid ? a.state + (size_t)sc * a.S : nullptr;
  double R[9], W[3], xl[3], vl[3], Rl[9], wl[3], fd[3];
  int cnt = 0;
  if (valid) {
    for (int k = 0; k < 9; ++k) { R[k] = g[DAT_S_R(n) + 9 * i + k]; Rl[k] = g[DAT_S_RL(n) + k]; }
    for (int c = 0; c < 3; ++c) {
      W[c] = g[DAT_S_W(n) + 3 * i + c];
      xl[c] = g[DAT_S_XL(n) + c];
      vl[c] = g[DAT_S_VL(n) + c];
      wl[c] = g[DAT_S_WL(n) + c];
      fd[c] = fdes[(size_t)sc * 3 * n + 3 * i + c];
    }
    cnt = a.counter[sc];
  }
  const double* J = prm + DAT_P_J(n) + 9 * i;
  const double* Ji = prm + DAT_P_JINV(n) + 9 * i;
  double* mine = xs + lane * RO_X;
  const double* grp = xs + ls * n * RO_X;
  for (int s = 0; s < steps; ++s) {
    double dw[3] = {0, 0, 0};
    if (valid) {
      double f, M[3], Jw[3], wJw[3], t[3];
      ll_control_agent(R, W, J, fd, &f, M, a.ll_kind);
      mv3(J, W, Jw);
      cross3(W, Jw, wJw);
      for (int c = 0; c < 3; ++c) t[c] = M[c] - wJw[c];
      mv3(Ji, t, dw);
      double u[3] = {R[2] * f, R[5] * f, R[8] * f};  // f R e3
      double ub[3], m3[3];
      mtv3(Rl, u, ub);
      cross3(prm + DAT_P_RCOM(n) + 3 * i, ub, m3);
      for (int c = 0; c < 3; ++c) { mine[c] = u[c]; mine[3 + c] = m3[c]; }
    }
    __syncthreads();
    if (valid) {
      double dvc[3] = {0, 0, 0}, mom[3] = {0, 0, 0};
      for (int k = 0; k < n; ++k)
        for (int c = 0; c < 3; ++c) { dvc[c] += grp[k * RO_X + c]; mom[c] += grp[k * RO_X + 3 + c]; }
      const double mT = prm[DAT_P_MT];
      const double* xc = prm + DAT_P_XCOM;
      for (int c = 0; c < 3; ++c) dvc[c] /= mT;
      dvc[2] -= DAT_GRAVITY;
      double Jwl[3], wJwl[3], t[3], dwl[3];
      mv3(prm + DAT_P_JT, wl, Jwl);
      cross3(wl, Jwl, wJwl);
      for (int c = 0; c < 3; ++c) t[c] = mom[c] - wJwl[c];
      mv3(prm + DAT_P_JTI, t, dwl);
      double a1[3], a2[3], a3[3], sum[3], Rs[3], dvl[3];
      cross3(wl, xc, a1);
      cross3(wl, a1, a2);
      cross3(dwl, xc, a3);
      for (int c = 0; c < 3; ++c) sum[c] = a2[c] + a3[c];
      mv3(Rl, sum, Rs);
      for (int c = 0; c < 3; ++c) dvl[c] = dvc[c] - Rs[c];
      {
        double v[3], E[9], Rn[9];
        for (int c = 0; c < 3; ++c) v[c] = (W[c] + dw[c] * dt / 2.0) * dt;
        exp3(v, E);
        mm3(R, E, Rn);
        for (int k = 0; k < 9; ++k) R[k] = Rn[k];
        for (int c = 0; c < 3; ++c) W[c] += dw[c] * dt;
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
        for (int k = 0; k < 9; ++k) Rl[k] = Rn[k];
        for (int c = 0; c < 3; ++c) wl[c] += dwl[c] * dt;
      }
      cnt += 1;
      if (cnt >= 20) {  // _INTEGRATION_STEPS_PER_ROTATION_PROJECTION
        polar3(Rl);
        polar3(R);
        cnt = 0;
      }
    }
    __syncthreads();  // the sums are read before the next step overwrites them
  }
  if (valid) {
    for (int k = 0; k < 9; ++k) g[DAT_S_R(n) + 9 * i + k] = R[k];
    for (int c = 0; c < 3; ++c) g[DAT_S_W(n) + 3 * i + c] = W[c];
    if (i == 0) {
      for (int c = 0; c < 3; ++c) {
        g[DAT_S_XL(n) + c] = xl[c];
        g[DAT_S_VL(n) + c] = vl[c];
        g[DAT_S_WL(n) + c] = wl[c];
      }
      for (int k = 0; k < 9; ++k) g[DAT_S_RL(n) + k] = Rl[k];
      a.counter[sc] = cnt;
    }
  }
}

void launch_rollout(const KArgs& a, int B, hipStream_t stream, int steps, double dt, const double* fdes) {
  const int G = 64 / a.n;
  hipLaunchKernelGGL(k_rollout_agents, dim3((B + G - 1) / G), dim3(64), 0, stream, a, steps, dt, fdes);
}

// RQPLowLevelController.control (control/rqp_centralized.py:518-535) at the current states: thrust
// f (B x n) and moments M (B x n x 3) from f_des, one lane per (scenario, agent)
__global__ void k_low_level(KArgs a, const double* fdes, double* fo, double* Mo) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = a.n;
  if (t >= a.B * n) return;
  const int sc = t / n, i = t - sc * n;
  const double* prm = prm_of(a, sc);
  const double* st = a.state + (size_t)sc * a.S;
  ll_control_agent(st + DAT_S_R(n) + 9 * i, st + DAT_S_W(n) + 3 * i, prm + DAT_P_J(n) + 9 * i,
                   fdes + (size_t)sc * 3 * n + 3 * i, fo + t, Mo + 3 * (size_t)t, a.ll_kind);
}

// rigid payload (system/rigid_payload.py:93-130): `steps` steps of dt with the forces f held, one lane per scenario
__global__ void k_rp_rollout(KArgs a, int steps, double dt, const double* f) {
  const int sc = blockIdx.x * blockDim.x + threadIdx.x;
  if (sc >= a.B) return;
  const int n = a.n;
  const double* prm = prm_of(a, sc);
  double* st = a.state + (size_t)sc * a.S;
  int cnt = a.counter[sc];
  for (int s = 0; s < steps; ++s) rp_step(prm, n, st, &cnt, f + (size_t)sc * 3 * n, dt);
  a.counter[sc] = cnt;
}

__global__ void k_desired(KArgs a, double* acc) {
  const int sc = blockIdx.x * blockDim.x + threadIdx.x;
  if (sc >= a.B) return;
  const double* st = a.state + (size_t)sc * a.S;
  double* o = acc + (size_t)sc * 6;
  int f = (a.nforest > 0) ? (a.scen_forest ? a.scen_forest[sc] : 0) : -1;
  if (f < 0 || a.mountain == nullptr) {
    double m0[DAT_MOUNTAIN_SIZE] = {30.0, 0.0, 25.0, 1e300, 0.0};
    desired_accel_forest(st, a.n, m0, 1.5, o);
  } else {
    desired_accel_forest(st, a.n, a.mountain + (size_t)f * DAT_MOUNTAIN_SIZE, 1.5, o);
  }
}

__global__ void k_warm(KArgs a) {
  const int sc = blockIdx.x * blockDim.x + threadIdx.x;
  if (sc >= a.B) return;
  const int n = a.n, N3 = 3 * n;
  const double* prm = prm_of(a, sc);
  const double* feq = prm + DAT_P_FEQ(n);
  if (a.cf) {
    for (int i = 0; i < n; ++i)
      for (int c = 0; c < N3; ++c) {
        a.cf[((size_t)sc * n + i) * N3 + c] = feq[c];
        a.clam[((size_t)sc * n + i) * N3 + c] = 0.0;
      }
    for (int c = 0; c < N3; ++c) a.cfbar[(size_t)sc * N3 + c] = feq[c];
  }
  if (a.dlamF) {
    double s3[3] = {0, 0, 0};
    for (int k = 0; k < n; ++k)
      for (int c = 0; c < 3; ++c) s3[c] += feq[3 * k + c];
    for (int c = 0; c < N3; ++c) { a.dlamF[(size_t)sc * N3 + c] = 0.0; a.dlamM[(size_t)sc * N3 + c] = 0.0; }
    for (int i = 0; i < n; ++i) {
      double* pv = a.dprev + ((size_t)sc * n + i) * 9;
      for (int c = 0; c < 3; ++c) { pv[c] = feq[3 * i + c]; pv[3 + c] = s3[c] - feq[3 * i + c]; }
      double rf[3], jr[3];
      cross3(prm + DAT_P_RCOM(n) + 3 * i, pv, rf);
      mv3(prm + DAT_P_JTI, rf, jr);
      for (int c = 0; c < 3; ++c) pv[6 + c] = -jr[c];
    }
  }
  if (a.pf)
    for (int c = 0; c < N3; ++c) a.pf[(size_t)sc * N3 + c] = feq[c];
  for (int c = 0; c < N3; ++c) a.fdes[(size_t)sc * N3 + c] = feq[c];
  // the previous step's ADMM / DD iteration count and slowest IPM count select the IPM start (C-ADMM
  // warm regime) and the drain order: a reset handle behaves exactly like a freshly created one
  a.iters[sc] = 0;
  if (a.ipmx) a.ipmx[sc] = 0;
}

__global__ void k_env(KArgs a, double* lhs, double* rhs, int* nrow, unsigned char* col, double* md) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = a.n;
  if (t >= a.B * n) return;
  const int sc = t / n, i = t % n;
  const double* prm = prm_of(a, sc);
  const double* st = a.state + (size_t)sc * a.S;
  const double* trees;
  int nt, k = 0;
  unsigned mask;
  forest_of(a, sc, &trees, &nt);
  double L[DAT_NENV][3], R[DAT_NENV];
  bool cent = (a.cf == nullptr && a.dlamF == nullptr);
  EnvOut e = env_rows(prm, n, st, trees, nt, cent ? -1 : i, cent ? prm[DAT_P_AENVC] : prm[DAT_P_AENVD], &mask, L, R);
  double* lo = lhs + (size_t)t * DAT_NENV * 3;
  double* ro = rhs + (size_t)t * DAT_NENV;
  for (int r = 0; r < DAT_NENV; ++r) {
    for (int c = 0; c < 3; ++c) lo[3 * r + c] = 0.0;
    ro[r] = 0.0;
  }
#pragma unroll
  for (int r = 0; r < DAT_NENV; ++r) {
    if (!((mask >> r) & 1u)) continue;
    for (int c = 0; c < 3; ++c) lo[3 * k + c] = L[r][c];
    ro[k] = R[r];
    ++k;
  }
  nrow[t] = k;
  col[t] = (unsigned char)e.collision;
  md[t] = e.min_env_dist;
}

// ------------------------------------------------------------------------------------------------
// raw batched agent QPs: RQPPrimalSolver.solve (control/rqp_cadmm.py:482-501, control/rqp_dd.py:475-505)
// ------------------------------------------------------------------------------------------------
// One lane per item (a scenario's state / parameters / forest, one agent, its own multipliers).
// Not a hot path: the scenario data live in lane registers / scratch (PlainRef), as in k_cent.
struct AgentQPArgs {
  int count;
  const int *scen, *agent;
  const double *acc, *lam, *rho, *fbar, *c9;
  double* x;
  int *status, *iters;
  unsigned char* col;
  double* mind;
  double* best;
};

__global__ __launch_bounds__(64) void k_agent_qp(KArgs a, AgentQPArgs q) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = k < q.count;
  const int n = a.n, N3 = 3 * n;
  const bool dd = a.dlamF != nullptr;
  const int sc = valid ? q.scen[k] : 0, i = valid ? q.agent[k] : 0;
  const double* prm = prm_of(a, sc);
  const double* st = a.state + (size_t)sc * a.S;
  QPShared S;
  QPLane<1> P;
  EnvRows E;
  double Rt_all[NMAX * 9];
  int nr = NBASE;
  EnvOut env;
  env.collision = 0;
  env.min_env_dist = 0.0;
  if (valid) {
    for (int j = 0; j < n; ++j) make_Rt(prm + DAT_P_RCOM(n) + 3 * j, st + DAT_S_RL(n), Rt_all + 9 * j);
    build_shared(S, prm, n, st, q.acc + (size_t)k * 6, prm[DAT_P_KFD], prm[DAT_P_KMD], 3, !dd);
    if (dd) {
      lane_dd_static(P, prm, i);
    } else {
      lane_cadmm_static(P, prm, i);
    }
    const double* trees;
    int nt;
    unsigned emask;
    forest_of(a, sc, &trees, &nt);
    double lhs[DAT_NENV][3], rhs[DAT_NENV];
    env = env_rows(prm, n, st, trees, nt, i, prm[DAT_P_AENVD], &emask, lhs, rhs);
    set_env_rows(P, E, S, emask, lhs, rhs);
    nr = rows_needed(P.emask);
    if (dd) {
      set_dd_price(P, prm, n, i, q.c9 + (size_t)k * 9);
    } else {
      lane_cadmm_dynamic(P, prm, n, i, Rt_all, q.lam + (size_t)k * N3, q.fbar + (size_t)k * N3, q.rho[k]);
    }
  }
  nr = wave_max(nr);
  if (!valid) return;
  double y[1][3], w[6];
  const PlainRef<QPShared> shr{&S};
  const EnvPlain er{&E};
  const RtPtr rtr{Rt_all + 9 * i};
  double* bst = q.best + (size_t)k * best_size(1);
  // the C-ADMM agent QP as the closed loop solves it: rows certified infeasible are held (k_cadmm_tail)
  if (!dd && !P.infeasible && dvl_rows_infeasible(shr, er, P.emask)) P.infeasible = 1;
  IPMOut o = dd ? ipm_solve_rows<MODE_DD, 1>(nr, shr, er, rtr, P, prm + DAT_P_FEQ(n) + 3 * i, y, w, bst, IPM_MAX_ITER,
                                             a.qp_tol)
                : ipm_solve_rows<MODE_CADMM, 1, IPM_FAST_REDO>(nr, shr, er, rtr, P, prm + DAT_P_FEQ(n) + 3 * i, y, w, bst,
                                                IPM_MAX_ITER, a.qp_tol);
  if (dd) {
    double* xo = q.x + (size_t)k * 9;
    for (int c = 0; c < 3; ++c) xo[c] = y[0][c];
    for (int c = 0; c < 6; ++c) xo[3 + c] = w[c];
  } else {
    double* xo = q.x + (size_t)k * N3;
    const double rho = q.rho[k];
    for (int j = 0; j < n; ++j) {
      if (j == i) {
        for (int c = 0; c < 3; ++c) xo[3 * j + c] = y[0][c];
      } else {
        cadmm_free_block(Rt_all + 9 * j, q.lam + (size_t)k * N3 + 3 * j, q.fbar + (size_t)k * N3 + 3 * j, o.pi, rho,
                         xo + 3 * j);
      }
    }
  }
  // in-band accepts (rare: per lane, no wavefront reduction)
  if (o.inband) atomicAdd(a.counters + CNT_INBAND, 1);
  if (inband_loose(o)) atomicAdd(a.counters + CNT_INBAND + 1, 1);
  atomicAdd(a.counters + CNT_REF, (unsigned long long)o.refs);
  atomicAdd(a.counters + CNT_REF + 1, (unsigned long long)o.corrs);
  q.status[k] = o.status;
  q.iters[k] = o.iters;
  q.col[k] = (unsigned char)env.collision;
  q.mind[k] = env.min_env_dist;
}

}  // namespace

// ================================================================================================
// handle + C-ABI
// ================================================================================================
constexpr int DAT_MAX_SUB = 4;  // sub-batches of the C-ADMM closed loop (dat_set_sub_batches)
struct dat_handle {
  dat_config cfg;
  int P = 0, S = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipEvent_t ek = nullptr;       // C-ADMM: after k_bucket
  double cadmm_ms = 0.0;         // summed device time of k_cadmm
  int persistent_blocks = 1024;  // C-ADMM: resident k_cadmm blocks (CUs x 4 wavefronts)
  double qp_tol = IPM_TOL;       // IPM stopping tolerance (dat_set_qp_tolerance)
  double* params = nullptr;
  int ppp = 0;
  bool have_params = false;
  double *state = nullptr, *acc = nullptr, *fdes = nullptr;
  int* counter = nullptr;
  double* trees = nullptr;
  int* tree_off = nullptr;
  int* scen_forest = nullptr;
  double* mountain = nullptr;
  int nforest = 0;
  double *cf = nullptr, *cfbar = nullptr, *clam = nullptr;
  int *rlist = nullptr, *rres = nullptr;  // C-ADMM: robust lists, resume records
  double *dlamF = nullptr, *dlamM = nullptr, *dprev = nullptr, *dHinv = nullptr;
  double* pf = nullptr;
  double* best = nullptr;
  int *iters = nullptr, *qstatus = nullptr;
  double *mind = nullptr, *err = nullptr;
  unsigned char* col = nullptr;
  unsigned long long* counters = nullptr;  // DAT_NCOUNTERS: [CNT_STRIDE k + .] of env class k (C-ADMM); [0..2] otherwise
  int *need = nullptr, *slist = nullptr, *scount = nullptr, *ipmx = nullptr;
  double* erows = nullptr;     // C-ADMM: env rows of the step, k_env_class -> k_cadmm
  unsigned* emask = nullptr;
  long long hl_steps = 0;
  double hl_ms = 0.0;
  // host clock marks of the last dat_closed_loop call: its start, then each HL step's k_cadmm / k_dd /
  // k_cent completion (ms on a steady clock); consecutive differences are the per-step times of a
  // back-to-back run (dat_get_step_marks)
  std::vector<double> marks;
  double* acc_seq = nullptr;  // dat_control_steps: K x B x 6 desired accelerations (grown on demand)
  size_t acc_seq_cap = 0;
  // C-ADMM closed loop on sub-batches (dat_set_sub_batches): contiguous scenario ranges, each with its own
  // stream, so one sub-batch's kernels fill the drain tail and the short kernels of the others
  int nsub = 1;
  std::vector<hipEvent_t> sub_ev;  // closed_loop_sub: k_cadmm start / end events per sub-batch and step
  hipStream_t sub_stream[DAT_MAX_SUB] = {};
  hipEvent_t sub_done[DAT_MAX_SUB] = {};
  hipEvent_t ev_start = nullptr, ev_end = nullptr;
  // C-ADMM with a forest: per sub-batch the stream of the concurrent tail launch and its start / end events
  hipStream_t tail_stream = nullptr;  // C-ADMM, one sub-batch: the tail-routed scenarios' launch beside k_cadmm
  hipEvent_t tail_ev[2] = {};
  double* wrec = nullptr;  // C-ADMM: the tail's warm-start records (B n WREC_SIZE)
  double agent_qp_ms = 0.0;  // device time of the last dat_solve_agent_qp_batch launch
  int ll_kind = 0;  // LL_PD (example/rqp_example.py:113) or LL_SM
  std::vector<void*> allocs;
};

// C-ADMM scenario slots per k_cadmm wavefront: floor(64/n), fewer when the batch would not give
// every CU a wavefront.  A small batch is then spread one wavefront per CU (a wavefront's ADMM pass
// waits for the slowest of fewer lanes).  Not further: wavefronts sharing a CU pair's instruction
// cache at different points of the ~100 KB unrolled IPM slow each other down (C2, 1,024 scenarios,
// target blocks 1024 / 256 / 64 / floor(64/n) packing: 14.7 / 13.0 / 14.4 / 14.2 ms per step).
int cadmm_slots(const dat_handle* h, int B, int n) {
  const int gmax = 64 / n;
  int pb = h->persistent_blocks / 4 > 0 ? h->persistent_blocks / 4 : 1;
  const int g = (B + pb - 1) / pb;
  return g < 1 ? 1 : (g > gmax ? gmax : g);
}

namespace {

template <typename T>
int dalloc(dat_handle* h, T** p, size_t count) {
  *p = nullptr;
  if (count == 0) return 0;
  HIPCHK(hipMalloc((void**)p, count * sizeof(T)));
  HIPCHK(hipMemsetAsync(*p, 0, count * sizeof(T), h->stream));
  h->allocs.push_back(*p);
  return 0;
}

void dfree(dat_handle* h, void* p) {
  if (!p) return;
  for (auto& q : h->allocs)
    if (q == p) q = nullptr;
  (void)hipFree(p);
}

KArgs kargs(dat_handle* h) {
  KArgs a;
  memset(&a, 0, sizeof(a));
  const dat_config& c = h->cfg;
  a.B = c.batch;
  a.n = c.n;
  a.G = cadmm_slots(h, c.batch, c.n);
  a.P = h->P;
  a.S = h->S;
  a.ppp = h->ppp;
  a.params = h->params;
  a.state = h->state;
  a.counter = h->counter;
  a.acc = h->acc;
  a.fdes = h->fdes;
  a.trees = h->trees;
  a.tree_off = h->tree_off;
  a.scen_forest = h->scen_forest;
  a.nforest = h->nforest;
  a.mountain = h->mountain;
  a.max_iter = c.max_iter;
  a.res_tol = c.res_tol;
  a.use_total_res = c.use_total_res;
  a.rho0 = c.rho0;
  a.tau = c.tau_incr;
  a.rho_max = c.rho_max;
  a.record_err = c.record_err;
  a.qp_tol = h->qp_tol;
  a.ksteps = 1;
  a.cf = h->cf;
  a.cfbar = h->cfbar;
  a.clam = h->clam;
  a.dlamF = h->dlamF;
  a.dlamM = h->dlamM;
  a.dprev = h->dprev;
  a.dHinv = h->dHinv;
  a.pf = h->pf;
  a.best = h->best;
  a.iters = h->iters;
  a.qstatus = h->qstatus;
  a.mind = h->mind;
  a.col = h->col;
  a.err = h->err;
  a.counters = h->counters;
  a.need = h->need;
  a.ipmx = h->ipmx;
  a.erows = h->erows;
  a.emask = h->emask;
  a.slist = h->slist;
  a.scount = h->scount;
  a.qhead = h->scount ? h->scount + 2 * NCLS : nullptr;
  a.rlist = h->rlist;
  a.rres = h->rres;
  a.ll_kind = h->ll_kind;
  a.wrec = h->wrec;
  a.tail_prev = h->nforest > 0 ? TAIL_PREV : INT_MAX;
  a.tail_pass = h->nforest > 0 ? TAIL_PASS : INT_MAX;
  // the concurrent tail launch needs a stream of its own beside the step's: with sub-batches (4 streams) a fifth
  // and more would share the box's GPU_MAX_HW_QUEUES = 4 hardware queues with them and serialise the sub-batches
  a.route = h->cfg.mode == DAT_MODE_CADMM && h->nforest > 0 && h->nsub == 1;
  // (created on first use: a stream made at dat_create would take a hardware queue from the sub-batch streams)
  if (a.route && !h->tail_stream &&
      (hipStreamCreateWithFlags(&h->tail_stream, hipStreamNonBlocking) != hipSuccess ||
       hipEventCreateWithFlags(&h->tail_ev[0], hipEventDisableTiming) != hipSuccess ||
       hipEventCreateWithFlags(&h->tail_ev[1], hipEventDisableTiming) != hipSuccess))
    a.route = 0;  // (no stream: the wedged scenarios go through k_cadmm's hand-over, same results)
  a.tmode = 0;
#ifdef DAT_NO_TAIL  // A/B builds only (tools/build_var.sh): the round-5 schedule, no tail rule
  a.tail_prev = a.tail_pass = INT_MAX;
  a.route = 0;
#endif
  return a;
}

size_t dd_lds(int n, bool env) {
  int G = 64 / n, NT = G * n;
  return sizeof(double) * (al2((size_t)NT * 9) + 2 * al2((size_t)G * 3 * n) + al2((size_t)NT * DD_ES) +
                           (size_t)G * RT_STRIDE * n + 64 * DD_RS) +
         sizeof(QPShared) * (size_t)G + sizeof(double) * dd_area_doubles(env) + sizeof(int) * 192;
}
size_t dd_setup_lds(int n) {
  int N = 6 * n;
  return sizeof(double) * (81 * (size_t)n + 9 * (size_t)n + dd_setup_hs(n) + N);
}

// the C-ADMM drain of one control step: k_cadmm (env classes 3, 2, 1, 0) with a forest, k_cadmm0 without.
// k_cadmm_tail: one scenario slot per block (G = 1).  Its scenarios are few -- stalled ADMM loops next to trees,
// 101 sequential passes -- and a slot of its own per scenario keeps one scenario's pass from waiting for the
// slowest agent QP of the others'.  With a forest two launches: the tail-routed scenarios on the sub-batch's
// tail stream, started with k_cadmm (their lists are known after k_bucket), and the hand-over lists after
// k_cadmm on the step's stream, which then waits for the first.
constexpr int TAIL_BLOCKS = 256;
int launch_cadmm(const dat_handle* h, const KArgs& a, int blocks, hipStream_t st) {
  KArgs r = a;
  r.G = 1;
  if (h->nforest > 0) {
    if (a.route) {
      KArgs t = r;
      t.tmode = 1;
      const hipStream_t ts = h->tail_stream;
      HIPCHK(hipEventRecord(h->tail_ev[0], st));
      HIPCHK(hipStreamWaitEvent(ts, h->tail_ev[0], 0));
      hipLaunchKernelGGL(k_cadmm_tail, dim3(TAIL_BLOCKS), dim3(64), cadmm_tail_lds_bytes(a.n, NCLS - 1), ts, t);
      HIPCHK(hipEventRecord(h->tail_ev[1], ts));
    }
    hipLaunchKernelGGL(k_cadmm, dim3(blocks), dim3(64), cadmm_lds_bytes(a.n, a.G, NCLS - 1), st, a);
    hipLaunchKernelGGL(k_cadmm_tail, dim3(TAIL_BLOCKS), dim3(64), cadmm_tail_lds_bytes(r.n, NCLS - 1), st, r);
    if (a.route) HIPCHK(hipStreamWaitEvent(st, h->tail_ev[1], 0));
  } else {
    hipLaunchKernelGGL(k_cadmm0, dim3(blocks), dim3(64), cadmm_lds_bytes(a.n, a.G, 0), st, a);
    hipLaunchKernelGGL(k_cadmm0_tail, dim3(TAIL_BLOCKS), dim3(64), cadmm_tail_lds_bytes(r.n, 0), st, r);
  }
  return 0;
}

// ksteps > 1 (dat_control_steps): that many control steps fused into one drain, acc_seq ksteps x B x 6
int launch_hl(dat_handle* h, int ksteps = 1, const double* acc_seq = nullptr) {
  KArgs a = kargs(h);
  a.ksteps = ksteps;
  if (acc_seq) a.acc = acc_seq;
  const int n = h->cfg.n, B = h->cfg.batch;
  if (!h->have_params) return fail("dat_set_params has not been called");
  if (h->cfg.record_err && h->err)
    HIPCHK(hipMemsetAsync(h->err, 0xff, sizeof(double) * (size_t)B * (h->cfg.max_iter + 1), h->stream));  // NaN pad
  HIPCHK(hipEventRecord(h->e0, h->stream));
  if (h->cfg.mode == DAT_MODE_CADMM) {
    int G = 64 / n;
    int blocks = (B + G - 1) / G;
    hipLaunchKernelGGL(k_env_class, dim3(blocks), dim3(64), 0, h->stream, a);
    hipLaunchKernelGGL(k_bucket, dim3(1), dim3(BUCKET_T), 0, h->stream, B, (const int*)h->need, h->slist, h->scount);
    HIPCHK(hipEventRecord(h->ek, h->stream));
    const int Gc = a.G, cblocks = (B + Gc - 1) / Gc;
    if (launch_cadmm(h, a, std::min(cblocks, h->persistent_blocks), h->stream)) return -1;
  } else if (h->cfg.mode == DAT_MODE_DD) {
    if (n > DD_REG_NMAX)  // [H | I] in LDS: beyond the default 64 KB dynamic LDS from n = 11 on
      HIPCHK(hipFuncSetAttribute((const void*)k_dd_setup<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)dd_setup_lds(n)));
    switch (n <= DD_REG_NMAX ? n : 0) {
      case 3: hipLaunchKernelGGL(k_dd_setup<3>, dim3(B), dim3(64), dd_setup_lds(n), h->stream, a); break;
      case 4: hipLaunchKernelGGL(k_dd_setup<4>, dim3(B), dim3(64), dd_setup_lds(n), h->stream, a); break;
      case 5: hipLaunchKernelGGL(k_dd_setup<5>, dim3(B), dim3(64), dd_setup_lds(n), h->stream, a); break;
      case 6: hipLaunchKernelGGL(k_dd_setup<6>, dim3(B), dim3(64), dd_setup_lds(n), h->stream, a); break;
      case 7: hipLaunchKernelGGL(k_dd_setup<7>, dim3(B), dim3(64), dd_setup_lds(n), h->stream, a); break;
      case 8: hipLaunchKernelGGL(k_dd_setup<8>, dim3(B), dim3(64), dd_setup_lds(n), h->stream, a); break;
      default: hipLaunchKernelGGL(k_dd_setup<0>, dim3(B), dim3(64), dd_setup_lds(n), h->stream, a); break;
    }
    hipLaunchKernelGGL(k_dd_key, dim3((B + 63) / 64), dim3(64), 0, h->stream, a);
    hipLaunchKernelGGL(k_bucket, dim3(1), dim3(BUCKET_T), 0, h->stream, B, (const int*)h->need, h->slist, h->scount);
    HIPCHK(hipEventRecord(h->ek, h->stream));
    int G = 64 / n;
    int blocks = (B + G - 1) / G;
    if (h->nforest > 0)
      hipLaunchKernelGGL(k_dd<true>, dim3(std::min(blocks, h->persistent_blocks)), dim3(64), dd_lds(n, h->nforest > 0), h->stream, a);
    else
      hipLaunchKernelGGL(k_dd<false>, dim3(std::min(blocks, h->persistent_blocks)), dim3(64), dd_lds(n, h->nforest > 0), h->stream, a);
  } else {
    HIPCHK(launch_cent(n, B, h->stream, a));
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(h->e1, h->stream));
  return 0;
}

// kernel arguments of the C-ADMM sub-batch of scenarios [off, off + Bs) (dat_set_sub_batches): every
// per-scenario array offset, the env-row image a disjoint block of the SoA buffer (stride Bs n), the
// class table its own; counters shared (atomics)
template <class T>
T* offp(T* p, size_t k) { return p ? p + k : p; }
KArgs sub_kargs(dat_handle* h, int off, int Bs, int s) {
  KArgs a = kargs(h);
  const size_t n = h->cfg.n, N3 = 3 * n, o = (size_t)off;
  a.B = Bs;
  a.G = cadmm_slots(h, Bs, (int)n);
  if (a.ppp) a.params += o * a.P;
  a.state += o * a.S;
  a.counter += o;
  a.acc += o * 6;
  a.fdes += o * N3;
  a.scen_forest = offp(a.scen_forest, o);
  a.cf += o * n * N3;
  a.cfbar += o * N3;
  a.clam += o * n * N3;
  a.best += o * n * best_size(1);
  a.iters += o;
  a.qstatus += o * n;
  a.mind += o;
  a.col += o;
  a.err = offp(a.err, o * (a.max_iter + 1));
  a.need += o;
  a.ipmx += o;
  a.slist += o;
  a.rlist += o;
  a.rres += o * RRES_INTS;
  a.wrec += o * n * WREC_SIZE;
  a.scount = h->scount + SCOUNT_INTS * s;
  a.qhead = a.scount + 2 * NCLS;
  a.erows += (size_t)4 * DAT_NENV * n * o;
  a.emask += o * n;
  return a;
}

int finish_hl(dat_handle* h, int ksteps = 1) {
  HIPCHK(hipEventSynchronize(h->e1));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, h->e0, h->e1));
  h->hl_ms += ms;
  if (h->cfg.mode != DAT_MODE_CENTRALIZED) {  // k_cadmm / k_dd: from after k_bucket to the end of the step
    float mk = 0.f;
    HIPCHK(hipEventElapsedTime(&mk, h->ek, h->e1));
    h->cadmm_ms += mk;
  }
  h->hl_steps += ksteps;
  return 0;
}

}  // namespace

extern "C" {

#ifdef DAT_CAPTURE_LOOSE
int dat_get_captures(double* out, int* count) {
  HIPCHK(hipDeviceSynchronize());
  unsigned int k = 0;
  HIPCHK(hipMemcpyFromSymbol(&k, HIP_SYMBOL(dat::g_ncap), sizeof(k)));
  *count = (int)k;
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(dat::g_cap), sizeof(double) * CAP_MAX * CAP_DOUBLES));
  return 0;
}
#endif
#ifdef DAT_ITER_HIST
int dat_get_iter_hist(unsigned long long* out) {
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(dat::g_iter_hist), sizeof(unsigned long long) * 64));
  unsigned long long z[64] = {0};
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(dat::g_iter_hist), z, sizeof(z)));
  return 0;
}
#endif
#ifdef DAT_PHASE_PROF
// development builds only (tools/phase_prof.py): the IPM phase cycle sums, reset after the read
int dat_get_phase_cycles(unsigned long long* out) {
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(dat::g_phase), sizeof(unsigned long long) * 16));
  unsigned long long z[16] = {0};
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(dat::g_phase), z, sizeof(z)));
  return 0;
}
#endif

void dat_default_config(dat_config* c) {
  memset(c, 0, sizeof(*c));
  c->device = 0;
  c->mode = DAT_MODE_CADMM;
  c->n = 3;
  c->batch = 1;
  c->dt = 1e-3;
  c->hl_every = 10;
  c->max_iter = 100;
  c->res_tol = 1e-2;
  c->use_total_res = 1;
  c->rho0 = 1.0;
  c->tau_incr = 1.0;
  c->rho_max = 2.0;
  c->record_err = 0;
}

const char* dat_last_error(void) { return g_err.c_str(); }

int dat_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

int dat_create(const dat_config* cfg, dat_handle** out) {
  if (!cfg || !out) return fail("dat_create: null argument");
  *out = nullptr;
  const dat_config& c = *cfg;
  if (c.n < 3 || c.n > NMAX) return fail("dat_create: n must be in [3, 16]");
  if (c.mode == DAT_MODE_DD && c.n > NMAX_DD) return fail("dat_create: DD supports n <= 16");
  if (c.mode == DAT_MODE_CENTRALIZED && c.n > NMAX_CENT) return fail("dat_create: centralized supports n <= 16");
  if (c.mode < 0 || c.mode > 2) return fail("dat_create: bad mode");
  if (c.batch < 1) return fail("dat_create: batch must be >= 1");
  if (c.max_iter < 0) return fail("dat_create: max_iter must be >= 0");
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (c.device < 0 || c.device >= ndev) return fail("dat_create: no such HIP device");
  HIPCHK(hipSetDevice(c.device));
  dat_handle* h = new dat_handle();
  h->cfg = c;
  h->P = DAT_PARAM_SIZE(c.n);
  h->S = DAT_STATE_SIZE(c.n);
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&h->e0) != hipSuccess || hipEventCreate(&h->e1) != hipSuccess ||
      hipEventCreate(&h->ek) != hipSuccess) {
    delete h;
    return fail("dat_create: stream/event creation failed");
  }
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c.device) == hipSuccess && ncu > 0)
    h->persistent_blocks = 4 * ncu;  // k_cadmm: one wavefront per SIMD (register-bound), 4 SIMDs per CU
  const size_t B = c.batch, n = c.n, N3 = 3 * n;
  int rc = 0;
  rc |= dalloc(h, &h->state, B * h->S);
  rc |= dalloc(h, &h->counter, B);
  rc |= dalloc(h, &h->acc, B * 6);
  rc |= dalloc(h, &h->fdes, B * N3);
  rc |= dalloc(h, &h->iters, B);
  rc |= dalloc(h, &h->qstatus, B * n);
  rc |= dalloc(h, &h->mind, B);
  rc |= dalloc(h, &h->col, B);
  rc |= dalloc(h, &h->counters, DAT_NCOUNTERS);
  if (c.record_err) rc |= dalloc(h, &h->err, B * (c.max_iter + 1));
  if (c.mode == DAT_MODE_CADMM) {
    rc |= dalloc(h, &h->need, B);
    rc |= dalloc(h, &h->ipmx, B);
    rc |= dalloc(h, &h->erows, (size_t)B * n * DAT_NENV * 4);
    rc |= dalloc(h, &h->emask, (size_t)B * n);
    rc |= dalloc(h, &h->slist, B);
    rc |= dalloc(h, &h->scount, SCOUNT_INTS * DAT_MAX_SUB);  // one class table per sub-batch
    rc |= dalloc(h, &h->cf, B * n * N3);
    rc |= dalloc(h, &h->cfbar, B * N3);
    rc |= dalloc(h, &h->clam, B * n * N3);
    rc |= dalloc(h, &h->rres, B * RRES_INTS);
    rc |= dalloc(h, &h->rlist, B);
    rc |= dalloc(h, &h->wrec, B * n * WREC_SIZE);
  } else if (c.mode == DAT_MODE_DD) {
    rc |= dalloc(h, &h->need, B);
    rc |= dalloc(h, &h->ipmx, B);
    rc |= dalloc(h, &h->slist, B);
    rc |= dalloc(h, &h->scount, SCOUNT_INTS);
    rc |= dalloc(h, &h->dlamF, B * N3);
    rc |= dalloc(h, &h->dlamM, B * N3);
    rc |= dalloc(h, &h->dprev, B * n * 9);
#if DAT_DD_WARM
    rc |= dalloc(h, &h->wrec, B * n * WREC_SIZE);
#endif
    rc |= dalloc(h, &h->dHinv, B * 36 * n * n);
  } else {
    rc |= dalloc(h, &h->pf, B * N3);
  }
  // lane-private IPM best-iterate records
  // best-iterate records: one per agent QP lane (centralized: one per lane of the scenario's 16-lane slot)
  rc |= dalloc(h, &h->best, c.mode == DAT_MODE_CENTRALIZED ? B * 16 * (size_t)best_size(1) : B * n * (size_t)best_size(1));
  if (rc) {
    std::string m = g_err;
    dat_destroy(h);
    return fail(m);
  }
  if (dat_reset_counters(h)) {
    std::string m = g_err;
    dat_destroy(h);
    return fail(m);
  }
  if (c.mode == DAT_MODE_CADMM) {  // the tail's workgroup may exceed the default 64 KB of dynamic LDS
    const int tl = (int)cadmm_tail_lds_bytes(c.n);
    if (hipFuncSetAttribute((const void*)k_cadmm_tail, hipFuncAttributeMaxDynamicSharedMemorySize, tl) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_cadmm0_tail, hipFuncAttributeMaxDynamicSharedMemorySize, tl) != hipSuccess) {
      dat_destroy(h);
      return fail("dat_create: tail kernel LDS attribute");
    }
  }
  // LDS budgets
  size_t lds = c.mode == DAT_MODE_CADMM ? cadmm_lds_bytes(c.n, 64 / c.n) : (c.mode == DAT_MODE_DD ? dd_setup_lds(c.n) : 0);
  if (lds > 160 * 1024) {
    dat_destroy(h);
    return fail("dat_create: LDS budget exceeded");
  }
  *out = h;
  return 0;
}

int dat_destroy(dat_handle* h) {
  if (!h) return 0;
  (void)hipSetDevice(h->cfg.device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  for (void* p : h->allocs)
    if (p) (void)hipFree(p);
  if (h->acc_seq) (void)hipFree(h->acc_seq);
  for (int s = 1; s < DAT_MAX_SUB; ++s) {
    if (h->sub_stream[s]) (void)hipStreamDestroy(h->sub_stream[s]);
    if (h->sub_done[s]) (void)hipEventDestroy(h->sub_done[s]);
  }
  if (h->tail_stream) {
    (void)hipStreamSynchronize(h->tail_stream);
    (void)hipStreamDestroy(h->tail_stream);
  }
  for (int e = 0; e < 2; ++e)
    if (h->tail_ev[e]) (void)hipEventDestroy(h->tail_ev[e]);
  if (h->ev_start) (void)hipEventDestroy(h->ev_start);
  if (h->ev_end) (void)hipEventDestroy(h->ev_end);
  for (hipEvent_t e : h->sub_ev) (void)hipEventDestroy(e);
  if (h->e0) (void)hipEventDestroy(h->e0);
  if (h->e1) (void)hipEventDestroy(h->e1);
  if (h->ek) (void)hipEventDestroy(h->ek);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

int dat_set_params(dat_handle* h, const double* params, int per_scenario) {
  if (!h || !params) return fail("dat_set_params: null argument");
  HIPCHK(hipSetDevice(h->cfg.device));
  size_t count = (per_scenario ? (size_t)h->cfg.batch : 1) * h->P;
  if (h->params) dfree(h, h->params);
  if (dalloc(h, &h->params, count)) return -1;
  HIPCHK(hipMemcpyAsync(h->params, params, count * sizeof(double), hipMemcpyHostToDevice, h->stream));
  h->ppp = per_scenario ? 1 : 0;
  h->have_params = true;
  return dat_reset_warm_start(h);
}

int dat_set_forests(dat_handle* h, int num_forests, const int* tree_offsets, const double* tree_pos,
                    const int* scenario_forest, const double* mountain) {
  if (!h) return fail("dat_set_forests: null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  HIPCHK(hipStreamSynchronize(h->stream));
  dfree(h, h->trees);
  dfree(h, h->tree_off);
  dfree(h, h->scen_forest);
  dfree(h, h->mountain);
  h->trees = nullptr;
  h->tree_off = nullptr;
  h->scen_forest = nullptr;
  h->mountain = nullptr;
  h->nforest = 0;
  if (num_forests <= 0) return 0;
  if (!tree_offsets || !tree_pos) return fail("dat_set_forests: null forest data");
  const int T = tree_offsets[num_forests];
  if (T < 0) return fail("dat_set_forests: bad offsets");
  for (int f = 0; f < num_forests; ++f)
    if (tree_offsets[f + 1] < tree_offsets[f]) return fail("dat_set_forests: offsets must be non-decreasing");
  if (dalloc(h, &h->trees, (size_t)(T > 0 ? T : 1) * 3) || dalloc(h, &h->tree_off, num_forests + 1)) return -1;
  if (T > 0) {
    // each forest's trees sorted by x: env_rows scans only the x-window of its vision range
    std::vector<double> sorted((size_t)3 * T);
    std::vector<int> idx;
    for (int f = 0; f < num_forests; ++f) {
      const int b = tree_offsets[f], e = tree_offsets[f + 1];
      idx.resize(e - b);
      for (int k = 0; k < e - b; ++k) idx[k] = b + k;
      std::stable_sort(idx.begin(), idx.end(), [&](int u, int v) { return tree_pos[3 * u] < tree_pos[3 * v]; });
      for (int k = 0; k < e - b; ++k)
        for (int c = 0; c < 3; ++c) sorted[(size_t)3 * (b + k) + c] = tree_pos[(size_t)3 * idx[k] + c];
    }
    HIPCHK(hipMemcpyAsync(h->trees, sorted.data(), sizeof(double) * 3 * T, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  HIPCHK(hipMemcpyAsync(h->tree_off, tree_offsets, sizeof(int) * (num_forests + 1), hipMemcpyHostToDevice, h->stream));
  if (scenario_forest) {
    for (int s = 0; s < h->cfg.batch; ++s)
      if (scenario_forest[s] >= num_forests) return fail("dat_set_forests: scenario_forest out of range");
    if (dalloc(h, &h->scen_forest, h->cfg.batch)) return -1;
    HIPCHK(hipMemcpyAsync(h->scen_forest, scenario_forest, sizeof(int) * h->cfg.batch, hipMemcpyHostToDevice, h->stream));
  }
  if (mountain) {
    if (dalloc(h, &h->mountain, (size_t)num_forests * DAT_MOUNTAIN_SIZE)) return -1;
    HIPCHK(hipMemcpyAsync(h->mountain, mountain, sizeof(double) * num_forests * DAT_MOUNTAIN_SIZE, hipMemcpyHostToDevice,
                          h->stream));
  }
  h->nforest = num_forests;
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int dat_set_tolerance(dat_handle* h, double res_tol, int use_total_res) {
  if (!h) return fail("null handle");
  h->cfg.res_tol = res_tol;
  h->cfg.use_total_res = use_total_res;
  return 0;
}

int dat_set_qp_tolerance(dat_handle* h, double tol) {
  if (!h) return fail("null handle");
  if (!(tol >= 1e-12 && tol <= 1e-7)) return fail("dat_set_qp_tolerance: tol must lie in [1e-12, 1e-7]");
  h->qp_tol = tol;
  return 0;
}

int dat_set_max_iter(dat_handle* h, int max_iter) {
  if (!h) return fail("null handle");
  if (max_iter < 0) return fail("dat_set_max_iter: negative");
  if (h->cfg.record_err && max_iter > h->cfg.max_iter) {
    HIPCHK(hipSetDevice(h->cfg.device));
    HIPCHK(hipStreamSynchronize(h->stream));
    dfree(h, h->err);
    h->err = nullptr;
    if (dalloc(h, &h->err, (size_t)h->cfg.batch * (max_iter + 1))) return -1;
  }
  h->cfg.max_iter = max_iter;
  return 0;
}

int dat_reset_warm_start(dat_handle* h) {
  if (!h) return fail("null handle");
  if (!h->have_params) return fail("dat_reset_warm_start: params not set");
  HIPCHK(hipSetDevice(h->cfg.device));
  KArgs a = kargs(h);
  hipLaunchKernelGGL(k_warm, dim3((h->cfg.batch + 63) / 64), dim3(64), 0, h->stream, a);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int dat_set_state(dat_handle* h, const double* state, const int* counters) {
  if (!h || !state) return fail("dat_set_state: null argument");
  HIPCHK(hipSetDevice(h->cfg.device));
  HIPCHK(hipMemcpyAsync(h->state, state, sizeof(double) * (size_t)h->cfg.batch * h->S, hipMemcpyHostToDevice, h->stream));
  if (counters)
    HIPCHK(hipMemcpyAsync(h->counter, counters, sizeof(int) * h->cfg.batch, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int dat_get_state(dat_handle* h, double* state, int* counters) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (state)
    HIPCHK(hipMemcpyAsync(state, h->state, sizeof(double) * (size_t)h->cfg.batch * h->S, hipMemcpyDeviceToHost, h->stream));
  if (counters)
    HIPCHK(hipMemcpyAsync(counters, h->counter, sizeof(int) * h->cfg.batch, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int dat_control_step(dat_handle* h, const double* state, const double* acc_des, double* f_des, int* iters,
                     int* qp_status, double* min_env_dist, unsigned char* collision, double* err_seq) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  const size_t B = h->cfg.batch, n = h->cfg.n;
  if (state) HIPCHK(hipMemcpyAsync(h->state, state, sizeof(double) * B * h->S, hipMemcpyHostToDevice, h->stream));
  KArgs a = kargs(h);
  if (acc_des) {
    HIPCHK(hipMemcpyAsync(h->acc, acc_des, sizeof(double) * B * 6, hipMemcpyHostToDevice, h->stream));
  } else {
    hipLaunchKernelGGL(k_desired, dim3((B + 63) / 64), dim3(64), 0, h->stream, a, h->acc);
    HIPCHK(hipGetLastError());
  }
  if (launch_hl(h)) return -1;
  if (f_des) HIPCHK(hipMemcpyAsync(f_des, h->fdes, sizeof(double) * B * 3 * n, hipMemcpyDeviceToHost, h->stream));
  if (iters) HIPCHK(hipMemcpyAsync(iters, h->iters, sizeof(int) * B, hipMemcpyDeviceToHost, h->stream));
  if (qp_status) HIPCHK(hipMemcpyAsync(qp_status, h->qstatus, sizeof(int) * B * n, hipMemcpyDeviceToHost, h->stream));
  if (min_env_dist) HIPCHK(hipMemcpyAsync(min_env_dist, h->mind, sizeof(double) * B, hipMemcpyDeviceToHost, h->stream));
  if (collision) HIPCHK(hipMemcpyAsync(collision, h->col, B, hipMemcpyDeviceToHost, h->stream));
  if (err_seq) {
    if (!h->err) return fail("dat_control_step: err_seq requested but record_err = 0");
    HIPCHK(hipMemcpyAsync(err_seq, h->err, sizeof(double) * B * (h->cfg.max_iter + 1), hipMemcpyDeviceToHost, h->stream));
  }
  if (finish_hl(h)) return -1;
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int dat_control_steps(dat_handle* h, int steps, const double* acc_seq, double* f_des, int* iters, int* qp_status) {
  if (!h || !acc_seq) return fail("dat_control_steps: null argument");
  if (steps <= 0) return fail("dat_control_steps: steps must be >= 1");
  if (h->cfg.mode != DAT_MODE_CADMM && h->cfg.mode != DAT_MODE_DD)
    return fail("dat_control_steps: C-ADMM and DD handles only");
  if (h->nforest > 0) return fail("dat_control_steps: handles without a forest only (env rows change with the state)");
  if (h->cfg.record_err) return fail("dat_control_steps: record_err must be 0");
  HIPCHK(hipSetDevice(h->cfg.device));
  const size_t B = h->cfg.batch, n = h->cfg.n, need = (size_t)steps * B * 6;
  if (need > h->acc_seq_cap) {
    if (h->acc_seq) HIPCHK(hipFree(h->acc_seq));
    h->acc_seq = nullptr;
    h->acc_seq_cap = 0;
    HIPCHK(hipMalloc(&h->acc_seq, sizeof(double) * need));
    h->acc_seq_cap = need;
  }
  HIPCHK(hipMemcpyAsync(h->acc_seq, acc_seq, sizeof(double) * need, hipMemcpyHostToDevice, h->stream));
  if (launch_hl(h, steps, h->acc_seq)) return -1;
  if (f_des) HIPCHK(hipMemcpyAsync(f_des, h->fdes, sizeof(double) * B * 3 * n, hipMemcpyDeviceToHost, h->stream));
  if (iters) HIPCHK(hipMemcpyAsync(iters, h->iters, sizeof(int) * B, hipMemcpyDeviceToHost, h->stream));
  if (qp_status) HIPCHK(hipMemcpyAsync(qp_status, h->qstatus, sizeof(int) * B * n, hipMemcpyDeviceToHost, h->stream));
  if (finish_hl(h, steps)) return -1;
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int dat_rollout(dat_handle* h, int steps, const double* f_des) {
  if (!h) return fail("null handle");
  if (steps <= 0) return 0;
  HIPCHK(hipSetDevice(h->cfg.device));
  const size_t B = h->cfg.batch, n = h->cfg.n;
  if (f_des) HIPCHK(hipMemcpyAsync(h->fdes, f_des, sizeof(double) * B * 3 * n, hipMemcpyHostToDevice, h->stream));
  if (!h->have_params) return fail("dat_rollout: params not set");
  KArgs a = kargs(h);
  launch_rollout(a, (int)B, h->stream, steps, h->cfg.dt, (const double*)h->fdes);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

// the closed loop on sub-batches: hl_steps x (desired acceleration, env classes, class sort, C-ADMM drain,
// rollout) per sub-batch on its own stream, no synchronisation between the sub-batches or the steps
int closed_loop_sub(dat_handle* h, int hl_steps) {
  if (!h->have_params) return fail("dat_set_params has not been called");
  const int B = h->cfg.batch, n = h->cfg.n, S = h->nsub;
  auto now_ms = [] {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  h->marks.clear();
  h->marks.push_back(now_ms());
  // k_cadmm launch spans: a start / end event pair per sub-batch and step, on the sub-batch's stream
  while (h->sub_ev.size() < 2 * (size_t)S * hl_steps) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    h->sub_ev.push_back(e);
  }
  HIPCHK(hipEventRecord(h->ev_start, h->stream));
  for (int s = 1; s < S; ++s) HIPCHK(hipStreamWaitEvent(h->sub_stream[s], h->ev_start, 0));
  for (int k = 0; k < hl_steps; ++k) {
    for (int s = 0; s < S; ++s) {
      const int off = (int)((long long)B * s / S), Bs = (int)((long long)B * (s + 1) / S) - off;
      hipStream_t st = h->sub_stream[s];
      KArgs a = sub_kargs(h, off, Bs, s);
      hipLaunchKernelGGL(k_desired, dim3((Bs + 63) / 64), dim3(64), 0, st, a, (double*)a.acc);
      const int G = 64 / n;
      hipLaunchKernelGGL(k_env_class, dim3((Bs + G - 1) / G), dim3(64), 0, st, a);
      hipLaunchKernelGGL(k_bucket, dim3(1), dim3(BUCKET_T), 0, st, Bs, (const int*)a.need, a.slist, a.scount);
      const hipEvent_t* ev = h->sub_ev.data() + 2 * ((size_t)k * S + s);
      HIPCHK(hipEventRecord(ev[0], st));
      if (launch_cadmm(h, a, std::min((Bs + a.G - 1) / a.G, h->persistent_blocks), st)) return -1;
      HIPCHK(hipEventRecord(ev[1], st));
      launch_rollout(a, Bs, st, h->cfg.hl_every, h->cfg.dt, (const double*)a.fdes);
      HIPCHK(hipGetLastError());
    }
  }
  for (int s = 1; s < S; ++s) {
    HIPCHK(hipEventRecord(h->sub_done[s], h->sub_stream[s]));
    HIPCHK(hipStreamWaitEvent(h->stream, h->sub_done[s], 0));
  }
  HIPCHK(hipEventRecord(h->ev_end, h->stream));
  HIPCHK(hipEventSynchronize(h->ev_end));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, h->ev_start, h->ev_end));
  // hl_ms: the whole run's device time (the sub-batches' kernels overlap); cadmm_ms: the sum of the
  // k_cadmm launch spans (S launches per HL step: dat_get_kernel_ms / (hl_steps S) is one launch)
  h->hl_ms += ms;
  for (size_t j = 0; j < (size_t)S * hl_steps; ++j) {
    float mk = 0.f;
    HIPCHK(hipEventElapsedTime(&mk, h->sub_ev[2 * j], h->sub_ev[2 * j + 1]));
    h->cadmm_ms += mk;
  }
  h->hl_steps += hl_steps;
  h->marks.push_back(now_ms());
  return 0;
}

int dat_closed_loop(dat_handle* h, int hl_steps) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (h->nsub > 1) {
    if (closed_loop_sub(h, hl_steps)) return -1;
    HIPCHK(hipStreamSynchronize(h->stream));
    return 0;
  }
  const size_t B = h->cfg.batch;
  KArgs a = kargs(h);
  auto now_ms = [] {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  h->marks.clear();
  h->marks.push_back(now_ms());
  for (int s = 0; s < hl_steps; ++s) {
    hipLaunchKernelGGL(k_desired, dim3((B + 63) / 64), dim3(64), 0, h->stream, a, h->acc);
    if (launch_hl(h)) return -1;
    launch_rollout(a, (int)B, h->stream, h->cfg.hl_every, h->cfg.dt, (const double*)h->fdes);
    HIPCHK(hipGetLastError());
    // waits for this step's control kernel; the rollout still runs while the next step is enqueued
    if (finish_hl(h)) return -1;
    h->marks.push_back(now_ms());
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int dat_get_refinement_counters(dat_handle* h, long long* passes, long long* corrections) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  unsigned long long c[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(c, h->counters + CNT_REF, sizeof(c), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (passes) *passes = (long long)c[0];
  if (corrections) *corrections = (long long)c[1];
  return 0;
}

int dat_get_step_marks(dat_handle* h, double* marks_ms, int max_marks) {
  if (!h) return fail("null handle");
  const int m = (int)h->marks.size();
  if (marks_ms)
    for (int k = 0; k < m && k < max_marks; ++k) marks_ms[k] = h->marks[k] - h->marks[0];
  return m;
}

int dat_get_counters(dat_handle* h, long long* qp_solves, long long* ipm_iters, long long* ipm_row_iters,
                     long long* hl_steps, double* hl_kernel_ms) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  unsigned long long cc[DAT_NCOUNTERS] = {};
  HIPCHK(hipMemcpyAsync(cc, h->counters, sizeof(cc), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  unsigned long long c[3] = {cc[0], cc[1], cc[2]};
  if (h->cfg.mode == DAT_MODE_CADMM)
    for (int k = 1; k < NCLS; ++k)
      for (int j = 0; j < 3; ++j) c[j] += cc[CNT_STRIDE * k + j];
  if (qp_solves) *qp_solves = (long long)c[0];
  if (ipm_iters) *ipm_iters = (long long)c[1];
  if (ipm_row_iters) *ipm_row_iters = (long long)c[2];
  if (hl_steps) *hl_steps = h->hl_steps;
  if (hl_kernel_ms) *hl_kernel_ms = h->hl_ms;
  return 0;
}

int dat_get_class_counters(dat_handle* h, int env_class, long long* qp_solves, long long* ipm_iters,
                           long long* ipm_row_iters, double* kernel_ms) {
  if (!h) return fail("null handle");
  if (h->cfg.mode != DAT_MODE_CADMM) return fail("dat_get_class_counters: C-ADMM handles only");
  if (env_class < 0 || env_class >= NCLS) return fail("dat_get_class_counters: env_class must be in [0, 4)");
  HIPCHK(hipSetDevice(h->cfg.device));
  unsigned long long c[3] = {0, 0, 0};
  HIPCHK(hipMemcpyAsync(c, h->counters + CNT_STRIDE * env_class, sizeof(c), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (qp_solves) *qp_solves = (long long)c[0];
  if (ipm_iters) *ipm_iters = (long long)c[1];
  if (ipm_row_iters) *ipm_row_iters = (long long)c[2];
  if (kernel_ms) *kernel_ms = h->cadmm_ms;
  return 0;
}

int dat_get_class_occupancy(dat_handle* h, int env_class, long long* slot_ipm_iters, long long* wave_admm_iters) {
  if (!h) return fail("null handle");
  if (h->cfg.mode != DAT_MODE_CADMM) return fail("dat_get_class_occupancy: C-ADMM handles only");
  if (env_class < 0 || env_class >= NCLS) return fail("dat_get_class_occupancy: env_class must be in [0, 4)");
  HIPCHK(hipSetDevice(h->cfg.device));
  unsigned long long c[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(c, h->counters + CNT_STRIDE * env_class + 3, sizeof(c), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (slot_ipm_iters) *slot_ipm_iters = (long long)c[0];
  if (wave_admm_iters) *wave_admm_iters = (long long)c[1];
  return 0;
}

int dat_reset_counters(dat_handle* h) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  HIPCHK(hipMemsetAsync(h->counters, 0, DAT_NCOUNTERS * sizeof(unsigned long long), h->stream));
  {  // the running minimum of the env distance starts at +inf
    static const unsigned long long inf = dist_key(HUGE_VAL);
    HIPCHK(hipMemcpyAsync(h->counters + CNT_COLL + 1, &inf, sizeof(inf), hipMemcpyHostToDevice, h->stream));
  }
  h->cadmm_ms = 0.0;
  HIPCHK(hipStreamSynchronize(h->stream));
  h->hl_steps = 0;
  h->hl_ms = 0.0;
  return 0;
}

int dat_set_sub_batches(dat_handle* h, int count) {
  if (!h) return fail("null handle");
  if (count < 1 || count > DAT_MAX_SUB) return fail("dat_set_sub_batches: count must be in [1, 4]");
  if (count > 1 && h->cfg.mode != DAT_MODE_CADMM) return fail("dat_set_sub_batches: C-ADMM handles only");
  if (count > h->cfg.batch) return fail("dat_set_sub_batches: more sub-batches than scenarios");
  if (count > 1 && h->cfg.record_err) return fail("dat_set_sub_batches: record_err must be 0");
  HIPCHK(hipSetDevice(h->cfg.device));
  h->sub_stream[0] = h->stream;
  for (int s = 1; s < count; ++s) {
    if (!h->sub_stream[s]) HIPCHK(hipStreamCreateWithFlags(&h->sub_stream[s], hipStreamNonBlocking));
    if (!h->sub_done[s]) HIPCHK(hipEventCreateWithFlags(&h->sub_done[s], hipEventDisableTiming));
  }
  if (!h->ev_start) HIPCHK(hipEventCreate(&h->ev_start));
  if (!h->ev_end) HIPCHK(hipEventCreate(&h->ev_end));
  h->nsub = count;
  return 0;
}

int dat_set_persistent_blocks(dat_handle* h, int blocks) {
  if (!h) return fail("null handle");
  if (blocks < 0) return fail("dat_set_persistent_blocks: negative");
  if (blocks == 0) {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, h->cfg.device) != hipSuccess || ncu <= 0)
      ncu = 256;
    blocks = 4 * ncu;
  }
  h->persistent_blocks = blocks;
  return 0;
}

int dat_synchronize(dat_handle* h) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int dat_env_rows(dat_handle* h, double* lhs, double* rhs, int* nrow, unsigned char* collision, double* min_dist) {
  if (!h || !lhs || !rhs || !nrow || !collision || !min_dist) return fail("dat_env_rows: null argument");
  if (!h->have_params) return fail("dat_env_rows: params not set");
  HIPCHK(hipSetDevice(h->cfg.device));
  const size_t B = h->cfg.batch, n = h->cfg.n, T = B * n;
  double *dl, *dr, *dm;
  int* dn;
  unsigned char* dc;
  HIPCHK(hipMalloc(&dl, sizeof(double) * T * DAT_NENV * 3));
  HIPCHK(hipMalloc(&dr, sizeof(double) * T * DAT_NENV));
  HIPCHK(hipMalloc(&dm, sizeof(double) * T));
  HIPCHK(hipMalloc(&dn, sizeof(int) * T));
  HIPCHK(hipMalloc(&dc, T));
  KArgs a = kargs(h);
  hipLaunchKernelGGL(k_env, dim3((T + 63) / 64), dim3(64), 0, h->stream, a, dl, dr, dn, dc, dm);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(lhs, dl, sizeof(double) * T * DAT_NENV * 3, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(rhs, dr, sizeof(double) * T * DAT_NENV, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(nrow, dn, sizeof(int) * T, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(collision, dc, T, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(min_dist, dm, sizeof(double) * T, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(dl);
  (void)hipFree(dr);
  (void)hipFree(dm);
  (void)hipFree(dn);
  (void)hipFree(dc);
  if (e != hipSuccess) return fail(std::string("dat_env_rows: ") + hipGetErrorString(e));
  return 0;
}

int dat_solve_agent_qp_batch(dat_handle* h, int count, const int* scenario, const int* agent, const double* acc_des,
                             const double* lam, const double* rho, const double* f_mean, const double* c9, double* x,
                             int* status, int* ipm_iters, unsigned char* collision, double* min_env_dist) {
  if (!h) return fail("null handle");
  if (count < 0) return fail("dat_solve_agent_qp_batch: negative count");
  if (count == 0) return 0;
  if (!h->have_params) return fail("dat_solve_agent_qp_batch: params not set");
  const int mode = h->cfg.mode, n = h->cfg.n, N3 = 3 * n;
  if (mode == DAT_MODE_CENTRALIZED) return fail("dat_solve_agent_qp_batch: C-ADMM or DD handles only");
  const bool dd = mode == DAT_MODE_DD;
  if (!scenario || !agent || !acc_des || !x || !status) return fail("dat_solve_agent_qp_batch: null argument");
  if (dd ? !c9 : (!lam || !rho || !f_mean)) return fail("dat_solve_agent_qp_batch: missing multipliers");
  for (int k = 0; k < count; ++k) {
    if (scenario[k] < 0 || scenario[k] >= h->cfg.batch) return fail("dat_solve_agent_qp_batch: scenario out of range");
    if (agent[k] < 0 || agent[k] >= n) return fail("dat_solve_agent_qp_batch: agent out of range");
    if (!dd && !(rho[k] > 0.0))
      return fail("dat_solve_agent_qp_batch: rho must be > 0 (at rho = 0 the copies f_j, j != i, are not unique)");
  }
  HIPCHK(hipSetDevice(h->cfg.device));
  const size_t C = count, nx = dd ? 9 : N3;
  std::vector<void*> tmp;
  auto dev = [&](size_t bytes, const void* src) -> void* {
    void* p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 8) != hipSuccess) return nullptr;
    tmp.push_back(p);
    if (src && hipMemcpyAsync(p, src, bytes, hipMemcpyHostToDevice, h->stream) != hipSuccess) return nullptr;
    return p;
  };
  AgentQPArgs q;
  memset(&q, 0, sizeof(q));
  q.count = count;
  q.scen = (const int*)dev(sizeof(int) * C, scenario);
  q.agent = (const int*)dev(sizeof(int) * C, agent);
  q.acc = (const double*)dev(sizeof(double) * C * 6, acc_des);
  if (dd) {
    q.c9 = (const double*)dev(sizeof(double) * C * 9, c9);
  } else {
    q.lam = (const double*)dev(sizeof(double) * C * N3, lam);
    q.rho = (const double*)dev(sizeof(double) * C, rho);
    q.fbar = (const double*)dev(sizeof(double) * C * N3, f_mean);
  }
  q.x = (double*)dev(sizeof(double) * C * nx, nullptr);
  q.status = (int*)dev(sizeof(int) * C, nullptr);
  q.iters = (int*)dev(sizeof(int) * C, nullptr);
  q.col = (unsigned char*)dev(C, nullptr);
  q.mind = (double*)dev(sizeof(double) * C, nullptr);
  q.best = (double*)dev(sizeof(double) * C * best_size(1), nullptr);
  bool ok = q.scen && q.agent && q.acc && q.x && q.status && q.iters && q.col && q.mind && q.best &&
            (dd ? q.c9 != nullptr : (q.lam && q.rho && q.fbar));
  hipError_t e = hipSuccess;
  if (ok) {
    KArgs a = kargs(h);
    e = hipEventRecord(h->e0, h->stream);
    hipLaunchKernelGGL(k_agent_qp, dim3((count + 63) / 64), dim3(64), 0, h->stream, a, q);
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipEventRecord(h->e1, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(x, q.x, sizeof(double) * C * nx, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(status, q.status, sizeof(int) * C, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && ipm_iters) e = hipMemcpyAsync(ipm_iters, q.iters, sizeof(int) * C, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && collision) e = hipMemcpyAsync(collision, q.col, C, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && min_env_dist)
      e = hipMemcpyAsync(min_env_dist, q.mind, sizeof(double) * C, hipMemcpyDeviceToHost, h->stream);
  }
  hipError_t es = hipStreamSynchronize(h->stream);
  if (ok && e == hipSuccess && es == hipSuccess) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, h->e0, h->e1) == hipSuccess) h->agent_qp_ms = ms;
  }
  for (void* p : tmp) (void)hipFree(p);
  if (!ok) return fail("dat_solve_agent_qp_batch: device allocation failed");
  if (e != hipSuccess) return fail(std::string("dat_solve_agent_qp_batch: ") + hipGetErrorString(e));
  if (es != hipSuccess) return fail(std::string("dat_solve_agent_qp_batch: ") + hipGetErrorString(es));
  return 0;
}

int dat_set_low_level(dat_handle* h, int kind) {
  if (!h) return fail("null handle");
  if (kind != DAT_LL_PD && kind != DAT_LL_SM) return fail("dat_set_low_level: kind must be DAT_LL_PD or DAT_LL_SM");
  h->ll_kind = kind;
  return 0;
}

int dat_low_level_control(dat_handle* h, const double* f_des, double* thrust, double* moment) {
  if (!h || !thrust || !moment) return fail("dat_low_level_control: null argument");
  if (!h->have_params) return fail("dat_low_level_control: params not set");
  HIPCHK(hipSetDevice(h->cfg.device));
  const size_t B = h->cfg.batch, n = h->cfg.n;
  if (f_des) HIPCHK(hipMemcpyAsync(h->fdes, f_des, sizeof(double) * B * 3 * n, hipMemcpyHostToDevice, h->stream));
  double *df = nullptr, *dm = nullptr;
  HIPCHK(hipMalloc(&df, sizeof(double) * B * n));
  if (hipMalloc(&dm, sizeof(double) * B * n * 3) != hipSuccess) {
    (void)hipFree(df);
    return fail("dat_low_level_control: hipMalloc failed");
  }
  KArgs a = kargs(h);
  hipLaunchKernelGGL(k_low_level, dim3((B * n + 63) / 64), dim3(64), 0, h->stream, a, (const double*)h->fdes, df, dm);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(thrust, df, sizeof(double) * B * n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(moment, dm, sizeof(double) * B * n * 3, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(df);
  (void)hipFree(dm);
  if (e != hipSuccess) return fail(std::string("dat_low_level_control: ") + hipGetErrorString(e));
  return 0;
}

int dat_get_kernel_ms(dat_handle* h, double* ms) {
  if (!h || !ms) return fail("dat_get_kernel_ms: null argument");
  *ms = h->cadmm_ms;
  return 0;
}

int dat_get_agent_qp_ms(dat_handle* h, double* ms) {
  if (!h || !ms) return fail("dat_get_agent_qp_ms: null argument");
  *ms = h->agent_qp_ms;
  return 0;
}

int dat_get_robust_redos(dat_handle* h, long long* redos) {
  if (!h) return fail("dat_get_robust_redos: null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  unsigned long long c = 0;
  HIPCHK(hipMemcpyAsync(&c, h->counters + CNT_ROB, sizeof(c), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (redos) *redos = (long long)c;
  return 0;
}

int dat_get_tail_counters(dat_handle* h, long long* out) {
  if (!h || !out) return fail("dat_get_tail_counters: null argument");
  HIPCHK(hipSetDevice(h->cfg.device));
  unsigned long long c[6] = {};
  HIPCHK(hipMemcpyAsync(c, h->counters + CNT_TAIL, sizeof(c), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  for (int k = 0; k < 6; ++k) out[k] = (long long)c[k];
  return 0;
}

int dat_get_collision_stats(dat_handle* h, long long* collisions, double* min_env_dist) {
  if (!h) return fail("dat_get_collision_stats: null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  unsigned long long c[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(c, h->counters + CNT_COLL, sizeof(c), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (collisions) *collisions = (long long)c[0];
  if (min_env_dist) *min_env_dist = dist_of_key(c[1]);
  return 0;
}

int dat_get_inband_exits(dat_handle* h, long long* inband, long long* beyond_clarabel_tol) {
  if (!h) return fail("dat_get_inband_exits: null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  unsigned long long c[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(c, h->counters + CNT_INBAND, sizeof(c), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (inband) *inband = (long long)c[0];
  if (beyond_clarabel_tol) *beyond_clarabel_tol = (long long)c[1];
  return 0;
}

int dat_rp_rollout(dat_handle* h, int steps, const double* f) {
  if (!h) return fail("null handle");
  if (steps <= 0) return 0;
  if (!h->have_params) return fail("dat_rp_rollout: params not set");
  HIPCHK(hipSetDevice(h->cfg.device));
  const size_t B = h->cfg.batch, n = h->cfg.n;
  if (f) HIPCHK(hipMemcpyAsync(h->fdes, f, sizeof(double) * B * 3 * n, hipMemcpyHostToDevice, h->stream));
  KArgs a = kargs(h);
  hipLaunchKernelGGL(k_rp_rollout, dim3((B + 63) / 64), dim3(64), 0, h->stream, a, steps, h->cfg.dt,
                     (const double*)h->fdes);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

}  // extern "C"
