// dat_cpu.hip -- the CPU baseline of bench.py: the C4 closed loop on the host's cores.
//
// SURVEY.md 8(d) "CPU baseline plan": the reference's cvxpy + Clarabel path cannot run here or on
// the GPU box, so the reported CPU baseline is a C++ fp64 restatement of the same controller loop,
// one scenario per OpenMP thread, compiled -O3 for x86-64-v3 (AVX2 / FMA; built in the dev
// container, run on the GPU box's host).  Per scenario and high-level step it runs what the GPU
// runs:
//   desired acceleration (example/rqp_example.py:33-59)                       desired_accel_forest
//   RQPCADMMController.control (control/rqp_cadmm.py:631-675): per agent the env CBF rows
//     (:307-373, env_rows), RQPPrimalSolver.solve (:482-501, ipm_solve), consensus mean and the
//     matrix inf-norm residual (:582-600), dual update (:627-629); warm f, f_mean, lambda persist
//   hl_every simulation steps: LL SO(3) PD + dynamics + integration (sim_step)
// using the same per-lane __host__ __device__ functions as the kernels (dat_core.hpp / dat_qp.hpp),
// so the CPU and GPU do identical arithmetic per scenario.  This is a measured baseline, not the
// product: the package never loads it.
#include <omp.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../distributed_aerial_transportation_amd/csrc/dat_qp.hpp"

using namespace dat;

#if defined(DAT_IPM_STATS)
long long g_ith[2][8][32];  // tools/ipm_stats.py: IPM iterations by start and active env rows
#endif

namespace {
constexpr int NMAXC = 16;

struct Ctx {
  int n, B, P, S;
  std::vector<double> params, state, cf, cfbar, clam, fdes, trees, mountain;
  std::vector<int> counter, tree_off, scen_forest, iters;
  int nforest = 0;
  long long qp = 0, ipm = 0;
};

// One C-ADMM control step of scenario sc (control/rqp_cadmm.py:631-675).
void cadmm_step(Ctx& c, int sc, long long* qp, long long* ipm) {
  const int n = c.n, N3 = 3 * n;
  const double* prm = c.params.data();
  double* st = c.state.data() + (size_t)sc * c.S;
  const double* trees = nullptr;
  int nt = 0;
  const double* mnt = nullptr;
  const double m0[DAT_MOUNTAIN_SIZE] = {30.0, 0.0, 25.0, 1e300, 0.0};
  if (c.nforest > 0) {
    const int f = c.scen_forest.empty() ? 0 : c.scen_forest[sc];
    trees = c.trees.data() + 3 * (size_t)c.tree_off[f];
    nt = c.tree_off[f + 1] - c.tree_off[f];
    mnt = c.mountain.data() + (size_t)f * DAT_MOUNTAIN_SIZE;
  }
  double acc[6];
  desired_accel_forest(st, n, mnt ? mnt : m0, 1.5, acc);
  QPShared S;
  build_shared(S, prm, n, st, acc, prm[DAT_P_KFD], prm[DAT_P_KMD], 3, true);
  double Rt_all[NMAXC * 9];
  for (int j = 0; j < n; ++j) make_Rt(prm + DAT_P_RCOM(n) + 3 * j, st + DAT_S_RL(n), Rt_all + 9 * j);
  QPLane<1> P[NMAXC];
  EnvRows E[NMAXC];
  for (int i = 0; i < n; ++i) {
    lane_cadmm_static(P[i], prm, i);
    unsigned emask = 0;
    double lhs[DAT_NENV][3], rhs[DAT_NENV];
    env_rows(prm, n, st, trees, nt, i, prm[DAT_P_AENVD], &emask, lhs, rhs);
    set_env_rows(P[i], E[i], S, emask, lhs, rhs);
    // rows certified infeasible are held (the GPU's tail certifies them once per scenario-step)
    if (dvl_rows_infeasible(PlainRef<QPShared>{&S}, EnvPlain{&E[i]}, P[i].emask)) P[i].infeasible = 1;
  }
  double* cf = c.cf.data() + (size_t)sc * n * N3;
  double* fb = c.cfbar.data() + (size_t)sc * N3;
  double* lam = c.clam.data() + (size_t)sc * n * N3;
  const double* feq = prm + DAT_P_FEQ(n);
  const double tol = 1e-2, rho0 = 1.0, tau = 1.0, rho_max = 2.0;
  const int max_iter = 100;
  double rho = rho0;
  int it = 0;
  const int prev_it = c.iters[sc];  // the previous step's ADMM iterations
  // the GPU's tail rule (dat_kargs.hpp, with a forest): the warm start and stall exit of pass it >= 1 when the
  // previous step took more than TAIL_PREV passes or it >= TAIL_PASS; the passes the tail kernel runs keep the
  // agent QPs' warm-start records (from the step's start when routed, from the first unclean pass or TAIL_PASS)
  const int tprev = c.nforest > 0 ? TAIL_PREV : 1 << 30, tpass = c.nforest > 0 ? TAIL_PASS : 1 << 30;
  double wrec[NMAXC][WREC_SIZE];
  for (int i = 0; i < n; ++i) wrec[i][0] = 0.0;
  bool in_tail = prev_it > tprev;
  for (;;) {
    in_tail = in_tail || it >= tpass;
    const bool wson = it >= 1 && (prev_it > tprev || it >= tpass);
    bool unclean = false;
    for (int i = 0; i < n; ++i) {
      lane_cadmm_dynamic(P[i], prm, n, i, Rt_all, lam + i * N3, fb, rho);
      P[i].tuned = it == 0 || prev_it <= 3;  // as k_cadmm (tuned IPM start: first pass / warm regime)
      double y[1][3], w[6], best[best_size(1)];
      IPMOut o = ipm_solve_rows<MODE_CADMM, 1, IPM_FAST_REDO, true>(
          rows_needed(P[i].emask), PlainRef<QPShared>{&S}, EnvPlain{&E[i]}, RtPtr{Rt_all + 9 * i}, P[i], feq + 3 * i, y,
          w, best, 50, 1e-10, in_tail ? wrec[i] : nullptr, wson);
      unclean = unclean || o.stiff;
      ++*qp;
      *ipm += o.iters;
#if defined(DAT_IPM_STATS)
      ++g_ith[P[i].tuned ? 1 : 0][__builtin_popcount(P[i].emask) & 7][o.iters < 31 ? o.iters : 31];
#endif
      double* fi = cf + i * N3;
      if (o.status == ST_OPTIMAL) {
        for (int j = 0; j < n; ++j) {
          if (j == i) {
            for (int k = 0; k < 3; ++k) fi[3 * j + k] = y[0][k];
          } else {
            cadmm_free_block(Rt_all + 9 * j, lam + i * N3 + 3 * j, fb + 3 * j, o.pi, rho, fi + 3 * j);
          }
        }
      } else if (o.status == ST_FAILED) {
        for (int k = 0; k < N3; ++k) fi[k] = feq[k];
      }
    }
    in_tail = in_tail || (unclean && c.nforest > 0);
    ++it;
    rho = std::min(rho * tau, rho_max);
    for (int k = 0; k < N3; ++k) {
      double s = 0.0;
      for (int i = 0; i < n; ++i) s += cf[i * N3 + k];
      fb[k] = s / n;
    }
    double res = 0.0;
    for (int i = 0; i < n; ++i)
      for (int r = 0; r < 3; ++r) {
        double s = 0.0;
        for (int j = 0; j < n; ++j) s += std::fabs(cf[i * N3 + 3 * j + r] - fb[3 * j + r]);
        res = std::max(res, s);
      }
    if (res < tol || it > max_iter) break;
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < N3; ++k) lam[i * N3 + k] += rho * (cf[i * N3 + k] - fb[k]);
  }
  double* fd = c.fdes.data() + (size_t)sc * N3;
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) fd[3 * i + k] = cf[i * N3 + 3 * i + k];
  c.iters[sc] = it;
}
}  // namespace

extern "C" {

#if defined(DAT_IPM_STATS) && !defined(__HIP_DEVICE_COMPILE__)
void datcpu_ipm_ith(long long* out) {  // [tuned start][active env rows][IPM iterations] solves
  long long* g = &g_ith[0][0][0];
  for (int k = 0; k < 512; ++k) { out[k] = g[k]; g[k] = 0; }
}
void datcpu_ipm_stats(long long* out) {
  for (int k = 0; k < 16; ++k) { out[k] = dat::g_ipm_stats[k]; dat::g_ipm_stats[k] = 0; }
  for (int k = 0; k < 72; ++k) { out[16 + k] = dat::g_ipm_hist[k / 24][k % 24]; dat::g_ipm_hist[k / 24][k % 24] = 0; }
}
#endif

void* datcpu_create(int n, int B, const double* params) {
  if (n < 3 || n > NMAXC || B < 1 || !params) return nullptr;
  Ctx* c = new Ctx();
  c->n = n;
  c->B = B;
  c->P = DAT_PARAM_SIZE(n);
  c->S = DAT_STATE_SIZE(n);
  c->params.assign(params, params + c->P);
  const size_t N3 = 3 * (size_t)n;
  c->state.assign((size_t)B * c->S, 0.0);
  c->counter.assign(B, 0);
  c->iters.assign(B, 0);
  c->fdes.assign((size_t)B * N3, 0.0);
  c->cf.assign((size_t)B * n * N3, 0.0);
  c->cfbar.assign((size_t)B * N3, 0.0);
  c->clam.assign((size_t)B * n * N3, 0.0);
  const double* feq = params + DAT_P_FEQ(n);
  for (int b = 0; b < B; ++b) {  // warm start f = f_mean = f_eq, lambda = 0 (control/rqp_cadmm.py:577-580)
    for (int i = 0; i < n; ++i) std::memcpy(&c->cf[((size_t)b * n + i) * N3], feq, sizeof(double) * N3);
    std::memcpy(&c->cfbar[(size_t)b * N3], feq, sizeof(double) * N3);
    std::memcpy(&c->fdes[(size_t)b * N3], feq, sizeof(double) * N3);
  }
  return c;
}

void datcpu_destroy(void* h) { delete (Ctx*)h; }

// trees of each forest must be sorted by x (as dat_set_forests stores them for the GPU)
int datcpu_set_forests(void* h, int num_forests, const int* tree_offsets, const double* tree_pos,
                       const int* scenario_forest, const double* mountain) {
  Ctx* c = (Ctx*)h;
  if (!c || num_forests < 0) return -1;
  c->nforest = num_forests;
  if (num_forests == 0) return 0;
  const int T = tree_offsets[num_forests];
  c->tree_off.assign(tree_offsets, tree_offsets + num_forests + 1);
  c->trees.assign(tree_pos, tree_pos + 3 * (size_t)T);
  c->mountain.assign(mountain, mountain + (size_t)num_forests * DAT_MOUNTAIN_SIZE);
  if (scenario_forest) c->scen_forest.assign(scenario_forest, scenario_forest + c->B);
  return 0;
}

int datcpu_set_state(void* h, const double* state) {
  Ctx* c = (Ctx*)h;
  if (!c || !state) return -1;
  c->state.assign(state, state + (size_t)c->B * c->S);
  std::fill(c->counter.begin(), c->counter.end(), 0);
  return 0;
}

// the constructor's warm state (f = f_mean = f_eq, lambda = 0, control/rqp_cadmm.py:577-580) and no
// step history (the previous step's ADMM iteration count selects the IPM start, as on the GPU: k_warm)
int datcpu_reset_warm(void* h) {
  Ctx* c = (Ctx*)h;
  if (!c) return -1;
  const size_t N3 = 3 * (size_t)c->n;
  const double* feq = c->params.data() + DAT_P_FEQ(c->n);
  std::fill(c->clam.begin(), c->clam.end(), 0.0);
  std::fill(c->iters.begin(), c->iters.end(), 0);
  for (int b = 0; b < c->B; ++b) {
    for (int i = 0; i < c->n; ++i) std::memcpy(&c->cf[((size_t)b * c->n + i) * N3], feq, sizeof(double) * N3);
    std::memcpy(&c->cfbar[(size_t)b * N3], feq, sizeof(double) * N3);
    std::memcpy(&c->fdes[(size_t)b * N3], feq, sizeof(double) * N3);
  }
  return 0;
}

// hl_steps closed-loop periods of scenarios [first, first + count) on `threads` OpenMP threads (0:
// default); returns the agent-QP solves and IPM iterations of the call.
int datcpu_closed_loop(void* h, int hl_steps, int first, int count, int threads, int hl_every, double dt,
                       long long* qp_solves, long long* ipm_iters) {
  Ctx* c = (Ctx*)h;
  if (!c || first < 0 || count < 0 || first + count > c->B) return -1;
  long long qp = 0, ipm = 0;
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads) reduction(+ : qp, ipm)
  for (int sc = first; sc < first + count; ++sc) {
    for (int k = 0; k < hl_steps; ++k) {
      cadmm_step(*c, sc, &qp, &ipm);
      double* st = c->state.data() + (size_t)sc * c->S;
      const double* fd = c->fdes.data() + (size_t)sc * 3 * c->n;
      for (int s = 0; s < hl_every; ++s) sim_step<NMAXC>(c->params.data(), c->n, st, &c->counter[sc], fd, dt);
    }
  }
  if (qp_solves) *qp_solves = qp;
  if (ipm_iters) *ipm_iters = ipm;
  return 0;
}

int datcpu_get(void* h, double* state, double* f_des, int* iters) {
  Ctx* c = (Ctx*)h;
  if (!c) return -1;
  if (state) std::memcpy(state, c->state.data(), sizeof(double) * c->state.size());
  if (f_des) std::memcpy(f_des, c->fdes.data(), sizeof(double) * c->fdes.size());
  if (iters) std::memcpy(iters, c->iters.data(), sizeof(int) * c->iters.size());
  return 0;
}

int datcpu_max_threads(void) { return omp_get_max_threads(); }

}  // extern "C"
