// Register-pressure probe (development tool, not built into the library): each kernel wraps one
// piece of the per-lane device code so `hipcc -Rpass-analysis=kernel-resource-usage` reports its
// VGPR / AGPR / scratch footprint in isolation.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -c tools/regprobe.hip -o /dev/null \
//         -Rpass-analysis=kernel-resource-usage
#include <hip/hip_runtime.h>

#include "../distributed_aerial_transportation_amd/csrc/dat_qp.hpp"

using namespace dat;

template <int NR>
__global__ __launch_bounds__(64) void probe_ipm_cadmm(const double* prm, const double* lam, const double* fb,
                                                      double* out, double* best) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  QPShared* sh = (QPShared*)smem;
  double* env = (double*)(sh + 1);
  double* rt = env + ENV_LDS_DOUBLES;
  const int lane = threadIdx.x;
  QPLane<1> P;
  lane_cadmm_static(P, prm, lane % 6);
  lane_cadmm_dynamic(P, prm, 6, lane % 6, rt, lam + 18 * lane, fb, 1.0);
  P.emask = NR > NBASE ? 1u : 0u;
  double y[1][3], w[6];
  IPMOut o = ipm_solve<MODE_CADMM, 1, NR>(LdsRef<QPShared>{sh, lane / 6}, EnvLds{env, lane}, RtLds{rt, 9 * (lane % 6)}, P,
                                          prm + DAT_P_FEQ(6), y, w, best + 21 * lane, 50, 1e-10);
  double* o8 = out + 16 * lane;
  for (int c = 0; c < 3; ++c) o8[c] = y[0][c];
  for (int c = 0; c < 6; ++c) o8[3 + c] = o.pi[c];
  o8[9] = o.iters;
}
template <int NR>
__global__ __launch_bounds__(64) void probe_ipm_cadmm_lrows(const double* prm, const double* lam, const double* fb,
                                                            double* out, double* best) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  QPShared* sh = (QPShared*)smem;
  double* env = (double*)(sh + 1);
  double* rt = env + ENV_LDS_DOUBLES;
  double* rows = rt + 64;
  const int lane = threadIdx.x;
  QPLane<1> P;
  lane_cadmm_static(P, prm, lane % 6);
  lane_cadmm_dynamic(P, prm, 6, lane % 6, rt, lam + 18 * lane, fb, 1.0);
  P.emask = NR > NBASE ? 1u : 0u;
  double y[1][3], w[6];
  IPMOut o = ipm_solve<MODE_CADMM, 1, NR>(LdsRef<QPShared>{sh, lane / 6}, EnvLds{env, lane}, RtLds{rt, 9 * (lane % 6)}, P,
                                          prm + DAT_P_FEQ(6), y, w, best + 21 * lane, 50, 1e-10, RowLds{rows, lane});
  double* o8 = out + 16 * lane;
  for (int c = 0; c < 3; ++c) o8[c] = y[0][c];
  for (int c = 0; c < 6; ++c) o8[3 + c] = o.pi[c];
  o8[9] = o.iters;
}
template __global__ void probe_ipm_cadmm_lrows<NBASE>(const double*, const double*, const double*, double*, double*);
template __global__ void probe_ipm_cadmm_lrows<NBASE + 5>(const double*, const double*, const double*, double*, double*);
template __global__ void probe_ipm_cadmm_lrows<DAT_MAXROW>(const double*, const double*, const double*, double*, double*);
template __global__ void probe_ipm_cadmm<NBASE + 5>(const double*, const double*, const double*, double*, double*);
template __global__ void probe_ipm_cadmm<NBASE>(const double*, const double*, const double*, double*, double*);
template __global__ void probe_ipm_cadmm<DAT_MAXROW>(const double*, const double*, const double*, double*, double*);

__global__ __launch_bounds__(64) void probe_env(const double* prm, const double* st, const double* trees, int nt,
                                                double* out) {
  double lhs[DAT_NENV][3], rhs[DAT_NENV];
  unsigned mask;
  EnvOut e = env_rows(prm, 6, st, trees, nt, threadIdx.x % 6, 1.5, &mask, lhs, rhs);
  double* o = out + 64 * threadIdx.x;
  for (int j = 0; j < DAT_NENV; ++j) {
    o[4 * j] = lhs[j][0];
    o[4 * j + 1] = lhs[j][1];
    o[4 * j + 2] = lhs[j][2];
    o[4 * j + 3] = rhs[j];
  }
  o[40] = e.min_env_dist + mask;
}

// ipm_solve with aux slots in the LDS row store (AUXM groups of per-iteration data out of registers)
template <int NR, unsigned AUXM>
__global__ __launch_bounds__(64) void probe_ipm_cadmm_aux(const double* prm, const double* lam, const double* fb,
                                                          double* out, double* best) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  QPShared* sh = (QPShared*)smem;
  double* env = (double*)(sh + 1);
  double* rt = env + ENV_LDS_DOUBLES;
  double* rows = rt + 64;
  const int lane = threadIdx.x;
  QPLane<1> P;
  lane_cadmm_static(P, prm, lane % 6);
  lane_cadmm_dynamic(P, prm, 6, lane % 6, rt, lam + 18 * lane, fb, 1.0);
  P.emask = NR > NBASE ? 1u : 0u;
  double y[1][3], w[6];
  IPMOut o = ipm_solve<MODE_CADMM, 1, NR, LdsRef<QPShared>, EnvLds, RtLds, RowLds, AUXM>(
      LdsRef<QPShared>{sh, lane / 6}, EnvLds{env, lane}, RtLds{rt, 9 * (lane % 6)}, P, prm + DAT_P_FEQ(6), y, w,
      best + 21 * lane, 50, 1e-10, RowLds{rows, lane});
  double* o8 = out + 16 * lane;
  for (int c = 0; c < 3; ++c) o8[c] = y[0][c];
  for (int c = 0; c < 6; ++c) o8[3 + c] = o.pi[c];
  o8[9] = o.iters;
}
#ifndef PROBE_AUXM
#define PROBE_AUXM 15
#endif
template __global__ void probe_ipm_cadmm_aux<NBASE, PROBE_AUXM>(const double*, const double*, const double*, double*, double*);
template __global__ void probe_ipm_cadmm_aux<NBASE + 5, PROBE_AUXM>(const double*, const double*, const double*, double*, double*);
template __global__ void probe_ipm_cadmm_aux<DAT_MAXROW, PROBE_AUXM>(const double*, const double*, const double*, double*, double*);
