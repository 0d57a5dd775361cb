// dat_cent.hip -- the centralized QP kernel (control/rqp_centralized.py:27-455), one lane per scenario,
// instantiated for every team size 3 <= n <= NMAX_CENT.  Its own translation unit: the per-n
// instantiations of the n-block IPM are compiled in parallel with dat.hip (distributed_aerial_
// transportation_amd/_lib.py) and linked into libdat.so.
#include <hip/hip_runtime.h>

#include "dat_kargs.hpp"

using namespace dat;

namespace {

// ------------------------------------------------------------------------------------------------
// centralized: one lane per scenario
// ------------------------------------------------------------------------------------------------
template <int NB>
__global__ __launch_bounds__(64) void k_cent(KArgs a) {
  const int sc = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = sc < a.B;
  const int n = NB;
  unsigned long long q = 0, ip = 0, rw = 0, ib = 0, lo = 0;
  const double* prm = valid ? prm_of(a, sc) : a.params;
  QPShared S;
  QPLane<NB> P;
  double Rt[NB][9];
  EnvRows E;
  EnvOut env;
  env.collision = 0;
  env.min_env_dist = 0.0;
  int nr = NBASE;
  if (valid) {
    const double* st = a.state + (size_t)sc * a.S;
    build_shared(S, prm, n, st, a.acc + (size_t)sc * 6, prm[DAT_P_KFC], prm[DAT_P_KMC], 2, false);
    lane_cent<NB>(P, prm, n, st, Rt);
    const double* trees;
    int nt;
    unsigned emask;
    forest_of(a, sc, &trees, &nt);
    double lhs[DAT_NENV][3], rhs[DAT_NENV];
    env = env_rows(prm, n, st, trees, nt, -1, prm[DAT_P_AENVC], &emask, lhs, rhs);
    set_env_rows(P, E, S, emask, lhs, rhs);
    nr = rows_needed(P.emask);
  }
  nr = wave_max(nr);
  if (valid) {
    double y[NB][3], w[6];
    IPMOut o = ipm_solve_rows<MODE_CENT, NB>(nr, PlainRef<QPShared>{&S}, EnvPlain{&E}, RtPtr{&Rt[0][0]}, P,
                                             prm + DAT_P_FEQ(n), y, w, a.best + (size_t)sc * best_size(NB),
                                             IPM_MAX_ITER, a.qp_tol);
    q = 1;
    ip = o.iters;
    ib = o.inband;
    lo = inband_loose(o);
    rw = (unsigned long long)o.iters * (__builtin_popcount(S.bmask) + __builtin_popcount(P.emask));
    double* pf = a.pf + (size_t)sc * 3 * n;
    if (o.status == ST_OPTIMAL)  // hold the previous solution otherwise (rqp_centralized.py:441-444)
      for (int k = 0; k < NB; ++k)
        for (int c = 0; c < 3; ++c) pf[3 * k + c] = y[k][c];
    for (int c = 0; c < 3 * n; ++c) a.fdes[(size_t)sc * 3 * n + c] = pf[c];
    for (int k = 0; k < n; ++k) a.qstatus[(size_t)sc * n + k] = o.status;
    a.iters[sc] = -1;
    a.col[sc] = (unsigned char)env.collision;
    a.mind[sc] = env.min_env_dist;
  }
  for (int off = 32; off > 0; off >>= 1) {
    q += __shfl_xor(q, off);
    ip += __shfl_xor(ip, off);
    rw += __shfl_xor(rw, off);
    ib += __shfl_xor(ib, off);
    lo += __shfl_xor(lo, off);
  }
  if (threadIdx.x == 0) {
    atomicAdd(a.counters, q);
    atomicAdd(a.counters + 1, ip);
    atomicAdd(a.counters + 2, rw);
    if (ib) atomicAdd(a.counters + CNT_INBAND, ib);
    if (lo) atomicAdd(a.counters + CNT_INBAND + 1, lo);
  }
}

}  // namespace

namespace dat {

hipError_t launch_cent(int n, int blocks, hipStream_t stream, const KArgs& a) {
  switch (n) {
#define DAT_CENT_CASE(NB) \
  case NB: hipLaunchKernelGGL(k_cent<NB>, dim3(blocks), dim3(64), 0, stream, a); break;
    DAT_CENT_CASE(3) DAT_CENT_CASE(4) DAT_CENT_CASE(5) DAT_CENT_CASE(6)
#undef DAT_CENT_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace dat
