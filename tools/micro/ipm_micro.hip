// Standalone IPM microbenchmark (development tool): batches of C-ADMM agent QPs built on the host
// from perturbed rest states of the n = 6 hexagon team, solved by ipm_solve on the GPU, one lane
// per QP.  Reports ns per QP and per IPM iteration.  Build variants with -D flags.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I<csrc> ipm_micro.hip -o ipm_micro
//   ./ipm_micro <params.bin> [num_qps] [reps]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "dat_qp.hpp"

using namespace dat;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int G = 10, NAG = 6;

__global__ __launch_bounds__(64) void k_micro(const QPShared* gsh, const QPLane<1>* glane, const EnvRows* genv,
                                              int nqp, double* out, int* iters) {
  __shared__ QPShared sh[G];
  __shared__ EnvRows er[64];
  const int lane = threadIdx.x;
  const int q = blockIdx.x * 64 + lane;
  if (lane < G) sh[lane] = gsh[blockIdx.x * G + lane];
  if (q < nqp) er[lane] = genv[q];
  __syncthreads();
  if (q >= nqp || lane >= G * NAG) return;
  QPLane<1> P = glane[q];
  const LdsRef<QPShared> shr{sh, lane / NAG};
  const LdsRef<EnvRows> err{er, lane};
  double y[1][3], w[6];
  IPMOut o = ipm_solve<MODE_CADMM, 1>(shr, err, P, y, w, 50, 1e-10);
  out[3 * q] = y[0][0];
  out[3 * q + 1] = y[0][1];
  out[3 * q + 2] = y[0][2];
  iters[q] = o.iters * 4 + o.status;
}

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: %s params.bin [nqp] [reps] [env_rows]\n", argv[0]); return 2; }
  const int n = NAG;
  std::vector<double> prm(DAT_PARAM_SIZE(NAG));
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(prm.data(), sizeof(double), prm.size(), f) != prm.size()) { fprintf(stderr, "bad params\n"); return 2; }
  fclose(f);
  int nblk = (argc > 2 ? atoi(argv[2]) : 262144) / 64;
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  const int nenv = argc > 4 ? atoi(argv[4]) : 0;
  const int nqp = nblk * 64;
  std::vector<QPShared> hsh((size_t)nblk * G);
  std::vector<QPLane<1>> hl(nqp);
  std::vector<EnvRows> he(nqp);
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  std::normal_distribution<double> N01(0.0, 1.0);
  const double* feq = prm.data() + DAT_P_FEQ(n);
  for (int b = 0; b < nblk; ++b)
    for (int s = 0; s < G; ++s) {
      // perturbed hover state
      std::vector<double> st(DAT_STATE_SIZE(n), 0.0);
      for (int i = 0; i < n; ++i) { st[9 * i] = st[9 * i + 4] = st[9 * i + 8] = 1.0; }
      double rv[3] = {0.05 * U(rng), 0.05 * U(rng), 0.05 * U(rng)}, Rl[9];
      exp3(rv, Rl);
      for (int k = 0; k < 9; ++k) st[DAT_S_RL(n) + k] = Rl[k];
      for (int c = 0; c < 3; ++c) {
        st[DAT_S_XL(n) + c] = U(rng);
        st[DAT_S_VL(n) + c] = (c == 0 ? 0.5 : 0.0) + 0.2 * U(rng);
        st[DAT_S_WL(n) + c] = 0.1 * U(rng);
      }
      double acc[6];
      for (int c = 0; c < 6; ++c) acc[c] = 0.5 * U(rng);
      QPShared& S = hsh[(size_t)b * G + s];
      build_shared(S, prm.data(), n, st.data(), acc, prm[DAT_P_KFD], prm[DAT_P_KMD], 3, true);
      double Rt_all[9 * NAG];
      for (int j = 0; j < n; ++j) make_Rt(prm.data() + DAT_P_RCOM(n) + 3 * j, st.data() + DAT_S_RL(n), Rt_all + 9 * j);
      std::vector<double> lam(3 * n), fbar(3 * n);
      for (int k = 0; k < 3 * n; ++k) { lam[k] = 0.1 * N01(rng); fbar[k] = feq[k] + 0.2 * N01(rng); }
      for (int i = 0; i < n; ++i) {
        const int q = b * 64 + s * n + i;
        QPLane<1>& P = hl[q];
        lane_cadmm_static(P, prm.data(), n, i, Rt_all + 9 * i);
        double lhs[DAT_NENV][3] = {}, rhs[DAT_NENV] = {};
        unsigned mask = 0;
        for (int j = 0; j < nenv && j < DAT_NENV; ++j) {
          double d[3] = {1.0 + 0.1 * U(rng), 0.3 * U(rng), 0.1 * U(rng)};
          for (int c = 0; c < 3; ++c) lhs[j][c] = 0.2 * d[c];
          rhs[j] = -3.0 - U(rng);
          mask |= 1u << j;
        }
        set_env_rows(P, he[q], S, mask, lhs, rhs);
        lane_cadmm_dynamic(P, prm.data(), n, i, Rt_all, lam.data(), fbar.data(), 1.0);
      }
    }
  QPShared* dsh;
  QPLane<1>* dl;
  EnvRows* de;
  double* dout;
  int* dit;
  CK(hipMalloc(&dsh, sizeof(QPShared) * hsh.size()));
  CK(hipMalloc(&dl, sizeof(QPLane<1>) * hl.size()));
  CK(hipMalloc(&de, sizeof(EnvRows) * he.size()));
  CK(hipMalloc(&dout, sizeof(double) * 3 * nqp));
  CK(hipMalloc(&dit, sizeof(int) * nqp));
  CK(hipMemcpy(dsh, hsh.data(), sizeof(QPShared) * hsh.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dl, hl.data(), sizeof(QPLane<1>) * hl.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(de, he.data(), sizeof(EnvRows) * he.size(), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_micro, dim3(nblk), dim3(64), 0, 0, dsh, dl, de, nqp, dout, dit);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_micro, dim3(nblk), dim3(64), 0, 0, dsh, dl, de, nqp, dout, dit);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  std::vector<int> it(nqp);
  CK(hipMemcpy(it.data(), dit, sizeof(int) * nqp, hipMemcpyDeviceToHost));
  long long tot = 0, nopt = 0, used = 0;
  int mx = 0;
  for (int q = 0; q < nqp; ++q) {
    if ((q % 64) >= G * NAG) continue;
    ++used;
    tot += it[q] / 4;
    nopt += (it[q] % 4) == 0;
    mx = it[q] / 4 > mx ? it[q] / 4 : mx;
  }
  // wave cost is set by its slowest lane: sum over waves of max iterations
  long long wave_it = 0;
  for (int b = 0; b < nblk; ++b) {
    int m = 0;
    for (int l = 0; l < G * NAG; ++l) m = it[b * 64 + l] / 4 > m ? it[b * 64 + l] / 4 : m;
    wave_it += m;
  }
  printf("{\"variant\": \"%s\", \"env_rows\": %d, \"qps\": %lld, \"ms\": %.4f, \"ns_per_qp\": %.3f, \"mean_iters\": %.3f, "
         "\"max_iters\": %d, \"optimal_frac\": %.5f, \"ns_per_lane_iter\": %.4f, \"wave_iters\": %lld}\n",
         VARIANT, nenv, used, best, best * 1e6 / used, (double)tot / used, mx, (double)nopt / used,
         best * 1e6 / tot, wave_it);
  return 0;
}
