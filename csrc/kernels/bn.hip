// Evaluation-mode BatchNorm folded into the preceding conv: w' = w * s,
// b' = (b - mean) * s + beta with s = gamma / sqrt(var + eps), once per model snapshot, so
// every evaluation conv is one kernel with a fused bias epilogue.  (Training BN is fused into
// the conv kernels: bnfuse.hpp.)
#include "common.hpp"
#include <algorithm>

namespace {

// eval fold: wf[s][co][k] = w[s][co][k] * s_c ; bf[s][co] = (b0 - rm) * s_c + beta, and (amax
// given) max |wf| of each slot folded into its zeroed operand-max slot (common.hpp) — the scale
// of the folded weights' fp16 pair, exactly what a separate max pass over wf returns.  blockIdx.y
// = slot.
template <typename T>
__global__ void bn_fold_kernel(const float* __restrict__ w, long long w_sstride, const float* __restrict__ cbias,
                               const float* __restrict__ gamma, const float* __restrict__ beta,
                               const float* __restrict__ rm, const float* __restrict__ rv, long long s_gstride,
                               float eps, T* __restrict__ wf, float* __restrict__ bf, int Cout, int K,
                               int* __restrict__ amax, int amax_ld) {
  const int s = blockIdx.y;
  const long long per = (long long)Cout * K;
  float m = 0.f;
  for (long long rem = blockIdx.x * (long long)blockDim.x + threadIdx.x; rem < per;
       rem += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(rem / K);
    const int k = (int)(rem - (long long)co * K);
    const long long p = (long long)s * s_gstride + co;
    const float sc = gamma[p] / sqrtf(rv[p] + eps);
    const float v = w[(long long)s * w_sstride + rem] * sc;
    wf[(long long)s * per + rem] = from_f<T>(v);
    m = fmaxf(m, fabsf(v));
    if (k == 0) {
      const float b0 = cbias ? cbias[p] : 0.f;
      bf[(long long)s * Cout + co] = (b0 - rm[p]) * sc + beta[p];
    }
  }
  if (amax) amax_fold(amax, amax_ld, s, m);
}

int egrid(long long n) { return (int)std::max(1LL, std::min(4096LL, (n + 255) / 256)); }

}  // namespace

// wf fp32 (the f32 flag must be set: the bf16 family is gone)
DBA_EXPORT int dba_bn_fold(const float* w, long long w_sstride, const float* cbias, const float* gamma,
                           const float* beta, const float* rm, const float* rv, long long s_gstride, float eps,
                           void* wf, float* bf, int slots, int Cout, int K, int f32, int* amax, int amax_ld,
                           void* stream) {
  if (!f32) return -102;
  const long long per = (long long)Cout * K;
  hipLaunchKernelGGL((bn_fold_kernel<float>), dim3(egrid(per), slots), dim3(256), 0, (hipStream_t)stream, w, w_sstride,
                     cbias, gamma, beta, rm, rv, s_gstride, eps, (float*)wf, bf, Cout, (int)K, amax, amax_ld);
  DBA_LAUNCH_CHECK();
}
