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

// a whole model fold in one launch (blockIdx.y = slot): the per-conv launches of a 20-conv
// ResNet fold were ~20 launch floors per evaluated snapshot.  The x grid is the concatenation
// of every conv's chunks of kFoldChunk elements (desc i owns blocks [boff_i, boff_{i+1})), so
// no block idles (a max-sized grid per desc dispatched ~4096 x 20 mostly-empty blocks).
struct FoldDesc {   // all int64 (built from a torch int64 host tensor)
  long long w, w_sstride, gamma, beta, rm, rv, s_gstride, wf, bf, Cout, K, amax, amax_ld, boff;
};
constexpr int kFoldBatch = 24;
constexpr int kFoldChunk = 2048;   // elements per 256-thread block (8 per thread)
struct FoldBatch {
  FoldDesc d[kFoldBatch];
  int n;
};
__global__ void bn_fold_batch_kernel(const FoldBatch b, float eps) {
  int i = 0;
  while (i + 1 < b.n && (long long)blockIdx.x >= b.d[i + 1].boff) ++i;
  const FoldDesc& d = b.d[i];
  const int s = blockIdx.y, Cout = (int)d.Cout, K = (int)d.K;
  const long long per = (long long)Cout * K;
  const float* gamma = (const float*)d.gamma; const float* beta = (const float*)d.beta;
  const float* rm = (const float*)d.rm; const float* rv = (const float*)d.rv;
  const float* w = (const float*)d.w;
  float* wf = (float*)d.wf; float* bf = (float*)d.bf;
  const long long base = ((long long)blockIdx.x - d.boff) * kFoldChunk;
  const long long end = base + kFoldChunk < per ? base + kFoldChunk : per;
  float m = 0.f;
  for (long long rem = base + threadIdx.x; rem < end; rem += blockDim.x) {
    const int co = (int)(rem / K);
    const int k = (int)(rem - (long long)co * K);
    const long long p = (long long)s * d.s_gstride + co;
    const float sc = gamma[p] / sqrtf(rv[p] + eps);
    const float v = w[(long long)s * d.w_sstride + rem] * sc;
    wf[(long long)s * per + rem] = v;
    m = fmaxf(m, fabsf(v));
    if (k == 0) bf[(long long)s * Cout + co] = (0.f - rm[p]) * sc + beta[p];
  }
  amax_fold((int*)d.amax, (int)d.amax_ld, s, m);
}

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

// n BN folds (no conv bias, fp32) of one model bank with `slots` slots in one launch per 24;
// desc: n x FoldDesc in HOST memory (passed by value: graph-capture safe)
DBA_EXPORT int dba_bn_fold_batch(const void* desc, int n, int slots, float eps, void* stream) {
  const FoldDesc* ds = (const FoldDesc*)desc;
  for (int i0 = 0; i0 < n; i0 += kFoldBatch) {
    FoldBatch b{};
    b.n = std::min(kFoldBatch, n - i0);
    long long nb = 0;
    for (int i = 0; i < b.n; ++i) {
      b.d[i] = ds[i0 + i];
      b.d[i].boff = nb;
      nb += (b.d[i].Cout * b.d[i].K + kFoldChunk - 1) / kFoldChunk;
    }
    hipLaunchKernelGGL(bn_fold_batch_kernel, dim3((unsigned)nb, slots), dim3(256), 0, (hipStream_t)stream, b, eps);
    const int rc = (int)hipGetLastError();
    if (rc != 0) return rc;
  }
  return 0;
}
