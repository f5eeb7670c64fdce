// Flat-buffer server-side kernels over whole model states:
//   * model-replacement scaling  w' = base + gamma (w - base)             (image_train.py:166-171)
//   * FedAvg apply + DP noise     dst += coef*upd + N(0, sigma) (hash RNG)  (helper.py:240-257)
//   * batched squared distances   ||p_i - m||^2 for ALL clients in one pass (RFA, helper.py:376-381)
//   * weighted sum                sum_i w_i p_i                            (Weiszfeld / FoolsGold)
//   * Gram matrix F F^T on the f32-input MFMA (v_mfma_f32_16x16x4_f32)     (FoolsGold cosine)
//   * anomaly-evasion distance loss  a*CE + (1-a)*||w - w_g||  on the grouped replicas
//     (helper.py:111-123, image_train.py:87-90, loan_train.py:114-117)
#include "common.hpp"
#include <algorithm>

namespace {

int egrid(long long n) { return (int)std::max(1LL, std::min(16384LL, (n + 255) / 256)); }

__global__ void scale_kernel(const float* __restrict__ w, const float* __restrict__ base, float gamma,
                             float* __restrict__ out, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = base[i] + (w[i] - base[i]) * gamma;
}

__global__ void noise_add_kernel(float* __restrict__ dst, const float* __restrict__ upd, long long n, float coef,
                                 float sigma, uint32_t seed, int noise) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float u = upd[i] * coef;
    if (noise) {
      const uint32_t c = (uint32_t)(i * 2);
      const float u1 = uniform01(seed, c), u2 = uniform01(seed, c + 1);
      u += sigma * sqrtf(-2.0f * __logf(u1)) * __cosf(6.283185307179586f * u2);
    }
    dst[i] += u;
  }
}

__global__ __launch_bounds__(256) void sqdist_kernel(const float* __restrict__ pts, long long p_rstride,
                                                     const float* __restrict__ m, long long n,
                                                     double* __restrict__ out) {
  __shared__ float red[4];
  const int i = blockIdx.y;
  const float* p = pts + (long long)i * p_rstride;
  float s = 0.f;
  for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) {
    const float d = p[k] - m[k];
    s += d * d;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out + i, (double)(red[0] + red[1] + red[2] + red[3]));
}

__global__ void wsum_kernel(const float* __restrict__ pts, long long p_rstride, const float* __restrict__ w, int npts,
                            float* __restrict__ out, long long n) {
  for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int i = 0; i < npts; ++i) s = fmaf(w[i], pts[(long long)i * p_rstride + k], s);
    out[k] = s;
  }
}

// out[i][j] += sum_k F[i][k] F[j][k] over this block's k-range; one wave per 16x16 tile
__global__ __launch_bounds__(64) void gram_kernel(const float* __restrict__ F, long long f_rstride, int n, int d,
                                                  int kchunk, float* __restrict__ out) {
  const int ti = blockIdx.x, tj = blockIdx.y;
  const int k0 = blockIdx.z * kchunk, k1 = min(d, k0 + kchunk);
  const int lane = threadIdx.x;
  const int r = lane & 15, kk = lane >> 4;
  const int ia = ti * 16 + r, ib = tj * 16 + r;
  const float* fa = F + (long long)ia * f_rstride;
  const float* fb = F + (long long)ib * f_rstride;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = k0; k < k1; k += 4) {
    const int kx = k + kk;
    const float a = (ia < n && kx < k1) ? fa[kx] : 0.f;
    const float b = (ib < n && kx < k1) ? fb[kx] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  const int j = tj * 16 + (lane & 15);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = ti * 16 + (lane >> 4) * 4 + q;
    if (i < n && j < n) atomicAdd(out + (long long)i * n + j, acc[q]);
  }
}

// nrm2[g] += ||w_g - base_g||^2 over the parameter region (replicas in their poison phase only)
__global__ __launch_bounds__(256) void distnorm_kernel(const float* __restrict__ w, long long ws,
                                                       const float* __restrict__ base, long long bs,
                                                       const int* __restrict__ trig, const int* __restrict__ active,
                                                       long long n, float* __restrict__ nrm2) {
  __shared__ float red[4];
  const int g = blockIdx.y;
  if (trig[g] < 0 || active[g] == 0) return;
  const float* wg = w + (long long)g * ws;
  const float* bg = base + (long long)g * bs;
  float s = 0.f;
  for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) {
    const float d = wg[k] - bg[k];
    s = fmaf(d, d, s);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(nrm2 + g, red[0] + red[1] + red[2] + red[3]);
}

// d/dw [a*CE + (1-a)*||w-b||] = a*g + (1-a)(w-b)/||w-b||  (0 at w == b, torch's norm subgradient)
__global__ void distgrad_kernel(const float* __restrict__ w, long long ws, const float* __restrict__ base,
                                long long bs, float* __restrict__ grads, long long n, const int* __restrict__ trig,
                                const int* __restrict__ active, float alpha, const float* __restrict__ nrm2) {
  const int g = blockIdx.y;
  if (trig[g] < 0 || active[g] == 0) return;
  const float nr = sqrtf(nrm2[g]);
  const float c = nr > 0.f ? (1.f - alpha) / nr : 0.f;
  const float* wg = w + (long long)g * ws;
  const float* bg = base + (long long)g * bs;
  float* gg = grads + (long long)g * n;
  for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x)
    gg[k] = fmaf(alpha, gg[k], c * (wg[k] - bg[k]));
}

}  // namespace

DBA_EXPORT int dba_dist_loss_grad(const float* w, long long ws, const float* base, long long bs, float* grads,
                                  long long n, int G, const int* trig, const int* active, float alpha, float* nrm2,
                                  void* stream) {
  const int bx = (int)std::max(1LL, std::min(256LL, (n + 2047) / 2048));
  hipLaunchKernelGGL(distnorm_kernel, dim3(bx, G), dim3(256), 0, (hipStream_t)stream, w, ws, base, bs, trig, active,
                     n, nrm2);
  hipLaunchKernelGGL(distgrad_kernel, dim3(bx, G), dim3(256), 0, (hipStream_t)stream, w, ws, base, bs, grads, n, trig,
                     active, alpha, nrm2);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_scale_from_base(const float* w, const float* base, float gamma, float* out, long long n,
                                   void* stream) {
  hipLaunchKernelGGL(scale_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, w, base, gamma, out, n);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_add_noise_scaled(float* dst, const float* upd, long long n, float coef, float sigma,
                                    unsigned seed, int noise, void* stream) {
  hipLaunchKernelGGL(noise_add_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, dst, upd, n, coef, sigma,
                     seed, noise);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_sq_dists(const float* pts, long long p_rstride, const float* m, int npts, long long n, double* out,
                            void* stream) {
  const int bx = (int)std::max(1LL, std::min(512LL, (n + 1023) / 1024));
  hipLaunchKernelGGL(sqdist_kernel, dim3(bx, npts), dim3(256), 0, (hipStream_t)stream, pts, p_rstride, m, n, out);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_weighted_sum(const float* pts, long long p_rstride, const float* w, int npts, float* out,
                                long long n, void* stream) {
  hipLaunchKernelGGL(wsum_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, pts, p_rstride, w, npts, out, n);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_gram(const float* F, long long f_rstride, int n, int d, float* out, void* stream) {
  const int t = (n + 15) / 16;
  const int kchunk = 1024;
  dim3 grid(t, t, std::max(1, (d + kchunk - 1) / kchunk));
  hipLaunchKernelGGL(gram_kernel, grid, dim3(64), 0, (hipStream_t)stream, F, f_rstride, n, d, kchunk, out);
  DBA_LAUNCH_CHECK();
}
