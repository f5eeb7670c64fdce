// Flat-buffer server-side kernels over whole model states.  No atomics:
// every cross-block reduction writes per-block partials summed in a fixed order, so results
// are bitwise reproducible.
//   * model-replacement scaling  w' = base + gamma (w - base)             (image_train.py:166-171)
//   * FedAvg delta sum (fp64) + apply + DP noise  dst += coef*sum_i(w_i - g) + N(0, sigma)
//                                 (hash RNG)  (helper.py:218-257)
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

// dst += coef*upd (+ N(0, sigma)); upd fp32 or fp64 (the FedAvg delta sum is kept in fp64)
template <typename U>
__global__ void noise_add_kernel(float* __restrict__ dst, const U* __restrict__ upd, long long n, float coef,
                                 float sigma, uint32_t seed, int noise) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float u = (float)(upd[i] * (U)coef);
    if (noise) {
      const uint32_t c = (uint32_t)(i * 2);
      const float u1 = uniform01(seed, c), u2 = uniform01(seed, c + 1);
      u += sigma * sqrtf(-2.0f * __logf(u1)) * __cosf(6.283185307179586f * u2);
    }
    dst[i] += u;
  }
}

// out[i] = sum_r (rows[r][i] - base[i]) in fp64, rows in order (FedAvg's per-rank delta sum:
// fp32 deltas summed in fp64 are exact, so the all-reduced total does not depend on how the
// clients are split over ranks)
__global__ void delta_sum_kernel(const float* __restrict__ rows, long long rstride, int nrows,
                                 const float* __restrict__ base, long long n, double* __restrict__ out) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const double b = base[i];
    double acc = 0.0;
    for (int r = 0; r < nrows; ++r) acc += (double)rows[(long long)r * rstride + i] - b;
    out[i] = acc;
  }
}

// deterministic two-pass squared distances: part[i][blk] = this block's sum (fp64), then
// sqdist_finalize sums the blocks of point i in block order
__global__ __launch_bounds__(256) void sqdist_kernel(const float* __restrict__ pts, long long p_rstride,
                                                     const float* __restrict__ m, long long n,
                                                     double* __restrict__ part) {
  __shared__ double red[4];
  const int i = blockIdx.y;
  const float* p = pts + (long long)i * p_rstride;
  double s = 0.0;
  for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) {
    const double d = (double)p[k] - (double)m[k];
    s += d * d;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[(long long)i * gridDim.x + blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ void sqdist_finalize(const double* __restrict__ part, int nblk, int npts, double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npts) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += part[(long long)i * nblk + b];
  out[i] = s;
}

template <typename O>
__global__ void wsum_kernel(const float* __restrict__ pts, long long p_rstride, const float* __restrict__ w, int npts,
                            O* __restrict__ out, long long n) {
  for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) {
    O s = 0;
    for (int i = 0; i < npts; ++i) s += (O)w[i] * (O)pts[(long long)i * p_rstride + k];
    out[k] = s;
  }
}

// Reproducible weighted sum (RFA's Weiszfeld average, FoolsGold's weighted gradient): every
// product q = w_i * p_ik * 2^E is exact in fp64 (two fp32 factors, a power-of-two scale) and is
// quantised ON ITS OWN onto a fixed two-limb grid, hi = floor(q), lo = floor((q - hi) * 2^53);
// the limbs are summed as int64 — over the rank's clients here, then over ranks by an int64
// all-reduce — which is exact and order-free, so the sum does not depend on which rank holds
// which client (world-1 == world-N bits).  E is chosen by the caller so |q| <= 2^52 / n (no
// overflow of either limb sum for n <= 512).  out: [2][n] int64 (hi sums, lo sums).
__global__ void wsum_fixed_kernel(const float* __restrict__ pts, long long p_rstride, const float* __restrict__ w,
                                  int npts, long long* __restrict__ out, long long n, double scale) {
  for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) {
    long long hs = 0, ls = 0;
    for (int i = 0; i < npts; ++i) {
      const double q = (double)w[i] * (double)pts[(long long)i * p_rstride + k] * scale;
      const double hi = floor(q);
      hs += (long long)hi;
      ls += (long long)floor((q - hi) * 0x1p53);
    }
    out[k] = hs;
    out[n + k] = ls;
  }
}

// slab[z][i][j] = sum over k-chunk z of F[i][k] F[j][k]; one wave per 16x16 tile (f32 MFMA),
// summed over z in order by gram_finalize (no atomics)
__global__ __launch_bounds__(64) void gram_kernel(const float* __restrict__ F, long long f_rstride, int n, int d,
                                                  int kchunk, float* __restrict__ slab) {
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
  float* out = slab + (long long)blockIdx.z * n * n;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = ti * 16 + (lane >> 4) * 4 + q;
    if (i < n && j < n) out[(long long)i * n + j] = acc[q];
  }
}

__global__ void gram_finalize(const float* __restrict__ slab, int nz, int nn, double* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nn) return;
  double s = 0.0;
  for (int z = 0; z < nz; ++z) s += (double)slab[(long long)z * nn + e];
  out[e] = s;
}

// part[g][blk] = this block's sum of (w_g - base_g)^2 over the parameter region (replicas in
// their poison phase only); distgrad_kernel sums a replica's parts in block order
__global__ __launch_bounds__(256) void distnorm_kernel(const float* __restrict__ w, long long ws,
                                                       const float* __restrict__ base, long long bs,
                                                       const int* __restrict__ trig, const int* __restrict__ active,
                                                       long long n, float* __restrict__ part) {
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
  if (threadIdx.x == 0) part[(long long)g * gridDim.x + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// d/dw [a*CE + (1-a)*||w-b||] = a*g + (1-a)(w-b)/||w-b||  (0 at w == b, torch's norm subgradient);
// block (0, g) also publishes ||w-b||^2 into nrm2[g]
__global__ void distgrad_kernel(const float* __restrict__ w, long long ws, const float* __restrict__ base,
                                long long bs, float* __restrict__ grads, long long n, const int* __restrict__ trig,
                                const int* __restrict__ active, float alpha, const float* __restrict__ part,
                                float* __restrict__ nrm2) {
  const int g = blockIdx.y;
  if (trig[g] < 0 || active[g] == 0) return;
  float n2 = 0.f;
  for (int b = 0; b < (int)gridDim.x; ++b) n2 += part[(long long)g * gridDim.x + b];
  if (blockIdx.x == 0 && threadIdx.x == 0) nrm2[g] = n2;
  const float nr = sqrtf(n2);
  const float c = nr > 0.f ? (1.f - alpha) / nr : 0.f;
  const float* wg = w + (long long)g * ws;
  const float* bg = base + (long long)g * bs;
  float* gg = grads + (long long)g * n;
  for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x)
    gg[k] = fmaf(alpha, gg[k], c * (wg[k] - bg[k]));
}

}  // namespace

// part: [G][256] fp32 workspace (no initialisation needed)
DBA_EXPORT int dba_dist_loss_grad(const float* w, long long ws, const float* base, long long bs, float* grads,
                                  long long n, int G, const int* trig, const int* active, float alpha, float* nrm2,
                                  float* part, void* stream) {
  const int bx = (int)std::max(1LL, std::min(256LL, (n + 2047) / 2048));
  hipLaunchKernelGGL(distnorm_kernel, dim3(bx, G), dim3(256), 0, (hipStream_t)stream, w, ws, base, bs, trig, active,
                     n, part);
  hipLaunchKernelGGL(distgrad_kernel, dim3(bx, G), dim3(256), 0, (hipStream_t)stream, w, ws, base, bs, grads, n, trig,
                     active, alpha, part, nrm2);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_scale_from_base(const float* w, const float* base, float gamma, float* out, long long n,
                                   void* stream) {
  hipLaunchKernelGGL(scale_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, w, base, gamma, out, n);
  DBA_LAUNCH_CHECK();
}

// upd fp64 (upd_f64) or fp32
DBA_EXPORT int dba_add_noise_scaled(float* dst, const void* upd, long long n, float coef, float sigma,
                                    unsigned seed, int noise, int upd_f64, void* stream) {
  if (upd_f64)
    hipLaunchKernelGGL(noise_add_kernel<double>, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, dst,
                       (const double*)upd, n, coef, sigma, seed, noise);
  else
    hipLaunchKernelGGL(noise_add_kernel<float>, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, dst,
                       (const float*)upd, n, coef, sigma, seed, noise);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_delta_sum(const float* rows, long long rstride, int nrows, const float* base, long long n,
                             double* out, void* stream) {
  hipLaunchKernelGGL(delta_sum_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, rows, rstride, nrows, base,
                     n, out);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_sqdist_blocks(long long n) { return (int)std::max(1LL, std::min(512LL, (n + 1023) / 1024)); }

// part: [npts][dba_sqdist_blocks(n)] fp64 workspace
DBA_EXPORT int dba_sq_dists(const float* pts, long long p_rstride, const float* m, int npts, long long n, double* out,
                            double* part, void* stream) {
  const int bx = dba_sqdist_blocks(n);
  hipLaunchKernelGGL(sqdist_kernel, dim3(bx, npts), dim3(256), 0, (hipStream_t)stream, pts, p_rstride, m, n, part);
  hipLaunchKernelGGL(sqdist_finalize, dim3((npts + 63) / 64), dim3(64), 0, (hipStream_t)stream, part, bx, npts, out);
  DBA_LAUNCH_CHECK();
}

// out fp64 (out_f64) or fp32
DBA_EXPORT int dba_weighted_sum(const float* pts, long long p_rstride, const float* w, int npts, void* out,
                                long long n, int out_f64, void* stream) {
  if (out_f64)
    hipLaunchKernelGGL(wsum_kernel<double>, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, pts, p_rstride, w, npts,
                       (double*)out, n);
  else
    hipLaunchKernelGGL(wsum_kernel<float>, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, pts, p_rstride, w, npts,
                       (float*)out, n);
  DBA_LAUNCH_CHECK();
}

// out [2][n] int64: the fixed-point limb sums of sum_i w[i] * pts[i] (wsum_fixed_kernel); scale = 2^E
DBA_EXPORT int dba_weighted_sum_fixed(const float* pts, long long p_rstride, const float* w, int npts, long long* out,
                                      long long n, double scale, void* stream) {
  hipLaunchKernelGGL(wsum_fixed_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, pts, p_rstride, w, npts, out,
                     n, scale);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_gram_chunks(int d) { return std::max(1, (d + 1023) / 1024); }

// slab: [dba_gram_chunks(d)][n][n] fp32 workspace; out [n][n] fp64
DBA_EXPORT int dba_gram(const float* F, long long f_rstride, int n, int d, double* out, float* slab, void* stream) {
  const int t = (n + 15) / 16;
  const int kchunk = 1024;
  const int nz = dba_gram_chunks(d);
  dim3 grid(t, t, nz);
  hipLaunchKernelGGL(gram_kernel, grid, dim3(64), 0, (hipStream_t)stream, F, f_rstride, n, d, kchunk, slab);
  hipLaunchKernelGGL(gram_finalize, dim3((n * n + 255) / 256), dim3(256), 0, (hipStream_t)stream, slab, nz, n * n, out);
  DBA_LAUNCH_CHECK();
}
