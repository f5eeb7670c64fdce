// Pooling, ReLU-mask backward and dropout for grouped NHWC bf16 activations
// (LoanNet dropout, loan_model.py:13-19).
#include "common.hpp"
#include <algorithm>

namespace {

int egrid(long long n) { return (int)std::max(1LL, std::min(16384LL, (n + 255) / 256)); }

__global__ void relu_mask_bwd_kernel(const uint16_t* __restrict__ dout, const uint16_t* __restrict__ out,
                                     uint16_t* __restrict__ din, long long n8) {
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n8; t += (long long)gridDim.x * blockDim.x) {
    uint4 d = *(const uint4*)(dout + t * 8);
    const uint4 o = *(const uint4*)(out + t * 8);
    uint16_t* dp = (uint16_t*)&d;
    const uint16_t* op = (const uint16_t*)&o;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (!(bf2f(op[e]) > 0.f)) dp[e] = 0;
    *(uint4*)(din + t * 8) = d;
  }
}

__global__ void relu_mask_bwd_tail(const uint16_t* __restrict__ dout, const uint16_t* __restrict__ out,
                                   uint16_t* __restrict__ din, long long beg, long long n) {
  const long long t = beg + blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t < n) din[t] = bf2f(out[t]) > 0.f ? dout[t] : (uint16_t)0;
}

// y[gn][ho][wo][c] = max window; ind = flat input index hi*W+wi (first max, like PyTorch)
__global__ void maxpool_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int* __restrict__ ind,
                               long long GN, int H, int W, int C, int Ho, int Wo, int k, int s, int p) {
  const long long total = GN * Ho * Wo * C;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    long long r = t / C;
    const int wo = (int)(r % Wo);
    r /= Wo;
    const int ho = (int)(r % Ho);
    const long long gn = r / Ho;
    float best = -INFINITY;
    int bi = -1;
    for (int i = 0; i < k; ++i) {
      const int hi = ho * s - p + i;
      if ((unsigned)hi >= (unsigned)H) continue;
      for (int j = 0; j < k; ++j) {
        const int wi = wo * s - p + j;
        if ((unsigned)wi >= (unsigned)W) continue;
        const float v = bf2f(x[((gn * H + hi) * W + wi) * C + c]);
        if (v > best || bi < 0 || v != v) { best = v; bi = hi * W + wi; }
      }
    }
    y[t] = f2bf(best);
    ind[t] = bi;
  }
}

// gather form of the max-pool backward (no atomics, deterministic)
__global__ void maxpool_bwd_kernel(const uint16_t* __restrict__ dy, const int* __restrict__ ind,
                                   uint16_t* __restrict__ dx, long long GN, int H, int W, int C, int Ho, int Wo, int k,
                                   int s, int p) {
  const long long total = GN * H * W * C;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    long long r = t / C;
    const int w = (int)(r % W);
    r /= W;
    const int h = (int)(r % H);
    const long long gn = r / H;
    const int me = h * W + w;
    const int ho0 = max(0, (h + p - k + s) / s), ho1 = min(Ho - 1, (h + p) / s);
    const int wo0 = max(0, (w + p - k + s) / s), wo1 = min(Wo - 1, (w + p) / s);
    float acc = 0.f;
    for (int ho = ho0; ho <= ho1; ++ho)
      for (int wo = wo0; wo <= wo1; ++wo) {
        const long long o = ((gn * Ho + ho) * Wo + wo) * C + c;
        if (ind[o] == me) acc += bf2f(dy[o]);
      }
    dx[t] = f2bf(acc);
  }
}

__global__ void avgpool_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, long long GN, int HW, int C) {
  const long long total = GN * C;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    const long long gn = t / C;
    float s = 0.f;
    for (int i = 0; i < HW; ++i) s += bf2f(x[(gn * HW + i) * C + c]);
    y[t] = f2bf(s / (float)HW);
  }
}

__global__ void avgpool_bwd_kernel(const uint16_t* __restrict__ dy, uint16_t* __restrict__ dx, long long GN, int HW,
                                   int C) {
  const long long total = GN * HW * C;
  const float inv = 1.0f / (float)HW;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    const long long gn = t / ((long long)HW * C);
    dx[t] = f2bf(bf2f(dy[gn * C + c]) * inv);
  }
}

// keep iff uniform(seed[g] + salt*0x9E3779B9, i_in_group) >= p ; y = x * keep / (1-p)
template <typename T>
__global__ void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, const int* __restrict__ seeds, uint32_t salt,
                               float p, long long per, int G) {
  const long long total = per * G;
  const float scale = 1.0f / (1.0f - p);
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int g = (int)(t / per);
    const uint32_t i = (uint32_t)(t - (long long)g * per);
    const uint32_t sd = (uint32_t)seeds[g] + salt * 0x9E3779B9u;
    const bool keep = uniform01(sd, i) >= p;
    y[t] = from_f<T>(keep ? to_f<T>(x[t]) * scale : 0.f);
  }
}

}  // namespace

DBA_EXPORT int dba_relu_mask_bwd(const void* dout, const void* out, void* din, long long n, void* stream) {
  const long long n8 = n / 8;
  if (n8 > 0)
    hipLaunchKernelGGL(relu_mask_bwd_kernel, dim3(egrid(n8)), dim3(256), 0, (hipStream_t)stream,
                       (const uint16_t*)dout, (const uint16_t*)out, (uint16_t*)din, n8);
  if (n8 * 8 < n)
    hipLaunchKernelGGL(relu_mask_bwd_tail, dim3(1), dim3(256), 0, (hipStream_t)stream, (const uint16_t*)dout,
                       (const uint16_t*)out, (uint16_t*)din, n8 * 8, n);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_maxpool(const void* x, void* y, int* ind, long long GN, int H, int W, int C, int Ho, int Wo, int k,
                           int s, int p, void* stream) {
  hipLaunchKernelGGL(maxpool_kernel, dim3(egrid(GN * Ho * Wo * C)), dim3(256), 0, (hipStream_t)stream,
                     (const uint16_t*)x, (uint16_t*)y, ind, GN, H, W, C, Ho, Wo, k, s, p);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_maxpool_bwd(const void* dy, const int* ind, void* dx, long long GN, int H, int W, int C, int Ho,
                               int Wo, int k, int s, int p, void* stream) {
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(egrid(GN * H * W * C)), dim3(256), 0, (hipStream_t)stream,
                     (const uint16_t*)dy, ind, (uint16_t*)dx, GN, H, W, C, Ho, Wo, k, s, p);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_avgpool(const void* x, void* y, long long GN, int HW, int C, void* stream) {
  hipLaunchKernelGGL(avgpool_kernel, dim3(egrid(GN * C)), dim3(256), 0, (hipStream_t)stream, (const uint16_t*)x,
                     (uint16_t*)y, GN, HW, C);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_avgpool_bwd(const void* dy, void* dx, long long GN, int HW, int C, void* stream) {
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(egrid(GN * HW * C)), dim3(256), 0, (hipStream_t)stream,
                     (const uint16_t*)dy, (uint16_t*)dx, GN, HW, C);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_dropout(const void* x, void* y, int is_f32, const int* seeds, unsigned salt, float p, long long per,
                           int G, void* stream) {
  if (is_f32)
    hipLaunchKernelGGL(dropout_kernel<float>, dim3(egrid(per * G)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)x, (float*)y, seeds, salt, p, per, G);
  else
    hipLaunchKernelGGL(dropout_kernel<uint16_t>, dim3(egrid(per * G)), dim3(256), 0, (hipStream_t)stream,
                       (const uint16_t*)x, (uint16_t*)y, seeds, salt, p, per, G);
  DBA_LAUNCH_CHECK();
}
