// Pooling, ReLU-mask backward and dropout for grouped NHWC activations (bf16 or fp32)
// (LoanNet dropout, loan_model.py:13-19).
#include "common.hpp"
#include <algorithm>

namespace {

int egrid(long long n) { return (int)std::max(1LL, std::min(16384LL, (n + 255) / 256)); }

template <typename T>
__global__ void relu_mask_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ out, T* __restrict__ din,
                                     long long n8) {
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n8; t += (long long)gridDim.x * blockDim.x) {
    float d[8], o[8];
    ld8(dout + t * 8, d);
    ld8(out + t * 8, o);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (!(o[e] > 0.f)) d[e] = 0.f;
    st8(din + t * 8, d);
  }
}

template <typename T>
__global__ void relu_mask_bwd_tail(const T* __restrict__ dout, const T* __restrict__ out, T* __restrict__ din,
                                   long long beg, long long n) {
  const long long t = beg + blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t < n) din[t] = to_f<T>(out[t]) > 0.f ? dout[t] : from_f<T>(0.f);
}

// y[gn][ho][wo][c] = max window; ind = flat input index hi*W+wi (first max, like PyTorch)
template <typename T>
__global__ void maxpool_kernel(const T* __restrict__ x, T* __restrict__ y, int* __restrict__ ind,
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
        const float v = to_f<T>(x[((gn * H + hi) * W + wi) * C + c]);
        if (v > best || bi < 0 || v != v) { best = v; bi = hi * W + wi; }
      }
    }
    y[t] = from_f<T>(best);
    if (ind) ind[t] = bi;
  }
}

// fp32, C % 4 == 0, fewer than 2^31 channel quads: 4 channels per thread (16-B loads / stores),
// 32-bit index arithmetic (the generic form's 64-bit divisions dominated MnistNet's evaluation
// pools: 162 us per launch, profiles/r5/mnist/); ind optional (evaluation needs no indices).
// Same selection rule per channel (first maximum in window order; a NaN wins).
__global__ void maxpool_v4_kernel(const float* __restrict__ x, float* __restrict__ y, int* __restrict__ ind,
                                  unsigned total4, int H, int W, int C4, int Ho, int Wo, int k, int s, int p) {
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total4; t += gridDim.x * blockDim.x) {
    const unsigned c4 = t % (unsigned)C4;
    unsigned r = t / (unsigned)C4;
    const int wo = (int)(r % (unsigned)Wo);
    r /= (unsigned)Wo;
    const int ho = (int)(r % (unsigned)Ho);
    const unsigned gn = r / (unsigned)Ho;
    const float4* __restrict__ xi = (const float4*)x + (long long)gn * H * W * C4 + c4;
    float b[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int bi[4] = {-1, -1, -1, -1};
    for (int i = 0; i < k; ++i) {
      const int hi = ho * s - p + i;
      if ((unsigned)hi >= (unsigned)H) continue;
      for (int j = 0; j < k; ++j) {
        const int wi = wo * s - p + j;
        if ((unsigned)wi >= (unsigned)W) continue;
        const float4 v4 = xi[(hi * W + wi) * C4];
        const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (v[e] > b[e] || bi[e] < 0 || v[e] != v[e]) { b[e] = v[e]; bi[e] = hi * W + wi; }
      }
    }
    ((float4*)y)[t] = make_float4(b[0], b[1], b[2], b[3]);
    if (ind) ((int4*)ind)[t] = make_int4(bi[0], bi[1], bi[2], bi[3]);
  }
}

// gather form of the max-pool backward (no atomics, deterministic)
template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ dy, const int* __restrict__ ind, T* __restrict__ dx,
                                   long long GN, int H, int W, int C, int Ho, int Wo, int k, int s, int p) {
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
        if (ind[o] == me) acc += to_f<T>(dy[o]);
      }
    dx[t] = from_f<T>(acc);
  }
}

// the fp32 gather form for C % 4 == 0, 4 channels per thread (16-B dy / index / dx accesses) and
// 32-bit index math (the form above spends 4 64-bit divisions per element: 105 us per Tiny
// lone-client step).  Same windows in the same (ho, wo) order per element, a non-matching window
// adding nothing (acc + 0 == acc: acc starts at +0 and is never -0): the same bits.
__global__ __launch_bounds__(256) void maxpool_bwd4_kernel(const float4* __restrict__ dy, const int4* __restrict__ ind,
                                                           float4* __restrict__ dx, int GN, int H, int W, int C4,
                                                           int Ho, int Wo, int k, int s, int p) {
  const int total = GN * H * W * C4;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int c4 = t % C4;
    int r = t / C4;
    const int w = r % W;
    r /= W;
    const int h = r % H, gn = r / H;
    const int me = h * W + w;
    const int ho0 = max(0, (h + p - k + s) / s), ho1 = min(Ho - 1, (h + p) / s);
    const int wo0 = max(0, (w + p - k + s) / s), wo1 = min(Wo - 1, (w + p) / s);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int ho = ho0; ho <= ho1; ++ho)
      for (int wo = wo0; wo <= wo1; ++wo) {
        const int o = ((gn * Ho + ho) * Wo + wo) * C4 + c4;
        const int4 id = ind[o];
        const float4 d = dy[o];
        if (id.x == me) acc.x += d.x;
        if (id.y == me) acc.y += d.y;
        if (id.z == me) acc.z += d.z;
        if (id.w == me) acc.w += d.w;
      }
    dx[t] = acc;
  }
}

template <typename T>
__global__ void avgpool_kernel(const T* __restrict__ x, T* __restrict__ y, long long GN, int HW, int C) {
  const long long total = GN * C;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    const long long gn = t / C;
    float s = 0.f;
    for (int i = 0; i < HW; ++i) s += to_f<T>(x[(gn * HW + i) * C + c]);
    y[t] = from_f<T>(s / (float)HW);
  }
}

template <typename T>
__global__ void avgpool_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, long long GN, int HW, int C) {
  const long long total = GN * HW * C;
  const float inv = 1.0f / (float)HW;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    const long long gn = t / ((long long)HW * C);
    dx[t] = from_f<T>(to_f<T>(dy[gn * C + c]) * inv);
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

#define EW_T(f32, call) do { if (f32) { typedef float T; call; } else { typedef uint16_t T; call; } } while (0)

DBA_EXPORT int dba_relu_mask_bwd(const void* dout, const void* out, void* din, long long n, int f32, void* stream) {
  const long long n8 = n / 8;
  hipStream_t st = (hipStream_t)stream;
  if (n8 > 0)
    EW_T(f32, hipLaunchKernelGGL((relu_mask_bwd_kernel<T>), dim3(egrid(n8)), dim3(256), 0, st, (const T*)dout,
                                 (const T*)out, (T*)din, n8));
  if (n8 * 8 < n)
    EW_T(f32, hipLaunchKernelGGL((relu_mask_bwd_tail<T>), dim3(1), dim3(256), 0, st, (const T*)dout, (const T*)out,
                                 (T*)din, n8 * 8, n));
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_maxpool(const void* x, void* y, int* ind, long long GN, int H, int W, int C, int Ho, int Wo, int k,
                           int s, int p, int f32, void* stream) {
  const long long total4 = GN * Ho * Wo * (C / 4);
  if (f32 && C % 4 == 0 && total4 < (1LL << 31) && !((uintptr_t)x & 15) && !((uintptr_t)y & 15) &&
      !((uintptr_t)ind & 15)) {
    hipLaunchKernelGGL(maxpool_v4_kernel, dim3(egrid(total4)), dim3(256), 0, (hipStream_t)stream, (const float*)x,
                       (float*)y, ind, (unsigned)total4, H, W, C / 4, Ho, Wo, k, s, p);
    DBA_LAUNCH_CHECK();
  }
  EW_T(f32, hipLaunchKernelGGL((maxpool_kernel<T>), dim3(egrid(GN * Ho * Wo * C)), dim3(256), 0, (hipStream_t)stream,
                               (const T*)x, (T*)y, ind, GN, H, W, C, Ho, Wo, k, s, p));
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_maxpool_bwd(const void* dy, const int* ind, void* dx, long long GN, int H, int W, int C, int Ho,
                               int Wo, int k, int s, int p, int f32, void* stream) {
  if (f32 && C % 4 == 0 && GN * H * W * C < (1LL << 31) && GN * Ho * Wo * C < (1LL << 31) &&
      !(((uintptr_t)dy | (uintptr_t)ind | (uintptr_t)dx) & 15)) {
    const long long total4 = GN * H * W * (C / 4);
    hipLaunchKernelGGL(maxpool_bwd4_kernel, dim3(egrid(total4)), dim3(256), 0, (hipStream_t)stream, (const float4*)dy,
                       (const int4*)ind, (float4*)dx, (int)GN, H, W, C / 4, Ho, Wo, k, s, p);
    DBA_LAUNCH_CHECK();
  }
  EW_T(f32, hipLaunchKernelGGL((maxpool_bwd_kernel<T>), dim3(egrid(GN * H * W * C)), dim3(256), 0, (hipStream_t)stream,
                               (const T*)dy, ind, (T*)dx, GN, H, W, C, Ho, Wo, k, s, p));
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_avgpool(const void* x, void* y, long long GN, int HW, int C, int f32, void* stream) {
  EW_T(f32, hipLaunchKernelGGL((avgpool_kernel<T>), dim3(egrid(GN * C)), dim3(256), 0, (hipStream_t)stream,
                               (const T*)x, (T*)y, GN, HW, C));
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_avgpool_bwd(const void* dy, void* dx, long long GN, int HW, int C, int f32, void* stream) {
  EW_T(f32, hipLaunchKernelGGL((avgpool_bwd_kernel<T>), dim3(egrid(GN * HW * C)), dim3(256), 0, (hipStream_t)stream,
                               (const T*)dy, (T*)dx, GN, HW, C));
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
