// Fused batch ingest: device-resident uint8 dataset -> gathered,
// converted, optionally h-flipped, trigger-stamped, relabelled batch in one pass.
// Replaces the reference's DataLoader workers + ToTensor + Python per-pixel trigger loop
// (image_helper.py:252-263,298-350) and LOAN's per-row feature writes (loan_train.py:99-107).
#include "common.hpp"
#include <algorithm>

namespace {

template <typename OutT>
__global__ void gather_images_kernel(const uint8_t* __restrict__ src, const int* __restrict__ labels,
                                     const int* __restrict__ idx, const uint8_t* __restrict__ masks,
                                     const int* __restrict__ trig, const int* __restrict__ poison_n, int target,
                                     const int* __restrict__ flip_seeds, OutT* __restrict__ out,
                                     int* __restrict__ yout, int G, int B, int H, int W, int C) {
  const long long total = (long long)G * B * H * W;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int w = (int)(t % W);
    long long r = t / W;
    const int h = (int)(r % H);
    r /= H;
    const int b = (int)(r % B);
    const int g = (int)(r / B);
    const int s = idx[g * B + b];
    OutT* o = out + t * C;
    if (s < 0) {
      for (int c = 0; c < C; ++c) o[c] = from_f<OutT>(0.f);
      if (h == 0 && w == 0) yout[g * B + b] = -1;
      continue;
    }
    int ws = w;
    if (flip_seeds && (hash2((uint32_t)flip_seeds[g], (uint32_t)b) & 1u)) ws = W - 1 - w;
    const int tg = trig[g];
    const bool pois = tg >= 0 && b < poison_n[g];
    const bool stamp = pois && masks[((long long)tg * H + h) * W + w];
    const uint8_t* p = src + (((long long)s * H + h) * W + ws) * C;
    for (int c = 0; c < C; ++c) o[c] = from_f<OutT>((stamp ? 255.f : (float)p[c]) * (1.0f / 255.0f));
    if (h == 0 && w == 0) yout[g * B + b] = pois ? target : labels[s];
  }
}

template <typename OutT>
__global__ void gather_rows_kernel(const float* __restrict__ src, const int* __restrict__ labels,
                                   const int* __restrict__ idx, const int* __restrict__ tcols,
                                   const float* __restrict__ tvals, int K, const int* __restrict__ trig,
                                   const int* __restrict__ poison_n, int target, OutT* __restrict__ out,
                                   int* __restrict__ yout, int G, int B, int F) {
  const long long total = (long long)G * B * F;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int f = (int)(t % F);
    const long long gb = t / F;
    const int b = (int)(gb % B), g = (int)(gb / B);
    const int s = idx[gb];
    if (s < 0) {
      out[t] = from_f<OutT>(0.f);
      if (f == 0) yout[gb] = -1;
      continue;
    }
    float v = src[(long long)s * F + f];
    const int tg = trig[g];
    const bool pois = tg >= 0 && b < poison_n[g];
    if (pois)
      for (int k = 0; k < K; ++k)
        if (tcols[tg * K + k] == f) v = tvals[tg * K + k];
    out[t] = from_f<OutT>(v);
    if (f == 0) yout[gb] = pois ? target : labels[s];
  }
}

int grid_for(long long n) { return (int)std::max(1LL, std::min(8192LL, (n + 255) / 256)); }

}  // namespace

DBA_EXPORT int dba_gather_images(const void* src, const int* labels, const int* idx, const void* masks, const int* trig,
                                 const int* poison_n, int target, const int* flip_seeds, void* out, int out_f32,
                                 int* yout, int G, int B, int H, int W, int C, void* stream) {
  const long long n = (long long)G * B * H * W;
  if (out_f32)
    hipLaunchKernelGGL(gather_images_kernel<float>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                       (const uint8_t*)src, labels, idx, (const uint8_t*)masks, trig, poison_n, target, flip_seeds,
                       (float*)out, yout, G, B, H, W, C);
  else
    hipLaunchKernelGGL(gather_images_kernel<uint16_t>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                       (const uint8_t*)src, labels, idx, (const uint8_t*)masks, trig, poison_n, target, flip_seeds,
                       (uint16_t*)out, yout, G, B, H, W, C);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_gather_rows(const float* src, const int* labels, const int* idx, const int* tcols, const float* tvals,
                               int K, const int* trig, const int* poison_n, int target, void* out, int out_f32,
                               int* yout, int G, int B, int F, void* stream) {
  const long long n = (long long)G * B * F;
  if (out_f32)
    hipLaunchKernelGGL(gather_rows_kernel<float>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, src, labels,
                       idx, tcols, tvals, K, trig, poison_n, target, (float*)out, yout, G, B, F);
  else
    hipLaunchKernelGGL(gather_rows_kernel<uint16_t>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, src,
                       labels, idx, tcols, tvals, K, trig, poison_n, target, (uint16_t*)out, yout, G, B, F);
  DBA_LAUNCH_CHECK();
}
