// Fused softmax cross-entropy forward + backward + correct count, per group (K9).
// Replaces log_softmax/cross_entropy/argmax/eq/sum and the per-batch `.item()` host syncs
// of the reference (image_train.py:85,104-105; test.py:34-37): counters stay on device.
#include "common.hpp"

namespace {

__global__ __launch_bounds__(256) void xent_kernel(const float* __restrict__ logits, const int* __restrict__ labels,
                                                   int B, int C, int mean, uint16_t* __restrict__ dl,
                                                   float* __restrict__ loss_out, float* __restrict__ corr_out) {
  __shared__ float sl[4], sc[4];
  __shared__ int scnt[4];
  const int g = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int* lab = labels + (long long)g * B;
  int cnt = 0;
  for (int b = tid; b < B; b += 256) cnt += lab[b] >= 0;
  // block-reduce the valid count
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, kWave);
  if (lane == 0) scnt[wid] = cnt;
  __syncthreads();
  const int n = scnt[0] + scnt[1] + scnt[2] + scnt[3];
  const float scale = (mean && n > 0) ? 1.0f / (float)n : 1.0f;
  float wl = 0.f, wc = 0.f;
  for (int b = wid; b < B; b += 4) {
    const float* x = logits + ((long long)g * B + b) * C;
    const int y = lab[b];
    float mx = -INFINITY;
    int am = 0x7fffffff;
    for (int c = lane; c < C; c += kWave) {
      const float v = x[c];
      if (v > mx || (v == mx && c < am)) { mx = v; am = c; }
    }
    // argmax: max value, then smallest index among ties (first max, like torch)
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(mx, o, kWave);
      const int oa = __shfl_xor(am, o, kWave);
      if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
    }
    float se = 0.f;
    for (int c = lane; c < C; c += kWave) se += __expf(x[c] - mx);
    se = wave_sum(se);
    const float lse = mx + __logf(se);
    if (y >= 0) {
      wl += lse - x[y];
      wc += (am == y) ? 1.f : 0.f;
    }
    if (dl) {
      uint16_t* d = dl + ((long long)g * B + b) * C;
      for (int c = lane; c < C; c += kWave) {
        float v = 0.f;
        if (y >= 0) v = (__expf(x[c] - lse) - (c == y ? 1.f : 0.f)) * scale;
        d[c] = f2bf(v);
      }
    }
  }
  if (lane == 0) { sl[wid] = wl; sc[wid] = wc; }
  __syncthreads();
  if (tid == 0) {
    const float L = sl[0] + sl[1] + sl[2] + sl[3];
    loss_out[g] = mean ? (n > 0 ? L / (float)n : 0.f) : L;
    corr_out[g] = sc[0] + sc[1] + sc[2] + sc[3];
  }
}

}  // namespace

DBA_EXPORT int dba_softmax_xent(const float* logits, const int* labels, int G, int B, int C, int mean, void* dl,
                                float* loss, float* correct, void* stream) {
  hipLaunchKernelGGL(xent_kernel, dim3(G), dim3(256), 0, (hipStream_t)stream, logits, labels, B, C, mean,
                     (uint16_t*)dl, loss, correct);
  DBA_LAUNCH_CHECK();
}
