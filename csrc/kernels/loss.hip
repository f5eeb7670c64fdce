// Fused softmax cross-entropy forward + backward + correct count, per group (K9).
// Replaces log_softmax/cross_entropy/argmax/eq/sum and the per-batch `.item()` host syncs
// of the reference (image_train.py:85,104-105; test.py:34-37): counters stay on device.
//
// One thread per row (C <= a few hundred classes: 10 CIFAR/MNIST, 200 Tiny, 9 LOAN): the
// row's max/argmax, log-sum-exp and gradient are thread-local loops, so a training step's
// 64-row batch costs one short pass instead of 16 serial wave-wide reductions per wave.
// Optionally accumulates the step's (loss, correct, valid rows) straight into the per-client
// per-internal-epoch statistics slots (train_result.csv rows), replacing the index-add
// kernels the trainer would otherwise launch after every step.
#include "common.hpp"

namespace {

template <typename T>
__global__ __launch_bounds__(256) void xent_kernel(const float* __restrict__ logits, const int* __restrict__ labels,
                                                   int B, int C, int mean, T* __restrict__ dl,
                                                   float* __restrict__ loss_out, double* __restrict__ loss64,
                                                   float* __restrict__ corr_out,
                                                   float* __restrict__ stats, long long stats_stride,
                                                   const int* __restrict__ slot, int max_slots,
                                                   const int* __restrict__ nvalid) {
  __shared__ double sl[4];
  __shared__ float sc[4];
  __shared__ int scnt[4];
  const int g = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int* lab = labels + (long long)g * B;
  int cnt = 0;
  for (int b = tid; b < B; b += 256) cnt += lab[b] >= 0;
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, kWave);
  if (lane == 0) scnt[wid] = cnt;
  __syncthreads();
  const int n = scnt[0] + scnt[1] + scnt[2] + scnt[3];
  const float scale = (mean && n > 0) ? 1.0f / (float)n : 1.0f;
  double wl = 0.0;    // per-row fp32 losses summed in fp64: independent of the row grouping
  float wc = 0.f;
  for (int b = tid; b < B; b += 256) {
    const float* x = logits + ((long long)g * B + b) * C;
    T* d = dl ? dl + ((long long)g * B + b) * C : nullptr;
    const int y = lab[b];
    if (y < 0) {
      if (d)
        for (int c = 0; c < C; ++c) d[c] = from_f<T>(0.f);
      continue;
    }
    // argmax = first maximum (torch semantics)
    float mx = x[0];
    int am = 0;
    for (int c = 1; c < C; ++c) {
      const float v = x[c];
      if (v > mx) { mx = v; am = c; }
    }
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += __expf(x[c] - mx);
    const float lse = mx + __logf(se);
    wl += (double)(lse - x[y]);
    wc += (am == y) ? 1.f : 0.f;
    if (d)
      for (int c = 0; c < C; ++c) d[c] = from_f<T>((__expf(x[c] - lse) - (c == y ? 1.f : 0.f)) * scale);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wl += __shfl_xor(wl, o, kWave);
  wc = wave_sum(wc);
  if (lane == 0) { sl[wid] = wl; sc[wid] = wc; }
  __syncthreads();
  if (tid == 0) {
    const double L = ((sl[0] + sl[1]) + sl[2]) + sl[3];
    const double l64 = mean ? (n > 0 ? L / (double)n : 0.0) : L;
    const float loss = (float)l64;
    if (loss64) loss64[g] = l64;
    const float corr = sc[0] + sc[1] + sc[2] + sc[3];
    loss_out[g] = loss;
    corr_out[g] = corr;
    if (stats) {
      const long long s = (long long)g * max_slots + slot[g];
      stats[s] += loss;
      stats[stats_stride + s] += corr;
      stats[2 * stats_stride + s] += (float)nvalid[g];
    }
  }
}

}  // namespace

// stats (optional): [3][stats_stride] fp32, slot [G] int, nvalid [G] int; dl fp32 (dl_f32) or bf16;
// loss64 (optional): the per-group loss unrounded (fp64; evaluation sums)
DBA_EXPORT int dba_softmax_xent(const float* logits, const int* labels, int G, int B, int C, int mean, void* dl,
                                float* loss, float* correct, float* stats, long long stats_stride, const int* slot,
                                int max_slots, const int* nvalid, int dl_f32, double* loss64, void* stream) {
  if (dl_f32)
    hipLaunchKernelGGL(xent_kernel<float>, dim3(G), dim3(256), 0, (hipStream_t)stream, logits, labels, B, C, mean,
                       (float*)dl, loss, loss64, correct, stats, stats_stride, slot, max_slots, nvalid);
  else
    hipLaunchKernelGGL(xent_kernel<uint16_t>, dim3(G), dim3(256), 0, (hipStream_t)stream, logits, labels, B, C, mean,
                       (uint16_t*)dl, loss, loss64, correct, stats, stats_stride, slot, max_slots, nvalid);
  DBA_LAUNCH_CHECK();
}
