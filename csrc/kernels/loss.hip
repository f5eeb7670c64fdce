// Fused softmax cross-entropy forward + backward + correct count, per group (K9).
// Replaces log_softmax/cross_entropy/argmax/eq/sum and the per-batch `.item()` host syncs
// of the reference (image_train.py:85,104-105; test.py:34-37): counters stay on device.
//
// A row belongs to a SEGMENT of L lanes (L = 16 up to 512 classes — Tiny-ImageNet's 200: 13
// per lane, 16 rows in flight per block — 64 beyond; heads of <= 16 classes — CIFAR / MNIST /
// LOAN — keep one thread per row, L = 1, where the segment shuffles cost more than the short
// serial loops): the lanes read the row's logits
// coalesced (class c on lane c % L), and max / argmax / sum-exp are fixed butterflies inside the
// segment, so a 256-thread block works on 256 / L rows at once.  (Round 1-5 form: one thread per
// row looping serially over C with row-strided reads — 92.6 us per 1024 x 200 evaluation chunk.)
//
// Large groups (evaluation chunks) are cut into 32-row slices, one block per (slice, group), so a
// launch fills the chip; each block writes its slice's (loss, correct) partial and a one-block-
// per-group finish launch sums the partials in slice order.  Training batches (<= 256 rows) are
// one slice: one launch, which also accumulates the step's (loss, correct, valid rows) straight
// into the per-client per-internal-epoch statistics slots (train_result.csv rows).
//
// Every order is fixed (segment butterflies, per-thread rows in order, a fixed block tree, slices
// in order) and depends on the group's own rows only: the bits do not depend on how many groups
// share the launch.
#include "common.hpp"

namespace {

constexpr int kXentThreads = 256;
constexpr int kXentSliceRows = 32;

template <int L>
__device__ __forceinline__ float seg_sum(float v) {
#pragma unroll
  for (int o = L / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// block-wide fixed-order sums of (fp64 loss, fp32 correct): waves' butterflies, then waves in order
__device__ __forceinline__ void xent_block_sum(double& wl, float& wc) {
  __shared__ double sl[kXentThreads / kWave];
  __shared__ float sc[kXentThreads / kWave];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wl += __shfl_xor(wl, o, kWave);
  wc = wave_sum(wc);
  if (lane == 0) { sl[wid] = wl; sc[wid] = wc; }
  __syncthreads();
  wl = ((sl[0] + sl[1]) + sl[2]) + sl[3];
  wc = ((sc[0] + sc[1]) + sc[2]) + sc[3];
}

__device__ __forceinline__ void xent_write(int g, double L, float corr, int n, int mean, float* loss_out,
                                           double* loss64, float* corr_out, float* stats, long long stats_stride,
                                           const int* slot, int max_slots, const int* nvalid) {
  const double l64 = mean ? (n > 0 ? L / (double)n : 0.0) : L;
  const float loss = (float)l64;
  if (loss64) loss64[g] = l64;
  loss_out[g] = loss;
  corr_out[g] = corr;
  if (stats) {
    const long long s = (long long)g * max_slots + slot[g];
    stats[s] += loss;
    stats[stats_stride + s] += corr;
    stats[2 * stats_stride + s] += (float)nvalid[g];
  }
}

// grid (slices, G); part [G][slices][2] fp64 when slices > 1
template <typename T, int L>
__global__ __launch_bounds__(kXentThreads) void xent_kernel(
    const float* __restrict__ logits, const int* __restrict__ labels, int B, int C, int mean, T* __restrict__ dl,
    float* __restrict__ loss_out, double* __restrict__ loss64, float* __restrict__ corr_out,
    float* __restrict__ stats, long long stats_stride, const int* __restrict__ slot, int max_slots,
    const int* __restrict__ nvalid, double* __restrict__ part) {
  const int g = blockIdx.y, S = gridDim.x;
  const int tid = threadIdx.x;
  const int* lab = labels + (long long)g * B;
  float scale = 1.0f;
  int n = 0;
  if (mean || S == 1) {
    // the group's valid rows (the mean's divisor): every block counts the whole group
    __shared__ int scnt[kXentThreads / kWave];
    int cnt = 0;
    for (int b = tid; b < B; b += kXentThreads) cnt += lab[b] >= 0;
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, kWave);
    if ((tid & 63) == 0) scnt[tid >> 6] = cnt;
    __syncthreads();
    n = scnt[0] + scnt[1] + scnt[2] + scnt[3];
    scale = (mean && n > 0) ? 1.0f / (float)n : 1.0f;
  }
  constexpr int kRows = kXentThreads / L;     // rows in flight per block
  const int seg = tid / L, sl = tid % L;
  const int r0 = S == 1 ? 0 : blockIdx.x * kXentSliceRows;
  const int r1 = S == 1 ? B : min(B, r0 + kXentSliceRows);
  double wl = 0.0;    // per-row fp32 losses summed in fp64 (segment leaders, rows in order)
  float wc = 0.f;
  for (int b = r0 + seg; b < r1; b += kRows) {
    const float* x = logits + ((long long)g * B + b) * C;
    T* d = dl ? dl + ((long long)g * B + b) * C : nullptr;
    const int y = lab[b];
    if (y < 0) {
      if (d)
        for (int c = sl; c < C; c += L) d[c] = from_f<T>(0.f);
      continue;
    }
    // argmax = first maximum (torch semantics): per lane in class order, then the smaller
    // index on ties across lanes
    float mx = -INFINITY;
    int am = C;
    for (int c = sl; c < C; c += L) {
      const float v = x[c];
      if (v > mx || am == C) { mx = v; am = c; }
    }
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) {
      const float om = __shfl_xor(mx, o, kWave);
      const int oa = __shfl_xor(am, o, kWave);
      if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
    }
    float se = 0.f;
    for (int c = sl; c < C; c += L) se += __expf(x[c] - mx);
    se = seg_sum<L>(se);
    const float lse = mx + __logf(se);
    if (sl == 0) {
      wl += (double)(lse - x[y]);
      wc += (am == y) ? 1.f : 0.f;
    }
    if (d)
      for (int c = sl; c < C; c += L) d[c] = from_f<T>((__expf(x[c] - lse) - (c == y ? 1.f : 0.f)) * scale);
  }
  xent_block_sum(wl, wc);
  if (tid != 0) return;
  if (S == 1) {
    xent_write(g, wl, wc, n, mean, loss_out, loss64, corr_out, stats, stats_stride, slot, max_slots, nvalid);
  } else {
    part[((long long)g * S + blockIdx.x) * 2] = wl;
    part[((long long)g * S + blockIdx.x) * 2 + 1] = (double)wc;
  }
}

// one block per group: the slice partials summed in slice order (fixed tree of the thread sums)
__global__ __launch_bounds__(kXentThreads) void xent_finish_kernel(
    const int* __restrict__ labels, int B, int S, int mean, const double* __restrict__ part,
    float* __restrict__ loss_out, double* __restrict__ loss64, float* __restrict__ corr_out,
    float* __restrict__ stats, long long stats_stride, const int* __restrict__ slot, int max_slots,
    const int* __restrict__ nvalid) {
  const int g = blockIdx.x, tid = threadIdx.x;
  __shared__ int scnt[kXentThreads / kWave];
  const int* lab = labels + (long long)g * B;
  int cnt = 0;
  for (int b = tid; b < B; b += kXentThreads) cnt += lab[b] >= 0;
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, kWave);
  if ((tid & 63) == 0) scnt[tid >> 6] = cnt;
  double wl = 0.0, wc = 0.0;
  for (int s = tid; s < S; s += kXentThreads) {
    wl += part[((long long)g * S + s) * 2];
    wc += part[((long long)g * S + s) * 2 + 1];
  }
  float wcf = (float)wc;   // slice counts are small integers: exact in fp32
  xent_block_sum(wl, wcf);
  if (tid != 0) return;
  const int n = scnt[0] + scnt[1] + scnt[2] + scnt[3];
  xent_write(g, wl, wcf, n, mean, loss_out, loss64, corr_out, stats, stats_stride, slot, max_slots, nvalid);
}

// the round-5 form (a thread per row, one block per group) for every shape: the A/B of the
// kernel bench (tools/bench_kernels xent rows); never set by the framework
int g_xent_r5 = 0;

template <typename T>
int xent_go(const float* logits, const int* labels, int G, int B, int C, int mean, T* dl, float* loss,
            double* loss64, float* correct, float* stats, long long stats_stride, const int* slot, int max_slots,
            const int* nvalid, double* part, hipStream_t st) {
  const int S = (B <= kXentThreads || part == nullptr || g_xent_r5) ? 1 : (B + kXentSliceRows - 1) / kXentSliceRows;
  const dim3 grid(S, G);
#define XENT_L(LL)                                                                                            \
  hipLaunchKernelGGL((xent_kernel<T, LL>), grid, dim3(kXentThreads), 0, st, logits, labels, B, C, mean, dl, loss, \
                     loss64, correct, stats, stats_stride, slot, max_slots, nvalid, part)
  // a thread per row for the 10-class heads (the segment shuffles cost more); 16-lane segments up
  // to 512 classes (Tiny's 200: 13 per lane, 16 rows in flight per block — 64-lane segments left
  // a 64-row group 16 serial passes: 41 vs 15 us for 10 x 64 x 200, tools/bench_kernels xent rows)
  if (C <= 16 || g_xent_r5) XENT_L(1);
  else if (C <= 512) XENT_L(16);
  else XENT_L(64);
#undef XENT_L
  if (S > 1)
    hipLaunchKernelGGL(xent_finish_kernel, dim3(G), dim3(kXentThreads), 0, st, labels, B, S, mean, part, loss,
                       loss64, correct, stats, stats_stride, slot, max_slots, nvalid);
  return (int)hipGetLastError();
}

}  // namespace

DBA_EXPORT int dba_xent_r5_set(int on) {
  const int prev = g_xent_r5;
  if (on >= 0) g_xent_r5 = on;
  return prev;
}

// doubles of the slice-partial workspace of a softmax_xent launch (0: one slice per group)
DBA_EXPORT long long dba_softmax_xent_part_doubles(int G, int B) {
  return B <= kXentThreads ? 0 : 2LL * G * ((B + kXentSliceRows - 1) / kXentSliceRows);
}

// stats (optional): [3][stats_stride] fp32, slot [G] int, nvalid [G] int; dl fp32 (dl_f32) or bf16;
// loss64 (optional): the per-group loss unrounded (fp64; evaluation sums); part: the
// dba_softmax_xent_part_doubles workspace (null: one slice per group, whatever B)
DBA_EXPORT int dba_softmax_xent(const float* logits, const int* labels, int G, int B, int C, int mean, void* dl,
                                float* loss, float* correct, float* stats, long long stats_stride, const int* slot,
                                int max_slots, const int* nvalid, int dl_f32, double* loss64, double* part,
                                void* stream) {
  if (G <= 0 || B <= 0 || C <= 0) return 0;
  if (dl_f32)
    return xent_go<float>(logits, labels, G, B, C, mean, (float*)dl, loss, loss64, correct, stats, stats_stride, slot,
                          max_slots, nvalid, part, (hipStream_t)stream);
  return xent_go<uint16_t>(logits, labels, G, B, C, mean, (uint16_t*)dl, loss, loss64, correct, stats, stats_stride,
                           slot, max_slots, nvalid, part, (hipStream_t)stream);
}

// ============================================================ fused classifier head (training)
// The CIFAR ResNets' head of a training step in TWO launches: global average pool of the last
// block output, the linear layer, softmax cross-entropy + correct count (+ the per-client
// statistics slots), and the head's backward — dlogits, the linear layer's bias and weight
// gradients and the gradient of the pooled features (the BN finish pass consumes it:
// xbn.hip bnx_tile_kernel's pooled mode).  Reference: models/resnet_cifar.py:97-100
// (avg_pool2d, view, linear) and image_train.py:85-92 (cross_entropy, backward).
// Replaces ~8 launches of a step (avgpool, the 1x1 linear conv, xent, two bias column sums,
// the FC weight gradient + its slab, the 1x1 data gradient, operand maxima).
//   head_rows_kernel  grid (row blocks of 4, replicas): pools its rows (every pixel load of a
//                     row issued at once), logits, cross-entropy, dlogits, the rows' pooled-
//                     feature gradient; writes pooled / dlogits rows and the block's (loss,
//                     correct) partial;
//   head_fin_kernel   grid (column blocks, replicas): the weight gradient (row quarters, then
//                     the quarters in a fixed order), the bias gradient, the partials in block
//                     order and the statistics slots.
// Arithmetic: the pool is avgpool_kernel's (channel sums in pixel order, / HW); every dot
// product is an exact-fp32 FMA chain in a fixed order (4 lanes x strided quarters for the
// logits, then a fixed butterfly; 4 row quarters for the weight gradient): fp32-level, deterministic, and
// a replica's bits depend on its own rows only.  K <= 16 classes, C <= 512 features, N <= 256
// rows, HW <= 64 pixels (checked on the host).  (A one-launch form with one block per replica
// was slower than the unfused ops: its pooling pass is one CU streaming the replica's whole
// last activation.)
namespace {

constexpr int kHeadK = 16, kHeadRows = 4, kHeadHW = 64;

__global__ __launch_bounds__(256) void head_rows_kernel(
    const float* __restrict__ feat, long long f_gstride, int N, int HW, int C, const float* __restrict__ W,
    long long w_sstride, const float* __restrict__ bias, long long b_sstride, int K, const int* __restrict__ labels,
    const int* __restrict__ nvalid, float* __restrict__ pooled, float* __restrict__ dlog, float* __restrict__ dpool,
    double* __restrict__ part, int mean) {
  __shared__ __attribute__((aligned(16))) float pl[kHeadRows * 512];   // the block's pooled rows
  __shared__ float lg[kHeadRows * kHeadK];                             // logits, then dlogits
  const int g = blockIdx.y, nb = gridDim.x, tid = threadIdx.x;
  const int nv = valid_rows(nvalid, g, N);
  const int r0 = blockIdx.x * kHeadRows, nr = max(0, min(kHeadRows, nv - r0));
  const int* lab = labels + (long long)g * N;
  const float* fg = feat + (long long)g * f_gstride;
  const float* Wg = W + (long long)g * w_sstride;
  // 1. pooled[n][c] = (sum over pixels in order) / HW: a thread's (row, 4-channel) item, all its
  //    pixel loads issued before the adds
  const int C4 = C >> 2;
  for (int e = tid; e < nr * C4; e += 256) {
    const int n = e / C4, c = (e - n * C4) * 4;
    const float* src = fg + (long long)(r0 + n) * HW * C + c;
    float4 v[kHeadHW / 4];
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i0 = 0; i0 < HW; i0 += kHeadHW / 4) {
#pragma unroll
      for (int i = 0; i < kHeadHW / 4; ++i)
        if (i0 + i < HW) v[i] = *(const float4*)(src + (long long)(i0 + i) * C);
#pragma unroll
      for (int i = 0; i < kHeadHW / 4; ++i)
        if (i0 + i < HW) { s.x += v[i].x; s.y += v[i].y; s.z += v[i].z; s.w += v[i].w; }
    }
    const float hw = (float)HW;
    const float4 p = make_float4(s.x / hw, s.y / hw, s.z / hw, s.w / hw);
    *(float4*)&pl[n * C + c] = p;
    *(float4*)(pooled + ((long long)g * N + r0 + n) * C + c) = p;
  }
  // the replica's valid labels (the mean's divisor)
  __shared__ int scnt[4];
  int cnt = 0;
  for (int b = tid; b < N; b += 256) cnt += lab[b] >= 0;
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, kWave);
  if ((tid & 63) == 0) scnt[tid >> 6] = cnt;
  __syncthreads();
  const int ncnt = scnt[0] + scnt[1] + scnt[2] + scnt[3];
  // 2. logits: 4 lanes per (row, class), quarter q sums c = q, q + 4, ... (FMA chain), then the
  //    butterfly (q0 + q1) + (q2 + q3), then + bias
  {
    const int p = tid >> 2, q = tid & 3;
    const bool live = p < nr * K;
    const int n = live ? p / K : 0, k = live ? p - n * K : 0;
    float s = 0.f;
    if (live) {
#pragma unroll 8
      for (int c = q; c < C; c += 4) s = fmaf(pl[n * C + c], Wg[k * C + c], s);
    }
    s += __shfl_xor(s, 1, kWave);
    s += __shfl_xor(s, 2, kWave);
    if (live && q == 0) lg[n * kHeadK + k] = s + bias[(long long)g * b_sstride + k];
  }
  static_assert(kHeadRows * kHeadK * 4 <= 256, "one pass of 4-lane groups");
  __syncthreads();
  // 3. softmax cross-entropy per row (xent_kernel's arithmetic, L = 1), dlogits into lg
  const float scale = (mean && ncnt > 0) ? 1.0f / (float)ncnt : 1.0f;
  double wl = 0.0;
  float wc = 0.f;
  if (tid < nr) {
    float* x = lg + tid * kHeadK;
    const int y = lab[r0 + tid];
    if (y < 0) {
      for (int c = 0; c < K; ++c) x[c] = 0.f;
    } else {
      float mx = x[0];
      int am = 0;
      for (int c = 1; c < K; ++c)
        if (x[c] > mx) { mx = x[c]; am = c; }
      float se = 0.f;
      for (int c = 0; c < K; ++c) se += __expf(x[c] - mx);
      const float lse = mx + __logf(se);
      wl = (double)(lse - x[y]);
      wc = (am == y) ? 1.f : 0.f;
      for (int c = 0; c < K; ++c) x[c] = (__expf(x[c] - lse) - (c == y ? 1.f : 0.f)) * scale;
    }
    for (int c = 0; c < K; ++c) dlog[((long long)g * N + r0 + tid) * kHeadK + c] = x[c];
  }
  xent_block_sum(wl, wc);   // (its barriers also publish the dlogits)
  if (tid == 0) {
    part[((long long)g * nb + blockIdx.x) * 2] = wl;
    part[((long long)g * nb + blockIdx.x) * 2 + 1] = (double)wc;
  }
  // 4. the rows' pooled-feature gradient: dpool[n][c] = sum_k dl[n][k] W[k][c] (classes in order)
  for (int e = tid; e < nr * C; e += 256) {
    const int n = e / C, c = e - n * C;
    float s = 0.f;
    for (int k = 0; k < K; ++k) s = fmaf(lg[n * kHeadK + k], Wg[k * C + c], s);
    dpool[((long long)g * N + r0 + n) * C + c] = s;
  }
}

// grid (column blocks of 64, replicas): the weight gradient dW[k][c] = sum over the valid rows
// of dl[n][k] pooled[n][c] — a wave per row quarter (rows q, q + 4, ...; FMA chains), the
// quarters added (q0 + q1) + (q2 + q3); column block 0 also the bias gradient (rows in order),
// (loss, correct) from the row blocks' partials in block order and the statistics slots
__global__ __launch_bounds__(256) void head_fin_kernel(
    int N, int C, int K, const int* __restrict__ labels, const int* __restrict__ nvalid,
    const float* __restrict__ pooled, const float* __restrict__ dlog, const double* __restrict__ part, int nb,
    float* __restrict__ dW, long long dw_gstride, float* __restrict__ db, long long db_gstride,
    float* __restrict__ loss_out, float* __restrict__ corr_out, float* __restrict__ stats, long long stats_stride,
    const int* __restrict__ slot, int max_slots, int mean) {
  const int g = blockIdx.y, tid = threadIdx.x;
  const int nv = valid_rows(nvalid, g, N);
  if (blockIdx.x == 0) {
    const int* lab = labels + (long long)g * N;
    __shared__ int scnt[4];
    int cnt = 0;
    for (int b = tid; b < N; b += 256) cnt += lab[b] >= 0;
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, kWave);
    if ((tid & 63) == 0) scnt[tid >> 6] = cnt;
    double wl = 0.0, wc = 0.0;
    for (int s = tid; s < nb; s += 256) {
      wl += part[((long long)g * nb + s) * 2];
      wc += part[((long long)g * nb + s) * 2 + 1];
    }
    float wcf = (float)wc;
    xent_block_sum(wl, wcf);
    if (tid == 0)
      xent_write(g, wl, wcf, scnt[0] + scnt[1] + scnt[2] + scnt[3], mean, loss_out, nullptr, corr_out, stats,
                 stats_stride, slot, max_slots, nvalid);
    if (nv > 0 && tid < K) {   // rows in order, 16 loads in flight per trip
      const float* dl = dlog + (long long)g * N * kHeadK;
      float s = 0.f;
      for (int n0 = 0; n0 < nv; n0 += 16) {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = n0 + r < nv ? dl[(n0 + r) * kHeadK + tid] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (n0 + r < nv) s += v[r];
      }
      db[(long long)g * db_gstride + tid] = s;
    }
  }
  if (nv == 0) return;   // an inactive replica: no gradients written
  __shared__ float sq[3][kHeadK][64];
  const float* dl = dlog + (long long)g * N * kHeadK;
  const float* pg = pooled + (long long)g * N * C;
  const int q = tid >> 6, c = blockIdx.x * 64 + (tid & 63);
  const bool live = c < C;
  float s[kHeadK];
#pragma unroll
  for (int k = 0; k < kHeadK; ++k) s[k] = 0.f;
  for (int n0 = q; n0 < nv; n0 += 16) {   // 4 of the quarter's rows per trip, loads first
    float p[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + 4 * r;
      p[r] = (live && n < nv) ? pg[(long long)n * C + c] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + 4 * r;
      if (n < nv) {
#pragma unroll
        for (int k = 0; k < kHeadK; ++k)
          if (k < K) s[k] = fmaf(dl[n * kHeadK + k], p[r], s[k]);
      }
    }
  }
  if (q > 0) {
#pragma unroll
    for (int k = 0; k < kHeadK; ++k) sq[q - 1][k][tid & 63] = s[k];
  }
  __syncthreads();
  if (q == 0 && live) {
#pragma unroll
    for (int k = 0; k < kHeadK; ++k)
      if (k < K)
        dW[(long long)g * dw_gstride + k * C + c] =
            (s[k] + sq[0][k][tid]) + (sq[1][k][tid] + sq[2][k][tid]);
  }
}

}  // namespace

// workspace doubles of dba_head_train (the row blocks' loss partials)
DBA_EXPORT long long dba_head_part_doubles(int G, int N) {
  return 2LL * G * ((N + kHeadRows - 1) / kHeadRows);
}

// feat [G][N][H][W][C] (replica stride f_gstride) fp32, W / bias the replicas' rows [G][K][C] /
// [G][K] (strides), labels [G][N] int (< 0: padding), nvalid [G]; pooled / dpool [G][N][C] fp32,
// dlog [G][N][16] fp32 and part (dba_head_part_doubles) workspaces / outputs; dW [G][K][C],
// db [G][K] (strides) overwritten for active replicas.
DBA_EXPORT int dba_head_train(const float* feat, long long f_gstride, int G, int N, int HW, int C, const float* W,
                              long long w_sstride, const float* bias, long long b_sstride, int K, const int* labels,
                              const int* nvalid, float* pooled, float* dlog, double* part, float* dW,
                              long long dw_gstride, float* db, long long db_gstride, float* dpool, float* loss,
                              float* correct, float* stats, long long stats_stride, const int* slot, int max_slots,
                              int mean, void* stream) {
  if (K < 1 || K > kHeadK || C > 512 || (C & 3) || N > 256 || HW > kHeadHW || HW < 1 ||
      (((uintptr_t)feat | (uintptr_t)pooled | (uintptr_t)dpool) & 15) || (f_gstride & 3))
    return -100;
  const int nb = (N + kHeadRows - 1) / kHeadRows;
  hipLaunchKernelGGL(head_rows_kernel, dim3(nb, G), dim3(256), 0, (hipStream_t)stream, feat, f_gstride, N, HW, C, W,
                     w_sstride, bias, b_sstride, K, labels, nvalid, pooled, dlog, dpool, part, mean);
  hipLaunchKernelGGL(head_fin_kernel, dim3((C + 63) / 64, G), dim3(256), 0, (hipStream_t)stream, N, C, K, labels, nvalid, pooled,
                     dlog, part, nb, dW, dw_gstride, db, db_gstride, loss, correct, stats, stats_stride, slot,
                     max_slots, mean);
  DBA_LAUNCH_CHECK();
}
