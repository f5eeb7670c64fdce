// Training-mode BatchNorm for grouped NHWC activations and the
// eval-mode BN fold into the preceding conv.
//
//   stats   : per-(group, channel) sum / sum-of-squares over the group's VALID rows
//             (fp32 per-block partials, no atomics and no pre-zeroed buffers; the finalize
//             pass sums them in fp64);
//   finalize: mean, 1/std, running-stat update (unbiased var, momentum) in place in the
//             flat replica state;
//   apply   : y -> (y-mean)*invstd*gamma + beta (+residual) (ReLU) over the valid rows only;
//   backward: one fused reduce (sum d, sum d*xhat with the ReLU mask recomputed from the
//             forward output) + one fused apply that also emits the residual-branch grad.
#include "common.hpp"
#include <algorithm>
#include <cstdlib>

namespace {

// Rows per reduction block: ~16K elements per block (8 passes of 256 threads x 8 channels),
// so narrow-spatial / wide-channel layers (ResNet stage 4: 16 px x 256 ch) still launch
// enough blocks to cover the chip instead of 2 per replica.
__host__ __device__ inline int rows_per_block(int C) {
  const int rpp = 256 / (C / 8);
  const int r = 16384 / C;
  return r > rpp ? r : rpp;
}

// Per-block partial sums (no atomics, no pre-zeroing): part[g][blk][0][c] = sum x (STATS)
// or sum d (BWD); part[g][blk][1][c] = sum x^2 or sum d*xhat.  Blocks past the valid rows
// write zeros so the finalize pass can sum every slot unconditionally.
// Last-block finalize (fin != nullptr): the blocks holding valid rows count their arrival on
// the replica's zeroed counter; the last one sums the replica's partials (fixed order, fp64)
// and finalises in the same launch — one launch per BN pass instead of reduce + finalize.
struct BnFin {
  int* counter;                                   // [G] zeroed (per-step arena)
  // forward: running stats and batch statistics
  float* rm; float* rv; long long s_gstride; float momentum, eps; float* mean_out; float* invstd_out;
  // backward: sums [G][2][C], dgamma / dbeta accumulation
  float* sums; float* dgamma; float* dbeta; long long g_gstride;
};

template <bool BWD>
__device__ void bn_last_block(const float* __restrict__ part, int nblk_grid, int nvb, int g, int C, double n,
                              const BnFin& f) {
  __shared__ double fr[2][256];
  const int tid = threadIdx.x;
  const int tpc = C >= 256 ? 1 : 256 / C;         // threads per channel
  const float* pg = part + (long long)g * nblk_grid * 2 * C;
  for (int c0 = 0; c0 < C; c0 += 256 / tpc) {
    const int c = c0 + tid / tpc, q = tid % tpc;
    double a0 = 0.0, a1 = 0.0;
    if (c < C) {
#pragma unroll 4
      for (int b = q; b < nvb; b += tpc) {
        a0 += (double)pg[(long long)b * 2 * C + c];
        a1 += (double)pg[(long long)b * 2 * C + C + c];
      }
    }
    fr[0][tid] = a0;
    fr[1][tid] = a1;
    __syncthreads();
    if (q == 0 && c < C) {
      double s0 = 0.0, s1 = 0.0;
      for (int k = 0; k < tpc; ++k) { s0 += fr[0][tid + k]; s1 += fr[1][tid + k]; }
      if (!BWD) {
        const int i = g * C + c;
        const double m = s0 / n;
        double var = s1 / n - m * m;
        var = var > 0 ? var : 0;
        f.mean_out[i] = (float)m;
        f.invstd_out[i] = (float)(1.0 / sqrt(var + (double)f.eps));
        float* prm = f.rm + (long long)g * f.s_gstride + c;
        float* prv = f.rv + (long long)g * f.s_gstride + c;
        const double unb = n > 1 ? var * n / (n - 1) : var;
        *prm = (float)((1.0 - f.momentum) * (*prm) + f.momentum * m);
        *prv = (float)((1.0 - f.momentum) * (*prv) + f.momentum * unb);
      } else {
        f.sums[((long long)g * 2) * C + c] = (float)s0;
        f.sums[((long long)g * 2 + 1) * C + c] = (float)s1;
        f.dbeta[(long long)g * f.g_gstride + c] += (float)s0;
        f.dgamma[(long long)g * f.g_gstride + c] += (float)s1;
      }
    }
    __syncthreads();
  }
}

template <bool BWD, typename T>
__global__ __launch_bounds__(256) void bn_reduce_kernel(const T* __restrict__ y, const T* __restrict__ dout,
                                                        const T* __restrict__ out, const float* __restrict__ mean,
                                                        const float* __restrict__ invstd, int relu,
                                                        const int* __restrict__ nvalid, int N, int HW, int C,
                                                        float* __restrict__ part, const BnFin fin) {
  __shared__ float red[2][256][8];
  __shared__ int last;
  const int g = blockIdx.y;
  const int R = N * HW;
  const int Rv = valid_rows(nvalid, g, N) * HW;
  const int rpb = rows_per_block(C);
  const int r0 = blockIdx.x * rpb;
  const int tid = threadIdx.x;
  float* pg = part + ((long long)g * gridDim.x + blockIdx.x) * 2 * C;
  if (r0 >= Rv) {
    if (fin.counter) {
      // no valid row in this block: with fin only the valid blocks' partials are summed; an
      // inactive replica's statistics are zeroed by its block 0 (forward)
      if (!BWD && Rv == 0 && blockIdx.x == 0)
        for (int c = tid; c < C; c += 256) { fin.mean_out[g * C + c] = 0.f; fin.invstd_out[g * C + c] = 0.f; }
      return;
    }
    for (int c = tid; c < 2 * C; c += 256) pg[c] = 0.f;
    return;
  }
  const int r1 = min(Rv, r0 + rpb);
  const int tpr = C / 8;                 // threads per row
  const int rpp = 256 / tpr;             // rows per pass
  const int cg = tid % tpr, rr = tid / tpr;
  float s0[8], s1[8], mu[8], is[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s0[e] = 0.f; s1[e] = 0.f; }
  if (BWD) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { mu[e] = mean[g * C + cg * 8 + e]; is[e] = invstd[g * C + cg * 8 + e]; }
  }
  const long long gbase = (long long)g * R * C;
  for (int r = r0 + rr; r < r1; r += rpp) {
    const long long o = gbase + (long long)r * C + cg * 8;
    float yp[8];
    ld8(y + o, yp);
    if (!BWD) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float v = yp[e]; s0[e] += v; s1[e] += v * v; }
    } else {
      float dp[8], op[8];
      ld8(dout + o, dp);
      if (relu) ld8(out + o, op);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float d = dp[e];
        if (relu && !(op[e] > 0.f)) d = 0.f;
        const float xh = (yp[e] - mu[e]) * is[e];
        s0[e] += d; s1[e] += d * xh;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][tid][e] = s0[e]; red[1][tid][e] = s1[e]; }
  __syncthreads();
  if (tid < tpr) {
    for (int k = 1; k < rpp; ++k) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { s0[e] += red[0][tid + k * tpr][e]; s1[e] += red[1][tid + k * tpr][e]; }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      pg[tid * 8 + e] = s0[e];
      pg[C + tid * 8 + e] = s1[e];
    }
  }
  if (!fin.counter) return;
  const int nvb = (Rv + rpb - 1) / rpb;   // blocks with valid rows (this replica)
  __threadfence();                          // partials visible device-wide before the arrival
  __syncthreads();
  if (tid == 0) last = atomicAdd(fin.counter + g, 1) == nvb - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  bn_last_block<BWD>(part, gridDim.x, nvb, g, C, (double)Rv, fin);
}

// sums the nblk partials of (g, c): a block covers cpb = min(64, C) channels with 256 / cpb
// threads per channel (all 256 threads busy for narrow layers), two independent fp64 chains
// per thread, then an LDS reduction.  Returns with threadIdx.x < cpb holding the totals.
__device__ __forceinline__ int bn_cpb(int C) { return C < 64 ? C : 64; }

__device__ __forceinline__ void sum_partials(const float* __restrict__ part, int nblk, int C, int g, int c, bool cok,
                                             double& s0, double& s1) {
  __shared__ double red[2][256];
  const int cpb = bn_cpb(C), tpc = 256 / cpb;
  const int q = threadIdx.x / cpb;
  double a0 = 0, a1 = 0, b0 = 0, b1 = 0;
  if (cok && q < tpc) {
    const float* pg = part + (long long)g * nblk * 2 * C + c;
    int b = q;
    for (; b + tpc < nblk; b += 2 * tpc) {
      a0 += pg[(long long)b * 2 * C];
      a1 += pg[(long long)b * 2 * C + C];
      b0 += pg[(long long)(b + tpc) * 2 * C];
      b1 += pg[(long long)(b + tpc) * 2 * C + C];
    }
    if (b < nblk) { a0 += pg[(long long)b * 2 * C]; a1 += pg[(long long)b * 2 * C + C]; }
  }
  red[0][threadIdx.x] = a0 + b0;
  red[1][threadIdx.x] = a1 + b1;
  __syncthreads();
  s0 = 0; s1 = 0;
  if ((int)threadIdx.x < cpb) {
    for (int k = 0; k < tpc; ++k) { s0 += red[0][k * cpb + threadIdx.x]; s1 += red[1][k * cpb + threadIdx.x]; }
  }
}

__global__ void bn_finalize_kernel(const float* __restrict__ part, int nblk, const int* __restrict__ nvalid, int N,
                                   int HW, int C, float* __restrict__ rm, float* __restrict__ rv, long long s_gstride,
                                   float momentum, float eps, float* __restrict__ mean, float* __restrict__ invstd,
                                   int G) {
  const int g = blockIdx.y;
  const int cpb = bn_cpb(C);
  const int c = blockIdx.x * cpb + (int)(threadIdx.x % cpb);
  double s0, s1;
  sum_partials(part, nblk, C, g, c, c < C, s0, s1);
  if ((int)threadIdx.x >= cpb || c >= C) return;
  const int i = g * C + c;
  const double n = (double)valid_rows(nvalid, g, N) * HW;
  if (n <= 0) { mean[i] = 0.f; invstd[i] = 0.f; return; }
  const double m = s0 / n;
  double var = s1 / n - m * m;
  var = var > 0 ? var : 0;
  mean[i] = (float)m;
  invstd[i] = (float)(1.0 / sqrt(var + (double)eps));
  float* prm = rm + (long long)g * s_gstride + c;
  float* prv = rv + (long long)g * s_gstride + c;
  const double unb = n > 1 ? var * n / (n - 1) : var;
  *prm = (float)((1.0 - momentum) * (*prm) + momentum * m);
  *prv = (float)((1.0 - momentum) * (*prv) + momentum * unb);
}

// finalize from the conv-epilogue partials (xgemm.hip bn_tile_stats): part[g][c][2][nblk] fp64,
// one block per (channel, replica), every thread sums a fixed stride of 32-row groups in
// fp64, then a fixed LDS tree — the order depends on nblk only.
__global__ __launch_bounds__(256) void bn_finalize_part_kernel(const double* __restrict__ part, int nblk,
                                                               const int* __restrict__ nvalid, int N, int HW, int C,
                                                               float* __restrict__ rm, float* __restrict__ rv,
                                                               long long s_gstride, float momentum, float eps,
                                                               float* __restrict__ mean, float* __restrict__ invstd) {
  __shared__ double red[2][256];
  const int c = blockIdx.x, g = blockIdx.y, tid = threadIdx.x;
  const double* __restrict__ p = part + ((long long)g * C + c) * 2 * nblk;
  double a0 = 0, a1 = 0;
#pragma unroll 4
  for (int b = tid; b < nblk; b += 256) {
    a0 += p[b];
    a1 += p[nblk + b];
  }
  red[0][tid] = a0;
  red[1][tid] = a1;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) {
      red[0][tid] += red[0][tid + w];
      red[1][tid] += red[1][tid + w];
    }
    __syncthreads();
  }
  if (tid != 0) return;
  const int i = g * C + c;
  const double n = (double)valid_rows(nvalid, g, N) * HW;
  if (n <= 0) { mean[i] = 0.f; invstd[i] = 0.f; return; }
  const double m = red[0][0] / n;
  double var = red[1][0] / n - m * m;
  var = var > 0 ? var : 0;
  mean[i] = (float)m;
  invstd[i] = (float)(1.0 / sqrt(var + (double)eps));
  float* prm = rm + (long long)g * s_gstride + c;
  float* prv = rv + (long long)g * s_gstride + c;
  const double unb = n > 1 ? var * n / (n - 1) : var;
  *prm = (float)((1.0 - momentum) * (*prm) + momentum * m);
  *prv = (float)((1.0 - momentum) * (*prv) + momentum * unb);
}

// Elementwise passes: 256 % (C/8) == 0, so every thread of the grid-stride loop always owns
// the same 8 channels; their per-(replica, channel) coefficients are loaded once per replica
// change instead of 4-7 scalar loads per element.
template <typename T>
__global__ void bn_apply_kernel(const T* __restrict__ y, const float* __restrict__ mean,
                                const float* __restrict__ invstd, const float* __restrict__ gamma,
                                const float* __restrict__ beta, long long p_gstride, const T* __restrict__ res,
                                int relu, T* __restrict__ out, const int* __restrict__ nvalid, int G, int N,
                                int HW, int C, int* __restrict__ amax, int amax_ld) {
  // grid (blocks, G): only the replica's VALID rows are touched (inactive replicas exit at
  // once; padded rows are never read downstream — every consumer gates on nvalid)
  const int g = blockIdx.y;
  const int c8 = C / 8;
  const int total = valid_rows(nvalid, g, N) * HW * c8;
  const int tid0 = blockIdx.x * blockDim.x + threadIdx.x;
  if ((int)(blockIdx.x * blockDim.x) >= total) return;   // whole block idle (block-uniform)
  const int c0 = (tid0 % c8) * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = c0 + e;
    sc[e] = invstd[g * C + c] * gamma[(long long)g * p_gstride + c];
    sh[e] = beta[(long long)g * p_gstride + c] - mean[g * C + c] * sc[e];
  }
  const long long base = (long long)g * N * HW * c8;
  float vmax = 0.f;
  for (int t = tid0; t < total; t += gridDim.x * blockDim.x) {
    const long long o = (base + t) * 8;
    float yp[8], rp[8], op[8];
    ld8(y + o, yp);
    if (res) ld8(res + o, rp);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = fmaf(yp[e], sc[e], sh[e]);
      if (res) v += rp[e];
      if (relu) v = fmaxf(v, 0.f);
      op[e] = v;
      vmax = fmaxf(vmax, fabsf(v));
    }
    st8(out + o, op);
  }
  if (amax) amax_fold(amax, amax_ld, g, vmax);
}

// dy = gamma*is/n * (n*d - sum d - xhat * sum d*xhat) = A*d + B*y + K per (replica, channel)
template <typename T>
__global__ void bn_bwd_apply_kernel(const T* __restrict__ dout, const T* __restrict__ out,
                                    const T* __restrict__ y, const float* __restrict__ mean,
                                    const float* __restrict__ invstd, const float* __restrict__ gamma,
                                    long long p_gstride, const float* __restrict__ sums, int relu,
                                    T* __restrict__ dy, T* __restrict__ dres,
                                    const int* __restrict__ nvalid, int G, int N, int HW, int C,
                                    int* __restrict__ amax, int amax_ld) {
  const int g = blockIdx.y;
  const int c8 = C / 8;
  const int nv = valid_rows(nvalid, g, N) * HW;
  const int total = nv * c8;
  const int tid0 = blockIdx.x * blockDim.x + threadIdx.x;
  if ((int)(blockIdx.x * blockDim.x) >= total) return;   // whole block idle (block-uniform)
  const int c0 = (tid0 % c8) * 8;
  const float n = (float)nv;
  float A[8], B[8], K[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = c0 + e;
    const float is = invstd[g * C + c];
    const float ga = gamma[(long long)g * p_gstride + c] * is;
    const float sd = sums[((long long)g * 2) * C + c];
    const float sdx = sums[((long long)g * 2 + 1) * C + c];
    A[e] = ga;
    B[e] = -ga * is * sdx / n;
    K[e] = -ga * sd / n - B[e] * mean[g * C + c];
  }
  const long long base = (long long)g * N * HW * c8;
  float vmax = 0.f;
  for (int t = tid0; t < total; t += gridDim.x * blockDim.x) {
    const long long o = (base + t) * 8;
    float dp[8], yp[8], op[8], p1[8];
    ld8(dout + o, dp);
    ld8(y + o, yp);
    if (relu) ld8(out + o, op);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (relu && !(op[e] > 0.f)) dp[e] = 0.f;
      p1[e] = fmaf(A[e], dp[e], fmaf(B[e], yp[e], K[e]));
      vmax = fmaxf(vmax, fabsf(p1[e]));
    }
    st8(dy + o, p1);
    if (dres) st8(dres + o, dp);
  }
  if (amax) amax_fold(amax, amax_ld, g, vmax);
}

// sums the backward partials into sums[g][2][C] and accumulates dgamma / dbeta
__global__ void bn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, float* __restrict__ sums,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta, long long g_gstride,
                                       int G, int C) {
  const int g = blockIdx.y;
  const int cpb = bn_cpb(C);
  const int c = blockIdx.x * cpb + (int)(threadIdx.x % cpb);
  double s0, s1;
  sum_partials(part, nblk, C, g, c, c < C, s0, s1);
  if ((int)threadIdx.x >= cpb || c >= C) return;
  sums[((long long)g * 2) * C + c] = (float)s0;
  sums[((long long)g * 2 + 1) * C + c] = (float)s1;
  dbeta[(long long)g * g_gstride + c] += (float)s0;
  dgamma[(long long)g * g_gstride + c] += (float)s1;
}


// Backward apply with the finalize folded in, for small launches (a lone client's grouped
// step, where the separate finalize launch is ~5 us of latency for a few KB of work): every
// block first sums its replica's reduce partials for ALL channels itself — sum_partials, the
// finalize's exact fixed order, rounded to fp32 like the finalize's stored sums — so the
// coefficients, and every output bit, equal the reduce / finalize / apply path; block 0 alone
// accumulates dgamma / dbeta.  The partials are 2 * C * nblk = 8192 fp32 per replica for every
// ResNet stage (rows_per_block), L2-resident after the first block of an XCD reads them; the
// grid is capped (grid-stride rows) so few blocks repeat the sum.
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_fin_kernel(
    const T* __restrict__ dout, const T* __restrict__ out, const T* __restrict__ y, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma, long long p_gstride,
    const float* __restrict__ part, int nblk, float* __restrict__ dgamma, float* __restrict__ dbeta,
    long long g_gstride, int relu, T* __restrict__ dy, T* __restrict__ dres, const int* __restrict__ nvalid, int N,
    int HW, int C, int* __restrict__ amax, int amax_ld) {
  __shared__ float sums[2][2048];              // C <= 2048 (bn_layout_ok)
  const int g = blockIdx.y;
  const int c8 = C / 8;
  const int nv = valid_rows(nvalid, g, N) * HW;
  const int total = nv * c8;
  if (blockIdx.x != 0 && (int)(blockIdx.x * blockDim.x) >= total) return;   // block-uniform
  const int cpb = bn_cpb(C);
  for (int cb = 0; cb < C; cb += cpb) {
    const int c = cb + (int)(threadIdx.x % cpb);
    double s0, s1;
    sum_partials(part, nblk, C, g, c, c < C, s0, s1);
    if ((int)threadIdx.x < cpb && c < C) {
      sums[0][c] = (float)s0;
      sums[1][c] = (float)s1;
      if (blockIdx.x == 0) {
        dbeta[(long long)g * g_gstride + c] += (float)s0;
        dgamma[(long long)g * g_gstride + c] += (float)s1;
      }
    }
    __syncthreads();   // sum_partials' LDS is reused by the next channel group
  }
  const int tid0 = blockIdx.x * blockDim.x + threadIdx.x;
  if ((int)(blockIdx.x * blockDim.x) >= total) return;
  const int c0 = (tid0 % c8) * 8;
  const float n = (float)nv;
  float A[8], B[8], K[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = c0 + e;
    const float is = invstd[g * C + c];
    const float ga = gamma[(long long)g * p_gstride + c] * is;
    const float sd = sums[0][c];
    const float sdx = sums[1][c];
    A[e] = ga;
    B[e] = -ga * is * sdx / n;
    K[e] = -ga * sd / n - B[e] * mean[g * C + c];
  }
  const long long base = (long long)g * N * HW * c8;
  float vmax = 0.f;
  for (int t = tid0; t < total; t += gridDim.x * blockDim.x) {
    const long long o = (base + t) * 8;
    float dp[8], yp[8], op[8], p1[8];
    ld8(dout + o, dp);
    ld8(y + o, yp);
    if (relu) ld8(out + o, op);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (relu && !(op[e] > 0.f)) dp[e] = 0.f;
      p1[e] = fmaf(A[e], dp[e], fmaf(B[e], yp[e], K[e]));
      vmax = fmaxf(vmax, fabsf(p1[e]));
    }
    st8(dy + o, p1);
    if (dres) st8(dres + o, dp);
  }
  if (amax) amax_fold(amax, amax_ld, g, vmax);
}

// ---------------------------------------------------------------- narrow-spatial layers
// One block owns 8 channels of one replica for ALL of its valid rows (<= 16K rows: ResNet
// stages 2-4 at batch 64), so statistics, finalize (running stats), and apply — or the
// whole backward — run in ONE launch with no cross-block synchronisation.  Replaces the
// reduce / finalize / apply chain (3 launches) where the per-launch latency, not the bytes,
// sets the cost (a lone attacker's grouped step).
__device__ __forceinline__ void block_sum16(float (&a)[8], float (&b)[8], float (*red)[4][8]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    a[e] = wave_sum(a[e]);
    b[e] = wave_sum(b[e]);
  }
  if (lane == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { red[0][w][e] = a[e]; red[1][w][e] = b[e]; }
  }
  __syncthreads();
}

template <typename T>
__global__ __launch_bounds__(256) void bn_small_fwd_kernel(
    const T* __restrict__ y, const int* __restrict__ nvalid, int N, int HW, int C,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ rm, float* __restrict__ rv,
    long long p_gstride, float momentum, float eps, const T* __restrict__ res, int relu,
    T* __restrict__ out, float* __restrict__ mean, float* __restrict__ invstd, int* __restrict__ amax,
    int amax_ld) {
  __shared__ float red[2][4][8];
  __shared__ float coef[2][8];
  const int g = blockIdx.y, c0 = blockIdx.x * 8, tid = threadIdx.x;
  const int R = valid_rows(nvalid, g, N) * HW;
  if (R == 0) {
    if (tid < 8) { mean[g * C + c0 + tid] = 0.f; invstd[g * C + c0 + tid] = 0.f; }
    return;
  }
  const long long base = (long long)g * N * HW * C + c0;
  float s0[8], s1[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s0[e] = 0.f; s1[e] = 0.f; }
  // R <= 4 * 256 (the single-launch threshold): the thread's rows are loaded once, all in
  // flight together, and kept in registers for the apply pass (same summation order)
  constexpr int RPT = 4;
  const bool cached = R <= RPT * 256;
  float yc[RPT][8];
  if (cached) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int r = tid + k * 256;
      if (r < R) ld8(y + base + (long long)r * C, yc[k]);
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      if (tid + k * 256 < R) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float x = yc[k][e]; s0[e] += x; s1[e] = fmaf(x, x, s1[e]); }
      }
    }
  } else {
    for (int r = tid; r < R; r += 256) {
      float p[8];
      ld8(y + base + (long long)r * C, p);
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float x = p[e]; s0[e] += x; s1[e] = fmaf(x, x, s1[e]); }
    }
  }
  block_sum16(s0, s1, red);
  if (tid < 8) {
    const double S0 = (double)red[0][0][tid] + red[0][1][tid] + red[0][2][tid] + red[0][3][tid];
    const double S1 = (double)red[1][0][tid] + red[1][1][tid] + red[1][2][tid] + red[1][3][tid];
    const double n = (double)R;
    const double m = S0 / n;
    double var = S1 / n - m * m;
    var = var > 0 ? var : 0;
    const int c = c0 + tid;
    const float is = (float)(1.0 / sqrt(var + (double)eps));
    mean[g * C + c] = (float)m;
    invstd[g * C + c] = is;
    float* prm = rm + (long long)g * p_gstride + c;
    float* prv = rv + (long long)g * p_gstride + c;
    const double unb = n > 1 ? var * n / (n - 1) : var;
    *prm = (float)((1.0 - momentum) * (*prm) + momentum * m);
    *prv = (float)((1.0 - momentum) * (*prv) + momentum * unb);
    const float sc = is * gamma[(long long)g * p_gstride + c];
    coef[0][tid] = sc;
    coef[1][tid] = beta[(long long)g * p_gstride + c] - (float)m * sc;
  }
  __syncthreads();
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { sc[e] = coef[0][e]; sh[e] = coef[1][e]; }
  float vmax = 0.f;
  auto apply_row = [&](long long o, const float (&p)[8]) __attribute__((always_inline)) {
    float rp[8], op[8];
    if (res) ld8(res + o, rp);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = fmaf(p[e], sc[e], sh[e]);
      if (res) x += rp[e];
      if (relu) x = fmaxf(x, 0.f);
      op[e] = x;
      vmax = fmaxf(vmax, fabsf(x));
    }
    st8(out + o, op);
  };
  if (cached) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int r = tid + k * 256;
      if (r < R) apply_row(base + (long long)r * C, yc[k]);
    }
  } else {
    for (int r = tid; r < R; r += 256) {
      const long long o = base + (long long)r * C;
      float p[8];
      ld8(y + o, p);
      apply_row(o, p);
    }
  }
  if (amax) amax_fold(amax, amax_ld, g, vmax);
}

template <typename T>
__global__ __launch_bounds__(256) void bn_small_bwd_kernel(
    const T* __restrict__ dout, const T* __restrict__ out, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ gamma,
    long long p_gstride, int relu, float* __restrict__ dgamma, float* __restrict__ dbeta, long long g_gstride,
    T* __restrict__ dy, T* __restrict__ dres, const int* __restrict__ nvalid, int N, int HW, int C,
    int* __restrict__ amax, int amax_ld) {
  __shared__ float red[2][4][8];
  __shared__ float coef[3][8];
  const int g = blockIdx.y, c0 = blockIdx.x * 8, tid = threadIdx.x;
  const int R = valid_rows(nvalid, g, N) * HW;
  if (R == 0) return;
  const long long base = (long long)g * N * HW * C + c0;
  float mu[8], is[8], s0[8], s1[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = mean[g * C + c0 + e];
    is[e] = invstd[g * C + c0 + e];
    s0[e] = 0.f;
    s1[e] = 0.f;
  }
  // R <= 4 * 256: the thread's rows of dout (ReLU-masked) and y are loaded once, all in
  // flight together, and kept in registers for the apply pass (same summation order)
  constexpr int RPT = 4;
  const bool cached = R <= RPT * 256;
  float dc[RPT][8], yc[RPT][8];
  auto load_row = [&](long long o, float (&dp)[8], float (&yp)[8]) __attribute__((always_inline)) {
    float op[8];
    ld8(dout + o, dp);
    ld8(y + o, yp);
    if (relu) ld8(out + o, op);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (relu && !(op[e] > 0.f)) dp[e] = 0.f;
  };
  auto acc_row = [&](const float (&dp)[8], const float (&yp)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s0[e] += dp[e];
      s1[e] = fmaf(dp[e], (yp[e] - mu[e]) * is[e], s1[e]);
    }
  };
  if (cached) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int r = tid + k * 256;
      if (r < R) load_row(base + (long long)r * C, dc[k], yc[k]);
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k)
      if (tid + k * 256 < R) acc_row(dc[k], yc[k]);
  } else {
    for (int r = tid; r < R; r += 256) {
      float dp[8], yp[8];
      load_row(base + (long long)r * C, dp, yp);
      acc_row(dp, yp);
    }
  }
  block_sum16(s0, s1, red);
  if (tid < 8) {
    const float sd = red[0][0][tid] + red[0][1][tid] + red[0][2][tid] + red[0][3][tid];
    const float sdx = red[1][0][tid] + red[1][1][tid] + red[1][2][tid] + red[1][3][tid];
    const int c = c0 + tid;
    dbeta[(long long)g * g_gstride + c] += sd;
    dgamma[(long long)g * g_gstride + c] += sdx;
    const float n = (float)R;
    const float ga = gamma[(long long)g * p_gstride + c] * is[tid];
    const float B = -ga * is[tid] * sdx / n;
    coef[0][tid] = ga;
    coef[1][tid] = B;
    coef[2][tid] = -ga * sd / n - B * mu[tid];
  }
  __syncthreads();
  float A[8], B[8], K[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { A[e] = coef[0][e]; B[e] = coef[1][e]; K[e] = coef[2][e]; }
  float vmax = 0.f;
  auto apply_row = [&](long long o, const float (&dp)[8], const float (&yp)[8]) __attribute__((always_inline)) {
    float p1[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      p1[e] = fmaf(A[e], dp[e], fmaf(B[e], yp[e], K[e]));
      vmax = fmaxf(vmax, fabsf(p1[e]));
    }
    st8(dy + o, p1);
    if (dres) st8(dres + o, dp);
  };
  if (cached) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int r = tid + k * 256;
      if (r < R) apply_row(base + (long long)r * C, dc[k], yc[k]);
    }
  } else {
    for (int r = tid; r < R; r += 256) {
      const long long o = base + (long long)r * C;
      float dp[8], yp[8];
      load_row(o, dp, yp);
      apply_row(o, dp, yp);
    }
  }
  if (amax) amax_fold(amax, amax_ld, g, vmax);
}

// eval fold: wf[s][co][k] = w[s][co][k] * s_c ; bf[s][co] = (b0 - rm) * s_c + beta
template <typename T>
__global__ void bn_fold_kernel(const float* __restrict__ w, long long w_sstride, const float* __restrict__ cbias,
                               const float* __restrict__ gamma, const float* __restrict__ beta,
                               const float* __restrict__ rm, const float* __restrict__ rv, long long s_gstride,
                               float eps, T* __restrict__ wf, float* __restrict__ bf, int slots, int Cout,
                               int K) {
  const long long per = (long long)Cout * K;
  const long long total = per * slots;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int s = (int)(t / per);
    const long long rem = t - s * per;
    const int co = (int)(rem / K);
    const int k = (int)(rem - (long long)co * K);
    const long long p = (long long)s * s_gstride + co;
    const float sc = gamma[p] / sqrtf(rv[p] + eps);
    wf[t] = from_f<T>(w[(long long)s * w_sstride + rem] * sc);
    if (k == 0) {
      const float b0 = cbias ? cbias[p] : 0.f;
      bf[(long long)s * Cout + co] = (b0 - rm[p]) * sc + beta[p];
    }
  }
}

int egrid(long long n) { return (int)std::max(1LL, std::min(16384LL, (n + 255) / 256)); }

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

// launches of at most this many replicas fold the backward finalize into the apply
// (DBA_BN_BWD_FUSE_G, default 4; 0 = off; dba_bn_bwd_fuse_set for tests)
int& bwd_fuse_g() {
  static int g = env_int("DBA_BN_BWD_FUSE_G", 4);
  return g;
}

// per-replica grid for the row-gated elementwise passes: ~16K blocks over the launch
dim3 ggrid(int G, int N, int HW, int C) {
  const long long per = (long long)N * HW * (C / 8);
  const long long cap = std::max(1LL, 16384LL / std::max(1, G));
  return dim3((unsigned)std::max(1LL, std::min(cap, (per + 255) / 256)), G);
}

}  // namespace

DBA_EXPORT int dba_bn_partial_blocks(int N, int HW, int C) { return ceil_div((long long)N * HW, rows_per_block(C)); }

// folded backward finalize for launches of <= g replicas (0: off); returns the previous value
DBA_EXPORT int dba_bn_bwd_fuse_set(int g) {
  const int prev = bwd_fuse_g();
  if (g >= 0) bwd_fuse_g() = g;
  return prev;
}

// Channel-layout contract of every BN launcher (returns -102 otherwise): C % 8 == 0 and
// 256 % (C / 8) == 0, so a thread of the grid-stride elementwise passes always owns the same
// 8 channels (ggrid), and rows_per_block(C) >= 1.
static bool bn_layout_ok(int C) { return C > 0 && C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0; }

#define BN_T(f32, call) do { if (f32) { typedef float T; call; } else { typedef uint16_t T; call; } } while (0)

// part: [G][nblk][2][C] fp32 workspace (no initialisation needed); y fp32 (f32) or bf16
// counter (optional): [G] zeroed ints — the statistics are finalised by the last reduce block
// (one launch); without it a separate finalize launch runs
DBA_EXPORT int dba_bn_stats(const void* y, const int* nvalid, int G, int N, int HW, int C, float* part, float* rm,
                            float* rv, long long s_gstride, float momentum, float eps, float* mean, float* invstd,
                            int f32, int* counter, void* stream) {
  if (!bn_layout_ok(C)) return -102;
  hipStream_t st = (hipStream_t)stream;
  const int nblk = ceil_div((long long)N * HW, rows_per_block(C));
  BnFin fin{};
  if (counter) {
    fin.counter = counter; fin.rm = rm; fin.rv = rv; fin.s_gstride = s_gstride; fin.momentum = momentum;
    fin.eps = eps; fin.mean_out = mean; fin.invstd_out = invstd;
  }
  BN_T(f32, hipLaunchKernelGGL((bn_reduce_kernel<false, T>), dim3(nblk, G), dim3(256), 0, st, (const T*)y, nullptr,
                               nullptr, nullptr, nullptr, 0, nvalid, N, HW, C, part, fin));
  if (!counter)
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(ceil_div(C, C < 64 ? C : 64), G), dim3(256), 0, st, part, nblk, nvalid,
                       N, HW, C, rm, rv, s_gstride, momentum, eps, mean, invstd, G);
  DBA_LAUNCH_CHECK();
}

// mean / invstd / running stats from the partials a conv epilogue folded (dba_xconv_fwd bnpart)
DBA_EXPORT int dba_bn_finalize_part(const double* part, int nblk, const int* nvalid, int G, int N, int HW, int C,
                                    float* rm, float* rv, long long s_gstride, float momentum, float eps, float* mean,
                                    float* invstd, void* stream) {
  if (!bn_layout_ok(C)) return -102;
  hipLaunchKernelGGL(bn_finalize_part_kernel, dim3(C, G), dim3(256), 0, (hipStream_t)stream, part, nblk, nvalid, N, HW,
                     C, rm, rv, s_gstride, momentum, eps, mean, invstd);
  DBA_LAUNCH_CHECK();
}

// amax (optional, a zeroed slot [kAmaxSub][amax_ld], common.hpp): folds max |out| per replica for an
// fp16-pair consumer (fp32 only)
DBA_EXPORT int dba_bn_apply(const void* y, const float* mean, const float* invstd, const float* gamma, const float* beta,
                            long long p_gstride, const void* res, int relu, void* out, const int* nvalid, int G, int N,
                            int HW, int C, int f32, int* amax, int amax_ld, void* stream) {
  if (!bn_layout_ok(C)) return -102;
  BN_T(f32, hipLaunchKernelGGL((bn_apply_kernel<T>), ggrid(G, N, HW, C), dim3(256), 0, (hipStream_t)stream,
                               (const T*)y, mean, invstd, gamma, beta, p_gstride, (const T*)res, relu, (T*)out, nvalid,
                               G, N, HW, C, amax, amax_ld));
  DBA_LAUNCH_CHECK();
}

// part: [G][nblk][2][C] workspace followed by sums [G][2][C] (fp32, no initialisation needed)
DBA_EXPORT int dba_bn_bwd(const void* dout, const void* out, const void* y, const float* mean, const float* invstd,
                          const float* gamma, long long p_gstride, int relu, float* dgamma, float* dbeta,
                          long long g_gstride, void* dy, void* dres, float* part, const int* nvalid, int G, int N,
                          int HW, int C, int f32, int* amax, int amax_ld, int* counter, void* stream) {
  if (!bn_layout_ok(C)) return -102;
  hipStream_t st = (hipStream_t)stream;
  const int nblk = ceil_div((long long)N * HW, rows_per_block(C));
  float* sums = part + (long long)G * nblk * 2 * C;
  BnFin fin{};
  if (counter) {
    fin.counter = counter; fin.sums = sums; fin.dgamma = dgamma; fin.dbeta = dbeta; fin.g_gstride = g_gstride;
  }
  BN_T(f32, hipLaunchKernelGGL((bn_reduce_kernel<true, T>), dim3(nblk, G), dim3(256), 0, st, (const T*)y,
                               (const T*)dout, (const T*)out, mean, invstd, relu, nvalid, N, HW, C, part, fin));
  // launches of few replicas (a lone client's step): the finalize folds into the apply
  // (bn_bwd_apply_fin_kernel, same bits); DBA_BN_BWD_FUSE_G=0 keeps three launches
  if (!counter && G <= bwd_fuse_g()) {
    dim3 ga = ggrid(G, N, HW, C);
    ga.x = std::min(ga.x, 128u);
    BN_T(f32, hipLaunchKernelGGL((bn_bwd_apply_fin_kernel<T>), ga, dim3(256), 0, st, (const T*)dout, (const T*)out,
                                 (const T*)y, mean, invstd, gamma, p_gstride, part, nblk, dgamma, dbeta, g_gstride,
                                 relu, (T*)dy, (T*)dres, nvalid, N, HW, C, amax, amax_ld));
    DBA_LAUNCH_CHECK();
  }
  if (!counter)
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(ceil_div(C, C < 64 ? C : 64), G), dim3(256), 0, st, part, nblk,
                       sums, dgamma, dbeta, g_gstride, G, C);
  BN_T(f32, hipLaunchKernelGGL((bn_bwd_apply_kernel<T>), ggrid(G, N, HW, C), dim3(256), 0, st, (const T*)dout,
                               (const T*)out, (const T*)y, mean, invstd, gamma, p_gstride, sums, relu, (T*)dy,
                               (T*)dres, nvalid, G, N, HW, C, amax, amax_ld));
  DBA_LAUNCH_CHECK();
}

// single-launch BN forward for rows-per-replica <= 16384 (see bn_small_fwd_kernel)
DBA_EXPORT int dba_bn_small_fwd(const void* y, const int* nvalid, int G, int N, int HW, int C, const float* gamma,
                                const float* beta, float* rm, float* rv, long long p_gstride, float momentum, float eps,
                                const void* res, int relu, void* out, float* mean, float* invstd, int f32,
                                int* amax, int amax_ld, void* stream) {
  if (C % 8 != 0) return -102;
  BN_T(f32, hipLaunchKernelGGL((bn_small_fwd_kernel<T>), dim3(C / 8, G), dim3(256), 0, (hipStream_t)stream,
                               (const T*)y, nvalid, N, HW, C, gamma, beta, rm, rv, p_gstride, momentum, eps,
                               (const T*)res, relu, (T*)out, mean, invstd, amax, amax_ld));
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_bn_small_bwd(const void* dout, const void* out, const void* y, const float* mean,
                                const float* invstd, const float* gamma, long long p_gstride, int relu, float* dgamma,
                                float* dbeta, long long g_gstride, void* dy, void* dres, const int* nvalid, int G,
                                int N, int HW, int C, int f32, int* amax, int amax_ld, void* stream) {
  if (C % 8 != 0) return -102;
  BN_T(f32, hipLaunchKernelGGL((bn_small_bwd_kernel<T>), dim3(C / 8, G), dim3(256), 0, (hipStream_t)stream,
                               (const T*)dout, (const T*)out, (const T*)y, mean, invstd, gamma, p_gstride, relu,
                               dgamma, dbeta, g_gstride, (T*)dy, (T*)dres, nvalid, N, HW, C, amax, amax_ld));
  DBA_LAUNCH_CHECK();
}

// wf in fp32 (f32) or bf16
DBA_EXPORT int dba_bn_fold(const float* w, long long w_sstride, const float* cbias, const float* gamma,
                           const float* beta, const float* rm, const float* rv, long long s_gstride, float eps,
                           void* wf, float* bf, int slots, int Cout, int K, int f32, void* stream) {
  const long long n = (long long)slots * Cout * K;
  BN_T(f32, hipLaunchKernelGGL((bn_fold_kernel<T>), dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, w, w_sstride,
                               cbias, gamma, beta, rm, rv, s_gstride, eps, (T*)wf, bf, slots, Cout, K));
  DBA_LAUNCH_CHECK();
}
