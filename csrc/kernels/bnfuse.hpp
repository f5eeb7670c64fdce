// Training BatchNorm fused into the conv kernels (gfx950): the statistics of a conv output are
// reduced by the kernel that produces it, and the normalisation is applied by the kernels that
// CONSUME it, so a conv-BN-ReLU costs no launch of its own.
//
// Reference semantics: BatchNorm2d in train mode followed by ReLU / a residual add
// (/root/reference/models/resnet_cifar.py:31-36, driven by image_train.py:84-102): biased
// variance to normalise, unbiased variance into the running statistics (momentum 0.1).
//
// Forward.  The producing conv's epilogue (xconv.hpp xconv_kernel / xhalo.hpp xhalo_kernel, stem.hip) reduces its
// tile of the raw output y into LEVEL-0 records, one per (32-row group, channel):
//     {sum y, sum y^2, max y, min y}        (sums in fp64, sequential over the 32 rows)
// and one small launch (bnx_finalize_kernel, a block per (channel, replica)) sums a channel's
// records in a fixed order and finalises: mean, 1/std, the running-stat update, the affine form
// scale = gamma/std, shift = beta - mean*scale of the BN (+ReLU) output, and an exact bound of
// that output's max |.| (from the per-channel max / min of y) for the fp16-pair operand scale
// of its consumers.  The output itself is never stored when its only consumers are convs: the
// consuming conv's A staging (and the weight gradient's x staging) computes
// relu(fma(y, scale, shift)) per element — bit-identical to a separate BN-apply pass.
//
// Backward.  The data gradient g of a BN(+ReLU) output comes from a dgrad whose epilogue masks
// it (d = g where the output is > 0), stores d, and reduces level-0 records
//     {sum d, sum d*xhat_a, sum d*xhat_b, max |d|}     (xhat = (y - mean) * invstd, fp32)
// for the BN a of the output and, when the output is a residual sum of two BNs (a shortcut
// conv), the BN b of the other branch; the finalize launch accumulates dbeta += sum d,
// dgamma += sum d*xhat and the affine form of the BN input gradient
//     dy = fma(A, d, fma(B, y, K)),  A = gamma*invstd, B = -A*invstd*sum(d*xhat)/n,
//     K = -A*sum(d)/n - B*mean
// (bn.hip's formulas), with a bound of max |dy| for its fp16-pair scale.  The weight gradient of
// the conv below stages dy from (d, y) on the fly and stores it once for that conv's data
// gradient.
//
// Every order is fixed (groups of 32 rows; the finalize's per-thread strides and LDS tree depend
// on the replica's group count only) and independent of the tile shape of the launch, so the
// bits do not depend on how many replicas share a launch: a tile (32 / 64 / 128 rows) always
// covers whole groups; split-K launches, the standalone pass (xbn.hip bnx_tile_kernel) and the
// epilogues produce the same records.  (An in-kernel two-level ticket finalisation was measured
// first: its serial tail after the last tile cost 12-20 us per conv — more than this launch.
// Round 6 measured exact integer records accumulated with device-scope atomics and finalised
// by their first consumer: 39-46 fewer launches per step, but the atomics — 8-10 per (tile,
// channel), performed past the per-XCD L2s — made the producing convs 9-20 us slower each:
// lone step 1667 -> 1882 us, 10-client step 2948 -> 3355 us; profiles/r6/acc/.)
#pragma once
#include "common.hpp"

__host__ __device__ __forceinline__ int ceil_div_d(int a, int b) { return (a + b - 1) / b; }

constexpr int kBnGrp = 32;                 // rows per level-0 group
// per-BN coefficient rows [G][kBnRows][C] (fp32)
enum { kCMean = 0, kCInv, kCScale, kCShift, kCYmax, kCYmin, kCA, kCB, kCK, kBnRows };

struct BnFuse {
  int mode;                 // 0 none, 1 forward statistics of the output, 2 backward (mask + reduce)
  int C;                    // channels of the output (= the conv's Ncol)
  int ngrp;                 // 32-row groups per replica (from the replica's row count)
  double* rec0;             // [G][C][ngrp][4] level-0 records (channel-major: the finalize reads a channel's run)
  // BN a: forward — the BN of this output; backward — the BN whose output's gradient this is
  float* coef_a;            // [G][kBnRows][C]
  const float* gamma_a; const float* beta_a; float* rm_a; float* rv_a;
  long long p_gstride;      // replica stride of gamma / beta / running stats (flat state rows)
  float momentum, eps;
  int relu;                 // forward: the lazy output has a ReLU (its bound)
  int* amax_a; int amax_ld; // forward: bound slot of the lazy output; backward: of dy_a
  // backward only
  const float* ya; const float* yb; long long y_gstride;   // pre-BN values of BN a / b
  float* coef_b; const float* gamma_b; int* amax_b;
  float* dgamma_a; float* dbeta_a; float* dgamma_b; float* dbeta_b; long long gr_gstride;
  const float* mask_out;    // d = g where mask_out > 0 (the materialised BN output), else
  int mask_lazy;            //   where fma(ya, scale_a, shift_a) > 0 (mask_lazy), else d = g
};

__device__ __forceinline__ void bnf_store_rec(double* p, double a, double b, double c, double d) {
  ((double2*)p)[0] = make_double2(a, b);
  ((double2*)p)[1] = make_double2(c, d);
}

// combine record v into accumulator a (sums in order; max / min or max |d|)
__device__ __forceinline__ void bnf_acc(double (&a)[4], const double (&v)[4], int mode) {
  a[0] += v[0];
  a[1] += v[1];
  if (mode == 1) {
    a[2] = fmax(a[2], v[2]);
    a[3] = fmin(a[3], v[3]);
  } else {
    a[2] += v[2];
    a[3] = fmax(a[3], v[3]);
  }
}
__device__ __forceinline__ void bnf_init(double (&a)[4], int mode) {
  a[0] = 0.0; a[1] = 0.0;
  a[2] = mode == 1 ? -INFINITY : 0.0;
  a[3] = mode == 1 ? INFINITY : 0.0;
}

// per-channel finalisation of replica g from its level-1 sum a (n valid rows); returns the
// channel's bound contribution (forward: max |relu?(fma(y, scale, shift))|; backward: max |dy_a|,
// and *bound_b: max |dy_b|)
__device__ __forceinline__ float bnf_finalize_channel(const BnFuse& f, int g, int c, const double (&a)[4], double n,
                                                      float* bound_b) {
  const int C = f.C;
  float* ca = f.coef_a + (long long)g * kBnRows * C;
  if (f.mode == 1) {
    const double m = a[0] / n;
    double var = a[1] / n - m * m;
    var = var > 0 ? var : 0;
    const float mean = (float)m, inv = (float)(1.0 / sqrt(var + (double)f.eps));
    float* prm = f.rm_a + (long long)g * f.p_gstride + c;
    float* prv = f.rv_a + (long long)g * f.p_gstride + c;
    const double unb = n > 1 ? var * n / (n - 1) : var;
    *prm = (float)((1.0 - f.momentum) * (*prm) + f.momentum * m);
    *prv = (float)((1.0 - f.momentum) * (*prv) + f.momentum * unb);
    const float sc = inv * f.gamma_a[(long long)g * f.p_gstride + c];
    const float sh = f.beta_a[(long long)g * f.p_gstride + c] - mean * sc;
    const float ymax = (float)a[2], ymin = (float)a[3];
    ca[kCMean * C + c] = mean;
    ca[kCInv * C + c] = inv;
    ca[kCScale * C + c] = sc;
    ca[kCShift * C + c] = sh;
    ca[kCYmax * C + c] = ymax;
    ca[kCYmin * C + c] = ymin;
    float hi = fmaf(ymax, sc, sh), lo = fmaf(ymin, sc, sh);
    if (f.relu) { hi = fmaxf(hi, 0.f); lo = fmaxf(lo, 0.f); }
    return fmaxf(fabsf(hi), fabsf(lo));
  }
  // backward: bn.hip bn_bwd_apply's coefficients from the fp32-rounded sums
  const float fn = (float)n;
  const float sd = (float)a[0], dmax = (float)a[3];
  auto one = [&](float* cb, const float* gam, float* dgam, float* dbet, float sdx) __attribute__((always_inline)) {
    dbet[(long long)g * f.gr_gstride + c] += sd;
    dgam[(long long)g * f.gr_gstride + c] += sdx;
    const float is = cb[kCInv * C + c], mean = cb[kCMean * C + c];
    const float ga = gam[(long long)g * f.p_gstride + c] * is;
    const float B = -ga * is * sdx / fn;
    const float K = -ga * sd / fn - B * mean;
    cb[kCA * C + c] = ga;
    cb[kCB * C + c] = B;
    cb[kCK * C + c] = K;
    const float hi = fmaf(B, cb[kCYmax * C + c], K), lo = fmaf(B, cb[kCYmin * C + c], K);
    return (fabsf(ga) * dmax + fmaxf(fabsf(hi), fabsf(lo))) * (1.f + 0x1p-10f);
  };
  const float ba = one(ca, f.gamma_a, f.dgamma_a, f.dbeta_a, (float)a[1]);
  if (f.coef_b) *bound_b = fmaxf(*bound_b, one(f.coef_b + (long long)g * kBnRows * C, f.gamma_b, f.dgamma_b,
                                               f.dbeta_b, (float)a[2]));
  return ba;
}

// level-0 records of a tile staged in LDS: Ct [BM][BN] fp32 (forward: y; backward: d, already
// masked) of rows m0.. / columns n0.. of replica g; orow[r] >= 0 marks a valid row and is its
// element offset in the replica's [M][C] output (the offset of ya / yb too)
template <int BM, int BN>
__device__ __forceinline__ void bnf_tile_records(const BnFuse& f, const float* Ct, const long long* orow, int g,
                                                 int m0, int n0, int Mv) {
  constexpr int NG = BM / kBnGrp;
  static_assert(BM % kBnGrp == 0, "tiles cover whole groups");
  const int gv = ceil_div_d(Mv, kBnGrp);
  const int C = f.C;
  const float* ya = f.mode == 2 ? f.ya + (long long)g * f.y_gstride : nullptr;
  const float* yb = (f.mode == 2 && f.yb) ? f.yb + (long long)g * f.y_gstride : nullptr;
  const float* ca = f.coef_a + (long long)g * kBnRows * C;
  const float* cb = f.coef_b ? f.coef_b + (long long)g * kBnRows * C : nullptr;
  for (int e = threadIdx.x; e < NG * BN; e += 256) {
    const int grp = e / BN, cc = e - grp * BN, n = n0 + cc;
    const int b = m0 / kBnGrp + grp;
    if (n >= C || b >= gv) continue;
    double a[4];
    bnf_init(a, f.mode);
    if (f.mode == 1) {
#pragma unroll 8
      for (int r = 0; r < kBnGrp; ++r) {
        const int row = grp * kBnGrp + r;
        if (orow[row] < 0) continue;
        const double v = (double)Ct[row * BN + cc];
        a[0] += v;
        a[1] = fma(v, v, a[1]);
        a[2] = fmax(a[2], v);
        a[3] = fmin(a[3], v);
      }
    } else {
      const float ma = ca[kCMean * C + n], ia = ca[kCInv * C + n];
      const float mb = cb ? cb[kCMean * C + n] : 0.f, ib = cb ? cb[kCInv * C + n] : 0.f;
      // the group's BN inputs first, all loads in flight (a load per row in the ordered loop
      // below cost one memory latency per 4 rows: +8-12 us per data-gradient launch)
      float yav[kBnGrp], ybv[kBnGrp];
#pragma unroll
      for (int r = 0; r < kBnGrp; ++r) {
        const long long o = orow[grp * kBnGrp + r];
        yav[r] = o >= 0 ? ya[o + n] : 0.f;
        ybv[r] = (o >= 0 && yb) ? yb[o + n] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < kBnGrp; ++r) {
        const int row = grp * kBnGrp + r;
        if (orow[row] < 0) continue;
        const float d = Ct[row * BN + cc];
        const float xa = (yav[r] - ma) * ia;
        a[0] += (double)d;
        a[1] = fma((double)d, (double)xa, a[1]);
        if (yb) a[2] = fma((double)d, (double)((ybv[r] - mb) * ib), a[2]);
        a[3] = fmax(a[3], (double)fabsf(d));
      }
    }
    bnf_store_rec(f.rec0 + (((long long)g * C + n) * f.ngrp + b) * 4, a[0], a[1], a[2], a[3]);
  }
}

// the backward mask of an output element vector (4 consecutive channels n.. at row offset o of
// replica g): d = g where the BN(+ReLU) output is > 0
__device__ __forceinline__ float4 bnf_mask4(const BnFuse& f, int g, long long o, int n, float4 v) {
  if (f.mask_out) {
    const float4 m = *(const float4*)(f.mask_out + (long long)g * f.y_gstride + o + n);
    v.x = m.x > 0.f ? v.x : 0.f; v.y = m.y > 0.f ? v.y : 0.f; v.z = m.z > 0.f ? v.z : 0.f; v.w = m.w > 0.f ? v.w : 0.f;
  } else if (f.mask_lazy) {
    const float* ca = f.coef_a + (long long)g * kBnRows * f.C;
    const float4 y = *(const float4*)(f.ya + (long long)g * f.y_gstride + o + n);
    const float4 sc = *(const float4*)(ca + kCScale * f.C + n), sh = *(const float4*)(ca + kCShift * f.C + n);
    v.x = fmaf(y.x, sc.x, sh.x) > 0.f ? v.x : 0.f;
    v.y = fmaf(y.y, sc.y, sh.y) > 0.f ? v.y : 0.f;
    v.z = fmaf(y.z, sc.z, sh.z) > 0.f ? v.z : 0.f;
    v.w = fmaf(y.w, sc.w, sh.w) > 0.f ? v.w : 0.f;
  }
  return v;
}

// One block per (channel, replica): the channel's level-0 records summed in a fixed order
// (thread t: groups t, t + 256, ... in order; then a fixed pairwise LDS tree), finalised by
// thread 0; the bound folds into the zeroed slot with an integer atomicMax (exact, any order).
__device__ __forceinline__ void bnf_finalize_block(const BnFuse& f, int g, int c, int Mv) {
  __shared__ double red[256][4];
  const int tid = threadIdx.x;
  const int gv = ceil_div_d(Mv, kBnGrp);
  double a[4];
  bnf_init(a, f.mode);
  const double* r = f.rec0 + ((long long)g * f.C + c) * f.ngrp * 4;
  for (int b = tid; b < gv; b += 256) {
    const double2 lo = ((const double2*)(r + b * 4))[0], hi = ((const double2*)(r + b * 4))[1];
    const double v[4] = {lo.x, lo.y, hi.x, hi.y};
    bnf_acc(a, v, f.mode);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) red[tid][q] = a[q];
  __syncthreads();
  // the fixed pairwise tree (tid <- tid + w, w = 128 .. 1): the two cross-wave levels through
  // LDS, the six in-wave levels as shuffles — the same pairs in the same order as an LDS level
  // each, without their barriers (every combine is commutative)
  if (tid < 128) {
    const double v[4] = {red[tid + 128][0], red[tid + 128][1], red[tid + 128][2], red[tid + 128][3]};
    double x[4] = {red[tid][0], red[tid][1], red[tid][2], red[tid][3]};
    bnf_acc(x, v, f.mode);
#pragma unroll
    for (int q = 0; q < 4; ++q) red[tid][q] = x[q];
  }
  __syncthreads();
  if (tid >= 64) return;
  double x[4];
  {
    const double v[4] = {red[tid + 64][0], red[tid + 64][1], red[tid + 64][2], red[tid + 64][3]};
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = red[tid][q];
    bnf_acc(x, v, f.mode);
  }
#pragma unroll
  for (int w = 32; w > 0; w >>= 1) {
    double v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = __shfl_down(x[q], w, 64);
    bnf_acc(x, v, f.mode);   // (lanes >= w compute values no later level reads)
  }
  if (tid != 0) return;
  const double t[4] = {x[0], x[1], x[2], x[3]};
  float bb = 0.f;
  const float ba = bnf_finalize_channel(f, g, c, t, (double)Mv, &bb);
  if (f.amax_a && ba > 0.f) atomicMax(f.amax_a + (c % kAmaxSub) * f.amax_ld + g, __float_as_int(ba));
  if (f.amax_b && bb > 0.f) atomicMax(f.amax_b + (c % kAmaxSub) * f.amax_ld + g, __float_as_int(bb));
}

namespace {
__global__ __launch_bounds__(256) void bnx_finalize_kernel(const BnFuse f, const int* __restrict__ nvalid, int N,
                                                           int HW) {
  const int Mv = valid_rows(nvalid, blockIdx.y, N) * HW;
  if (Mv > 0) bnf_finalize_block(f, blockIdx.y, blockIdx.x, Mv);   // (inactive replicas: consumers skip them)
}

// the finalize launch of a fused BN pass (after its producer in stream order)
inline int bnx_finalize_go(const BnFuse& f, const int* nvalid, int G, int N, int HW, hipStream_t st) {
  hipLaunchKernelGGL(bnx_finalize_kernel, dim3(f.C, G), dim3(256), 0, st, f, nvalid, N, HW);
  return (int)hipGetLastError();
}
}  // namespace
