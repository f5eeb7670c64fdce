// Training BatchNorm fused into the conv kernels (gfx950): the statistics of a conv output are
// reduced by the kernel that produces it, and the normalisation is applied by the kernels that
// CONSUME it, so a conv-BN-ReLU costs no launch of its own.
//
// Reference semantics: BatchNorm2d in train mode followed by ReLU / a residual add
// (/root/reference/models/resnet_cifar.py:31-36, driven by image_train.py:84-102): biased
// variance to normalise, unbiased variance into the running statistics (momentum 0.1).
//
// Forward.  The producing conv's epilogue (xgemm.hip xconv / xhalo, stem.hip) reduces its
// tile of the raw output y into LEVEL-0 records, one per (32-row group, channel):
//     {sum y, sum y^2, max y, min y}        (sums in fp64, sequential over the 32 rows)
// Every 512 rows (16 groups) form a super group (SG); the tile blocks of an SG draw tickets on
// the SG's counter and the last one sums the SG's 16 records in group order into a LEVEL-1
// record; those SG finalisers draw tickets on the replica's counter and the last one sums the
// SG records in order and finalises: mean, 1/std, the running-stat update, the affine form
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
// conv), the BN b of the other branch; the same two-level tickets finalise dbeta += sum d,
// dgamma += sum d*xhat and the affine form of the BN input gradient
//     dy = fma(A, d, fma(B, y, K)),  A = gamma*invstd, B = -A*invstd*sum(d*xhat)/n,
//     K = -A*sum(d)/n - B*mean
// (bn.hip's formulas), with a bound of max |dy| for its fp16-pair scale.  The weight gradient of
// the conv below stages dy from (d, y) on the fly and stores it once for that conv's data
// gradient.
//
// Every order is fixed (groups of 32 rows, SGs of 16 groups, SGs in order) and independent of
// the tile shape of the launch, so the bits do not depend on how many replicas share a launch:
// a tile (32 / 64 / 128 rows, 512 % rows == 0) always covers whole groups of one SG; split-K
// launches, the separate split-K reduce and the standalone kernels (bn.hip bnx_*) produce the
// same records.  Hand-offs between the blocks of one launch: every record is stored
// write-through (sc1) and drained by every storing wave (vmcnt(0)) before a workgroup barrier
// and ONE agent-scope atomic add per workgroup; the workgroup whose add returns expected-1
// reads the records with sc1 loads only — the first row of MI355X_MICROARCH.md's hand-off table
// (§ visibility: "ONE lane of each storing workgroup, for ALL that workgroup's stores: an
// agent-scope atomic add ... the workgroup whose add came last, told by the value its add
// returned ... loads, all sc1").  No block waits for another, so the grid always drains.
#pragma once
#include "common.hpp"

__host__ __device__ __forceinline__ int ceil_div_d(int a, int b) { return (a + b - 1) / b; }

constexpr int kBnGrp = 32;                 // rows per level-0 group
constexpr int kBnSg = 512;                 // rows per super group
constexpr int kBnGpS = kBnSg / kBnGrp;     // groups per super group
// per-BN coefficient rows [G][kBnRows][C] (fp32)
enum { kCMean = 0, kCInv, kCScale, kCShift, kCYmax, kCYmin, kCA, kCB, kCK, kBnRows };

struct BnFuse {
  int mode;                 // 0 none, 1 forward statistics of the output, 2 backward (mask + reduce)
  int C;                    // channels of the output (= the conv's Ncol)
  int ngrp, nsg;            // groups / super groups per replica (from the replica's row count)
  double* rec0;             // [G][ngrp][C][4]
  double* rec1;             // [G][nsg][C][4]
  int* cnt1;                // [G][nsg] zeroed
  int* cnt2;                // [G] zeroed
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

// ---- write-through record stores / loads (aux 16 = sc1)
typedef __attribute__((ext_vector_type(4))) unsigned int bnf_u32x4;
__device__ __forceinline__ void bnf_store_rec(double* base, long long rec_index, long long nrec, double a, double b,
                                              double c, double d) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)0x7fffffff, 0x00020000);
  const int off = (int)(rec_index * 32);
  (void)nrec;
  const double2 lo = make_double2(a, b), hi = make_double2(c, d);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(bnf_u32x4, lo), r, off, 0, 16);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(bnf_u32x4, hi), r, off + 16, 0, 16);
}
__device__ __forceinline__ void bnf_load_rec(const double* base, long long rec_index, double (&v)[4]) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), (short)0, (int)0x7fffffff, 0x00020000);
  const int off = (int)(rec_index * 32);
  const double2 lo = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
  const double2 hi = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, 16));
  v[0] = lo.x; v[1] = lo.y; v[2] = hi.x; v[3] = hi.y;
}

// block-level ticket: every thread calls; true in every thread of the block whose add was the
// expected-th.  The counter is reset by that block (reusable by the next launch / replay).
__device__ __forceinline__ bool bnf_arrive(int* cnt, int expected) {
  __shared__ int bnf_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == expected - 1;
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bnf_last = last;
  }
  __syncthreads();
  const bool last = bnf_last;
  if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler: loads stay below
  return last;
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

// the replica finaliser (one block): sums the nsg_v level-1 records of every channel in SG order
__device__ __forceinline__ void bnf_finalize_replica(const BnFuse& f, int g, int nsg_v, double n) {
  __shared__ float bnf_red[2][4];
  float ba = 0.f, bb = 0.f;
  for (int c = threadIdx.x; c < f.C; c += blockDim.x) {
    double a[4];
    bnf_init(a, f.mode);
    for (int s = 0; s < nsg_v; ++s) {
      double v[4];
      bnf_load_rec(f.rec1, ((long long)g * f.nsg + s) * f.C + c, v);
      bnf_acc(a, v, f.mode);
    }
    ba = fmaxf(ba, bnf_finalize_channel(f, g, c, a, n, &bb));
  }
  ba = wave_max(ba);
  bb = wave_max(bb);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { bnf_red[0][w] = ba; bnf_red[1][w] = bb; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (int)(blockDim.x + 63) >> 6;
    float x = 0.f, y = 0.f;
    for (int k = 0; k < nw; ++k) { x = fmaxf(x, bnf_red[0][k]); y = fmaxf(y, bnf_red[1][k]); }
    // the slot is zeroed and this block is its only writer (sub-slot 0 of common.hpp's layout)
    if (f.amax_a) f.amax_a[g] = __float_as_int(x);
    if (f.amax_b) f.amax_b[g] = __float_as_int(y);
  }
}

// the SG finaliser (one block): sums the SG's level-0 records in group order into its level-1
// record, then the replica ticket
__device__ __forceinline__ void bnf_finalize_sg(const BnFuse& f, int g, int s, int Mv) {
  const int gv = ceil_div_d(Mv, kBnGrp);
  const int b0 = s * kBnGpS, b1 = min(gv, b0 + kBnGpS);
  for (int c = threadIdx.x; c < f.C; c += blockDim.x) {
    double a[4];
    bnf_init(a, f.mode);
    for (int b = b0; b < b1; ++b) {
      double v[4];
      bnf_load_rec(f.rec0, ((long long)g * f.ngrp + b) * f.C + c, v);
      bnf_acc(a, v, f.mode);
    }
    bnf_store_rec(f.rec1, ((long long)g * f.nsg + s) * f.C + c, 0, a[0], a[1], a[2], a[3]);
  }
  const int nsg_v = ceil_div_d(Mv, kBnSg);
  if (bnf_arrive(f.cnt2 + g, nsg_v)) bnf_finalize_replica(f, g, nsg_v, (double)Mv);
}

// after a tile block stored its level-0 records (rows m0.. of the replica, BM rows, one of
// tiles_n column tiles): the SG ticket and, for the last arriver, the SG finalisation
__device__ __forceinline__ void bnf_tile_done(const BnFuse& f, int g, int m0, int BM, int tiles_n, int Mv) {
  const int s = m0 / kBnSg;
  const int rows = min(kBnSg, Mv - s * kBnSg);
  if (bnf_arrive(f.cnt1 + (long long)g * f.nsg + s, ceil_div_d(rows, BM) * tiles_n)) bnf_finalize_sg(f, g, s, Mv);
}

// level-0 records of a tile staged in LDS: Ct [BM][BN] fp32 (forward: y; backward: d, already
// masked) of rows m0.. / columns n0.. of replica g; orow[r] >= 0 marks a valid row and is its
// element offset in the replica's [M][C] output (the offset of ya / yb too)
template <int BM, int BN>
__device__ __forceinline__ void bnf_tile_records(const BnFuse& f, const float* Ct, const long long* orow, int g,
                                                 int m0, int n0, int Mv) {
  constexpr int NG = BM / kBnGrp;
  static_assert(BM % kBnGrp == 0 && kBnSg % BM == 0, "tiles cover whole groups of one super group");
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
#pragma unroll 4
      for (int r = 0; r < kBnGrp; ++r) {
        const int row = grp * kBnGrp + r;
        const long long o = orow[row];
        if (o < 0) continue;
        const float d = Ct[row * BN + cc];
        const float xa = (ya[o + n] - ma) * ia;
        a[0] += (double)d;
        a[1] = fma((double)d, (double)xa, a[1]);
        if (yb) a[2] = fma((double)d, (double)((yb[o + n] - mb) * ib), a[2]);
        a[3] = fmax(a[3], (double)fabsf(d));
      }
    }
    bnf_store_rec(f.rec0, ((long long)g * f.ngrp + b) * C + n, 0, a[0], a[1], a[2], a[3]);
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
