// Reference-precision (fp32) convolution family for gfx950: scaled fp16-pair MFMA.
//
// The reference trains and evaluates in fp32 (image_train.py:84-91, models/resnet_cifar.py:
// 67-104).  gfx950 has no xf32 MFMA and its exact f32-input MFMA runs at 1/16 of the 16-bit
// rate, so these kernels keep fp32 operands in HBM and split every operand element x, scaled
// by a power of two 2^s fixed per launch from the operand's max |x| (xmfma.hpp HScale), into
// two fp16 planes while staging it into LDS:
//
//     x * 2^s = h + l + e,   h = f16(x * 2^s),   l = f16(x * 2^s - h),   |e| <= 2^-22 |x|
//
// and sum the plane products hh + hl + lh (3 MFMAs per product, fp32 accumulation; the
// dropped ll term is <= 2^-22 |xy|) on the f16 MFMA: fp32-level error (tests/test_gpu_f32.py
// against fp64) at 1/3 of the 16-bit peak, ~5x the exact f32 MFMA's.  The operand maxima are
// folded by the producing kernels' epilogues (common.hpp amax_fold), so the scales cost no
// extra pass.  (Round 2-4 also carried 2- and 3-plane bf16 splits; the fp16 pair replaced
// them on every pass, measured under the branch-matched fp64 oracle: profiles/split_policy_r3.md.)
//
// Kernels (all deterministic: fixed reduction orders, no float atomics; the in-launch split-K
// combine draws integer arrival tickets that only pick WHICH block sums the slabs):
//   xconv_kernel    implicit-GEMM conv forward (bias / residual / ReLU epilogue) and data
//                   gradient; a stride-s data gradient runs as s*s parity classes, each an
//                   implicit GEMM over its own taps (no zero-tap MFMA work), in one launch;
//   xwgrad_kernel   weight gradient: C[cout][k] = sum_m dy[m][cout] * im2col(x)[m][k], both
//                   operands transposed to reduction-major while staging; split over m into
//                   fp32 slabs summed in a fixed order by xwgrad_reduce_kernel;
//   xsplitk_reduce  split-K slabs of small forward launches + epilogue (when the caller has
//                   no arrival counters: otherwise sk_combine sums them in the launch);
//   xtranspose      forward weights -> parity-class packed data-gradient weights;
//   xcolsum         bias gradient (column sums, fixed order).
#include "common.hpp"
#include "bnfuse.hpp"
#include "xmfma.hpp"
#include "xwgrad_halo.hpp"
#include <algorithm>
#include <type_traits>
#include <utility>
#include <cstdlib>

namespace {

// ============================================================================ conv
struct XClass {
  int nI, nJ;      // taps of the class along kh / kw
  int bh, bw;      // source pixel = (p*sp + bh + dsg*i, q*sp + bw + dsg*j)
  int oh, ow;      // output pixel = (p*os + oh, q*os + ow)
  int Hq, Wq;      // GEMM row grid per image
  long long boff;  // offset of the class's packed weights [Ncol][nI*nJ*Cs] in a slot
};

struct XArgs {
  const float* src; long long src_gstride;   // [G][N][Hs][Ws][Cs]
  const float* w; long long w_sstride;       // per slot: classes' [Ncol][K_c] blocks
  const int* wsel;
  const float* bias; long long b_sstride;
  const float* res;                          // output layout
  float* out; long long out_gstride;         // [G][N][Ho][Wo][Ncol] (or split-K slabs)
  const int* nvalid;
  int N, Hs, Ws, Cs, Ncol, Ho, Wo;
  int sp, os, dsg, relu;
  int splitk, tiles_n;
  int kslab;                                 // xconv KS: split-K slabs summed in the block (1: none)
  long long zstride;                         // split-K: slab z at out + z * zstride
  const int* amax_src;                       // H: max |src| slot [kAmaxSub][amax_src_ld] (common.hpp)
  const int* amax_w;                         // H: max |w| slot, indexed by weight slot
  int* amax_out;                             // optional: fold max |out| (zeroed slot)
  int amax_src_ld, amax_w_ld, amax_out_ld;
  const uint16_t* wp;                        // the weights pre-split (xsplit_w_kernel): per slot
  long long wp_sstride;                      //    2 planes of wp_sstride/2 fp16, scaled like amax_w
  // in-launch split-K combine (xconv_kernel sk_combine): slab z of replica g at
  // sk_ws + z * zstride + g * sk_gstride; sk_cnt: zeroed arrival counters, one per
  // (replica, tile, class); out / out_gstride stay the real output
  float* sk_ws; long long sk_gstride;
  int* sk_cnt;
  // training BN fused into the conv (bnfuse.hpp): forward statistics / backward mask + reduce of
  // the OUTPUT (bf.mode), and the lazy BN(+ReLU) A operand: the source holds the pre-BN values y
  // and every staged element is relu?(fma(y, scale, shift)) (lz_coef: the source BN's
  // coefficient rows [G][kBnRows][Cs]; zero outside the image)
  BnFuse bf;
  const float* lz_coef;
  int lz_relu;
  // fused downsampling shortcut (evaluation, xhalo_kernel SC): out += the 1x1
  // stride-2 conv of x2 [G][N][sc_H][sc_W][sc_C] with pre-split weights (sc_wp: per slot 2 planes
  // of Ncol x sc_C fp16) + its bias, as extra k-steps of the same accumulators
  const float* sc_src; long long sc_gstride;
  int sc_H, sc_W, sc_C;
  const uint16_t* sc_wp; long long sc_wp_sstride;
  const int* sc_amax_src; int sc_amax_src_ld;
  const int* sc_amax_w; int sc_amax_w_ld;
  const float* sc_bias; long long sc_b_sstride;
  XClass cls[4];
};

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4v;

// In-launch split-K combine (the CDNA4 guide's counter hand-off, write-through form) for a
// lone client's 32 x 128 tiles: every K-slice block stores its fp32 tile slab write-through
// (sc1: no release fence), drains it (every wave s_waitcnt vmcnt(0), then the barrier), and
// one lane draws a ticket on the tile's agent-scope counter; the block drawing S-1 reads the
// other slabs with sc1 loads (no acquire: every load of a handed-off byte bypasses L1), ALL of
// them in flight at once, and sums them into Ct in z order 0..S-1 — xsplitk_reduce_kernel's
// order, so every output bit is unchanged — then runs the normal epilogue (bias / residual /
// ReLU / BN statistics / max).  No block waits on another (the last arriver does the work), so
// the grid always drains.  Replaces the separate reduce launch and lets the epilogue fold BN
// statistics of split launches.  Returns false for the blocks that are done.
constexpr int kSkMax = 8;   // slabs an in-launch combine takes (sk_ok)
template <int BM, int BN>
__device__ __forceinline__ bool sk_combine(const XArgs& a, float* Ct, const long long* orow, int g, int zc, int kz,
                                           int n0, int* flag) {
  constexpr int C4 = BN / 4, IT = BM * C4 / 256;
  static_assert(BM * C4 % 256 == 0, "whole float4 passes");
  const int tid = threadIdx.x, S = a.splitk;
  const float* base = a.sk_ws + (long long)g * a.sk_gstride;
  int off[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int e = tid + it * 256, row = e / C4, cc = (e - row * C4) * 4, n = n0 + cc;
    const long long o = orow[row];
    off[it] = (o < 0 || n >= a.Ncol) ? kOOB : (int)((o + n) * 4);
  }
  {
    const __amdgpu_buffer_rsrc_t rs = rsrc(base + (long long)kz * a.zstride, a.sk_gstride * 4);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = tid + it * 256, row = e / C4, cc = (e - row * C4) * 4;
      const float4 v = *(const float4*)&Ct[row * BN + cc];
      if (off[it] != kOOB)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), rs, off[it], 0, 16);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its slab
  __syncthreads();
  if (tid == 0) {
    int* cnt = a.sk_cnt + ((long long)g * gridDim.x + blockIdx.x) * (gridDim.z / S) + zc;
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == S - 1;
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // reusable
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // loads stay below the ticket
  float4 w[kSkMax][IT];
#pragma unroll
  for (int z = 0; z < kSkMax; ++z) {
    if (z < S && z != kz) {
      const __amdgpu_buffer_rsrc_t rz = rsrc(base + (long long)z * a.zstride, a.sk_gstride * 4);
#pragma unroll
      for (int it = 0; it < IT; ++it)
        w[z][it] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rz, off[it], 0, 16));
    }
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int e = tid + it * 256, row = e / C4, cc = (e - row * C4) * 4;
    float4* cp = (float4*)&Ct[row * BN + cc];
    const float4 own = *cp;
    float4 v = kz == 0 ? own : w[0][it];
#pragma unroll
    for (int z = 1; z < kSkMax; ++z) {
      if (z < S) {
        const float4 u = z == kz ? own : w[z][it];
        v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
      }
    }
    if (off[it] != kOOB) *cp = v;
  }
  __syncthreads();
  return true;
}

// register budget (minimum workgroups per CU): 3 lets the 128x64 / 64x128 / 32x128 tiles keep
// their accumulators in VGPRs within 168 registers (3 waves per SIMD, no spills; the 128x128
// tiles stay at 2, LDS-bound).  Those tiles run the short-K stride-2 and 1x1 convs, whose
// prologue / epilogue a third resident workgroup hides: eval.l2.0.conv1 163 vs 156 TF,
// l2.0.sc 43 vs 33, training l2.0.conv1 fwd 134 vs 120, l3/l4 dgrad +7 %, headline 3.25 vs
// 3.16 rounds/s same box (profiles/r4/minb3/).  (1 -> 2 changed nothing: profiles/r4/minb/.)
// The 128x128 eval tiles are operand-fetch bound (profiles/r4/ximg/README.md), not MFMA bound.
#ifndef XCONV_MINB
#define XCONV_MINB 3
#endif
// KS: the K range runs as a.kslab slabs inside the block — each slab's MFMAs accumulate from
// zero, are scaled back (HScale) and added to a running fp32 sum in slab order — the exact
// arithmetic of a.kslab split-K launches summed in z order (xsplitk_reduce / sk_combine), so a
// grouped launch reproduces a lone client's split-K bits without the slab round trip through
// HBM or the separate reduce / statistics pass
// (A 4-stage register pipeline for the lone client's 32 x 128 tiles — loads issued 4 k-steps
// ahead instead of 2 — measured no faster: lone step 1.640 / 1.638 vs 1.646 / 1.589 ms, same
// box, profiles/r5/deep/.  Those launches are not bound by operand-load latency.)
template <int BM, int BN, int WM, int WN, int VEC, bool PW = false, bool LZ = false, bool KS = false>
__global__ __launch_bounds__(256, KS ? 2 : XCONV_MINB) void xconv_kernel(const XArgs a) {
  static_assert(!LZ || VEC >= 4, "lazy BN operand: 4-channel vectors");
  static_assert(!PW || VEC >= 4, "pre-split weights: vector loads");
  constexpr int P = 2;
  constexpr int TM = BM / WM, TN = BN / WN, MI = TM / 32, NJ = TN / 32;
  static_assert(WM * WN == 4 && MI >= 1 && NJ >= 1, "wave tiling");
  constexpr int ROWS = BM + BN, PL = ROWS * 4;   // uint4 per plane image
  constexpr int RA = BM / 32, RB = BN / 32;      // 4-element quarters per thread (A, B)
  static_assert(BM * BN <= 2 * P * PL * 4, "epilogue tile fits the LDS images");
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * P * PL];
  __shared__ long long orow[BM];
  __shared__ __attribute__((aligned(16))) float lzc[LZ ? 1024 : 4];   // lazy operand: scale | shift

  const int zc = blockIdx.z / a.splitk, kz = blockIdx.z - zc * a.splitk;
  const XClass c = a.cls[zc];
  const int g = blockIdx.y;
  const int HqWq = c.Hq * c.Wq;
  const int Mv = valid_rows(a.nvalid, g, a.N) * HqWq;
  const int tn = blockIdx.x % a.tiles_n, tm = blockIdx.x / a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mv) return;
  const int slot = a.wsel ? a.wsel[g] : g;
  const int Cs = a.Cs;
  if constexpr (LZ) {   // the source BN's scale / shift (Cs <= 512: checked on the host)
    const float* cf = a.lz_coef + (long long)g * kBnRows * Cs;
    for (int c = threadIdx.x; c < Cs; c += 256) {
      lzc[c] = cf[kCScale * Cs + c];
      lzc[512 + c] = cf[kCShift * Cs + c];
    }
  }
  const int K = c.nI * c.nJ * Cs;
  const int nkt = (K + 31) >> 5;
  const int kt0 = (int)((long long)nkt * kz / a.splitk), kt1 = (int)((long long)nkt * (kz + 1) / a.splitk);
  const float* __restrict__ src = a.src + (long long)g * a.src_gstride;
  const float* __restrict__ Bp = a.w + (long long)slot * a.w_sstride + c.boff;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int kq = tid & 7, r0 = tid >> 3;

  if (tid < BM) {
    const int m = m0 + tid;
    long long o = -1;
    if (m < Mv) {
      if (a.splitk > 1) {
        o = (long long)m * a.Ncol;
      } else {
        const int img = m / HqWq, rem = m - img * HqWq, p = rem / c.Wq, q = rem - p * c.Wq;
        o = (((long long)img * a.Ho + p * a.os + c.oh) * a.Wo + q * a.os + c.ow) * a.Ncol;
      }
    }
    orow[tid] = o;
  }
  // the thread's A rows (source pixel bases) and B rows (weight rows)
  // 32-bit element offsets (a replica's source is < 2^31 elements: checked on the host); an
  // invalid row gets an out-of-range ah so the bounds test alone zero-fills it
  int abase[RA], ah[RA], aw[RA];
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    const int m = m0 + r0 + 32 * i;
    abase[i] = 0; ah[i] = -(1 << 20); aw[i] = 0;
    if (m < Mv) {
      const int img = m / HqWq, rem = m - img * HqWq, p = rem / c.Wq, q = rem - p * c.Wq;
      ah[i] = p * a.sp + c.bh;
      aw[i] = q * a.sp + c.bw;
      abase[i] = ((img * a.Hs + ah[i]) * a.Ws + aw[i]) * Cs;
    }
  }
  // B rows: element offsets within the class's weight block (-1: past Ncol)
  int boffs[RB];
#pragma unroll
  for (int j = 0; j < RB; ++j) {
    const int n = n0 + r0 + 32 * j;
    boffs[j] = n < a.Ncol ? n * K : -1;
  }
  const __amdgpu_buffer_rsrc_t rA = rsrc(src, (long long)a.N * a.Hs * a.Ws * Cs * 4);
  const __amdgpu_buffer_rsrc_t rB = rsrc(Bp, (long long)a.Ncol * K * 4);
  // PW: the two fp16 planes of the weights (same element offsets, 2 B each)
  const uint16_t* Bh = PW ? a.wp + (long long)slot * a.wp_sstride + c.boff : nullptr;
  const __amdgpu_buffer_rsrc_t rBh = rsrc(Bh, (long long)a.Ncol * K * 2);
  const __amdgpu_buffer_rsrc_t rBl = rsrc(PW ? Bh + (a.wp_sstride >> 1) : nullptr, (long long)a.Ncol * K * 2);
  // reduction state of the thread's quarter: element k = kt*32 + kq*4 is channel kc of tap (ki, kj)
  int ki = 0, kj = 0, kc = 0;
  if (nkt > 0) {
    const int k = kt0 * 32 + kq * 4;
    const int t = k / Cs;
    kc = k - t * Cs;
    ki = t / c.nJ;
    kj = t - ki * c.nJ;
  }
  // two register stages: step kt+1 (stage (kt+1)&1) is split into the other LDS buffer in the
  // gaps of step kt's MFMAs, and each quarter's registers are reloaded with step kt+3 right
  // after its split, so a load has ~2 MFMA steps to land
  float4 ra[2][RA], rb[2][RB];
  int g_kb = 0, g_toff = 0, g_dh = 0, g_dw = 0;   // VEC >= 4: the prepared step's geometry
  bool g_kv = false;
  int g_kc = 0;                                   // LZ: the prepared step's first channel
  int s_kq[2][RA];                                // LZ: per stage / A quarter: channel | in-image << 16
  int e_off[4], e_dh[4], e_dw[4];                 // VEC 1: per element
  bool e_kv[4];
  auto gprep = [&]() __attribute__((always_inline)) {   // the step at the current reduction state, then advance it
    g_kb = (ki * c.nJ + kj) * Cs + kc;   // == kt*32 + kq*4
    g_kc = kc;
    if constexpr (VEC >= 4) {
      g_kv = ki < c.nI;
      g_dh = a.dsg * ki;
      g_dw = a.dsg * kj;
      g_toff = (g_dh * a.Ws + g_dw) * Cs + kc;   // uniform across the rows
    } else {
      int ii = ki, jj = kj, cc = kc;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        e_kv[e] = ii < c.nI;
        e_dh[e] = a.dsg * ii;
        e_dw[e] = a.dsg * jj;
        e_off[e] = (e_dh[e] * a.Ws + e_dw[e]) * Cs + cc;
        if (++cc == Cs) {
          cc = 0;
          if (++jj == c.nJ) { jj = 0; ++ii; }
        }
      }
    }
    // k += 32 (Cs % 32 == 0: at most one tap boundary)
    kc += 32;
    if constexpr (VEC == 32) {
      if (kc >= Cs) {
        kc -= Cs;
        if (++kj == c.nJ) { kj = 0; ++ki; }
      }
    } else {
      while (kc >= Cs) {
        kc -= Cs;
        if (++kj == c.nJ) { kj = 0; ++ki; }
      }
    }
  };
  auto gq = [&](int st, int q) __attribute__((always_inline)) {   // quarter q (A rows first) of the prepared step -> stage st
    if (q < RA) {
      if constexpr (VEC >= 4) {
        const bool ok = g_kv && (unsigned)(ah[q] + g_dh) < (unsigned)a.Hs && (unsigned)(aw[q] + g_dw) < (unsigned)a.Ws;
        ra[st][q] = bload4(rA, ok ? (abase[q] + g_toff) * 4 : kOOB);
        if constexpr (LZ) s_kq[st][q] = g_kc | ((int)ok << 16);
      } else {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool ok = e_kv[e] && (unsigned)(ah[q] + e_dh[e]) < (unsigned)a.Hs &&
                          (unsigned)(aw[q] + e_dw[e]) < (unsigned)a.Ws;
          v[e] = bload1(rA, ok ? (abase[q] + e_off[e]) * 4 : kOOB);
        }
        ra[st][q] = make_float4(v[0], v[1], v[2], v[3]);
      }
    } else {
      const int j = q - RA;
      if constexpr (PW) {   // planes, as the bits of one float4
        const int off = (boffs[j] >= 0 && g_kb < K) ? (boffs[j] + g_kb) * 2 : kOOB;
        const uint2 h = bload8(rBh, off), l = bload8(rBl, off);
        rb[st][j] = __builtin_bit_cast(float4, make_uint4(h.x, h.y, l.x, l.y));
      } else if constexpr (VEC >= 4) {
        rb[st][j] = bload4(rB, (boffs[j] >= 0 && g_kb < K) ? (boffs[j] + g_kb) * 4 : kOOB);
      } else {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = bload1(rB, (boffs[j] >= 0 && g_kb + e < K) ? (boffs[j] + g_kb + e) * 4 : kOOB);
        rb[st][j] = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  };
  auto gload = [&](int st) __attribute__((always_inline)) {
    gprep();
#pragma unroll
    for (int q = 0; q < RA + RB; ++q) gq(st, q);
  };
  // quarter q of stage st -> LDS buffer buf
  HScale hs;
  hs.init(amax_read(a.amax_src, a.amax_src_ld, g), amax_read(a.amax_w, a.amax_w_ld, slot));
  auto lput_q = [&](int buf, int st, int q) __attribute__((always_inline)) {
    uint4* L = lds + buf * P * PL;
    uint2 sp[P];
    if (q < RA) {
      if constexpr (LZ) {   // relu?(fma(y, scale, shift)) in the image, 0 in the padding
        const int kq4 = s_kq[st][q] & 0xffff;
        const bool ok = (s_kq[st][q] >> 16) != 0;
        const float4 sc = *(const float4*)&lzc[kq4], sh = *(const float4*)&lzc[512 + kq4];
        float4 v = ra[st][q];
        v.x = fmaf(v.x, sc.x, sh.x); v.y = fmaf(v.y, sc.y, sh.y); v.z = fmaf(v.z, sc.z, sh.z); v.w = fmaf(v.w, sc.w, sh.w);
        if (a.lz_relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
        if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
        split4h(v.x, v.y, v.z, v.w, hs.ma, sp);
      } else {
        split4h(ra[st][q].x, ra[st][q].y, ra[st][q].z, ra[st][q].w, hs.ma, sp);
      }
      lds_put<P, false, BM>(L, PL, 0, r0 + 32 * q, kq, sp);
    } else {
      const int j = q - RA;
      if constexpr (PW) {
        const uint4 u = __builtin_bit_cast(uint4, rb[st][j]);
        sp[0] = make_uint2(u.x, u.y);
        sp[1] = make_uint2(u.z, u.w);
      } else {
        split4h(rb[st][j].x, rb[st][j].y, rb[st][j].z, rb[st][j].w, hs.mb, sp);
      }
      lds_put<P, false, BN>(L, PL, BM, r0 + 32 * j, kq, sp);
    }
  };

  f32x16_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if constexpr (LZ) __syncthreads();   // lzc
  // KS: the running sum of the finished slabs, the next slab boundary
  [[maybe_unused]] f32x16_t ssum[KS ? MI : 1][KS ? NJ : 1];
  [[maybe_unused]] int zs = 1, kb_next = KS ? (int)((long long)nkt / a.kslab) : 0;
  auto slab_end = [&](int kt_done) __attribute__((always_inline)) {   // after step kt_done
    if constexpr (KS) {
      if (kt_done + 1 == kb_next) {
        hs.finish(acc);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              ssum[i][j][r] = zs == 1 ? acc[i][j][r] : ssum[i][j][r] + acc[i][j][r];
              acc[i][j][r] = 0.f;
            }
        ++zs;
        kb_next = (int)((long long)nkt * zs / a.kslab);
      }
    }
  };
  if (kt0 < kt1) {
    // loads past the slice's last step are harmless (past K they zero-fill), so the loop body
    // has no branches and the accumulators stay in place across iterations
    gload(0);
    gload(1);
    gprep();   // step kt0+2
#pragma unroll
    for (int q = 0; q < RA + RB; ++q) {
      lput_q(0, 0, q);
      gq(0, q);
    }
    __syncthreads();
    // step kt (offset from kt0 even: LDS buffer 0, successor in register stage 1; odd: swapped)
    int kt = kt0;
    for (; kt + 1 < kt1; kt += 2) {
      gprep();   // step kt+3
      mma_step<MI, NJ, P, true, false, BM, BN, RA + RB>(lds, PL, wm * TM, wn * TN, acc, lane, [&](int q) __attribute__((always_inline)) {
        lput_q(1, 1, q);
        gq(1, q);
      });
      slab_end(kt);
      __syncthreads();
      gprep();   // step kt+4
      mma_step<MI, NJ, P, true, false, BM, BN, RA + RB>(lds + P * PL, PL, wm * TM, wn * TN, acc, lane, [&](int q) __attribute__((always_inline)) {
        lput_q(0, 0, q);
        gq(0, q);
      });
      slab_end(kt + 1);
      __syncthreads();
    }
    if (kt < kt1) {
      mma_step<MI, NJ, P, true, false, BM, BN, 0>(lds, PL, wm * TM, wn * TN, acc, lane, [&](int) {});
      slab_end(kt);
    }
  }
  if constexpr (KS) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = ssum[i][j];
  } else {
    hs.finish(acc);
  }

  // ---- epilogue: fp32 tile through LDS, row-contiguous stores with bias / residual / ReLU
  __syncthreads();
  float* Ct = reinterpret_cast<float*>(lds);
  const int fr = lane & 31, hf = lane >> 5;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        Ct[(wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf) * BN + wn * TN + j * 32 + fr] = acc[i][j][r];
  __syncthreads();
  bool fin = a.splitk == 1;
  if constexpr (BM == 32 && BN == 128) {   // the only tile sk_ok admits
    if (!fin && a.sk_cnt) {
      __shared__ int sk_last;
      if (!sk_combine<BM, BN>(a, Ct, orow, g, zc, kz, n0, &sk_last)) return;
      fin = true;
    }
  }
  const int bfm = fin ? a.bf.mode : 0;   // fused training BN of the output (bnfuse.hpp)
  float* out = a.out + (long long)g * a.out_gstride + (fin ? 0 : (long long)kz * a.zstride);
  const float* bias = (fin && a.bias) ? a.bias + (long long)slot * a.b_sstride : nullptr;
  const float* res = (fin && a.res) ? a.res + (long long)g * a.out_gstride : nullptr;
  const bool relu = fin && a.relu;
  float vmax = 0.f;
  if ((a.Ncol & 3) == 0) {
    constexpr int C4 = BN / 4;
    for (int e = tid; e < BM * C4; e += 256) {
      const int row = e / C4, cc = (e - row * C4) * 4;
      const int n = n0 + cc;
      const long long o = orow[row];
      if (o < 0 || n >= a.Ncol) continue;
      float4 v = *(const float4*)&Ct[row * BN + cc];
      if (bias) { v.x += bias[n]; v.y += bias[n + 1]; v.z += bias[n + 2]; v.w += bias[n + 3]; }
      if (res) {
        const float4 rv = *(const float4*)(res + o + n);
        v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
      }
      if (relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
      if (bfm == 2) {   // backward: d = the gradient where the BN(+ReLU) output is > 0
        v = bnf_mask4(a.bf, g, o, n, v);
        *(float4*)&Ct[row * BN + cc] = v;
      }
      vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      *(float4*)(out + o + n) = v;
    }
  } else {
    for (int e = tid; e < BM * BN; e += 256) {
      const int row = e / BN, cc = e - row * BN;
      const int n = n0 + cc;
      const long long o = orow[row];
      if (o < 0 || n >= a.Ncol) continue;
      float v = Ct[row * BN + cc];
      if (bias) v += bias[n];
      if (res) v += res[o + n];
      if (relu) v = fmaxf(v, 0.f);
      vmax = fmaxf(vmax, fabsf(v));
      out[o + n] = v;
    }
  }
  if (fin && a.amax_out) amax_fold(a.amax_out, a.amax_out_ld, g, vmax);
  if (bfm) {
    __syncthreads();   // d in Ct (backward)
    bnf_tile_records<BM, BN>(a.bf, Ct, orow, g, m0, n0, Mv);
  }
}

// ======================================================================= halo conv
// Stride-1 3x3 conv (pad 1) and the stride-1 data gradient, for the narrow ResNet stages
// (W 32 / 16, Cs 32 / 64): the block's input patch ((TR+2) x (W+2) pixels x Cs) is loaded and
// split into bf16 planes ONCE and every tap's A fragments are read from it at the tap's pixel
// offset.  The implicit GEMM (xconv_kernel) re-stages and re-splits every input element once
// per tap (9x), which makes the split VALU — not the MFMA — the bound of these layers.  The
// weights stream through the same two-stage register/LDS pipeline as in xconv_kernel; the
// k-step order (tap-major, 32 channels per step) and the MFMA sequence per output element are
// the same, so both kernels compute identical bits.
// Patch image: pixel pp (patch column c = pp % (W + 2)) holds CH 16-B chunks, chunk q at
// q ^ hswz.  CH 4 (Cs 32): swizzle by pixel, (pp >> 2) & 3 — conflict-free.  CH 8 (Cs 64,
// 128 B per pixel, two pixels per 256-B bank row): a ds_read_b128 lane group of a wave reads
// 8 pixels of one patch row (columns c0+{0..3, 12..15}) and 8 of the next (c0+{4..11}), or the
// mirror image; the bank slot is 8 * (c & 1) + (q ^ swz) & 7, and swz = (c >> 1) & 7 maps those
// 16 pixels to 16 distinct slots for every tap column c0 (the former (pp >> 1) & 7 put pixels
// 16 apart on one slot: 2-way conflicts on ~29 % of the LDS cycles, profiles/pmc_eval_r3.md).

// SC (evaluation, a downsampling block's conv2 at W 16): the block's 1x1 stride-2 shortcut conv
// (32 input channels: one k-step) runs after the 18 3x3 steps from its own LDS tile
// (x2[2h][2w] of the block's 128 output pixels, loaded and split at the start), with its own
// fp16 scales (the accumulators are rescaled once, exactly) and pre-split weights; its output is
// never written or read back as a residual (reference models/resnet_cifar.py:24-36).
template <int W, int CS, int BM, int BN, int WM, int WN, bool PRE = false, bool LZ = false, bool SC = false>
__global__ __launch_bounds__(256) void xhalo_kernel(const XArgs a) {
  static_assert(!SC || (PRE && !LZ), "fused shortcut: evaluation, pre-split weights");
  constexpr int P = 2;
  constexpr int TR = BM / W, PW = W + 2, PR = TR + 2, PP = PR * PW;
  constexpr int CH = CS / 8, PATCH = PP * CH;             // uint4 per plane
  constexpr int TM = BM / WM, TN = BN / WN, MI = TM / 32, NJ = TN / 32;
  static_assert(WM * WN == 4 && MI >= 1 && NJ >= 1 && BM % W == 0, "tiling");
  constexpr int RB = BN / 32;                             // weight quarters per thread
  constexpr int BPL = BN * 4;                             // uint4 per weight plane (BN rows x 64 B)
  constexpr int NK = 9 * CS / 32;                         // k-steps
  constexpr int CB = CS / 32;                             // channel blocks per tap
  static_assert(BM * BN <= P * PATCH * 4, "epilogue tile fits the patch");
  constexpr int NKT = NK + (SC ? 1 : 0);                  // + the shortcut's k-step
  constexpr int SPL = BM * 4;                             // SC: uint4 per plane of the shortcut tile
  __shared__ __attribute__((aligned(16))) uint4 patch[P * PATCH];
  __shared__ __attribute__((aligned(16))) uint4 bring[2 * P * BPL];
  __shared__ __attribute__((aligned(16))) uint4 scbuf[SC ? P * SPL : 4];
  __shared__ long long orow[BM];

  const int g = blockIdx.y;
  const int HT = a.Ho / TR;                               // row tiles per image
  const int tn = blockIdx.x % a.tiles_n, tm = blockIdx.x / a.tiles_n;
  const int img = tm / HT, h0 = (tm - img * HT) * TR;
  const int n0 = tn * BN;
  const int nv_img = valid_rows(a.nvalid, g, a.N);
  if (img >= nv_img) return;
  const int slot = a.wsel ? a.wsel[g] : g;
  const int K = 9 * CS;
  const float* __restrict__ src = a.src + (long long)g * a.src_gstride;
  const float* __restrict__ Bp = a.w + (long long)slot * a.w_sstride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int kq = tid & 7, r0 = tid >> 3;
  const bool flip = a.dsg < 0;                            // data gradient: tap (i, j) reads (2-i, 2-j)

  if (tid < BM)
    orow[tid] = (((long long)img * a.Ho + h0 + tid / W) * a.Wo + tid % W) * a.Ncol;

  // ---- the input patch: rows h0-1 .. h0+TR, cols -1 .. W, loaded to registers, split once
  // into P planes (after the block-wide max under H)
  constexpr int Q4 = CS / 4;                              // float4 quarters per pixel
  constexpr int NE = (PP * Q4 + 255) / 256;
  float4 pv[NE];
  {
    const __amdgpu_buffer_rsrc_t rA = rsrc(src, (long long)a.N * a.Hs * a.Ws * CS * 4);
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + 256 * u;
      const int pp = e / Q4, q = e - pp * Q4;
      const int pr = pp / PW, pc = pp - pr * PW;
      const int h = h0 - 1 + pr, w = pc - 1;
      const bool ok = e < PP * Q4 && (unsigned)h < (unsigned)a.Hs && (unsigned)w < (unsigned)a.Ws;
      pv[u] = bload4(rA, ok ? (((img * a.Hs + h) * a.Ws + w) * CS + q * 4) * 4 : kOOB);
    }
  }
  // SC: the shortcut tile, x2[img][2(h0 + r)][2c][0 .. 32) of the block's BM output pixels
  constexpr int NS = SC ? BM * 8 / 256 : 1;
  [[maybe_unused]] float4 sv[NS];
  if constexpr (SC) {
    const __amdgpu_buffer_rsrc_t rS = rsrc(a.sc_src + (long long)g * a.sc_gstride,
                                           (long long)a.N * a.sc_H * a.sc_W * 32 * 4);
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int e = tid + 256 * u, px = e >> 3, q = e & 7;
      const int h = 2 * (h0 + px / W), w = 2 * (px % W);
      const bool ok = h < a.sc_H && w < a.sc_W;
      sv[u] = bload4(rS, ok ? (((img * a.sc_H + h) * a.sc_W + w) * 32 + q * 4) * 4 : kOOB);
    }
  }
  HScale hs;
  hs.init(amax_read(a.amax_src, a.amax_src_ld, g), amax_read(a.amax_w, a.amax_w_ld, slot));
  [[maybe_unused]] int s_sc = 0;
  if constexpr (SC) {
    const int sx = hexp(amax_read(a.sc_amax_src, a.sc_amax_src_ld, g));
    s_sc = sx + hexp(amax_read(a.sc_amax_w, a.sc_amax_w_ld, slot));
    const float m = __uint_as_float((uint32_t)(sx + 127) << 23);
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int e = tid + 256 * u;
      uint2 sp[P];
      split4h(sv[u].x, sv[u].y, sv[u].z, sv[u].w, m, sp);
      lds_put<P, false, BM>(scbuf, SPL, 0, e >> 3, e & 7, sp);
    }
  }
  const float* lzc = LZ ? a.lz_coef + (long long)g * kBnRows * CS : nullptr;
  auto patch_put = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + 256 * u;
      if (e >= PP * Q4) break;
      const int pp = e / Q4, q = e - pp * Q4;
      uint2 sp[P];
      if constexpr (LZ) {   // relu?(fma(y, scale, shift)) in the image, 0 in the padding
        const int pr = pp / PW, pc = pp - pr * PW;
        const int h = h0 - 1 + pr, w = pc - 1;
        const bool ok = (unsigned)h < (unsigned)a.Hs && (unsigned)w < (unsigned)a.Ws;
        const float4 sc = *(const float4*)(lzc + kCScale * CS + q * 4), sh = *(const float4*)(lzc + kCShift * CS + q * 4);
        float4 v = pv[u];
        v.x = fmaf(v.x, sc.x, sh.x); v.y = fmaf(v.y, sc.y, sh.y); v.z = fmaf(v.z, sc.z, sh.z); v.w = fmaf(v.w, sc.w, sh.w);
        if (a.lz_relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
        if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
        split4h(v.x, v.y, v.z, v.w, hs.ma, sp);
      } else {
        split4h(pv[u].x, pv[u].y, pv[u].z, pv[u].w, hs.ma, sp);
      }
      const int o = pp * CH + ((q >> 1) ^ hswz<W, CS>(pp, pp % PW));
#pragma unroll
      for (int p = 0; p < P; ++p) ((uint2*)&patch[p * PATCH + o])[q & 1] = sp[p];
    }
  };

  // ---- weights: two-stage pipeline (k-step t: tap t / CB, channels (t % CB) * 32 ..)
  int boffs[RB];
#pragma unroll
  for (int j = 0; j < RB; ++j) {
    const int n = n0 + r0 + 32 * j;
    boffs[j] = n < a.Ncol ? n * K : -1;
  }
  const __amdgpu_buffer_rsrc_t rB = rsrc(Bp, (long long)a.Ncol * K * 4);
  const uint16_t* Bh = PRE ? a.wp + (long long)slot * a.wp_sstride : nullptr;
  const __amdgpu_buffer_rsrc_t rBh = rsrc(Bh, (long long)a.Ncol * K * 2);
  const __amdgpu_buffer_rsrc_t rBl = rsrc(PRE ? Bh + (a.wp_sstride >> 1) : nullptr, (long long)a.Ncol * K * 2);
  float4 rb[2][RB];
  [[maybe_unused]] const uint16_t* Sh = SC ? a.sc_wp + (long long)slot * a.sc_wp_sstride : nullptr;
  [[maybe_unused]] const __amdgpu_buffer_rsrc_t rSh = rsrc(Sh, SC ? (long long)a.Ncol * 32 * 2 : 0);
  [[maybe_unused]] const __amdgpu_buffer_rsrc_t rSl = rsrc(SC ? Sh + (a.sc_wp_sstride >> 1) : nullptr,
                                                           SC ? (long long)a.Ncol * 32 * 2 : 0);
  auto gq = [&](int t, int st, int j) __attribute__((always_inline)) {   // quarter j of weight step t -> stage st
    const int kb = t * 32 + kq * 4;
    if (SC && t >= NK) {   // the shortcut's weights [Ncol][32]
      const int off = (boffs[j] >= 0 && t == NK) ? ((n0 + r0 + 32 * j) * 32 + kq * 4) * 2 : kOOB;
      const uint2 h = bload8(rSh, off), l = bload8(rSl, off);
      rb[st][j] = __builtin_bit_cast(float4, make_uint4(h.x, h.y, l.x, l.y));
      return;
    }
    if constexpr (PRE) {
      const int off = (boffs[j] >= 0 && kb < K) ? (boffs[j] + kb) * 2 : kOOB;
      const uint2 h = bload8(rBh, off), l = bload8(rBl, off);
      rb[st][j] = __builtin_bit_cast(float4, make_uint4(h.x, h.y, l.x, l.y));
    } else {
      rb[st][j] = bload4(rB, (boffs[j] >= 0 && kb < K) ? (boffs[j] + kb) * 4 : kOOB);
    }
  };
  auto gload = [&](int t, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < RB; ++j) gq(t, st, j);
  };
  auto lput_q = [&](int buf, int st, int q) __attribute__((always_inline)) {
    if (q >= RB) return;
    uint2 sp[P];
    if constexpr (PRE) {
      const uint4 u = __builtin_bit_cast(uint4, rb[st][q]);
      sp[0] = make_uint2(u.x, u.y);
      sp[1] = make_uint2(u.z, u.w);
    } else {
      split4h(rb[st][q].x, rb[st][q].y, rb[st][q].z, rb[st][q].w, hs.mb, sp);
    }
    lds_put<P, false, BN>(bring + buf * P * BPL, BPL, 0, r0 + 32 * q, kq, sp);
  };

  f32x16_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int fr = lane & 31, hf = lane >> 5;
  // patch pixel of each A fragment row at tap offset (0, 0)
  int apix[MI], acol[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = wm * TM + i * 32 + fr;
    apix[i] = (m / W) * PW + (m % W);
    acol[i] = m % W;
  }
  auto mma = [&](int t, int buf, int stn) __attribute__((always_inline)) {
    const bool scs = SC && t >= NK;
    const int tap = t / CB, cb = t - tap * CB;
    int ti = tap / 3, tj = tap - ti * 3;
    if (flip) { ti = 2 - ti; tj = 2 - tj; }
    const int toff = ti * PW + tj;
    const uint4* L = bring + buf * P * BPL;
    if (scs && t == NK) {   // the shortcut's products accumulate at their own scale (exact rescale)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = ldexpf(acc[i][j][r], s_sc - hs.s);
      hs.s = s_sc;
    }
    sfor<2>([&](auto KK) __attribute__((always_inline)) {
      const int ch = decltype(KK)::value * 2 + hf;
      uint4 af[P][MI], bfr[P][NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if (scs) {
          const int m = wm * TM + i * 32 + fr;
          const int o = m * 4 + (ch ^ ((m >> 2) & 3));
#pragma unroll
          for (int p = 0; p < P; ++p) af[p][i] = scbuf[p * SPL + o];
          continue;
        }
        const int pp = apix[i] + toff;
        const int o = pp * CH + ((cb * 4 + ch) ^ hswz<W, CS>(pp, acol[i] + tj));
#pragma unroll
        for (int p = 0; p < P; ++p) af[p][i] = patch[p * PATCH + o];
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = wn * TN + j * 32 + fr;
        const int o = n * 4 + (ch ^ ((n >> 2) & 3));
#pragma unroll
        for (int p = 0; p < P; ++p) bfr[p][j] = L[p * BPL + o];
      }
      mma_half<MI, NJ, P, true, RB, decltype(KK)::value>(af, bfr, acc, [&](int q) __attribute__((always_inline)) {
        lput_q(buf ^ 1, stn, q);
        gq(t + 3, stn, q);   // reload: step t+3 (past NK: zero-filled, never read)
      });
    });
  };


  gload(0, 0);
  gload(1, 1);
  patch_put();
#pragma unroll
  for (int q = 0; q < RB; ++q) {
    lput_q(0, 0, q);
    gq(2, 0, q);
  }
  __syncthreads();   // patch + first weight step
  int t = 0;
  for (; t + 1 < NKT; t += 2) {
    mma(t, 0, 1);
    __syncthreads();
    mma(t + 1, 1, 0);
    __syncthreads();
  }
  if (t < NKT) {
    mma(t, 0, 1);   // (its filler writes a buffer nobody reads)
    __syncthreads();
  }
  hs.finish(acc);

  // ---- epilogue through the (drained) patch memory
  float* Ct = reinterpret_cast<float*>(patch);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        Ct[(wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf) * BN + wn * TN + j * 32 + fr] = acc[i][j][r];
  __syncthreads();
  float* out = a.out + (long long)g * a.out_gstride;
  const float* bias = a.bias ? a.bias + (long long)slot * a.b_sstride : nullptr;
  const float* bias2 = (SC && a.sc_bias) ? a.sc_bias + (long long)slot * a.sc_b_sstride : nullptr;
  const float* res = a.res ? a.res + (long long)g * a.out_gstride : nullptr;
  constexpr int C4 = BN / 4;
  float vmax = 0.f;
  for (int e = tid; e < BM * C4; e += 256) {
    const int row = e / C4, cc = (e - row * C4) * 4;
    const int n = n0 + cc;
    if (n >= a.Ncol) continue;
    const long long o = orow[row];
    float4 v = *(const float4*)&Ct[row * BN + cc];
    if (bias2) {   // conv2's and the shortcut's folded biases, summed first (as ximg_kernel)
      const float4 b1 = bias ? *(const float4*)(bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
      v.x += b1.x + bias2[n]; v.y += b1.y + bias2[n + 1]; v.z += b1.z + bias2[n + 2]; v.w += b1.w + bias2[n + 3];
    } else if (bias) {
      v.x += bias[n]; v.y += bias[n + 1]; v.z += bias[n + 2]; v.w += bias[n + 3];
    }
    if (res) {
      const float4 rv = *(const float4*)(res + o + n);
      v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
    }
    if (a.relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
    if (a.bf.mode == 2) {   // backward: d = the gradient where the BN(+ReLU) output is > 0
      v = bnf_mask4(a.bf, g, o, n, v);
      *(float4*)&Ct[row * BN + cc] = v;
    }
    vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    *(float4*)(out + o + n) = v;
  }
  if (a.amax_out) amax_fold(a.amax_out, a.amax_out_ld, g, vmax);
  if (a.bf.mode) {
    __syncthreads();   // d in Ct (backward)
    const int Mv = nv_img * a.Ho * a.Wo;
    bnf_tile_records<BM, BN>(a.bf, Ct, orow, g, tm * BM, n0, Mv);
  }
}

// ================================================================ whole-image halo conv
// Stride-1 3x3 pad-1 evaluation forward of the small-image stages (W 16 / 8 / 4: ResNet stages
// 2-4 on 32x32 inputs; fp16 pair, weights pre-split at the eval fold).  The implicit GEMM
// re-fetches every input element once per tap, and at these shapes its operand fetch — not
// the MFMA — bounds it (eval.layer3 / 4 ran +37 / +43 % faster with the in-loop global loads
// removed, against +5 % without the in-loop barriers: profiles/r4/ximg).  Here a block owns
// IMGS whole images (BM = 128 or 256 output pixels) x BN output channels; the reduction runs
// channel-chunk-major (chunk of 32 channels, then its 9 taps): each chunk's zero-padded patch
// (IMGS x (W+2)^2 pixels x 32 channels) is loaded once, split once into the LDS patch, and
// read by all 9 taps at their pixel offsets — (W+2)^2 / W^2 = 1.27x / 1.56x / 2.25x of the
// image bytes instead of 9x.  The next chunk's patch is loaded into registers while the
// current chunk's 9 k-steps run (8 steps to land).
// 4 waves, 2 blocks per CU, one patch buffer: the next chunk is split + stored after the
// chunk's last barrier (one more barrier per chunk).  (An 8-wave BM-256 form with two patch
// buffers, the next chunk split in the MFMA gaps, was measured slower — one block per CU
// exposes its prologue / epilogue: eval.layer3 254 vs 314 TF, profiles/r4/ximg/README.md.)
// Weights: the two-stage register / LDS ring of xhalo_kernel.  Epilogue straight from the
// accumulators (a 32-lane row is 32 consecutive output channels: 128-B segments).
// (A fused downsampling shortcut as extra one-tap chunks — each refilling the patch, its loads
// prefetched only two k-steps ahead — measured slower than the shortcut conv + this kernel with a
// residual epilogue: 17 x 1024 images, layer3.0 1534 vs 1467 us, layer4.0 1370 vs 1142 us,
// profiles/r5/down/kbench_ximg_sc.log; the W-16 halo kernel's fused form wins: xhalo_kernel SC.)
// Deterministic; the chunk-major k order makes its bits differ from the tap-major implicit
// GEMM's (both fp32 level: tests hold both to the fp64 oracle).
template <int W, int IMGS, int BN, int WM, int WN, bool PRE>
__global__ __launch_bounds__(256) void ximg_kernel(const XArgs a) {
  constexpr int P = 2, NT = 256;
  constexpr int PW = W + 2, PI = PW * PW, PP = IMGS * PI;   // padded pixels per image / patch
  constexpr int CC = 32, CH = CC / 8, Q4 = CC / 4;          // chunk channels, 16-B chunks, float4 per pixel
  constexpr int PATCH = PP * CH;                            // uint4 per plane
  constexpr int BM = IMGS * W * W;
  constexpr int TM = BM / WM, TN = BN / WN, MI = TM / 32, NJ = TN / 32;
  static_assert(WM * WN == NT / 64 && MI >= 1 && NJ >= 1 && BM == 128, "tiling");
  constexpr int RPT = NT / 8;                               // weight rows staged per pass
  static_assert(BN % RPT == 0, "weight rows");
  constexpr int RB = BN / RPT, BPL = BN * 4;
  __shared__ __attribute__((aligned(16))) uint4 patch[P * PATCH];
  __shared__ __attribute__((aligned(16))) uint4 bring[2 * P * BPL];

  const int g = blockIdx.y;
  const int tn = blockIdx.x % a.tiles_n, tm = blockIdx.x / a.tiles_n;
  const int img0 = tm * IMGS, n0 = tn * BN;
  const int nv = min(valid_rows(a.nvalid, g, a.N), a.N);
  if (img0 >= nv) return;
  const int slot = a.wsel ? a.wsel[g] : g;
  const int Cs = a.Cs, K = 9 * Cs, NC = Cs / CC, NK = 9 * NC;
  const float* __restrict__ src = a.src + (long long)g * a.src_gstride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int kq = tid & 7, r0 = tid >> 3;
  const int fr = lane & 31, hf = lane >> 5;

  // ---- patch chunks: chunk cc of images img0 .. img0+IMGS-1, zero padding / invalid images
  constexpr int NE = (PP * Q4 + NT - 1) / NT;
  float4 pv[NE];
  const __amdgpu_buffer_rsrc_t rA = rsrc(src, (long long)a.N * W * W * Cs * 4);
  auto pload = [&](int cc) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + NT * u;
      const int pp = e / Q4, q = e - pp * Q4;
      const int im = pp / PI, rem = pp - im * PI;
      const int h = rem / PW - 1, w = rem % PW - 1, img = img0 + im;
      const bool ok = e < PP * Q4 && img < nv && (unsigned)h < (unsigned)W && (unsigned)w < (unsigned)W;
      pv[u] = bload4(rA, ok ? (((img * W + h) * W + w) * Cs + cc * CC + q * 4) * 4 : kOOB);
    }
  };
  HScale hs;
  auto ppiece = [&](int u, float m) __attribute__((always_inline)) {   // piece u of pv -> the patch
    const int e = tid + NT * u;
    if (e >= PP * Q4) return;
    const int pp = e / Q4, q = e - pp * Q4;
    const int prow = (pp % PI) / PW;   // patch row: the swizzle key
    uint2 sp[P];
    split4h(pv[u].x, pv[u].y, pv[u].z, pv[u].w, m, sp);
    const int o = pp * CH + ((q >> 1) ^ (prow & 3));
#pragma unroll
    for (int p = 0; p < P; ++p) ((uint2*)&patch[p * PATCH + o])[q & 1] = sp[p];
  };

  // ---- weights (pre-split planes, or fp32 split while staging: the same bits): two-stage
  // pipeline, k-step t = chunk t / 9, tap t % 9
  int bn_[RB];
#pragma unroll
  for (int j = 0; j < RB; ++j) {
    const int n = n0 + r0 + RPT * j;
    bn_[j] = n < a.Ncol ? n : -1;
  }
  const uint16_t* Bh = PRE ? a.wp + (long long)slot * a.wp_sstride : nullptr;
  const __amdgpu_buffer_rsrc_t rBh = rsrc(Bh, (long long)a.Ncol * K * 2);
  const __amdgpu_buffer_rsrc_t rBl = rsrc(PRE ? Bh + (a.wp_sstride >> 1) : nullptr, (long long)a.Ncol * K * 2);
  const __amdgpu_buffer_rsrc_t rB = rsrc(a.w + (long long)slot * a.w_sstride, (long long)a.Ncol * K * 4);
  uint4 rb[2][RB];
  auto gq = [&](int t, int st, int j) __attribute__((always_inline)) {
    const bool ok = bn_[j] >= 0 && t < NK;
    const int cc = t / 9, tap = t - cc * 9;
    const int kb = bn_[j] * K + tap * Cs + cc * CC + kq * 4;
    if constexpr (PRE) {
      const uint2 h = bload8(rBh, ok ? kb * 2 : kOOB), l = bload8(rBl, ok ? kb * 2 : kOOB);
      rb[st][j] = make_uint4(h.x, h.y, l.x, l.y);
    } else {
      rb[st][j] = __builtin_bit_cast(uint4, bload4(rB, ok ? kb * 4 : kOOB));
    }
  };
  auto lput_q = [&](int buf, int st, int q) __attribute__((always_inline)) {
    uint2 sp[P];
    if constexpr (PRE) {
      sp[0] = make_uint2(rb[st][q].x, rb[st][q].y);
      sp[1] = make_uint2(rb[st][q].z, rb[st][q].w);
    } else {
      const float4 v = __builtin_bit_cast(float4, rb[st][q]);
      split4h(v.x, v.y, v.z, v.w, hs.mb, sp);
    }
    lds_put<P, false, BN>(bring + buf * P * BPL, BPL, 0, r0 + RPT * q, kq, sp);
  };

  f32x16_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // patch pixel and patch row of each A fragment row at tap (0, 0).  LDS image: pixel pp holds
  // 4 16-B chunks, chunk c at c ^ (patch row & 3) — the rows of a 32-lane fragment read (W 8: 4
  // rows of 8 pixels, W 4: 2 images x 4 rows of 4) then hit 16 distinct 16-B bank slots in each
  // ds_read_b128 lane group at every tap (the 32-wide halo conv's (pp >> 2) & 3 left 2-way
  // conflicts here: SQ_LDS_BANK_CONFLICT 8.0e7 per launch, profiles/r4/final2/)
  int apix[MI], arow[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = wm * TM + i * 32 + fr;
    const int im = m / (W * W), rem = m - im * (W * W);
    apix[i] = im * PI + (rem / W) * PW + rem % W;
    arow[i] = rem / W;
  }
  // k-step t from weight buffer buf; fill: the weight ring's next step
  auto mma = [&](int t, int buf, int stn) __attribute__((always_inline)) {
    const int tap = t % 9, ti = tap / 3, tj = tap - ti * 3;
    const int toff = ti * PW + tj;
    const uint4* L = bring + buf * P * BPL;
    sfor<2>([&](auto KK) __attribute__((always_inline)) {
      const int ch = decltype(KK)::value * 2 + hf;
      uint4 af[P][MI], bfr[P][NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int pp = apix[i] + toff;
        const int o = pp * CH + (ch ^ ((arow[i] + ti) & 3));
#pragma unroll
        for (int p = 0; p < P; ++p) af[p][i] = patch[p * PATCH + o];
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = wn * TN + j * 32 + fr;
        const int o = n * 4 + (ch ^ ((n >> 2) & 3));
#pragma unroll
        for (int p = 0; p < P; ++p) bfr[p][j] = L[p * BPL + o];
      }
      mma_half<MI, NJ, P, true, RB, decltype(KK)::value>(af, bfr, acc, [&](int q) __attribute__((always_inline)) {
        lput_q(buf ^ 1, stn, q);
        gq(t + 3, stn, q);   // reload: step t+3 (past NK: zero-filled, never read)
      });
    });
  };
  auto step = [&](int t, int buf, int stn) __attribute__((always_inline)) {
    const int c = t / 9;
    mma(t, buf, stn);
    __syncthreads();
    if (t - 9 * c == 8 && c + 1 < NC) {   // the chunk's last k-step, another follows
#pragma unroll
      for (int u = 0; u < NE; ++u) ppiece(u, hs.ma);   // every read of the old patch is done
      if (c + 2 < NC) pload(c + 2);
      __syncthreads();
    }
  };

  hs.init(amax_read(a.amax_src, a.amax_src_ld, g), amax_read(a.amax_w, a.amax_w_ld, slot));
#pragma unroll
  for (int q = 0; q < RB; ++q) {
    gq(0, 0, q);
    gq(1, 1, q);
  }
  pload(0);
#pragma unroll
  for (int u = 0; u < NE; ++u) ppiece(u, hs.ma);
  if (NC > 1) pload(1);
#pragma unroll
  for (int q = 0; q < RB; ++q) {
    lput_q(0, 0, q);
    gq(2, 0, q);
  }
  __syncthreads();   // patch (chunk 0) + first weight step
  int t = 0;
  for (; t + 1 < NK; t += 2) {
    step(t, 0, 1);
    step(t + 1, 1, 0);
  }
  if (t < NK) step(t, 0, 1);
  hs.finish(acc);

  // ---- epilogue from the accumulators: bias, residual, ReLU, max
  float* out = a.out + (long long)g * a.out_gstride;
  const float* bias = a.bias ? a.bias + (long long)slot * a.b_sstride : nullptr;
  const float* res = a.res ? a.res + (long long)g * a.out_gstride : nullptr;
  float vmax = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = n0 + wn * TN + j * 32 + fr;
    if (n >= a.Ncol) continue;
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
        if (img0 + m / (W * W) >= nv) continue;
        const long long o = (long long)(img0 * W * W + m) * a.Ncol + n;
        float v = acc[i][j][r];
        if (bias) v += bv;
        if (res) v += res[o];
        if (a.relu) v = fmaxf(v, 0.f);
        vmax = fmaxf(vmax, fabsf(v));
        out[o] = v;
      }
  }
  if (a.amax_out) amax_fold(a.amax_out, a.amax_out_ld, g, vmax);
}

// sum of split-K slabs ws[z][g][m][n] (fixed z order) + bias (+ residual) (ReLU), valid rows
__global__ __launch_bounds__(256) void xsplitk_reduce_kernel(const float* __restrict__ ws, int S, long long zstride,
                                                             long long gstride, const int* __restrict__ nvalid, int N,
                                                             int HoWo, int Ncol, const float* __restrict__ bias,
                                                             long long b_sstride, const int* __restrict__ wsel,
                                                             const float* __restrict__ res, int relu,
                                                             float* __restrict__ out, int* __restrict__ amax_out,
                                                             int amax_ld) {
  const int g = blockIdx.y;
  const long long total = (long long)valid_rows(nvalid, g, N) * HoWo * Ncol;
  const float* __restrict__ bp = bias ? bias + (long long)(wsel ? wsel[g] : g) * b_sstride : nullptr;
  const long long base = (long long)g * gstride;
  float vmax = 0.f;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    float v = ws[base + e];
    for (int z = 1; z < S; ++z) v += ws[z * zstride + base + e];
    if (bp) v += bp[e % Ncol];
    if (res) v += res[base + e];
    if (relu) v = fmaxf(v, 0.f);
    vmax = fmaxf(vmax, fabsf(v));
    out[base + e] = v;
  }
  if (amax_out) amax_fold(amax_out, amax_ld, g, vmax);
}

// ============================================================================ wgrad
// x / magic division for the row decode (n < 2^24: exact after one correction)
struct FDiv {
  int d; float inv;
};
__device__ __forceinline__ int fdiv(int n, FDiv f) {
  int q = (int)((float)n * f.inv);
  if ((q + 1) * f.d <= n) ++q;
  if (q * f.d > n) --q;
  return q;
}

struct XWArgs {
  const float* dy; long long dy_gstride;   // [G][N*Ho*Wo][Cout]
  const float* x; long long x_gstride;     // [G][N][H][W][Cin]
  float* ws;                               // slabs [Z][G][Cout][K] (Z > 1)
  float* dw; long long dw_gstride;         // [G][Cout][K] (+=)
  const int* nvalid;
  int N, H, W, Cin, Ho, Wo, Cout, KW, stride, pad, K;
  int tiles_k, mchunk;
  const int* amax_dy;                      // max |dy| / |x| slots (common.hpp)
  const int* amax_x;
  int amax_dy_ld, amax_x_ld;
  FDiv dHoWo, dWo;
  // lazy x operand (bnfuse.hpp, XLZ): x = relu?(fma(y, scale, shift)) of the BN that produced
  // the conv's input (x points at y; zero in the padding).  (A lazy dy staged from (d, y) was
  // measured slower than bnx_dy_kernel's stored dy: profiles/r4/bnx/ab_steps.md.)
  const float* x_coef; int x_relu;
};

template <int BNO, int BK, int WN_, int WK_, int VEC, bool XLZ = false>
__global__ __launch_bounds__(256) void xwgrad_kernel(const XWArgs a) {
  constexpr int P = 2;
  constexpr int TNo = BNO / WN_, TK = BK / WK_, MI = TNo / 32, NJ = TK / 32;
  static_assert(WN_ * WK_ == 4 && MI >= 1 && NJ >= 1, "wave tiling");
  static_assert(BK == 128, "x micro-tiles: one per thread");
  constexpr int ROWS = BNO + BK, PL = ROWS * 4;
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * P * PL];

  const int g = blockIdx.y, z = blockIdx.z;
  const int tk = blockIdx.x % a.tiles_k, tn = blockIdx.x / a.tiles_k;
  const int n0 = tn * BNO, k0 = tk * BK;
  const int HoWo = a.Ho * a.Wo;
  const int Mv = valid_rows(a.nvalid, g, a.N) * HoWo;
  const int mb = z * a.mchunk, me = min(Mv, mb + a.mchunk);
  if (mb >= me) return;     // the reduce sums only the slabs of z < ceil(Mv / mchunk)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid / WK_, wk = wid % WK_;
  const float* __restrict__ dy = a.dy + (long long)g * a.dy_gstride;
  const float* __restrict__ x = a.x + (long long)g * a.x_gstride;
  const int m4 = tid & 7;     // micro-tile rows m4*4 .. m4*4+3 of the 32-row m tile

  // dy micro-tile: 4 m x 4 cout (threads < BNO*2)
  const int dn4 = tid >> 3;
  const bool dact = dn4 < BNO / 4;
  const int dn = n0 + dn4 * 4;
  // x micro-tile: 4 m x 4 k; the thread's k (tap, channel) are fixed for the whole block
  const int xk4 = tid >> 3;
  int xkh[4], xkw[4], xc[4];
  bool xkv[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = k0 + xk4 * 4 + e;
    xkv[e] = k < a.K;
    const int t = k / a.Cin;
    xc[e] = k - t * a.Cin;
    xkh[e] = t / a.KW;
    xkw[e] = t - xkh[e] * a.KW;
  }

  float dv[2][4][4], xv[2][4][4];   // [stage][m][n or k]
  unsigned s_xok[2] = {0u, 0u};     // XLZ: in-image bit (r * 4 + e) per stage
  float xsc[4], xsh[4];
  if constexpr (XLZ) {
    const float* cf = a.x_coef + (long long)g * kBnRows * a.Cin;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      xsc[e] = xkv[e] ? cf[kCScale * a.Cin + xc[e]] : 0.f;
      xsh[e] = xkv[e] ? cf[kCShift * a.Cin + xc[e]] : 0.f;
    }
  }

  // bounds-checked buffer loads (32-bit in-replica offsets: checked on the host)
  const __amdgpu_buffer_rsrc_t rD = rsrc(dy, (long long)a.N * HoWo * a.Cout * 4);
  const __amdgpu_buffer_rsrc_t rX = rsrc(x, (long long)a.N * a.H * a.W * a.Cin * 4);
  // dy rows (part 0) or x rows (part 1) of m-step mt -> stage st
  auto gpart = [&](int mt, int st, int part) __attribute__((always_inline)) {
    const int m0 = mt + m4 * 4;
    if constexpr (VEC == 4) {
      if (part == 0) {
        if (dact) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float4 v = bload4(rD, (m0 + r < me && dn < a.Cout) ? ((m0 + r) * a.Cout + dn) * 4 : kOOB);
            dv[st][r][0] = v.x; dv[st][r][1] = v.y; dv[st][r][2] = v.z; dv[st][r][3] = v.w;
          }
        }
        return;
      }
      unsigned okm = 0u;
      if (a.Wo % 4 == 0) {
        // the 4 rows are consecutive output pixels of one output row: decode once
        int img = 0, p = 0, q = 0;
        if (m0 < me) {
          img = fdiv(m0, a.dHoWo);
          const int rem = m0 - img * HoWo;
          p = fdiv(rem, a.dWo);
          q = rem - p * a.Wo;
        }
        const int h = p * a.stride - a.pad + xkh[0];
        const bool hok = xkv[0] && (unsigned)h < (unsigned)a.H;
        const int xrow = (img * a.H + h) * a.W;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int w = (q + r) * a.stride - a.pad + xkw[0];
          const bool ok = m0 + r < me && hok && (unsigned)w < (unsigned)a.W;
          const float4 v = bload4(rX, ok ? ((xrow + w) * a.Cin + xc[0]) * 4 : kOOB);
          xv[st][r][0] = v.x; xv[st][r][1] = v.y; xv[st][r][2] = v.z; xv[st][r][3] = v.w;
          okm |= ok ? (0xfu << (r * 4)) : 0u;
        }
      } else {
        // narrow outputs (Wo 2 / 1: the 64-wide stem's last stage): the 4 rows may span output
        // rows or images, decoded per row; the same 4 channel vectors as the scalar path loads
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + r;
          int img = 0, p = 0, q = 0;
          if (m < me) {
            img = fdiv(m, a.dHoWo);
            const int rem = m - img * HoWo;
            p = fdiv(rem, a.dWo);
            q = rem - p * a.Wo;
          }
          const int h = p * a.stride - a.pad + xkh[0], w = q * a.stride - a.pad + xkw[0];
          const bool ok = m < me && xkv[0] && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
          const float4 v = bload4(rX, ok ? (((img * a.H + h) * a.W + w) * a.Cin + xc[0]) * 4 : kOOB);
          xv[st][r][0] = v.x; xv[st][r][1] = v.y; xv[st][r][2] = v.z; xv[st][r][3] = v.w;
          okm |= ok ? (0xfu << (r * 4)) : 0u;
        }
      }
      if constexpr (XLZ) s_xok[st] = okm;
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + r;
        const bool mv = m < me;
        if (part == 0) {
          if (dact) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              dv[st][r][e] = bload1(rD, (mv && dn + e < a.Cout) ? (m * a.Cout + dn + e) * 4 : kOOB);
          }
          continue;
        }
        int img = 0, p = 0, q = 0;
        if (mv) {
          img = fdiv(m, a.dHoWo);
          const int rem = m - img * HoWo;
          p = fdiv(rem, a.dWo);
          q = rem - p * a.Wo;
        }
        const int hb = p * a.stride - a.pad, wb = q * a.stride - a.pad;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int h = hb + xkh[e], w = wb + xkw[e];
          const bool ok = mv && xkv[e] && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
          xv[st][r][e] = bload1(rX, ok ? (((img * a.H + h) * a.W + w) * a.Cin + xc[e]) * 4 : kOOB);
          if constexpr (XLZ) {
            if (r == 0 && e == 0) s_xok[st] = 0u;
            s_xok[st] |= ok ? (1u << (r * 4 + e)) : 0u;
          }
        }
      }
    }
  };
  auto gload = [&](int mt, int st) __attribute__((always_inline)) {
    gpart(mt, st, 0);
    gpart(mt, st, 1);
  };
  // piece q of stage st -> LDS buffer buf: q < 4 transposes dy column e = q, q >= 4 x column q-4
  HScale hs;
  hs.init(amax_read(a.amax_dy, a.amax_dy_ld, g), amax_read(a.amax_x, a.amax_x_ld, g));
  auto lput_q = [&](int buf, int st, int q) __attribute__((always_inline)) {
    uint4* L = lds + buf * P * PL;
    uint2 sp[P];
    if constexpr (XLZ) {
      if (q >= 4) {
        const int e = q - 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = fmaf(xv[st][r][e], xsc[e], xsh[e]);
          if (a.x_relu) v = fmaxf(v, 0.f);
          xv[st][r][e] = ((s_xok[st] >> (r * 4 + e)) & 1u) ? v : 0.f;
        }
      }
    }
    if (q < 4) {
      if (dact) {
        split4h(dv[st][0][q], dv[st][1][q], dv[st][2][q], dv[st][3][q], hs.ma, sp);
        lds_put<P, true, BNO>(L, PL, 0, dn4 * 4 + q, m4, sp);
      }
    } else {
      const int e = q - 4;
      split4h(xv[st][0][e], xv[st][1][e], xv[st][2][e], xv[st][3][e], hs.mb, sp);
      lds_put<P, true, BK>(L, PL, BNO, xk4 * 4 + e, m4, sp);
    }
  };

  f32x16_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // rows past the chunk zero-fill, so the loads of the steps past its end are harmless
  // two register stages; a stage's dy (x) registers are reloaded with the step two ahead as
  // soon as its 4 dy (x) pieces are split (see xconv_kernel)
  auto fill = [&](int buf, int st, int q, int mnext) __attribute__((always_inline)) {
    lput_q(buf, st, q);
    if (q == 3) gpart(mnext, st, 0);
    if (q == 7) gpart(mnext, st, 1);
  };
  gload(mb, 0);
  gload(mb + 32, 1);
#pragma unroll
  for (int q = 0; q < 8; ++q) fill(0, 0, q, mb + 64);
  __syncthreads();
  int mt = mb;
  for (; mt + 32 < me; mt += 64) {
    mma_step<MI, NJ, P, true, true, BNO, BK, 8>(lds, PL, wn * TNo, wk * TK, acc, lane,
                                             [&](int q) __attribute__((always_inline)) { fill(1, 1, q, mt + 96); });
    __syncthreads();
    mma_step<MI, NJ, P, true, true, BNO, BK, 8>(lds + P * PL, PL, wn * TNo, wk * TK, acc, lane,
                                             [&](int q) __attribute__((always_inline)) { fill(0, 0, q, mt + 128); });
    __syncthreads();
  }
  if (mt < me) mma_step<MI, NJ, P, true, true, BNO, BK, 0>(lds, PL, wn * TNo, wk * TK, acc, lane, [&](int) {});
  hs.finish(acc);

  // acc[i][j][r]: cout row n = n0 + wn*TNo + i*32 + (r&3) + 8*(r>>2) + 4*hf, k col = k0 + wk*TK + j*32 + fr
  const int fr = lane & 31, hf = lane >> 5;
  const bool direct = gridDim.z == 1;
  float* dst = direct ? a.dw + (long long)g * a.dw_gstride
                      : a.ws + ((long long)z * gridDim.y + g) * (long long)a.Cout * a.K;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k = k0 + wk * TK + j * 32 + fr;
      if (k >= a.K) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wn * TNo + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
        if (n >= a.Cout) continue;
        const long long o = (long long)n * a.K + k;
        if (direct) dst[o] += acc[i][j][r];
        else dst[o] = acc[i][j][r];
      }
    }
}

// dw[g] += sum over the first ceil(Mv_g / mchunk) slabs, in z order
__global__ __launch_bounds__(256) void xwgrad_reduce_kernel(const float* __restrict__ ws, int G, long long per,
                                                            const int* __restrict__ nvalid, int N, int HoWo,
                                                            int mchunk, float* __restrict__ dw, long long dw_gstride) {
  const int g = blockIdx.y;
  const int Mv = valid_rows(nvalid, g, N) * HoWo;
  const int nz = (Mv + mchunk - 1) / mchunk;
  if (nz == 0) return;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < per; e += (long long)gridDim.x * 256) {
    float v = 0.f;
    for (int z = 0; z < nz; ++z) v += ws[((long long)z * G + g) * per + e];
    dw[(long long)g * dw_gstride + e] += v;
  }
}

// the deferred weight-gradient reductions of a whole backward pass in one launch
// (blockIdx.y = descriptor, blockIdx.z = replica): same fixed z order as xwgrad_reduce_kernel
struct XWRDesc {   // all int64 (built from a torch int64 host tensor)
  long long ws, dw, dw_gstride, per, nvalid, N, HoWo, mchunk, G, unused;
};
constexpr int kXWRBatch = 24;
struct XWRBatch {
  XWRDesc d[kXWRBatch];
};

// ZG z-groups x (256 / ZG) lanes per block, a float4 of elements per lane: each lane sums the
// slabs z = zg, zg + ZG, ... (unrolled, so several slab loads are in flight instead of one
// serial chain of nz loads), then the group sums meet in LDS in z-group order.  ZG (16 for
// many slabs, 4 otherwise) and so the order depend on nz only (per-replica geometry), never
// on G: deterministic and world-size independent.
template <int ZG, bool V4>
__device__ __forceinline__ void xwr_body(const float* __restrict__ ws, long long zs, long long per, int nz,
                                         float* __restrict__ dw, float4* red) {
  constexpr int LN = 256 / ZG;   // lanes per z-group
  const int lane = threadIdx.x % LN, zg = threadIdx.x / LN;
  for (long long e0 = blockIdx.x * (LN * 4LL); e0 < per; e0 += (long long)gridDim.x * LN * 4) {
    const long long e = e0 + lane * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < per) {
#pragma unroll 4
      for (int z = zg; z < nz; z += ZG) {
        float4 v;
        if constexpr (V4) {
          v = *(const float4*)(ws + z * zs + e);
        } else {
          const float* p = ws + z * zs + e;
          v.x = p[0];
          v.y = e + 1 < per ? p[1] : 0.f;
          v.z = e + 2 < per ? p[2] : 0.f;
          v.w = e + 3 < per ? p[3] : 0.f;
        }
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    }
    if (zg > 0) red[(zg - 1) * LN + lane] = acc;
    __syncthreads();
    if (zg == 0 && e < per) {
#pragma unroll
      for (int q = 0; q < ZG - 1; ++q) {
        const float4 r = red[q * LN + lane];
        acc.x += r.x; acc.y += r.y; acc.z += r.z; acc.w += r.w;
      }
      const float a4[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (e + k < per) dw[e + k] += a4[k];
    }
    __syncthreads();
  }
}

template <bool V4>
__global__ __launch_bounds__(256) void xwgrad_reduce_batch_kernel(const XWRBatch b) {
  __shared__ float4 red[240];
  const XWRDesc& d = b.d[blockIdx.y];
  const int g = blockIdx.z;
  if (g >= (int)d.G) return;
  const int* nvalid = (const int*)d.nvalid;
  const int Mv = valid_rows(nvalid, g, (int)d.N) * (int)d.HoWo;
  const int nz = (Mv + (int)d.mchunk - 1) / (int)d.mchunk;
  if (nz == 0) return;
  const float* __restrict__ ws = (const float*)d.ws + (long long)g * d.per;
  float* __restrict__ dw = (float*)d.dw + (long long)g * d.dw_gstride;
  if (nz >= 32) xwr_body<16, V4>(ws, d.G * d.per, d.per, nz, dw, red);
  else xwr_body<4, V4>(ws, d.G * d.per, d.per, nz, dw, red);
}

// ====================================================================== dgrad weights
// wt[slot][class (ph,pw)][cin][i][j][cout] = w[slot][cout][kh0+i*s][kw0+j*s][cin]
// (kh0 = (ph + pad) % s): every tap belongs to exactly one parity class.
struct XTDesc {   // all int64 (built from a torch int64 host tensor)
  long long w, wt, w_sstride, Cout, KH, KW, Cin, stride, pad, unused;
};
constexpr int kXTBatch = 24;   // descriptors per launch, passed by value (graph-capture safe)
struct XTBatch {
  XTDesc d[kXTBatch];
};

// One 32 x 32 (cout x cin) tile of one tap per block iteration, transposed through LDS:
// coalesced reads along cin, coalesced writes along cout (the element-wise gather it replaces
// read every weight from a different cache line).  blockIdx.z = slot.
__global__ __launch_bounds__(256) void xtranspose_kernel(const XTBatch b, int slots, const int* __restrict__ nvalid) {
  __shared__ float tile[32][33];
  const XTDesc& d = b.d[blockIdx.y];
  const int s = (int)d.stride, KH = (int)d.KH, KW = (int)d.KW, Cin = (int)d.Cin, Cout = (int)d.Cout;
  const int pad = (int)d.pad;
  const int sl = blockIdx.z;
  if (nvalid && nvalid[sl] == 0) return;
  const int per = Cout * KH * KW * Cin;
  const float* __restrict__ w = (const float*)d.w + (long long)sl * d.w_sstride;
  float* __restrict__ wt = (float*)d.wt + (long long)sl * per;
  const int nco = (Cout + 31) >> 5, nci = (Cin + 31) >> 5;
  const int ntiles = KH * KW * nco * nci;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int tap = t / (nco * nci), rr = t - tap * nco * nci;
    const int cot = rr / nci, cit = rr - cot * nci;
    const int kh = tap / KW, kw = tap - kh * KW;
    // the tap's parity class (ph, pw): kh0 = (ph + pad) % s == kh % s
    const int kh0 = kh % s, kw0 = kw % s;
    const int ph = ((kh0 - pad) % s + s) % s, pw = ((kw0 - pad) % s + s) % s;
    const int cls = ph * s + pw;
    int base = 0, nI = 0, nJ = 0;
    for (int c = 0; c <= cls; ++c) {
      const int a = c / s, bb = c - a * s;
      const int h0 = (a + pad) % s, w0 = (bb + pad) % s;
      nI = h0 < KH ? (KH - h0 + s - 1) / s : 0;
      nJ = w0 < KW ? (KW - w0 + s - 1) / s : 0;
      if (c < cls) base += Cin * nI * nJ * Cout;
    }
    const int i = (kh - kh0) / s, j = (kw - kw0) / s;
#pragma unroll
    for (int k = ty; k < 32; k += 8) {
      const int co = cot * 32 + k, ci = cit * 32 + tx;
      tile[k][tx] = (co < Cout && ci < Cin) ? w[((co * KH + kh) * KW + kw) * Cin + ci] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int k = ty; k < 32; k += 8) {
      const int ci = cit * 32 + k, co = cot * 32 + tx;
      if (ci < Cin && co < Cout) wt[base + ((ci * nI + i) * nJ + j) * Cout + co] = tile[tx][k];
    }
    __syncthreads();
  }
}

// w [slots][per] fp32 (slot stride sstride) -> planes [slots][2][per] fp16 of w * 2^sb, sb from
// the slot's max |w| exactly as HScale computes it: a weight operand split once for all the
// blocks (and launches) that stage it
__device__ __forceinline__ void xsplit_w_body(const float* __restrict__ w, long long sstride, long long per,
                                              const int* __restrict__ amax, int ld, uint16_t* __restrict__ out,
                                              int sl, long long e0, long long e1, long long step) {
  const int sb = hexp(amax_read(amax, ld, sl));
  const float mb = __uint_as_float((uint32_t)(sb + 127) << 23);
  const float* __restrict__ src = w + (long long)sl * sstride;
  uint16_t* __restrict__ oh = out + (long long)sl * 2 * per;
  uint16_t* __restrict__ ol = oh + per;
  for (long long e = e0 + threadIdx.x * 4LL; e < e1; e += step) {
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = e + i < per ? src[e + i] : 0.f;
    uint2 sp[2];
    split4h(v[0], v[1], v[2], v[3], mb, sp);
    const uint16_t* h = (const uint16_t*)&sp[0];
    const uint16_t* l = (const uint16_t*)&sp[1];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (e + i < per) { oh[e + i] = h[i]; ol[e + i] = l[i]; }
  }
}
__global__ __launch_bounds__(256) void xsplit_w_kernel(const float* __restrict__ w, long long sstride, long long per,
                                                       const int* __restrict__ amax, int ld,
                                                       uint16_t* __restrict__ out) {
  xsplit_w_body(w, sstride, per, amax, ld, out, blockIdx.y, blockIdx.x * 1024LL, per, (long long)gridDim.x * 1024);
}
// a whole model fold's weight splits in one launch (blockIdx.y = slot): the x grid is the
// concatenation of every weight's chunks of kXSChunk elements (desc i owns blocks [boff_i,
// boff_{i+1})); a max-sized grid per desc left most blocks of the small convs idle
struct XSDesc {   // all int64 (built from a torch int64 host tensor)
  long long w, sstride, per, amax, ld, out, boff;
};
constexpr int kXSBatch = 24, kXSChunk = 4096;
struct XSBatch {
  XSDesc d[kXSBatch];
  int n;
};
__global__ __launch_bounds__(256) void xsplit_w_batch_kernel(const XSBatch b) {
  int i = 0;
  while (i + 1 < b.n && (long long)blockIdx.x >= b.d[i + 1].boff) ++i;
  const XSDesc& d = b.d[i];
  const long long e0 = ((long long)blockIdx.x - d.boff) * kXSChunk;
  const long long e1 = e0 + kXSChunk < d.per ? e0 + kXSChunk : d.per;
  xsplit_w_body((const float*)d.w, d.sstride, d.per, (const int*)d.amax, (int)d.ld, (uint16_t*)d.out, blockIdx.y, e0,
                e1, 1024);
}

// max |x| of n segments (offset, length) of every replica's flat row (the conv weights of a
// model replica: one launch per training step instead of one per conv); out[s][g]
// One block per 4096-element chunk of a segment (the segments' chunks laid end to end: block c
// belongs to the segment whose chunk range holds c), four 16-B loads per thread in flight; a
// 2-D grid of (64 chunks x segments) blocks left most of them idle on the small segments and
// read scalars.  The max is order-free (exact integer fold), so the tiling is free.
constexpr int kAmaxSegs = 64, kAmaxChunk = 4096;
struct AmaxSegs {
  long long off[kAmaxSegs];
  int len[kAmaxSegs];
  int start[kAmaxSegs + 1];   // first chunk of each segment (prefix sum of ceil(len / 4096))
  int n;
};
__global__ __launch_bounds__(256) void amax_segments_kernel(const float* __restrict__ base, long long gstride,
                                                            const AmaxSegs segs, int ld, int* __restrict__ out) {
  const int c = blockIdx.x, g = blockIdx.y;
  int sg = 0;
  while (sg + 1 < segs.n && segs.start[sg + 1] <= c) ++sg;
  const float* __restrict__ p = base + (long long)g * gstride + segs.off[sg];
  const int n = segs.len[sg], e0 = (c - segs.start[sg]) * kAmaxChunk;
  const bool v4 = ((segs.off[sg] | gstride) & 3) == 0 && ((uintptr_t)base & 15) == 0;
  float m = 0.f;
  float4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = e0 + (k * 256 + threadIdx.x) * 4;
    if (v4 && e + 3 < n) {
      v[k] = *(const float4*)(p + e);
    } else {
      v[k].x = e < n ? p[e] : 0.f;
      v[k].y = e + 1 < n ? p[e + 1] : 0.f;
      v[k].z = e + 2 < n ? p[e + 2] : 0.f;
      v[k].w = e + 3 < n ? p[e + 3] : 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) m = fmaxf(m, fmaxf(fmaxf(fabsf(v[k].x), fabsf(v[k].y)), fmaxf(fabsf(v[k].z), fabsf(v[k].w))));
  amax_fold(out + (long long)sg * kAmaxSub * ld, ld, g, m);
}

// max |x| of each replica's valid prefix (nvalid[g] * per_item elements, or n_per_g), as the
// float's bit pattern: the fp16-pair scale source (HScale).  Integer atomicMax of non-negative
// float bits: exact and order-independent (deterministic); out is zeroed by the launcher.
__global__ __launch_bounds__(256) void amax_kernel(const float* __restrict__ x, long long gstride, long long n_per_g,
                                                   const int* __restrict__ nvalid, long long per_item, int vec,
                                                   int* __restrict__ out, int ld) {
  const int g = blockIdx.y;
  const long long n = nvalid ? (long long)nvalid[g] * per_item : n_per_g;
  const float* __restrict__ p = x + (long long)g * gstride;
  float m = 0.f;
  if (vec) {
    const long long n4 = n >> 2;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n4; e += (long long)gridDim.x * 256) {
      const float4 v = ((const float4*)p)[e];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    for (long long e = n4 * 4 + blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256)
      m = fmaxf(m, fabsf(p[e]));
  } else {
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) m = fmaxf(m, fabsf(p[e]));
  }
  amax_fold(out, ld, g, m);
}

// bias gradient db[g][c] += sum over the valid rows of dy[g][r][c], deterministic, in two
// passes: xcolsum_part sums fixed 256-row chunks (4 row lanes x 64 columns per block, fp64,
// the lanes met in LDS in lane order) into part[g][chunk][c]; xcolsum_fin sums the chunks in
// chunk order.  The chunking depends on the replica's own valid rows only.  (The former single
// pass ran ONE block per 32 columns with a 4608-long serial add chain per thread for MnistNet's
// conv1 — 36864 rows x 20 channels: 278 us per launch, 70 % of the MNIST training stream,
// profiles/r5/mnist/streams_before.md.)
constexpr int kColRows = 256;
__global__ __launch_bounds__(256) void xcolsum_part_kernel(const float* __restrict__ dy, long long dy_gstride,
                                                           int rows_per_img, const int* __restrict__ nvalid, int N,
                                                           int C, double* __restrict__ part, int nchunk) {
  __shared__ double red[4][64];
  const int g = blockIdx.y, ch = blockIdx.x;
  const int R = valid_rows(nvalid, g, N) * rows_per_img;
  const int r0 = ch * kColRows, r1 = min(R, r0 + kColRows);
  const int tc = threadIdx.x & 63, tr = threadIdx.x >> 6;
  const float* __restrict__ d = dy + (long long)g * dy_gstride;
  for (int c0 = 0; c0 < C; c0 += 64) {
    const int c = c0 + tc;
    double s = 0.0;
    if (c < C)
#pragma unroll 4
      for (int r = r0 + tr; r < r1; r += 4) s += d[(long long)r * C + c];
    red[tr][tc] = s;
    __syncthreads();
    if (tr == 0 && c < C)
      part[((long long)g * nchunk + ch) * C + c] = ((red[0][tc] + red[1][tc]) + red[2][tc]) + red[3][tc];
    __syncthreads();
  }
}
// one wave per column: lane l sums chunks l, l + 64, ... (fp64), then the wave's fixed
// butterfly — the same order at any launch geometry
__global__ __launch_bounds__(256) void xcolsum_fin_kernel(const double* __restrict__ part, int rows_per_img,
                                                          const int* __restrict__ nvalid, int N, int C, int nchunk,
                                                          float* __restrict__ db, long long db_gstride) {
  const int g = blockIdx.y, c = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= C) return;
  const int R = valid_rows(nvalid, g, N) * rows_per_img;
  const int nc = (R + kColRows - 1) / kColRows;
  double t = 0.0;
  for (int k = lane; k < nc; k += 64) t += part[((long long)g * nchunk + k) * C + c];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
  if (lane == 0) db[(long long)g * db_gstride + c] += (float)t;
}

// ===================================================== fused training BN: standalone pass
// A tile pass over a MATERIALISED tensor, for the producers whose epilogue cannot reduce: the
// split-K slabs of multi-replica launches (summed here in z order, xsplitk_reduce's order, plus
// the dgrad's accumulated branch), stride-s data gradients, the global average pool's gradient,
// max-pool gradients.  Same 128-row tiles of whole groups, same level-0 records
// (bnf_tile_records) and finalize launch as the conv epilogues, so the statistics are
// the same bits whichever kernel produced them.  mode 1: statistics of the value (stored to dst
// when dst is given); mode 2: d = mask(value) -> dst (may alias src).  value = src, or the sum of
// S slabs ws[z] (+ accum), or pool[g][img][c] * pool_scale (elementwise.hip avgpool_bwd's value).
__global__ __launch_bounds__(256) void bnx_tile_kernel(const BnFuse f, const float* src, float* dst,
                                                       long long gstride, const int* __restrict__ nvalid, int N,
                                                       int HW, const float* __restrict__ pool, float pool_scale,
                                                       const float* __restrict__ ws, int S, long long zstride,
                                                       const float* __restrict__ accum) {
  constexpr int BM = 128, BN = 64, C4 = BN / 4;
  __shared__ __attribute__((aligned(16))) float Ct[BM * BN];
  __shared__ long long orow[BM];
  const int g = blockIdx.y, tid = threadIdx.x, C = f.C;
  const int tiles_n = ceil_div_d(C, BN);
  const int tn = blockIdx.x % tiles_n, tm = blockIdx.x / tiles_n;
  const int Mv = valid_rows(nvalid, g, N) * HW;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mv) return;
  if (tid < BM) orow[tid] = m0 + tid < Mv ? (long long)(m0 + tid) * C : -1;
  __syncthreads();
  const long long base = (long long)g * gstride;
  for (int e = tid; e < BM * C4; e += 256) {
    const int row = e / C4, cc = (e - row * C4) * 4, n = n0 + cc;
    const long long o = orow[row];
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (o >= 0 && n < C) {
      if (ws) {
        v = *(const float4*)(ws + base + o + n);
        for (int z = 1; z < S; ++z) {
          const float4 u = *(const float4*)(ws + z * zstride + base + o + n);
          v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
        }
      } else if (pool) {
        const float4 u = *(const float4*)(pool + ((long long)g * N + (m0 + row) / HW) * C + n);
        v = make_float4(u.x * pool_scale, u.y * pool_scale, u.z * pool_scale, u.w * pool_scale);
      } else {
        v = *(const float4*)(src + base + o + n);
      }
      if (accum) {
        const float4 r = *(const float4*)(accum + base + o + n);
        v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
      }
      if (f.mode == 2) v = bnf_mask4(f, g, o, n, v);
      if (dst) *(float4*)(dst + base + o + n) = v;
    }
    *(float4*)&Ct[row * BN + cc] = v;
  }
  __syncthreads();
  bnf_tile_records<BM, BN>(f, Ct, orow, g, m0, n0, Mv);
}

// The materialised output of a training BN (+ residual) (+ ReLU) (bnfuse.hpp): out =
// relu?(fma(ya, scale_a, shift_a) + r), r = res (identity shortcut) or fma(yb, scale_b, shift_b)
// (a shortcut conv's BN; relu_b: a lazy BN+ReLU output, e.g. the stem's) or 0 — bn.hip
// bn_apply's arithmetic; folds max |out| for the fp16-pair operand scale of its consumers.
// Valid rows only.
__global__ __launch_bounds__(256) void bnx_apply_kernel(const float* __restrict__ ya, const float* __restrict__ ca,
                                                        const float* __restrict__ res, const float* __restrict__ yb,
                                                        const float* __restrict__ cb, int relu_b, int relu,
                                                        float* __restrict__ out,
                                                        long long gstride, const int* __restrict__ nvalid, int N,
                                                        int HW, int C, int* __restrict__ amax, int amax_ld) {
  const int g = blockIdx.y;
  const int C4 = C >> 2;
  const long long total = (long long)valid_rows(nvalid, g, N) * HW * C4;
  const long long base = (long long)g * gstride;
  const float* cag = ca + (long long)g * kBnRows * C;
  const float* cbg = cb ? cb + (long long)g * kBnRows * C : nullptr;
  float vmax = 0.f;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int c = (int)(t % C4) * 4;
    const long long o = base + t * 4;
    const float4 y = *(const float4*)(ya + o);
    const float4 sc = *(const float4*)(cag + kCScale * C + c), sh = *(const float4*)(cag + kCShift * C + c);
    float4 v = make_float4(fmaf(y.x, sc.x, sh.x), fmaf(y.y, sc.y, sh.y), fmaf(y.z, sc.z, sh.z), fmaf(y.w, sc.w, sh.w));
    if (res) {
      const float4 r = *(const float4*)(res + o);
      v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
    } else if (yb) {
      const float4 u = *(const float4*)(yb + o);
      const float4 sb = *(const float4*)(cbg + kCScale * C + c), hb = *(const float4*)(cbg + kCShift * C + c);
      float4 b = make_float4(fmaf(u.x, sb.x, hb.x), fmaf(u.y, sb.y, hb.y), fmaf(u.z, sb.z, hb.z), fmaf(u.w, sb.w, hb.w));
      if (relu_b) { b.x = fmaxf(b.x, 0.f); b.y = fmaxf(b.y, 0.f); b.z = fmaxf(b.z, 0.f); b.w = fmaxf(b.w, 0.f); }
      v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
    }
    if (relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
    vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    *(float4*)(out + o) = v;
  }
  if (amax) amax_fold(amax, amax_ld, g, vmax);
}

// The input gradient of a training BN, stored: dy = fma(A, d, fma(B, y, K)) per channel
// (bnfuse.hpp; bn.hip bn_bwd_apply's arithmetic) over the valid rows, and the max |dy| slot
// folded for its fp16-pair consumers (measured faster than the weight gradient staging dy
// from (d, y) on the fly: profiles/r4/bnx/ab_steps.md).
__global__ __launch_bounds__(256) void bnx_dy_kernel(const float* __restrict__ d, const float* __restrict__ y,
                                                     const float* __restrict__ coef, float* __restrict__ dy,
                                                     long long gstride, const int* __restrict__ nvalid, int N, int HW,
                                                     int C, int* __restrict__ amax, int amax_ld) {
  const int g = blockIdx.y;
  const int C4 = C >> 2;
  const long long total = (long long)valid_rows(nvalid, g, N) * HW * C4;
  const long long base = (long long)g * gstride;
  const float* cf = coef + (long long)g * kBnRows * C;
  float vmax = 0.f;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int c = (int)(t % C4) * 4;
    const long long o = base + t * 4;
    const float4 dv = *(const float4*)(d + o), yv = *(const float4*)(y + o);
    const float4 A = *(const float4*)(cf + kCA * C + c), B = *(const float4*)(cf + kCB * C + c),
                 K = *(const float4*)(cf + kCK * C + c);
    const float4 v = make_float4(fmaf(A.x, dv.x, fmaf(B.x, yv.x, K.x)), fmaf(A.y, dv.y, fmaf(B.y, yv.y, K.y)),
                                 fmaf(A.z, dv.z, fmaf(B.z, yv.z, K.z)), fmaf(A.w, dv.w, fmaf(B.w, yv.w, K.w)));
    vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    *(float4*)(dy + o) = v;
  }
  if (amax) amax_fold(amax, amax_ld, g, vmax);
}

// ============================================================================ host
int bnx_tile_go(const BnFuse& f, const float* src, float* dst, long long gstride, const int* nvalid, int G, int N,
                int HW, const float* pool, float pool_scale, const float* ws, int S, long long zstride,
                const float* accum, hipStream_t st) {
  if (f.C & 3) return -102;
  const dim3 grid((unsigned)(ceil_div((long long)N * HW, 128) * ceil_div(f.C, 64)), G);
  hipLaunchKernelGGL(bnx_tile_kernel, grid, dim3(256), 0, st, f, src, dst, gstride, nvalid, N, HW, pool, pool_scale, ws,
                     S, zstride, accum);
  const int rc = (int)hipGetLastError();
  return rc != 0 ? rc : bnx_finalize_go(f, nvalid, G, N, HW, st);
}

template <int BM, int BN, int WM, int WN, int VEC, bool PW, bool LZ = false, bool KS = false>
int xconv_go(const XArgs& a, long long Mmax, int G, int nclass, hipStream_t st) {
  XArgs b = a;
  b.tiles_n = ceil_div(a.Ncol, BN);
  const dim3 grid((unsigned)(ceil_div(Mmax, BM) * b.tiles_n), G, nclass * a.splitk);
  hipLaunchKernelGGL((xconv_kernel<BM, BN, WM, WN, VEC, PW, LZ, KS>), grid, dim3(256), 0, st, b);
  DBA_LAUNCH_CHECK();
}

// a split forward of a grouped launch as in-block slabs (xconv_kernel KS): 32-channel vectors,
// Ncol > 64 (the stage-3 / 4 convs xsplitk splits), 64 x 128 tiles (the running sum doubles the
// accumulators), at most kKslabMax slabs (more go through HBM + the reduce / BN pass).  Serial
// slabs cost the launch its split-K parallelism: at 8 slabs (stage 4) the 10-client step's split
// convs took 385 vs 352 us with the reduce passes included (profiles/r4/kslab/).
// split-K policy (per-replica geometry only: any setting keeps world-1 == world-N bits):
// target tiles, minimum k-steps per slab, maximum slabs, maximum in-block slabs (KS)
struct SplitPolicy {
  int target = 128, min_k = 8, max_s = 8, kslab_max = 2;
  int dgrad_ks = 1;   // grouped stride-1 data gradients as in-block slabs too (else split + reduce pass)
};
SplitPolicy& split_policy() {
  static SplitPolicy p;
  return p;
}
int xconv_ks(const XArgs& a, long long M, int G, int vec, hipStream_t st) {
  if (a.kslab > split_policy().kslab_max || a.Ncol <= 64 || a.Cs % 32 || vec < 4 || a.splitk != 1 || a.kslab < 2) return -100;
  if (a.lz_coef) return xconv_go<64, 128, 2, 2, 32, false, true, true>(a, M, G, 1, st);
  if (a.wp) return xconv_go<64, 128, 2, 2, 32, true, false, true>(a, M, G, 1, st);
  return xconv_go<64, 128, 2, 2, 32, false, false, true>(a, M, G, 1, st);
}

template <int VEC, bool PW = false, bool LZ = false>
int xconv_tile(const XArgs& a, long long Mmax, int G, int nclass, int bm, hipStream_t st) {
  if (a.Ncol <= 32) return xconv_go<128, 32, 4, 1, VEC, PW, LZ>(a, Mmax, G, nclass, st);
  if (a.Ncol <= 64) {
    if (bm == 64) return xconv_go<64, 64, 2, 2, VEC, PW, LZ>(a, Mmax, G, nclass, st);
    return xconv_go<128, 64, 2, 2, VEC, PW, LZ>(a, Mmax, G, nclass, st);
  }
  if (bm == 32) return xconv_go<32, 128, 1, 4, VEC, PW, LZ>(a, Mmax, G, nclass, st);
  if (bm == 64) return xconv_go<64, 128, 2, 2, VEC, PW, LZ>(a, Mmax, G, nclass, st);
  return xconv_go<128, 128, 2, 2, VEC, PW, LZ>(a, Mmax, G, nclass, st);
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <int W, int CS, int BM, int BN, int WM, int WN, bool PRE = false, bool LZ = false, bool SC = false>
int xhalo_go(const XArgs& a, int G, hipStream_t st) {
  XArgs b = a;
  b.tiles_n = ceil_div(a.Ncol, BN);
  const dim3 grid((unsigned)(a.N * (a.Ho / (BM / W)) * b.tiles_n), G, 1);
  hipLaunchKernelGGL((xhalo_kernel<W, CS, BM, BN, WM, WN, PRE, LZ, SC>), grid, dim3(256), 0, st, b);
  DBA_LAUNCH_CHECK();
}

// the whole-image halo conv (ximg_kernel): evaluation forward, 3x3 stride-1 pad-1, square
// W 8 / 4, Cs % 32 == 0, no fused BN / lazy operands (dba_ximg_set(0): off — the tests' A/B
// against the implicit GEMM)
template <int W, int IMGS, int BN, int WM, int WN>
int ximg_go(const XArgs& a, int G, hipStream_t st) {
  XArgs b = a;
  b.tiles_n = ceil_div(a.Ncol, BN);
  const dim3 grid((unsigned)(ceil_div(a.N, IMGS) * b.tiles_n), G, 1);
  if (a.wp) hipLaunchKernelGGL((ximg_kernel<W, IMGS, BN, WM, WN, true>), grid, dim3(256), 0, st, b);
  else hipLaunchKernelGGL((ximg_kernel<W, IMGS, BN, WM, WN, false>), grid, dim3(256), 0, st, b);
  DBA_LAUNCH_CHECK();
}
int& ximg_on() {
  static int on = 1;
  return on;
}
int ximg_try(const XArgs& a, int G, int KH, int KW, hipStream_t st) {
  const XClass& c = a.cls[0];
  if (!ximg_on() || KH != 3 || KW != 3 || a.sp != 1 || a.os != 1 || a.dsg != 1 || a.splitk != 1 || c.nI != 3 ||
      c.nJ != 3 || c.bh != -1 || c.bw != -1)
    return -100;
  if (a.Hs != a.Ho || a.Ws != a.Wo || a.Ho != a.Wo || a.Cs % 32 != 0 || a.Ncol % 32 != 0) return -100;
  if (a.bf.mode || a.lz_coef) return -100;
  if (!aligned16(a.src) || a.src_gstride % 4 || !aligned16(a.w) || a.w_sstride % 4) return -100;
  if (a.wp && (((uintptr_t)a.wp & 15) || a.wp_sstride % 8)) return -100;
  if (a.sc_src) return -100;   // the fused shortcut: xhalo_kernel only (see ximg_kernel)
  if (a.Wo == 8) return a.Ncol >= 128 ? ximg_go<8, 2, 128, 2, 2>(a, G, st) : ximg_go<8, 2, 64, 2, 2>(a, G, st);
  if (a.Wo == 4) return a.Ncol >= 128 ? ximg_go<4, 8, 128, 2, 2>(a, G, st) : ximg_go<4, 8, 64, 2, 2>(a, G, st);
  return -100;
}

bool flip_dgrad(const XArgs& a) { return a.dsg < 0; }

int& wgrad_halo_on() {
  static int on = 1;
  return on;
}

// the halo kernel's shapes: 3x3 stride-1 pad-1 (fwd) or its stride-1 data gradient, one class,
// square W 32 (Cs 32, Ncol <= 32) or W 16 (Cs 64, Ncol <= 64), aligned fp32 operands.  (8-row
// W-32 tiles were faster in isolation, not in the overlapped bench: profiles/r2_halo_tiles_ab.md;
// a persistent weight-stationary W-32 form tied in isolation and held CUs the training stream
// needs: 3.06 vs 3.20 rounds/s, profiles/halo_ws_r3.md.)
int xhalo_try(const XArgs& a, int G, int KH, int KW, hipStream_t st) {
  const XClass& c = a.cls[0];
  if (KH != 3 || KW != 3 || a.sp != 1 || a.os != 1 || a.splitk != 1 || c.nI != 3 || c.nJ != 3) return -100;
  if (!(a.dsg == 1 ? (c.bh == -1 && c.bw == -1) : (c.bh == 1 && c.bw == 1))) return -100;
  if (a.Hs != a.Ho || a.Ws != a.Wo || a.Ho != a.Wo || (a.Ncol & 3) != 0) return -100;
  if (!aligned16(a.src) || !aligned16(a.w) || a.src_gstride % 4 || a.w_sstride % 4) return -100;
  if (a.lz_coef && (a.wp || flip_dgrad(a))) return -108;   // lazy BN operand: training forward
  if (a.Wo == 32 && a.Cs == 32 && a.Ncol <= 32 && a.Ho % 4 == 0 && !a.sc_src) {
    if (a.lz_coef) return xhalo_go<32, 32, 128, 32, 4, 1, false, true>(a, G, st);
    if (a.wp) return xhalo_go<32, 32, 128, 32, 4, 1, true>(a, G, st);
    return xhalo_go<32, 32, 128, 32, 4, 1>(a, G, st);
  }
  // W 16 / Cs 64 (8-row tiles x 64 channels): the implicit GEMM's re-split of every input
  // element per tap is what bounds that shape
  if (a.Wo == 16 && a.Cs == 64 && a.Ncol <= 64 && a.Ho % 8 == 0) {
    if (a.sc_src) {   // the fused downsampling shortcut: 32 input channels, pre-split weights
      if (!a.wp || a.sc_C != 32 || !aligned16(a.sc_src) || a.sc_gstride % 4 || ((uintptr_t)a.sc_wp & 15) ||
          a.sc_wp_sstride % 8 || flip_dgrad(a))
        return -100;
      return xhalo_go<16, 64, 128, 64, 2, 2, true, false, true>(a, G, st);
    }
    if (a.lz_coef) return xhalo_go<16, 64, 128, 64, 2, 2, false, true>(a, G, st);
    if (a.wp) return xhalo_go<16, 64, 128, 64, 2, 2, true>(a, G, st);
    return xhalo_go<16, 64, 128, 64, 2, 2>(a, G, st);
  }
  return -100;
}

// the implicit GEMM's tile rows for a launch (xconv_tile maps it to the kernel's BM).  Small
// launches (a lone client's grouped step) take 64-row tiles, the smallest (a lone client's
// stage-3/4 convs: 32-64 tiles of 64 rows) 32-row tiles with one 32x32 MFMA tile per wave.
int xconv_bm(long long Mmax, int Ncol, int G, int nclass, int splitk) {
  constexpr int kBm32Below = 256;
  const int bn = Ncol <= 32 ? 32 : Ncol <= 64 ? 64 : 128;
  const long long blocks = (long long)ceil_div(Mmax, 128) * ceil_div(Ncol, bn) * G * nclass * splitk;
  int bm = (bn > 32 && blocks < 512) ? 64 : 128;
  if (bn == 128 && 2 * blocks < kBm32Below) bm = 32;
  return bm;
}

// arrival counters an in-launch split-K combine needs: one per (replica, tile, class)
long long xconv_sk_count(long long Mmax, int Ncol, int G, int nclass, int splitk) {
  const int bn = Ncol <= 32 ? 32 : Ncol <= 64 ? 64 : 128;
  const int bm = Ncol <= 32 ? 128 : xconv_bm(Mmax, Ncol, G, nclass, splitk);
  return (long long)ceil_div(Mmax, bm) * ceil_div(Ncol, bn) * G * nclass;
}

// the in-launch combine applies: counters given and enough of them, 4-column output vectors,
// a replica's slab addressable by a 32-bit buffer offset
// (lone-client 32 x 128 tiles only: at 128-row tiles the reducer's serial slab read costs more
// than the launch it saves — 10-client step 2.20 -> 2.33 ms, profiles/r3_sk_inlaunch.md)
bool sk_ok(const int* cnt, long long cnt_n, long long M, int Ncol, int G, int nclass, int s) {
  return cnt && s <= kSkMax && Ncol > 64 && xconv_bm(M, Ncol, G, nclass, s) == 32 && (Ncol & 3) == 0 &&
         M * Ncol < (1LL << 29) && cnt_n >= xconv_sk_count(M, Ncol, G, nclass, s);
}

int xconv_dispatch(const XArgs& a, long long Mmax, int G, int nclass, int vec, hipStream_t st) {
  // The tile shape never changes a result bit: every output element sees the same k-step
  // order and the same plane-product order within a step.
  if (!a.amax_src || !a.amax_w) return -109;   // the fp16 pair needs both operand maxima
  const int bm = xconv_bm(Mmax, a.Ncol, G, nclass, a.splitk);
  if (vec == 4 && a.Cs % 32 == 0) vec = 32;
  if (a.lz_coef) {   // lazy BN operand (training forward; the launcher checked wp and vec)
    if (vec == 32) return xconv_tile<32, false, true>(a, Mmax, G, nclass, bm, st);
    return xconv_tile<4, false, true>(a, Mmax, G, nclass, bm, st);
  }
  if (a.wp && vec >= 4) {
    if (vec == 32) return xconv_tile<32, true>(a, Mmax, G, nclass, bm, st);
    return xconv_tile<4, true>(a, Mmax, G, nclass, bm, st);
  }
  if (vec == 32) return xconv_tile<32>(a, Mmax, G, nclass, bm, st);
  return vec == 4 ? xconv_tile<4>(a, Mmax, G, nclass, bm, st) : xconv_tile<1>(a, Mmax, G, nclass, bm, st);
}

// split-K factor of a forward launch (1 = none).  Decided from the PER-REPLICA geometry only
// (never from the group count G): the K-slicing sets the summation order, so a client's
// bits must not depend on how many other clients share its launch (world-1 vs world-N runs
// place different client groups on a rank).  Splits a replica below ~128 tiles of 64 rows
// (a lone client's stage-3/4 convs) into slabs of >= 8 k-steps.
int xsplitk(long long M, int /*G*/, int Ncol, int K) {
  const int bn = Ncol <= 32 ? 32 : Ncol <= 64 ? 64 : 128;
  // 128: a lone client's stage-3 convs (64 tiles of 64 rows) split in two — lone step 1.95 ->
  // 1.85 ms, the 10-client round's training time unchanged (202.4 vs 202.6 ms, r2c_iter1);
  // finer slabs were slower in the bench (348 -> 368 ms per round, profiles/sk_r3/)
  const int kTarget = split_policy().target, kMinK = split_policy().min_k;   // tiles; k-steps per slab
  const int kMaxS = std::min(kSkMax, split_policy().max_s);                  // slabs
  const long long tiles = (long long)ceil_div(M, 64) * ceil_div(Ncol, bn);
  if (tiles >= kTarget) return 1;
  const int nkt = (K + 31) / 32;
  int s = (int)std::min<long long>(kMaxS, (kTarget + tiles - 1) / tiles);
  while (s > 1 && nkt / s < kMinK) --s;
  return s;
}

struct ClassGeom {
  int n;
  XClass c[4];
};

// parity classes of a stride-s data gradient (see xtranspose_kernel for the weight order)
ClassGeom dgrad_classes(int H, int W, int Cin, int Cout, int KH, int KW, int s, int pad) {
  ClassGeom cg{};
  cg.n = s * s;
  long long off = 0;
  for (int ci = 0; ci < s * s; ++ci) {
    const int ph = ci / s, pw = ci - ph * s;
    const int kh0 = (ph + pad) % s, kw0 = (pw + pad) % s;
    XClass& c = cg.c[ci];
    c.nI = kh0 < KH ? (KH - kh0 + s - 1) / s : 0;
    c.nJ = kw0 < KW ? (KW - kw0 + s - 1) / s : 0;
    c.bh = (ph + pad - kh0) / s;
    c.bw = (pw + pad - kw0) / s;
    c.oh = ph;
    c.ow = pw;
    c.Hq = ph < H ? (H - ph + s - 1) / s : 0;
    c.Wq = pw < W ? (W - pw + s - 1) / s : 0;
    c.boff = off;
    off += (long long)Cin * c.nI * c.nJ * Cout;
  }
  return cg;
}

}  // namespace

// patch-reuse weight gradient (xwgrad_halo.hip) on / off (tests: A/B against the implicit GEMM
// on the same slabs); returns the previous
// the split-K policy (negative: keep); returns 0 (tools / A-B runs: tools.bench_step --split)
DBA_EXPORT int dba_xsplit_policy(int target, int min_k, int max_s, int kslab_max, int dgrad_ks) {
  SplitPolicy& p = split_policy();
  if (dgrad_ks >= 0) p.dgrad_ks = dgrad_ks;
  if (target > 0) p.target = target;
  if (min_k > 0) p.min_k = min_k;
  if (max_s > 0) p.max_s = std::min(max_s, kSkMax);
  if (kslab_max > 0) p.kslab_max = kslab_max;
  return 0;
}

DBA_EXPORT int dba_xwgrad_halo_set(int on) {
  const int prev = wgrad_halo_on();
  if (on >= 0) wgrad_halo_on() = on;
  return prev;
}

// whole-image halo conv (ximg_kernel) on / off (tests: A/B against the implicit GEMM); returns the previous
DBA_EXPORT int dba_ximg_set(int on) {
  const int prev = ximg_on();
  if (on >= 0) ximg_on() = on;
  return prev;
}

// workspace floats a split-K forward launch of this shape needs (0: none)
DBA_EXPORT long long dba_xconv_ws_floats(int G, int N, int Ho, int Wo, int Cin, int Cout, int KH, int KW) {
  const long long M = (long long)N * Ho * Wo;
  const int s = xsplitk(M, G, Cout, KH * KW * Cin);
  return s > 1 ? (long long)s * G * M * Cout : 0;
}

// arrival counters (int32, zeroed) the in-launch split-K combine of this shape needs (0: it
// does not split, or the combine is off / not applicable: the separate reduce launch runs)
DBA_EXPORT long long dba_xconv_sk_ints(int G, int N, int Ho, int Wo, int Cin, int Cout, int KH, int KW) {
  const long long M = (long long)N * Ho * Wo;
  const int s = xsplitk(M, G, Cout, KH * KW * Cin);
  const long long n = s > 1 ? xconv_sk_count(M, Cout, G, 1, s) : 0;
  return (n > 0 && sk_ok((const int*)1, n, M, Cout, G, 1, s)) ? n : 0;
}

// y = act(conv(x, w) + bias + res), fp32 NHWC; w [slots][Cout][KH][KW][Cin]
DBA_EXPORT int dba_xconv_fwd(const float* x, long long x_gstride, const float* w, long long w_sstride,
                             const int* wsel, const float* bias, long long b_sstride, const float* res, float* out,
                             long long out_gstride, const int* nvalid, int G, int N, int H, int W, int Cin, int Ho,
                             int Wo, int Cout, int KH, int KW, int stride, int pad, int relu, const int* amax_x,
                             int amax_x_ld, const int* amax_w, int amax_w_ld, int* amax_out, int amax_out_ld,
                             const uint16_t* wp, long long wp_sstride, float* ws, long long ws_floats, int* sk_cnt,
                             long long sk_cnt_n, const void* bnf, const float* lz_coef, int lz_relu, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if ((long long)N * H * W * Cin >= (1LL << 29)) return -103;   // 32-bit in-replica byte offsets
  const long long M = (long long)N * Ho * Wo;
  const int K = KH * KW * Cin;
  const int vec = (Cin % 4 == 0 && aligned16(x) && aligned16(w) && x_gstride % 4 == 0 && w_sstride % 4 == 0) ? 4 : 1;
  XArgs a{};
  a.src = x; a.src_gstride = x_gstride; a.w = w; a.w_sstride = w_sstride; a.wsel = wsel;
  a.bias = bias; a.b_sstride = b_sstride; a.res = res; a.out = out; a.out_gstride = out_gstride;
  a.nvalid = nvalid; a.N = N; a.Hs = H; a.Ws = W; a.Cs = Cin; a.Ncol = Cout; a.Ho = Ho; a.Wo = Wo;
  a.sp = stride; a.os = 1; a.dsg = 1; a.relu = relu; a.splitk = 1;
  a.amax_src = amax_x; a.amax_w = amax_w; a.amax_out = amax_out;
  a.amax_src_ld = amax_x_ld; a.amax_w_ld = amax_w_ld; a.amax_out_ld = amax_out_ld;
  a.wp = wp; a.wp_sstride = wp_sstride;
  a.cls[0] = XClass{KH, KW, -pad, -pad, 0, 0, Ho, Wo, 0};
  if (!amax_x || !amax_w) return -109;   // the fp16 pair needs both operand maxima
  if (bnf) {
    a.bf = *(const BnFuse*)bnf;
    if (a.bf.mode != 1 || bias || res || relu || (Cout & 3) || a.bf.C != Cout) return -108;
  }
  if (lz_coef) {
    if (wp || vec < 4 || Cin > 512) return -108;
    a.lz_coef = lz_coef; a.lz_relu = lz_relu;
  }
  // a fused BN's finalize launch follows its producer (bnx_tile_go launches its own)
  auto fin = [&](int rc) { return (rc == 0 && a.bf.mode) ? bnx_finalize_go(a.bf, nvalid, G, N, Ho * Wo, st) : rc; };
  if (stride == 1) {
    int rc = ximg_try(a, G, KH, KW, st);
    if (rc == -100) rc = xhalo_try(a, G, KH, KW, st);
    if (rc != -100) return fin(rc);
  }
  const int s = xsplitk(M, G, Cout, K);
  const bool ws_ok = s > 1 && ws != nullptr && ws_floats >= (long long)s * G * M * Cout;
  if (s > 1 && !(ws_ok && sk_ok(sk_cnt, sk_cnt_n, M, Cout, G, 1, s))) {
    // grouped launch: the slabs summed inside each block (same bits as the split launches)
    XArgs b = a;
    b.kslab = s;
    const int rc = xconv_ks(b, M, G, vec, st);
    if (rc != -100) return fin(rc);
  }
  if (ws_ok && sk_ok(sk_cnt, sk_cnt_n, M, Cout, G, 1, s)) {
    // in-launch combine (sk_combine): one launch, BN statistics folded by the reducing block
    XArgs b = a;
    b.splitk = s;
    b.zstride = (long long)G * M * Cout;
    b.sk_ws = ws; b.sk_gstride = M * Cout; b.sk_cnt = sk_cnt;
    return fin(xconv_dispatch(b, M, G, 1, vec, st));
  }
  if (ws_ok) {
    XArgs b = a;
    b.splitk = s;
    b.out = ws;
    b.out_gstride = M * Cout;
    b.zstride = (long long)G * M * Cout;
    const int rc = xconv_dispatch(b, M, G, 1, vec, st);
    if (rc != 0) return rc;
    if (a.bf.mode)   // the slabs summed + the statistics in one pass, the epilogue's records (bnfuse.hpp)
      return bnx_tile_go(a.bf, nullptr, out, out_gstride, nvalid, G, N, Ho * Wo, nullptr, 0.f, ws, s, b.zstride,
                         nullptr, st);
    const long long per = M * Cout;
    const dim3 grid((unsigned)std::max(1LL, std::min(1024LL, (per + 255) / 256)), G);
    hipLaunchKernelGGL(xsplitk_reduce_kernel, grid, dim3(256), 0, st, (const float*)ws, s, b.zstride, per, nvalid, N,
                       Ho * Wo, Cout, bias, b_sstride, wsel, res, relu, out, amax_out, amax_out_ld);
    DBA_LAUNCH_CHECK();
  }
  return fin(xconv_dispatch(a, M, G, 1, vec, st));
}

// The conv2 of a downsampling BasicBlock with its 1x1 stride-2 shortcut fused (evaluation, BN
// folded): out = relu(conv3x3(a, w2) + b2 + conv1x1_s2(x2, wsc) + bsc), one launch, the shortcut's
// output never materialised (xhalo_kernel SC: the W-16 stage, 64 channels from 32; 17 x 1024
// images 1348 vs 1886 us for the shortcut conv + the residual-epilogue conv2,
// profiles/r5/down/kbench_ximg_sc.log).  a [G][N][Ho][Wo][C] fp32, x2
// [G][N][H2][W2][C2] fp32 (Ho = ceil(H2 / 2)), w2 / wsc pre-split fp16-pair planes per slot.
// Returns -100 for shapes without a fused kernel (the caller runs the two convs).
DBA_EXPORT int dba_xdown_fwd(const float* a_, long long a_gstride, const float* w2, long long w2_sstride,
                             const uint16_t* w2p, long long w2p_sstride, const int* wsel, const float* b2,
                             long long b_sstride, const float* x2, long long x2_gstride, const uint16_t* wscp,
                             long long wscp_sstride, const float* bsc, long long bsc_sstride, float* out,
                             long long out_gstride, const int* nvalid, int G, int N, int Ho, int Wo, int C, int H2,
                             int W2, int C2, const int* amax_a, int amax_a_ld, const int* amax_w2, int amax_w2_ld,
                             const int* amax_x2, int amax_x2_ld, const int* amax_wsc, int amax_wsc_ld, int* amax_out,
                             int amax_out_ld, void* stream) {
  if (!amax_a || !amax_w2 || !amax_x2 || !amax_wsc || !w2p || !wscp) return -109;
  if ((Ho - 1) * 2 >= H2 || (Wo - 1) * 2 >= W2 || (long long)N * H2 * W2 * C2 >= (1LL << 29) ||
      (long long)N * Ho * Wo * C >= (1LL << 29))
    return -103;
  XArgs a{};
  a.src = a_; a.src_gstride = a_gstride; a.w = w2; a.w_sstride = w2_sstride; a.wsel = wsel;
  a.bias = b2; a.b_sstride = b_sstride; a.res = nullptr; a.out = out; a.out_gstride = out_gstride;
  a.nvalid = nvalid; a.N = N; a.Hs = Ho; a.Ws = Wo; a.Cs = C; a.Ncol = C; a.Ho = Ho; a.Wo = Wo;
  a.sp = 1; a.os = 1; a.dsg = 1; a.relu = 1; a.splitk = 1;
  a.amax_src = amax_a; a.amax_w = amax_w2; a.amax_out = amax_out;
  a.amax_src_ld = amax_a_ld; a.amax_w_ld = amax_w2_ld; a.amax_out_ld = amax_out_ld;
  a.wp = w2p; a.wp_sstride = w2p_sstride;
  a.sc_src = x2; a.sc_gstride = x2_gstride; a.sc_H = H2; a.sc_W = W2; a.sc_C = C2;
  a.sc_wp = wscp; a.sc_wp_sstride = wscp_sstride;
  a.sc_amax_src = amax_x2; a.sc_amax_src_ld = amax_x2_ld; a.sc_amax_w = amax_wsc; a.sc_amax_w_ld = amax_wsc_ld;
  a.sc_bias = bsc; a.sc_b_sstride = bsc_sstride;
  a.cls[0] = XClass{3, 3, -1, -1, 0, 0, Ho, Wo, 0};
  return xhalo_try(a, G, 3, 3, (hipStream_t)stream);
}

// dX of a conv from class-packed transposed weights (dba_xtranspose); accum (optional) is
// added in.  dy [G][N][Ho][Wo][Cout] -> dx [G][N][H][W][Cin]
DBA_EXPORT int dba_xconv_dgrad(const float* dy, long long dy_gstride, const float* wt, long long wt_sstride,
                               const int* wsel, const float* accum, float* dx, long long dx_gstride,
                               const int* nvalid, int G, int N, int H, int W, int Cin, int Ho, int Wo, int Cout,
                               int KH, int KW, int stride, int pad, const int* amax_dy, int amax_dy_ld,
                               const int* amax_w, int amax_w_ld, const uint16_t* wp, long long wp_sstride, float* ws,
                               long long ws_floats, int* sk_cnt, long long sk_cnt_n, const void* bnf, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if ((long long)N * Ho * Wo * Cout >= (1LL << 29)) return -103;   // 32-bit in-replica byte offsets
  const ClassGeom cg = dgrad_classes(H, W, Cin, Cout, KH, KW, stride, pad);
  const int vec = (Cout % 4 == 0 && aligned16(dy) && aligned16(wt) && dy_gstride % 4 == 0 && wt_sstride % 4 == 0) ? 4 : 1;
  XArgs a{};
  a.src = dy; a.src_gstride = dy_gstride; a.w = wt; a.w_sstride = wt_sstride; a.wsel = wsel;
  a.bias = nullptr; a.b_sstride = 0; a.res = accum; a.out = dx; a.out_gstride = dx_gstride;
  a.nvalid = nvalid; a.N = N; a.Hs = Ho; a.Ws = Wo; a.Cs = Cout; a.Ncol = Cin; a.Ho = H; a.Wo = W;
  a.sp = 1; a.os = stride; a.dsg = -1; a.relu = 0; a.splitk = 1;
  a.amax_src = amax_dy; a.amax_w = amax_w;
  a.amax_src_ld = amax_dy_ld; a.amax_w_ld = amax_w_ld;
  a.wp = wp; a.wp_sstride = wp_sstride;
  if (bnf) {   // the backward BN mask + reduce of the gradient (stride-1 data gradients: one class)
    a.bf = *(const BnFuse*)bnf;
    if (a.bf.mode != 2 || stride != 1 || (Cin & 3) || a.bf.C != Cin) return -108;
  }
  long long Mmax = 0;
  for (int i = 0; i < cg.n; ++i) {
    a.cls[i] = cg.c[i];
    Mmax = std::max(Mmax, (long long)N * cg.c[i].Hq * cg.c[i].Wq);
  }
  auto fin = [&](int rc) { return (rc == 0 && a.bf.mode) ? bnx_finalize_go(a.bf, nvalid, G, N, H * W, st) : rc; };
  if (stride == 1) {
    const int rc = xhalo_try(a, G, KH, KW, st);
    if (rc != -100) return fin(rc);
    const long long M = (long long)N * H * W;
    const int s = xsplitk(M, G, Cin, KH * KW * Cout);
    const bool ws_ok = s > 1 && ws != nullptr && ws_floats >= (long long)s * G * M * Cin;
    if (ws_ok && sk_ok(sk_cnt, sk_cnt_n, M, Cin, G, 1, s)) {
      XArgs b = a;
      b.splitk = s;
      b.zstride = (long long)G * M * Cin;
      b.sk_ws = ws; b.sk_gstride = M * Cin; b.sk_cnt = sk_cnt;
      return fin(xconv_dispatch(b, M, G, 1, vec, st));
    }
    if (s > 1 && split_policy().dgrad_ks) {
      // grouped launch: the slabs summed inside each block in z order, then the accumulated
      // input and the BN mask / records in the epilogue — the lone client's in-launch combine
      // arithmetic (sk_combine), without the slab round trip and the standalone BN pass
      XArgs b = a;
      b.kslab = s;
      const int rc = xconv_ks(b, M, G, vec, st);
      if (rc != -100) return fin(rc);
    }
    if (ws_ok) {
      XArgs b = a;
      b.splitk = s;
      b.out = ws;
      b.out_gstride = M * Cin;
      b.zstride = (long long)G * M * Cin;
      const int rc = xconv_dispatch(b, M, G, 1, vec, st);
      if (rc != 0) return rc;
      if (a.bf.mode)   // slabs + accum summed, masked and reduced in one pass (bnfuse.hpp)
        return bnx_tile_go(a.bf, nullptr, dx, dx_gstride, nvalid, G, N, H * W, nullptr, 0.f, ws, s, b.zstride, accum,
                           st);
      const long long per = M * Cin;
      const dim3 grid((unsigned)std::max(1LL, std::min(1024LL, (per + 255) / 256)), G);
      hipLaunchKernelGGL(xsplitk_reduce_kernel, grid, dim3(256), 0, st, (const float*)ws, s, b.zstride, per, nvalid,
                         N, H * W, Cin, nullptr, 0LL, wsel, accum, 0, dx, (int*)nullptr, 0);
      DBA_LAUNCH_CHECK();
    }
  }
  return fin(xconv_dispatch(a, Mmax, G, cg.n, vec, st));
}

// class-packed data-gradient weights for n convs.  desc: n x XTDesc in HOST memory, read
// here and passed to the kernel by value (safe under HIP graph capture); nvalid (optional,
// slots == replicas) skips inactive slots.
DBA_EXPORT int dba_xtranspose(const void* desc, int n, int slots, long long max_per, const int* nvalid,
                              void* stream) {
  const XTDesc* ds = (const XTDesc*)desc;
  for (int i0 = 0; i0 < n; i0 += kXTBatch) {
    XTBatch b{};
    const int m = std::min(kXTBatch, n - i0);
    for (int i = 0; i < m; ++i) b.d[i] = ds[i0 + i];
    const dim3 grid((unsigned)std::max(1LL, std::min(1024LL, (max_per + 1023) / 1024)), m, slots);
    hipLaunchKernelGGL(xtranspose_kernel, grid, dim3(256), 0, (hipStream_t)stream, b, slots, nvalid);
    const int rc = (int)hipGetLastError();
    if (rc != 0) return rc;
  }
  return 0;
}

// slab floats dba_xwgrad needs for this shape (0: accumulates straight into dw)
// The m-chunking (Z slabs) is decided from the PER-REPLICA geometry only (see xsplitk): ~256
// blocks per replica (a lone client fills the chip), chunks of >= 256 rows.
DBA_EXPORT long long dba_xwgrad_ws_floats(int G, int N, int Ho, int Wo, int Cin, int Cout, int KH, int KW, int* mchunk_out) {
  const int K = KH * KW * Cin;
  // the narrow stages' 3x3 convs: the patch-reuse kernel's slabs (xwgrad_halo.hip: SPB strips
  // of 8 rows each; the implicit GEMM takes the same slabs where that kernel declines)
  const int hrows = (KH == 3 && KW == 3) ? xwgrad_halo_rows(Ho, Wo, Cin, Cout) : 0;
  if (hrows > 0 && (long long)N * Ho * Wo > hrows) {
    const long long M = (long long)N * Ho * Wo, Z = (M + hrows - 1) / hrows;
    if (mchunk_out) *mchunk_out = hrows;
    return Z * G * Cout * K;
  }
  const int bno = Cout <= 32 ? 32 : Cout <= 64 ? 64 : 128;
  const long long tiles = (long long)ceil_div(Cout, bno) * ceil_div(K, 128);
  const long long M = (long long)N * Ho * Wo;
  constexpr int kTarget = 256, kMinRows = 256;   // blocks per replica; rows per slab
  long long Z = std::max(1LL, std::min((kTarget + tiles - 1) / tiles, M / kMinRows));
  int mchunk = (int)((M + Z - 1) / Z);
  mchunk = (mchunk + 31) / 32 * 32;
  Z = (M + mchunk - 1) / mchunk;
  if (mchunk_out) *mchunk_out = mchunk;
  return Z > 1 ? Z * G * Cout * K : 0;
}

// dw[g] += sum_m dy (x) im2col(x) (fp32, deterministic); dw [G][Cout][KH][KW][Cin] rows
// defer != 0: the slab reduction (Z > 1) is left to dba_xwgrad_reduce_batch (one launch for
// the whole backward pass)
DBA_EXPORT int dba_xwgrad(const float* dy, long long dy_gstride, const float* x, long long x_gstride, float* dw,
                          long long dw_gstride, const int* nvalid, int G, int N, int H, int W, int Cin, int Ho,
                          int Wo, int Cout, int KH, int KW, int stride, int pad, const int* amax_dy,
                          int amax_dy_ld, const int* amax_x, int amax_x_ld, float* ws, long long ws_floats, int defer,
                          const float* x_coef, int x_relu, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int mchunk = 0;
  const long long need = dba_xwgrad_ws_floats(G, N, Ho, Wo, Cin, Cout, KH, KW, &mchunk);
  if (need > 0 && (ws == nullptr || ws_floats < need)) return -101;
  const long long M = (long long)N * Ho * Wo;
  const int Z = (int)((M + mchunk - 1) / mchunk);
  XWArgs a{};
  a.dy = dy; a.dy_gstride = dy_gstride; a.x = x; a.x_gstride = x_gstride; a.ws = ws; a.dw = dw;
  a.dw_gstride = dw_gstride; a.nvalid = nvalid; a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Ho = Ho; a.Wo = Wo;
  a.Cout = Cout; a.KW = KW; a.stride = stride; a.pad = pad; a.K = KH * KW * Cin;
  a.mchunk = mchunk;
  a.amax_dy = amax_dy; a.amax_x = amax_x;
  a.amax_dy_ld = amax_dy_ld; a.amax_x_ld = amax_x_ld;
  a.x_coef = x_coef; a.x_relu = x_relu;
  a.dHoWo = FDiv{Ho * Wo, 1.0f / (float)(Ho * Wo)};
  a.dWo = FDiv{Wo, 1.0f / (float)Wo};
  a.tiles_k = ceil_div(a.K, 128);
  if ((long long)N * Ho * Wo * Cout >= (1LL << 29) || (long long)N * H * W * Cin >= (1LL << 29)) return -103;
  if (Z > 1 && wgrad_halo_on() && stride == 1 && pad == 1 && KH == 3 && KW == 3 && H == Ho && W == Wo &&
      Cin == Cout && mchunk == xwgrad_halo_rows(Ho, Wo, Cin, Cout)) {
    // patch reuse: each staged input element feeds all 9 taps (xwgrad_halo.hip)
    XWHArgs h{dy, dy_gstride, x, x_gstride, ws, nvalid, N, H, amax_dy, amax_dy_ld, amax_x, amax_x_ld, x_coef, x_relu};
    const int rc = xwgrad_halo_launch(h, G, W, Cin, st);
    if (rc != -100) {
      if (rc != 0 || defer) return rc;
      const long long per = (long long)Cout * a.K;
      const dim3 g2((unsigned)std::max(1LL, std::min(1024LL, (per + 255) / 256)), G);
      hipLaunchKernelGGL(xwgrad_reduce_kernel, g2, dim3(256), 0, st, (const float*)ws, G, per, nvalid, N, Ho * Wo,
                         mchunk, dw, dw_gstride);
      DBA_LAUNCH_CHECK();
    }
  }
  const bool v4 = Cin % 4 == 0 && Cout % 4 == 0 && aligned16(dy) && aligned16(x) && dy_gstride % 4 == 0 &&
                  x_gstride % 4 == 0;
  // output-channel tile: 128 for wide layers (64 for a lone client's stage-3/4 weight gradients
  // when a launch would be short of blocks measured within run-to-run spread: lone step 1.774 ->
  // 1.763 ms, scripts/gpu/r2c_iter10.sh).  The tile never changes a bit (same per-element row
  // order within a slab); Z came from the per-replica geometry above.
  if (!amax_dy || !amax_x) return -109;   // the fp16 pair needs both operand maxima
  const int bno = Cout <= 32 ? 32 : Cout <= 64 ? 64 : 128;
  const dim3 grid((unsigned)(ceil_div(Cout, bno) * a.tiles_k), G, Z);
#define XW_GO(BNO_, WN__, WK__, V_, X_) \
  hipLaunchKernelGGL((xwgrad_kernel<BNO_, 128, WN__, WK__, V_, X_>), grid, dim3(256), 0, st, a)
#define XW_P(V_, X_)                                  \
  do {                                                \
    if (bno == 32) XW_GO(32, 1, 4, V_, X_);           \
    else if (bno == 64) XW_GO(64, 2, 2, V_, X_);      \
    else XW_GO(128, 2, 2, V_, X_);                    \
  } while (0)
  if (x_coef) {
    if (v4) XW_P(4, true); else XW_P(1, true);
  } else {
    if (v4) XW_P(4, false); else XW_P(1, false);
  }
#undef XW_P
#undef XW_GO
  if (Z > 1 && !defer) {
    const long long per = (long long)Cout * a.K;
    const dim3 g2((unsigned)std::max(1LL, std::min(1024LL, (per + 255) / 256)), G);
    hipLaunchKernelGGL(xwgrad_reduce_kernel, g2, dim3(256), 0, st, (const float*)ws, G, per, nvalid, N, Ho * Wo,
                       mchunk, dw, dw_gstride);
  }
  DBA_LAUNCH_CHECK();
}

// out [slots][2][per] fp16 planes of w (see xsplit_w_kernel); amax: the weights' max slot
DBA_EXPORT int dba_xsplit_w(const float* w, long long sstride, long long per, int slots, const int* amax, int ld,
                            uint16_t* out, void* stream) {
  const dim3 grid((unsigned)std::max(1LL, std::min(1024LL, (per + 1023) / 1024)), slots);
  hipLaunchKernelGGL(xsplit_w_kernel, grid, dim3(256), 0, (hipStream_t)stream, w, sstride, per, amax, ld, out);
  DBA_LAUNCH_CHECK();
}

// the fp16-pair planes of n weight operands (one model fold) in one launch per 24; desc: n x XSDesc
// in HOST memory (passed by value), every operand with `slots` slots
DBA_EXPORT int dba_xsplit_w_batch(const void* desc, int n, int slots, void* stream) {
  const XSDesc* ds = (const XSDesc*)desc;
  for (int i0 = 0; i0 < n; i0 += kXSBatch) {
    XSBatch b{};
    b.n = std::min(kXSBatch, n - i0);
    long long nb = 0;
    for (int i = 0; i < b.n; ++i) {
      b.d[i] = ds[i0 + i];
      b.d[i].boff = nb;
      nb += (b.d[i].per + kXSChunk - 1) / kXSChunk;
    }
    hipLaunchKernelGGL(xsplit_w_batch_kernel, dim3((unsigned)nb, slots), dim3(256), 0, (hipStream_t)stream, b);
    const int rc = (int)hipGetLastError();
    if (rc != 0) return rc;
  }
  return 0;
}

// out: n zeroed amax slots [n][kAmaxSub][ld] (common.hpp): max |x| of segment s of replica g;
// segs: n x (offset, length) int64 pairs in HOST memory (passed by value: safe under graph
// capture), n <= 64
DBA_EXPORT int dba_amax_segments(const float* base, long long gstride, const long long* segs, int n, int G, int* out,
                                 int ld, void* stream) {
  if (n > kAmaxSegs || n < 1) return -105;
  AmaxSegs a{};
  a.n = n;
  for (int i = 0; i < n; ++i) {
    a.off[i] = segs[2 * i];
    a.len[i] = (int)segs[2 * i + 1];
    a.start[i + 1] = a.start[i] + std::max(1, ceil_div(a.len[i], kAmaxChunk));
  }
  const dim3 grid((unsigned)a.start[n], G);
  hipLaunchKernelGGL(amax_segments_kernel, grid, dim3(256), 0, (hipStream_t)stream, base, gstride, a, ld, out);
  DBA_LAUNCH_CHECK();
}

// folds max |x| over replica g's valid prefix into the zeroed slot out [kAmaxSub][ld]
DBA_EXPORT int dba_amax(const float* x, long long gstride, long long n_per_g, const int* nvalid, long long per_item,
                        int G, int* out, int ld, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int vec = aligned16(x) && gstride % 4 == 0;
  const long long per = nvalid ? per_item * (n_per_g / std::max(1LL, per_item)) : n_per_g;
  const dim3 grid((unsigned)std::max(1LL, std::min(256LL, (per + 4095) / 4096)), G);
  hipLaunchKernelGGL(amax_kernel, grid, dim3(256), 0, st, x, gstride, n_per_g, nvalid, per_item, vec, out, ld);
  DBA_LAUNCH_CHECK();
}

// part: [G][ceil(N * rows_per_img / 256)][C] fp64 workspace (dba_xcolsum_part_doubles)
DBA_EXPORT long long dba_xcolsum_part_doubles(int G, int N, int rows_per_img, int C) {
  return (long long)G * ceil_div((long long)N * rows_per_img, kColRows) * C;
}
DBA_EXPORT int dba_xcolsum(const float* dy, long long dy_gstride, int rows_per_img, const int* nvalid, int G, int N,
                           int C, float* db, long long db_gstride, double* part, void* stream) {
  const int nchunk = ceil_div((long long)N * rows_per_img, kColRows);
  hipLaunchKernelGGL(xcolsum_part_kernel, dim3(nchunk, G), dim3(256), 0, (hipStream_t)stream, dy, dy_gstride,
                     rows_per_img, nvalid, N, C, part, nchunk);
  hipLaunchKernelGGL(xcolsum_fin_kernel, dim3(ceil_div(C, 4), G), dim3(256), 0, (hipStream_t)stream, part,
                     rows_per_img, nvalid, N, C, nchunk, db, db_gstride);
  DBA_LAUNCH_CHECK();
}

// desc: n x XWRDesc in HOST memory (passed to the kernel by value: safe under graph capture)
DBA_EXPORT int dba_xwgrad_reduce_batch(const void* desc, int n, int Gmax, long long max_per, void* stream) {
  const XWRDesc* ds = (const XWRDesc*)desc;
  for (int i0 = 0; i0 < n; i0 += kXWRBatch) {
    XWRBatch b{};
    const int m = std::min(kXWRBatch, n - i0);
    for (int i = 0; i < m; ++i) b.d[i] = ds[i0 + i];
    bool v4 = true;
    for (int i = 0; i < m; ++i) v4 = v4 && b.d[i].per % 4 == 0 && b.d[i].ws % 16 == 0;
    const dim3 grid((unsigned)std::max(1LL, std::min(256LL, (max_per + 255) / 256)), m, Gmax);
    if (v4) hipLaunchKernelGGL(xwgrad_reduce_batch_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, b);
    else hipLaunchKernelGGL(xwgrad_reduce_batch_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, b);
    const int rc = (int)hipGetLastError();
    if (rc != 0) return rc;
  }
  return 0;
}

// the fused-BN standalone pass (bnx_tile_kernel) over a materialised tensor or a pooled gradient;
// bnf: a BnFuse in host memory (passed by value: graph-capture safe)
DBA_EXPORT int dba_bnx_rows(const void* bnf, const float* src, float* dst, long long gstride, const int* nvalid, int G,
                            int N, int HW, const float* pool, float pool_scale, void* stream) {
  const BnFuse f = *(const BnFuse*)bnf;
  if (f.mode < 1 || f.mode > 2 || (f.mode == 2 && (!dst || !f.ya))) return -108;
  return bnx_tile_go(f, src, dst, gstride, nvalid, G, N, HW, pool, pool_scale, nullptr, 1, 0, nullptr,
                     (hipStream_t)stream);
}

// sizeof(BnFuse) (the Python ctypes mirror checks its layout against it)
DBA_EXPORT int dba_bnfuse_size() { return (int)sizeof(BnFuse); }

DBA_EXPORT int dba_bnx_apply(const float* ya, const float* ca, const float* res, const float* yb, const float* cb,
                             int relu_b, int relu, float* out, long long gstride, const int* nvalid, int G, int N, int HW, int C,
                             int* amax, int amax_ld, void* stream) {
  if (C & 3) return -102;
  const long long per = (long long)N * HW * (C / 4);
  const long long cap = std::max(1LL, 8192LL / std::max(1, G));
  const dim3 grid((unsigned)std::max(1LL, std::min(cap, (per + 255) / 256)), G);
  hipLaunchKernelGGL(bnx_apply_kernel, grid, dim3(256), 0, (hipStream_t)stream, ya, ca, res, yb, cb, relu_b, relu, out,
                     gstride,
                     nvalid, N, HW, C, amax, amax_ld);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_bnx_dy(const float* d, const float* y, const float* coef, float* dy, long long gstride,
                          const int* nvalid, int G, int N, int HW, int C, int* amax, int amax_ld, void* stream) {
  if (C & 3) return -102;
  const long long per = (long long)N * HW * (C / 4);
  const long long cap = std::max(1LL, 8192LL / std::max(1, G));
  const dim3 grid((unsigned)std::max(1LL, std::min(cap, (per + 255) / 256)), G);
  hipLaunchKernelGGL(bnx_dy_kernel, grid, dim3(256), 0, (hipStream_t)stream, d, y, coef, dy, gstride, nvalid, N, HW, C,
                     amax, amax_ld);
  DBA_LAUNCH_CHECK();
}
