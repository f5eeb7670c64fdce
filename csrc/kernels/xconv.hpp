// Reference-precision (fp32) convolution family for gfx950: scaled fp16-pair MFMA — the
// shared part of its translation units (xconv_fwd.hip, xconv_dgrad.hip): the launch arguments,
// the implicit-GEMM kernel (forward and data gradient), the split-K reduce and the host-side
// tile / split policy.
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
#pragma once
#include "common.hpp"
#include "bnfuse.hpp"
#include "xmfma.hpp"
#include <algorithm>
#include <type_traits>
#include <utility>
#include <cstdlib>

// state and helpers shared across the family's translation units (one instance in the library)
namespace xg {
struct SplitPolicy {
  int target = 128, min_k = 8, max_s = 8, kslab_max = 2;
  int dgrad_ks = 1;   // grouped stride-1 data gradients as in-block slabs too (else split + reduce pass)
};
SplitPolicy& split_policy();   // (xconv_fwd.hip)
// the fused-BN standalone pass over a materialised tensor or split-K slabs (xbn.hip)
int bnx_tile_go(const ::BnFuse& f, const float* src, float* dst, long long gstride, const int* nvalid, int G, int N,
                int HW, const float* pool, float pool_scale, const float* ws, int S, long long zstride,
                const float* accum, hipStream_t st);
}  // namespace xg
using xg::SplitPolicy;
using xg::split_policy;
using xg::bnx_tile_go;

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


// the implicit GEMM's tile rows for a launch (xconv_tile maps it to the kernel's BM).  Small
// launches (a lone client's grouped step) take 64-row tiles, the smallest (the stage-3/4 convs
// of 1-3 clients: 32-64 tiles of 64 rows per replica) 32-row tiles with one 32x32 MFMA tile per
// wave — which also admits them to the in-launch split-K combine (sk_ok).  (Round 6: 512, was
// 256 = the lone client only; a 2-client step's stage-3/4 convs then took the in-block-slab or
// slab + standalone BN pass forms: 7 bnx_tile launches of 16 us per step.)
int xconv_bm(long long Mmax, int Ncol, int G, int nclass, int splitk) {
  constexpr int kBm32Below = 512;
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

}  // namespace
