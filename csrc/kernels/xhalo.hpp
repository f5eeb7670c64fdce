// The halo-tiled 3x3 stride-1 conv (forward, data gradient, the evaluation down-block) of the
// fp32 family (xconv.hpp), shared by xconv_fwd.hip and xconv_dgrad.hip.
#pragma once
#include "xconv.hpp"

namespace {

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
  __shared__ __attribute__((aligned(16))) float lzs[LZ ? 2 * CS : 4];   // lazy operand: scale | shift
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
  // LZ: the source BN's scale / shift in LDS (from its coefficient rows)
  if constexpr (LZ) {
    const float* cf = a.lz_coef + (long long)g * kBnRows * CS;
    for (int c = tid; c < CS; c += 256) {
      lzs[c] = cf[kCScale * CS + c];
      lzs[CS + c] = cf[kCShift * CS + c];
    }
    __syncthreads();
  }
  const int src_bits = amax_read(a.amax_src, a.amax_src_ld, g);
  HScale hs;
  hs.init(src_bits, amax_read(a.amax_w, a.amax_w_ld, slot));
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
        const float4 sc = *(const float4*)&lzs[q * 4], sh = *(const float4*)&lzs[CS + q * 4];
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

template <int W, int CS, int BM, int BN, int WM, int WN, bool PRE = false, bool LZ = false, bool SC = false>
int xhalo_go(const XArgs& a, int G, hipStream_t st) {
  XArgs b = a;
  b.tiles_n = ceil_div(a.Ncol, BN);
  const dim3 grid((unsigned)(a.N * (a.Ho / (BM / W)) * b.tiles_n), G, 1);
  hipLaunchKernelGGL((xhalo_kernel<W, CS, BM, BN, WM, WN, PRE, LZ, SC>), grid, dim3(256), 0, st, b);
  DBA_LAUNCH_CHECK();
}

bool flip_dgrad(const XArgs& a) { return a.dsg < 0; }

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

}  // namespace
