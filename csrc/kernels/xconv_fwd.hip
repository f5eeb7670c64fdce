// fp32 family, forward pass (xconv.hpp): the conv launcher (halo / whole-image / implicit-GEMM
// tiles, split-K in-launch or in-block, fused training-BN statistics and lazy BN operands), the
// evaluation down-block, and the whole-image halo conv of the 8 / 4-wide evaluation stages.
#include "xhalo.hpp"

namespace xg {
SplitPolicy& split_policy() {
  static SplitPolicy p;
  return p;
}
}  // namespace xg

namespace {

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
                             long long sk_cnt_n, const void* bnf, const float* lz_coef, int lz_relu,
                             void* stream) {
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
  if ((H2 - 1) / 2 + 1 != Ho || (W2 - 1) / 2 + 1 != Wo || (long long)N * H2 * W2 * C2 >= (1LL << 29) ||
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
