// Evaluation BasicBlock of the 32-wide ResNet stage in ONE launch (fp32 reference precision,
// scaled fp16-pair MFMA operands, BN folded into both convs):
//
//     y = relu(conv2(h) + b2 + x),   h = relu(conv1(x) + b1)       (3x3, stride 1, pad 1)
//
// The unfused form is two halo-conv launches that each read an input tensor with 4-row tiles
// (1.5x its bytes with the halo rows) and write an output tensor, and the second re-reads x
// for the residual: ~5 activation-tensor volumes of HBM traffic per block for ~0.5 ms of MFMA
// work per 17k images (the stage is HBM-bound, profiles/pmc_eval_r3.md).  Here a workgroup
// owns 8 output rows of one image: it loads input rows h0-2 .. h0+9 once (12 rows: 1.5x),
// splits them into the fp16 pair ONCE into an LDS patch, computes conv1 over the 10 rows
// conv2 needs (the 2 halo rows are recomputed: 1.25x conv1 work), rewrites the patch memory
// with the split mid activation h (never leaves LDS), computes conv2, and stores y with the
// residual read back in exact fp32 (the just-read rows are L2-resident): 2.5 volumes.
//
// Numerics are those of the two-launch form: per output element the same tap-major k-step
// order and MFMA plane products (xhalo.hpp xhalo_kernel), conv1's operand scales from the
// replica's max |x| and the weight slot's max |w|.  The mid activation's scale is this
// block's own max |h| (a power of two with max * 2^s in [2^14, 2^15)) instead of the
// replica's: the split is scale-invariant wherever no fp16 subnormal occurs, and a larger
// scale only moves fewer lo-plane elements into subnormals, so the mid operand is at least as
// precise.  Deterministic (no atomics but the exact integer max of the output's amax slot).
//
// STEM variant (layer1.0 of the CIFAR ResNets, reference models/resnet_cifar.py:80-88 +
// 14-37): x = relu(stem(img) + b0) is itself computed here from the 3-channel image, so the
// 32-channel stem output (128 B per pixel written and read back: a full activation volume
// each way, plus the stem launch) never reaches HBM.  The workgroup loads image rows
// h0-3 .. h0+10 (14 rows x 34 cols x 3 channels, 5.6 KB) into LDS and computes the stem for
// the 12 patch rows on the MFMAs (K = 27 taps x channels padded to 32: two 16-deep halves,
// 3 plane products each; the A fragments are gathered from the fp32 image rows and split
// with this block's max |img| as scale, the B fragments are the stem's pre-split planes).
// Each wave owns the stem tiles of the two output rows its conv2 tiles cover (same MFMA
// layout), so the residual stays in 32 VGPRs in fp32 (the exact values conv1 was fed, before
// their split); the four edge rows are one tile each.  The stem output is re-split into the
// patch with its block max as scale (the mid activation's rule).  The stem thus runs in the
// split-MFMA precision of every other conv (2^-22 relative per product) instead of the
// separate launch's exact fp32 FMAs (stem.hip) — within the fp32-level tolerance the tests
// hold every conv to.
#include "common.hpp"
#include "xmfma.hpp"

namespace {

struct XBArgs {
  const float* x; long long x_gstride;     // [G][N][32][32][32] block input (= residual)
  float* out; long long out_gstride;       // [G][N][32][32][32]
  const int* wsel;                         // replica -> weight slot (null: identity)
  const uint16_t* w1p; const uint16_t* w2p;   // pre-split fp16 planes per slot: [2][32 * 288]
  long long wp_sstride;                    //   (xsplit_w_kernel, scaled like amax_w*)
  const float* b1; const float* b2; long long b_sstride;
  const int* nvalid;
  int N;
  const int* amax_x; int amax_x_ld;        // max |x| per replica
  const int* amax_w1; const int* amax_w2; int amax_w_ld;   // max |w| per slot
  int* amax_out; int amax_out_ld;          // optional: max |y| folded per replica
  // STEM only (x is then the [G][N][32][32][3] image): the stem's pre-split planes per slot
  // ([2][32 * 27], w0_sstride apart), folded bias and max |w0| slot (ld amax_w_ld)
  const uint16_t* w0p; long long w0_sstride;
  const float* b0; long long b0_sstride;
  const int* amax_w0;
};

constexpr int kW = 32, kC = 32, kTR = 8;      // image width, channels, output rows per block
constexpr int kPW = kW + 2;                  // patch columns (zero padding at 0 and 33)
constexpr int kPR = kTR + 4;                 // input patch rows (h0-2 .. h0+9)
constexpr int kMR = kTR + 2;                 // mid rows (h0-1 .. h0+8)
constexpr int kCH = kC / 8;                  // 16-B chunks per pixel per plane
constexpr int kPatch = kPR * kPW * kCH;      // uint4 per plane
constexpr int kK = 9 * kC;                   // reduction length per conv
constexpr int kBPL = kC * 4;                 // uint4 per weight plane of one k-step (32 rows x 64 B)
constexpr int kSteps = 18;                   // 9 k-steps (taps) of conv1, then 9 of conv2
constexpr int kCi = 3, kK0 = 9 * kCi;        // STEM: image channels, stem reduction length
constexpr int kIR = kPR + 2, kIW = kW + 2;   // STEM: image rows h0-3 .. h0+10, cols -1 .. 32
constexpr int kIm = kIR * kIW * kCi;         // STEM: image patch floats
static_assert(kPR * kW * kC * 4 <= 2 * kPatch * 16, "fp32 staging of the stem / mid rows fits the patch");

template <bool STEM>
__global__ __launch_bounds__(256) void xblock_kernel(const XBArgs a) {
  __shared__ __attribute__((aligned(16))) uint4 patch[2 * kPatch];
  __shared__ __attribute__((aligned(16))) uint4 bring[2 * 2 * kBPL];
  __shared__ float red[3][4];                // block maxima: image (STEM), stem output (STEM), mid
  __shared__ float im[STEM ? kIm : 1];

  const int g = blockIdx.y;
  const int img = blockIdx.x / (kW / kTR), h0 = (blockIdx.x % (kW / kTR)) * kTR;
  if (img >= valid_rows(a.nvalid, g, a.N)) return;
  const int slot = a.wsel ? a.wsel[g] : g;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kq = tid & 7, r0 = tid >> 3;
  const int fr = lane & 31, hf = lane >> 5;
  const float* __restrict__ src = a.x + (long long)g * a.x_gstride + (long long)img * kW * kW * (STEM ? kCi : kC);
  constexpr int Q4 = kC / 4;                       // float4 per pixel
  float* Ct = reinterpret_cast<float*>(patch);     // fp32 staging of whole rows (stem, mid, output)

  // fp32 rows [0, NR) staged in Ct (zeros on rows outside the image) -> the patch layout split
  // with this block's max (``red``: the waves' maxima), zero padding columns; returns the scale
  // exponent (a power of two with max * 2^s in [2^14, 2^15))
  auto resplit = [&](auto NRc, const float (&rmax)[4]) __attribute__((always_inline)) {
    constexpr int NR = decltype(NRc)::value;
    const float bmax = fmaxf(fmaxf(rmax[0], rmax[1]), fmaxf(rmax[2], rmax[3]));
    const int sexp = hexp(__float_as_int(bmax));
    const float m = __uint_as_float((uint32_t)(sexp + 127) << 23);
    constexpr int NM = NR * kW * Q4 / 256;           // float4 of the rows per thread
    float4 mv[NM];
#pragma unroll
    for (int u = 0; u < NM; ++u) mv[u] = *(const float4*)&Ct[(tid + 256 * u) * 4];
    __syncthreads();   // every staged value read: the patch memory takes the split rows
#pragma unroll
    for (int u = 0; u < NM; ++u) {
      const int e = tid + 256 * u;
      const int px = e / Q4, q = e - px * Q4;
      const int pp = (px / kW) * kPW + px % kW + 1;
      uint2 sp[2];
      split4h(mv[u].x, mv[u].y, mv[u].z, mv[u].w, m, sp);
      const int o = pp * kCH + ((q >> 1) ^ hswz<kW, kC>(pp, 0));
      ((uint2*)&patch[o])[q & 1] = sp[0];
      ((uint2*)&patch[kPatch + o])[q & 1] = sp[1];
    }
    // zero padding columns 0 and 33 of the rows (2 planes x 4 chunks each)
    for (int e = tid; e < NR * 2 * kCH * 2; e += 256) {
      const int pl = e & 1, c4 = (e >> 1) & (kCH - 1), side = (e >> 3) & 1, mr = e >> 4;
      patch[pl * kPatch + (mr * kPW + side * (kPW - 1)) * kCH + c4] = make_uint4(0u, 0u, 0u, 0u);
    }
    return sexp;
  };

  f32x16_t acc[3];
  auto zero = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  };
  HScale hs;
  [[maybe_unused]] f32x16_t res[2];   // STEM: the residual x of this wave's output tiles (fp32)

  if constexpr (!STEM) {
    // ---- input patch: rows h0-2 .. h0+9, cols -1 .. 32 (zeros outside the image)
    constexpr int NE = (kPR * kPW * Q4 + 255) / 256;
    float4 pv[NE];
    {
      const __amdgpu_buffer_rsrc_t rA = rsrc(src, (long long)kW * kW * kC * 4);
#pragma unroll
      for (int u = 0; u < NE; ++u) {
        const int e = tid + 256 * u;
        const int pp = e / Q4, q = e - pp * Q4;
        const int pr = pp / kPW, pc = pp - pr * kPW;
        const int h = h0 - 2 + pr, w = pc - 1;
        const bool ok = e < kPR * kPW * Q4 && (unsigned)h < (unsigned)kW && (unsigned)w < (unsigned)kW;
        pv[u] = bload4(rA, ok ? ((h * kW + w) * kC + q * 4) * 4 : kOOB);
      }
    }
    hs.init(amax_read(a.amax_x, a.amax_x_ld, g), amax_read(a.amax_w1, a.amax_w_ld, slot));
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + 256 * u;
      if (e >= kPR * kPW * Q4) break;
      const int pp = e / Q4, q = e - pp * Q4;
      uint2 sp[2];
      split4h(pv[u].x, pv[u].y, pv[u].z, pv[u].w, hs.ma, sp);
      const int o = pp * kCH + ((q >> 1) ^ hswz<kW, kC>(pp, 0));
      ((uint2*)&patch[o])[q & 1] = sp[0];
      ((uint2*)&patch[kPatch + o])[q & 1] = sp[1];
    }
  } else {
    // ---- image rows h0-3 .. h0+10, cols -1 .. 32 (zeros outside) -> LDS, fp32
    constexpr int NI = (kIm + 255) / 256;
    float iv[NI];
    {
      const __amdgpu_buffer_rsrc_t rI = rsrc(src, (long long)kW * kW * kCi * 4);
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        const int e = tid + 256 * u;
        const int r = e / (kIW * kCi), rem = e - r * (kIW * kCi);
        const int c = rem / kCi, ci = rem - c * kCi;
        const int h = h0 - 3 + r, w = c - 1;
        const bool ok = e < kIm && (unsigned)h < (unsigned)kW && (unsigned)w < (unsigned)kW;
        iv[u] = bload1(rI, ok ? ((h * kW + w) * kCi + ci) * 4 : kOOB);
      }
    }
    // the stem's B fragments: planes [32 couts][27], k = KK * 16 + hf * 8 + j (zero past 27)
    uint4 bst[2][2];   // [KK][plane]
    {
      const uint16_t* W0 = a.w0p + (long long)slot * a.w0_sstride;
      const long long lo = a.w0_sstride >> 1;
#pragma unroll
      for (int KK = 0; KK < 2; ++KK)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          uint32_t u[4];
#pragma unroll
          for (int j2 = 0; j2 < 4; ++j2) {
            const int k = KK * 16 + hf * 8 + 2 * j2;
            const uint32_t v0 = k < kK0 ? W0[p * lo + fr * kK0 + k] : 0u;
            const uint32_t v1 = k + 1 < kK0 ? W0[p * lo + fr * kK0 + k + 1] : 0u;
            u[j2] = v0 | (v1 << 16);
          }
          bst[KK][p] = make_uint4(u[0], u[1], u[2], u[3]);
        }
    }
    float m = 0.f;
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int e = tid + 256 * u;
      if (e >= kIm) break;
      im[e] = iv[u];
      m = fmaxf(m, fabsf(iv[u]));
    }
    m = wave_max(m);
    if (lane == 0) red[0][wid] = m;
    __syncthreads();   // image rows + their max
    const float imax = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    const int simg = hexp(__float_as_int(imax));
    const float mimg = __uint_as_float((uint32_t)(simg + 127) << 23);
    HScale h0s;
    h0s.s = simg + hexp(amax_read(a.amax_w0, a.amax_w_ld, slot));

    // ---- stem tiles: patch rows E (an edge row 0, 1, 10, 11), wid + 2, wid + 6 (the rows of
    // this wave's conv2 output tiles: kept as the residual)
    const int pr0 = wid < 2 ? wid : wid + 8;
    zero();
    sfor<2>([&](auto KKc) __attribute__((always_inline)) {
      constexpr int KK = decltype(KKc)::value;
      int d[8];   // image-patch offset of reduction element k (tap-major, channel-minor)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = KK * 16 + hf * 8 + j, tap = k / kCi, ci = k - tap * kCi;
        d[j] = k < kK0 ? ((tap / 3) * kIW + tap % 3) * kCi + ci : -1;
      }
      uint4 af[2][3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int pr = i == 0 ? pr0 : wid + 2 + 4 * (i - 1);
        const int base = (pr * kIW + fr) * kCi;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = d[j] >= 0 ? im[base + d[j]] : 0.f;
        uint2 s0[2], s1[2];
        split4h(v[0], v[1], v[2], v[3], mimg, s0);
        split4h(v[4], v[5], v[6], v[7], mimg, s1);
        af[0][i] = make_uint4(s0[0].x, s0[0].y, s1[0].x, s1[0].y);
        af[1][i] = make_uint4(s0[1].x, s0[1].y, s1[1].x, s1[1].y);
      }
      const uint4 bfr[2][1] = {{bst[KK][0]}, {bst[KK][1]}};
      f32x16_t (&ac)[3][1] = *reinterpret_cast<f32x16_t (*)[3][1]>(&acc[0]);
      mma_half<3, 1, 2, true, 0, KK>(af, bfr, ac, [](int) {});
    });
    h0s.finish(*reinterpret_cast<f32x16_t (*)[3][1]>(&acc[0]));
    const float bias0 = a.b0[(long long)slot * a.b0_sstride + fr];
    float smax = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int pr = i == 0 ? pr0 : wid + 2 + 4 * (i - 1);
      const bool in_img = (unsigned)(h0 - 2 + pr) < (unsigned)kW;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int px = (r & 3) + 8 * (r >> 2) + 4 * hf;
        const float v = in_img ? fmaxf(acc[i][r] + bias0, 0.f) : 0.f;
        smax = fmaxf(smax, v);
        Ct[(pr * kW + px) * kC + fr] = v;
        if (i > 0) res[i - 1][r] = v;
      }
    }
    smax = wave_max(smax);
    if (lane == 0) red[1][wid] = smax;
    __syncthreads();   // the staged stem rows + their max
    const int sst = resplit(std::integral_constant<int, kPR>{}, red[1]);
    hs.ma = __uint_as_float((uint32_t)(sst + 127) << 23);
    hs.s = sst + hexp(amax_read(a.amax_w1, a.amax_w_ld, slot));
  }

  // ---- weights: step t < 9 is conv1's tap t, t >= 9 conv2's tap t - 9 (32 couts x 32 channels)
  const uint16_t* W1 = a.w1p + (long long)slot * a.wp_sstride;
  const uint16_t* W2 = a.w2p + (long long)slot * a.wp_sstride;
  const long long half = a.wp_sstride >> 1;
  const __amdgpu_buffer_rsrc_t r1h = rsrc(W1, (long long)kC * kK * 2), r1l = rsrc(W1 + half, (long long)kC * kK * 2);
  const __amdgpu_buffer_rsrc_t r2h = rsrc(W2, (long long)kC * kK * 2), r2l = rsrc(W2 + half, (long long)kC * kK * 2);
  uint4 rb[2];
  auto gq = [&](int t, int st) __attribute__((always_inline)) {
    const int tt = t < 9 ? t : t - 9;
    const int off = t < kSteps ? (r0 * kK + tt * 32 + kq * 4) * 2 : kOOB;   // past the last step: zeros
    const uint2 h = t < 9 ? bload8(r1h, off) : bload8(r2h, off);
    const uint2 l = t < 9 ? bload8(r1l, off) : bload8(r2l, off);
    rb[st] = make_uint4(h.x, h.y, l.x, l.y);
  };
  auto lput = [&](int buf, int st) __attribute__((always_inline)) {
    const uint2 sp[2] = {make_uint2(rb[st].x, rb[st].y), make_uint2(rb[st].z, rb[st].w)};
    lds_put<2, false, kC>(bring + buf * 2 * kBPL, kBPL, 0, r0, kq, sp);
  };

  zero();

  // one k-step: the wave's MI output-row tiles (rows wid, wid + 4, wid + 8 of the phase's
  // row grid) at tap t % 9; A from the patch image (rows offset by the tap), B from the ring
  auto step = [&](auto MIc, int t, int buf, int stn) __attribute__((always_inline)) {
    constexpr int MI = decltype(MIc)::value;
    const int tap = t < 9 ? t : t - 9;
    const int ti = tap / 3, tj = tap - ti * 3;
    const uint4* L = bring + buf * 2 * kBPL;
    sfor<2>([&](auto KK) __attribute__((always_inline)) {
      const int ch = decltype(KK)::value * 2 + hf;
      uint4 af[2][MI], bfr[2][1];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int pp = (wid + 4 * i + ti) * kPW + fr + tj;
        const int o = pp * kCH + (ch ^ hswz<kW, kC>(pp, 0));
        af[0][i] = patch[o];
        af[1][i] = patch[kPatch + o];
      }
      const int o = fr * 4 + (ch ^ ((fr >> 2) & 3));
      bfr[0][0] = L[o];
      bfr[1][0] = L[kBPL + o];
      f32x16_t (&ac)[MI][1] = *reinterpret_cast<f32x16_t (*)[MI][1]>(&acc[0]);
      mma_half<MI, 1, 2, true, 1, decltype(KK)::value>(af, bfr, ac, [&](int) __attribute__((always_inline)) {
        lput(buf ^ 1, stn);
        gq(t + 3, stn);
      });
    });
  };
  auto run = [&](int t) __attribute__((always_inline)) {
    const int buf = t & 1, stn = buf ^ 1;
    if (t < 9 && wid < 2) step(std::integral_constant<int, 3>{}, t, buf, stn);
    else step(std::integral_constant<int, 2>{}, t, buf, stn);
    __syncthreads();
  };

  gq(0, 0);
  gq(1, 1);
  lput(0, 0);
  gq(2, 0);
  __syncthreads();   // patch + conv1's first weight step

  for (int t = 0; t < 9; ++t) run(t);

  // ---- mid activation: h = relu(conv1 + b1), zero on rows outside the image; staged in fp32
  // through the (dead) patch memory, then re-split with this block's scale into the patch layout
  hs.finish(*reinterpret_cast<f32x16_t (*)[3][1]>(&acc[0]));
  const float* b1 = a.b1 + (long long)slot * a.b_sstride;
  const float bias1 = b1[fr];
  float vmax = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int mr = wid + 4 * i;
    if (mr >= kMR) break;   // waves 2, 3 own two tiles
    const bool in_img = (unsigned)(h0 - 1 + mr) < (unsigned)kW;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int px = (r & 3) + 8 * (r >> 2) + 4 * hf;
      const float v = in_img ? fmaxf(acc[i][r] + bias1, 0.f) : 0.f;
      vmax = fmaxf(vmax, v);
      Ct[(mr * kW + px) * kC + fr] = v;
    }
  }
  vmax = wave_max(vmax);
  if (lane == 0) red[2][wid] = vmax;
  __syncthreads();
  const int smid = resplit(std::integral_constant<int, kMR>{}, red[2]);
  hs.ma = __uint_as_float((uint32_t)(smid + 127) << 23);
  hs.s = smid + hexp(amax_read(a.amax_w2, a.amax_w_ld, slot));
  zero();
  __syncthreads();

  for (int t = 9; t < kSteps; ++t) run(t);

  // ---- output: y = relu(conv2 + b2 + x), fp32, through LDS for row-contiguous stores
  hs.finish(*reinterpret_cast<f32x16_t (*)[2][1]>(&acc[0]));
  const float* b2 = a.b2 + (long long)slot * a.b_sstride;
  [[maybe_unused]] const float bias2 = STEM ? b2[fr] : 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float v = acc[i][r];
      if constexpr (STEM) v = fmaxf(v + bias2 + res[i][r], 0.f);   // the residual from registers
      Ct[((wid + 4 * i) * kW + (r & 3) + 8 * (r >> 2) + 4 * hf) * kC + fr] = v;
    }
  __syncthreads();
  const long long obase = (long long)h0 * kW * kC;
  float* out = a.out + (long long)g * a.out_gstride + (long long)img * kW * kW * kC + obase;
  [[maybe_unused]] const float* res_g = src + obase;
  float omax = 0.f;
#pragma unroll
  for (int u = 0; u < kTR * kW * Q4 / 256; ++u) {
    const int e = tid + 256 * u;
    float4 v = *(const float4*)&Ct[e * 4];
    if constexpr (!STEM) {
      const int c4 = (e % Q4) * 4;
      const float4 rv = *(const float4*)(res_g + e * 4);
      v.x = fmaxf(v.x + b2[c4] + rv.x, 0.f);
      v.y = fmaxf(v.y + b2[c4 + 1] + rv.y, 0.f);
      v.z = fmaxf(v.z + b2[c4 + 2] + rv.z, 0.f);
      v.w = fmaxf(v.w + b2[c4 + 3] + rv.w, 0.f);
    }
    omax = fmaxf(omax, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    *(float4*)(out + e * 4) = v;
  }
  if (a.amax_out) amax_fold(a.amax_out, a.amax_out_ld, g, omax);
}

}  // namespace

// y = relu(conv2(relu(conv1(x) + b1)) + b2 + x) for [G][N][32][32][32] fp32 activations with
// pre-split fp16-pair weights (both convs [slots][32][3][3][32], planes wp_sstride apart per
// slot).  Returns -100 for any other shape (the caller runs the two convs).
DBA_EXPORT int dba_xblock_fwd(const float* x, long long x_gstride, float* out, long long out_gstride, const int* wsel,
                              const uint16_t* w1p, const uint16_t* w2p, long long wp_sstride, const float* b1,
                              const float* b2, long long b_sstride, const int* nvalid, int G, int N, int H, int W,
                              int C, int Cout, const int* amax_x, int amax_x_ld, const int* amax_w1,
                              const int* amax_w2, int amax_w_ld, int* amax_out, int amax_out_ld, void* stream) {
  if (H != kW || W != kW || C != kC || Cout != kC || !amax_x || !amax_w1 || !amax_w2 || !w1p || !w2p || !b1 || !b2)
    return -100;
  if (((uintptr_t)x & 15) || ((uintptr_t)out & 15) || (x_gstride & 3) || (out_gstride & 3) || (wp_sstride & 7) ||
      ((uintptr_t)w1p & 15) || ((uintptr_t)w2p & 15))
    return -100;
  if ((long long)N * H * W * C >= (1LL << 29)) return -103;
  XBArgs a{x, x_gstride, out, out_gstride, wsel, w1p, w2p, wp_sstride, b1, b2, b_sstride, nvalid, N,
           amax_x, amax_x_ld, amax_w1, amax_w2, amax_w_ld, amax_out, amax_out_ld,
           nullptr, 0, nullptr, 0, nullptr};
  hipLaunchKernelGGL(xblock_kernel<false>, dim3((unsigned)(N * (kW / kTR)), G), dim3(256), 0, (hipStream_t)stream, a);
  DBA_LAUNCH_CHECK();
}

// The stem + the first identity BasicBlock of the 32-wide stage:
//   x = relu(stem(img) + b0),  y = relu(conv2(relu(conv1(x) + b1)) + b2 + x)
// for [G][N][32][32][3] fp32 images (stem [slots][32][3][3][3], pre-split planes [2][32 * 27]
// w0_sstride apart per slot; conv1 / conv2 as dba_xblock_fwd).  -100 for any other shape.
DBA_EXPORT int dba_xblock_stem_fwd(const float* img, long long img_gstride, float* out, long long out_gstride,
                                   const int* wsel, const uint16_t* w0p, long long w0_sstride, const float* b0,
                                   long long b0_sstride, const uint16_t* w1p, const uint16_t* w2p,
                                   long long wp_sstride, const float* b1, const float* b2, long long b_sstride,
                                   const int* nvalid, int G, int N, int H, int W, int Cin, int C,
                                   const int* amax_w0, const int* amax_w1, const int* amax_w2, int amax_w_ld,
                                   int* amax_out, int amax_out_ld, void* stream) {
  if (H != kW || W != kW || Cin != kCi || C != kC || !w0p || !b0 || !amax_w0 || !amax_w1 || !amax_w2 || !w1p ||
      !w2p || !b1 || !b2)
    return -100;
  if (((uintptr_t)img & 3) || ((uintptr_t)out & 15) || (out_gstride & 3) || (wp_sstride & 7) || (w0_sstride & 1) ||
      w0_sstride < 2 * kC * kK0 || ((uintptr_t)w1p & 15) || ((uintptr_t)w2p & 15))
    return -100;
  if ((long long)N * H * W * C >= (1LL << 29)) return -103;
  XBArgs a{img, img_gstride, out, out_gstride, wsel, w1p, w2p, wp_sstride, b1, b2, b_sstride, nvalid, N,
           nullptr, 0, amax_w1, amax_w2, amax_w_ld, amax_out, amax_out_ld,
           w0p, w0_sstride, b0, b0_sstride, amax_w0};
  hipLaunchKernelGGL(xblock_kernel<true>, dim3((unsigned)(N * (kW / kTR)), G), dim3(256), 0, (hipStream_t)stream, a);
  DBA_LAUNCH_CHECK();
}
