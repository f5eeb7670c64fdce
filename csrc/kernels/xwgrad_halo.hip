// Weight gradient of the stride-1 3x3 pad-1 convs of the narrow ResNet stages with patch reuse
// (gfx950, fp32 reference precision on the scaled fp16-pair MFMA):
//
//     dW[co][tap][ci] = sum_p dy[p][co] * x[p + off(tap)][ci]          (tap = 3 x 3, pad 1)
//
// The implicit-GEMM weight gradient (xwgrad.hip xwgrad_kernel) stages an im2col tile per
// 128-wide slice of K = 9 Cin, so every input element is loaded, (lazily BN-applied,) split and
// written to LDS once per tap — 9x — and the 288-wide K of the 32-channel stage runs as 3 tiles
// of 128 (25 % padding).  Here a workgroup owns whole images of one replica: per 8-row strip it
// stages the output gradient dy (8 rows x W pixels x C) and the input patch x (10 rows x (W+2)
// pixels with the zero halo) ONCE, split into fp16 pairs, as row-major [pixel][channel] LDS
// images, and every tap reads its B fragments from the same patch at the tap's pixel offset.
// Both operands are consumed reduction-major (k = pixels) with the gfx950 transposing LDS read
// ds_read_b64_tr_b16: a 16-lane group reads 4 pixel rows x 16 channels and each lane receives
// one channel's 4 pixels, so no transposing store pass is needed (cdna_hip_programming.md T10).
//
// Wave work: C = 32 (one 32 x 32 tile per tap): wave w owns taps w and w + 4 over the whole
// strip and tap 8 over a quarter of its k-steps (the four partial tap-8 tiles meet in LDS in
// wave order: balanced 2.25 tiles per wave).  C = 64: wave w owns output-channel tile w & 1 x
// input-channel tile w >> 1 for all 9 taps (9 accumulators).
//
// Output: one fp32 slab of the whole [C][9][C] gradient per workgroup (= per SPB strips), summed
// by the batched slab reduction of xwgrad.hip in slab order — the slab geometry depends on the
// replica's own shape only, so a client's bits do not depend on how many clients share the
// launch.  Deterministic (no atomics).  LDS image swizzle for C = 64 (128-B pixel rows): 16-B
// chunk k of pixel p at k ^ 4 ((p >> 1) & 1), which makes every transposing read of 4
// consecutive pixels (any alignment: the tap offsets) conflict-free; C = 32 needs none.
#include "common.hpp"
#include "bnfuse.hpp"
#include "xmfma.hpp"
#include "xwgrad_halo.hpp"

namespace {

typedef __attribute__((ext_vector_type(4))) short v4s;
typedef __attribute__((address_space(3))) v4s lds_v4s;

// element offset of (pixel p, channel c) in a [pixel][C] fp16 LDS image (16-B chunk swizzle)
template <int C>
__device__ __forceinline__ int img_off(int p, int c) {
  if constexpr (C == 64) return p * C + ((((c >> 3) ^ (((p >> 1) & 1) << 2))) << 3) + (c & 7);
  else return p * C + c;
}

// 4 fp16 (8 B) of a transposing read: this lane's 16-lane group reads rows (pixels) pix(q) and
// the group's 16-channel block; the lane supplies row q = (lane & 15) >> 2, channels 4 (lane & 3)
__device__ __forceinline__ uint2 tr_read(const uint16_t* img_base_plane, int elem_off) {
  const v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img_base_plane + elem_off));
  return __builtin_bit_cast(uint2, v);
}

template <int W, int C, int SPB, bool XLZ>
__global__ __launch_bounds__(256, 2) void xwgrad_halo_kernel(const XWHArgs a) {
  constexpr int TR = 8, PX = TR * W, PW = W + 2, PR = TR + 2, PP = PR * PW;
  constexpr int Q4 = C / 4;                        // float4 per pixel
  constexpr int NKS = PX / 16;                     // 16-pixel k-steps per strip
  constexpr int ND = PX * Q4 / 256, NX = (PP * Q4 + 255) / 256;
  static_assert(PX * Q4 % 256 == 0, "dy pieces");
  static_assert(W % 16 == 0 && (C == 32 || C == 64), "shapes");
  constexpr int DYE = PX * C, XE = PP * C;         // fp16 elements per plane image
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * DYE + 2 * XE];
  uint16_t* dyl = lds;                             // [2][PX][C]
  uint16_t* xl = lds + 2 * DYE;                    // [2][PP][C]

  const int g = blockIdx.y;
  const int HS = a.H / TR;                         // strips per image
  const int strip0 = blockIdx.x * SPB;             // first strip of the block (image-major)
  const int img = strip0 / HS;
  if (img >= valid_rows(a.nvalid, g, a.N)) return;   // the reducer sums only the valid slabs
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* __restrict__ dyg = a.dy + (long long)g * a.dy_gstride;
  const float* __restrict__ xg = a.x + (long long)g * a.x_gstride;
  const __amdgpu_buffer_rsrc_t rD = rsrc(dyg, (long long)a.N * a.H * W * C * 4);
  const __amdgpu_buffer_rsrc_t rX = rsrc(xg, (long long)a.N * a.H * W * C * 4);
  HScale hs;
  hs.init(amax_read(a.amax_dy, a.amax_dy_ld, g), amax_read(a.amax_x, a.amax_x_ld, g));
  // XLZ: a thread's staged pieces all hold the same 4 channels (256 % (C / 4) == 0)
  float4 lsc = make_float4(0.f, 0.f, 0.f, 0.f), lsh = lsc;
  if constexpr (XLZ) {
    const float* cf = a.x_coef + (long long)g * kBnRows * C + (tid % Q4) * 4;
    lsc = *(const float4*)(cf + kCScale * C);
    lsh = *(const float4*)(cf + kCShift * C);
  }

  // per lane: its transposing-read row / channel quad and the MFMA tile halves
  const int gi = lane & 15, rq = gi >> 2, cp = gi & 3;   // row q, channel quad p of the group
  const int g16 = (lane >> 4) & 1, hf = lane >> 5;       // channel half of the tile, k half

  constexpr int NACC = C == 32 ? 3 : 9;
  f32x16_t acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  // C = 32: taps (wid, wid + 4, 8) -> acc 0, 1, 2 (tap 8 on k-steps [NKS/4 wid, NKS/4 (wid+1)));
  // C = 64: co tile wid & 1, ci tile wid >> 1, acc[tap]
  const int cot = C == 64 ? (wid & 1) * 32 : 0, cit = C == 64 ? (wid >> 1) * 32 : 0;

  for (int s = 0; s < SPB; ++s) {
    const int h0 = ((strip0 + s) % HS) * TR;
    // ---- stage the strip: dy rows h0 .. h0+7 and the x patch rows h0-1 .. h0+8 (zero halo).
    // The loads are issued in three waves (dy, then each half of the patch) and each is split
    // and stored as soon as the next is in flight, so at most ~two thirds of the strip sit in
    // registers beside the accumulators (C = 64: 144 accumulator VGPRs live across strips)
    constexpr int NX1 = (NX + 1) / 2, NX2 = NX - NX1;
    float4 dv[ND], xv1[NX1], xv2[NX2 > 0 ? NX2 : 1];
    const int dbase = ((img * a.H + h0) * W) * C;
    auto xload = [&](int u) __attribute__((always_inline)) {
      const int e = tid + 256 * u, pp = e / Q4, q = e - pp * Q4;
      const int pr = pp / PW, pc = pp - pr * PW, h = h0 - 1 + pr, w = pc - 1;
      const bool ok = e < PP * Q4 && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)W;
      return bload4(rX, ok ? (((img * a.H + h) * W + w) * C + q * 4) * 4 : kOOB);
    };
    auto xput = [&](int u, float4 v) __attribute__((always_inline)) {
      const int e = tid + 256 * u;
      if (e >= PP * Q4) return;
      const int pp = e / Q4, q = e - pp * Q4;
      if constexpr (XLZ) {   // relu?(fma(y, scale, shift)) inside the image, 0 in the halo
        const int pr = pp / PW, pc = pp - pr * PW, h = h0 - 1 + pr, w = pc - 1;
        const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)W;
        v.x = fmaf(v.x, lsc.x, lsh.x); v.y = fmaf(v.y, lsc.y, lsh.y); v.z = fmaf(v.z, lsc.z, lsh.z);
        v.w = fmaf(v.w, lsc.w, lsh.w);
        if (a.x_relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
        if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      uint2 sp[2];
      split4h(v.x, v.y, v.z, v.w, hs.mb, sp);
      const int o = img_off<C>(pp, q * 4);
      *(uint2*)&xl[o] = sp[0];
      *(uint2*)&xl[XE + o] = sp[1];
    };
#pragma unroll
    for (int u = 0; u < ND; ++u) dv[u] = bload4(rD, (dbase + (tid + 256 * u) * 4) * 4);
#pragma unroll
    for (int u = 0; u < NX1; ++u) xv1[u] = xload(u);
    if (s > 0) __syncthreads();   // the previous strip's reads are done
#pragma unroll
    for (int u = 0; u < ND; ++u) {
      const int e = tid + 256 * u, p = e / Q4, q = e - p * Q4;
      uint2 sp[2];
      split4h(dv[u].x, dv[u].y, dv[u].z, dv[u].w, hs.ma, sp);
      const int o = img_off<C>(p, q * 4);
      *(uint2*)&dyl[o] = sp[0];
      *(uint2*)&dyl[DYE + o] = sp[1];
    }
#pragma unroll
    for (int u = 0; u < NX2; ++u) xv2[u] = xload(NX1 + u);
#pragma unroll
    for (int u = 0; u < NX1; ++u) xput(u, xv1[u]);
#pragma unroll
    for (int u = 0; u < NX2; ++u) xput(NX1 + u, xv2[u]);
    __syncthreads();

    // ---- the strip's k-steps: A = dy^T (rows co), B = shifted x (cols ci), k = 16 pixels
    auto afrag = [&](int ks, uint4 (&A)[2]) __attribute__((always_inline)) {
      const int m0 = ks * 16 + 8 * hf + rq;                 // pixel of row q, first read
      const int c = cot + 16 * g16 + 4 * cp;
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) {
        const uint2 u0 = tr_read(dyl + pl * DYE, img_off<C>(m0, c));
        const uint2 u1 = tr_read(dyl + pl * DYE, img_off<C>(m0 + 4, c));
        A[pl] = make_uint4(u0.x, u0.y, u1.x, u1.y);
      }
    };
    auto bfrag = [&](int ks, int tap, uint4 (&B)[2]) __attribute__((always_inline)) {
      const int ti = tap / 3, tj = tap - ti * 3;
      const int m0 = ks * 16 + 8 * hf + rq;                 // output pixel of row q (same row)
      const int pp0 = (m0 / W + ti) * PW + m0 % W + tj;     // its patch pixel at the tap
      const int c = cit + 16 * g16 + 4 * cp;
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) {
        const uint2 u0 = tr_read(xl + pl * XE, img_off<C>(pp0, c));
        const uint2 u1 = tr_read(xl + pl * XE, img_off<C>(pp0 + 4, c));
        B[pl] = make_uint4(u0.x, u0.y, u1.x, u1.y);
      }
    };
    // plane products in mma_half's order (the small ones first): hi*lo, lo*hi, hi*hi
    auto mma3 = [&](f32x16_t& d, const uint4 (&A)[2], const uint4 (&B)[2]) __attribute__((always_inline)) {
      d = mfma16<true>(A[0], B[1], d);
      d = mfma16<true>(A[1], B[0], d);
      d = mfma16<true>(A[0], B[0], d);
    };
    if constexpr (C == 32) {
      const int t1 = wid, t2 = wid + 4;
      const int q0 = (NKS / 4) * wid, q1 = q0 + NKS / 4;
#pragma unroll 2
      for (int ks = 0; ks < NKS; ++ks) {
        uint4 A[2], B1[2], B2[2];
        afrag(ks, A);
        bfrag(ks, t1, B1);
        bfrag(ks, t2, B2);
        mma3(acc[0], A, B1);
        mma3(acc[1], A, B2);
        if (ks >= q0 && ks < q1) {
          uint4 B3[2];
          bfrag(ks, 8, B3);
          mma3(acc[2], A, B3);
        }
      }
    } else {
#pragma unroll 1
      for (int ks = 0; ks < NKS; ++ks) {
        uint4 A[2];
        afrag(ks, A);
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          uint4 B[2];
          bfrag(ks, tap, B);
          mma3(acc[tap], A, B);
        }
      }
    }
  }
  hs.finish(*reinterpret_cast<f32x16_t (*)[NACC][1]>(&acc[0]));

  // ---- the block's slab [C][9][C] (co, tap, ci): acc lane layout row = co, col = ci
  float* slab = a.ws + ((long long)blockIdx.x * gridDim.y + g) * (long long)C * 9 * C;
  const int col = lane & 31;
  auto put = [&](const f32x16_t& v, int tap, int co0, int ci0) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * hf;
      slab[((long long)co * 9 + tap) * C + ci0 + col] = v[r];
    }
  };
  if constexpr (C == 32) {
    put(acc[0], wid, 0, 0);
    put(acc[1], wid + 4, 0, 0);
    // tap 8: the four waves' partial tiles summed in wave order through LDS
    __syncthreads();   // the strip images are no longer read
    float* red = reinterpret_cast<float*>(lds);   // [4][32 co][32 ci]
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wid * 1024 + ((r & 3) + 8 * (r >> 2) + 4 * hf) * 32 + col] = acc[2][r];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = tid * 4 + k, co = e >> 5, ci = e & 31;
      slab[((long long)co * 9 + 8) * C + ci] = ((red[e] + red[1024 + e]) + red[2048 + e]) + red[3072 + e];
    }
  } else {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) put(acc[tap], tap, cot, cit);
  }
}

template <int W, int C, int SPB>
int go(const XWHArgs& a, int G, hipStream_t st) {
  const int blocks = a.N * (a.H / 8) / SPB;
  if (a.x_coef) hipLaunchKernelGGL((xwgrad_halo_kernel<W, C, SPB, true>), dim3(blocks, G), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((xwgrad_halo_kernel<W, C, SPB, false>), dim3(blocks, G), dim3(256), 0, st, a);
  DBA_LAUNCH_CHECK();
}

}  // namespace

// rows per slab (mchunk) of the patch-reuse weight gradient for this shape, 0 = not handled
int xwgrad_halo_rows(int H, int W, int Cin, int Cout) {
  if (H != W || Cin != Cout) return 0;
  if (W == 32 && Cin == 32) return 2 * 8 * W;   // SPB 2: 128 slabs per 64-image replica
  if (W == 16 && Cin == 64) return 2 * 8 * W;   // SPB 2 (one image): 64 slabs
  return 0;
}

int xwgrad_halo_launch(const XWHArgs& a, int G, int W, int C, hipStream_t st) {
  if (xwgrad_halo_rows(a.H, W, C, C) == 0 || (a.H % 16) || !a.amax_dy || !a.amax_x) return -100;
  if (((uintptr_t)a.dy & 15) || ((uintptr_t)a.x & 15) || (a.dy_gstride & 3) || (a.x_gstride & 3)) return -100;
  if (W == 32 && C == 32) return go<32, 32, 2>(a, G, st);
  if (W == 16 && C == 64) return go<16, 64, 2>(a, G, st);
  return -100;
}
