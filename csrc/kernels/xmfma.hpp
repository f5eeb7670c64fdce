// Shared device helpers of the fp32 (split-plane MFMA) conv kernels (xconv.hpp, xhalo.hpp, xconv_fwd.hip, xwgrad.hip, xblock.hip):
// buffer loads with out-of-range zero fill, the scaled-fp16 pair split, the per-launch fp16
// scales (HScale), the swizzled LDS operand images and the compile-time MFMA / staging schedule
// (mma_half).  See xconv.hpp's header for the math.
#pragma once
#include "common.hpp"
#include <type_traits>
#include <utility>

namespace {

typedef __attribute__((ext_vector_type(2))) float f32x2v;

// bounds-checked loads: a raw buffer load whose byte offset is past num_records returns zeros,
// so out-of-image taps and past-K columns need no branch (offset kOOB)
constexpr int kOOB = (int)0x80000000;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}
__device__ __forceinline__ uint2 bload8(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, 0));
}
__device__ __forceinline__ float bload1(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}

// ---- fp16 pair split: x*2^s = h + l + e, h = f16(x*2^s), l = f16(x*2^s - h),
// |e| <= 2^-22 |x| (11 significant bits per plane against bf16's 8), 3 MFMAs per product
// (hh + hl + lh; the dropped ll term is <= 2^-22 |xy|).  fp16's exponent range is narrow, so
// each operand is scaled by a power of two fixed for the whole launch, chosen from the
// operand's max |x| (per replica / weight slot, computed by dba_amax or fused into the
// producing kernel): max * 2^s in [2^14, 2^15).  Scaling is exact, and the accumulators'
// 2^(sa+sb) is removed exactly in the epilogue; elements below max * 2^-17 keep an absolute
// error under max * 2^-40.
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2v;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;

__device__ __forceinline__ uint32_t cvt_pkh(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){a, b}, f16x2v));
}
__device__ __forceinline__ f32x2v unpkh(uint32_t u) {
  return __builtin_convertvector(__builtin_bit_cast(f16x2v, u), f32x2v);
}
__device__ __forceinline__ void split4h(float a, float b, float c, float d, float sc, uint2 (&o)[2]) {
  a *= sc; b *= sc; c *= sc; d *= sc;   // exact (power of two)
  const uint32_t h0 = cvt_pkh(a, b), h1 = cvt_pkh(c, d);
  const f32x2v u0 = unpkh(h0), u1 = unpkh(h1);
  o[0] = make_uint2(h0, h1);
  o[1] = make_uint2(cvt_pkh(a - u0.x, b - u0.y), cvt_pkh(c - u1.x, d - u1.y));   // exact residuals
}
constexpr int kSMax = 100;   // scale exponent cap (operands below 2^-85 stay unnormalised)
// scale exponent for a max |x| given as float bits (0 / subnormal max: the cap)
__device__ __forceinline__ int hexp(int maxbits) { return min(kSMax, 141 - (maxbits >> 23)); }
struct HScale {
  float ma = 1.f, mb = 1.f;   // fill multipliers 2^sa, 2^sb
  int s = 0;                  // the accumulators hold sum * 2^s
  __device__ __forceinline__ void init(int maxa, int maxb) {
    const int sa = hexp(maxa), sb = hexp(maxb);
    ma = __uint_as_float((uint32_t)(sa + 127) << 23);
    mb = __uint_as_float((uint32_t)(sb + 127) << 23);
    s = sa + sb;
  }
  template <int MI, int NJ>
  __device__ __forceinline__ void finish(f32x16_t (&acc)[MI][NJ]) const {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = ldexpf(acc[i][j][r], -s);
  }
};

// LDS images: per plane, rows of 32 reduction elements (64 B = 4 x 16-B chunks).  A row's
// 16-B chunk c is stored at chunk c ^ swz so the ds_read_b128 fragment reads (lane groups
// {0-3,12-15,20-27} / {4-11,16-19,28-31}) hit 16 distinct bank slots.
//   conv  (ROWPERM = false): physical row = logical row, swz = (row >> 2) & 3;
//   wgrad (ROWPERM = true) : operand rows are written 4 at a time (a transposed 4x4 micro
//     tile), so logical row n lives at physical (n & 3) * (R / 4) + (n >> 2) with swz = n & 3
//     — both the transposing ds_write_b64 stores and the fragment reads are conflict-free.
template <bool ROWPERM, int R>
__device__ __forceinline__ int prow(int n) {
  if constexpr (ROWPERM) return (n & 3) * (R / 4) + (n >> 2);
  else return n;
}
template <bool ROWPERM>
__device__ __forceinline__ int pswz(int n) {
  if constexpr (ROWPERM) return n & 3;
  else return (n >> 2) & 3;
}

// one 32-deep reduction step of a wave's MI x NJ block of 32x32 tiles from an LDS image:
// A rows [arow0, arow0 + 32 MI) of the region at row offset 0 (RA rows), B rows at RA + ...
// ``fill(q)`` (q = 0 .. NQ-1) is staging work of the NEXT step (split + LDS stores of one
// 4-element quarter per call), spread evenly between the MFMAs so the VALU split and the
// ds_write traffic issue in the MFMA gaps instead of after them.
// one 32x32x16 MFMA on fp16 split planes (H: the fp16 pair — the only split of the family)
template <bool H>
__device__ __forceinline__ f32x16_t mfma16(const uint4& a, const uint4& b, const f32x16_t& c) {
  static_assert(H, "fp16 pair");
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0,
                                                0, 0);
}

// compile-time loop: f(std::integral_constant<int, 0>) ... f(integral_constant<N-1>)
template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}
// plane product p of the P-plane split (total order <= P-1, the small ones first)
constexpr int prod_pa(int P, int p) {
  int k = 0;
  for (int s = P - 1; s >= 0; --s)
    for (int pa = 0; pa <= s; ++pa, ++k)
      if (k == p) return pa;
  return 0;
}
constexpr int prod_pb(int P, int p) {
  int k = 0;
  for (int s = P - 1; s >= 0; --s)
    for (int pa = 0; pa <= s; ++pa, ++k)
      if (k == p) return s - pa;
  return 0;
}

// the MFMAs of half-step KK (16 reduction elements) of a wave's MI x NJ tiles, with the
// staging fills fill(q) (q = 0 .. NQ-1, compile-time constants) of the NEXT step spread evenly
// between them, so the VALU split / ds_write / reload traffic issues in the MFMA gaps
template <int MI, int NJ, int P, bool H, int NQ, int KK, typename Fill>
__device__ __forceinline__ void mma_half(const uint4 (&af)[P][MI], const uint4 (&bfr)[P][NJ],
                                         f32x16_t (&acc)[MI][NJ], Fill&& fill) {
  constexpr int PER = P * (P + 1) / 2 * MI * NJ, T = 2 * PER;   // MFMAs per half / whole step
  sfor<PER>([&](auto C) __attribute__((always_inline)) {
    constexpr int c = decltype(C)::value;
    constexpr int p = c / (MI * NJ), i = (c / NJ) % MI, j = c % NJ;
    acc[i][j] = mfma16<H>(af[prod_pa(P, p)][i], bfr[prod_pb(P, p)][j], acc[i][j]);
    constexpr int cnt = KK * PER + c + 1;
    sfor<NQ>([&](auto Q) __attribute__((always_inline)) {
      constexpr int q = decltype(Q)::value;
      if constexpr (cnt * NQ >= (q + 1) * T && (cnt - 1) * NQ < (q + 1) * T) fill(q);
    });
  });
}

template <int MI, int NJ, int P, bool H, bool ROWPERM, int RA, int RB, int NQ, typename Fill>
__device__ __forceinline__ void mma_step(const uint4* __restrict__ L, int PL, int arow0, int brow0,
                                         f32x16_t (&acc)[MI][NJ], int lane, Fill&& fill) {
  const int fr = lane & 31, hf = lane >> 5;
  sfor<2>([&](auto KK) __attribute__((always_inline)) {
    const int ch = decltype(KK)::value * 2 + hf;
    uint4 af[P][MI], bfr[P][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int n = arow0 + i * 32 + fr;
      const int o = prow<ROWPERM, RA>(n) * 4 + (ch ^ pswz<ROWPERM>(n));
#pragma unroll
      for (int p = 0; p < P; ++p) af[p][i] = L[p * PL + o];
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = brow0 + j * 32 + fr;
      const int o = (RA + prow<ROWPERM, RB>(n)) * 4 + (ch ^ pswz<ROWPERM>(n));
#pragma unroll
      for (int p = 0; p < P; ++p) bfr[p][j] = L[p * PL + o];
    }
    mma_half<MI, NJ, P, H, NQ, decltype(KK)::value>(af, bfr, acc, fill);
  });
}

// store the P planes of 4 consecutive reduction elements (8-B slot q of logical row n)
template <int P, bool ROWPERM, int R>
__device__ __forceinline__ void lds_put(uint4* __restrict__ L, int PL, int roff, int n, int q, const uint2 (&s)[P]) {
  const int o = (roff + prow<ROWPERM, R>(n)) * 4 + ((q >> 1) ^ pswz<ROWPERM>(n));
#pragma unroll
  for (int p = 0; p < P; ++p) ((uint2*)&L[p * PL + o])[q & 1] = s[p];
}

// patch swizzle of the halo kernels (xhalo.hpp xhalo_kernel, xblock.hip): pixel pp (patch
// column col) holds CS / 8 16-B chunks, chunk q at q ^ hswz
template <int W, int CS>
__device__ __forceinline__ int hswz(int pp, int col) {
  constexpr int CH = CS / 8;                    // 16-B chunks per pixel (4 or 8)
  if constexpr (CH == 4) return (pp >> 2) & 3;
  else return (col >> 1) & 7;
}

}  // namespace
