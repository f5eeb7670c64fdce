// Generation-3 weight gradient for the convolutions pwgrad.hip does not tile: the strided
// stage-entry 3x3 convs, the 1x1 stride-2 shortcuts and the 3-channel stem
// (reference: ResNet-18 backward of models/resnet_cifar.py / resnet_tinyimagenet.py, the
// `loss.backward()` in image_train.py:120-123).
//
//   dW[co][j] (+)= sum over output pixels m of dY[m][co] * X_col[m][j],  j = (kh, kw, ci)
//
// The reduction axis is the pixel.  Both operands stay in their natural NHWC row layout in
// LDS and are consumed column-wise with gfx950's transposing read (ds_read_b64_tr_b16):
//   * dY tile  [KM pixels][BCO channels] — 16-B LDS-DMA chunks, 128-B panel rows swizzled;
//   * X  tile  [KM pixels][BJ im2col columns] — gathered straight from the image by the DMA:
//     16-B chunks (Cin % 8 == 0: one chunk = 8 channels of one tap); the 3-channel stem
//     (XB == 2, a tap row is 6 bytes) gathers single elements through registers instead
//     (sub-dword LDS-DMA does not land lane-contiguously);
//   * 3-deep LDS ring with counted vmcnt and raw barriers (DMA of k-steps t+1, t+2 in flight
//     while t computes), 32x32x16 MFMAs, optional in-block split of the pixel axis (WK);
//   * split-K over pixel runs chosen IN-KERNEL from the number of replicas active this step
//     (the launch lives in a HIP graph captured once for all G), fp32 atomics when split.
#include "common.hpp"
#include <algorithm>
#include <stdlib.h>
#include <type_traits>

namespace {

typedef short v4i16_t __attribute__((ext_vector_type(4)));

// f(integral_constant<0>) ... f(integral_constant<N-1>): compile-time indices, so register
// arrays indexed by them never fall back to scratch
template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

struct W3Args {
  const uint16_t* dy; long long dy_gstride;     // [G][N][Ho][Wo][Cout]
  const uint16_t* x; long long x_gstride;       // [G][N][H][W][Cin]
  float* dw; long long dw_gstride;              // [G][Cout][KH][KW][Cin] fp32 (accumulated)
  const int* nvalid;
  const uint16_t* zeros;
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad;
  int G, tiles, ncu, bpc;
  float atom_budget;                            // fp32 atomics a split-K launch may issue
};

// 16-byte-chunk XOR for a 64-channel (128-B) panel row: the 4 rows of a transposed read
// land on distinct bank slots (same rule as pwgrad.hip); 32-channel rows need none.
template <int PW>
__device__ __forceinline__ int swz(int row) {
  if constexpr (PW == 64) return ((row >> 1) & 1) << 2;
  else return 0;
}

template <int PW, int KM>
__device__ __forceinline__ int tile_off(int row, int col) {   // byte offset in a panelled tile
  const int panel = col / PW, cc = col - panel * PW;
  const int chunk = cc >> 3;
  return panel * (KM * PW * 2) + row * PW * 2 + ((chunk ^ swz<PW>(row)) << 4) + ((cc & 7) << 1);
}

template <int BCO, int BJ, int KM, int WCO, int WJ, int WK, int XB>
__global__ __launch_bounds__(256) void wgrad3_kernel(W3Args a) {
  static_assert(WCO * WJ * WK == 4, "4 waves");
  constexpr int NT = 256;
  constexpr int TCO = BCO / WCO, TJ = BJ / WJ;
  constexpr int MI = TCO / 32, NJ = TJ / 32;
  constexpr int PCO = BCO < 64 ? BCO : 64, PJ = BJ < 64 ? BJ : 64;
  static_assert(MI >= 1 && NJ >= 1 && KM % (16 * WK) == 0, "tile geometry");
  static_assert(XB == 16 || BJ == 32, "element gathers use unswizzled 32-column rows");
  constexpr int DYCH = KM * BCO / 8;                       // 16-B chunks of the dY tile
  constexpr int XEL = XB == 16 ? KM * BJ / 8 : 0;         // DMA chunks of the X tile
  constexpr int NXR = XB == 16 ? 0 : KM * BJ / NT;         // register-staged X elements per thread
  static_assert(XB == 16 || NXR == KM / (NT / BJ), "element path geometry");
  constexpr int NID = (DYCH + NT - 1) / NT, NIX = (XEL + NT - 1) / NT;
  constexpr int NI = NID + NIX;                            // DMA instructions per thread per stage
  static_assert(2 * NI <= 63, "vmcnt range");
  constexpr int DYB = NID * NT * 16, XBYTES = XB == 16 ? NIX * NT * 16 : KM * BJ * 2;
  constexpr int STAGE = DYB + XBYTES;
  constexpr int NBUF = XB == 16 ? 3 : 2;
  __shared__ __attribute__((aligned(16))) char lds[NBUF][STAGE];
  constexpr int kWaitKeep = (NI & 15) | ((NI >> 4) << 14) | (0x7 << 4) | (0xF << 8);   // vmcnt(NI)
  constexpr int kWaitAll = (0x7 << 4) | (0xF << 8);                                    // vmcnt(0)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = blockIdx.y;
  const int J = a.KH * a.KW * a.Cin;
  const int tiles_j = (J + BJ - 1) / BJ;
  const int co0 = (blockIdx.z / tiles_j) * BCO, j0 = (blockIdx.z % tiles_j) * BJ;
  const int HoWo = a.Ho * a.Wo;
  const int Mv = valid_rows(a.nvalid, g, a.N) * HoWo;
  if (Mv == 0) return;
  const int nks = (Mv + KM - 1) / KM;
  // split-K from the replicas active this step
  int active = 0;
  for (int r = 0; r < a.G; ++r) active += valid_rows(a.nvalid, r, a.N) > 0;
  const float by_cus = (float)(a.ncu * a.bpc) / (float)(active * a.tiles);
  const float by_atomics = a.atom_budget / ((float)active * a.Cout * J);
  const int S = max(1, min(min(nks, (int)gridDim.x), (int)fminf(by_cus, by_atomics)));
  if ((int)blockIdx.x >= S) return;
  const int per = (nks + S - 1) / S;
  const int t0 = blockIdx.x * per, t1 = min(nks, t0 + per);
  if (t0 >= t1) return;
  const bool atomic = S > 1;
  const uint16_t* __restrict__ dyg = a.dy + (long long)g * a.dy_gstride;
  const uint16_t* __restrict__ xg = a.x + (long long)g * a.x_gstride;

  // X staging: a thread's column (tap, ci) is the same for every k-step (the chunk swizzle
  // depends only on bit 1 of the row, and rows advance in steps of RS, a multiple of 4), so
  // the im2col decode is hoisted; rows walk forward by RS with carries instead of divisions.
  constexpr int CPR = XB == 16 ? PJ / 8 : BJ;      // X elements per tile row
  constexpr int RS = NT / CPR;                     // row step between a thread's elements
  constexpr int NPAN = XB == 16 ? BJ / PJ : 1;
  constexpr int IPP = KM / RS;                     // elements per thread per panel
  static_assert(KM % RS == 0 && RS % 4 == 0, "row walk");
  const int r0 = tid / CPR;
  int xci[NPAN], xdh[NPAN], xdw[NPAN];
  bool xjv[NPAN];
#pragma unroll
  for (int pn = 0; pn < NPAN; ++pn) {
    const int j = j0 + pn * PJ + (XB == 16 ? (((tid % CPR) ^ swz<PJ>(r0)) << 3) : tid % CPR);
    const int tap = j / a.Cin, kh = tap / a.KW;
    xjv[pn] = j < J;
    xci[pn] = j - tap * a.Cin;
    xdh[pn] = kh - a.pad;
    xdw[pn] = tap - kh * a.KW - a.pad;
  }
  const int dq = RS % a.Wo, dp = (RS / a.Wo) % a.Ho, dn = RS / HoWo;
  // calls f(k, pn, src) for the thread's IPP x NPAN X elements of k-step tt
  auto walk_x = [&](int tt, auto&& f) __attribute__((always_inline))  {
    int m = tt * KM + r0;
    int n = m / HoWo, p = (m - n * HoWo) / a.Wo;
    int q = m - n * HoWo - p * a.Wo;
    static_for<IPP>([&](auto kc) __attribute__((always_inline))  {
      constexpr int k = decltype(kc)::value;
      const int hb = p * a.stride, wb = q * a.stride;
      static_for<NPAN>([&](auto pc) __attribute__((always_inline))  {
        constexpr int pn = decltype(pc)::value;
        const int hi = hb + xdh[pn], wi = wb + xdw[pn];
        const uint16_t* src = a.zeros;
        if (m < Mv && xjv[pn] && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W)
          src = xg + (((long long)n * a.H + hi) * a.W + wi) * a.Cin + xci[pn];
        f(std::integral_constant<int, k>{}, std::integral_constant<int, pn>{}, src);
      });
      m += RS;
      q += dq;
      if (q >= a.Wo) { q -= a.Wo; ++p; }
      p += dp;
      if (p >= a.Ho) { p -= a.Ho; ++n; }
      n += dn;
    });
  };
  auto stage = [&](int tt, int buf) __attribute__((always_inline))  {
    const int mb = tt * KM;
    char* base = lds[buf];
#pragma unroll
    for (int i = 0; i < NID; ++i) {
      const int e = tid + NT * i;
      const uint16_t* src = a.zeros;
      if (e < DYCH) {
        const int panel = e / (KM * PCO / 8), rem = e - panel * (KM * PCO / 8);
        const int row = rem / (PCO / 8), cpos = rem - row * (PCO / 8);
        const int co = co0 + panel * PCO + ((cpos ^ swz<PCO>(row)) << 3);
        const int m = mb + row;
        if (m < Mv && co < a.Cout) src = dyg + (long long)m * a.Cout + co;
      }
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(base + (i * NT + wid * 64) * 16),
                                       16, 0, 0);
    }
    if constexpr (XB == 16) {
      walk_x(tt, [&](auto kc, auto pc, const uint16_t* src) __attribute__((always_inline))  {
        const int i = decltype(pc)::value * IPP + decltype(kc)::value;                // chunk e = tid + NT*i: panel pn, row r0 + RS*k
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(base + DYB + (i * NT + wid * 64) * 16),
                                         16, 0, 0);
      });
    }
  };
  // element path (Cin % 8 != 0, BJ == 32): gathered through registers
  uint16_t xr[NXR > 0 ? NXR : 1];
  auto gather_x = [&](int tt) __attribute__((always_inline))  {
    if constexpr (XB == 2) walk_x(tt, [&](auto kc, auto, const uint16_t* src) __attribute__((always_inline))  { xr[decltype(kc)::value] = *src; });
  };
  auto write_x = [&](int buf) __attribute__((always_inline))  {
    uint16_t* L = reinterpret_cast<uint16_t*>(lds[buf] + DYB);
#pragma unroll
    for (int i = 0; i < NXR; ++i) L[(r0 + RS * i) * BJ + (tid % CPR)] = xr[i];
  };

  const int wk = wid / (WCO * WJ), wr = wid - wk * (WCO * WJ);
  const int wco = wr / WJ, wj = wr - wco * WJ;
  // transposed-read lane geometry: 16-lane group G4, row q within a 4-row block, 4-col group p4
  const int G4 = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
  const int hsel = G4 >> 1;
  const int colA = wco * TCO + 16 * (G4 & 1) + 4 * p4;
  const int colB = wj * TJ + 16 * (G4 & 1) + 4 * p4;

  f32x16_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto compute = [&](int buf) __attribute__((always_inline))  {
    const char* Ldy = lds[buf];
    const char* Lx = lds[buf] + DYB;
#pragma unroll
    for (int ks = wk; ks < KM / 16; ks += WK) {
      union { bf16x8_t v; v4i16_t h[2]; } fa[MI], fb[NJ];
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        const int px = ks * 16 + 8 * hsel + 4 * t2 + q;
#pragma unroll
        for (int i = 0; i < MI; ++i)
          fa[i].h[t2] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4i16_t*)(Ldy + tile_off<PCO, KM>(px, colA + 32 * i)));
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          fb[j].h[t2] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4i16_t*)(Lx + tile_off<PJ, KM>(px, colB + 32 * j)));
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i].v, fb[j].v, acc[i][j], 0, 0, 0);
    }
  };

  if constexpr (XB == 16) {
    // 3-deep ring: k-steps tt+1, tt+2 in flight while tt computes; counted vmcnt + raw barrier
    stage(t0, 0);
    if (t0 + 1 < t1) {
      stage(t0 + 1, 1);
      __builtin_amdgcn_s_waitcnt(kWaitKeep);
    } else {
      __builtin_amdgcn_s_waitcnt(kWaitAll);
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    int cur = 0;
    for (int tt = t0; tt < t1; ++tt) {
      compute(cur);
      if (tt + 1 < t1) {
        asm volatile("" ::: "memory");
        if (tt + 2 < t1) {
          stage(tt + 2, cur == 0 ? 2 : cur - 1);     // buffer of k-step tt-1
          __builtin_amdgcn_s_waitcnt(kWaitKeep);
        } else {
          __builtin_amdgcn_s_waitcnt(kWaitAll);
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        cur = cur == 2 ? 0 : cur + 1;
      }
    }
  } else {
    // double buffer: dY by DMA, X gathered into registers; both for tt+1 in flight during tt
    stage(t0, 0);
    gather_x(t0);
    write_x(0);
    __syncthreads();
    int cur = 0;
    for (int tt = t0; tt < t1; ++tt) {
      const bool more = tt + 1 < t1;
      if (more) {
        stage(tt + 1, cur ^ 1);
        gather_x(tt + 1);
      }
      compute(cur);
      if (more) write_x(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  }

  if constexpr (WK > 1) {   // fold the pixel groups' partials into group 0 through the idle ring
    static_assert((WK - 1) * WCO * WJ * MI * NJ * 16 * 64 * 4 <= NBUF * STAGE, "reduction fits the ring");
    float* red = reinterpret_cast<float*>(&lds[0][0]);
    __syncthreads();
    if (wk > 0) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            red[(((((wk - 1) * WCO * WJ + wr) * MI + i) * NJ + j) * 16 + r) * 64 + lane] = acc[i][j][r];
    }
    __syncthreads();
    if (wk > 0) return;
#pragma unroll
    for (int k2 = 1; k2 < WK; ++k2)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            acc[i][j][r] += red[(((((k2 - 1) * WCO * WJ + wr) * MI + i) * NJ + j) * 16 + r) * 64 + lane];
  }
  // D[co][j]: lane -> column j (lane & 31), registers -> co rows
  float* __restrict__ dwg = a.dw + (long long)g * a.dw_gstride;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = j0 + wj * TJ + 32 * j + (lane & 31);
    if (col >= J) continue;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wco * TCO + 32 * i + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
        if (co >= a.Cout) continue;
        float* d = dwg + (long long)co * J + col;
        if (atomic) atomicAdd(d, acc[i][j][r]);
        else *d += acc[i][j][r];                    // sole writer of this element
      }
  }
}

int num_cus_3() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <int BCO, int BJ, int KM, int WCO, int WJ, int WK, int XB>
int launch_w3(const W3Args& a0, int G, hipStream_t st) {
  constexpr int NT = 256;
  constexpr int NID = (KM * BCO / 8 + NT - 1) / NT;
  constexpr int STAGE = NID * NT * 16 + KM * BJ * 2;
  W3Args a = a0;
  const int J = a.KH * a.KW * a.Cin;
  a.G = G;
  a.tiles = ceil_div(a.Cout, BCO) * ceil_div(J, BJ);
  a.ncu = num_cus_3();
  a.bpc = std::max(1, std::min(8, (160 * 1024) / ((XB == 16 ? 3 : 2) * STAGE)));
  const int nks = ceil_div((long long)a.N * a.Ho * a.Wo, KM);
  // grid.x = the largest split any activity pattern can ask for (one active replica)
  const char* ab = getenv("DBA_W3_ATOMICS");
  a.atom_budget = ab ? (float)atof(ab) : 1.2e7f;
  const double s1 = std::min((double)a.ncu * a.bpc / a.tiles, (double)a.atom_budget / ((double)a.Cout * J));
  const int smax = std::max(1, std::min(nks, (int)s1));
  dim3 grid(smax, G, a.tiles);
  hipLaunchKernelGGL((wgrad3_kernel<BCO, BJ, KM, WCO, WJ, WK, XB>), grid, dim3(NT), 0, st, a);
  DBA_LAUNCH_CHECK();
}

}  // namespace

// dW (+)= weight gradient of a general conv (any stride / pad / kernel).  Needs Cout % 8 == 0;
// Cin % 8 == 0 uses 16-B im2col chunks, other Cin (the 3-channel stem) element gathers.
// Returns -100 for shapes it does not handle.
DBA_EXPORT int dba_wgrad3(const void* dy, long long dy_gstride, const void* x, long long x_gstride, float* dw,
                          long long dw_gstride, const int* nvalid, const void* zeros, int G, int N, int H, int W,
                          int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad, void* stream) {
  if (Cout % 8 != 0) return -100;
  W3Args a{(const uint16_t*)dy, dy_gstride, (const uint16_t*)x, x_gstride, dw, dw_gstride, nvalid,
           (const uint16_t*)zeros, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, G, 1, 256, 1, 3.0e6f};
  hipStream_t st = (hipStream_t)stream;
  const int J = KH * KW * Cin;
  if (Cin % 8 != 0) {
    if (Cout > 64) return -100;
    return launch_w3<32, 32, 128, 1, 1, 4, 2>(a, G, st);
  }
  if (J <= 32) return launch_w3<64, 32, 64, 2, 1, 2, 16>(a, G, st);
  // 128x128 tiles (1 block per CU) only when they alone fill the chip twice over
  const long long big = (long long)ceil_div(Cout, 128) * ceil_div(J, 128) * G;
  if (Cout >= 128 && J >= 128 && big >= 2LL * num_cus_3()) return launch_w3<128, 128, 64, 2, 2, 1, 16>(a, G, st);
  return launch_w3<64, 64, 64, 2, 2, 1, 16>(a, G, st);
}
