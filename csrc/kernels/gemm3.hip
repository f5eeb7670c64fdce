// Generation-3 implicit-GEMM convolution (gfx950): the wide layers whose source channel
// count is a multiple of 64 (ResNet stages 3-4, the stage-entry convs, the stride-1 data
// gradients run as forward convs of dY).
//
// vs conv2.hip (register-staged, 2 LDS buffers, padded rows, one __syncthreads per k-step
// that drains every load):
//   * A (activation rows) and B (weight rows) stream global -> LDS by LDS-DMA
//     (global_load_lds_dwordx4): no staging registers, no ds_write pass;
//   * an NS-deep LDS ring (NS = 2 by default: 64 KB, two blocks per CU — measured faster than
//     NS = 3 at one block per CU) with counted vmcnt and a raw s_barrier; k-step kc+NS-1 is
//     issued before kc computes;
//   * 128-B LDS rows with a 16-B chunk XOR swizzle (chunk ^ ((row >> 1) & 7)) applied on the DMA
//     SOURCE address (the LDS image must be lane-linear): every ds_read_b128 lane group of a
//     32-row fragment read hits 16 distinct bank slots;
//   * Cs % 64 == 0, so one k-step is one tap x 64 contiguous channels: each A row is a single
//     128-B run of the source pixel (or the zero page), no per-chunk tap decode.
// The epilogue (fp32 tile staged through the drained ring, bias / residual / ReLU, 16-B
// stores) matches conv2.hip.
#include "common.hpp"
#include <algorithm>
#include <cstdlib>

namespace {

struct G3Args {
  const uint16_t* src; long long src_gstride;   // [G][N][Hs][Ws][Cs]
  const uint16_t* w; long long w_sstride;       // [slots][Ncol][K]
  const int* wsel;
  const float* bias; long long b_sstride;
  const uint16_t* res;                          // [G][M][Ncol]
  void* out; long long out_gstride;             // [G][M][Ncol]
  const int* nvalid;
  const uint16_t* zeros;
  int N, Hs, Ws, Cs, Ho, Wo, Ncol, KH, KW, stride, pad, relu;
  int tiles_n;
  long long out_zstride;                        // split-K: fp32 slab of K-slice z at out + z * out_zstride
};

__device__ __forceinline__ int g3swz(int row) { return (row >> 1) & 7; }

template <int BM, int BN, int NS, typename OutT>
__global__ __launch_bounds__(256) void igemm3_kernel(G3Args a) {
  constexpr int TM = BM / 2, TN = BN / 2;            // 2x2 waves
  constexpr int MI = TM / 32, NJ = TN / 32;
  constexpr int CHA = BM * 8, CHB = BN * 8;          // 16-B chunks per stage
  constexpr int NIA = CHA / 256, NIB = CHB / 256;
  constexpr int NI = NIA + NIB;                      // DMA instructions per thread per stage
  constexpr int STG = CHA + CHB;
  static_assert(BM * BN * 4 <= NS * STG * 16, "epilogue tile fits the ring");
  constexpr int KEEP = NI * (NS - 2);                // DMA instructions left in flight at a wait
  constexpr int kWaitKeep = (KEEP & 15) | ((KEEP >> 4) << 14) | (0x7 << 4) | (0xF << 8);
  constexpr int kWaitAll = (0x7 << 4) | (0xF << 8);
  __shared__ __attribute__((aligned(16))) uint4 ring[NS][STG];

  const int g = blockIdx.y;
  const int HoWo = a.Ho * a.Wo;
  const int Mv = valid_rows(a.nvalid, g, a.N) * HoWo;
  const int tn = blockIdx.x % a.tiles_n, tm = blockIdx.x / a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mv) return;
  const int K = a.KH * a.KW * a.Cs;
  // split-K (gridDim.z > 1, small launches): this block reduces k-steps [kb, kb + nk) into its
  // own fp32 slab; splitk_reduce_kernel sums the slabs and applies the epilogue
  const int nk_all = K / 64;
  const int kb = (int)((long long)nk_all * blockIdx.z / gridDim.z);
  const int nk = (int)((long long)nk_all * (blockIdx.z + 1) / gridDim.z) - kb;
  const uint16_t* __restrict__ src = a.src + (long long)g * a.src_gstride;
  const int slot = a.wsel ? a.wsel[g] : g;
  const uint16_t* __restrict__ Wp = a.w + (long long)slot * a.w_sstride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // per-thread DMA rows (fixed for the block): A row -> source pixel, B row -> weight row
  int an[NIA], ap[NIA], aq[NIA], acs[NIA];
#pragma unroll
  for (int i = 0; i < NIA; ++i) {
    const int e = tid + 256 * i, row = e >> 3;
    acs[i] = (e & 7) ^ g3swz(row);
    const int m = m0 + row;
    if (m < Mv) {
      const int n = m / HoWo, rem = m - n * HoWo;
      an[i] = n;
      ap[i] = (rem / a.Wo) * a.stride - a.pad;
      aq[i] = (rem - (rem / a.Wo) * a.Wo) * a.stride - a.pad;
    } else {
      an[i] = -1; ap[i] = 0; aq[i] = 0;
    }
  }
  const uint16_t* brow[NIB];
#pragma unroll
  for (int i = 0; i < NIB; ++i) {
    const int e = tid + 256 * i, row = e >> 3;
    brow[i] = n0 + row < a.Ncol ? Wp + (long long)(n0 + row) * K + ((e & 7) ^ g3swz(row)) * 8 : nullptr;
  }

  auto stage = [&](int kc, int buf) {
    const int tap = (kc * 64) / a.Cs, c0 = kc * 64 - tap * a.Cs;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
#pragma unroll
    for (int i = 0; i < NIA; ++i) {
      const uint16_t* p = a.zeros;
      const int hs = ap[i] + kh, ws = aq[i] + kw;
      if (an[i] >= 0 && (unsigned)hs < (unsigned)a.Hs && (unsigned)ws < (unsigned)a.Ws)
        p = src + (((long long)an[i] * a.Hs + hs) * a.Ws + ws) * a.Cs + c0 + acs[i] * 8;
      __builtin_amdgcn_global_load_lds((const void*)p,
                                       (__attribute__((address_space(3))) void*)&ring[buf][i * 256 + wid * 64],
                                       16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NIB; ++i) {
      const uint16_t* p = brow[i] ? brow[i] + kc * 64 : a.zeros;
      __builtin_amdgcn_global_load_lds((const void*)p,
                                       (__attribute__((address_space(3))) void*)&ring[buf][CHA + i * 256 + wid * 64],
                                       16, 0, 0);
    }
  };

  f32x16_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // NS-deep ring: k-step kc+NS-1 is issued at the top of iteration kc (into the buffer of
  // kc-1, retired by the previous barrier) and the wait at the bottom leaves NS-2 stages in
  // flight across the raw barrier.
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) stage(kb + s, s);
  if (nk >= NS - 1) {
    // all NS-1 prologue stages were issued: wait for k-step 0 only
    __builtin_amdgcn_s_waitcnt(kWaitKeep);
  } else {
    __builtin_amdgcn_s_waitcnt(kWaitAll);      // short K: fewer stages in flight, drain them
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const int fr = lane & 31, hi = lane >> 5;
  int cur = 0;
  for (int kc = 0; kc < nk; ++kc) {
    const int pre = kc + NS - 1;
    if (pre < nk) stage(kb + pre, cur == 0 ? NS - 1 : cur - 1);
    const uint4* L = ring[cur];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int ch = kk * 2 + hi;
      bf16x8_t af[MI], bfr[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wm * TM + i * 32 + fr;
        af[i] = *(const bf16x8_t*)&L[row * 8 + (ch ^ g3swz(row))];
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int row = wn * TN + j * 32 + fr;
        bfr[j] = *(const bf16x8_t*)&L[CHA + row * 8 + (ch ^ g3swz(row))];
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kc + 1 < nk) {
      asm volatile("" ::: "memory");
      // k-step kc+1 must have landed; the younger ones may stay in flight
      if (kc + NS - 1 < nk) __builtin_amdgcn_s_waitcnt(kWaitKeep);
      else __builtin_amdgcn_s_waitcnt(kWaitAll);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      cur = cur == NS - 1 ? 0 : cur + 1;
    }
  }

  // ---- epilogue: fp32 tile through the (drained) ring, 8-wide pass with bias / res / ReLU
  __syncthreads();
  float* Cst = reinterpret_cast<float*>(&ring[0][0]);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        const int col = wn * TN + j * 32 + fr;
        Cst[row * BN + col] = acc[i][j][r];
      }
  __syncthreads();
  OutT* out = (OutT*)a.out + (long long)g * a.out_gstride + (long long)blockIdx.z * a.out_zstride;
  const float* bias = a.bias ? a.bias + (long long)slot * a.b_sstride : nullptr;
  const uint16_t* res = a.res ? a.res + (long long)g * a.out_gstride : nullptr;
  constexpr int CH8 = BN / 8;
  for (int e = tid; e < BM * CH8; e += 256) {
    const int row = e / CH8, c8 = (e - row * CH8) * 8;
    const int m = m0 + row;
    const int n = n0 + c8;
    if (m >= Mv || n >= a.Ncol) continue;
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = Cst[row * BN + c8 + t];
    const long long o = (long long)m * a.Ncol + n;
    if (bias) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] += bias[n + t];
    }
    if (res) {
      const uint4 rv = *(const uint4*)(res + o);
      const uint16_t* rp = (const uint16_t*)&rv;
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] += bf2f(rp[t]);
    }
    if (a.relu) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = fmaxf(v[t], 0.f);
    }
    if constexpr (sizeof(OutT) == 2) {
      uint4 pk;
      uint16_t* pp = (uint16_t*)&pk;
#pragma unroll
      for (int t = 0; t < 8; ++t) pp[t] = f2bf(v[t]);
      *(uint4*)((uint16_t*)out + o) = pk;
    } else {
#pragma unroll
      for (int t = 0; t < 8; ++t) ((float*)out)[o + t] = v[t];
    }
  }
}

template <int BM, int BN, int NS, typename OutT>
int launch3(G3Args a, int G, hipStream_t st, int splitk = 1) {
  const long long M = (long long)a.N * a.Ho * a.Wo;
  a.tiles_n = ceil_div(a.Ncol, BN);
  dim3 grid((unsigned)(ceil_div(M, BM) * a.tiles_n), G, splitk);
  hipLaunchKernelGGL((igemm3_kernel<BM, BN, NS, OutT>), grid, dim3(256), 0, st, a);
  DBA_LAUNCH_CHECK();
}

// Sum of the split-K slabs ws[z][g][m][n] + bias (+ residual) (ReLU) -> bf16, valid rows only.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int S, long long zstride,
                                                            long long ws_gstride, const int* __restrict__ nvalid,
                                                            int N, int HoWo, int Ncol, const float* __restrict__ bias,
                                                            long long b_sstride, const int* __restrict__ wsel,
                                                            const uint16_t* __restrict__ res, long long out_gstride,
                                                            int relu, uint16_t* __restrict__ out) {
  const int g = blockIdx.y;
  const long long total = (long long)valid_rows(nvalid, g, N) * HoWo * (Ncol / 8);
  const float* __restrict__ src = ws + (long long)g * ws_gstride;
  const float* __restrict__ bp = bias ? bias + (long long)(wsel ? wsel[g] : g) * b_sstride : nullptr;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const long long e = t * 8;
    const int n = (int)(e % Ncol);
    float v[8];
    {
      const float4 a0 = *(const float4*)(src + e), a1 = *(const float4*)(src + e + 4);
      v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w; v[4] = a1.x; v[5] = a1.y; v[6] = a1.z; v[7] = a1.w;
    }
    for (int z = 1; z < S; ++z) {
      const float* q = src + z * zstride + e;
      const float4 a0 = *(const float4*)q, a1 = *(const float4*)(q + 4);
      v[0] += a0.x; v[1] += a0.y; v[2] += a0.z; v[3] += a0.w; v[4] += a1.x; v[5] += a1.y; v[6] += a1.z; v[7] += a1.w;
    }
    if (bp) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += bp[n + i];
    }
    const long long o = (long long)g * out_gstride + e;
    if (res) {
      const uint4 rv = *(const uint4*)(res + o);
      const uint16_t* rp = (const uint16_t*)&rv;
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += bf2f(rp[i]);
    }
    uint4 pk;
    uint16_t* pp = (uint16_t*)&pk;
#pragma unroll
    for (int i = 0; i < 8; ++i) pp[i] = f2bf(relu ? fmaxf(v[i], 0.f) : v[i]);
    *(uint4*)(out + o) = pk;
  }
}

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

// launches with fewer 128x128 tiles than this take the small-tile path
bool g3_small(long long M, int G, int Cout) {
  static const int limit = env_int("DBA_G3_SMALL_LIMIT", 512);
  return M * G / 128 * ((Cout + 127) / 128) < limit;
}

// tile shape (BM x BN, ring depth) by code — DBA_G3_SMALL_TILE / DBA_G3_BIG_TILE pick one for
// the small / large launch classes (sweeps: scripts/gpu/g3_tiles.sh)
int launch3_tile(int code, const G3Args& a, int G, hipStream_t st) {
  switch (code) {
    case 1: return launch3<64, 64, 4, uint16_t>(a, G, st);
    case 2: return launch3<64, 128, 3, uint16_t>(a, G, st);
    case 3: return launch3<128, 64, 3, uint16_t>(a, G, st);
    case 4: return launch3<128, 128, 2, uint16_t>(a, G, st);
    case 5: return launch3<128, 128, 3, uint16_t>(a, G, st);
    case 6: return launch3<64, 64, 3, uint16_t>(a, G, st);
    default: return launch3<64, 128, 4, uint16_t>(a, G, st);
  }
}

int* g3_tiles() {
  static int t[2] = {env_int("DBA_G3_SMALL_TILE", 2), env_int("DBA_G3_BIG_TILE", 4)};
  return t;
}

// split factor for a small launch: enough K-slices to put ~256 blocks on the chip, at least
// 4 k-steps per slice (1 = no split; DBA_G3_SPLITK=0 disables)
int g3_splitk(long long M, int G, int Cout, int K) {
  static const bool off = getenv("DBA_G3_SPLITK") && atoi(getenv("DBA_G3_SPLITK")) == 0;
  if (off) return 1;
  const long long blocks = (long long)ceil_div(M, 64) * ceil_div(Cout, 128) * G;
  if (blocks >= 192) return 1;
  const int nk = K / 64;
  int s = (int)std::min<long long>(8, (256 + blocks - 1) / blocks);
  while (s > 1 && nk / s < 4) --s;
  return s;
}

}  // namespace

// Select the tile codes of the small / large launch classes (launch3_tile); -1 keeps one.
// Returns the previous pair packed as small * 16 + big.
DBA_EXPORT int dba_conv3_set_tiles(int small_tile, int big_tile) {
  int* t = g3_tiles();
  const int prev = t[0] * 16 + t[1];
  if (small_tile >= 0) t[0] = small_tile;
  if (big_tile >= 0) t[1] = big_tile;
  return prev;
}

// fp32 workspace (floats) dba_conv3_fwd needs for a split-K launch of this shape (0: none)
DBA_EXPORT long long dba_conv3_splitk_floats(int G, int N, int Ho, int Wo, int Cin, int Cout, int KH, int KW,
                                             int out_f32) {
  if (Cin % 64 != 0 || Cout % 8 != 0 || Cout < 128 || out_f32) return 0;
  const long long M = (long long)N * Ho * Wo;
  if (!g3_small(M, G, Cout)) return 0;
  const int s = g3_splitk(M, G, Cout, KH * KW * Cin);
  return s > 1 ? (long long)s * G * M * Cout : 0;
}

// Forward conv (or a stride-1 data gradient expressed as one, with tap-flipped transposed
// weights) for Cs % 64 == 0, Ncol % 8 == 0, Ncol >= 128.  Returns -100 otherwise (caller
// falls back to conv2.hip).
DBA_EXPORT int dba_conv3_fwd(const void* x, long long x_gstride, const void* w, long long w_sstride, const int* wsel,
                             const float* bias, long long b_sstride, const void* res, void* out, long long out_gstride,
                             int out_f32, const int* nvalid, const void* zeros, int G, int N, int H, int W, int Cin,
                             int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad, int relu, void* ws,
                             long long ws_floats, void* stream) {
  if (Cin % 64 != 0 || Cout % 8 != 0 || Cout < 128 || out_f32) return -100;
  const long long M = (long long)N * Ho * Wo;
  G3Args a{(const uint16_t*)x, x_gstride, (const uint16_t*)w, w_sstride, wsel, bias, b_sstride,
           (const uint16_t*)res, out, out_gstride, nvalid, (const uint16_t*)zeros,
           N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, relu, 1, 0};
  const int small_tile = g3_tiles()[0], big_tile = g3_tiles()[1];
  if (g3_small(M, G, Cout)) {
    // small launches (grouped training steps): the block count cannot cover the chip, so
    // per-block latency rules — 64-row M tiles with a 3-deep LDS ring (tile code 2, swept in
    // scripts/gpu/g3_tiles.sh: 64x128/3 187 ms vs 64x128/4 192-202 ms per bench round)
    static const bool small_off = getenv("DBA_G3_SMALL") && atoi(getenv("DBA_G3_SMALL")) == 0;
    if (small_off) return -100;
    const int s = g3_splitk(M, G, Cout, KH * KW * Cin);
    if (s > 1 && ws != nullptr && ws_floats >= (long long)s * G * M * Cout) {
      // a lone client's stage-4 conv is 32 blocks of 36 k-steps: split K over s slabs
      G3Args b = a;
      b.out = ws;
      b.out_gstride = M * Cout;
      b.out_zstride = (long long)G * M * Cout;
      b.bias = nullptr;
      b.res = nullptr;
      b.relu = 0;
      const int rc = launch3<64, 128, 4, float>(b, G, (hipStream_t)stream, s);
      if (rc != 0) return rc;
      const long long per = M * (Cout / 8);
      const dim3 grid((unsigned)std::max(1LL, std::min(2048LL, (per + 255) / 256)), G);
      hipLaunchKernelGGL(splitk_reduce_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const float*)ws, s,
                         b.out_zstride, b.out_gstride, nvalid, N, Ho * Wo, Cout, bias, b_sstride, wsel,
                         (const uint16_t*)res, out_gstride, relu, (uint16_t*)out);
      DBA_LAUNCH_CHECK();
    }
    return launch3_tile(small_tile, a, G, (hipStream_t)stream);
  }
  return launch3_tile(big_tile, a, G, (hipStream_t)stream);
}
