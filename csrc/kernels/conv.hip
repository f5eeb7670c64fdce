// Implicit-GEMM convolution on CDNA4 matrix cores (gfx950), NHWC, bf16 in / fp32 accumulate.
//
// Replaces the reference's cuDNN conv/linear calls for every model:
//   * forward            y[m, co]  = sum_k  X~[m, k] * W[co, k]     (+bias, +residual, ReLU)
//   * data gradient      dx[m, ci] = sum_k dY~[m, k] * Wt[ci, k]    (Wt = W with Cin/Cout swapped)
//   * weight gradient    dW[co, j] = sum_m  dY[m, co] * X~[m, j]    (split-K over rows, fp32 atomics)
// where X~ / dY~ are the im2col gathers done on the fly while staging tiles into LDS
// (k = tap * C + c, tap = kh * KW + kw; linears are 1x1 convs on [N,1,1,F]).
//
// Grouped execution: blockIdx.z is the replica/job group; each group selects its weight
// slot through `wsel` (eval: many jobs share one folded model) and owns `nvalid[g]` valid
// samples — tiles past them exit immediately, so partial last batches and finished clients
// cost nothing.  Tiles are 2x2 waves of 16x16x32 bf16 MFMAs; LDS rows are padded to 80 B so
// the 16-B fragment reads of 16 consecutive rows hit 16 distinct bank slots.
#include "common.hpp"
#include <algorithm>

namespace {

constexpr int BK = 32;
constexpr int LDSP = 40;  // u16 per LDS row (32 + 8 pad)

struct IgemmArgs {
  const uint16_t* src; long long src_gstride;   // A source activations [G][N][Hs][Ws][Cs]
  const uint16_t* w; long long w_sstride;       // B operand [slots][Ncol][K] (K contiguous)
  const int* wsel;
  const float* bias; long long b_sstride;       // [slots][Ncol] fp32 or null
  const uint16_t* res; long long res_gstride;   // [G][M][Ncol] bf16 or null
  void* out; long long out_gstride;             // [G][M][Ncol]
  const int* nvalid;
  int N, Hs, Ws, Cs, Ho, Wo, Ncol, KH, KW, stride, pad, relu;
};

// MODE 0: forward conv gather (source = conv input), MODE 1: data-gradient gather (source = dY)
template <int MODE>
__device__ __forceinline__ bool src_pos(const IgemmArgs& a, int p, int q, int kh, int kw, int& hs, int& ws) {
  if (MODE == 0) {
    hs = p * a.stride - a.pad + kh;
    ws = q * a.stride - a.pad + kw;
    return (unsigned)hs < (unsigned)a.Hs && (unsigned)ws < (unsigned)a.Ws;
  } else {
    int th = p + a.pad - kh, tw = q + a.pad - kw;
    if (th < 0 || tw < 0) return false;
    if (a.stride != 1) {
      if ((th % a.stride) | (tw % a.stride)) return false;
      th /= a.stride;
      tw /= a.stride;
    }
    hs = th; ws = tw;
    return th < a.Hs && tw < a.Ws;
  }
}

template <int BM, int BN, int MODE, bool FAST, typename OutT>
__global__ __launch_bounds__(256) void igemm_kernel(IgemmArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t As[2][BM][LDSP];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][BN][LDSP];
  constexpr int MI = BM / 32, NJ = BN / 32, RA = BM / 64;
  const int g = blockIdx.z;
  const int HoWo = a.Ho * a.Wo;
  const int Mv = valid_rows(a.nvalid, g, a.N) * HoWo;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  if (m0 >= Mv) return;
  const int K = a.KH * a.KW * a.Cs;
  const int nk = (K + BK - 1) / BK;
  const uint16_t* __restrict__ src = a.src + (long long)g * a.src_gstride;
  const int slot = a.wsel ? a.wsel[g] : g;
  const uint16_t* __restrict__ Wp = a.w + (long long)slot * a.w_sstride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // ---- per-thread A rows (FAST path: each thread stages RA rows x one 16-B k segment)
  int rn[RA], rp[RA], rq[RA];
  bool rv[RA];
  const int aseg = tid & 3;
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    const int m = m0 + (tid >> 2) + 64 * i;
    rv[i] = m < Mv;
    const int mm = rv[i] ? m : 0;
    rn[i] = mm / HoWo;
    const int rem = mm - rn[i] * HoWo;
    rp[i] = rem / a.Wo;
    rq[i] = rem - rp[i] * a.Wo;
  }

  uint4 ra[RA];
  uint4 rb;
  uint16_t ga[BM * BK / 256], gb[(BN * BK + 255) / 256];

  auto load_tiles = [&](int kc) {
    if constexpr (FAST) {
      const int k0 = kc * BK;
      const int tap = k0 / a.Cs;
      const int c0 = k0 - tap * a.Cs + aseg * 8;
      const int kh = tap / a.KW, kw = tap - kh * a.KW;
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        int hs, ws;
        ra[i] = make_uint4(0, 0, 0, 0);
        if (rv[i] && src_pos<MODE>(a, rp[i], rq[i], kh, kw, hs, ws))
          ra[i] = *(const uint4*)(src + (((long long)rn[i] * a.Hs + hs) * a.Ws + ws) * a.Cs + c0);
      }
      if (tid < BN * 4) {
        const int n = n0 + (tid >> 2);
        rb = make_uint4(0, 0, 0, 0);
        if (n < a.Ncol) rb = *(const uint4*)(Wp + (long long)n * K + k0 + (tid & 3) * 8);
      }
    } else {
#pragma unroll
      for (int e = 0; e < BM * BK / 256; ++e) {
        const int idx = tid + 256 * e;
        const int r = idx >> 5, kk = idx & 31;
        const int m = m0 + r, k = kc * BK + kk;
        uint16_t v = 0;
        if (m < Mv && k < K) {
          const int n = m / HoWo, rem = m - n * HoWo, p = rem / a.Wo, q = rem - p * a.Wo;
          const int tap = k / a.Cs, c = k - tap * a.Cs, kh = tap / a.KW, kw = tap - kh * a.KW;
          int hs, ws;
          if (src_pos<MODE>(a, p, q, kh, kw, hs, ws))
            v = src[(((long long)n * a.Hs + hs) * a.Ws + ws) * a.Cs + c];
        }
        ga[e] = v;
      }
#pragma unroll
      for (int e = 0; e < (BN * BK + 255) / 256; ++e) {
        const int idx = tid + 256 * e;
        uint16_t v = 0;
        if (idx < BN * BK) {
          const int r = idx >> 5, kk = idx & 31;
          const int n = n0 + r, k = kc * BK + kk;
          if (n < a.Ncol && k < K) v = Wp[(long long)n * K + k];
        }
        gb[e] = v;
      }
    }
  };
  auto store_tiles = [&](int buf) {
    if constexpr (FAST) {
#pragma unroll
      for (int i = 0; i < RA; ++i) *(uint4*)&As[buf][(tid >> 2) + 64 * i][aseg * 8] = ra[i];
      if (tid < BN * 4) *(uint4*)&Bs[buf][tid >> 2][(tid & 3) * 8] = rb;
    } else {
#pragma unroll
      for (int e = 0; e < BM * BK / 256; ++e) {
        const int idx = tid + 256 * e;
        As[buf][idx >> 5][idx & 31] = ga[e];
      }
#pragma unroll
      for (int e = 0; e < (BN * BK + 255) / 256; ++e) {
        const int idx = tid + 256 * e;
        if (idx < BN * BK) Bs[buf][idx >> 5][idx & 31] = gb[e];
      }
    }
  };

  f32x4_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  int cur = 0;
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  for (int kc = 0; kc < nk; ++kc) {
    if (kc + 1 < nk) load_tiles(kc + 1);
    bf16x8_t af[MI], bfr[NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i) af[i] = *(const bf16x8_t*)&As[cur][wm * (BM / 2) + i * 16 + fr][fk];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bfr[j] = *(const bf16x8_t*)&Bs[cur][wn * (BN / 2) + j * 16 + fr][fk];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (kc + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ---- epilogue: bias, residual, ReLU, store
  OutT* out = (OutT*)a.out + (long long)g * a.out_gstride;
  const float* bias = a.bias ? a.bias + (long long)slot * a.b_sstride : nullptr;
  const uint16_t* res = a.res ? a.res + (long long)g * a.res_gstride : nullptr;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = n0 + wn * (BN / 2) + j * 16 + fr;
    if (n >= a.Ncol) continue;
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 16 + (lane >> 4) * 4 + r;
        if (m >= Mv) continue;
        float v = acc[i][j][r] + bv;
        const long long o = (long long)m * a.Ncol + n;
        if (res) v += bf2f(res[o]);
        if (a.relu) v = fmaxf(v, 0.f);
        out[o] = from_f<OutT>(v);
      }
    }
  }
}

// ------------------------------------------------------------------ weight gradient
struct WgradArgs {
  const uint16_t* dy; long long dy_gstride;   // [G][N][Ho][Wo][Cout]
  const uint16_t* x; long long x_gstride;     // [G][N][H][W][Cin]
  float* dw; long long dw_gstride;            // [G][Cout][KH][KW][Cin] fp32 (accumulated)
  const int* nvalid;
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, rows_per_split;
};

template <bool FAST>
__global__ __launch_bounds__(256) void wgrad_kernel(WgradArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t As[2][64][LDSP];   // [co][m]
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][64][LDSP];   // [j][m]
  const int g = blockIdx.z;
  const int HoWo = a.Ho * a.Wo;
  const int Mv = valid_rows(a.nvalid, g, a.N) * HoWo;
  const int mbeg = blockIdx.y * a.rows_per_split;
  if (mbeg >= Mv) return;
  const int mend = min(Mv, mbeg + a.rows_per_split);
  const int J = a.KH * a.KW * a.Cin;
  const int tiles_j = (J + 63) / 64;
  const int co0 = (blockIdx.x / tiles_j) * 64, j0 = (blockIdx.x % tiles_j) * 64;
  const uint16_t* __restrict__ dy = a.dy + (long long)g * a.dy_gstride;
  const uint16_t* __restrict__ x = a.x + (long long)g * a.x_gstride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int ml = tid >> 3, seg = tid & 7;   // staging: 32 rows x 8 segments of 8 channels

  // B column segment decode (fixed per thread)
  const int jj = j0 + seg * 8;
  const int tap = jj / a.Cin, ci = jj - tap * a.Cin;
  const int kh = tap / a.KW, kw = tap - kh * a.KW;

  uint16_t va[8], vb[8];
  auto load_tiles = [&](int mb) {
    const int m = mb + ml;
    const bool mv = m < mend;
    int n = 0, p = 0, q = 0;
    if (mv) { n = m / HoWo; const int rem = m - n * HoWo; p = rem / a.Wo; q = rem - p * a.Wo; }
    const int hi = p * a.stride - a.pad + kh, wi = q * a.stride - a.pad + kw;
    const bool xin = mv && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W && jj < J;
    if constexpr (FAST) {
      uint4 t = make_uint4(0, 0, 0, 0);
      if (mv && co0 + seg * 8 < a.Cout) t = *(const uint4*)(dy + (long long)m * a.Cout + co0 + seg * 8);
      const uint16_t* tp = (const uint16_t*)&t;
#pragma unroll
      for (int e = 0; e < 8; ++e) va[e] = tp[e];
      uint4 u = make_uint4(0, 0, 0, 0);
      if (xin) u = *(const uint4*)(x + (((long long)n * a.H + hi) * a.W + wi) * a.Cin + ci);
      const uint16_t* up = (const uint16_t*)&u;
#pragma unroll
      for (int e = 0; e < 8; ++e) vb[e] = up[e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int co = co0 + seg * 8 + e;
        va[e] = (mv && co < a.Cout) ? dy[(long long)m * a.Cout + co] : (uint16_t)0;
        const int j = jj + e;
        uint16_t v = 0;
        if (mv && j < J) {
          const int t2 = j / a.Cin, c2 = j - t2 * a.Cin, kh2 = t2 / a.KW, kw2 = t2 - kh2 * a.KW;
          const int h2 = p * a.stride - a.pad + kh2, w2 = q * a.stride - a.pad + kw2;
          if ((unsigned)h2 < (unsigned)a.H && (unsigned)w2 < (unsigned)a.W)
            v = x[(((long long)n * a.H + h2) * a.W + w2) * a.Cin + c2];
        }
        vb[e] = v;
      }
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      As[buf][seg * 8 + e][ml] = va[e];
      Bs[buf][seg * 8 + e][ml] = vb[e];
    }
  };

  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  load_tiles(mbeg);
  store_tiles(0);
  __syncthreads();
  int cur = 0;
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  for (int mb = mbeg; mb < mend; mb += BK) {
    const bool more = mb + BK < mend;
    if (more) load_tiles(mb + BK);
    bf16x8_t af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = *(const bf16x8_t*)&As[cur][wm * 32 + i * 16 + fr][fk];
#pragma unroll
    for (int j = 0; j < 2; ++j) bfr[j] = *(const bf16x8_t*)&Bs[cur][wn * 32 + j * 16 + fr][fk];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (more) store_tiles(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  float* dw = a.dw + (long long)g * a.dw_gstride;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = j0 + wn * 32 + j * 16 + fr;
    if (col >= J) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (co < a.Cout) atomicAdd(dw + (long long)co * J + col, acc[i][j][r]);
      }
  }
}

// dW^T for the data gradient: [slots][Co][T][Ci] -> [slots][Ci][T][Co]; with `flip` the taps
// are also reversed (t -> T-1-t), turning a stride-1 dgrad into a forward conv (halo kernel).
// One block row per slot, 32-bit indexing; output-ordered (coalesced writes).
__global__ void transpose_w_kernel(const uint16_t* __restrict__ w, long long w_sstride, uint16_t* __restrict__ wt,
                                   int Co, int T, int Ci, int flip) {
  const int s = blockIdx.y;
  const int per = Co * T * Ci;
  const uint16_t* ws = w + (long long)s * w_sstride;
  uint16_t* wo = wt + (long long)s * per;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < per; i += gridDim.x * blockDim.x) {
    const int co = i % Co;
    const int r = i / Co;
    const int t = r % T;
    const int ci = r / T;
    const int ts = flip ? T - 1 - t : t;
    wo[i] = ws[(co * T + ts) * Ci + ci];
  }
}

// bias gradient: db[g][c] += sum over valid rows of dy[g][m][c].  Blocks own runs of
// `rpb` rows; for C <= 256 a block's 256 threads are (256 / C) row lanes x C channels, for
// wider layers they walk 256-channel chunks row by row (coalesced).  Each block adds its
// per-channel sums with one float atomic per channel (MnistNet conv1: 36,864 rows x 20
// channels per replica — a single column-walking thread per channel took ~4 ms).
__global__ __launch_bounds__(256) void colsum_kernel(const uint16_t* __restrict__ dy, long long dy_gstride,
                                                     int rows_per_sample, const int* nvalid, int N, int C,
                                                     float* __restrict__ db, long long db_gstride, int rpb) {
  __shared__ float red[256];
  const int g = blockIdx.y, tid = threadIdx.x;
  const int rows = valid_rows(nvalid, g, N) * rows_per_sample;
  const int r0 = blockIdx.x * rpb;
  if (r0 >= rows) return;
  const int r1 = min(rows, r0 + rpb);
  const uint16_t* __restrict__ p = dy + (long long)g * dy_gstride;
  float* __restrict__ d = db + (long long)g * db_gstride;
  if (C <= 256) {
    const int lanes = 256 / C, rr = tid / C, c = tid - rr * C;
    float s = 0.f;
    if (rr < lanes)
      for (int r = r0 + rr; r < r1; r += lanes) s += bf2f(p[(long long)r * C + c]);
    red[tid] = s;
    __syncthreads();
    if (tid < C) {
      float t = 0.f;
      for (int k = 0; k < lanes; ++k) t += red[k * C + tid];
      atomicAdd(d + tid, t);
    }
    return;
  }
  for (int c = tid; c < C; c += 256) {
    float s = 0.f;
    for (int r = r0; r < r1; ++r) s += bf2f(p[(long long)r * C + c]);
    atomicAdd(d + c, s);
  }
}

template <int BM, int BN, int MODE, bool FAST, typename OutT>
int launch_igemm(const IgemmArgs& a, int G, hipStream_t st) {
  const int M = a.N * a.Ho * a.Wo;
  dim3 grid(ceil_div(M, BM), ceil_div(a.Ncol, BN), G);
  hipLaunchKernelGGL((igemm_kernel<BM, BN, MODE, FAST, OutT>), grid, dim3(256), 0, st, a);
  DBA_LAUNCH_CHECK();
}

template <int MODE, typename OutT>
int dispatch_igemm(const IgemmArgs& a, int G, hipStream_t st) {
  const bool fast = (a.Cs % 32) == 0;
  const int M = a.N * a.Ho * a.Wo;
  const bool small_n = a.Ncol <= 32;
  const bool small_m = (long long)M * G < 256LL * 128 * 2;   // too few 128-row tiles to fill the chip
  if (fast) {
    if (small_n) return small_m ? launch_igemm<64, 32, MODE, true, OutT>(a, G, st) : launch_igemm<128, 32, MODE, true, OutT>(a, G, st);
    return small_m ? launch_igemm<64, 64, MODE, true, OutT>(a, G, st) : launch_igemm<128, 64, MODE, true, OutT>(a, G, st);
  }
  if (small_n) return launch_igemm<64, 32, MODE, false, OutT>(a, G, st);
  return launch_igemm<64, 64, MODE, false, OutT>(a, G, st);
}

}  // namespace

DBA_EXPORT int dba_conv_fwd(const void* x, long long x_gstride, const void* w, long long w_sstride, const int* wsel,
                            const float* bias, long long b_sstride, const void* res, long long res_gstride,
                            void* out, long long out_gstride, int out_f32, const int* nvalid, int G, int N, int H,
                            int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad, int relu,
                            void* stream) {
  IgemmArgs a{(const uint16_t*)x, x_gstride, (const uint16_t*)w, w_sstride, wsel, bias, b_sstride,
              (const uint16_t*)res, res_gstride, out, out_gstride, nvalid, N, H, W, Cin, Ho, Wo, Cout, KH, KW,
              stride, pad, relu};
  hipStream_t st = (hipStream_t)stream;
  return out_f32 ? dispatch_igemm<0, float>(a, G, st) : dispatch_igemm<0, uint16_t>(a, G, st);
}

// wt: transposed weights [slots][Cin][KH][KW][Cout]; dx: [G][N][H][W][Cin]
DBA_EXPORT int dba_conv_dgrad(const void* dy, long long dy_gstride, const void* wt, long long wt_sstride,
                              const int* wsel, void* dx, long long dx_gstride, const int* nvalid, int G, int N, int H,
                              int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad,
                              void* stream) {
  // source = dY [N][Ho][Wo][Cout], output rows = input pixels [N][H][W], output channels = Cin
  IgemmArgs a{(const uint16_t*)dy, dy_gstride, (const uint16_t*)wt, wt_sstride, wsel, nullptr, 0, nullptr, 0, dx,
              dx_gstride, nvalid, N, Ho, Wo, Cout, H, W, Cin, KH, KW, stride, pad, 0};
  return dispatch_igemm<1, uint16_t>(a, G, (hipStream_t)stream);
}

DBA_EXPORT int dba_conv_wgrad(const void* dy, long long dy_gstride, const void* x, long long x_gstride, float* dw,
                              long long dw_gstride, const int* nvalid, int G, int N, int H, int W, int Cin, int Ho,
                              int Wo, int Cout, int KH, int KW, int stride, int pad, void* stream) {
  const int M = N * Ho * Wo;
  // split the row reduction so the launch has >= ~2048 blocks
  const int J = KH * KW * Cin;
  const long long tiles = (long long)ceil_div(Cout, 64) * ceil_div(J, 64) * G;
  int splits = (int)std::max(1LL, std::min((long long)ceil_div(M, BK), 2048 / std::max(1LL, tiles)));
  int rows = ceil_div(M, splits);
  rows = ceil_div(rows, BK) * BK;
  splits = ceil_div(M, rows);
  WgradArgs a{(const uint16_t*)dy, dy_gstride, (const uint16_t*)x, x_gstride, dw, dw_gstride, nvalid, N, H, W, Cin,
              Ho, Wo, Cout, KH, KW, stride, pad, rows};
  dim3 grid((unsigned)(ceil_div(Cout, 64) * ceil_div(J, 64)), splits, G);
  const bool fast = (Cin % 8 == 0) && (Cout % 8 == 0);
  if (fast) hipLaunchKernelGGL(wgrad_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(wgrad_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, a);
  DBA_LAUNCH_CHECK();
}

// w[s][co][t][ci] -> wt[s][ci][t'][co] through a 64x64 LDS tile: 16-byte loads along ci,
// 16-byte stores along co (the naive kernel above reads with a T*Ci stride).  Slots whose
// replica is inactive this step (nvalid[s] == 0, slot == replica) are skipped.
__global__ __launch_bounds__(256) void transpose_w_tiled_kernel(const uint16_t* __restrict__ w, long long w_sstride,
                                                                uint16_t* __restrict__ wt, int Co, int T, int Ci,
                                                                int flip, const int* __restrict__ nvalid) {
  __shared__ uint16_t tile[64][64 + 2];
  const int s = blockIdx.z;
  if (nvalid && nvalid[s] == 0) return;
  const int t = blockIdx.y;
  const int tci = (Ci + 63) / 64;
  const int co0 = (blockIdx.x / tci) * 64, ci0 = (blockIdx.x % tci) * 64;
  const uint16_t* ws = w + (long long)s * w_sstride;
  uint16_t* wo = wt + (long long)s * Co * T * Ci;
  const int tid = threadIdx.x;
  const int ts = flip ? T - 1 - t : t;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + 256 * i;               // 64 rows x 8 chunks
    const int r = e >> 3, c8 = (e & 7) * 8;
    const int co = co0 + r, ci = ci0 + c8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (co < Co && ci < Ci) v = *(const uint4*)(ws + ((long long)co * T + ts) * Ci + ci);
    const uint16_t* pv = (const uint16_t*)&v;
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[r][c8 + j] = pv[j];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + 256 * i;
    const int r = e >> 3, c8 = (e & 7) * 8;    // r: ci within tile, c8: co chunk
    const int ci = ci0 + r, co = co0 + c8;
    if (ci >= Ci || co >= Co) continue;
    uint4 v;
    uint16_t* pv = (uint16_t*)&v;
#pragma unroll
    for (int j = 0; j < 8; ++j) pv[j] = tile[c8 + j][r];
    *(uint4*)(wo + ((long long)ci * T + t) * Co + co) = v;
  }
}

// ---------------------------------------------------------------- batched transposes
// Every data-gradient weight transpose of a training step in ONE launch (the step's weights
// are fixed from the forward to the SGD update, so all of them can be produced up front):
// one LDS-tiled 64x64 block per (layer, tap, tile), descriptors passed by value.  A lone
// attacker's latency-bound step otherwise pays a dependent launch per layer.
namespace {
constexpr int kMaxTDesc = 32;
struct TDesc {
  const uint16_t* w;
  uint16_t* wt;
  long long ws;
  int Co, T, Ci, flip, tiles, tile0;
};
struct TBatch {
  TDesc d[kMaxTDesc];
  int n;
  const int* nvalid;
};

__global__ __launch_bounds__(256) void transpose_w_batch_kernel(const TBatch b) {
  __shared__ uint16_t tile[64][64 + 2];
  const int s = blockIdx.y;
  if (b.nvalid && b.nvalid[s] == 0) return;
  int k = 0;
  while (k + 1 < b.n && (int)blockIdx.x >= b.d[k + 1].tile0) ++k;
  const TDesc& d = b.d[k];
  const int Co = d.Co, T = d.T, Ci = d.Ci;
  const int local = blockIdx.x - d.tile0;
  const int tci = (Ci + 63) / 64, tco = (Co + 63) / 64;
  const int t = local / (tci * tco);
  const int rem = local - t * tci * tco;
  const int co0 = (rem / tci) * 64, ci0 = (rem % tci) * 64;
  const uint16_t* ws = d.w + (long long)s * d.ws;
  uint16_t* wo = d.wt + (long long)s * Co * T * Ci;
  const int tid = threadIdx.x;
  const int ts = d.flip ? T - 1 - t : t;
  const bool vec = (Ci % 8 == 0) && (Co % 8 == 0);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + 256 * i;
    const int r = e >> 3, c8 = (e & 7) * 8;
    const int co = co0 + r, ci = ci0 + c8;
    if (vec) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (co < Co && ci < Ci) v = *(const uint4*)(ws + ((long long)co * T + ts) * Ci + ci);
      const uint16_t* pv = (const uint16_t*)&v;
#pragma unroll
      for (int j = 0; j < 8; ++j) tile[r][c8 + j] = pv[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        tile[r][c8 + j] = (co < Co && ci + j < Ci) ? ws[((long long)co * T + ts) * Ci + ci + j] : (uint16_t)0;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + 256 * i;
    const int r = e >> 3, c8 = (e & 7) * 8;
    const int ci = ci0 + r, co = co0 + c8;
    if (ci >= Ci || co >= Co) continue;
    uint16_t* dst = wo + ((long long)ci * T + t) * Co + co;
    if (vec) {
      uint4 v;
      uint16_t* pv = (uint16_t*)&v;
#pragma unroll
      for (int j = 0; j < 8; ++j) pv[j] = tile[c8 + j][r];
      *(uint4*)dst = v;
    } else {
      for (int j = 0; j < 8 && co + j < Co; ++j) dst[j] = tile[c8 + j][r];
    }
  }
}

}  // namespace

// n descriptors of 9 words each: {w, wt, ws, Co, T, Ci, flip, (unused), (unused)} as int64
DBA_EXPORT int dba_transpose_w_batch(const long long* desc, int n, int slots, const int* nvalid, void* stream) {
  if (n <= 0) return 0;
  if (n > kMaxTDesc) return -101;
  TBatch b;
  int tiles = 0;
  for (int k = 0; k < n; ++k) {
    const long long* q = desc + 9 * k;
    TDesc& d = b.d[k];
    d.w = (const uint16_t*)q[0];
    d.wt = (uint16_t*)q[1];
    d.ws = q[2];
    d.Co = (int)q[3];
    d.T = (int)q[4];
    d.Ci = (int)q[5];
    d.flip = (int)q[6];
    d.tiles = ceil_div(d.Co, 64) * ceil_div(d.Ci, 64) * d.T;
    d.tile0 = tiles;
    tiles += d.tiles;
  }
  b.n = n;
  b.nvalid = nvalid;
  hipLaunchKernelGGL(transpose_w_batch_kernel, dim3(tiles, slots), dim3(256), 0, (hipStream_t)stream, b);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_transpose_w(const void* w, long long w_sstride, void* wt, int slots, int Co, int T, int Ci,
                               int flip, const int* nvalid, void* stream) {
  if (Co % 8 == 0 && Ci % 8 == 0) {
    dim3 grid(ceil_div(Co, 64) * ceil_div(Ci, 64), T, slots);
    hipLaunchKernelGGL(transpose_w_tiled_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const uint16_t*)w,
                       w_sstride, (uint16_t*)wt, Co, T, Ci, flip, nvalid);
    DBA_LAUNCH_CHECK();
  }
  const int per = Co * T * Ci;
  const int bx = std::max(1, std::min(256, (per + 255) / 256));
  hipLaunchKernelGGL(transpose_w_kernel, dim3(bx, slots), dim3(256), 0, (hipStream_t)stream, (const uint16_t*)w,
                     w_sstride, (uint16_t*)wt, Co, T, Ci, flip);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_colsum(const void* dy, long long dy_gstride, int rows_per_sample, const int* nvalid, int G, int N,
                          int C, float* db, long long db_gstride, void* stream) {
  const long long rows = (long long)N * rows_per_sample;
  const int rpb = C <= 256 ? 256 : 64;
  dim3 grid(std::max(1, ceil_div(rows, rpb)), G);
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const uint16_t*)dy, dy_gstride,
                     rows_per_sample, nvalid, N, C, db, db_gstride, rpb);
  DBA_LAUNCH_CHECK();
}
