// fp32 family, weight-gradient pass: the implicit-GEMM weight gradient (both operands
// transposed to reduction-major while staging, fp32 slabs over output pixels), the batched
// slab reduction of a backward pass, the bias column sums; the narrow stages' 3x3 convs go to
// the patch-reuse kernel (xwgrad_halo.hip).
#include "common.hpp"
#include "bnfuse.hpp"
#include "xmfma.hpp"
#include "xwgrad_halo.hpp"
#include <algorithm>

namespace {

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

int& wgrad_halo_on() {
  static int on = 1;
  return on;
}

}  // namespace

DBA_EXPORT int dba_xwgrad_halo_set(int on) {
  const int prev = wgrad_halo_on();
  if (on >= 0) wgrad_halo_on() = on;
  return prev;
}

// whole-image halo conv (ximg_kernel) on / off (tests: A/B against the implicit GEMM); returns the previous

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
