// Implicit-GEMM convolution, generation 2 (gfx950): the hot path for every conv / linear
// whose source channel count is a multiple of 8 (all ResNet-18 layers, both passes).
//
// vs conv.hip (kept for odd channel counts):
//   * v_mfma_f32_32x32x16_bf16 (half the LDS operand traffic per FLOP of 16x16x32);
//   * BK = 64 per barrier, double-buffered LDS with register-staged prefetch: the global
//     gathers of step k+1 are in flight while step k's MFMAs run;
//   * LDS rows padded to 144 B: the 32 lanes of a fragment read hit 32 distinct bank slots
//     (row*36 dwords mod 64 is a bijection over 16 consecutive rows);
//   * the output tile is staged through LDS in fp32 and written back in 16-byte bf16 chunks
//     (bias / residual / ReLU applied in that pass) instead of 2-byte scattered stores;
//   * linearised block index with the N-tile fastest, so blocks sharing an A (activation)
//     row panel are dispatched back to back.
// Source segments of 8 channels never straddle a tap (Cs % 8 == 0), so every A load is one
// aligned 16-B vector load whatever the tap geometry (stem 7x7/s2, 3x3, 1x1 shortcut, linear).
#include "common.hpp"
#include <algorithm>

namespace {

constexpr int BK2 = 64;
typedef short v4i16_t __attribute__((ext_vector_type(4)));
constexpr int LP = BK2 + 8;   // u16 per LDS row (144 B)

struct Igemm2Args {
  const uint16_t* src; long long src_gstride;   // [G][N][Hs][Ws][Cs]
  const uint16_t* w; long long w_sstride;       // [slots][Ncol][K]
  const int* wsel;
  const float* bias; long long b_sstride;
  const uint16_t* res;                          // [G][M][Ncol] (same layout as out)
  void* out; long long out_gstride;             // [G][M][Ncol]
  const int* nvalid;
  int N, Hs, Ws, Cs, Ho, Wo, Ncol, KH, KW, stride, pad, relu;
  int tiles_n;
};

template <int MODE>
__device__ __forceinline__ bool src_pos2(const Igemm2Args& a, int p, int q, int kh, int kw, int& hs, int& ws) {
  if constexpr (MODE == 0) {
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

// BT: the B operand is read straight from the FORWARD weight tensor [Co][T][Ci] in its
// natural K-major order (k = tap*Co + co rows, Ci columns; tap-flipped when MODE == 0, i.e.
// a stride-1 data gradient run as a forward conv) and consumed with ds_read_b64_tr_b16
// transposed reads — no separate weight-transpose pass.  B LDS rows are padded by 64 B so
// the 4 rows of a transposed read hit distinct banks.
template <int BM, int BN, int WM, int WN, int MODE, typename OutT, bool BT = false>
__global__ __launch_bounds__(256) void igemm2_kernel(Igemm2Args a) {
  constexpr int TM = BM / WM, TN = BN / WN;          // wave tile
  constexpr int MI = TM / 32, NJ = TN / 32;          // 32x32 MFMA tiles per wave
  constexpr int RA = BM * 8 / 256;                   // A 16-B loads per thread per k-step
  constexpr int RB = (BN * 8 + 255) / 256;           // B 16-B loads per thread
  // BT: u16 per B row (k-major), padded so the row pitch is 16 dwords mod 64: the 4 rows of a
  // transposed read (64 B of columns each per 32-lane half) land on distinct banks
  constexpr int LPT = BN + 2 * ((16 - BN / 2) & 63);
  static_assert(WM * WN == 4, "4 waves");
  static_assert(MI >= 1 && NJ >= 1, "wave tile >= 32x32");
  constexpr int LDS_B = BT ? BK2 * LPT : BN * LP;    // u16 per B buffer
  constexpr int LDS_AB = 2 * (BM * LP + LDS_B);      // u16
  constexpr int LDS_C = BM * BN * 2;                  // u16 (fp32 staging)
  __shared__ __attribute__((aligned(16))) uint16_t smem[LDS_AB > LDS_C ? LDS_AB : LDS_C];
  uint16_t (*As)[BM][LP] = reinterpret_cast<uint16_t (*)[BM][LP]>(smem);
  uint16_t (*Bs)[BN][LP] = reinterpret_cast<uint16_t (*)[BN][LP]>(smem + 2 * BM * LP);
  uint16_t (*Bt)[BK2][LPT] = reinterpret_cast<uint16_t (*)[BK2][LPT]>(smem + 2 * BM * LP);

  const int g = blockIdx.y;
  const int HoWo = a.Ho * a.Wo;
  // MODE 2 (stride-2 data gradient): output rows are grouped by pixel-parity class
  // (py, px); every row of a block shares it, so whole k-steps whose tap parity cannot
  // reach the class are skipped (3/4 of a 3x3 stride-2 scatter GEMM is structurally zero).
  const int HoWo2 = MODE == 2 ? HoWo / 4 : HoWo;
  const int Mv = valid_rows(a.nvalid, g, a.N) * HoWo2;
  const int tn = blockIdx.x % a.tiles_n;
  int tm = blockIdx.x / a.tiles_n, cls = 0;
  if constexpr (MODE == 2) {
    const int tpc = (a.N * HoWo2 + BM - 1) / BM;   // row tiles per class
    cls = tm / tpc;
    tm -= cls * tpc;
  }
  const int py = cls >> 1, px = cls & 1;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mv) return;
  const int K = a.KH * a.KW * a.Cs;
  const int cpt = a.Cs / BK2;                      // MODE 2: k-steps per tap (Cs % 64 == 0)
  const int kh0 = (py + a.pad) & 1, kw0 = (px + a.pad) & 1;
  const int nvw = MODE == 2 ? (a.KW - kw0 + 1) / 2 : 1;
  const int nvh = MODE == 2 ? (a.KH - kh0 + 1) / 2 : 1;
  const int nk = MODE == 2 ? nvh * nvw * cpt : (K + BK2 - 1) / BK2;
  auto kc_of = [&](int j) -> int {
    if constexpr (MODE != 2) return j;
    const int chunk = j % cpt, t = j / cpt;
    const int ih = t / nvw, iw = t - ih * nvw;
    return ((kh0 + 2 * ih) * a.KW + kw0 + 2 * iw) * cpt + chunk;
  };
  const uint16_t* __restrict__ src = a.src + (long long)g * a.src_gstride;
  const int slot = a.wsel ? a.wsel[g] : g;
  const uint16_t* __restrict__ Wp = a.w + (long long)slot * a.w_sstride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  // staging geometry: A load i covers row (tid>>3) + 32*i, segment tid&7 (8 channels)
  const int seg = tid & 7;
  int rbase[RA], rp[RA], rq[RA];
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    if (m < Mv) {
      const int n = m / HoWo2, rem = m - n * HoWo2;
      if constexpr (MODE == 2) {
        const int w2 = a.Wo >> 1;
        rp[i] = 2 * (rem / w2) + py;
        rq[i] = 2 * (rem - (rem / w2) * w2) + px;
      } else {
        rp[i] = rem / a.Wo;
        rq[i] = rem - rp[i] * a.Wo;
      }
      rbase[i] = n;
    } else {
      rbase[i] = -1; rp[i] = 0; rq[i] = 0;
    }
  }
  uint4 ra[RA], rb[RB];

  auto load_tiles = [&](int kc) {
    const int k = kc * BK2 + seg * 8;
    const bool kin = k < K;
    const int tap = k / a.Cs;
    const int c = k - tap * a.Cs;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      int hs, ws;
      ra[i] = make_uint4(0, 0, 0, 0);
      if (kin && rbase[i] >= 0 && src_pos2<MODE>(a, rp[i], rq[i], kh, kw, hs, ws))
        ra[i] = *(const uint4*)(src + (((long long)rbase[i] * a.Hs + hs) * a.Ws + ws) * a.Cs + c);
    }
    if constexpr (!BT) {
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const int r = (tid >> 3) + 32 * i;
        rb[i] = make_uint4(0, 0, 0, 0);
        if (r < BN && kin && n0 + r < a.Ncol) rb[i] = *(const uint4*)(Wp + (long long)(n0 + r) * K + k);
      }
    } else {
      // B^T tile [BK2 rows k][BN cols n], 16-B chunks along n: k -> (tap, co) of the source
      // channel axis; element = W[co][tap'][n] with tap' = T-1-tap for the flipped (MODE 0) form
      constexpr int CPR = BN / 8;                    // chunks per B row
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const int e = tid + 256 * i;
        const int kr = e / CPR, cn = (e - kr * CPR) * 8;
        const int kg = kc * BK2 + kr;
        rb[i] = make_uint4(0, 0, 0, 0);
        if (kr < BK2 && kg < K && n0 + cn < a.Ncol) {
          const int T = a.KH * a.KW;
          int tap, co;
          if (a.Cs % BK2 == 0) {          // one tap per k-step: hoistable, no per-row division
            tap = (kc * BK2) / a.Cs;
            co = kc * BK2 - tap * a.Cs + kr;
          } else {
            tap = kg / a.Cs;
            co = kg - tap * a.Cs;
          }
          const int tsrc = MODE == 0 ? T - 1 - tap : tap;
          rb[i] = *(const uint4*)(Wp + ((long long)co * T + tsrc) * a.Ncol + n0 + cn);
        }
      }
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < RA; ++i) *(uint4*)&As[buf][(tid >> 3) + 32 * i][seg * 8] = ra[i];
    if constexpr (!BT) {
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const int r = (tid >> 3) + 32 * i;
        if (r < BN) *(uint4*)&Bs[buf][r][seg * 8] = rb[i];
      }
    } else {
      constexpr int CPR = BN / 8;
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const int e = tid + 256 * i;
        const int kr = e / CPR, cn = (e - kr * CPR) * 8;
        if (kr < BK2) *(uint4*)&Bt[buf][kr][cn] = rb[i];
      }
    }
  };

  f32x16_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    load_tiles(kc_of(0));
    store_tiles(0);
  }
  __syncthreads();
  const int fr = lane & 31, fk = (lane >> 5) * 8;
  int cur = 0;
  for (int kc = 0; kc < nk; ++kc) {
    if (kc + 1 < nk) load_tiles(kc_of(kc + 1));
#pragma unroll
    for (int kk = 0; kk < BK2; kk += 16) {
      bf16x8_t af[MI], bfr[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = *(const bf16x8_t*)&As[cur][wm * TM + i * 32 + fr][kk + fk];
      if constexpr (!BT) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[j] = *(const bf16x8_t*)&Bs[cur][wn * TN + j * 32 + fr][kk + fk];
      } else {
        // transposed read (T10): lane 4q+p of 16-lane group G4 addresses row k = kk+8h+4t+q,
        // columns 16*(G4&1)+4p..+3; lane i of the group receives column i, rows in elements
        const int G4 = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          union { bf16x8_t v; v4i16_t h[2]; } u;
#pragma unroll
          for (int t2 = 0; t2 < 2; ++t2)
            u.h[t2] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16_t*)
                &Bt[cur][kk + 8 * (G4 >> 1) + 4 * t2 + q][wn * TN + j * 32 + 16 * (G4 & 1) + 4 * p4]);
          bfr[j] = u.v;
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kc + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ---- epilogue: stage fp32 tile in LDS, then 8-wide vector pass with bias/res/ReLU
  float* Cst = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = wn * TN + j * 32 + fr;
        Cst[row * BN + col] = acc[i][j][r];
      }
  __syncthreads();
  OutT* out = (OutT*)a.out + (long long)g * a.out_gstride;
  const float* bias = a.bias ? a.bias + (long long)slot * a.b_sstride : nullptr;
  const uint16_t* res = a.res ? a.res + (long long)g * a.out_gstride : nullptr;
  constexpr int CH = BN / 8;                         // 8-col chunks per row
  const bool full_n = (n0 + BN <= a.Ncol) && (a.Ncol % 8 == 0);
  for (int e = tid; e < BM * CH; e += 256) {
    const int row = e / CH, c8 = (e - row * CH) * 8;
    const int mr = m0 + row;
    if (mr >= Mv) continue;
    int m = mr;
    if constexpr (MODE == 2) {   // class-local row -> pixel index
      const int w2 = a.Wo >> 1;
      const int nimg = mr / HoWo2, rem = mr - nimg * HoWo2;
      const int pp = 2 * (rem / w2) + py, qq = 2 * (rem - (rem / w2) * w2) + px;
      m = (nimg * a.Ho + pp) * a.Wo + qq;
    }
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = Cst[row * BN + c8 + t];
    const int n = n0 + c8;
    const long long o = (long long)m * a.Ncol + n;
    if (full_n) {
      if (bias) {
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] += bias[n + t];
      }
      if (res) {
        const uint4 rv = *(const uint4*)(res + o);
        const uint16_t* rp2 = (const uint16_t*)&rv;
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] += bf2f(rp2[t]);
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
    } else {
      for (int t = 0; t < 8 && n + t < a.Ncol; ++t) {
        float x = v[t] + (bias ? bias[n + t] : 0.f);
        if (res) x += bf2f(res[o + t]);
        if (a.relu) x = fmaxf(x, 0.f);
        out[o + t] = from_f<OutT>(x);
      }
    }
  }
}

// ------------------------------------------------------------- small-channel sources
// Stems / first layers with Cs < 8 (CIFAR 3x3x3, Tiny 7x7x3, MNIST 5x5x1): every thread
// gathers ONE output row's receptive field (k = tap*Cs + c, contiguous within a kernel row
// in NHWC) straight into its LDS row; K <= 160 is consumed in 32-wide MFMA k-steps.
// HALO: CIFAR-stem geometry (3x3, stride 1, pad 1, Cs 3, 256 % Wo == 0, 16-B aligned rows):
// the block's 256 output pixels are 256/Wo whole image rows, so the input rows they need are
// copied once into an LDS halo with 16-B loads and every receptive field is read from there.
template <typename OutT, int KMAX, bool HALO = false>
__global__ __launch_bounds__(256) void igemm_small_kernel(Igemm2Args a) {
  constexpr int BM = 256, BN = 32;
  constexpr int LPs = KMAX + 8;
  // operand tiles, then (aliased) the fp32 output tile of the staged epilogue: a 160-B row
  // stride keeps both the MFMA-layout writes and the row-per-thread 16-B reads conflict-free
  constexpr int CP = 40;
  constexpr int HALO_BYTES = HALO ? 4096 : 0;   // (256/Wo + 2) rows x (Wo + 2) px x 3 ch, Wo <= 64
  constexpr int AB_BYTES = (BM + BN) * LPs * 2 + HALO_BYTES, C_BYTES = BM * CP * 4;
  __shared__ __attribute__((aligned(16))) uint8_t smem[AB_BYTES > C_BYTES ? AB_BYTES : C_BYTES];
  uint16_t(*As)[LPs] = (uint16_t(*)[LPs])smem;
  uint16_t(*Bs)[LPs] = (uint16_t(*)[LPs])(smem + BM * LPs * 2);
  float(*Cst)[CP] = (float(*)[CP])smem;
  const int g = blockIdx.y;
  const int HoWo = a.Ho * a.Wo;
  const int Mv = valid_rows(a.nvalid, g, a.N) * HoWo;
  const int tn = blockIdx.x % a.tiles_n, tm = blockIdx.x / a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mv) return;
  const int K = a.KH * a.KW * a.Cs;
  const int Kp = (K + 31) & ~31;
  const uint16_t* __restrict__ src = a.src + (long long)g * a.src_gstride;
  const int slot = a.wsel ? a.wsel[g] : g;
  const uint16_t* __restrict__ Wp = a.w + (long long)slot * a.w_sstride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if constexpr (HALO) {
    constexpr int HC = 3;                       // channels
    const int R = BM / a.Wo;                    // output rows per block
    const int RW = (a.Ws + 2) * HC;             // halo row: one zero pixel each side
    uint16_t* halo = (uint16_t*)(smem + (BM + BN) * LPs * 2);
    const int n = m0 / HoWo, p0 = (m0 - n * HoWo) / a.Wo;
    const uint16_t* __restrict__ img = src + (long long)n * a.Hs * a.Ws * HC;
    for (int e = tid; e < (R + 2) * RW; e += 256) halo[e] = 0;
    __syncthreads();
    const int vpr = a.Ws * HC / 8;              // 16-B vectors per input row
    for (int e = tid; e < (R + 2) * vpr; e += 256) {
      const int hr = e / vpr, v = e - hr * vpr, hs = p0 - 1 + hr;
      if ((unsigned)hs < (unsigned)a.Hs) {
        const uint4 d = *(const uint4*)(img + (long long)hs * a.Ws * HC + v * 8);
        const uint16_t* dp = (const uint16_t*)&d;
#pragma unroll
        for (int t = 0; t < 8; ++t) halo[hr * RW + HC + v * 8 + t] = dp[t];
      }
    }
    __syncthreads();
    const int pr = tid / a.Wo, q = tid - pr * a.Wo;
    const bool live = m0 + tid < Mv;
    uint16_t vals[32];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int j = 0; j < 9; ++j) vals[kh * 9 + j] = live ? halo[(pr + kh) * RW + q * HC + j] : (uint16_t)0;
#pragma unroll
    for (int k = 27; k < 32; ++k) vals[k] = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint4 pk;
      uint16_t* pp = (uint16_t*)&pk;
#pragma unroll
      for (int t = 0; t < 8; ++t) pp[t] = vals[j * 8 + t];
      *(uint4*)&As[tid][j * 8] = pk;
    }
  } else if constexpr (KMAX == 32) {
    // A (K <= 32: CIFAR 3x3x3, MNIST 5x5x1): the row's whole receptive field is loaded into
    // registers first — unrolled, branch-free clamped loads, so all of them are in flight at
    // once instead of one global-load latency per tap — then written as four 16-B LDS stores
    const int m = m0 + tid;
    const int mm = m < Mv ? m : Mv - 1;
    const int n = mm / HoWo, rem = mm - n * HoWo, p = rem / a.Wo, q = rem - p * a.Wo;
    const int hs0 = p * a.stride - a.pad, ws0 = q * a.stride - a.pad;
    const uint16_t* __restrict__ img = src + (long long)n * a.Hs * a.Ws * a.Cs;
    uint16_t vals[32];
    int kh = 0, kw = 0, c = 0;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const int hs = hs0 + kh, ws = ws0 + kw;
      const bool in = k < K && m < Mv && (unsigned)hs < (unsigned)a.Hs && (unsigned)ws < (unsigned)a.Ws;
      const int hc = min(max(hs, 0), a.Hs - 1), wc = min(max(ws, 0), a.Ws - 1);
      const uint16_t t = img[(hc * a.Ws + wc) * a.Cs + min(c, a.Cs - 1)];
      vals[k] = in ? t : (uint16_t)0;
      if (++c == a.Cs) {
        c = 0;
        if (++kw == a.KW) { kw = 0; ++kh; }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint4 pk;
      uint16_t* pp = (uint16_t*)&pk;
#pragma unroll
      for (int t = 0; t < 8; ++t) pp[t] = vals[j * 8 + t];
      *(uint4*)&As[tid][j * 8] = pk;
    }
  } else {  // A: one row per thread
    const int m = m0 + tid;
    uint16_t* dst = As[tid];
    if (m < Mv) {
      const int n = m / HoWo, rem = m - n * HoWo, p = rem / a.Wo, q = rem - p * a.Wo;
      int k = 0;
      for (int kh = 0; kh < a.KH; ++kh) {
        const int hs = p * a.stride - a.pad + kh;
        const bool hin = (unsigned)hs < (unsigned)a.Hs;
        for (int kw = 0; kw < a.KW; ++kw) {
          const int ws = q * a.stride - a.pad + kw;
          const bool in = hin && (unsigned)ws < (unsigned)a.Ws;
          const uint16_t* s = src + (((long long)n * a.Hs + hs) * a.Ws + ws) * a.Cs;
          for (int c = 0; c < a.Cs; ++c) dst[k++] = in ? s[c] : (uint16_t)0;
        }
      }
      for (; k < Kp; ++k) dst[k] = 0;
    } else {
      for (int k = 0; k < Kp; ++k) dst[k] = 0;
    }
  }
  for (int e = tid; e < BN * Kp; e += 256) {   // B: [BN][Kp], zero-padded
    const int r = e / Kp, k = e - r * Kp;
    Bs[r][k] = (k < K && n0 + r < a.Ncol) ? Wp[(long long)(n0 + r) * K + k] : (uint16_t)0;
  }
  __syncthreads();
  // 4 waves x (64 rows x 32 cols): 2 MFMA 32x32 tiles per wave
  f32x16_t acc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  const int fr = lane & 31, fk = (lane >> 5) * 8;
  for (int kk = 0; kk < Kp; kk += 16) {
    const bf16x8_t b = *(const bf16x8_t*)&Bs[fr][kk + fk];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bf16x8_t av = *(const bf16x8_t*)&As[wid * 64 + i * 32 + fr][kk + fk];
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, b, acc[i], 0, 0, 0);
    }
  }
  OutT* out = (OutT*)a.out + (long long)g * a.out_gstride;
  const float* bias = a.bias ? a.bias + (long long)slot * a.b_sstride : nullptr;
  const uint16_t* res = a.res ? a.res + (long long)g * a.out_gstride : nullptr;
  const int n = n0 + fr;
  if constexpr (sizeof(OutT) == 2) {
    if (a.Ncol % 8 == 0) {
      // staged epilogue: acc (+bias) -> LDS fp32 tile -> each thread owns one output row and
      // writes its up-to-32 channels as 16-B stores (the MFMA layout would give 2-B stores)
      __syncthreads();   // every wave is done reading As / Bs
      const float bv = (bias && n < a.Ncol) ? bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          Cst[wid * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)][fr] = acc[i][r] + bv;
      __syncthreads();
      // lane -> (row, 8-channel chunk) with the chunk fastest: a wave stores 16 rows x 64 B
      // contiguous per instruction when Ncol == 32
#pragma unroll
      for (int it = 0; it < BM * (BN / 8) / 256; ++it) {
        const int idx = it * 256 + tid, row = idx / (BN / 8), c = idx % (BN / 8);
        const int m = m0 + row;
        if (m >= Mv || n0 + c * 8 + 8 > a.Ncol) continue;
        const long long o = (long long)m * a.Ncol + n0 + c * 8;
        const float4 lo = *(const float4*)&Cst[row][c * 8], hi = *(const float4*)&Cst[row][c * 8 + 4];
        float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        if (res) {
          const uint4 rv = *(const uint4*)(res + o);
          const uint16_t* rp = (const uint16_t*)&rv;
#pragma unroll
          for (int t = 0; t < 8; ++t) v[t] += bf2f(rp[t]);
        }
        uint4 pk;
        uint16_t* pp = (uint16_t*)&pk;
#pragma unroll
        for (int t = 0; t < 8; ++t) pp[t] = f2bf(a.relu ? fmaxf(v[t], 0.f) : v[t]);
        *(uint4*)((uint16_t*)out + o) = pk;
      }
      return;
    }
  }
  if (n >= a.Ncol) return;
  const float bv = bias ? bias[n] : 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wid * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (m >= Mv) continue;
      const long long o = (long long)m * a.Ncol + n;
      float v = acc[i][r] + bv;
      if (res) v += bf2f(res[o]);
      if (a.relu) v = fmaxf(v, 0.f);
      out[o] = from_f<OutT>(v);
    }
}

template <int BM, int BN, int WM, int WN, int MODE, typename OutT, bool BT = false>
int launch2(Igemm2Args a, int G, hipStream_t st) {
  const int M = a.N * a.Ho * a.Wo;
  a.tiles_n = ceil_div(a.Ncol, BN);
  const int tiles_m = MODE == 2 ? 4 * ceil_div(M / 4, BM) : ceil_div(M, BM);
  dim3 grid((unsigned)(tiles_m * a.tiles_n), G);
  hipLaunchKernelGGL((igemm2_kernel<BM, BN, WM, WN, MODE, OutT, BT>), grid, dim3(256), 0, st, a);
  DBA_LAUNCH_CHECK();
}

template <int MODE, typename OutT, bool BT = false>
int dispatch2(Igemm2Args a, int G, hipStream_t st) {
  const long long M = (long long)a.N * a.Ho * a.Wo;
  if (a.Ncol <= 32) return launch2<128, 32, 4, 1, MODE, OutT, BT>(a, G, st);
  if (a.Ncol <= 64) return launch2<128, 64, 2, 2, MODE, OutT, BT>(a, G, st);
  // wide outputs: 128x128 tiles unless the launch would not fill the chip
  if (M * G / 128 * ((a.Ncol + 127) / 128) >= 512) return launch2<128, 128, 2, 2, MODE, OutT, BT>(a, G, st);
  return launch2<64, 128, 1, 4, MODE, OutT, BT>(a, G, st);
}

}  // namespace

// Returns -100 when the shape is not handled here (caller falls back to conv.hip kernels).
DBA_EXPORT int dba_conv2_fwd(const void* x, long long x_gstride, const void* w, long long w_sstride, const int* wsel,
                             const float* bias, long long b_sstride, const void* res, void* out, long long out_gstride,
                             int out_f32, const int* nvalid, int G, int N, int H, int W, int Cin, int Ho, int Wo,
                             int Cout, int KH, int KW, int stride, int pad, int relu, void* stream) {
  Igemm2Args a{(const uint16_t*)x, x_gstride, (const uint16_t*)w, w_sstride, wsel, bias, b_sstride,
               (const uint16_t*)res, out, out_gstride, nvalid, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, relu, 1};
  hipStream_t st = (hipStream_t)stream;
  if (Cin % 8 == 0)
    return out_f32 ? dispatch2<0, float>(a, G, st) : dispatch2<0, uint16_t>(a, G, st);
  if (Cin < 8 && KH * KW * Cin <= 160) {
    a.tiles_n = ceil_div(Cout, 32);
    dim3 grid((unsigned)(ceil_div((long long)N * Ho * Wo, 256) * a.tiles_n), G);
    const bool k32 = KH * KW * Cin <= 32;
    if (out_f32) {
      if (k32) hipLaunchKernelGGL((igemm_small_kernel<float, 32>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((igemm_small_kernel<float, 160>), grid, dim3(256), 0, st, a);
    } else {
      const bool halo = KH == 3 && KW == 3 && Cin == 3 && stride == 1 && pad == 1 && Wo == W && Ho == H &&
                        Wo <= 64 && 256 % Wo == 0 && (Ho * Wo) % 256 == 0 && (W * 3) % 8 == 0 &&
                        ((uintptr_t)x % 16) == 0 && (x_gstride * 2) % 16 == 0 &&
                        (256 / Wo + 2) * (Wo + 2) * 3 * 2 <= 4096;
      if (halo) hipLaunchKernelGGL((igemm_small_kernel<uint16_t, 32, true>), grid, dim3(256), 0, st, a);
      else if (k32) hipLaunchKernelGGL((igemm_small_kernel<uint16_t, 32>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((igemm_small_kernel<uint16_t, 160>), grid, dim3(256), 0, st, a);
    }
    DBA_LAUNCH_CHECK();
  }
  return -100;
}

// Data gradient straight from the FORWARD weights w [slots][Cout][KH][KW][Cin] (no transpose
// pass): stride 1 (pad = (K-1)/2) runs as a forward conv of dY with tap-flipped weights
// (MODE 0), other strides as the scatter-form implicit GEMM (MODE 1).  accum as below.
DBA_EXPORT int dba_conv2_dgrad_w(const void* dy, long long dy_gstride, const void* w, long long w_sstride,
                                 const int* wsel, const void* accum, void* dx, long long dx_gstride,
                                 const int* nvalid, int G, int N, int H, int W, int Cin, int Ho, int Wo, int Cout,
                                 int KH, int KW, int stride, int pad, void* stream) {
  if (Cout % 8 != 0 || Cin % 8 != 0) return -100;
  hipStream_t st = (hipStream_t)stream;
  if (stride == 1 && KH == KW && pad == (KH - 1) / 2) {
    Igemm2Args a{(const uint16_t*)dy, dy_gstride, (const uint16_t*)w, w_sstride, wsel, nullptr, 0,
                 (const uint16_t*)accum, dx, dx_gstride, nvalid, N, Ho, Wo, Cout, H, W, Cin, KH, KW, 1, KH - 1 - pad,
                 0, 1};
    return dispatch2<0, uint16_t, true>(a, G, st);
  }
  Igemm2Args a{(const uint16_t*)dy, dy_gstride, (const uint16_t*)w, w_sstride, wsel, nullptr, 0,
               (const uint16_t*)accum, dx, dx_gstride, nvalid, N, Ho, Wo, Cout, H, W, Cin, KH, KW, stride, pad, 0, 1};
  return dispatch2<1, uint16_t, true>(a, G, st);
}

// accum (nullable, same layout as dx): dx = dgrad + accum (the other branch's input gradient)
DBA_EXPORT int dba_conv2_dgrad(const void* dy, long long dy_gstride, const void* wt, long long wt_sstride,
                               const int* wsel, const void* accum, void* dx, long long dx_gstride, const int* nvalid,
                               int G, int N, int H, int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW,
                               int stride, int pad, void* stream) {
  if (Cout % 8 != 0) return -100;
  Igemm2Args a{(const uint16_t*)dy, dy_gstride, (const uint16_t*)wt, wt_sstride, wsel, nullptr, 0,
               (const uint16_t*)accum, dx, dx_gstride, nvalid, N, Ho, Wo, Cout, H, W, Cin, KH, KW, stride, pad, 0, 1};
  if (stride == 2 && Cout % BK2 == 0 && H % 2 == 0 && W % 2 == 0)
    return dispatch2<2, uint16_t>(a, G, (hipStream_t)stream);
  return dispatch2<1, uint16_t>(a, G, (hipStream_t)stream);
}
