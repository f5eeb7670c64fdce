// Halo-tiled weight gradient for the stride-1 3x3 convolutions (ResNet-18 stages 1-4):
//   dW[co][kh][kw][ci] += sum over pixels of dY[px][co] * X[px shifted by (kh-1, kw-1)][ci]
//
// The reduction axis is the PIXEL, but NHWC stores pixels as rows with channels
// contiguous — both MFMA operands need their k (pixel) index inside a lane.  gfx950's
// transposing LDS read (ds_read_b64_tr_b16) delivers exactly that from the natural
// row-major images, so the tiles stream global -> LDS untouched (LDS-DMA) and are
// consumed column-wise:
//   * A = dY^T (32 output channels x 16 pixels), B = X_tap (16 pixels x 32 input channels);
//   * a block owns a (CO x CI) channel slice of one client replica and a contiguous run of
//     (image, row-segment) tiles; per tile it stages the dY tile [SR*W][CO] and the input
//     halo [(SR+2) x (W+2)][CI] once and reuses the halo for all 9 taps (no im2col);
//   * one wave per (32-co, 32-ci, kernel row kh) owns 3 accumulators (kw = 0..2);
//   * 3-deep LDS ring: tiles t+1 and t+2 land by DMA while tile t computes; counted vmcnt
//     and a raw barrier (one per tile) keep the youngest DMA in flight across it;
//   * 64-channel images use a 16-byte-chunk XOR swizzle (bit 2 of the chunk by bit 1 of the
//     pixel) so the 4 rows of every transposed read hit distinct bank slots;
//   * the block's partial dW leaves by fp32 atomics (split-K over pixel runs) into the flat
//     gradient buffer.
#include "common.hpp"
#include <algorithm>

namespace {

typedef short v4i16_t __attribute__((ext_vector_type(4)));

struct PwArgs {
  const uint16_t* dy; long long dy_gstride;     // [G][N][H][W][Cout]
  const uint16_t* x; long long x_gstride;       // [G][N][H][W][Cin]
  float* dw; long long dw_gstride;              // [G][Cout][3][3][Cin] (fp32, accumulated)
  const int* nvalid;
  const uint16_t* zeros;
  int N, H, Cout, Cin;
  int G, slices, ncu;                           // launch geometry for the in-kernel split-K choice
};

// Split-K factor S (pixel runs per output slice), chosen IN-KERNEL from the number of
// replicas active this step (the launch is captured once in a HIP graph for all G): enough
// blocks to cover the CUs, but the S x |dW| fp32 atomics (~1.3 TB/s chip-wide) must not
// outweigh the MFMA work.  A lone attacker finishing its poison epochs gets ~10x the blocks
// of a step where all G clients train.
__device__ __forceinline__ int split_k(const PwArgs& a, int tiles) {
  int active = 0;
  for (int g = 0; g < a.G; ++g) active += valid_rows(a.nvalid, g, a.N) > 0;
  active = active > 0 ? active : 1;
  const float by_cus = (float)a.ncu / (float)(active * a.slices);
  const float by_atomics = 3.0e6f / ((float)active * a.Cout * a.Cin * 9);
  const int S = (int)fminf(by_cus, by_atomics);
  return max(1, min(min(tiles, (int)gridDim.x), S));
}

template <int CH>
__device__ __forceinline__ int swz_px(int px) {   // chunk XOR for a CH-channel image row
  if constexpr (CH == 64) return ((px >> 1) & 1) << 2;
  else return 0;
}

// byte offset of (row, channel col) in a CH-channel image with the swizzle; col % 4 == 0
template <int CH>
__device__ __forceinline__ int img_off(int row, int col) {
  const int chunk = col >> 3;
  return row * CH * 2 + ((chunk ^ swz_px<CH>(row)) << 4) + ((col & 7) << 1);
}

// A tile is SR rows of one image (NIMG == 1) or NIMG whole images (SR == H), the latter for
// the small-spatial stages so each DMA round trip carries enough pixels.
// WK > 1 splits each tile's pixels over WK wave groups (more waves for the narrow layers);
// their partial sums meet in LDS before the atomics.
template <int CO, int CI, int W, int SR, int NIMG, int WK>
__global__ __launch_bounds__((CO / 32) * (CI / 32) * 3 * WK * 64) void pwgrad_kernel(PwArgs a) {
  constexpr int NCO = CO / 32, NCI = CI / 32;
  constexpr int NW = NCO * NCI * 3 * WK;
  constexpr int NR = NCO * NCI * 3;               // waves per pixel group
  constexpr int NT = NW * 64;
  constexpr int IP = SR * W;                      // pixels per image slab
  constexpr int TP = NIMG * IP;                   // pixels per tile
  constexpr int HP = W + 2, HR = SR + 2;
  constexpr int HIMG = HR * HP;                   // halo pixels per image slab
  constexpr int DYCH = TP * CO / 8;               // 16-B chunks of the dY tile
  constexpr int HCH = NIMG * HIMG * CI / 8;       // 16-B chunks of the halo
  constexpr int NI = (DYCH + HCH + NT - 1) / NT;  // DMA instructions per thread per tile
  constexpr int BUF = NI * NT;                    // chunks per buffer
  static_assert(TP % (16 * WK) == 0 && W % 4 == 0, "tile geometry");
  static_assert((WK - 1) * NR * 3 * 16 * 64 * 4 <= 3 * BUF * 16, "wave-group reduction fits the LDS ring");
  __shared__ __attribute__((aligned(16))) uint4 lds[3][BUF];
  constexpr int kWaitKeep = (NI & 15) | ((NI >> 4) << 14) | (0x7 << 4) | (0xF << 8);   // vmcnt(NI)
  constexpr int kWaitAll = (0x7 << 4) | (0xF << 8);                                    // vmcnt(0)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = blockIdx.y;
  const int nci_blk = a.Cin / CI;
  const int co0 = (blockIdx.z / nci_blk) * CO, ci0 = (blockIdx.z % nci_blk) * CI;
  const int segs = a.H / SR;
  const int nimg = valid_rows(a.nvalid, g, a.N);
  const int T = NIMG == 1 ? nimg * segs : (nimg + NIMG - 1) / NIMG;
  if (T == 0) return;
  const int S = split_k(a, NIMG == 1 ? a.N * segs : (a.N + NIMG - 1) / NIMG);
  if ((int)blockIdx.x >= S) return;
  const int per = (T + S - 1) / S;
  const int t0 = blockIdx.x * per, t1 = min(T, t0 + per);
  if (t0 >= t1) return;
  const bool atomic = S > 1;
  const int HW = a.H * W;
  const uint16_t* __restrict__ dyg = a.dy + (long long)g * a.dy_gstride;
  const uint16_t* __restrict__ xg = a.x + (long long)g * a.x_gstride;

  auto stage = [&](int tt, int buf) {
    int n0, row0;
    if (NIMG == 1) { n0 = tt / segs; row0 = (tt - n0 * segs) * SR; }
    else { n0 = tt * NIMG; row0 = 0; }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int e = tid + NT * i;
      const uint16_t* p = a.zeros;
      if (e < DYCH) {
        const int px = e / (CO / 8), cs = e - px * (CO / 8);
        const int j = px / IP, pl = px - j * IP;
        if (n0 + j < nimg)
          p = dyg + ((long long)(n0 + j) * HW + row0 * W + pl) * a.Cout + co0 + ((cs ^ swz_px<CO>(px)) << 3);
      } else if (e < DYCH + HCH) {
        const int e2 = e - DYCH;
        const int hp = e2 / (CI / 8), cs = e2 - hp * (CI / 8);
        const int j = hp / HIMG, hl = hp - j * HIMG;
        const int hr = hl / HP, hc = hl - hr * HP;
        const int ih = row0 - 1 + hr, iw = hc - 1;
        if (n0 + j < nimg && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)W)
          p = xg + (((long long)(n0 + j) * a.H + ih) * W + iw) * a.Cin + ci0 + ((cs ^ swz_px<CI>(hp)) << 3);
      }
      __builtin_amdgcn_global_load_lds((const void*)p,
                                       (__attribute__((address_space(3))) void*)&lds[buf][i * NT + wid * 64],
                                       16, 0, 0);
    }
  };

  // wave roles
  const int wr = wid % NR, wk = wid / NR;         // role within the pixel group, pixel group
  const int kh = wr % 3;
  const int wci = (wr / 3) % NCI, wco = wr / (3 * NCI);
  // transposed-read lane geometry (T10): group G = lane>>4, q = row in the 4-row block, p = 4-col group
  const int G4 = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
  const int hsel = G4 >> 1;                       // k half (rows 8h..8h+7)
  const int colA = wco * 32 + 16 * (G4 & 1) + 4 * p4;   // co within the slice
  const int colB = wci * 32 + 16 * (G4 & 1) + 4 * p4;   // ci within the slice

  f32x16_t acc[3];
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[k][r] = 0.f;

  // 3-deep ring: tiles tt+1, tt+2 in flight while tt computes; counted vmcnt + raw barrier
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
    const char* Lb = reinterpret_cast<const char*>(lds[cur]);
    const char* Ldy = Lb;
    const char* Lx = Lb + DYCH * 16;
#pragma unroll 2
    for (int ks = wk; ks < TP / 16; ks += WK) {
      union { bf16x8_t v; v4i16_t h[2]; } fa, fb[3];
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        const int px = ks * 16 + 8 * hsel + 4 * t2 + q;          // pixel (k index) this lane addresses
        fa.h[t2] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4i16_t*)(Ldy + img_off<CO>(px, colA)));
        const int j = px / IP, pl = px - j * IP;
        const int r = pl / W, c = pl - r * W;
        const int hp0 = j * HIMG + (r + kh) * HP + c;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
          fb[kw].h[t2] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4i16_t*)(Lx + img_off<CI>(hp0 + kw, colB)));
      }
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) acc[kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa.v, fb[kw].v, acc[kw], 0, 0, 0);
    }
    if (tt + 1 < t1) {
      asm volatile("" ::: "memory");
      if (tt + 2 < t1) {
        stage(tt + 2, cur == 0 ? 2 : cur - 1);     // buffer of tile tt-1
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

  if constexpr (WK > 1) {   // fold the pixel groups' partials into group 0 through the (idle) LDS ring
    float* red = reinterpret_cast<float*>(&lds[0][0]);
    __syncthreads();
    if (wk > 0) {
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int r = 0; r < 16; ++r) red[((((wk - 1) * NR + wr) * 3 + kw) * 16 + r) * 64 + lane] = acc[kw][r];
    }
    __syncthreads();
    if (wk > 0) return;
#pragma unroll
    for (int k2 = 1; k2 < WK; ++k2)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[kw][r] += red[((((k2 - 1) * NR + wr) * 3 + kw) * 16 + r) * 64 + lane];
  }
  // D[co][ci]: lane -> ci column (lane & 31), registers -> co rows
  float* __restrict__ dwg = a.dw + (long long)g * a.dw_gstride;
  const int ci = ci0 + wci * 32 + (lane & 31);
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + wco * 32 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
      float* d = dwg + ((long long)(co * 3 + kh) * 3 + kw) * a.Cin + ci;
      if (atomic) atomicAdd(d, acc[kw][r]);
      else *d += acc[kw][r];                      // sole writer of this element
    }
}

int num_cus_w() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <int CO, int CI, int W, int SR, int NIMG, int WK>
int launch_pw(const PwArgs& a, int G, hipStream_t st) {
  if (a.H % SR != 0 || a.Cout % CO != 0 || a.Cin % CI != 0 || (NIMG > 1 && SR != a.H)) return -100;
  const int slices = (a.Cout / CO) * (a.Cin / CI);
  const int tiles = NIMG == 1 ? a.N * (a.H / SR) : (a.N + NIMG - 1) / NIMG;
  PwArgs b = a;
  b.G = G;
  b.slices = slices;
  b.ncu = num_cus_w();
  // grid.x = the largest split any activity pattern can ask for (one active replica)
  const double s1 = std::min((double)b.ncu / slices, 3.0e6 / ((double)a.Cout * a.Cin * 9));
  const int smax = std::max(1, std::min(tiles, (int)s1));
  dim3 grid(smax, G, slices);
  hipLaunchKernelGGL((pwgrad_kernel<CO, CI, W, SR, NIMG, WK>), grid, dim3((CO / 32) * (CI / 32) * 3 * WK * 64), 0,
                     st, b);
  DBA_LAUNCH_CHECK();
}

}  // namespace

// dW (+)= wgrad of a stride-1 3x3 pad-1 conv.  Returns -100 for shapes it does not tile.
DBA_EXPORT int dba_pwgrad(const void* dy, long long dy_gstride, const void* x, long long x_gstride, float* dw,
                          long long dw_gstride, const int* nvalid, const void* zeros, int G, int N, int H, int W,
                          int Cin, int Cout, void* stream) {
  PwArgs a{(const uint16_t*)dy, dy_gstride, (const uint16_t*)x, x_gstride, dw, dw_gstride, nvalid,
           (const uint16_t*)zeros, N, H, Cout, Cin, G, 1, 256};
  hipStream_t st = (hipStream_t)stream;
  if (Cin == 32 && Cout == 32 && W == 32) return launch_pw<32, 32, 32, 8, 1, 2>(a, G, st);
  if (Cin % 64 == 0 && Cout % 64 == 0) {
    if (W == 16) return launch_pw<64, 64, 16, 8, 1, 1>(a, G, st);
    if (W == 8) return launch_pw<64, 64, 8, 8, 1, 1>(a, G, st);
    if (W == 4 && H == 4) return launch_pw<64, 64, 4, 4, 4, 1>(a, G, st);
  }
  return -100;
}
