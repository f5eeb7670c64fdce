// Persistent register-weight halo convolution for the stride-1 3x3 layers of ResNet-18
// (CIFAR stages 1-3: 32ch@32x32, 64ch@16x16, 128ch@8x8; Tiny stages 1-2) — forward, eval
// (BN folded into bias) and, with in-kernel flip-transposed weights, the data gradient.
//
// Design (CDNA4 / gfx950):
//   * operand swap: the WEIGHTS are the MFMA A operand (32 output channels x 16 k) and live
//     in VGPRs for the whole kernel (each wave owns one 32-channel slice: 9*C/16 fragments),
//     the activations are the B operand read from LDS.  One ds_read_b128 per
//     v_mfma_f32_32x32x16_bf16 — well inside the LDS budget — and no weight traffic per tile;
//   * output lanes = pixels: each lane holds 4 runs of 4 consecutive channels of ONE pixel,
//     so the epilogue (bias / residual / ReLU) stores 8-byte NHWC chunks straight from the
//     accumulators — no LDS staging tile, no extra barrier;
//   * persistent blocks: the grid is sized to the chip (not to the problem), every block
//     walks a contiguous run of (group, image, row-segment) tiles, reloading weights only
//     when its run crosses a group (client model) boundary.  The run boundaries are
//     derived in-kernel from nvalid[] so inactive/padded replicas cost nothing and the
//     launch is HIP-graph-capturable;
//   * the halo (SR+2 rows x W+2 cols x C channels) of tiles t+1, t+2 streams global -> LDS
//     by LDS-DMA (global_load_lds_dwordx4, no staging registers) into a 3-buffer ring while
//     tile t computes: one raw barrier per tile with a counted vmcnt, so the youngest DMA
//     stays in flight across it.  Border padding is DMA'd from a zero page;
//   * LDS image is unpadded (lane-linear, as LDS-DMA requires) with a 16-byte-chunk XOR
//     swizzle applied on the SOURCE address, chosen per geometry so the 16 lanes of every
//     ds_read_b128 lane group hit 16 distinct bank slots (see swz());
//   * B fragments are double-buffered one k-step ahead of the MFMAs that consume them.
// Data-gradient mode (tr = 1): dX = conv(dY, W^T flipped) — the weight fragments are
// gathered transposed+flipped from the forward [Cout][3][3][Cin] tensor while loading them
// into registers, so no separate transpose kernel runs.
#include "common.hpp"
#include <algorithm>
#include <cstdlib>

namespace {

struct PconvArgs {
  const uint16_t* src; long long src_gstride;   // [G][N][H][W][C]
  const uint16_t* w; long long w_sstride;       // fwd: [slots][COUT][3][3][C]; tr: [slots][C][3][3][COUT]
  const int* wsel;
  const float* bias; long long b_sstride;
  const uint16_t* res;                          // [G][N][H][W][COUT]
  uint16_t* out; long long out_gstride;
  const int* nvalid;
  const uint16_t* zeros;                        // >= 16 zero bytes (source of halo padding)
  int G, N, H, relu, tr;
};

// LDS position of halo pixel (hr, hc).  Stride 1: row-major with pitch W+2.  Stride 2:
// columns de-interleaved by parity (even half, then odd half, W+1 slots each), so the
// stride-2 pixel walk of an output row reads CONSECUTIVE positions.
template <int S, int W>
__device__ __forceinline__ int hpos(int hr, int hc) {
  if constexpr (S == 1) return hr * (W + 2) + hc;
  else return hr * 2 * (W + 1) + (hc & 1) * (W + 1) + (hc >> 1);
}

// 16-byte-chunk swizzle inside a pixel (CP chunks per pixel): every ds_read_b128 lane group
// of a B-fragment read hits 16 distinct bank slots (checked exhaustively over all taps for
// each geometry used).
template <int S, int CP, int W>
__device__ __forceinline__ int swz(int hr, int hc) {
  if constexpr (S == 1) {
    if constexpr (CP == 4) {
      const int q = hr * (W + 2) + hc;
      return (q >> 2) & 3;
    } else if constexpr (CP == 8) {
      return (hc >> 1) & 7;
    } else {
      return ((hr & 1) << 3) | (hc & 7);
    }
  } else {
    if constexpr (CP == 4) return (hc >> 3) & 3;
    else return (((hr >> 1) & 1) << 2) | ((hc >> 2) & 3);
  }
}

// W = OUTPUT width; S = stride (1, or 2 for the stage-entry convs, forward only)
template <int C, int COUT, int W, int MI, int NWC, int WPE, bool TR, int S = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void pconv_kernel(PconvArgs a) {
  constexpr int CP = C / 8;                 // 16-B chunks per pixel
  constexpr int HP = S == 1 ? W + 2 : 2 * (W + 1);   // halo row pitch (positions)
  constexpr int WIN = W * S;                // input width
  constexpr int NWP = 4 / NWC;              // waves along pixels
  constexpr int BPX = NWP * MI * 32;        // output pixels per tile
  constexpr int SR = BPX / W;               // output rows per tile
  constexpr int HR = S * SR + (S == 1 ? 2 : 1);
  constexpr int HALO = HR * HP * CP;        // chunks per halo image
  constexpr int NCH = (HALO + 255) / 256;   // staged chunks per thread
  constexpr int KSTEPS = 9 * C / 16;
  constexpr int CSTEPS = C / 16;
  static_assert(BPX % W == 0 && NWC * 32 == COUT, "tile geometry");
  __shared__ __attribute__((aligned(16))) uint4 lds[3][NCH * 256];
  // s_waitcnt immediate: vmcnt = n, expcnt / lgkmcnt = no wait (gfx9 encoding)
  constexpr int kWaitKeep = (NCH & 15) | ((NCH >> 4) << 14) | (0x7 << 4) | (0xF << 8);
  constexpr int kWaitAll = (0x7 << 4) | (0xF << 8);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wc = wid % NWC, wp = wid / NWC;
  const int segs = a.H / SR;
  const int HWo = a.H * W;
  const int HIN = a.H * S;                  // input height

  // ---- this block's contiguous run [v0, v1) of valid tiles
  int V = 0;
  for (int g = 0; g < a.G; ++g) V += valid_rows(a.nvalid, g, a.N) * segs;
  const int per = (V + gridDim.x - 1) / gridDim.x;
  const int v0 = blockIdx.x * per;
  const int v1 = min(V, v0 + per);
  if (v0 >= v1) return;
  int g = 0, t = v0;
  for (;;) {
    const int nt = valid_rows(a.nvalid, g, a.N) * segs;
    if (t < nt) break;
    t -= nt;
    ++g;
  }

  bf16x8_t wreg[KSTEPS];
  float4 breg[4];                           // this lane's 16 output channels' bias
  auto load_weights = [&](int gg) {
    const int slot = a.wsel ? a.wsel[gg] : gg;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
      breg[jj] = a.bias ? *(const float4*)(a.bias + (long long)slot * a.b_sstride + wc * 32 + jj * 8 + (lane >> 5) * 4)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
    const uint16_t* __restrict__ Wp = a.w + (long long)slot * a.w_sstride;
    const int row = wc * 32 + (lane & 31);
    [[maybe_unused]] __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)Wp, (short)0, C * 9 * COUT * 2, 0x00020000);
    [[maybe_unused]] const int vlane = ((lane >> 5) * 8 * 9 * COUT + row) * 2;
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      const int k = s * 16 + (lane >> 5) * 8;
      if constexpr (!TR) {
        wreg[s] = *(const bf16x8_t*)(Wp + (long long)row * (9 * C) + k);
      } else {
        // transposed + tap-flipped gather from the forward [C][3][3][COUT] tensor: k = tap*C + co,
        // element (co + j, 8 - tap, row).  Buffer loads: the per-lane part of the offset is one
        // VGPR, the (s, j) part a scalar constant — no per-load 64-bit address registers.
        const int c16 = s % CSTEPS, tap = s / CSTEPS;
        union { bf16x8_t v; uint16_t u[8]; } tmp;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          tmp.u[j] = __builtin_amdgcn_raw_buffer_load_b16(
              rsrc, vlane, ((c16 * 16 + j) * 9 + 8 - tap) * COUT * 2, 0);
        wreg[s] = tmp.v;
      }
    }
  };

  // LDS slot e (lane-linear per DMA instruction) holds global chunk (e % CP) ^ swz of pixel e / CP
  auto stage = [&](int gg, int tt, int buf) {
    const int n = tt / segs, sg = tt - n * segs;
    const int row0 = sg * SR * S - 1;
    const uint16_t* __restrict__ s = a.src + (long long)gg * a.src_gstride + (long long)n * HIN * WIN * C;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int e = tid + 256 * i;
      const uint16_t* p = a.zeros;
      if (e < HALO) {
        const int cs = e % CP, pix = e / CP;
        const int hr = pix / HP, rem = pix - hr * HP;
        int hc = rem;
        if constexpr (S == 2) hc = rem < W + 1 ? 2 * rem : 2 * (rem - (W + 1)) + 1;
        const int ih = row0 + hr, iw = hc - 1;
        if ((unsigned)ih < (unsigned)HIN && (unsigned)iw < (unsigned)WIN)
          p = s + ((long long)ih * WIN + iw) * C + (cs ^ swz<S, CP, W>(hr, hc)) * 8;
      }
      __builtin_amdgcn_global_load_lds((const void*)p,
                                       (__attribute__((address_space(3))) void*)&lds[buf][i * 256 + wid * 64],
                                       16, 0, 0);
    }
  };

  auto next_tile = [&](int& gg, int& tt) {
    ++tt;
    while (tt >= valid_rows(a.nvalid, gg, a.N) * segs) { tt = 0; ++gg; }
  };
  // 3-deep LDS ring: tiles v+1 and v+2 are in flight while tile v computes.  Waits are
  // counted (vmcnt = one tile's DMA instructions) and the barrier is a raw s_barrier, so
  // the younger tile's DMA stays in flight across it (a __syncthreads would drain it).
  load_weights(g);
  stage(g, t, 0);
  int gb = g, tb = t;               // most recently staged tile
  if (v0 + 1 < v1) {
    next_tile(gb, tb);
    stage(gb, tb, 1);
    __builtin_amdgcn_s_waitcnt(kWaitKeep);
  } else {
    __builtin_amdgcn_s_waitcnt(kWaitAll);
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // per-lane pixel coordinates of the wave's MI fragments inside a tile
  int pr[MI], pc[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int p = (wp * MI + i) * 32 + (lane & 31);
    pr[i] = p / W;
    pc[i] = p - pr[i] * W;
  }
  const int hi = lane >> 5;
  int cur = 0;
  for (int v = v0; v < v1; ++v) {
    // keep the per-step LDS address math inside the k-loop (not hoisted into VGPRs for all
    // KSTEPS x MI fragments across the tile loop)
#pragma unroll
    for (int i = 0; i < MI; ++i) asm volatile("" : "+v"(pr[i]), "+v"(pc[i]));
    const int n_img = t / segs, sg_img = t - n_img * segs;
    const long long mbase = (long long)n_img * HWo + (long long)sg_img * SR * W;
    uint16_t* __restrict__ o = a.out + (long long)g * a.out_gstride;
    const uint16_t* __restrict__ rs = a.res ? a.res + (long long)g * a.out_gstride : nullptr;
    uint2 rres[MI][4];
    if (rs) {   // issued early: their latency hides under the k-loop
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          rres[i][jj] = *(const uint2*)(rs + (mbase + (wp * MI + i) * 32 + (lane & 31)) * COUT + wc * 32 + jj * 8 + hi * 4);
    }
    f32x16_t acc[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    const uint4* L = lds[cur];
    bf16x8_t bq[2][MI];
    auto loadB = [&](int st, bf16x8_t* q) {
      const int tap = st / CSTEPS, c16 = st - tap * CSTEPS;
      const int kh = tap / 3, kw = tap - kh * 3;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int hr = S * pr[i] + kh, hc = S * pc[i] + kw;
        q[i] = *(const bf16x8_t*)&L[hpos<S, W>(hr, hc) * CP + ((c16 * 2 + hi) ^ swz<S, CP, W>(hr, hc))];
      }
    };
    loadB(0, bq[0]);
#pragma unroll
    for (int st = 0; st < KSTEPS; ++st) {
      if (st + 1 < KSTEPS) loadB(st + 1, bq[(st + 1) & 1]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wreg[st], bq[st & 1][i], acc[i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- epilogue: lane = pixel, 4 runs of 4 consecutive channels (residual loads were
    // issued before the k-loop; bias lives in registers)
    {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const long long m = mbase + (wp * MI + i) * 32 + (lane & 31);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int ch = wc * 32 + jj * 8 + hi * 4;
          float v[4] = {acc[i][jj * 4] + breg[jj].x, acc[i][jj * 4 + 1] + breg[jj].y,
                        acc[i][jj * 4 + 2] + breg[jj].z, acc[i][jj * 4 + 3] + breg[jj].w};
          if (rs) {
            const uint2 rv = rres[i][jj];
            v[0] += __uint_as_float(rv.x << 16);
            v[1] += __uint_as_float(rv.x & 0xffff0000u);
            v[2] += __uint_as_float(rv.y << 16);
            v[3] += __uint_as_float(rv.y & 0xffff0000u);
          }
          if (a.relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          uint2 pk;
          pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          *(uint2*)(o + m * COUT + ch) = pk;
        }
      }
    }

    if (v + 1 < v1) {
      asm volatile("" ::: "memory");
      const bool has2 = v + 2 < v1;
      if (has2) {
        next_tile(gb, tb);
        stage(gb, tb, cur == 0 ? 2 : cur - 1);   // buffer of tile v-1 (retired by the last barrier)
        __builtin_amdgcn_s_waitcnt(kWaitKeep);  // tile v+1 landed; v+2 stays in flight
      } else {
        __builtin_amdgcn_s_waitcnt(kWaitAll);
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      int gn = g, tn = t;
      next_tile(gn, tn);
      if (gn != g) load_weights(gn);
      g = gn;
      t = tn;
      cur = cur == 2 ? 0 : cur + 1;
    }
  }
}

int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <int C, int COUT, int W, int MI, int NWC, int WPE, int S = 1>
int launch_pconv(const PconvArgs& a, hipStream_t st) {
  constexpr int BPX = (4 / NWC) * MI * 32;
  constexpr int SR = BPX / W;
  if (a.H % SR != 0) return -100;
  const long long tiles = (long long)a.G * a.N * (a.H / SR);
  // Bounded persistence: at least one wave of blocks per CU slot, but no block walks more than
  // ~kTilesPerBlock tiles, so CUs turn over every few tens of microseconds.  A fully
  // persistent grid would hold every CU's LDS for the whole launch and starve the
  // (higher-priority) training stream that runs concurrently with evaluation.
  static const int tpb = [] {
    const char* e = getenv("DBA_PCONV_TPB");
    const int v = e ? atoi(e) : 8;
    return v > 0 ? v : 8;
  }();
  const long long by_turnover = (tiles + tpb - 1) / tpb;
  const int grid = (int)std::max(1LL, std::min(tiles, std::max((long long)num_cus() * WPE, by_turnover)));
  if constexpr (S == 1) {
    if (a.tr)
      hipLaunchKernelGGL((pconv_kernel<C, COUT, W, MI, NWC, WPE, true, 1>), dim3(grid), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((pconv_kernel<C, COUT, W, MI, NWC, WPE, false, 1>), dim3(grid), dim3(256), 0, st, a);
  } else {
    if (a.tr) return -100;
    hipLaunchKernelGGL((pconv_kernel<C, COUT, W, MI, NWC, WPE, false, S>), dim3(grid), dim3(256), 0, st, a);
  }
  DBA_LAUNCH_CHECK();
}

}  // namespace

// 3x3 pad-1 conv (tr = 0) or, at stride 1, its data gradient (tr = 1, w = the forward
// weight).  H, W = OUTPUT size.  Geometries (C, Cout, W, stride): (32,32,32,1), (64,64,16,1),
// and the stage-entry convs (32,64,16,2), (64,128,8,2) (128/256-channel stride-1 layers need
// 288+ weight VGPRs per wave: they stay on the implicit-GEMM kernel).  Returns -100 otherwise.
DBA_EXPORT int dba_pconv(const void* x, long long x_gstride, const void* w, long long w_sstride, const int* wsel,
                         const float* bias, long long b_sstride, const void* res, void* out, long long out_gstride,
                         const int* nvalid, const void* zeros, int G, int N, int H, int W, int C, int Cout, int tr,
                         int relu, int stride, void* stream) {
  PconvArgs a{(const uint16_t*)x, x_gstride, (const uint16_t*)w, w_sstride, wsel, bias, b_sstride,
              (const uint16_t*)res, (uint16_t*)out, out_gstride, nvalid, (const uint16_t*)zeros, G, N, H, relu, tr};
  hipStream_t st = (hipStream_t)stream;
  if (stride == 1) {
    if (C == 32 && Cout == 32 && W == 32) return launch_pconv<32, 32, 32, 2, 1, 2>(a, st);
    if (C == 64 && Cout == 64 && W == 16) return launch_pconv<64, 64, 16, 4, 2, 1>(a, st);
  } else if (stride == 2 && !tr) {
    if (C == 32 && Cout == 64 && W == 16) return launch_pconv<32, 64, 16, 2, 2, 1, 2>(a, st);
    if (C == 64 && Cout == 128 && W == 8) return launch_pconv<64, 128, 8, 2, 4, 1, 2>(a, st);
  }
  return -100;
}
