// Halo-tiled direct convolution for stride-1 convs (3x3 pad 1, 1x1 pad 0) — the bulk of
// ResNet-18's FLOPs in both the forward and (via flipped weights) the data-gradient pass.
//
// Why: an im2col implicit GEMM re-gathers every input pixel once per tap (9x for 3x3) from
// L1/L2; at CIFAR shapes (Cin = Cout = 32..128) that gather traffic, not the matrix cores,
// bounds the kernel.  Here a block owns NI segments of SR whole output rows; it stages the
// segments' input rows + halo ONCE into LDS (zero-padded borders, each pixel padded to C+8
// elements so the 32 lanes of an MFMA fragment read — 32 consecutive pixels — hit distinct
// bank slots), then walks taps x 16-channel chunks reading A fragments straight out of the
// halo at the tap's offset: no im2col, no barrier inside the K loop.  Weight fragments
// (16 B per lane, contiguous in [Cout][KH][KW][C]) stream from L2 into registers one step
// ahead.  Output goes through an fp32 LDS staging tile and leaves as 16-byte bf16 chunks
// with bias / residual / ReLU fused.
#include "common.hpp"
#include <algorithm>

namespace {

struct HaloArgs {
  const uint16_t* src; long long src_gstride;   // [G][N][H][W][C]
  const uint16_t* w; long long w_sstride;       // [slots][Cout][KH][KW][C]
  const int* wsel;
  const float* bias; long long b_sstride;
  const uint16_t* res;
  void* out; long long out_gstride;             // [G][N][H][W][Cout]
  const int* nvalid;
  int N, H, W, C, Cout, KH, pad, relu;
  int SR, NI, tiles_n;
};

template <int MI, int NJ, typename OutT>
__global__ __launch_bounds__(256) void halo_conv_kernel(HaloArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  constexpr int BM = 4 * MI * 32, BN = NJ * 32;
  const int g = blockIdx.y;
  const int HW = a.H * a.W;
  const int Mv = valid_rows(a.nvalid, g, a.N) * HW;
  const int tn = blockIdx.x % a.tiles_n, tm = blockIdx.x / a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mv) return;
  const int KW = a.KH;
  const int HR = a.SR + a.KH - 1, HW2 = a.W + KW - 1, PS = a.C + 8;
  const int segs_per_img = a.H / a.SR;
  const uint16_t* __restrict__ src = a.src + (long long)g * a.src_gstride;
  const int slot = a.wsel ? a.wsel[g] : g;
  const uint16_t* __restrict__ Wp = a.w + (long long)slot * a.w_sstride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int s0 = tm * a.NI;                   // first segment of this block
  const int K = a.KH * a.KH * a.C;
  const int KP = K + 8;                       // padded B row (distinct bank slots per lane)
  const int halo_elems = a.NI * (a.SR + a.KH - 1) * (a.W + a.KH - 1) * (a.C + 8);
  uint16_t* Bs = smem + ((halo_elems + 7) & ~7);

  // ---- stage input rows + halo of all NI segments (16-byte chunks, zero outside image)
  {
    const int c8n = a.C / 8;
    const int per_seg = HR * HW2 * c8n;
    const int total = a.NI * per_seg;
    for (int e = tid; e < total; e += 256) {
      const int seg = e / per_seg;
      int r = e - seg * per_seg;
      const int hr = r / (HW2 * c8n);
      r -= hr * HW2 * c8n;
      const int hc = r / c8n, c8 = r - hc * c8n;
      const int s = s0 + seg;
      const int n = s / segs_per_img;
      const int row = (s - n * segs_per_img) * a.SR + hr - a.pad;
      const int col = hc - a.pad;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n * HW < Mv && (unsigned)row < (unsigned)a.H && (unsigned)col < (unsigned)a.W)
        v = *(const uint4*)(src + (((long long)n * a.H + row) * a.W + col) * a.C + c8 * 8);
      *(uint4*)&smem[((seg * HR + hr) * HW2 + hc) * PS + c8 * 8] = v;
    }
  }
  // ---- stage this block's weight panel [BN][K] once (shared by the 4 waves)
  {
    const int k8n = K / 8;
    for (int e = tid; e < BN * k8n; e += 256) {
      const int r = e / k8n, k8 = e - r * k8n;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n0 + r < a.Cout) v = *(const uint4*)(Wp + (long long)(n0 + r) * K + k8 * 8);
      *(uint4*)&Bs[r * KP + k8 * 8] = v;
    }
  }
  // per-lane A-fragment base (pixel of each 32-row MFMA tile)
  int abase[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int ml = wid * MI * 32 + i * 32 + (lane & 31);
    const int seg = ml / (a.SR * a.W);
    const int rem = ml - seg * a.SR * a.W;
    const int r = rem / a.W, c = rem - r * a.W;
    abase[i] = ((seg * HR + r) * HW2 + c) * PS + (lane >> 5) * 8;
  }
  __syncthreads();

  const int steps = K / 16;
  const int cpt = a.C / 16;                   // 16-channel chunks per tap
  int bbase[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) bbase[j] = (j * 32 + (lane & 31)) * KP + (lane >> 5) * 8;
  f32x16_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  int tap = 0, cc = 0;
  for (int s = 0; s < steps; ++s) {
    const int kh = tap / KW, kw = tap - kh * KW;
    const int aoff = (kh * HW2 + kw) * PS + cc * 16;
    bf16x8_t bfr[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bfr[j] = *(const bf16x8_t*)&Bs[bbase[j] + s * 16];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const bf16x8_t av = *(const bf16x8_t*)&smem[abase[i] + aoff];
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bfr[j], acc[i][j], 0, 0, 0);
    }
    if (++cc == cpt) { cc = 0; ++tap; }
  }

  // ---- epilogue through an fp32 LDS staging tile (reuses the halo buffer)
  __syncthreads();
  float* Cst = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wid * MI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        Cst[row * BN + j * 32 + (lane & 31)] = acc[i][j][r];
      }
  __syncthreads();
  OutT* out = (OutT*)a.out + (long long)g * a.out_gstride;
  const float* bias = a.bias ? a.bias + (long long)slot * a.b_sstride : nullptr;
  const uint16_t* res = a.res ? a.res + (long long)g * a.out_gstride : nullptr;
  constexpr int CH = BN / 8;
  const bool full_n = (n0 + BN <= a.Cout) && (a.Cout % 8 == 0);
  for (int e = tid; e < BM * CH; e += 256) {
    const int row = e / CH, c8 = (e - row * CH) * 8;
    const int m = m0 + row;
    if (m >= Mv) continue;
    const int n = n0 + c8;
    const long long o = (long long)m * a.Cout + n;
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = Cst[row * BN + c8 + t];
    if (full_n) {
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
    } else {
      for (int t = 0; t < 8 && n + t < a.Cout; ++t) {
        float x = v[t] + (bias ? bias[n + t] : 0.f);
        if (res) x += bf2f(res[o + t]);
        if (a.relu) x = fmaxf(x, 0.f);
        out[o + t] = from_f<OutT>(x);
      }
    }
  }
}

template <int MI, int NJ, typename OutT>
int launch_halo(HaloArgs a, int G, size_t lds, hipStream_t st) {
  constexpr int BM = 4 * MI * 32, BN = NJ * 32;
  const long long M = (long long)a.N * a.H * a.W;
  a.tiles_n = (a.Cout + BN - 1) / BN;
  const size_t need = std::max(lds, (size_t)BM * BN * 4);
  static bool attr_set = false;   // > 64 KB of dynamic LDS must be opted into (gfx950: 160 KB per CU)
  if (need > 65536 && !attr_set) {
    hipFuncSetAttribute((const void*)halo_conv_kernel<MI, NJ, OutT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    attr_set = true;
  }
  dim3 grid((unsigned)(((M + BM - 1) / BM) * a.tiles_n), G);
  hipLaunchKernelGGL((halo_conv_kernel<MI, NJ, OutT>), grid, dim3(256), need, st, a);
  DBA_LAUNCH_CHECK();
}

}  // namespace

// Stride-1 conv with KH == KW in {1, 3}, pad == (KH-1)/2 (or the dgrad's KH-1-pad), C % 16 == 0.
// Returns -100 (not handled) for shapes whose halo does not fit LDS or do not tile.
DBA_EXPORT int dba_halo_conv(const void* x, long long x_gstride, const void* w, long long w_sstride, const int* wsel,
                             const float* bias, long long b_sstride, const void* res, void* out,
                             long long out_gstride, int out_f32, const int* nvalid, int G, int N, int H, int W, int C,
                             int Cout, int KH, int pad, int relu, void* stream) {
  if (C % 16 != 0 || (KH != 1 && KH != 3) || pad != (KH - 1) / 2) return -100;
  // Halo tiling pays where activations dominate the operand traffic: narrow outputs
  // (ResNet stage 1).  Wide layers are weight-dominated and go to the gen-2 GEMM.
  if (Cout > 32) return -100;
  const int MI = 2;
  const int BM = 4 * MI * 32;
  if (BM % W != 0) return -100;
  int SR = std::min(H, BM / W);
  if (H % SR != 0 || BM % (SR * W) != 0) return -100;
  const int NI = BM / (SR * W);
  const size_t halo = ((size_t)NI * (SR + KH - 1) * (W + KH - 1) * (C + 8) + 7) / 8 * 8;
  const size_t lds = (halo + 32 * ((size_t)KH * KH * C + 8)) * 2;
  if (lds > 96 * 1024) return -100;
  HaloArgs a{(const uint16_t*)x, x_gstride, (const uint16_t*)w, w_sstride, wsel, bias, b_sstride,
             (const uint16_t*)res, out, out_gstride, nvalid, N, H, W, C, Cout, KH, pad, relu, SR, NI, 1};
  hipStream_t st = (hipStream_t)stream;
  (void)MI;
  return out_f32 ? launch_halo<2, 1, float>(a, G, lds, st) : launch_halo<2, 1, uint16_t>(a, G, lds, st);
}
