// Image stems: direct convolution of a few-channel input in exact fp32 on the VALU (gfx950).
//
// The first conv of every image model reads Cin = 3 (MnistNet: 1) channels: K = KH*KW*Cin =
// 27 (CIFAR ResNet, models/resnet_cifar.py:72), 147 (Tiny ResNet 7x7/2, resnet_tinyimagenet.py:
// 143) or 25 (MnistNet 5x5, MnistNet.py:11).  On the implicit-GEMM MFMA kernels (xconv.hpp)
// such a conv is one 32-deep k-step per tile, so the launch is all prologue and epilogue, and
// each element is split into fp16 planes for 3 MFMAs whose work is <2 % of the FLOPs of the
// next layer (profiles/kbench_r2_fp32_f16pair.json: 19 TFLOP/s, output-write bound at ~1.4 TB/s).
// Here: TPP threads per output pixel, each owning CPT consecutive output channels; the slot's
// weights sit in LDS transposed to [k][Cout] so a thread reads its CPT channels of one tap with
// one ds_read_b128 per 4 channels (lanes of different channel groups hit different 16-B
// slots); the pixel's receptive field streams through registers one kernel row at a time.
// Every output is an fp32 FMA chain in fixed (kh, kw, ci) order: exact fp32 arithmetic and
// deterministic.  Epilogue: bias, residual, ReLU, the fp16-pair max slot of the output
// (common.hpp amax_fold) and, for a training BN, the level-0 records of the fused BN statistics
// (bnfuse.hpp bnf_tile_records' definition).
#include "common.hpp"
#include "bnfuse.hpp"

namespace {

struct StemArgs {
  const float* x; long long x_gstride;      // [G][N][H][W][CIN]
  const float* w; long long w_sstride;      // [slots][COUT][KH][KW][CIN]
  const int* wsel;
  const float* bias; long long b_sstride;   // [slots][COUT] (optional)
  const float* res;                         // output layout (optional)
  float* out; long long out_gstride;        // [G][N][Ho][Wo][COUT]
  const int* nvalid;
  int N, H, W, Ho, Wo, stride, pad, relu;
  int* amax_out; int amax_ld;
  BnFuse bf;                                // fused training BN statistics (bnfuse.hpp), mode 1
};

template <int KH, int KW, int CIN, int COUT, int CPT, int ITER>
__global__ __launch_bounds__(256) void xstem_kernel(const StemArgs a) {
  constexpr int K = KH * KW * CIN;
  constexpr int TPP = COUT / CPT;            // threads per pixel
  constexpr int PIX = 256 / TPP;             // pixels per block
  static_assert(COUT % CPT == 0 && CPT % 4 == 0, "channel groups of 4");
  __shared__ __attribute__((aligned(16))) float wt[K * COUT];          // [k][COUT]
  __shared__ __attribute__((aligned(16))) float tile[PIX * COUT];       // BN statistics tile

  const int g = blockIdx.y;
  const int tid = threadIdx.x;
  const int HoWo = a.Ho * a.Wo;
  const int Mv = valid_rows(a.nvalid, g, a.N) * HoWo;
  const bool want_stats = a.bf.mode == 1;
  const int mb = blockIdx.x * (ITER * PIX);
  if (mb >= Mv) return;   // no valid pixel in the block's tiles
  const int slot = a.wsel ? a.wsel[g] : g;
  const float* __restrict__ wg = a.w + (long long)slot * a.w_sstride;
  for (int e = tid; e < K * COUT; e += 256) {   // conflict-free LDS writes (the reads hit L1)
    const int k = e / COUT, c = e - k * COUT;
    wt[e] = wg[c * K + k];
  }
  __syncthreads();

  const int pl = tid / TPP, cg = tid - pl * TPP;
  const int c0 = cg * CPT;
  float vmax = 0.f;
  const float* bp = a.bias ? a.bias + (long long)slot * a.b_sstride + c0 : nullptr;
  for (int it = 0; it < ITER; ++it) {   // the weights in LDS serve ITER pixel tiles
    const int m0 = mb + it * PIX;
    const int m = m0 + pl;
    const bool live = pl < PIX && m < Mv;
    float acc[CPT];
#pragma unroll
    for (int c = 0; c < CPT; ++c) acc[c] = 0.f;
    if (live) {
      const int img = m / HoWo, rem = m - img * HoWo, p = rem / a.Wo, q = rem - p * a.Wo;
      const float* __restrict__ xg = a.x + (long long)g * a.x_gstride + (long long)img * a.H * a.W * CIN;
      const int h0 = p * a.stride - a.pad, w0 = q * a.stride - a.pad;
#pragma unroll 1
      for (int kh = 0; kh < KH; ++kh) {
        const int h = h0 + kh;
        const bool hok = (unsigned)h < (unsigned)a.H;
        float xr[KW * CIN];
#pragma unroll
        for (int kw = 0; kw < KW; ++kw) {
          const int w = w0 + kw;
          const bool ok = hok && (unsigned)w < (unsigned)a.W;
#pragma unroll
          for (int ci = 0; ci < CIN; ++ci) xr[kw * CIN + ci] = ok ? xg[((long long)h * a.W + w) * CIN + ci] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < KW * CIN; ++j) {
          const float4* wr = (const float4*)&wt[(kh * KW * CIN + j) * COUT + c0];
#pragma unroll
          for (int c4 = 0; c4 < CPT / 4; ++c4) {
            const float4 wv = wr[c4];
            acc[c4 * 4 + 0] = fmaf(wv.x, xr[j], acc[c4 * 4 + 0]);
            acc[c4 * 4 + 1] = fmaf(wv.y, xr[j], acc[c4 * 4 + 1]);
            acc[c4 * 4 + 2] = fmaf(wv.z, xr[j], acc[c4 * 4 + 2]);
            acc[c4 * 4 + 3] = fmaf(wv.w, xr[j], acc[c4 * 4 + 3]);
          }
        }
      }
      const long long o = (long long)g * a.out_gstride + (long long)m * COUT + c0;
#pragma unroll
      for (int c4 = 0; c4 < CPT / 4; ++c4) {
        float4 v = make_float4(acc[c4 * 4], acc[c4 * 4 + 1], acc[c4 * 4 + 2], acc[c4 * 4 + 3]);
        if (bp) { v.x += bp[c4 * 4]; v.y += bp[c4 * 4 + 1]; v.z += bp[c4 * 4 + 2]; v.w += bp[c4 * 4 + 3]; }
        if (a.res) {
          const float4 r = *(const float4*)(a.res + o + c4 * 4);
          v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
        }
        if (a.relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
        vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        *(float4*)(a.out + o + c4 * 4) = v;
        acc[c4 * 4] = v.x; acc[c4 * 4 + 1] = v.y; acc[c4 * 4 + 2] = v.z; acc[c4 * 4 + 3] = v.w;
      }
    }
    if (want_stats) {   // statistics of the raw output (fused BN implies no bias / residual / ReLU)
      if (pl < PIX) {
#pragma unroll
        for (int c = 0; c < CPT; ++c) tile[pl * COUT + c0 + c] = live ? acc[c] : 0.f;
      }
      __syncthreads();
      if (a.bf.mode == 1) {   // level-0 records (bnfuse.hpp bnf_tile_records' order)
        const int gv = ceil_div_d(Mv, kBnGrp);
        for (int e = tid; e < (PIX / 32) * COUT; e += 256) {
          const int grp = e / COUT, c = e - grp * COUT, b = m0 / 32 + grp;
          if (b >= gv) continue;
          double r4[4];
          bnf_init(r4, 1);
          for (int r = 0; r < 32; ++r) {
            if (m0 + grp * 32 + r >= Mv) break;
            const double v = (double)tile[(grp * 32 + r) * COUT + c];
            r4[0] += v;
            r4[1] = fma(v, v, r4[1]);
            r4[2] = fmax(r4[2], v);
            r4[3] = fmin(r4[3], v);
          }
          bnf_store_rec(a.bf.rec0 + (((long long)g * COUT + c) * a.bf.ngrp + b) * 4, r4[0], r4[1], r4[2], r4[3]);
        }
      }
      __syncthreads();
    }
  }
  if (a.amax_out) amax_fold(a.amax_out, a.amax_ld, g, vmax);
}

template <int KH, int KW, int CIN, int COUT, int CPT>
int stem_go(const StemArgs& a, int G, hipStream_t st) {
  constexpr int PIX = 256 / (COUT / CPT);
  constexpr int ITER = 4;   // pixel tiles per block: one weight load (LDS transpose) per 4 tiles
  if (a.bf.mode && PIX % 32 != 0) return -100;
  const long long M = (long long)a.N * a.Ho * a.Wo;
  const dim3 grid((unsigned)ceil_div(M, PIX * ITER), G);
  hipLaunchKernelGGL((xstem_kernel<KH, KW, CIN, COUT, CPT, ITER>), grid, dim3(256), 0, st, a);
  const int rc = (int)hipGetLastError();
  if (rc != 0 || !a.bf.mode) return rc;
  return bnx_finalize_go(a.bf, a.nvalid, G, a.N, a.Ho * a.Wo, st);   // the fused BN's finalize
}

}  // namespace

// y = act(conv(x, w) + bias + res) for the stem shapes (fp32 NHWC, exact fp32 FMA chains);
// returns -100 for any other shape (the caller takes the MFMA family).
DBA_EXPORT int dba_xstem_fwd(const float* x, long long x_gstride, const float* w, long long w_sstride, const int* wsel,
                             const float* bias, long long b_sstride, const float* res, float* out,
                             long long out_gstride, const int* nvalid, int G, int N, int H, int W, int Cin, int Ho,
                             int Wo, int Cout, int KH, int KW, int stride, int pad, int relu, int* amax_out,
                             int amax_ld, const void* bnf, void* stream) {
  if (((uintptr_t)out & 15) || (out_gstride & 3) || (res && ((uintptr_t)res & 15))) return -100;
  StemArgs a{};
  a.x = x; a.x_gstride = x_gstride; a.w = w; a.w_sstride = w_sstride; a.wsel = wsel;
  a.bias = bias; a.b_sstride = b_sstride; a.res = res; a.out = out; a.out_gstride = out_gstride;
  a.nvalid = nvalid; a.N = N; a.H = H; a.W = W; a.Ho = Ho; a.Wo = Wo; a.stride = stride; a.pad = pad;
  a.relu = relu; a.amax_out = amax_out; a.amax_ld = amax_ld;
  if (bnf) {
    a.bf = *(const BnFuse*)bnf;
    if (a.bf.mode != 1 || bias || res || relu || a.bf.C != Cout) return -108;
  }
  hipStream_t st = (hipStream_t)stream;
  if (KH == 3 && KW == 3 && Cin == 3 && Cout == 32) return stem_go<3, 3, 3, 32, 8>(a, G, st);
  if (KH == 7 && KW == 7 && Cin == 3 && Cout == 64) return stem_go<7, 7, 3, 64, 8>(a, G, st);
  if (KH == 5 && KW == 5 && Cin == 1 && Cout == 20 && !a.bf.mode) return stem_go<5, 5, 1, 20, 4>(a, G, st);
  return -100;
}
