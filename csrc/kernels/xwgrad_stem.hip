// Weight gradient of the 3-channel 3x3 stride-1 pad-1 stem conv (gfx950, fp32):
//
//     dW[co][kh][kw][ci] = sum_p dy[p][co] * x[p + (kh - 1, kw - 1)][ci]       (32 x 27 outputs)
//
// the autograd of the reference stem (/root/reference/models/resnet_cifar.py:72, conv1 of the
// CIFAR ResNets; the Tiny-ImageNet stem has the same 3 -> 32 3x3 form on 64-wide images).  The
// implicit-GEMM weight gradient runs it as a K = 27 GEMM with scalar (VEC 1) staging and the
// output rows split over a handful of 32 x 128 tiles: ~7 TFLOP/s.  The product is tiny
// (2 * 27 * 32 FLOP per pixel) and the dy read (128 B per pixel) dominates, so this is a
// bandwidth kernel: a workgroup owns 256 consecutive pixels (256 / W whole image rows of one
// replica), reads its dy tile once with coalesced 16-B loads into LDS, builds the 256 x 27 patch
// matrix from a zero-padded (rows + 2) x (W + 2) x 3 image window, and reduces the outer
// products with exact fp32 FMAs (no operand split: 4 x 4 register tiles, 2 LDS reads per 16
// FMAs).  Four row groups meet in LDS in a fixed order; the workgroup's [32][27] partial is one
// slab of the batched slab reduction (xwgrad.hip xwgrad_reduce_batch_kernel, slab order).
//
// Lazy input gradient: when the stem's BN input gradient is not stored (the stem has no data
// gradient, so the weight gradient is its only consumer) dy = fma(A, d, fma(B, y, K)) is formed
// while staging — bit-identical to xbn.hip bnx_dy_kernel — from the finished output gradient d,
// the BN input y and the BN's backward rows (bnfuse.hpp), which saves that pass and its 128 B per
// pixel round trip.
//
// Slab geometry (256 rows) is per replica, so the bits do not depend on how many replicas share
// the launch; no atomics.
#include "common.hpp"
#include "bnfuse.hpp"

namespace {

struct XWSArgs {
  const float* d; long long d_gstride;     // [G][N][H][W][32]: dy, or the finished BN output gradient
  const float* y;                          // lazy: the BN input (same layout / stride as d)
  const float* coef;                       // lazy: BN rows [G][kBnRows][32] (A, B, K), else null
  const float* x; long long x_gstride;     // [G][N][H][W][3] input image
  float* ws;                               // slabs [Z][G][32 * 27], Z = N * H * W / 256
  const int* nvalid;
  int N, H;
};

constexpr int kCo = 32, kK = 27, kPix = 256;

template <int W>
__global__ __launch_bounds__(256, 2) void xwgrad_stem_kernel(const XWSArgs a) {
  constexpr int R = kPix / W;                  // image rows per workgroup
  constexpr int RW = (R + 2) * (W + 2) * 3;    // zero-padded input window (floats)
  __shared__ float4 dys[kPix * 8];             // [p][co / 4]   (reused for the row-group sums)
  __shared__ float4 pat[kPix * 7];             // [p][k / 4], k padded 27 -> 28 with a zero
  __shared__ float raw[RW];
  const int g = blockIdx.y, z = blockIdx.x, G = gridDim.y, tid = threadIdx.x;
  const int Mv = valid_rows(a.nvalid, g, a.N) * a.H * W;
  if (z * kPix >= Mv) return;                  // (the reduction reads the first Mv / 256 slabs)
  const int img = (z * R) / a.H, h0 = (z * R) - img * a.H;

  // input window rows h0 - 1 .. h0 + R, columns -1 .. W (zero outside the image)
  const float* xi = a.x + (long long)g * a.x_gstride + (long long)img * a.H * W * 3;
  for (int e = tid; e < RW; e += 256) {
    const int rr = e / ((W + 2) * 3), rem = e - rr * ((W + 2) * 3);
    const int cc = rem / 3, ci = rem - cc * 3;
    const int h = h0 + rr - 1, w = cc - 1;
    raw[e] = (h >= 0 && h < a.H && w >= 0 && w < W) ? xi[((long long)h * W + w) * 3 + ci] : 0.f;
  }
  // dy tile: 256 consecutive pixels x 32 channels, 16-B coalesced (lazy: formed from d, y)
  const long long base = (long long)g * a.d_gstride + ((long long)img * a.H + h0) * W * kCo;
  const float4* d4 = (const float4*)(a.d + base);
  const int q = tid & 7;                       // this thread's channel quad (constant: 256 % 8 == 0)
  if (a.coef) {
    const float* cf = a.coef + (long long)g * kBnRows * kCo;
    const float4 A = ((const float4*)(cf + kCA * kCo))[q], B = ((const float4*)(cf + kCB * kCo))[q];
    const float4 K = ((const float4*)(cf + kCK * kCo))[q];
    const float4* y4 = (const float4*)(a.y + base);
    float4 dv[8], yv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      dv[i] = d4[tid + 256 * i];
      yv[i] = y4[tid + 256 * i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float4 v;
      v.x = fmaf(A.x, dv[i].x, fmaf(B.x, yv[i].x, K.x));
      v.y = fmaf(A.y, dv[i].y, fmaf(B.y, yv[i].y, K.y));
      v.z = fmaf(A.z, dv[i].z, fmaf(B.z, yv[i].z, K.z));
      v.w = fmaf(A.w, dv[i].w, fmaf(B.w, yv[i].w, K.w));
      dys[tid + 256 * i] = v;
    }
  } else {
    float4 dv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) dv[i] = d4[tid + 256 * i];
#pragma unroll
    for (int i = 0; i < 8; ++i) dys[tid + 256 * i] = dv[i];
  }
  __syncthreads();
  // patch matrix row of pixel tid: k = (kh * 3 + kw) * 3 + ci
  {
    const int r = tid / W, c = tid - r * W;
    float pv[28];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int ci = 0; ci < 3; ++ci) pv[(kh * 3 + kw) * 3 + ci] = raw[((r + kh) * (W + 2) + c + kw) * 3 + ci];
    pv[27] = 0.f;
#pragma unroll
    for (int j = 0; j < 7; ++j) pat[tid * 7 + j] = make_float4(pv[4 * j], pv[4 * j + 1], pv[4 * j + 2], pv[4 * j + 3]);
  }
  __syncthreads();
  // row group rg sums pixels 64 rg .. 64 rg + 63; lane l owns channels 4 (l & 7).. x taps 4 (l >> 3)..
  const int rg = tid >> 6, l = tid & 63, coq = l & 7, kq = l >> 3;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  if (kq < 7) {
#pragma unroll 4
    for (int p = rg * 64; p < rg * 64 + 64; ++p) {
      const float4 dv = dys[p * 8 + coq], pv = pat[p * 7 + kq];
      const float dd[4] = {dv.x, dv.y, dv.z, dv.w}, xx[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(dd[i], xx[j], acc[i][j]);
    }
  }
  __syncthreads();                             // dys free: row-group partials [rg][l][16]
  float* red = (float*)dys;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) red[(rg * 64 + l) * 16 + i * 4 + j] = acc[i][j];
  __syncthreads();
  float* slab = a.ws + ((long long)z * G + g) * (kCo * kK);
  for (int e = tid; e < 64 * 16; e += 256) {
    const int ll = e >> 4, ij = e & 15;
    const int co = 4 * (ll & 7) + (ij >> 2), k = 4 * (ll >> 3) + (ij & 3);
    if (k >= kK) continue;
    const float v = ((red[e] + red[1024 + e]) + red[2048 + e]) + red[3072 + e];
    slab[co * kK + k] = v;
  }
}

template <int W>
int go(const XWSArgs& a, int G, hipStream_t st) {
  const int blocks = a.N * a.H * W / kPix;
  hipLaunchKernelGGL(xwgrad_stem_kernel<W>, dim3(blocks, G), dim3(256), 0, st, a);
  DBA_LAUNCH_CHECK();
}

}  // namespace

// slab floats of the stem weight gradient (slabs of 256 rows: mchunk = 256), 0 = shape not taken
DBA_EXPORT long long dba_xwgrad_stem_ws_floats(int G, int N, int H, int W, int Cin, int Cout) {
  if (Cin != 3 || Cout != kCo || (W != 32 && W != 64) || H % (kPix / W)) return 0;
  return (long long)N * H * W / kPix * G * (kCo * kK);
}

// dy [G][N][H][W][32] (or, coef != null, the finished BN output gradient d with the BN input y
// and its backward rows: dy = fma(A, d, fma(B, y, K))), x [G][N][H][W][3] -> slabs ws (reduced
// by dba_xwgrad_reduce_batch with mchunk 256, per = 32 * 27)
DBA_EXPORT int dba_xwgrad_stem(const float* d, long long d_gstride, const float* y, const float* coef, const float* x,
                               long long x_gstride, float* ws, const int* nvalid, int G, int N, int H, int W,
                               void* stream) {
  if (dba_xwgrad_stem_ws_floats(G, N, H, W, 3, kCo) == 0) return -100;
  if (((uintptr_t)d & 15) || (d_gstride & 3) || (coef && (((uintptr_t)y & 15) || ((uintptr_t)coef & 15)))) return -101;
  XWSArgs a{d, d_gstride, y, coef, x, x_gstride, ws, nvalid, N, H};
  hipStream_t st = (hipStream_t)stream;
  return W == 32 ? go<32>(a, G, st) : go<64>(a, G, st);
}
