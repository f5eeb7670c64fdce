// fp32 family, the fused training BN's standalone passes (bnfuse.hpp): the tile pass over a
// materialised tensor / split-K slabs / a pooled gradient, the stored block output (apply), the
// stored BN input gradient (dy).
#include "common.hpp"
#include "bnfuse.hpp"
#include <algorithm>

namespace {

// ===================================================== fused training BN: standalone pass
// A tile pass over a MATERIALISED tensor, for the producers whose epilogue cannot reduce: the
// split-K slabs of multi-replica launches (summed here in z order, xsplitk_reduce's order, plus
// the dgrad's accumulated branch), stride-s data gradients, the global average pool's gradient,
// max-pool gradients.  Same 128-row tiles of whole groups, same level-0 records
// (bnf_tile_records) and finalize launch as the conv epilogues, so the statistics are the same bits whichever
// kernel produced them.  mode 1: statistics of the value (stored to dst
// when dst is given); mode 2: d = mask(value) -> dst (may alias src).  value = src, or the sum of
// S slabs ws[z] (+ accum), or pool[g][img][c] * pool_scale (elementwise.hip avgpool_bwd's value).
__global__ __launch_bounds__(256) void bnx_tile_kernel(const BnFuse f, const float* src, float* dst,
                                                       long long gstride, const int* __restrict__ nvalid, int N,
                                                       int HW, const float* __restrict__ pool, float pool_scale,
                                                       const float* __restrict__ ws, int S, long long zstride,
                                                       const float* __restrict__ accum) {
  constexpr int BM = 128, BN = 64, C4 = BN / 4;
  __shared__ __attribute__((aligned(16))) float Ct[BM * BN];
  __shared__ long long orow[BM];
  const int g = blockIdx.y, tid = threadIdx.x, C = f.C;
  const int tiles_n = ceil_div_d(C, BN);
  const int tn = blockIdx.x % tiles_n, tm = blockIdx.x / tiles_n;
  const int Mv = valid_rows(nvalid, g, N) * HW;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mv) return;
  if (tid < BM) orow[tid] = m0 + tid < Mv ? (long long)(m0 + tid) * C : -1;
  __syncthreads();
  const long long base = (long long)g * gstride;
  for (int e = tid; e < BM * C4; e += 256) {
    const int row = e / C4, cc = (e - row * C4) * 4, n = n0 + cc;
    const long long o = orow[row];
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (o >= 0 && n < C) {
      if (ws) {
        v = *(const float4*)(ws + base + o + n);
        for (int z = 1; z < S; ++z) {
          const float4 u = *(const float4*)(ws + z * zstride + base + o + n);
          v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
        }
      } else if (pool) {
        const float4 u = *(const float4*)(pool + ((long long)g * N + (m0 + row) / HW) * C + n);
        v = make_float4(u.x * pool_scale, u.y * pool_scale, u.z * pool_scale, u.w * pool_scale);
      } else {
        v = *(const float4*)(src + base + o + n);
      }
      if (accum) {
        const float4 r = *(const float4*)(accum + base + o + n);
        v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
      }
      if (f.mode == 2) v = bnf_mask4(f, g, o, n, v);
      if (dst) *(float4*)(dst + base + o + n) = v;
    }
    *(float4*)&Ct[row * BN + cc] = v;
  }
  __syncthreads();
  bnf_tile_records<BM, BN>(f, Ct, orow, g, m0, n0, Mv);
}

// The materialised output of a training BN (+ residual) (+ ReLU) (bnfuse.hpp): out =
// relu?(fma(ya, scale_a, shift_a) + r), r = res (identity shortcut) or fma(yb, scale_b, shift_b)
// (a shortcut conv's BN; relu_b: a lazy BN+ReLU output, e.g. the stem's) or 0 — bn.hip
// bn_apply's arithmetic; folds max |out| for the fp16-pair operand scale of its consumers.
// Valid rows only.
__global__ __launch_bounds__(256) void bnx_apply_kernel(const float* __restrict__ ya, const float* __restrict__ ca,
                                                        const float* __restrict__ res, const float* __restrict__ yb,
                                                        const float* __restrict__ cb, int relu_b, int relu,
                                                        float* __restrict__ out,
                                                        long long gstride, const int* __restrict__ nvalid, int N,
                                                        int HW, int C, int* __restrict__ amax, int amax_ld) {
  const int g = blockIdx.y;
  const int C4 = C >> 2;
  const long long total = (long long)valid_rows(nvalid, g, N) * HW * C4;
  const long long base = (long long)g * gstride;
  const float* cag = ca + (long long)g * kBnRows * C;
  const float* cbg = cb ? cb + (long long)g * kBnRows * C : nullptr;
  float vmax = 0.f;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int c = (int)(t % C4) * 4;
    const long long o = base + t * 4;
    const float4 y = *(const float4*)(ya + o);
    const float4 sc = *(const float4*)(cag + kCScale * C + c), sh = *(const float4*)(cag + kCShift * C + c);
    float4 v = make_float4(fmaf(y.x, sc.x, sh.x), fmaf(y.y, sc.y, sh.y), fmaf(y.z, sc.z, sh.z), fmaf(y.w, sc.w, sh.w));
    if (res) {
      const float4 r = *(const float4*)(res + o);
      v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
    } else if (yb) {
      const float4 u = *(const float4*)(yb + o);
      const float4 sb = *(const float4*)(cbg + kCScale * C + c), hb = *(const float4*)(cbg + kCShift * C + c);
      float4 b = make_float4(fmaf(u.x, sb.x, hb.x), fmaf(u.y, sb.y, hb.y), fmaf(u.z, sb.z, hb.z), fmaf(u.w, sb.w, hb.w));
      if (relu_b) { b.x = fmaxf(b.x, 0.f); b.y = fmaxf(b.y, 0.f); b.z = fmaxf(b.z, 0.f); b.w = fmaxf(b.w, 0.f); }
      v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
    }
    if (relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
    vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    *(float4*)(out + o) = v;
  }
  if (amax) amax_fold(amax, amax_ld, g, vmax);
}

// The input gradient of a training BN, stored: dy = fma(A, d, fma(B, y, K)) per channel
// (bnfuse.hpp; bn.hip bn_bwd_apply's arithmetic) over the valid rows, and the max |dy| slot
// folded for its fp16-pair consumers (measured faster than the weight gradient staging dy
// from (d, y) on the fly: profiles/r4/bnx/ab_steps.md).
__global__ __launch_bounds__(256) void bnx_dy_kernel(const float* __restrict__ d, const float* __restrict__ y,
                                                     const float* __restrict__ coef, float* __restrict__ dy,
                                                     long long gstride, const int* __restrict__ nvalid, int N, int HW,
                                                     int C, int* __restrict__ amax, int amax_ld) {
  const int g = blockIdx.y;
  const int C4 = C >> 2;
  const long long total = (long long)valid_rows(nvalid, g, N) * HW * C4;
  const long long base = (long long)g * gstride;
  const float* cf = coef + (long long)g * kBnRows * C;
  float vmax = 0.f;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int c = (int)(t % C4) * 4;
    const long long o = base + t * 4;
    const float4 dv = *(const float4*)(d + o), yv = *(const float4*)(y + o);
    const float4 A = *(const float4*)(cf + kCA * C + c), B = *(const float4*)(cf + kCB * C + c),
                 K = *(const float4*)(cf + kCK * C + c);
    const float4 v = make_float4(fmaf(A.x, dv.x, fmaf(B.x, yv.x, K.x)), fmaf(A.y, dv.y, fmaf(B.y, yv.y, K.y)),
                                 fmaf(A.z, dv.z, fmaf(B.z, yv.z, K.z)), fmaf(A.w, dv.w, fmaf(B.w, yv.w, K.w)));
    vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    *(float4*)(dy + o) = v;
  }
  if (amax) amax_fold(amax, amax_ld, g, vmax);
}

}  // namespace

namespace xg {
int bnx_tile_go(const BnFuse& f, const float* src, float* dst, long long gstride, const int* nvalid, int G, int N,
                int HW, const float* pool, float pool_scale, const float* ws, int S, long long zstride,
                const float* accum, hipStream_t st) {
  if (f.C & 3) return -102;
  const dim3 grid((unsigned)(ceil_div((long long)N * HW, 128) * ceil_div(f.C, 64)), G);
  hipLaunchKernelGGL(bnx_tile_kernel, grid, dim3(256), 0, st, f, src, dst, gstride, nvalid, N, HW, pool, pool_scale, ws,
                     S, zstride, accum);
  const int rc = (int)hipGetLastError();
  return rc != 0 ? rc : bnx_finalize_go(f, nvalid, G, N, HW, st);   // the pass's BN finalize
}
}  // namespace xg
using xg::bnx_tile_go;

DBA_EXPORT int dba_bnx_rows(const void* bnf, const float* src, float* dst, long long gstride, const int* nvalid, int G,
                            int N, int HW, const float* pool, float pool_scale, void* stream) {
  const BnFuse f = *(const BnFuse*)bnf;
  if (f.mode < 1 || f.mode > 2 || (f.mode == 2 && (!dst || !f.ya))) return -108;
  return bnx_tile_go(f, src, dst, gstride, nvalid, G, N, HW, pool, pool_scale, nullptr, 1, 0, nullptr,
                     (hipStream_t)stream);
}

// sizeof(BnFuse) (the Python ctypes mirror checks its layout against it)

DBA_EXPORT int dba_bnfuse_size() { return (int)sizeof(BnFuse); }

DBA_EXPORT int dba_bnx_apply(const float* ya, const float* ca, const float* res, const float* yb, const float* cb,
                             int relu_b, int relu, float* out, long long gstride, const int* nvalid, int G, int N, int HW, int C,
                             int* amax, int amax_ld, void* stream) {
  if (C & 3) return -102;
  const long long per = (long long)N * HW * (C / 4);
  const long long cap = std::max(1LL, 8192LL / std::max(1, G));
  const dim3 grid((unsigned)std::max(1LL, std::min(cap, (per + 255) / 256)), G);
  hipLaunchKernelGGL(bnx_apply_kernel, grid, dim3(256), 0, (hipStream_t)stream, ya, ca, res, yb, cb, relu_b, relu, out,
                     gstride,
                     nvalid, N, HW, C, amax, amax_ld);
  DBA_LAUNCH_CHECK();
}

DBA_EXPORT int dba_bnx_dy(const float* d, const float* y, const float* coef, float* dy, long long gstride,
                          const int* nvalid, int G, int N, int HW, int C, int* amax, int amax_ld, void* stream) {
  if (C & 3) return -102;
  const long long per = (long long)N * HW * (C / 4);
  const long long cap = std::max(1LL, 8192LL / std::max(1, G));
  const dim3 grid((unsigned)std::max(1LL, std::min(cap, (per + 255) / 256)), G);
  hipLaunchKernelGGL(bnx_dy_kernel, grid, dim3(256), 0, (hipStream_t)stream, d, y, coef, dy, gstride, nvalid, N, HW, C,
                     amax, amax_ld);
  DBA_LAUNCH_CHECK();
}
