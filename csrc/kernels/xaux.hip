// fp32 family, operand helpers: fp16-pair weight planes split once per fold / step (single and
// batched), and the operand max |x| slots (segment and per-replica forms).
#include "common.hpp"
#include "xmfma.hpp"
#include <algorithm>

namespace {

// w [slots][per] fp32 (slot stride sstride) -> planes [slots][2][per] fp16 of w * 2^sb, sb from
// the slot's max |w| exactly as HScale computes it: a weight operand split once for all the
// blocks (and launches) that stage it
__device__ __forceinline__ void xsplit_w_body(const float* __restrict__ w, long long sstride, long long per,
                                              const int* __restrict__ amax, int ld, uint16_t* __restrict__ out,
                                              int sl, long long e0, long long e1, long long step) {
  const int sb = hexp(amax_read(amax, ld, sl));
  const float mb = __uint_as_float((uint32_t)(sb + 127) << 23);
  const float* __restrict__ src = w + (long long)sl * sstride;
  uint16_t* __restrict__ oh = out + (long long)sl * 2 * per;
  uint16_t* __restrict__ ol = oh + per;
  for (long long e = e0 + threadIdx.x * 4LL; e < e1; e += step) {
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = e + i < per ? src[e + i] : 0.f;
    uint2 sp[2];
    split4h(v[0], v[1], v[2], v[3], mb, sp);
    const uint16_t* h = (const uint16_t*)&sp[0];
    const uint16_t* l = (const uint16_t*)&sp[1];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (e + i < per) { oh[e + i] = h[i]; ol[e + i] = l[i]; }
  }
}
__global__ __launch_bounds__(256) void xsplit_w_kernel(const float* __restrict__ w, long long sstride, long long per,
                                                       const int* __restrict__ amax, int ld,
                                                       uint16_t* __restrict__ out) {
  xsplit_w_body(w, sstride, per, amax, ld, out, blockIdx.y, blockIdx.x * 1024LL, per, (long long)gridDim.x * 1024);
}
// a whole model fold's weight splits in one launch (blockIdx.y = slot): the x grid is the
// concatenation of every weight's chunks of kXSChunk elements (desc i owns blocks [boff_i,
// boff_{i+1})); a max-sized grid per desc left most blocks of the small convs idle
struct XSDesc {   // all int64 (built from a torch int64 host tensor)
  long long w, sstride, per, amax, ld, out, boff;
};
constexpr int kXSBatch = 24, kXSChunk = 4096;
struct XSBatch {
  XSDesc d[kXSBatch];
  int n;
};
__global__ __launch_bounds__(256) void xsplit_w_batch_kernel(const XSBatch b) {
  int i = 0;
  while (i + 1 < b.n && (long long)blockIdx.x >= b.d[i + 1].boff) ++i;
  const XSDesc& d = b.d[i];
  const long long e0 = ((long long)blockIdx.x - d.boff) * kXSChunk;
  const long long e1 = e0 + kXSChunk < d.per ? e0 + kXSChunk : d.per;
  xsplit_w_body((const float*)d.w, d.sstride, d.per, (const int*)d.amax, (int)d.ld, (uint16_t*)d.out, blockIdx.y, e0,
                e1, 1024);
}

// max |x| of n segments (offset, length) of every replica's flat row (the conv weights of a
// model replica: one launch per training step instead of one per conv); out[s][g]
// One block per 4096-element chunk of a segment (the segments' chunks laid end to end: block c
// belongs to the segment whose chunk range holds c), four 16-B loads per thread in flight; a
// 2-D grid of (64 chunks x segments) blocks left most of them idle on the small segments and
// read scalars.  The max is order-free (exact integer fold), so the tiling is free.
constexpr int kAmaxSegs = 64, kAmaxChunk = 4096;
struct AmaxSegs {
  long long off[kAmaxSegs];
  int len[kAmaxSegs];
  int start[kAmaxSegs + 1];   // first chunk of each segment (prefix sum of ceil(len / 4096))
  int n;
};
__global__ __launch_bounds__(256) void amax_segments_kernel(const float* __restrict__ base, long long gstride,
                                                            const AmaxSegs segs, int ld, int* __restrict__ out) {
  const int c = blockIdx.x, g = blockIdx.y;
  int sg = 0;
  while (sg + 1 < segs.n && segs.start[sg + 1] <= c) ++sg;
  const float* __restrict__ p = base + (long long)g * gstride + segs.off[sg];
  const int n = segs.len[sg], e0 = (c - segs.start[sg]) * kAmaxChunk;
  const bool v4 = ((segs.off[sg] | gstride) & 3) == 0 && ((uintptr_t)base & 15) == 0;
  float m = 0.f;
  float4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = e0 + (k * 256 + threadIdx.x) * 4;
    if (v4 && e + 3 < n) {
      v[k] = *(const float4*)(p + e);
    } else {
      v[k].x = e < n ? p[e] : 0.f;
      v[k].y = e + 1 < n ? p[e + 1] : 0.f;
      v[k].z = e + 2 < n ? p[e + 2] : 0.f;
      v[k].w = e + 3 < n ? p[e + 3] : 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) m = fmaxf(m, fmaxf(fmaxf(fabsf(v[k].x), fabsf(v[k].y)), fmaxf(fabsf(v[k].z), fabsf(v[k].w))));
  amax_fold(out + (long long)sg * kAmaxSub * ld, ld, g, m);
}

// max |x| of each replica's valid prefix (nvalid[g] * per_item elements, or n_per_g), as the
// float's bit pattern: the fp16-pair scale source (HScale).  Integer atomicMax of non-negative
// float bits: exact and order-independent (deterministic); out is zeroed by the launcher.
__global__ __launch_bounds__(256) void amax_kernel(const float* __restrict__ x, long long gstride, long long n_per_g,
                                                   const int* __restrict__ nvalid, long long per_item, int vec,
                                                   int* __restrict__ out, int ld) {
  const int g = blockIdx.y;
  const long long n = nvalid ? (long long)nvalid[g] * per_item : n_per_g;
  const float* __restrict__ p = x + (long long)g * gstride;
  float m = 0.f;
  if (vec) {
    const long long n4 = n >> 2;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n4; e += (long long)gridDim.x * 256) {
      const float4 v = ((const float4*)p)[e];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    for (long long e = n4 * 4 + blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256)
      m = fmaxf(m, fabsf(p[e]));
  } else {
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) m = fmaxf(m, fabsf(p[e]));
  }
  amax_fold(out, ld, g, m);
}

}  // namespace

DBA_EXPORT int dba_xsplit_w(const float* w, long long sstride, long long per, int slots, const int* amax, int ld,
                            uint16_t* out, void* stream) {
  const dim3 grid((unsigned)std::max(1LL, std::min(1024LL, (per + 1023) / 1024)), slots);
  hipLaunchKernelGGL(xsplit_w_kernel, grid, dim3(256), 0, (hipStream_t)stream, w, sstride, per, amax, ld, out);
  DBA_LAUNCH_CHECK();
}

// the fp16-pair planes of n weight operands (one model fold) in one launch per 24; desc: n x XSDesc
// in HOST memory (passed by value), every operand with `slots` slots

DBA_EXPORT int dba_xsplit_w_batch(const void* desc, int n, int slots, void* stream) {
  const XSDesc* ds = (const XSDesc*)desc;
  for (int i0 = 0; i0 < n; i0 += kXSBatch) {
    XSBatch b{};
    b.n = std::min(kXSBatch, n - i0);
    long long nb = 0;
    for (int i = 0; i < b.n; ++i) {
      b.d[i] = ds[i0 + i];
      b.d[i].boff = nb;
      nb += (b.d[i].per + kXSChunk - 1) / kXSChunk;
    }
    hipLaunchKernelGGL(xsplit_w_batch_kernel, dim3((unsigned)nb, slots), dim3(256), 0, (hipStream_t)stream, b);
    const int rc = (int)hipGetLastError();
    if (rc != 0) return rc;
  }
  return 0;
}

// out: n zeroed amax slots [n][kAmaxSub][ld] (common.hpp): max |x| of segment s of replica g;
// segs: n x (offset, length) int64 pairs in HOST memory (passed by value: safe under graph
// capture), n <= 64

DBA_EXPORT int dba_amax_segments(const float* base, long long gstride, const long long* segs, int n, int G, int* out,
                                 int ld, void* stream) {
  if (n > kAmaxSegs || n < 1) return -105;
  AmaxSegs a{};
  a.n = n;
  for (int i = 0; i < n; ++i) {
    a.off[i] = segs[2 * i];
    a.len[i] = (int)segs[2 * i + 1];
    a.start[i + 1] = a.start[i] + std::max(1, ceil_div(a.len[i], kAmaxChunk));
  }
  const dim3 grid((unsigned)a.start[n], G);
  hipLaunchKernelGGL(amax_segments_kernel, grid, dim3(256), 0, (hipStream_t)stream, base, gstride, a, ld, out);
  DBA_LAUNCH_CHECK();
}

// folds max |x| over replica g's valid prefix into the zeroed slot out [kAmaxSub][ld]

DBA_EXPORT int dba_amax(const float* x, long long gstride, long long n_per_g, const int* nvalid, long long per_item,
                        int G, int* out, int ld, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int vec = aligned16(x) && gstride % 4 == 0;
  const long long per = nvalid ? per_item * (n_per_g / std::max(1LL, per_item)) : n_per_g;
  const dim3 grid((unsigned)std::max(1LL, std::min(256LL, (per + 4095) / 4096)), G);
  hipLaunchKernelGGL(amax_kernel, grid, dim3(256), 0, st, x, gstride, n_per_g, nvalid, per_item, vec, out, ld);
  DBA_LAUNCH_CHECK();
}

// part: [G][ceil(N * rows_per_img / 256)][C] fp64 workspace (dba_xcolsum_part_doubles)
