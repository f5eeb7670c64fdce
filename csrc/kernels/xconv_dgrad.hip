// fp32 family, data-gradient pass (xconv.hpp): stride-s gradients as parity classes of the
// implicit GEMM, the halo-tiled stride-1 gradient, the fused BN mask + statistics of the
// gradient, and the class-packed transposed weights (one launch per backward pass).
#include "xhalo.hpp"

namespace {

// ====================================================================== dgrad weights
// wt[slot][class (ph,pw)][cin][i][j][cout] = w[slot][cout][kh0+i*s][kw0+j*s][cin]
// (kh0 = (ph + pad) % s): every tap belongs to exactly one parity class.
struct XTDesc {   // all int64 (built from a torch int64 host tensor)
  long long w, wt, w_sstride, Cout, KH, KW, Cin, stride, pad, unused;
};
constexpr int kXTBatch = 24;   // descriptors per launch, passed by value (graph-capture safe)
struct XTBatch {
  XTDesc d[kXTBatch];
};

// One 32 x 32 (cout x cin) tile of one tap per block iteration, transposed through LDS:
// coalesced reads along cin, coalesced writes along cout (the element-wise gather it replaces
// read every weight from a different cache line).  blockIdx.z = slot.
__global__ __launch_bounds__(256) void xtranspose_kernel(const XTBatch b, int slots, const int* __restrict__ nvalid) {
  __shared__ float tile[32][33];
  const XTDesc& d = b.d[blockIdx.y];
  const int s = (int)d.stride, KH = (int)d.KH, KW = (int)d.KW, Cin = (int)d.Cin, Cout = (int)d.Cout;
  const int pad = (int)d.pad;
  const int sl = blockIdx.z;
  if (nvalid && nvalid[sl] == 0) return;
  const int per = Cout * KH * KW * Cin;
  const float* __restrict__ w = (const float*)d.w + (long long)sl * d.w_sstride;
  float* __restrict__ wt = (float*)d.wt + (long long)sl * per;
  const int nco = (Cout + 31) >> 5, nci = (Cin + 31) >> 5;
  const int ntiles = KH * KW * nco * nci;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int tap = t / (nco * nci), rr = t - tap * nco * nci;
    const int cot = rr / nci, cit = rr - cot * nci;
    const int kh = tap / KW, kw = tap - kh * KW;
    // the tap's parity class (ph, pw): kh0 = (ph + pad) % s == kh % s
    const int kh0 = kh % s, kw0 = kw % s;
    const int ph = ((kh0 - pad) % s + s) % s, pw = ((kw0 - pad) % s + s) % s;
    const int cls = ph * s + pw;
    int base = 0, nI = 0, nJ = 0;
    for (int c = 0; c <= cls; ++c) {
      const int a = c / s, bb = c - a * s;
      const int h0 = (a + pad) % s, w0 = (bb + pad) % s;
      nI = h0 < KH ? (KH - h0 + s - 1) / s : 0;
      nJ = w0 < KW ? (KW - w0 + s - 1) / s : 0;
      if (c < cls) base += Cin * nI * nJ * Cout;
    }
    const int i = (kh - kh0) / s, j = (kw - kw0) / s;
#pragma unroll
    for (int k = ty; k < 32; k += 8) {
      const int co = cot * 32 + k, ci = cit * 32 + tx;
      tile[k][tx] = (co < Cout && ci < Cin) ? w[((co * KH + kh) * KW + kw) * Cin + ci] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int k = ty; k < 32; k += 8) {
      const int ci = cit * 32 + k, co = cot * 32 + tx;
      if (ci < Cin && co < Cout) wt[base + ((ci * nI + i) * nJ + j) * Cout + co] = tile[tx][k];
    }
    __syncthreads();
  }
}

struct ClassGeom {
  int n;
  XClass c[4];
};

// parity classes of a stride-s data gradient (see xtranspose_kernel for the weight order)
ClassGeom dgrad_classes(int H, int W, int Cin, int Cout, int KH, int KW, int s, int pad) {
  ClassGeom cg{};
  cg.n = s * s;
  long long off = 0;
  for (int ci = 0; ci < s * s; ++ci) {
    const int ph = ci / s, pw = ci - ph * s;
    const int kh0 = (ph + pad) % s, kw0 = (pw + pad) % s;
    XClass& c = cg.c[ci];
    c.nI = kh0 < KH ? (KH - kh0 + s - 1) / s : 0;
    c.nJ = kw0 < KW ? (KW - kw0 + s - 1) / s : 0;
    c.bh = (ph + pad - kh0) / s;
    c.bw = (pw + pad - kw0) / s;
    c.oh = ph;
    c.ow = pw;
    c.Hq = ph < H ? (H - ph + s - 1) / s : 0;
    c.Wq = pw < W ? (W - pw + s - 1) / s : 0;
    c.boff = off;
    off += (long long)Cin * c.nI * c.nJ * Cout;
  }
  return cg;
}

}  // namespace

DBA_EXPORT int dba_xconv_dgrad(const float* dy, long long dy_gstride, const float* wt, long long wt_sstride,
                               const int* wsel, const float* accum, float* dx, long long dx_gstride,
                               const int* nvalid, int G, int N, int H, int W, int Cin, int Ho, int Wo, int Cout,
                               int KH, int KW, int stride, int pad, const int* amax_dy, int amax_dy_ld,
                               const int* amax_w, int amax_w_ld, const uint16_t* wp, long long wp_sstride, float* ws,
                               long long ws_floats, int* sk_cnt, long long sk_cnt_n, const void* bnf, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if ((long long)N * Ho * Wo * Cout >= (1LL << 29)) return -103;   // 32-bit in-replica byte offsets
  const ClassGeom cg = dgrad_classes(H, W, Cin, Cout, KH, KW, stride, pad);
  const int vec = (Cout % 4 == 0 && aligned16(dy) && aligned16(wt) && dy_gstride % 4 == 0 && wt_sstride % 4 == 0) ? 4 : 1;
  XArgs a{};
  a.src = dy; a.src_gstride = dy_gstride; a.w = wt; a.w_sstride = wt_sstride; a.wsel = wsel;
  a.bias = nullptr; a.b_sstride = 0; a.res = accum; a.out = dx; a.out_gstride = dx_gstride;
  a.nvalid = nvalid; a.N = N; a.Hs = Ho; a.Ws = Wo; a.Cs = Cout; a.Ncol = Cin; a.Ho = H; a.Wo = W;
  a.sp = 1; a.os = stride; a.dsg = -1; a.relu = 0; a.splitk = 1;
  a.amax_src = amax_dy; a.amax_w = amax_w;
  a.amax_src_ld = amax_dy_ld; a.amax_w_ld = amax_w_ld;
  a.wp = wp; a.wp_sstride = wp_sstride;
  if (bnf) {   // the backward BN mask + reduce of the gradient (stride-1 data gradients: one class)
    a.bf = *(const BnFuse*)bnf;
    if (a.bf.mode != 2 || stride != 1 || (Cin & 3) || a.bf.C != Cin) return -108;
  }
  long long Mmax = 0;
  for (int i = 0; i < cg.n; ++i) {
    a.cls[i] = cg.c[i];
    Mmax = std::max(Mmax, (long long)N * cg.c[i].Hq * cg.c[i].Wq);
  }
  auto fin = [&](int rc) { return (rc == 0 && a.bf.mode) ? bnx_finalize_go(a.bf, nvalid, G, N, H * W, st) : rc; };
  if (stride == 1) {
    const int rc = xhalo_try(a, G, KH, KW, st);
    if (rc != -100) return fin(rc);
    const long long M = (long long)N * H * W;
    const int s = xsplitk(M, G, Cin, KH * KW * Cout);
    const bool ws_ok = s > 1 && ws != nullptr && ws_floats >= (long long)s * G * M * Cin;
    if (ws_ok && sk_ok(sk_cnt, sk_cnt_n, M, Cin, G, 1, s)) {
      XArgs b = a;
      b.splitk = s;
      b.zstride = (long long)G * M * Cin;
      b.sk_ws = ws; b.sk_gstride = M * Cin; b.sk_cnt = sk_cnt;
      return fin(xconv_dispatch(b, M, G, 1, vec, st));
    }
    if (s > 1 && split_policy().dgrad_ks) {
      // grouped launch: the slabs summed inside each block in z order, then the accumulated
      // input and the BN mask / records in the epilogue — the lone client's in-launch combine
      // arithmetic (sk_combine), without the slab round trip and the standalone BN pass
      XArgs b = a;
      b.kslab = s;
      const int rc = xconv_ks(b, M, G, vec, st);
      if (rc != -100) return fin(rc);
    }
    if (ws_ok) {
      XArgs b = a;
      b.splitk = s;
      b.out = ws;
      b.out_gstride = M * Cin;
      b.zstride = (long long)G * M * Cin;
      const int rc = xconv_dispatch(b, M, G, 1, vec, st);
      if (rc != 0) return rc;
      if (a.bf.mode)   // slabs + accum summed, masked and reduced in one pass (bnfuse.hpp)
        return bnx_tile_go(a.bf, nullptr, dx, dx_gstride, nvalid, G, N, H * W, nullptr, 0.f, ws, s, b.zstride, accum,
                           st);
      const long long per = M * Cin;
      const dim3 grid((unsigned)std::max(1LL, std::min(1024LL, (per + 255) / 256)), G);
      hipLaunchKernelGGL(xsplitk_reduce_kernel, grid, dim3(256), 0, st, (const float*)ws, s, b.zstride, per, nvalid,
                         N, H * W, Cin, nullptr, 0LL, wsel, accum, 0, dx, (int*)nullptr, 0);
      DBA_LAUNCH_CHECK();
    }
  }
  return fin(xconv_dispatch(a, Mmax, G, cg.n, vec, st));
}

// class-packed data-gradient weights for n convs.  desc: n x XTDesc in HOST memory, read
// here and passed to the kernel by value (safe under HIP graph capture); nvalid (optional,
// slots == replicas) skips inactive slots.

DBA_EXPORT int dba_xtranspose(const void* desc, int n, int slots, long long max_per, const int* nvalid,
                              void* stream) {
  const XTDesc* ds = (const XTDesc*)desc;
  for (int i0 = 0; i0 < n; i0 += kXTBatch) {
    XTBatch b{};
    const int m = std::min(kXTBatch, n - i0);
    for (int i = 0; i < m; ++i) b.d[i] = ds[i0 + i];
    const dim3 grid((unsigned)std::max(1LL, std::min(1024LL, (max_per + 1023) / 1024)), m, slots);
    hipLaunchKernelGGL(xtranspose_kernel, grid, dim3(256), 0, (hipStream_t)stream, b, slots, nvalid);
    const int rc = (int)hipGetLastError();
    if (rc != 0) return rc;
  }
  return 0;
}

// slab floats dba_xwgrad needs for this shape (0: accumulates straight into dw)
// The m-chunking (Z slabs) is decided from the PER-REPLICA geometry only (see xsplitk): ~256
// blocks per replica (a lone client fills the chip), chunks of >= 256 rows.
