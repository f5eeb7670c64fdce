// Training BatchNorm fused into the conv kernels (gfx950): the statistics of a conv output are
// reduced by the kernel that produces it, and the normalisation is applied by the kernels that
// CONSUME it, so a conv-BN-ReLU costs no launch of its own.
//
// Reference semantics: BatchNorm2d in train mode followed by ReLU / a residual add
// (/root/reference/models/resnet_cifar.py:31-36, driven by image_train.py:84-102): biased
// variance to normalise, unbiased variance into the running statistics (momentum 0.1).
//
// Forward.  The producing conv's epilogue (xconv.hpp xconv_kernel / xhalo.hpp xhalo_kernel, stem.hip) reduces each
// 32-row group of its tile of the raw output y, per channel, in fp64 in row order:
//     {sum y, sum y^2, max y, min y}
// converts the two sums to EXACT INTEGERS on a fixed 2^-80 grid (three int64 limbs, bnf_limbs),
// adds its groups' limbs and agent-scope atomically adds them into the BN's accumulator record
// (one of nsub spread copies per channel; max / min as atomic maxima of non-negative float bits).
// Integer addition is exact and associative, so the accumulated sums — and everything derived
// from them — have the same bits in any tile order, tile shape and replica grouping.  The
// coefficients (mean, 1/std, the running-stat update, scale = gamma/std, shift = beta - mean *
// scale, a bound of the BN (+ReLU) output's max |.| for the fp16-pair operand scale of its
// consumers) are derived from the record by ITS FIRST CONSUMER (bnf_coef_fwd): the consuming conv
// or apply pass computes them in its prologue and one designated block per replica writes the
// coefficient rows / running statistics / bound the later kernels read — no launch of their own.
// (bnx_finalize_kernel remains for consumers that are not record-aware.)  The output itself is
// never stored when its only consumers are convs: their staging computes relu(fma(y, scale,
// shift)) per element.
//
// Backward.  The data gradient g of a BN(+ReLU) output comes from a dgrad whose epilogue masks
// it (d = g where the output is > 0), stores d, and accumulates the same way
//     {sum d, sum d*xhat_a, sum d*xhat_b, max |d|}     (xhat = (y - mean) * invstd, fp32)
// for the BN a of the output and, when the output is a residual sum of two BNs (a shortcut
// conv), the BN b of the other branch; the record's consumer (bnx_dy_kernel / the stem's weight
// gradient) accumulates dbeta += sum d, dgamma += sum d*xhat once per replica and applies the
// affine form of the BN input gradient
//     dy = fma(A, d, fma(B, y, K)),  A = gamma*invstd, B = -A*invstd*sum(d*xhat)/n,
//     K = -A*sum(d)/n - B*mean
// (bn.hip's formulas), with a bound of max |dy| for its fp16-pair scale.
//
// (Rounds 3-5 kept fp64 level-0 records per 32-row group, summed by a finalize launch per BN
// in a fixed pairwise tree: 37 of a lone client's 144 launches per training step.  An in-kernel
// ticket finalisation of those records was measured first: its serial tail after the last tile
// cost 12-20 us per conv.)
#pragma once
#include "common.hpp"

__host__ __device__ __forceinline__ int ceil_div_d(int a, int b) { return (a + b - 1) / b; }

constexpr int kBnGrp = 32;                 // rows per level-0 group
// per-BN coefficient rows [G][kBnRows][C] (fp32)
enum { kCMean = 0, kCInv, kCScale, kCShift, kCYmax, kCYmin, kCA, kCB, kCK, kBnRows };

// accumulator record: int64 slots per (replica, channel, spread copy)
constexpr int kAccF = 8;    // forward: sum y (3 limbs), sum y^2 (3 limbs), bits max(y, 0), bits max(-y, 0)
constexpr int kAccB = 10;   // backward: sum d, sum d*xhat_a, sum d*xhat_b (3 limbs each), bits max |d|
constexpr unsigned long long kAccPoison = 0x7fc00000ull;   // a NaN's bits in a max slot: a non-finite
                                                           // or out-of-grid group poisons the BN

struct BnFuse {
  int mode;                 // 0 none, 1 forward statistics of the output, 2 backward (mask + reduce)
  int C;                    // channels of the output (= the conv's Ncol)
  int nsub;                 // spread copies of each channel's record (atomic contention)
  long long* acc;           // [G][C][nsub][kAccF | kAccB] zeroed int64 accumulators
  // BN a: forward — the BN of this output; backward — the BN whose output's gradient this is
  float* coef_a;            // [G][kBnRows][C]
  const float* gamma_a; const float* beta_a; float* rm_a; float* rv_a;
  long long p_gstride;      // replica stride of gamma / beta / running stats (flat state rows)
  float momentum, eps;
  int relu;                 // forward: the lazy output has a ReLU (its bound)
  int* amax_a; int amax_ld; // forward: bound slot of the lazy output; backward: of dy_a
  // backward only
  const float* ya; const float* yb; long long y_gstride;   // pre-BN values of BN a / b
  float* coef_b; const float* gamma_b; int* amax_b;
  float* dgamma_a; float* dbeta_a; float* dgamma_b; float* dbeta_b; long long gr_gstride;
  const float* mask_out;    // d = g where mask_out > 0 (the materialised BN output), else
  int mask_lazy;            //   where fma(ya, scale_a, shift_a) > 0 (mask_lazy), else d = g
  int which;                // finalising a backward record: 0 BN a, 1 BN b (its pointers then in the a fields)
};

__device__ __forceinline__ int bnf_kacc(int mode) { return mode == 1 ? kAccF : kAccB; }

// v = h + m 2^-40 + l 2^-80 (+ < 2^-80), 0 <= m, l < 2^40: an fp64 group sum on the fixed grid;
// false (poison) when |v| >= 2^40 or v is not finite
__device__ __forceinline__ bool bnf_limbs(double v, long long* out) {
  if (!(fabs(v) < 0x1p40)) return false;
  const double fh = floor(v);
  const double r = (v - fh) * 0x1p40;
  const double fm = floor(r);
  out[0] = (long long)fh;
  out[1] = (long long)fm;
  out[2] = (long long)floor((r - fm) * 0x1p40);
  return true;
}
__device__ __forceinline__ double bnf_unlimb(const long long* s) {
  return __dadd_rn(__dadd_rn((double)s[0], __dmul_rn((double)s[1], 0x1p-40)), __dmul_rn((double)s[2], 0x1p-80));
}
__device__ __forceinline__ unsigned long long bnf_fbits(float v) {   // v >= 0 or NaN
  return v != v ? kAccPoison : (unsigned long long)__float_as_uint(v);
}

// a channel's record reduced over its nsub spread copies by tpc consecutive lanes (tpc a power
// of two; lane `part` of the group takes copies part, part + tpc, ..., then an xor butterfly over
// the group): exact integer sums s[0..nl) and maxima s[nl..ka), the same value in every lane of
// the group.  EVERY lane of the wave calls it (the butterfly); `live` lanes read.
__device__ __forceinline__ void bnf_gather(const BnFuse& f, int g, int c, int part, int tpc, bool live,
                                           long long (&s)[kAccB]) {
  const int ka = bnf_kacc(f.mode), nl = f.mode == 1 ? 6 : 9;
#pragma unroll
  for (int k = 0; k < kAccB; ++k) s[k] = 0;
  if (live) {
    const long long* rec = f.acc + ((long long)g * f.C + c) * f.nsub * ka;
    for (int u = part; u < f.nsub; u += tpc) {
      const long long* r = rec + (long long)u * ka;
      for (int k = 0; k < nl; ++k) s[k] += r[k];
      for (int k = nl; k < ka; ++k) s[k] = (long long)max((unsigned long long)s[k], (unsigned long long)r[k]);
    }
  }
  for (int o = 1; o < tpc; o <<= 1) {
#pragma unroll
    for (int k = 0; k < kAccB; ++k) {
      const long long v = __shfl_xor(s[k], o, kWave);
      if (k < nl) s[k] += v;
      else s[k] = (long long)max((unsigned long long)s[k], (unsigned long long)v);
    }
  }
}

// the reduced record -> the double[4] of the finalisation: forward {sum y, sum y^2, max y, min y}
// (the range widened to contain 0), backward {sum d, sum d*xhat (BN a: which 0, BN b: which 1),
// sum d*xhat_b, max |d|}; NaN sums if poisoned
__device__ __forceinline__ void bnf_decode(const long long (&s)[kAccB], int mode, int which, double (&a)[4]) {
  const unsigned long long m0 = (unsigned long long)s[mode == 1 ? 6 : 9];
  const unsigned long long m1 = mode == 1 ? (unsigned long long)s[7] : 0ull;
  const bool poison = m0 >= kAccPoison || m1 >= kAccPoison;
  a[0] = poison ? (double)NAN : bnf_unlimb(s);
  a[1] = bnf_unlimb(s + (which ? 6 : 3));
  if (mode == 1) {
    a[2] = (double)__uint_as_float((unsigned)m0);
    a[3] = -(double)__uint_as_float((unsigned)m1);
  } else {
    a[2] = bnf_unlimb(s + 6);
    a[3] = (double)__uint_as_float((unsigned)m0);
  }
}

__device__ __forceinline__ void bnf_init(double (&a)[4], int mode) {
  a[0] = 0.0; a[1] = 0.0;
  a[2] = mode == 1 ? -INFINITY : 0.0;
  a[3] = mode == 1 ? INFINITY : 0.0;
}

// forward coefficients of channel c from its sums (n valid rows): mean, 1/std, scale, shift
// and the bound max |relu?(fma(y, scale, shift))| over the channel's range.  Every operation is
// an explicitly rounded intrinsic (no FMA contraction): the standalone finalize and every
// record-aware consumer — different kernels, different inlining — compute the same bits.
struct BnfFwd { double m, var; float mean, inv, sc, sh, ymax, ymin, bound; };
__device__ __forceinline__ BnfFwd bnf_coef_fwd(const BnFuse& f, int g, int c, const double (&a)[4], double n) {
  BnfFwd k;
  k.m = __ddiv_rn(a[0], n);
  const double var = __dsub_rn(__ddiv_rn(a[1], n), __dmul_rn(k.m, k.m));
  k.var = var > 0 ? var : 0;
  k.mean = (float)k.m;
  k.inv = (float)__ddiv_rn(1.0, __dsqrt_rn(__dadd_rn(k.var, (double)f.eps)));
  k.sc = __fmul_rn(k.inv, f.gamma_a[(long long)g * f.p_gstride + c]);
  k.sh = __fsub_rn(f.beta_a[(long long)g * f.p_gstride + c], __fmul_rn(k.mean, k.sc));
  k.ymax = (float)a[2];
  k.ymin = (float)a[3];
  float hi = fmaf(k.ymax, k.sc, k.sh), lo = fmaf(k.ymin, k.sc, k.sh);
  if (f.relu) { hi = fmaxf(hi, 0.f); lo = fmaxf(lo, 0.f); }
  k.bound = fmaxf(fabsf(hi), fabsf(lo));
  return k;
}
// ... and the BN's writes: running statistics (unbiased variance, momentum) and coefficient rows
__device__ __forceinline__ void bnf_write_fwd(const BnFuse& f, int g, int c, const BnfFwd& k, double n) {
  const int C = f.C;
  float* ca = f.coef_a + (long long)g * kBnRows * C;
  float* prm = f.rm_a + (long long)g * f.p_gstride + c;
  float* prv = f.rv_a + (long long)g * f.p_gstride + c;
  const double unb = n > 1 ? __ddiv_rn(__dmul_rn(k.var, n), __dsub_rn(n, 1.0)) : k.var;
  const double mo = (double)f.momentum, om = __dsub_rn(1.0, mo);
  *prm = (float)__dadd_rn(__dmul_rn(om, (double)*prm), __dmul_rn(mo, k.m));
  *prv = (float)__dadd_rn(__dmul_rn(om, (double)*prv), __dmul_rn(mo, unb));
  ca[kCMean * C + c] = k.mean;
  ca[kCInv * C + c] = k.inv;
  ca[kCScale * C + c] = k.sc;
  ca[kCShift * C + c] = k.sh;
  ca[kCYmax * C + c] = k.ymax;
  ca[kCYmin * C + c] = k.ymin;
}

// backward coefficients (bn.hip bn_bwd_apply's, from the fp32-rounded sums) of channel c of the
// BN whose forward rows are cb / parameters gam: dy = fma(A, d, fma(B, y, K)) and a bound of
// max |dy|; sdx = sum d * xhat of that BN
struct BnfBwd { float sd, sdx, A, B, K, bound; };
__device__ __forceinline__ BnfBwd bnf_coef_bwd(const BnFuse& f, int g, int c, const float* cb, const float* gam,
                                               const double (&a)[4], double sdx, double n) {
  const int C = f.C;
  BnfBwd k;
  const float fn = (float)n;
  k.sd = (float)a[0];
  k.sdx = (float)sdx;
  const float is = cb[kCInv * C + c], mean = cb[kCMean * C + c];
  k.A = __fmul_rn(gam[(long long)g * f.p_gstride + c], is);
  k.B = __fdiv_rn(__fmul_rn(__fmul_rn(-k.A, is), k.sdx), fn);
  k.K = __fsub_rn(__fdiv_rn(__fmul_rn(-k.A, k.sd), fn), __fmul_rn(k.B, mean));
  const float hi = fmaf(k.B, cb[kCYmax * C + c], k.K), lo = fmaf(k.B, cb[kCYmin * C + c], k.K);
  k.bound = __fmul_rn(__fadd_rn(__fmul_rn(fabsf(k.A), (float)a[3]), fmaxf(fabsf(hi), fabsf(lo))), 1.f + 0x1p-10f);
  return k;
}
__device__ __forceinline__ void bnf_write_bwd(const BnFuse& f, int g, int c, float* cb, float* dgam, float* dbet,
                                              const BnfBwd& k) {
  const int C = f.C;
  dbet[(long long)g * f.gr_gstride + c] = __fadd_rn(dbet[(long long)g * f.gr_gstride + c], k.sd);
  dgam[(long long)g * f.gr_gstride + c] = __fadd_rn(dgam[(long long)g * f.gr_gstride + c], k.sdx);
  cb[kCA * C + c] = k.A;
  cb[kCB * C + c] = k.B;
  cb[kCK * C + c] = k.K;
}

// per-channel finalisation of replica g from its sums a (n valid rows), with every write;
// returns the channel's bound contribution (forward: max |relu?(fma(y, scale, shift))|;
// backward: max |dy_a|, and *bound_b: max |dy_b|)
__device__ __forceinline__ float bnf_finalize_channel(const BnFuse& f, int g, int c, const double (&a)[4], double n,
                                                      float* bound_b) {
  if (f.mode == 1) {
    const BnfFwd k = bnf_coef_fwd(f, g, c, a, n);
    bnf_write_fwd(f, g, c, k, n);
    return k.bound;
  }
  float* ca = f.coef_a + (long long)g * kBnRows * f.C;
  const BnfBwd ka = bnf_coef_bwd(f, g, c, ca, f.gamma_a, a, a[1], n);
  bnf_write_bwd(f, g, c, ca, f.dgamma_a, f.dbeta_a, ka);
  if (f.coef_b) {
    float* cbp = f.coef_b + (long long)g * kBnRows * f.C;
    const BnfBwd kb = bnf_coef_bwd(f, g, c, cbp, f.gamma_b, a, a[2], n);
    bnf_write_bwd(f, g, c, cbp, f.dgamma_b, f.dbeta_b, kb);
    *bound_b = fmaxf(*bound_b, kb.bound);
  }
  return ka.bound;
}

// ---- record-aware consumers: a pending BN's coefficients derived in the consumer's prologue
// lanes per channel of a block-wide record reduction (a power of two <= 8, <= nsub)
__device__ __forceinline__ int bnf_tpc(int C, int nsub) {
  int t = 1;
  while (t < 8 && t * 2 * C <= 256 && t < nsub) t *= 2;
  return t;
}

// EVERY thread of the block calls it.  The forward coefficients of the pending BN f for replica
// g (n = Mv valid rows) into sc[c] / sh[c] (LDS, c < f.C); returns the block-wide bound of the
// BN (+ReLU) output.  write: this block is the BN's designated writer (coefficient rows, running
// statistics, the bound slot for later consumers).  Same arithmetic as bnx_finalize_kernel.
__device__ __forceinline__ float bnf_consume_fwd(const BnFuse& f, int g, int Mv, float* sc, float* sh, bool write) {
  __shared__ float bred[4];
  const int C = f.C, tpc = bnf_tpc(C, f.nsub), per = 256 / tpc;
  float bnd = 0.f;
  for (int c0 = 0; c0 < C; c0 += per) {
    const int c = c0 + (int)threadIdx.x / tpc, part = (int)threadIdx.x % tpc;
    long long s[kAccB];
    bnf_gather(f, g, c, part, tpc, c < C, s);
    if (c < C && part == 0) {
      double a[4];
      bnf_decode(s, 1, 0, a);
      const BnfFwd k = bnf_coef_fwd(f, g, c, a, (double)Mv);
      sc[c] = k.sc;
      sh[c] = k.sh;
      if (k.bound > 0.f) bnd = fmaxf(bnd, k.bound);
      if (write) bnf_write_fwd(f, g, c, k, (double)Mv);
    }
  }
  bnd = wave_max(bnd);
  if ((threadIdx.x & 63) == 0) bred[threadIdx.x >> 6] = bnd;
  __syncthreads();
  bnd = fmaxf(fmaxf(bred[0], bred[1]), fmaxf(bred[2], bred[3]));
  if (write && threadIdx.x == 0 && f.amax_a && bnd > 0.f) atomicMax(f.amax_a + g, __float_as_int(bnd));
  __syncthreads();   // sc / sh visible; bred free for another call
  return bnd;
}

// EVERY thread calls it.  The backward coefficients A / B / K of the pending BN record f (which:
// BN a 0, BN b 1 — f's `a` fields then hold that BN's pointers) for replica g into A / B / K
// (LDS); write: the designated writer block accumulates dgamma / dbeta, writes the A / B / K
// rows and folds the dy bound into the BN's slot (f.amax_a).
__device__ __forceinline__ void bnf_consume_bwd(const BnFuse& f, int which, int g, int Mv, float* A, float* B,
                                                float* K, bool write) {
  __shared__ float bredb[4];
  const int C = f.C, tpc = bnf_tpc(C, f.nsub), per = 256 / tpc;
  float* cb = f.coef_a + (long long)g * kBnRows * C;
  float bnd = 0.f;
  for (int c0 = 0; c0 < C; c0 += per) {
    const int c = c0 + (int)threadIdx.x / tpc, part = (int)threadIdx.x % tpc;
    long long s[kAccB];
    bnf_gather(f, g, c, part, tpc, c < C, s);
    if (c < C && part == 0) {
      double a[4];
      bnf_decode(s, 2, 0, a);
      const BnfBwd k = bnf_coef_bwd(f, g, c, cb, f.gamma_a, a, which ? a[2] : a[1], (double)Mv);
      A[c] = k.A;
      B[c] = k.B;
      K[c] = k.K;
      bnd = fmaxf(bnd, k.bound);
      if (write) bnf_write_bwd(f, g, c, cb, f.dgamma_a, f.dbeta_a, k);
    }
  }
  bnd = wave_max(bnd);
  if ((threadIdx.x & 63) == 0) bredb[threadIdx.x >> 6] = bnd;
  __syncthreads();
  bnd = fmaxf(fmaxf(bredb[0], bredb[1]), fmaxf(bredb[2], bredb[3]));
  if (write && threadIdx.x == 0 && f.amax_a && bnd > 0.f) atomicMax(f.amax_a + g, __float_as_int(bnd));
  __syncthreads();   // A / B / K visible; bredb free for another call
}

// a tile's statistics staged in LDS: Ct [BM][BN] fp32 (forward: y; backward: d, already masked)
// of rows m0.. / columns n0.. of replica g; orow[r] >= 0 marks a valid row and is its element
// offset in the replica's [M][C] output (the offset of ya / yb too).  Each 32-row group is
// reduced in fp64 in row order and put on the integer grid, the tile's groups are added, and
// the tile's column sums go to the accumulator with agent-scope atomics (spread copy: the tile
// index modulo nsub).  EVERY thread of the block calls it (it reuses Ct's memory after a barrier).
template <int BM, int BN>
__device__ __forceinline__ void bnf_tile_records(const BnFuse& f, float* Ct, const long long* orow, int g,
                                                 int m0, int n0, int Mv) {
  constexpr int NG = BM / kBnGrp;
  static_assert(BM % kBnGrp == 0, "tiles cover whole groups");
  constexpr int PER = (NG * BN + 255) / 256;      // (group, column) pairs per thread
  constexpr int KA = kAccB;                        // LDS stride of a pair's limbs
  static_assert(NG * BN * KA * 8 <= BM * BN * 4, "limbs fit the tile's memory");
  const int gv = ceil_div_d(Mv, kBnGrp);
  const int C = f.C, mode = f.mode;
  const float* ya = mode == 2 ? f.ya + (long long)g * f.y_gstride : nullptr;
  const float* yb = (mode == 2 && f.yb) ? f.yb + (long long)g * f.y_gstride : nullptr;
  const float* ca = f.coef_a + (long long)g * kBnRows * C;
  const float* cb = f.coef_b ? f.coef_b + (long long)g * kBnRows * C : nullptr;
  long long lim[PER][KA];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
#pragma unroll
    for (int k = 0; k < KA; ++k) lim[u][k] = 0;
    const int e = threadIdx.x + 256 * u;
    const int grp = e / BN, cc = e - grp * BN, n = n0 + cc;
    const int b = m0 / kBnGrp + grp;
    if (e >= NG * BN || n >= C || b >= gv) continue;
    double a[4];
    bnf_init(a, mode);
    if (mode == 1) {
#pragma unroll 8
      for (int r = 0; r < kBnGrp; ++r) {
        const int row = grp * kBnGrp + r;
        if (orow[row] < 0) continue;
        const double v = (double)Ct[row * BN + cc];
        a[0] += v;
        a[1] = fma(v, v, a[1]);
        a[2] = fmax(a[2], v);
        a[3] = fmin(a[3], v);
      }
      bool ok = bnf_limbs(a[0], lim[u]) && bnf_limbs(a[1], lim[u] + 3);
      const float hi = (float)fmax(a[2], 0.0), lo = (float)fmax(-a[3], 0.0);
      lim[u][6] = (long long)(ok ? bnf_fbits(hi) : kAccPoison);
      lim[u][7] = (long long)bnf_fbits(lo);
      if (a[2] != a[2] || a[3] != a[3]) lim[u][6] = (long long)kAccPoison;
    } else {
      const float ma = ca[kCMean * C + n], ia = ca[kCInv * C + n];
      const float mb = cb ? cb[kCMean * C + n] : 0.f, ib = cb ? cb[kCInv * C + n] : 0.f;
      // the group's BN inputs first, all loads in flight (a load per row in the ordered loop
      // below cost one memory latency per 4 rows: +8-12 us per data-gradient launch)
      float yav[kBnGrp], ybv[kBnGrp];
#pragma unroll
      for (int r = 0; r < kBnGrp; ++r) {
        const long long o = orow[grp * kBnGrp + r];
        yav[r] = o >= 0 ? ya[o + n] : 0.f;
        ybv[r] = (o >= 0 && yb) ? yb[o + n] : 0.f;
      }
      bool fin = true;
#pragma unroll
      for (int r = 0; r < kBnGrp; ++r) {
        const int row = grp * kBnGrp + r;
        if (orow[row] < 0) continue;
        const float d = Ct[row * BN + cc];
        const float xa = (yav[r] - ma) * ia;
        a[0] += (double)d;
        a[1] = fma((double)d, (double)xa, a[1]);
        if (yb) a[2] = fma((double)d, (double)((ybv[r] - mb) * ib), a[2]);
        fin = fin && d == d;
        a[3] = fmax(a[3], (double)fabsf(d));
      }
      const bool ok = fin && bnf_limbs(a[0], lim[u]) && bnf_limbs(a[1], lim[u] + 3) && bnf_limbs(a[2], lim[u] + 6);
      lim[u][9] = (long long)(ok ? bnf_fbits((float)a[3]) : kAccPoison);
    }
  }
  __syncthreads();   // every thread is done reading Ct
  const int ka = bnf_kacc(mode), nl = mode == 1 ? 6 : 9;
  const int sub = (m0 / BM) % f.nsub;
  constexpr int TPC = 256 / BN;   // threads sharing a column when 256 % BN == 0
  if constexpr (256 % BN == 0 && KA * (256 - BN) * 8 <= BM * BN * 4) {
    // a thread's pairs all lie in column threadIdx.x % BN: their limbs add in registers, then the
    // column's TPC threads meet in LDS (lane-contiguous int64 slots), then one atomic set per column
    long long t[KA];
#pragma unroll
    for (int k = 0; k < KA; ++k) t[k] = 0;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
#pragma unroll
      for (int k = 0; k < KA; ++k)
        if (k < nl) t[k] += lim[u][k];
        else t[k] = (long long)max((unsigned long long)t[k], (unsigned long long)lim[u][k]);
    }
    const int cc = threadIdx.x % BN, j = threadIdx.x / BN;
    if constexpr (TPC > 1) {
      long long* L = reinterpret_cast<long long*>(Ct);
      if (j > 0) {
#pragma unroll
        for (int k = 0; k < KA; ++k) L[(k * (TPC - 1) + j - 1) * BN + cc] = t[k];
      }
      __syncthreads();
      if (j == 0) {
#pragma unroll
        for (int i = 0; i < TPC - 1; ++i)
#pragma unroll
          for (int k = 0; k < KA; ++k) {
            const long long v = L[(k * (TPC - 1) + i) * BN + cc];
            if (k < nl) t[k] += v;
            else t[k] = (long long)max((unsigned long long)t[k], (unsigned long long)v);
          }
      }
    }
    const int n = n0 + cc;
    if (j == 0 && n < C) {
      unsigned long long* dst = (unsigned long long*)(f.acc + (((long long)g * C + n) * f.nsub + sub) * ka);
      for (int k = 0; k < nl; ++k)
        if (t[k] != 0) __hip_atomic_fetch_add(dst + k, (unsigned long long)t[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int k = nl; k < ka; ++k)
        if (t[k] != 0) __hip_atomic_fetch_max(dst + k, (unsigned long long)t[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (TPC > 1) __syncthreads();   // (LDS reads done before the caller reuses Ct)
    return;
  }
  long long* L = reinterpret_cast<long long*>(Ct);
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int e = threadIdx.x + 256 * u;
    if (e < NG * BN) {
#pragma unroll
      for (int k = 0; k < KA; ++k) L[e * KA + k] = lim[u][k];
    }
  }
  __syncthreads();
  for (int cc = threadIdx.x; cc < BN; cc += 256) {
    const int n = n0 + cc;
    if (n >= C) continue;
    long long t[KA];
#pragma unroll
    for (int k = 0; k < KA; ++k) t[k] = 0;
#pragma unroll
    for (int grp = 0; grp < NG; ++grp) {
      const long long* q = L + (grp * BN + cc) * KA;
      for (int k = 0; k < nl; ++k) t[k] += q[k];
      for (int k = nl; k < ka; ++k) t[k] = (long long)max((unsigned long long)t[k], (unsigned long long)q[k]);
    }
    unsigned long long* dst = (unsigned long long*)(f.acc + (((long long)g * C + n) * f.nsub + sub) * ka);
    for (int k = 0; k < nl; ++k)
      if (t[k] != 0) __hip_atomic_fetch_add(dst + k, (unsigned long long)t[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int k = nl; k < ka; ++k)
      if (t[k] != 0) __hip_atomic_fetch_max(dst + k, (unsigned long long)t[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// the backward mask of an output element vector (4 consecutive channels n.. at row offset o of
// replica g): d = g where the BN(+ReLU) output is > 0
__device__ __forceinline__ float4 bnf_mask4(const BnFuse& f, int g, long long o, int n, float4 v) {
  if (f.mask_out) {
    const float4 m = *(const float4*)(f.mask_out + (long long)g * f.y_gstride + o + n);
    v.x = m.x > 0.f ? v.x : 0.f; v.y = m.y > 0.f ? v.y : 0.f; v.z = m.z > 0.f ? v.z : 0.f; v.w = m.w > 0.f ? v.w : 0.f;
  } else if (f.mask_lazy) {
    const float* ca = f.coef_a + (long long)g * kBnRows * f.C;
    const float4 y = *(const float4*)(f.ya + (long long)g * f.y_gstride + o + n);
    const float4 sc = *(const float4*)(ca + kCScale * f.C + n), sh = *(const float4*)(ca + kCShift * f.C + n);
    v.x = fmaf(y.x, sc.x, sh.x) > 0.f ? v.x : 0.f;
    v.y = fmaf(y.y, sc.y, sh.y) > 0.f ? v.y : 0.f;
    v.z = fmaf(y.z, sc.z, sh.z) > 0.f ? v.z : 0.f;
    v.w = fmaf(y.w, sc.w, sh.w) > 0.f ? v.w : 0.f;
  }
  return v;
}

// The standalone finalisation of a BN's record (consumers that do not derive the coefficients
// themselves): a thread per (channel, replica) sums the channel's spread copies and finalises;
// the bound folds into the zeroed slot with an integer atomicMax (exact, any order).
namespace {
__global__ __launch_bounds__(64) void bnx_finalize_kernel(const BnFuse f, const int* __restrict__ nvalid, int N,
                                                          int HW) {
  const int g = blockIdx.y, c = blockIdx.x * 64 + threadIdx.x;
  const int Mv = valid_rows(nvalid, g, N) * HW;
  if (Mv <= 0) return;   // (inactive replicas: consumers skip them)
  float ba = 0.f, bb = 0.f;
  long long s[kAccB];
  bnf_gather(f, g, c, 0, 1, c < f.C, s);
  if (c < f.C) {
    double a[4];
    bnf_decode(s, f.mode, f.which, a);
    ba = bnf_finalize_channel(f, g, c, a, (double)Mv, &bb);
  }
  ba = wave_max(ba);
  bb = wave_max(bb);
  if (threadIdx.x == 0) {
    const int s = blockIdx.x % kAmaxSub;
    if (f.amax_a && ba > 0.f) atomicMax(f.amax_a + s * f.amax_ld + g, __float_as_int(ba));
    if (f.amax_b && bb > 0.f) atomicMax(f.amax_b + s * f.amax_ld + g, __float_as_int(bb));
  }
}

// the finalize launch of a fused BN pass (after its producer in stream order)
inline int bnx_finalize_go(const BnFuse& f, const int* nvalid, int G, int N, int HW, hipStream_t st) {
  hipLaunchKernelGGL(bnx_finalize_kernel, dim3((f.C + 63) / 64, G), dim3(64), 0, st, f, nvalid, N, HW);
  return (int)hipGetLastError();
}
}  // namespace
