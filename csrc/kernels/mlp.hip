// Persistent LoanNet trainer: ONE workgroup per client runs a whole segment of that client's
// local SGD steps (reference loan_train.py:98-127, models/loan_model.py:10-27) without
// returning to the host.
//
// The grouped trainer (fl/trainer.py) replays a captured graph per step: gather, three
// linear layers forward + backward, dropout, cross-entropy, SGD — ~20 launches of a few
// microseconds each for 64 x 91 inputs, so a LOAN round (clients of up to several thousand
// steps) is bound by launch latency (0.66 s of a 0.78 s round).  Here the
// client's parameters and momentum live in LDS for the segment (LoanNet has 5.5 k
// parameters), every step is a handful of LDS-resident fp32 VALU GEMMs separated by
// workgroup barriers, and the host launches one kernel per segment between phase events
// (snapshots / model-replacement scaling at internal-epoch ends).
//
// Per step, in the trainer's order (fl/trainer.py _step_ops): gather the batch rows with the
// feature trigger and label swap of the first poison_n rows (data.hip gather_rows_kernel);
// z1 = x W1^T + b1 -> ReLU -> dropout(0.5, salt 0); z2 -> ReLU -> dropout(salt 1); logits =
// a2 W3^T + b3 (the reference's Linear -> Dropout -> ReLU equals ReLU -> Dropout: the mask
// scales by 2 or zeroes); softmax cross-entropy with the batch mean, correct count and the
// per-epoch statistics slot (loss.hip xent_kernel: same __expf / __logf, fp64 row-loss sum);
// backward; SGD with momentum, weight decay, per-step lr and fresh-optimizer flag, FoolsGold
// gradient accumulation (optim.hip sgd_kernel: same expressions).  The dropout masks use the
// framework's counter hash with the step's seed (elementwise.hip dropout_kernel), so the
// masks are those of the graph path.  Arithmetic is exact fp32 FMA in a fixed order (the
// graph path runs the layers on the split-fp16 MFMA family), so the two paths agree to fp32
// rounding, not bitwise; every sum has a fixed order, so the kernel is deterministic.
#include "common.hpp"

namespace {

constexpr int kB = 64, kF = 91, kH1 = 46, kH2 = 23, kC = 9;   // batch, LoanNet dims
constexpr int kH1p = 48, kH2p = 24, kFp = 96;                 // zero-padded row counts
constexpr int kPmax = 6144;                                   // flat parameter floats (aligned entries)
constexpr int kT = 512;                                       // threads: 8 waves, 2 per SIMD
// row stride of the feature-major activation images: 68 floats (272 B) puts consecutive rows
// one 16-B bank slot apart, so lanes walking rows (the weight-gradient loops) read without
// LDS bank conflicts (a 64-float stride put every lane on the same slot)
constexpr int kLD = kB + 4;
constexpr int kLG = kC + 4;                                   // dlogits row stride (odd: conflict-free)

struct MlpArgs {
  const int* sched; int D, t0, t1, G;        // step descriptors [T][D] (fl/trainer.py _GroupBuffers)
  float* state; long long s_stride;          // [G][S] replica states: parameters first
  float* mom; float* fg;                     // [G][P] momentum, FoolsGold sums (null: off)
  int P;
  int o_w1, o_b1, o_w2, o_b2, o_w3, o_b3;    // entry offsets in the flat state
  const float* rows; const int* labels;      // training rows [n][kF], labels [n]
  const int* tcols; const float* tvals; int K; int target;   // feature triggers [n_trig][K]
  float* stats; long long stats_stride; int max_slots;       // [3][G * max_slots]
  float* nan_flag;
  float momentum, wd;
  long long* prof;                           // diagnostics (tools/bench_mlp --prof): [T][8] phase clocks, or null
};

struct MlpLds {
  float prm[kPmax], mom[kPmax];
  float xT[kFp * kLD];                                     // batch, feature-major (rows >= kF zero)
  float a1T[kH1p * kLD], a2T[kH2p * kLD];                  // post-dropout activations
  float lg[kB * kLG];                                      // dlogits
  float d1T[kH1p * kLD], d2T[kH2p * kLD];                  // pre-activation gradients
  int y[kB];
  double wl[4];
  float wc[4];
};

__device__ __forceinline__ void sgd1(MlpLds& s, const MlpArgs& a, float* fgr, int o, float gr, float lr, bool first) {
  const float p = s.prm[o];
  if (fgr) fgr[o] += gr;
  const float d = gr + a.wd * p;
  const float m = first ? d : a.momentum * s.mom[o] + d;
  s.mom[o] = m;
  s.prm[o] = p - lr * m;
}

// One 32 x 32 fp32 output tile D[i][j] = sum_k A(i, k) B(k, j), k < 2 nks, on the exact-fp32
// MFMA (v_mfma_f32_32x32x2_f32: lane l supplies A(l % 32, l / 32) and B(l / 32, l % 32) of
// each 2-deep step; it holds D rows (r & 3) + 8 (r >> 2) + 4 (l / 32), column l % 32).  The
// fp32 matrix rate is twice the VALU FMA rate, and each operand value read from LDS feeds a
// 32-wide outer product instead of 2-4 register-blocked FMAs (the VALU version was bound by
// LDS return bandwidth and load latency: tools/bench_mlp --prof).
template <typename FA, typename FB>
__device__ __forceinline__ f32x16_t mm_tile(int nks, FA fa, FB fb) {
  f32x16_t acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int lane = threadIdx.x & 63, r32 = lane & 31, kh = lane >> 5;
#pragma unroll 4
  for (int ks = 0; ks < nks; ++ks) {
    const int k = 2 * ks + kh;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa(r32, k), fb(k, r32), acc, 0, 0, 0);
  }
  return acc;
}
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// outstanding global loads (__syncthreads' workgroup release fence would also wait vmcnt(0),
// i.e. for the next step's prefetched batch rows, which must stay in flight across the step)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ int tile_row(int r) { return (r & 3) + 8 * (r >> 2) + 4 * ((threadIdx.x & 63) >> 5); }

__global__ __launch_bounds__(kT) void mlp_train_kernel(const MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  MlpLds& s = *reinterpret_cast<MlpLds*>(smem);
  const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int G = a.G, GB = G * kB;
  float* st = a.state + (long long)g * a.s_stride;
  float* mg = a.mom + (long long)g * a.P;
  float* fgr = a.fg ? a.fg + (long long)g * a.P : nullptr;

  // a client whose steps ended before this segment has nothing to do
  if (!a.sched[(long long)a.t0 * a.D + GB + 3 * G + g]) return;

  for (int i = tid; i < a.P; i += kT) {
    s.prm[i] = st[i];
    s.mom[i] = mg[i];
  }
  for (int i = tid; i < kH1p * kLD; i += kT) s.a1T[i] = s.d1T[i] = 0.f;
  for (int i = tid; i < kFp * kLD; i += kT) s.xT[i] = 0.f;
  for (int i = tid; i < kH2p * kLD; i += kT) s.a2T[i] = s.d2T[i] = 0.f;
  for (int i = tid; i < kB * kLG; i += kT) s.lg[i] = 0.f;
  __syncthreads();

  // Step descriptors and batch rows are fetched ONE STEP AHEAD into registers (the HBM
  // latency of the random row gather and of the descriptor reads overlaps the current step's
  // compute) and staged into LDS at the end of the step.  A client's active steps are
  // contiguous from its first (fl/plan.py, native pack_steps), so the loop ends at its first
  // inactive step.
  constexpr int NG = (kB * kF + kT - 1) / kT;   // gathered elements per thread
  struct Desc { int poison_n, trig, first, active, nvalid, slot; uint32_t seed; float lr; };
  auto desc = [&](int t) __attribute__((always_inline)) {
    Desc q{0, -1, 0, 0, 0, 0, 0u, 0.f};
    if (t >= a.t1) return q;
    const int* f8 = a.sched + (long long)t * a.D + GB;
    q.poison_n = f8[g]; q.trig = f8[G + g]; q.first = f8[2 * G + g]; q.active = f8[3 * G + g];
    q.nvalid = f8[4 * G + g]; q.slot = f8[5 * G + g]; q.seed = (uint32_t)f8[6 * G + g];
    q.lr = __int_as_float(f8[7 * G + g]);
    return q;
  };
  float gv[NG];
  int gy = -1;
  // the gather in two halves, so no wave waits on a global load mid-step: the row indices
  // (and the label-row index) are loaded first, the rows themselves one phase later, once the
  // indices have landed; the values are consumed by stage() at the end of the step
  int gi[NG];
  int gl = -1;
  auto gather_idx = [&](int t, const Desc& q, int tid) __attribute__((always_inline)) {
    if (!q.active) return;
    const int* idx = a.sched + (long long)t * a.D + g * kB;
#pragma unroll
    for (int u = 0; u < NG; ++u) {
      const int e = tid + kT * u;
      gi[u] = e < kB * kF ? idx[e / kF] : -1;
    }
    if (tid < kB) gl = idx[tid];
  };
  auto gather_rows = [&](const Desc& q, int tid) __attribute__((always_inline)) {
    if (!q.active) return;
    // raw row values only: selecting on them here (zero for padded rows, trigger values)
    // would make the wave wait for the loads mid-step; stage() applies both
#pragma unroll
    for (int u = 0; u < NG; ++u) {
      const int e = tid + kT * u;
      gv[u] = a.rows[(long long)max(gi[u], 0) * kF + e % kF];
    }
    if (tid < kB && gl >= 0) gy = a.labels[gl];
  };
  auto gather = [&](int t, const Desc& q, int tid) __attribute__((always_inline)) {
    gather_idx(t, q, tid);
    gather_rows(q, tid);
  };
  auto stage = [&](const Desc& q, int tid) __attribute__((always_inline)) {   // registers -> xT / y
#pragma unroll
    for (int u = 0; u < NG; ++u) {
      const int e = tid + kT * u;
      if (e < kB * kF) {
        const int b = e / kF, f = e - b * kF;
        float v = gi[u] < 0 ? 0.f : gv[u];
        if (gi[u] >= 0 && q.trig >= 0 && b < q.poison_n)   // feature trigger of the poisoned rows
          for (int k = 0; k < a.K; ++k)
            if (a.tcols[q.trig * a.K + k] == f) v = a.tvals[q.trig * a.K + k];
        s.xT[f * kLD + b] = v;
      }
    }
    if (tid < kB) s.y[tid] = gl < 0 ? -1 : ((q.trig >= 0 && tid < q.poison_n) ? a.target : gy);
  };

  Desc cur = desc(a.t0);
  gather(a.t0, cur, tid);
  stage(cur, tid);
  for (int t = a.t0; t < a.t1; ++t) {
    if (!cur.active) break;
    // an opaque per-step copy of the thread index: everything derived from it (a step's
    // hundreds of per-thread LDS / global addresses) is recomputed inside the step instead of
    // being hoisted out of the step loop, where it spilled to scratch
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wid = tid >> 6;
    const int poison_n = cur.poison_n, first = cur.first, nvalid = cur.nvalid, slot = cur.slot;
    const uint32_t seed = cur.seed;
    const float lr = cur.lr;
    (void)poison_n;
    const Desc nxt = desc(t + 1);
#define PROF(k) if (a.prof && tid == 0) a.prof[(long long)(t - a.t0) * 8 + (k)] = (long long)__builtin_readcyclecounter()
    PROF(0);
    lds_barrier();   // xT / y of step t staged
    gather_idx(t + 1, nxt, tid);   // the next step's batch: indices now, rows after layer 1

    const int c32 = lane & 31;
    // ---- layer 1: [64 x 91] x W1^T -> 2 x 2 tiles (waves 0-3), + b1, ReLU, dropout (salt 0)
    if (wid < 4) {
      const int mt = wid & 1, nt = wid >> 1;
      const f32x16_t z = mm_tile(
          (kF + 1) / 2, [&](int i, int k) { return s.xT[k * kLD + mt * 32 + i]; },
          [&](int k, int j) {
            const int u = nt * 32 + j;
            return (u < kH1 && k < kF) ? s.prm[a.o_w1 + u * kF + k] : 0.f;
          });
      const int j = nt * 32 + c32;
      if (j < kH1) {
        const float bj = s.prm[a.o_b1 + j];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int b = mt * 32 + tile_row(r);
          const bool keep = uniform01(seed, (uint32_t)(b * kH1 + j)) >= 0.5f;
          s.a1T[j * kLD + b] = keep ? fmaxf(z[r] + bj, 0.f) * 2.0f : 0.f;
        }
      }
    }
    gather_rows(nxt, tid);   // lands while this step computes
    PROF(1);
    lds_barrier();

    // ---- layer 2: 2 tiles (waves 0-1), + b2, ReLU, dropout (salt 1)
    if (wid < 2) {
      const int mt = wid;
      const f32x16_t z = mm_tile(
          kH1 / 2, [&](int i, int k) { return s.a1T[k * kLD + mt * 32 + i]; },
          [&](int k, int j) { return j < kH2 ? s.prm[a.o_w2 + j * kH1 + k] : 0.f; });
      const int j = c32;
      if (j < kH2) {
        const float bj = s.prm[a.o_b2 + j];
        const uint32_t sd1 = seed + 0x9E3779B9u;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int b = mt * 32 + tile_row(r);
          const bool keep = uniform01(sd1, (uint32_t)(b * kH2 + j)) >= 0.5f;
          s.a2T[j * kLD + b] = keep ? fmaxf(z[r] + bj, 0.f) * 2.0f : 0.f;
        }
      }
    }
    PROF(2);
    lds_barrier();

    // ---- layer 3 logits: 2 tiles (waves 0-1) -> lg
    if (wid < 2) {
      const int mt = wid;
      const f32x16_t z = mm_tile(
          kH2p / 2, [&](int i, int k) { return s.a2T[k * kLD + mt * 32 + i]; },
          [&](int k, int c) { return (c < kC && k < kH2) ? s.prm[a.o_w3 + c * kH2 + k] : 0.f; });
      if (c32 < kC) {
        const float bc = s.prm[a.o_b3 + c32];
#pragma unroll
        for (int r = 0; r < 16; ++r) s.lg[(mt * 32 + tile_row(r)) * kLG + c32] = z[r] + bc;
      }
    }
    lds_barrier();

    // ---- softmax cross-entropy (one row per thread of wave 0): dlogits into lg
    if (wid == 0) {
      const int b = lane;
      float x[kC];
#pragma unroll
      for (int c = 0; c < kC; ++c) x[c] = s.lg[b * kLG + c];
      const int y = s.y[b];
      const float scale = nvalid > 0 ? 1.0f / (float)nvalid : 1.0f;
      double wl = 0.0;
      float wc = 0.f;
      if (y < 0) {
#pragma unroll
        for (int c = 0; c < kC; ++c) s.lg[b * kLG + c] = 0.f;
      } else {
        float mx = x[0];
        int am = 0;
#pragma unroll
        for (int c = 1; c < kC; ++c)
          if (x[c] > mx) { mx = x[c]; am = c; }
        float se = 0.f;
#pragma unroll
        for (int c = 0; c < kC; ++c) se += __expf(x[c] - mx);
        const float lse = mx + __logf(se);
        float xy = x[0];
#pragma unroll
        for (int c = 1; c < kC; ++c)
          if (c == y) xy = x[c];
        wl = (double)(lse - xy);
        wc = am == y ? 1.f : 0.f;
#pragma unroll
        for (int c = 0; c < kC; ++c) s.lg[b * kLG + c] = (__expf(x[c] - lse) - (c == y ? 1.f : 0.f)) * scale;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) wl += __shfl_xor(wl, o, kWave);
      wc = wave_sum(wc);
      if (lane == 0) {
        const double l64 = nvalid > 0 ? wl / (double)nvalid : 0.0;
        const float loss = (float)l64;
        const long long si = (long long)g * a.max_slots + slot;
        a.stats[si] += loss;
        a.stats[a.stats_stride + si] += wc;
        a.stats[2 * a.stats_stride + si] += (float)nvalid;
        if (loss != loss) atomicAdd(a.nan_flag, 1.0f);   // reference LoanNet raises on NaN
      }
    }
    PROF(3);
    lds_barrier();

    // ---- d(layer-2 output) = dlogits W3, masked by a2's dropout / ReLU: 2 tiles (waves 0-1)
    if (wid < 2) {
      const int mt = wid;
      const f32x16_t z = mm_tile(
          (kC + 1) / 2, [&](int i, int k) { return k < kC ? s.lg[(mt * 32 + i) * kLG + k] : 0.f; },
          [&](int k, int j) { return (k < kC && j < kH2) ? s.prm[a.o_w3 + k * kH2 + j] : 0.f; });
      const int j = c32;
      if (j < kH2) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int b = mt * 32 + tile_row(r);
          s.d2T[j * kLD + b] = s.a2T[j * kLD + b] > 0.f ? z[r] * 2.0f : 0.f;
        }
      }
    }
    PROF(4);
    lds_barrier();

    // ---- d(layer-1 output) = d2 W2 (waves 0-3, reads W2) | layer-3 weight gradient + SGD
    // (wave 4: W3 is no longer read) | layer-3 bias gradient (wave 5)
    if (wid < 4) {
      const int mt = wid & 1, nt = wid >> 1;
      const f32x16_t z = mm_tile(
          kH2p / 2, [&](int i, int k) { return s.d2T[k * kLD + mt * 32 + i]; },
          [&](int k, int j) {
            const int u = nt * 32 + j;
            return (u < kH1 && k < kH2) ? s.prm[a.o_w2 + k * kH1 + u] : 0.f;
          });
      const int k = nt * 32 + c32;
      if (k < kH1) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int b = mt * 32 + tile_row(r);
          s.d1T[k * kLD + b] = s.a1T[k * kLD + b] > 0.f ? z[r] * 2.0f : 0.f;
        }
      }
    } else if (wid == 4) {
      const f32x16_t gw = mm_tile(
          kB / 2, [&](int c, int b) { return c < kC ? s.lg[b * kLG + c] : 0.f; },
          [&](int b, int j) { return j < kH2 ? s.a2T[j * kLD + b] : 0.f; });
      const int j = c32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = tile_row(r);
        if (c < kC && j < kH2) sgd1(s, a, fgr, a.o_w3 + c * kH2 + j, gw[r], lr, first);
      }
    } else if (wid == 5 && lane < kC) {
      float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f;
#pragma unroll
      for (int b = 0; b < kB; b += 4) {
        p0 += s.lg[b * kLG + lane];
        p1 += s.lg[(b + 1) * kLG + lane];
        p2 += s.lg[(b + 2) * kLG + lane];
        p3 += s.lg[(b + 3) * kLG + lane];
      }
      sgd1(s, a, fgr, a.o_b3 + lane, (p0 + p1) + (p2 + p3), lr, first);
    }
    PROF(5);
    lds_barrier();

    // ---- layer-1 (6 tiles, waves 0-5) / layer-2 (2 tiles, waves 6-7) weight gradients + SGD,
    // then the layer-1 / layer-2 bias gradients
    if (wid < 6) {
      const int jt = wid / 3, ft = wid % 3;
      const f32x16_t gw = mm_tile(
          kB / 2, [&](int i, int b) { const int j = jt * 32 + i; return j < kH1 ? s.d1T[j * kLD + b] : 0.f; },
          [&](int b, int f) { const int ff = ft * 32 + f; return ff < kF ? s.xT[ff * kLD + b] : 0.f; });
      const int f = ft * 32 + c32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = jt * 32 + tile_row(r);
        if (j < kH1 && f < kF) sgd1(s, a, fgr, a.o_w1 + j * kF + f, gw[r], lr, first);
      }
    } else {
      const int kt = wid - 6;
      const f32x16_t gw = mm_tile(
          kB / 2, [&](int j, int b) { return j < kH2 ? s.d2T[j * kLD + b] : 0.f; },
          [&](int b, int k) { const int kk = kt * 32 + k; return kk < kH1 ? s.a1T[kk * kLD + b] : 0.f; });
      const int k = kt * 32 + c32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = tile_row(r);
        if (j < kH2 && k < kH1) sgd1(s, a, fgr, a.o_w2 + j * kH1 + k, gw[r], lr, first);
      }
    }
    if (tid < kH1 + kH2) {
      const bool l1 = tid < kH1;
      const int u = l1 ? tid : tid - kH1;
      const float* dT = l1 ? s.d1T : s.d2T;
      float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int b = 0; b < kB; b += 4) {
        const float4 v = *(const float4*)&dT[u * kLD + b];
        p.x += v.x; p.y += v.y; p.z += v.z; p.w += v.w;
      }
      sgd1(s, a, fgr, (l1 ? a.o_b1 : a.o_b2) + u, (p.x + p.y) + (p.z + p.w), lr, first);
    }
    PROF(6);
    lds_barrier();   // xT and the weights of step t are no longer read
    stage(nxt, tid);
    cur = nxt;
#undef PROF
  }

  for (int i = tid; i < a.P; i += kT) {
    st[i] = s.prm[i];
    mg[i] = s.mom[i];
  }
}

}  // namespace

DBA_EXPORT int dba_mlp_lds_bytes() { return (int)sizeof(MlpLds); }

// Segment [t0, t1) of the step table for every client of a G-replica group, LoanNet only
// (in 91, hidden 46 / 23, out 9, batch 64: -100 otherwise — the caller keeps the graph path).
DBA_EXPORT int dba_mlp_train(const int* sched, int D, int t0, int t1, int G, int B, float* state, long long s_stride,
                             float* mom, float* fg, int P, const int* offs, int F, int H1, int H2, int C,
                             const float* rows, const int* labels, const int* tcols, const float* tvals, int K,
                             int target, float* stats, long long stats_stride, int max_slots, float* nan_flag,
                             float momentum, float wd, long long* prof, void* stream) {
  if (B != kB || F != kF || H1 != kH1 || H2 != kH2 || C != kC || P > kPmax || D != G * B + 8 * G) return -100;
  if (t1 <= t0) return 0;
  MlpArgs a{sched, D, t0, t1, G, state, s_stride, mom, fg, P, offs[0], offs[1], offs[2], offs[3], offs[4], offs[5],
            rows, labels, tcols, tvals, K, target, stats, stats_stride, max_slots, nan_flag, momentum, wd, prof};
  // the dynamic-LDS attribute is per device: set once for every device this process launches on
  // (a device that refuses the ~118 KB budget declines the launch: the caller keeps the graph path)
  static unsigned long long attr_set = 0ull;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -100;
  if (!(attr_set >> dev & 1ull)) {
    const hipError_t e = hipFuncSetAttribute((const void*)mlp_train_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)sizeof(MlpLds));
    if (e != hipSuccess) return -100;
    attr_set |= 1ull << dev;
  }
  hipLaunchKernelGGL(mlp_train_kernel, dim3(G), dim3(kT), sizeof(MlpLds), (hipStream_t)stream, a);
  DBA_LAUNCH_CHECK();
}
