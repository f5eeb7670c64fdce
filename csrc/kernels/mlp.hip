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
constexpr int kH1p = 48, kH2p = 24, kCp = 12;                 // padded to 4-wide blocks
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
  float w1t[kF * kH1p], w2t[kH1 * kH2p], w3t[kH2 * kCp];   // transposed weights [in][out]
  float xT[kF * kLD];                                      // batch, feature-major
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
  for (int i = tid; i < kH2p * kLD; i += kT) s.a2T[i] = s.d2T[i] = 0.f;
  for (int i = tid; i < kB * kLG; i += kT) s.lg[i] = 0.f;
  __syncthreads();
  auto transpose_w = [&]() __attribute__((always_inline)) {
    for (int e = tid; e < kF * kH1p; e += kT) {
      const int f = e / kH1p, j = e - f * kH1p;
      s.w1t[e] = j < kH1 ? s.prm[a.o_w1 + j * kF + f] : 0.f;
    }
    for (int e = tid; e < kH1 * kH2p; e += kT) {
      const int k = e / kH2p, j = e - k * kH2p;
      s.w2t[e] = j < kH2 ? s.prm[a.o_w2 + j * kH1 + k] : 0.f;
    }
    for (int e = tid; e < kH2 * kCp; e += kT) {
      const int k = e / kCp, c = e - k * kCp;
      s.w3t[e] = c < kC ? s.prm[a.o_w3 + c * kH2 + k] : 0.f;
    }
  };
  transpose_w();

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
  auto gather = [&](int t, const Desc& q, int tid) __attribute__((always_inline)) {   // step t's rows -> registers
    if (!q.active) return;
    const int* idx = a.sched + (long long)t * a.D + g * kB;
#pragma unroll
    for (int u = 0; u < NG; ++u) {
      const int e = tid + kT * u;
      const int b = e / kF, f = e - b * kF;
      const int r = e < kB * kF ? idx[b] : -1;
      float v = 0.f;
      if (r >= 0) {
        v = a.rows[(long long)r * kF + f];
        if (q.trig >= 0 && b < q.poison_n)
          for (int k = 0; k < a.K; ++k)
            if (a.tcols[q.trig * a.K + k] == f) v = a.tvals[q.trig * a.K + k];
      }
      gv[u] = v;
    }
    if (tid < kB) {
      const int r = idx[tid];
      gy = r < 0 ? -1 : ((q.trig >= 0 && tid < q.poison_n) ? a.target : a.labels[r]);
    }
  };
  auto stage = [&](int tid) __attribute__((always_inline)) {   // registers -> xT / y (no reader in flight)
#pragma unroll
    for (int u = 0; u < NG; ++u) {
      const int e = tid + kT * u;
      if (e < kB * kF) {
        const int b = e / kF, f = e - b * kF;
        s.xT[f * kLD + b] = gv[u];
      }
    }
    if (tid < kB) s.y[tid] = gy;
  };

  Desc cur = desc(a.t0);
  gather(a.t0, cur, tid);
  stage(tid);
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
    __syncthreads();   // xT / y of step t staged
    gather(t + 1, nxt, tid);   // lands while this step computes

    // ---- layer 1: 2 x 4 (row, unit) blocks, 384 threads
    if (tid < (kB / 2) * (kH1p / 4)) {
      const int b0 = (tid & 31) * 2, j0 = (tid >> 5) * 4;
      float acc[2][4] = {};
#pragma unroll 7
      for (int f = 0; f < kF; ++f) {
        const float2 xv = *(const float2*)&s.xT[f * kLD + b0];
        const float4 wv = *(const float4*)&s.w1t[f * kH1p + j0];
        const float xs[2] = {xv.x, xv.y}, ws[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[i][k] = fmaf(xs[i], ws[k], acc[i][k]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int j = j0 + k;
        if (j >= kH1) break;
        const float bj = s.prm[a.o_b1 + j];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int b = b0 + i;
          const bool keep = uniform01(seed, (uint32_t)(b * kH1 + j)) >= 0.5f;
          s.a1T[j * kLD + b] = keep ? fmaxf(acc[i][k] + bj, 0.f) * 2.0f : 0.f;
        }
      }
    }
    PROF(1);
    __syncthreads();

    // ---- layer 2: 2 x 4 blocks, 192 threads
    if (tid < (kB / 2) * (kH2p / 4)) {
      const int b0 = (tid & 31) * 2, j0 = (tid >> 5) * 4;
      float acc[2][4] = {};
#pragma unroll 2
      for (int k = 0; k < kH1; ++k) {
        const float2 xv = *(const float2*)&s.a1T[k * kLD + b0];
        const float4 wv = *(const float4*)&s.w2t[k * kH2p + j0];
        const float xs[2] = {xv.x, xv.y}, ws[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[i][q] = fmaf(xs[i], ws[q], acc[i][q]);
      }
      const uint32_t sd1 = seed + 0x9E3779B9u;   // salt 1
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = j0 + q;
        if (j >= kH2) break;
        const float bj = s.prm[a.o_b2 + j];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int b = b0 + i;
          const bool keep = uniform01(sd1, (uint32_t)(b * kH2 + j)) >= 0.5f;
          s.a2T[j * kLD + b] = keep ? fmaxf(acc[i][q] + bj, 0.f) * 2.0f : 0.f;
        }
      }
    }
    PROF(2);
    __syncthreads();

    // ---- layer 3 + softmax cross-entropy (one row per thread of wave 0)
    if (wid == 0) {
      const int b = lane;
      float x[kC];
#pragma unroll
      for (int c = 0; c < kC; ++c) x[c] = 0.f;
      for (int k = 0; k < kH2; ++k) {
        const float av = s.a2T[k * kLD + b];
#pragma unroll
        for (int c = 0; c < kC; ++c) x[c] = fmaf(av, s.w3t[k * kCp + c], x[c]);
      }
#pragma unroll
      for (int c = 0; c < kC; ++c) x[c] += s.prm[a.o_b3 + c];
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
    __syncthreads();

    // ---- d(layer-2 output): dlogits W3, masked by the dropout / ReLU of a2
    for (int e = tid; e < kB * kH2; e += kT) {
      const int j = e / kB, b = e - j * kB;
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < kC; ++c) acc = fmaf(s.lg[b * kLG + c], s.prm[a.o_w3 + c * kH2 + j], acc);
      s.d2T[j * kLD + b] = s.a2T[j * kLD + b] > 0.f ? acc * 2.0f : 0.f;
    }
    PROF(4);
    __syncthreads();

    // ---- d(layer-1 output) (reads W2) | layer-3 gradients + SGD (W3 no longer read)
    for (int e = tid; e < kB * kH1; e += kT) {
      const int k = e / kB, b = e - k * kB;
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < kH2; ++j) acc = fmaf(s.d2T[j * kLD + b], s.prm[a.o_w2 + j * kH1 + k], acc);
      s.d1T[k * kLD + b] = s.a1T[k * kLD + b] > 0.f ? acc * 2.0f : 0.f;
    }
    for (int e = tid; e < kC * kH2 + kC; e += kT) {
      float gr = 0.f;
      if (e < kC * kH2) {
        const int c = e / kH2, j = e - c * kH2;
        for (int b = 0; b < kB; ++b) gr = fmaf(s.lg[b * kLG + c], s.a2T[j * kLD + b], gr);
        sgd1(s, a, fgr, a.o_w3 + e, gr, lr, first);
        s.w3t[j * kCp + c] = s.prm[a.o_w3 + e];
      } else {
        const int c = e - kC * kH2;
        for (int b = 0; b < kB; ++b) gr += s.lg[b * kLG + c];
        sgd1(s, a, fgr, a.o_b3 + c, gr, lr, first);
      }
    }
    PROF(5);
    __syncthreads();

    // ---- layer-1 / layer-2 weight + bias gradients and SGD: 4 x 4 (unit, input) blocks, the
    // block's inputs {q, q + n4, q + 2 n4, q + 3 n4} so consecutive lanes read consecutive
    // activation rows (conflict-free), its units 4 consecutive (a broadcast per lane group)
    constexpr int F4 = (kF + 3) / 4, K4 = (kH1 + 3) / 4;                 // 23, 12
    constexpr int N1 = ((kH1 + 3) / 4) * F4, N2 = ((kH2 + 3) / 4) * K4, NB = kH1 + kH2;
    static_assert(N1 + N2 + NB <= kT, "one pass");
    if (tid < N1 + N2) {
      const bool l1 = tid < N1;
      const int e2 = l1 ? tid : tid - N1;
      const int nin = l1 ? kF : kH1, nout = l1 ? kH1 : kH2, n4 = l1 ? F4 : K4;
      const int j0 = (e2 / n4) * 4, q = e2 % n4;
      const float* dT = l1 ? s.d1T : s.d2T;
      const float* inT = l1 ? s.xT : s.a1T;
      int jr[4], fr4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        jr[u] = min(j0 + u, nout - 1);            // clamped rows: their sums are discarded
        fr4[u] = min(q + u * n4, nin - 1);
      }
      float gw[4][4] = {};
#pragma unroll 2
      for (int b = 0; b < kB; b += 4) {
        float4 dv[4], xv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          dv[u] = *(const float4*)&dT[jr[u] * kLD + b];
          xv[u] = *(const float4*)&inT[fr4[u] * kLD + b];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            gw[u][v] = fmaf(dv[u].x, xv[v].x, gw[u][v]);
            gw[u][v] = fmaf(dv[u].y, xv[v].y, gw[u][v]);
            gw[u][v] = fmaf(dv[u].z, xv[v].z, gw[u][v]);
            gw[u][v] = fmaf(dv[u].w, xv[v].w, gw[u][v]);
          }
      }
      const int ow = l1 ? a.o_w1 : a.o_w2;
      float* wt = l1 ? s.w1t : s.w2t;
      const int ldt = l1 ? kH1p : kH2p;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = j0 + u;
        if (j >= nout) break;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int f = q + v * n4;
          if (f >= nin) break;
          const int o = ow + j * nin + f;
          sgd1(s, a, fgr, o, gw[u][v], lr, first);
          wt[f * ldt + j] = s.prm[o];
        }
      }
    } else if (tid < N1 + N2 + NB) {
      const int j = tid - N1 - N2;
      const bool l1 = j < kH1;
      const int u = l1 ? j : j - kH1;
      const float* dT = l1 ? s.d1T : s.d2T;
      float gr = 0.f;
      for (int b = 0; b < kB; ++b) gr += dT[u * kLD + b];
      sgd1(s, a, fgr, (l1 ? a.o_b1 : a.o_b2) + u, gr, lr, first);
    }
    PROF(6);
    __syncthreads();   // xT and the weights of step t are no longer read
    stage(tid);
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
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)mlp_train_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)sizeof(MlpLds));
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL(mlp_train_kernel, dim3(G), dim3(kT), sizeof(MlpLds), (hipStream_t)stream, a);
  DBA_LAUNCH_CHECK();
}
