// Host-side native runtime of the DBA-on-MI355X framework (C ABI, loaded via ctypes).
//
// The reference feeds every client batch through torch DataLoader worker processes
// (image_helper.py:252-263, num_workers=8) and schedules clients in a sequential Python
// loop (image_train.py:21).  Here the per-round work is planned once on the host and
// shipped to the GPU as one packed descriptor table:
//
//   * dba_pack_steps   — builds the [T, D] int32 step-descriptor table consumed by the
//                        HIP-graph-replayed grouped training step (one row per step, all
//                        clients of the rank side by side).
//   * dba_lpt_assign   — longest-processing-time placement of clients onto ranks
//                        (client-parallel data parallelism).
//   * dba_shard_index  — strided sharding of evaluation index lists across ranks.
//   * dba_balance_shares — water-filling shares of a round's image-sharded evaluation over
//                        ranks, given each rank's training + local-test load in the window.
//
// Row layout (D = G*B + 8*G int32 words):
//   idx[G*B] | poison_n[G] | trig[G] | first[G] | active[G] | nvalid[G] | slot[G] | seed[G] | lr[G] (f32 bits)
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <vector>

namespace {

inline uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

}  // namespace

extern "C" {

int dba_runtime_version() { return 4; }

uint32_t dba_hash2(uint32_t seed, uint32_t counter) { return lowbias32(counter ^ lowbias32(seed)); }

// Returns 0 on success, negative on a malformed schedule.
int dba_pack_steps(int G, int B, int T, int max_slots,
                   const int64_t* step_off,   // [G+1]   client g owns steps [step_off[g], step_off[g+1])
                   const int64_t* idx_off,    // [S+1]   step s owns idx_flat[idx_off[s], idx_off[s+1])
                   const int32_t* idx_flat,
                   const int32_t* poison_n, const int32_t* trig, const int32_t* first,
                   const int32_t* slot, const float* lr,   // [S] per step
                   const uint32_t* client_seed,            // [G]
                   int32_t* out) {                          // [T, D]
  const int64_t D = (int64_t)G * B + 8LL * G;
  for (int t = 0; t < T; ++t) {
    int32_t* row = out + (int64_t)t * D;
    int32_t* ridx = row;
    int32_t* f = row + (int64_t)G * B;
    int32_t* r_pn = f;
    int32_t* r_trig = f + G;
    int32_t* r_first = f + 2 * G;
    int32_t* r_act = f + 3 * G;
    int32_t* r_nv = f + 4 * G;
    int32_t* r_slot = f + 5 * G;
    int32_t* r_seed = f + 6 * G;
    int32_t* r_lr = f + 7 * G;
    for (int g = 0; g < G; ++g) {
      const int64_t ns = step_off[g + 1] - step_off[g];
      int32_t* gi = ridx + (int64_t)g * B;
      if (t < ns) {
        const int64_t s = step_off[g] + t;
        const int64_t n = idx_off[s + 1] - idx_off[s];
        if (n < 0 || n > B) return -1;
        std::memcpy(gi, idx_flat + idx_off[s], sizeof(int32_t) * n);
        for (int64_t k = n; k < B; ++k) gi[k] = -1;
        if (slot[s] < 0 || slot[s] >= max_slots) return -2;
        r_pn[g] = poison_n[s];
        r_trig[g] = trig[s];
        r_first[g] = first[s];
        r_act[g] = 1;
        r_nv[g] = (int32_t)n;
        r_slot[g] = slot[s];
        r_seed[g] = (int32_t)(dba_hash2(client_seed[g], (uint32_t)t) & 0x7fffffffU);
        std::memcpy(&r_lr[g], &lr[s], sizeof(float));
      } else {
        for (int k = 0; k < B; ++k) gi[k] = -1;
        r_pn[g] = 0; r_trig[g] = -1; r_first[g] = 0; r_act[g] = 0; r_nv[g] = 0;
        r_slot[g] = 0; r_seed[g] = 0; r_lr[g] = 0;
      }
    }
  }
  return 0;
}

// LPT: clients sorted by cost (desc, ties by index) go to the least-loaded rank
// (ties by lowest rank).  Deterministic: every rank computes the same placement.
void dba_lpt_assign(int n, const double* cost, int world, int32_t* owner, double* load_out) {
  std::vector<int> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cost[a] > cost[b]; });
  std::vector<double> load(world, 0.0);
  for (int i : order) {
    int best = 0;
    for (int r = 1; r < world; ++r)
      if (load[r] < load[best]) best = r;
    owner[i] = best;
    load[best] += cost[i];
  }
  if (load_out)
    for (int r = 0; r < world; ++r) load_out[r] = load[r];
}

// out = idx[rank::world]; returns the shard length.
int64_t dba_shard_index(const int64_t* idx, int64_t n, int rank, int world, int64_t* out) {
  int64_t k = 0;
  for (int64_t i = rank; i < n; i += world) out[k++] = idx[i];
  return k;
}

// Water-filling split of `work` units over ranks already carrying base[r] units in the same
// window: rank r gets share[r] = max(0, L - base[r]) / work with the level L chosen so the
// shares sum to 1 (the least-loaded ranks fill up first; a rank whose base alone exceeds the
// level gets nothing).  work <= 0: shares 1/world.  Deterministic (pure function of inputs):
// every rank computes the same shares.
void dba_balance_shares(int world, const double* base, double work, double* share) {
  if (world <= 0) return;
  if (!(work > 0.0)) {
    for (int r = 0; r < world; ++r) share[r] = 1.0 / world;
    return;
  }
  std::vector<double> b(base, base + world);
  std::sort(b.begin(), b.end());
  // the level lies between b[k-1] and b[k] for the first k with k*b[k] - sum(b[0..k)) >= work
  double level = 0.0, pref = 0.0;
  int k = 0;
  for (; k < world; ++k) {
    if (k > 0 && (double)k * b[k] - pref >= work) break;
    pref += b[k];
  }
  level = (work + pref) / k;
  double tot = 0.0;
  for (int r = 0; r < world; ++r) {
    share[r] = base[r] < level ? (level - base[r]) / work : 0.0;
    tot += share[r];
  }
  for (int r = 0; r < world; ++r) share[r] /= tot;   // exact sum 1 up to rounding
}

}  // extern "C"
