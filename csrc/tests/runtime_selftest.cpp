// Host self-test of the native runtime, built with -fsanitize=address,undefined by
// tests/test_native_sanitize.py (sanitizer runs on the host code).
// Exercises every entry point on randomized schedules, including malformed ones, and checks
// the packed descriptor rows against a straightforward re-derivation.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

extern "C" {
int dba_runtime_version();
uint32_t dba_hash2(uint32_t seed, uint32_t counter);
int dba_pack_steps(int G, int B, int T, int max_slots, const int64_t* step_off, const int64_t* idx_off,
                   const int32_t* idx_flat, const int32_t* poison_n, const int32_t* trig, const int32_t* first,
                   const int32_t* slot, const float* lr, const uint32_t* client_seed, int32_t* out);
void dba_lpt_assign(int n, const double* cost, int world, int32_t* owner, double* load_out);
int64_t dba_shard_index(const int64_t* idx, int64_t n, int rank, int world, int64_t* out);
}

#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "FAILED %s at %s:%d\n", #c, __FILE__, __LINE__); \
      return 1;                                                          \
    }                                                                    \
  } while (0)

int main() {
  std::mt19937 rng(1234);
  CHECK(dba_runtime_version() >= 3);
  for (int trial = 0; trial < 200; ++trial) {
    const int G = 1 + rng() % 12, B = 1 + rng() % 64, max_slots = 1 + rng() % 8;
    std::vector<int64_t> step_off(G + 1, 0);
    for (int g = 0; g < G; ++g) step_off[g + 1] = step_off[g] + (int64_t)(rng() % 20);
    const int64_t S = step_off[G];
    int T = 0;
    for (int g = 0; g < G; ++g) T = std::max<int>(T, (int)(step_off[g + 1] - step_off[g]));
    std::vector<int64_t> idx_off(S + 1, 0);
    for (int64_t s = 0; s < S; ++s) idx_off[s + 1] = idx_off[s] + 1 + rng() % B;
    std::vector<int32_t> idx(std::max<int64_t>(1, idx_off[S]));
    for (auto& v : idx) v = (int32_t)(rng() % 50000);
    std::vector<int32_t> pn(std::max<int64_t>(1, S)), trig(pn.size()), first(pn.size()), slot(pn.size());
    std::vector<float> lr(pn.size());
    for (int64_t s = 0; s < S; ++s) {
      pn[s] = rng() % 6; trig[s] = (int)(rng() % 5) - 1; first[s] = rng() % 2; slot[s] = rng() % max_slots;
      lr[s] = 0.001f * (1 + rng() % 100);
    }
    std::vector<uint32_t> seeds(G);
    for (auto& v : seeds) v = rng();
    const int64_t D = (int64_t)G * B + 8LL * G;
    std::vector<int32_t> out((size_t)std::max(T, 1) * D, 0x55555555);
    CHECK(dba_pack_steps(G, B, T, max_slots, step_off.data(), idx_off.data(), idx.data(), pn.data(), trig.data(),
                         first.data(), slot.data(), lr.data(), seeds.data(), out.data()) == 0);
    for (int t = 0; t < T; ++t)
      for (int g = 0; g < G; ++g) {
        const int32_t* row = out.data() + (int64_t)t * D;
        const int32_t* f = row + (int64_t)G * B;
        const int64_t ns = step_off[g + 1] - step_off[g];
        if (t < ns) {
          const int64_t s = step_off[g] + t, n = idx_off[s + 1] - idx_off[s];
          CHECK(f[3 * G + g] == 1 && f[4 * G + g] == n && f[g] == pn[s] && f[G + g] == trig[s]);
          CHECK(std::memcmp(row + (int64_t)g * B, idx.data() + idx_off[s], n * 4) == 0);
          for (int64_t k = n; k < B; ++k) CHECK(row[(int64_t)g * B + k] == -1);
          float l;
          std::memcpy(&l, &f[7 * G + g], 4);
          CHECK(l == lr[s]);
          CHECK(f[6 * G + g] == (int32_t)(dba_hash2(seeds[g], (uint32_t)t) & 0x7fffffffU));
        } else {
          CHECK(f[3 * G + g] == 0 && f[4 * G + g] == 0 && f[G + g] == -1);
        }
      }
    // malformed: a slot out of range must be rejected, not written past
    if (S > 0) {
      slot[0] = max_slots;
      CHECK(dba_pack_steps(G, B, T, max_slots, step_off.data(), idx_off.data(), idx.data(), pn.data(), trig.data(),
                           first.data(), slot.data(), lr.data(), seeds.data(), out.data()) == -2);
    }
  }
  // LPT: every client placed, loads add up, deterministic
  for (int trial = 0; trial < 100; ++trial) {
    const int n = 1 + rng() % 40, world = 1 + rng() % 8;
    std::vector<double> cost(n);
    for (auto& c : cost) c = 1 + rng() % 1000;
    std::vector<int32_t> own(n, -1), own2(n, -1);
    std::vector<double> load(world), load2(world);
    dba_lpt_assign(n, cost.data(), world, own.data(), load.data());
    dba_lpt_assign(n, cost.data(), world, own2.data(), load2.data());
    double tot = 0, ltot = 0;
    for (int i = 0; i < n; ++i) { CHECK(own[i] >= 0 && own[i] < world && own[i] == own2[i]); tot += cost[i]; }
    for (double l : load) ltot += l;
    CHECK(tot == ltot);
  }
  // sharding covers every element exactly once
  for (int world = 1; world <= 8; ++world) {
    const int64_t n = 1000 + world;
    std::vector<int64_t> idx(n), out(n), seen(n, 0);
    for (int64_t i = 0; i < n; ++i) idx[i] = i;
    for (int r = 0; r < world; ++r) {
      const int64_t k = dba_shard_index(idx.data(), n, r, world, out.data());
      for (int64_t i = 0; i < k; ++i) seen[out[i]]++;
    }
    for (int64_t i = 0; i < n; ++i) CHECK(seen[i] == 1);
  }
  std::printf("runtime selftest OK\n");
  return 0;
}
