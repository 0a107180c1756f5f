// gen.cpp — seeded synthetic effect streams, host side.
//
// Workload utility for bench.py and the parity tests: SplitMix64 streams in
// global stream order, then a stable counting sort into CSR-by-key order (the
// order the host batcher hands to ccrdt_*_apply).  This is input generation,
// not a compute path of the engine.
#include <algorithm>
#include <thread>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/ccrdt.h"
#include "../../include/ccrdt_gen.h"

namespace {
inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
inline uint64_t h(uint64_t seed, uint64_t p, uint64_t j) { return splitmix64(seed * 0x100000001B3ull + p * 16 + j); }
}  // namespace

extern "C" {

uint64_t ccrdt_splitmix64(uint64_t x) { return splitmix64(x); }

// topk_rmv stream.  Per stream position p:
//   key ~ U[0,n_keys); rmv with probability rmv_pm/1000; origin dc ~ U[0,D)
//   whose clock ticks once per op it originates (ts starts at 1).
//   add: id ~ U[0,n_players), score ~ U[1,score_max], ts = clock[dc].
//     With probability dup_pm/1000 the add re-delivers the key's previous add
//     (same element: exercises set semantics and ts <= Vc paths).
//   rmv: id = one of the key's last 4 added ids (random id if none);
//     VcRmv[d] = max(0, clock[d] - U[0,lag_max)) (0 = absent).
// After grouping by key (stable), with probability swap_pm/1000 an op is
// swapped with its successor inside the key (out-of-order delivery).
// rmv ops carry ts = row index into rmv_vc (rows in CSR order).
// Every DC clock starts at clock0 (0 for a fresh stream): batch b of a long
// stream passes clock0 >= the clocks the earlier batches reached (e.g.
// b * n_ops), so timestamps keep rising across batches (steady state).
int64_t ccrdt_gen_trmv_count(int64_t n_ops, uint64_t seed, int rmv_pm) {
  int64_t n = 0;
  for (int64_t p = 0; p < n_ops; ++p) n += (int64_t)(h(seed, p, 1) % 1000) < rmv_pm;
  return n;
}

int ccrdt_gen_trmv(int64_t n_ops, int64_t n_keys, int n_dc, int64_t n_players, int64_t score_max,
                   int rmv_pm, int lag_max, int dup_pm, int swap_pm, uint64_t seed,
                   int64_t clock0, uint64_t* key_ptr, uint8_t* kind, int64_t* id, int64_t* score,
                   uint8_t* dc, int64_t* ts, int64_t* rmv_vc) {
  if (n_ops < 0 || n_keys <= 0 || n_dc < 1 || n_dc > 8 || n_players < 1 || score_max < 1 ||
      lag_max < 1 || clock0 < 0)
    return CCRDT_EINVAL;
  std::vector<uint32_t> key(n_ops);
  std::vector<uint64_t> cnt(n_keys + 1, 0);
  for (int64_t p = 0; p < n_ops; ++p) {
    key[p] = (uint32_t)(h(seed, p, 0) % (uint64_t)n_keys);
    cnt[key[p] + 1]++;
  }
  for (int64_t k = 0; k < n_keys; ++k) cnt[k + 1] += cnt[k];
  memcpy(key_ptr, cnt.data(), (n_keys + 1) * 8);
  std::vector<uint64_t> fill(cnt.begin(), cnt.end() - 1);
  std::vector<int64_t> clock(n_dc, clock0);
  std::vector<int64_t> recent(n_keys * 4, 0);   // last 4 added ids per key
  std::vector<uint32_t> nrecent(n_keys, 0);
  std::vector<int64_t> last_sc(n_keys, 0), last_ts(n_keys, 0);
  std::vector<uint8_t> last_dc(n_keys, 0), has_last(n_keys, 0);
  // rmv rows are assigned in CSR order after the scatter; keep their clocks
  // per position temporarily in rmv_vc order of stream first.
  std::vector<int64_t> rvc_stream;  // [n_rmv_stream][n_dc]
  for (int64_t p = 0; p < n_ops; ++p) {
    const uint32_t k = key[p];
    const uint64_t dst = fill[k]++;
    const bool is_rmv = (int64_t)(h(seed, p, 1) % 1000) < rmv_pm;
    const uint8_t d = (uint8_t)(h(seed, p, 2) % (uint64_t)n_dc);
    clock[d] += 1;
    if (!is_rmv) {
      const bool dup = has_last[k] && (int64_t)(h(seed, p, 6) % 1000) < dup_pm;
      int64_t pid, sc, t;
      uint8_t odc;
      if (dup) {
        pid = recent[k * 4 + ((nrecent[k] + 3) & 3)];
        sc = last_sc[k];
        t = last_ts[k];
        odc = last_dc[k];
      } else {
        pid = (int64_t)(h(seed, p, 3) % (uint64_t)n_players);
        sc = 1 + (int64_t)(h(seed, p, 4) % (uint64_t)score_max);
        t = clock[d];
        odc = d;
      }
      kind[dst] = (uint8_t)(h(seed, p, 5) & 1);  // add or add_r: same effect
      id[dst] = pid;
      score[dst] = sc;
      dc[dst] = odc;
      ts[dst] = t;
      if (!dup) {
        recent[k * 4 + (nrecent[k] & 3)] = pid;
        nrecent[k] += 1;
        has_last[k] = 1;
        last_sc[k] = sc;
        last_ts[k] = t;
        last_dc[k] = odc;
      }
    } else {
      const int have = nrecent[k] > 4 ? 4 : (int)nrecent[k];
      int64_t pid;
      if (have) pid = recent[k * 4 + (h(seed, p, 3) % (uint64_t)have)];
      else pid = (int64_t)(h(seed, p, 3) % (uint64_t)n_players);
      kind[dst] = (uint8_t)(2 + (h(seed, p, 5) & 1));
      id[dst] = pid;
      score[dst] = 0;
      dc[dst] = d;
      ts[dst] = (int64_t)(rvc_stream.size() / n_dc);
      for (int j = 0; j < n_dc; ++j) {
        int64_t v = clock[j] - (int64_t)(h(seed, p, 7 + j) % (uint64_t)lag_max);
        rvc_stream.push_back(v < 0 ? 0 : v);
      }
    }
  }
  // optional adjacent swaps inside keys (out-of-order delivery)
  if (swap_pm > 0) {
    for (int64_t k = 0; k < n_keys; ++k) {
      for (uint64_t i = key_ptr[k]; i + 1 < key_ptr[k + 1]; ++i) {
        if ((int64_t)(h(seed ^ 0x5A5A, i, 0) % 1000) < swap_pm) {
          std::swap(kind[i], kind[i + 1]);
          std::swap(id[i], id[i + 1]);
          std::swap(score[i], score[i + 1]);
          std::swap(dc[i], dc[i + 1]);
          std::swap(ts[i], ts[i + 1]);
          ++i;
        }
      }
    }
  }
  // renumber rmv rows into CSR order
  int64_t r = 0;
  for (int64_t i = 0; i < n_ops; ++i) {
    if (kind[i] >= 2) {
      const int64_t src = ts[i];
      memcpy(rmv_vc + r * n_dc, rvc_stream.data() + src * n_dc, 8 * n_dc);
      ts[i] = r++;
    }
  }
  return CCRDT_OK;
}

}  // extern "C"

namespace {
// Walker alias table for O(1) Zipf(1) rank draws.
struct Alias {
  std::vector<double> prob;
  std::vector<uint32_t> alias;
  explicit Alias(int64_t n) : prob(n), alias(n) {
    std::vector<double> w(n);
    double sum = 0;
    for (int64_t r = 0; r < n; ++r) sum += (w[r] = 1.0 / (double)(r + 1));
    std::vector<int64_t> small, large;
    for (int64_t r = 0; r < n; ++r) {
      prob[r] = w[r] * (double)n / sum;
      (prob[r] < 1.0 ? small : large).push_back(r);
    }
    while (!small.empty() && !large.empty()) {
      const int64_t s = small.back(), l = large.back();
      small.pop_back();
      alias[s] = (uint32_t)l;
      prob[l] -= 1.0 - prob[s];
      if (prob[l] < 1.0) {
        large.pop_back();
        small.push_back(l);
      }
    }
    for (int64_t r : small) prob[r] = 1.0;
    for (int64_t r : large) prob[r] = 1.0;
  }
};
}  // namespace

extern "C" int ccrdt_gen_corpus(int64_t n_docs, int64_t doc_bytes, int64_t vocab, uint64_t seed,
                                int threads, uint8_t* bytes, uint64_t* doc_off) {
  if (n_docs < 0 || doc_bytes < 0 || vocab < 1 || vocab > (int64_t)0xFFFFFFFF || !doc_off ||
      (n_docs * doc_bytes > 0 && !bytes))
    return CCRDT_EINVAL;
  // vocabulary: word r = 1..12 lowercase letters from its hash
  std::vector<uint64_t> woff(vocab + 1);
  std::vector<uint8_t> wchars;
  wchars.reserve((size_t)vocab * 7);
  for (int64_t r = 0; r < vocab; ++r) {
    woff[r] = wchars.size();
    uint64_t x = splitmix64(seed ^ (0xC0FFEEull + (uint64_t)r * 0x9E3779B97F4A7C15ull));
    const int len = 1 + (int)(x % 12);
    for (int c = 0; c < len; ++c) {
      x = splitmix64(x);
      wchars.push_back((uint8_t)('a' + x % 26));
    }
  }
  woff[vocab] = wchars.size();
  const Alias al(vocab);
  for (int64_t d = 0; d <= n_docs; ++d) doc_off[d] = (uint64_t)(d * doc_bytes);
  if (threads < 1) threads = 1;
  auto work = [&](int t) {
    for (int64_t d = t; d < n_docs; d += threads) {
      uint8_t* out = bytes + d * doc_bytes;
      uint64_t x = splitmix64(seed * 0x100000001B3ull + (uint64_t)d);
      int64_t pos = 0;
      while (pos < doc_bytes) {
        x = splitmix64(x);
        const uint64_t i = x % (uint64_t)vocab;
        const double u = (double)(x >> 11) * (1.0 / 9007199254740992.0);
        const uint64_t r = u < al.prob[i] ? i : al.alias[i];
        for (uint64_t c = woff[r]; c < woff[r + 1] && pos < doc_bytes; ++c) out[pos++] = wchars[c];
        x = splitmix64(x);
        if (pos < doc_bytes) out[pos++] = (x % 12 == 0) ? (uint8_t)'\n' : (uint8_t)' ';
        if (pos < doc_bytes && (x >> 32) % 100 == 0) out[pos++] = (uint8_t)' ';
      }
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  return CCRDT_OK;
}
