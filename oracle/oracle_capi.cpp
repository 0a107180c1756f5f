// oracle_capi.cpp — ctypes-callable C API over ccrdt_oracle.hpp.
//
// TEST INFRASTRUCTURE ONLY (parity checker and bench.py cpu_baseline leg).
// Batch layouts mirror include/ccrdt.h so the same arrays feed both sides.
#include <cstdint>
#include <cstring>
#include <string>
#include <memory>
#include <thread>
#include <vector>

#include "ccrdt_oracle.hpp"

using namespace ccrdt_oracle;

namespace {
struct TrmvSet {
  std::vector<std::unique_ptr<NodePool>> pools;  // one per worker thread (declared first:
                                                 // destroyed after the keys' nodes)
  std::vector<TopkRmv> keys;
  int D;
};
struct LbSet {
  std::vector<Leaderboard> keys;
};
struct TkSet {
  std::vector<Topk> keys;
};
struct AvgSet {
  std::vector<Average> keys;
};

// Static partition of the keys over n_threads std::threads.  With `pools`,
// worker t allocates its containers' nodes from (*pools)[t] (NodePool); a key
// stays with the same worker for the same n_threads.
template <class F>
void parallel_keys(int64_t n_keys, int n_threads, F f,
                   std::vector<std::unique_ptr<NodePool>>* pools = nullptr) {
  const int nt = (n_threads <= 1 || n_keys < 2) ? 1 : n_threads;
  if (pools)
    while ((int)pools->size() < nt) pools->push_back(std::make_unique<NodePool>());
  auto run = [&](int t, int64_t b, int64_t e) {
    NodePool* prev = tl_pool;
    tl_pool = pools ? (*pools)[t].get() : nullptr;
    f(b, e);
    tl_pool = prev;
  };
  if (nt == 1) {
    run(0, 0, n_keys);
    return;
  }
  std::vector<std::thread> th;
  const int64_t chunk = (n_keys + nt - 1) / nt;
  for (int t = 0; t < nt; ++t) {
    const int64_t b = t * chunk, e = std::min<int64_t>(n_keys, b + chunk);
    if (b >= e) break;
    th.emplace_back([=, &run] { run(t, b, e); });
  }
  for (auto& x : th) x.join();
}

Vc dense_to_vc(const int64_t* row, int D) {
  Vc v;
  for (int d = 0; d < D; ++d)
    if (row[d] != 0) v[d] = row[d];
  return v;
}
}  // namespace

extern "C" {

// ------------------------------------------------------------- topk_rmv
void* orc_trmv_create(int64_t n_keys, int64_t k, int n_dc) {
  auto* s = new TrmvSet();
  s->keys.assign(n_keys, TopkRmv(k));
  s->D = n_dc;
  return s;
}
void orc_trmv_destroy(void* h) { delete (TrmvSet*)h; }

// Same op layout as ccrdt_trmv_ops.  Extra effects are op-indexed
// (ex_kind = 255 for none); any ex_* pointer may be null.
int orc_trmv_apply(void* h, const uint64_t* key_ptr, const uint8_t* kind, const int64_t* id,
                   const int64_t* score, const uint8_t* dc, const int64_t* ts,
                   const int64_t* rmv_vc, int n_threads, uint8_t* ex_kind, int64_t* ex_id,
                   int64_t* ex_score, uint8_t* ex_dc, int64_t* ex_ts, int64_t* ex_vc) {
  auto* s = (TrmvSet*)h;
  const int D = s->D;
  parallel_keys((int64_t)s->keys.size(), n_threads, [&](int64_t b, int64_t e) {
    for (int64_t k = b; k < e; ++k) {
      TopkRmv& st = s->keys[k];
      for (uint64_t i = key_ptr[k]; i < key_ptr[k + 1]; ++i) {
        RExtra x;
        if (kind[i] <= 1) x = st.update_add(id[i], score[i], dc[i], ts[i]);
        else x = st.update_rmv(id[i], dense_to_vc(rmv_vc + ts[i] * D, D));
        if (ex_kind) ex_kind[i] = x.kind == R_NOOP ? 255 : (uint8_t)x.kind;
        if (x.kind == R_ADD) {
          if (ex_id) ex_id[i] = x.elem.id;
          if (ex_score) ex_score[i] = x.elem.score;
          if (ex_dc) ex_dc[i] = (uint8_t)x.elem.dc;
          if (ex_ts) ex_ts[i] = x.elem.ts;
        } else if (x.kind == R_RMV) {
          if (ex_id) ex_id[i] = x.id;
          if (ex_vc)
            for (int d = 0; d < D; ++d) ex_vc[i * D + d] = vc_get(x.vc, d);
        }
      }
    }
  }, &s->pools);
  return 0;
}

// (the export's passes run on every host CPU, at most 16: a 2^20-key state of
// 370M Masked elements took ~40 s on one thread)
int export_threads() {
  const unsigned hw = std::thread::hardware_concurrency();
  return (int)std::min<unsigned>(16u, hw ? hw : 1u);
}

// Per key: |Observed|, |Masked| (all Ids), |Removals|.
void trmv_key_counts(const TrmvSet* s, std::vector<uint64_t>& co, std::vector<uint64_t>& cm,
                     std::vector<uint64_t>& cr) {
  const int64_t nk = (int64_t)s->keys.size();
  co.assign(nk, 0);
  cm.assign(nk, 0);
  cr.assign(nk, 0);
  parallel_keys(nk, export_threads(), [&](int64_t b, int64_t e) {
    for (int64_t k = b; k < e; ++k) {
      const TopkRmv& st = s->keys[k];
      uint64_t m = 0;
      for (auto& [i, set] : st.masked) m += set.size();
      co[k] = st.obs.size();
      cm[k] = m;
      cr[k] = st.removals.size();
    }
  });
}

void orc_trmv_sizes(void* h, int64_t* n_obs, int64_t* n_masked, int64_t* n_rows) {
  auto* s = (TrmvSet*)h;
  std::vector<uint64_t> co, cm, cr;
  trmv_key_counts(s, co, cm, cr);
  int64_t o = 0, m = 0, r = 0;
  for (size_t k = 0; k < co.size(); ++k) {
    o += co[k];
    m += cm[k];
    r += cr[k];
  }
  *n_obs = o;
  *n_masked = m;
  *n_rows = r;
}

// Canonical image, same layout as ccrdt_trmv_state: the per-key offsets from
// one counting pass, then every key written in parallel.
void orc_trmv_export(void* h, int64_t* vc, uint64_t* obs_ptr, int64_t* obs_id, int64_t* obs_score,
                     uint8_t* obs_dc, int64_t* obs_ts, uint64_t* m_ptr, int64_t* m_id,
                     int64_t* m_score, uint8_t* m_dc, int64_t* m_ts, uint64_t* r_ptr, int64_t* r_id,
                     int64_t* r_vc, uint8_t* min_valid, int64_t* min_id, int64_t* min_score,
                     uint8_t* min_dc, int64_t* min_ts) {
  auto* s = (TrmvSet*)h;
  const int D = s->D;
  const int64_t nk = (int64_t)s->keys.size();
  std::vector<uint64_t> co, cm, cr;
  trmv_key_counts(s, co, cm, cr);
  obs_ptr[0] = m_ptr[0] = r_ptr[0] = 0;
  for (int64_t k = 0; k < nk; ++k) {
    obs_ptr[k + 1] = obs_ptr[k] + co[k];
    m_ptr[k + 1] = m_ptr[k] + cm[k];
    r_ptr[k + 1] = r_ptr[k] + cr[k];
  }
  parallel_keys(nk, export_threads(), [&](int64_t b, int64_t e) {
    for (int64_t k = b; k < e; ++k) {
      const TopkRmv& st = s->keys[k];
      uint64_t po = obs_ptr[k], pm = m_ptr[k], pr = r_ptr[k];
      for (int d = 0; d < D; ++d) vc[k * D + d] = vc_get(st.vc, d);
      for (auto& [i, el] : st.obs) {  // std::map: sorted by id
        obs_id[po] = el.id;
        obs_score[po] = el.score;
        obs_dc[po] = (uint8_t)el.dc;
        obs_ts[po] = el.ts;
        ++po;
      }
      for (auto& [i, set] : st.masked) {  // by id, then term order inside
        for (auto& el : set) {
          m_id[pm] = el.id;
          m_score[pm] = el.score;
          m_dc[pm] = (uint8_t)el.dc;
          m_ts[pm] = el.ts;
          ++pm;
        }
      }
      for (auto& [i, v] : st.removals) {
        r_id[pr] = i;
        for (int d = 0; d < D; ++d) r_vc[pr * D + d] = vc_get(v, d);
        ++pr;
      }
      min_valid[k] = st.min ? 1 : 0;
      min_id[k] = st.min ? st.min->id : 0;
      min_score[k] = st.min ? st.min->score : 0;
      min_dc[k] = st.min ? (uint8_t)st.min->dc : 0;
      min_ts[k] = st.min ? st.min->ts : 0;
    }
  });
}

// downstream/2: op 0 add (dc, ts supplied), 1 rmv.  out_kind: 0 add 1 add_r
// 2 rmv 3 rmv_r 255 noop.
void orc_trmv_downstream(void* h, int64_t n, const uint64_t* key, const uint8_t* op,
                         const int64_t* id, const int64_t* score, const uint8_t* dc,
                         const int64_t* ts, uint8_t* out_kind) {
  auto* s = (TrmvSet*)h;
  for (int64_t i = 0; i < n; ++i) {
    const TopkRmv& st = s->keys[key[i]];
    int r = op[i] == 0 ? st.downstream_add(id[i], score[i], dc[i], ts[i]) : st.downstream_rmv(id[i]);
    out_kind[i] = r == R_NOOP ? 255 : (uint8_t)r;
  }
}

}  // extern "C"

// ================================================================ others
extern "C" {

// ---------------------------------------------------------------- average
// update/2 over a CSR batch; sum/num are in-out [n_keys].  Returns 1 if an op
// would crash the reference (N < 0: no function clause), else 0.
int orc_avg_apply(int64_t n_keys, const uint64_t* key_ptr, const int64_t* v, const int64_t* n,
                  int64_t* sum, int64_t* num) {
  for (int64_t k = 0; k < n_keys; ++k) {
    Average a;
    a.sum = sum[k];
    a.num = num[k];
    for (uint64_t i = key_ptr[k]; i < key_ptr[k + 1]; ++i)
      if (!a.add(v[i], n[i])) return 1;
    sum[k] = a.sum;
    num[k] = a.num;
  }
  return 0;
}
double orc_avg_value(int64_t sum, int64_t num) {
  Average a;
  a.sum = sum;
  a.num = num;
  return a.value();
}

// ------------------------------------------------------------------- topk
void* orc_topk_create(int64_t n_keys, int64_t k) { return new TkSet{std::vector<Topk>(n_keys, Topk(k))}; }
void orc_topk_destroy(void* h) { delete (TkSet*)h; }
void orc_topk_apply(void* h, const uint64_t* key_ptr, const int64_t* id, const int64_t* score) {
  auto* s = (TkSet*)h;
  for (size_t k = 0; k < s->keys.size(); ++k)
    for (uint64_t i = key_ptr[k]; i < key_ptr[k + 1]; ++i) s->keys[k].add(id[i], score[i]);
}
int64_t orc_topk_size(void* h) {
  int64_t n = 0;
  for (auto& t : ((TkSet*)h)->keys) n += t.top.size();
  return n;
}
// state sorted by id (sorted=0) or value/1 order (sorted=1)
void orc_topk_export(void* h, int value_order, uint64_t* ptr, int64_t* id, int64_t* score) {
  auto* s = (TkSet*)h;
  uint64_t p = 0;
  ptr[0] = 0;
  for (size_t k = 0; k < s->keys.size(); ++k) {
    auto v = value_order ? s->keys[k].value()
                         : std::vector<std::pair<i64, i64>>(s->keys[k].top.begin(), s->keys[k].top.end());
    for (auto& [i, sc] : v) {
      id[p] = i;
      score[p] = sc;
      ++p;
    }
    ptr[k + 1] = p;
  }
}

// ------------------------------------------------------------ leaderboard
void* orc_lb_create(int64_t n_keys, int64_t k) { return new LbSet{std::vector<Leaderboard>(n_keys, Leaderboard(k))}; }
void orc_lb_destroy(void* h) { delete (LbSet*)h; }
// kind 0 add, 1 add_r, 2 ban; ex_kind 255 none / 0 {add, {Id, Score}}
void orc_lb_apply(void* h, const uint64_t* key_ptr, const uint8_t* kind, const int64_t* id,
                  const int64_t* score, uint8_t* ex_kind, int64_t* ex_id, int64_t* ex_score) {
  auto* s = (LbSet*)h;
  for (size_t k = 0; k < s->keys.size(); ++k)
    for (uint64_t i = key_ptr[k]; i < key_ptr[k + 1]; ++i) {
      LExtra x = kind[i] == 2 ? s->keys[k].ban(id[i]) : s->keys[k].add(id[i], score[i]);
      if (ex_kind) ex_kind[i] = x.kind == L_ADD ? 0 : 255;
      if (x.kind == L_ADD) {
        if (ex_id) ex_id[i] = x.elem.id;
        if (ex_score) ex_score[i] = x.elem.score;
      }
    }
}
// The same fold with the boards split over n_threads threads (boards are
// independent objects: leaderboard.erl:215-286 touches one board per op).
void orc_lb_apply_mt(void* h, const uint64_t* key_ptr, const uint8_t* kind, const int64_t* id,
                     const int64_t* score, uint8_t* ex_kind, int64_t* ex_id, int64_t* ex_score, int n_threads) {
  auto* s = (LbSet*)h;
  if (n_threads < 1) n_threads = 1;
  const size_t nk = s->keys.size();
  std::vector<std::thread> th;
  for (int t = 0; t < n_threads; ++t)
    th.emplace_back([&, t] {
      for (size_t k = nk * t / n_threads; k < nk * (t + 1) / n_threads; ++k)
        for (uint64_t i = key_ptr[k]; i < key_ptr[k + 1]; ++i) {
          LExtra x = kind[i] == 2 ? s->keys[k].ban(id[i]) : s->keys[k].add(id[i], score[i]);
          if (ex_kind) ex_kind[i] = x.kind == L_ADD ? 0 : 255;
          if (x.kind == L_ADD) {
            if (ex_id) ex_id[i] = x.elem.id;
            if (ex_score) ex_score[i] = x.elem.score;
          }
        }
    });
  for (auto& x : th) x.join();
}
void orc_lb_sizes(void* h, int64_t* n_obs, int64_t* n_masked, int64_t* n_bans) {
  int64_t o = 0, m = 0, b = 0;
  for (auto& l : ((LbSet*)h)->keys) {
    o += l.obs.size();
    m += l.masked.size();
    b += l.bans.size();
  }
  *n_obs = o;
  *n_masked = m;
  *n_bans = b;
}
void orc_lb_export(void* h, uint64_t* obs_ptr, int64_t* obs_id, int64_t* obs_score, uint64_t* m_ptr,
                   int64_t* m_id, int64_t* m_score, uint64_t* b_ptr, int64_t* b_id, uint8_t* min_valid,
                   int64_t* min_id, int64_t* min_score) {
  auto* s = (LbSet*)h;
  uint64_t po = 0, pm = 0, pb = 0;
  obs_ptr[0] = m_ptr[0] = b_ptr[0] = 0;
  for (size_t k = 0; k < s->keys.size(); ++k) {
    const Leaderboard& l = s->keys[k];
    for (auto& [i, sc] : l.obs) {
      obs_id[po] = i;
      obs_score[po++] = sc;
    }
    for (auto& [i, sc] : l.masked) {
      m_id[pm] = i;
      m_score[pm++] = sc;
    }
    for (auto i : l.bans) b_id[pb++] = i;
    obs_ptr[k + 1] = po;
    m_ptr[k + 1] = pm;
    b_ptr[k + 1] = pb;
    min_valid[k] = l.min ? 1 : 0;
    min_id[k] = l.min ? l.min->id : 0;
    min_score[k] = l.min ? l.min->score : 0;
  }
}
// op 0 add, 1 ban; out 0 add, 1 add_r, 2 ban, 255 noop
void orc_lb_downstream(void* h, int64_t n, const uint64_t* key, const uint8_t* op, const int64_t* id,
                       const int64_t* score, uint8_t* out) {
  auto* s = (LbSet*)h;
  for (int64_t i = 0; i < n; ++i) {
    const Leaderboard& l = s->keys[key[i]];
    const int r = op[i] == 0 ? l.downstream_add(id[i], score[i]) : l.downstream_ban(id[i]);
    out[i] = r == L_NOOP ? 255 : (uint8_t)r;
  }
}
// cmp/2, min/1, get_largest/1 on explicit arguments (golden vectors)
int orc_lb_cmp(int a_nil, int64_t a_id, int64_t a_sc, int b_nil, int64_t b_id, int64_t b_sc) {
  std::optional<LPair> a, b;
  if (!a_nil) a = LPair{a_id, a_sc};
  if (!b_nil) b = LPair{b_id, b_sc};
  return lb_cmp(a, b) ? 1 : 0;
}
int orc_lb_minmax(int largest, int64_t n, const int64_t* id, const int64_t* sc, int64_t* out_id,
                  int64_t* out_sc) {
  std::map<i64, i64> m;
  for (int64_t i = 0; i < n; ++i) m[id[i]] = sc[i];
  auto r = largest ? Leaderboard::get_largest(m) : Leaderboard::lb_min(m);
  if (!r) return 0;
  *out_id = r->id;
  *out_sc = r->score;
  return 1;
}

// ------------------------------------------------ wordcount / worddocumentcount
struct WcSet {
  int wdc;
  std::vector<std::map<std::string, i64>> keys;
};
void* orc_wc_create(int64_t n_keys, int wdc) { return new WcSet{wdc, std::vector<std::map<std::string, i64>>(n_keys)}; }
void orc_wc_destroy(void* h) { delete (WcSet*)h; }
// key_ptr[n_keys+1] over docs; doc_off[n_docs+1] over bytes
void orc_wc_apply(void* h, const uint64_t* key_ptr, const uint64_t* doc_off, const uint8_t* bytes) {
  auto* s = (WcSet*)h;
  for (size_t k = 0; k < s->keys.size(); ++k)
    for (uint64_t d = key_ptr[k]; d < key_ptr[k + 1]; ++d) {
      std::string f((const char*)bytes + doc_off[d], doc_off[d + 1] - doc_off[d]);
      if (s->wdc) {
        WordDocCount w;
        w.counts.swap(s->keys[k]);
        w.add(f);
        w.counts.swap(s->keys[k]);
      } else {
        Wordcount w;
        w.counts.swap(s->keys[k]);
        w.add(f);
        w.counts.swap(s->keys[k]);
      }
    }
}
// The same fold with each key's documents split over n_threads threads: every
// thread folds add/2 over its documents into a map of its own (the +1s of
// wordcount.erl:78-85 / worddocumentcount.erl:78-86 commute), then the maps
// are summed into the key's map.  Used for the corpus-sized parity tests.
void orc_wc_apply_mt(void* h, const uint64_t* key_ptr, const uint64_t* doc_off, const uint8_t* bytes,
                     int n_threads) {
  auto* s = (WcSet*)h;
  if (n_threads < 1) n_threads = 1;
  for (size_t k = 0; k < s->keys.size(); ++k) {
    const uint64_t d0 = key_ptr[k], d1 = key_ptr[k + 1];
    std::vector<std::map<std::string, i64>> part(n_threads);
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t)
      th.emplace_back([&, t] {
        for (uint64_t d = d0 + t; d < d1; d += n_threads) {
          std::string f((const char*)bytes + doc_off[d], doc_off[d + 1] - doc_off[d]);
          if (s->wdc) {
            WordDocCount w;
            w.counts.swap(part[t]);
            w.add(f);
            w.counts.swap(part[t]);
          } else {
            Wordcount w;
            w.counts.swap(part[t]);
            w.add(f);
            w.counts.swap(part[t]);
          }
        }
      });
    for (auto& x : th) x.join();
    for (auto& m : part)
      for (auto& [w, c] : m) s->keys[k][w] += c;
  }
}
void orc_wc_sizes(void* h, int64_t* n_words, int64_t* n_bytes) {
  int64_t w = 0, b = 0;
  for (auto& m : ((WcSet*)h)->keys)
    for (auto& [s, c] : m) {
      ++w;
      b += (int64_t)s.size();
    }
  *n_words = w;
  *n_bytes = b;
}
// words sorted by bytes (std::string order = Erlang binary order) per key
void orc_wc_export(void* h, uint64_t* key_ptr, uint64_t* word_off, uint8_t* bytes, int64_t* count) {
  auto* s = (WcSet*)h;
  uint64_t w = 0, b = 0;
  key_ptr[0] = 0;
  word_off[0] = 0;
  for (size_t k = 0; k < s->keys.size(); ++k) {
    for (auto& [str, c] : s->keys[k]) {
      memcpy(bytes + b, str.data(), str.size());
      b += str.size();
      count[w] = c;
      word_off[++w] = b;
    }
    key_ptr[k + 1] = w;
  }
}

}  // extern "C"
