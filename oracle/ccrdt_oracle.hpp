// ccrdt_oracle.hpp — CPU restatement of antidote_ccrdt's six CCRDT types.
//
// TEST INFRASTRUCTURE ONLY.  This header is the parity oracle: tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg are the only
// callers.  The product path (antidote_ccrdt_amd/, libccrdt.so) never links
// or calls it, and has no CPU fallback.
//
// It restates the Erlang reference faithfully, using mutable ordered
// containers in place of the reference's persistent maps / gb_sets / sets:
//   * std::map<K,V>      ~ maps   (iteration order is irrelevant to every
//                                  result except value/1 list order, Q7,
//                                  which parity compares canonically)
//   * std::set<Elem>     ~ gb_sets with Erlang term order
//   * std::map<dc, ts>   ~ vc()   (sparse, missing => 0)
// DcIds are integer ranks that preserve Erlang term order between DcIds
// (SURVEY §8a Q1).  Tuple timestamps {0,0,n} of the reference tests map to n.
//
// Reference: /root/reference/src/antidote_ccrdt_*.erl (file:line cited at
// every function).  The reference cannot be compiled or run here (no
// erl/erlc/escript); parity is pinned by the reference's own EUnit vectors
// transcribed under tests/golden/ (see tests/golden/make_golden.py).
#pragma once
#include <algorithm>
#include <cstdint>
#include <map>
#include <optional>
#include <set>
#include <string>
#include <vector>

namespace ccrdt_oracle {
using i64 = int64_t;

// ===================================================================
// topk_rmv   (src/antidote_ccrdt_topk_rmv.erl)
// ===================================================================

// pair_internal() = {Score, Id, {DcId, Ts}}   (topk_rmv.erl:60)
// Field order below is the Erlang term order of that tuple.
struct RElem {
  i64 score;
  i64 id;
  int dc;
  i64 ts;
  bool operator<(const RElem& o) const {
    if (score != o.score) return score < o.score;
    if (id != o.id) return id < o.id;
    if (dc != o.dc) return dc < o.dc;
    return ts < o.ts;
  }
  bool operator==(const RElem& o) const {
    return score == o.score && id == o.id && dc == o.dc && ts == o.ts;
  }
};
// Node pools for the topk_rmv containers.  bench.py's threaded CPU baseline
// partitions keys over threads; with the default allocator every thread's
// map/set nodes go through glibc malloc.  A thread whose tl_pool is set
// (oracle_capi.cpp sets one per worker, owned by the oracle instance) takes
// nodes from its own chunks and recycles them on its own free lists; other
// threads use the heap.  A 16-byte header records the source.
struct NodePool {
  static constexpr size_t CHUNK = size_t(1) << 20;
  std::vector<char*> chunks;
  char* cur = nullptr;
  size_t left = 0;
  void* freel[16] = {};  // by 16-byte size class, blocks of <= 256 bytes
  NodePool() = default;
  NodePool(const NodePool&) = delete;
  NodePool& operator=(const NodePool&) = delete;
  ~NodePool() {
    for (char* c : chunks) ::operator delete(c);
  }
  void* get(size_t n) {
    const size_t cls = n / 16 - 1;
    if (freel[cls]) {
      void* p = freel[cls];
      freel[cls] = *(void**)p;
      return p;
    }
    if (left < n) {
      cur = (char*)::operator new(CHUNK);
      chunks.push_back(cur);
      left = CHUNK;
    }
    void* p = cur;
    cur += n;
    left -= n;
    return p;
  }
  void put(void* p, size_t n) {
    const size_t cls = n / 16 - 1;
    *(void**)p = freel[cls];
    freel[cls] = p;
  }
};
inline thread_local NodePool* tl_pool = nullptr;

template <class T>
struct PoolAlloc {
  using value_type = T;
  PoolAlloc() = default;
  template <class U>
  PoolAlloc(const PoolAlloc<U>&) {}
  T* allocate(size_t n) {
    const size_t bytes = (n * sizeof(T) + 16 + 15) & ~size_t(15);
    char* p;
    if (tl_pool && bytes <= 256) {
      p = (char*)tl_pool->get(bytes);
      *(uint64_t*)p = bytes;
    } else {
      p = (char*)::operator new(bytes);
      *(uint64_t*)p = 0;
    }
    return (T*)(p + 16);
  }
  void deallocate(T* t, size_t) {
    char* p = (char*)t - 16;
    const uint64_t h = *(uint64_t*)p;
    if (!h) ::operator delete(p);
    else if (tl_pool) tl_pool->put(p, h);  // else: freed with its pool
  }
  template <class U>
  bool operator==(const PoolAlloc<U>&) const { return true; }
  template <class U>
  bool operator!=(const PoolAlloc<U>&) const { return false; }
};
template <class K, class V>
using PMap = std::map<K, V, std::less<K>, PoolAlloc<std::pair<const K, V>>>;
template <class T>
using PSet = std::set<T, std::less<T>, PoolAlloc<T>>;

using Vc = PMap<int, i64>;

// cmp/2 (topk_rmv.erl:389-395): strict > on (Score, Id, Ts); DcId ignored.
// nil is std::nullopt: cmp(nil,_) = false, cmp(_,nil) = true.
inline bool rmv_cmp(const std::optional<RElem>& a, const std::optional<RElem>& b) {
  if (!a) return false;
  if (!b) return true;
  return a->score > b->score || (a->score == b->score && a->id > b->id) ||
         (a->score == b->score && a->id == b->id && a->ts > b->ts);
}

// vc_get_timestamp/2 (topk_rmv.erl:350-355): missing => 0.
inline i64 vc_get(const Vc& vc, int dc) {
  auto it = vc.find(dc);
  return it == vc.end() ? 0 : it->second;
}
// vc_update/3 (topk_rmv.erl:358-366).
inline void vc_update(Vc& vc, int dc, i64 ts) {
  auto it = vc.find(dc);
  if (it == vc.end()) vc[dc] = ts;
  else it->second = std::max(ts, it->second);
}
// merge_vcs/2 (topk_rmv.erl:378-386): fold Vc2 into Vc1, elementwise max,
// union of keys.
inline Vc merge_vcs(const Vc& vc1, const Vc& vc2) {
  Vc acc = vc1;
  for (const auto& [k, ts] : vc2) {
    auto it = acc.find(k);
    if (it == acc.end()) acc[k] = ts;
    else it->second = std::max(ts, it->second);
  }
  return acc;
}

// Effect kinds of topk_rmv (topk_rmv.erl:77-78).
enum RKind { R_ADD = 0, R_ADD_R = 1, R_RMV = 2, R_RMV_R = 3, R_NOOP = 4 };

// An extra effect returned by update/2 as {ok, State, [Effect]}:
// kind R_ADD  -> {add, {Id, Score, {Dc, Ts}}}           (topk_rmv.erl:295)
// kind R_RMV  -> {rmv, {Id, Removals[Id]}}               (topk_rmv.erl:237)
// kind R_NOOP -> {ok, State} (no extra effect)
struct RExtra {
  int kind = R_NOOP;
  RElem elem{};
  i64 id = 0;
  Vc vc;
};

// topkrmv() state (topk_rmv.erl:67-74).
struct TopkRmv {
  PMap<i64, RElem> obs;                  // Observed
  PMap<i64, PSet<RElem>> masked;         // Masked
  PMap<i64, Vc> removals;                // Removals
  Vc vc;                                 // replica Vc
  std::optional<RElem> min;              // Min ({nil,nil,nil} = nullopt)
  i64 size;                              // Size

  // new/1 (topk_rmv.erl:86-88); new/0 uses 100 (topk_rmv.erl:81-83).
  explicit TopkRmv(i64 k = 100) : size(k) {}

  // min_observed/1 (topk_rmv.erl:398-406): term-order smallest Obs value.
  std::optional<RElem> min_observed(const PMap<i64, RElem>& o) const {
    if (o.empty()) return std::nullopt;
    RElem best = o.begin()->second;
    for (const auto& [k, e] : o)
      if (e < best) best = e;
    return best;
  }

  // recompute_observed/5 (topk_rmv.erl:301-334).
  void recompute_observed(i64 id, const RElem& elem) {
    auto it = obs.find(id);
    if (it != obs.end()) {
      RElem old = it->second;
      if (rmv_cmp(elem, old)) {
        it->second = elem;
        if (min && old == *min) min = min_observed(obs);
      }
      return;
    }
    if ((i64)obs.size() < size) {
      obs[id] = elem;
      if (rmv_cmp(min, elem) || !min) min = elem;
      return;
    }
    if (rmv_cmp(elem, min)) {
      i64 min_id = min->id;
      obs.erase(min_id);
      obs[id] = elem;
      min = min_observed(obs);
    }
  }

  // add/4 (topk_rmv.erl:231-249).
  RExtra add(i64 id, i64 score, int dc, i64 ts) {
    RExtra ex;
    vc_update(vc, dc, ts);
    auto rit = removals.find(id);
    Vc rvc = rit == removals.end() ? Vc{} : rit->second;  // removals_get_vc :342-347
    if (vc_get(rvc, dc) >= ts) {                           // :234
      ex.kind = R_RMV;
      ex.id = id;
      ex.vc = rvc;
      return ex;
    }
    RElem e{score, id, dc, ts};
    masked[id].insert(e);  // gb_sets:add_element / singleton (:240-246)
    recompute_observed(id, e);
    return ex;
  }

  // rmv/3 (topk_rmv.erl:252-298).
  RExtra rmv(i64 id, const Vc& vc_rmv) {
    RExtra ex;
    // merge_vc/3 (:369-375)
    {
      auto it = removals.find(id);
      if (it == removals.end()) removals[id] = vc_rmv;
      else it->second = merge_vcs(it->second, vc_rmv);
    }
    // filter masked (:255-266)
    auto mit = masked.find(id);
    if (mit != masked.end()) {
      PSet<RElem> keep;
      for (const auto& e : mit->second)
        if (e.ts > vc_get(vc_rmv, e.dc)) keep.insert(e);
      if (keep.empty()) masked.erase(mit);
      else mit->second = std::move(keep);
    }
    // impacts observed? (:267-272)
    auto oit = obs.find(id);
    bool impacts = oit != obs.end() && vc_get(vc_rmv, oit->second.dc) >= oit->second.ts;
    if (!impacts) return ex;
    RElem removed = oit->second;
    obs.erase(oit);  // TmpObserved
    // Values = {largest(S) | I in NewMasked, I not in TmpObserved} (:276-281)
    std::optional<RElem> best;
    for (const auto& [i, s] : masked) {
      if (obs.count(i)) continue;
      const RElem& l = *s.rbegin();  // gb_sets:largest
      if (!best || *best < l) best = l;
    }
    if (!best) {  // (:283-289)
      if (min && removed == *min) min = min_observed(obs);
      return ex;
    }
    obs[best->id] = *best;  // (:291-295)
    min = min_observed(obs);
    ex.kind = R_ADD;
    ex.elem = *best;
    return ex;
  }

  // update/2 (topk_rmv.erl:140-148): add|add_r -> add/4, rmv|rmv_r -> rmv/3.
  RExtra update_add(i64 id, i64 score, int dc, i64 ts) { return add(id, score, dc, ts); }
  RExtra update_rmv(i64 id, const Vc& v) { return rmv(id, v); }

  // downstream/2 for {add, {Id, Score}} (topk_rmv.erl:103-115).  The host
  // supplies the DC rank and the clock value (?DC_META_DATA / ?TIME).
  int downstream_add(i64 id, i64 score, int dc, i64 ts) const {
    RElem e{score, id, dc, ts};
    auto it = obs.find(id);
    bool changes = it != obs.end() ? rmv_cmp(e, it->second) : rmv_cmp(e, min);
    return changes ? R_ADD : R_ADD_R;
  }
  // downstream/2 for {rmv, Id} (topk_rmv.erl:116-124): payload is the whole
  // replica Vc.
  int downstream_rmv(i64 id) const {
    if (!masked.count(id)) return R_NOOP;
    return obs.count(id) ? R_RMV : R_RMV_R;
  }

  // value/1 (topk_rmv.erl:91-95) — returned here sorted by Id (canonical).
  std::vector<std::pair<i64, i64>> value() const {
    std::vector<std::pair<i64, i64>> v;
    for (const auto& [k, e] : obs) v.push_back({e.id, e.score});
    return v;
  }
  // equal/2 (topk_rmv.erl:151-153).
  bool equal(const TopkRmv& o) const {
    if (size != o.size || obs.size() != o.obs.size()) return false;
    for (const auto& [k, e] : obs) {
      auto it = o.obs.find(k);
      if (it == o.obs.end() || !(it->second == e)) return false;
    }
    return true;
  }
};

// ===================================================================
// leaderboard   (src/antidote_ccrdt_leaderboard.erl)
// ===================================================================
struct LPair {  // pair() = {PlayerId, Score}
  i64 id, score;
  bool operator==(const LPair& o) const { return id == o.id && score == o.score; }
};
// cmp/2 (leaderboard.erl:289-294)
inline bool lb_cmp(const std::optional<LPair>& a, const std::optional<LPair>& b) {
  if (!a) return false;
  if (!b) return true;
  return a->score > b->score || (a->score == b->score && a->id > b->id);
}
enum LKind { L_ADD = 0, L_ADD_R = 1, L_BAN = 2, L_NOOP = 3 };
struct LExtra {
  int kind = L_NOOP;  // L_ADD -> {add, {Id, Score}} (leaderboard.erl:283)
  LPair elem{};
};
struct Leaderboard {
  std::map<i64, i64> obs, masked;
  std::set<i64> bans;
  std::optional<LPair> min;
  i64 size;
  explicit Leaderboard(i64 k = 100) : size(k) {}  // new/0,1 (:75-81)

  // min/1 (:297-303): head of lists:sort by cmp(Y,X) = smallest by (Score,Id)
  static std::optional<LPair> lb_min(const std::map<i64, i64>& m) {
    std::optional<LPair> best;
    for (const auto& [i, s] : m) {
      LPair p{i, s};
      if (!best || lb_cmp(*best, p)) best = p;
    }
    return best;
  }
  // get_largest/1 (:306-312): largest by (Score, Id)
  static std::optional<LPair> get_largest(const std::map<i64, i64>& m) {
    std::optional<LPair> best;
    for (const auto& [i, s] : m) {
      LPair p{i, s};
      if (!best || lb_cmp(p, *best)) best = p;
    }
    return best;
  }
  // add/3 (:215-261)
  LExtra add(i64 id, i64 score) {
    LExtra ex;
    if (bans.count(id)) return ex;
    auto it = obs.find(id);
    if (it != obs.end()) {
      if (score > it->second) {
        it->second = score;
        if (min && min->id == id) min = lb_min(obs);
      }
      return ex;
    }
    if ((i64)obs.size() == size) {
      if (lb_cmp(LPair{id, score}, min)) {
        LPair m = *min;
        masked.erase(id);
        obs[id] = score;
        obs.erase(m.id);
        masked[m.id] = m.score;
        min = lb_min(obs);
      } else {
        auto mit = masked.find(id);
        if (mit == masked.end() || score > mit->second) masked[id] = score;
      }
      return ex;
    }
    obs[id] = score;
    if (!min || lb_cmp(min, LPair{id, score})) min = LPair{id, score};
    return ex;
  }
  // ban/2 (:264-286)
  LExtra ban(i64 id) {
    LExtra ex;
    std::map<i64, i64> masked0 = masked;  // get_largest uses the pre-ban Masked
    bool in_obs = obs.count(id) > 0;
    masked.erase(id);
    obs.erase(id);
    bans.insert(id);
    if (!in_obs) return ex;
    auto ne = get_largest(masked0);
    if (!ne) {
      if (min && min->id == id) min = lb_min(obs);
      return ex;
    }
    masked.erase(ne->id);
    obs[ne->id] = ne->score;
    min = *ne;
    ex.kind = L_ADD;
    ex.elem = *ne;
    return ex;
  }
  // downstream/2 (:93-116)
  int downstream_add(i64 id, i64 score) const {
    if (bans.count(id)) return L_NOOP;
    auto it = obs.find(id);
    if (it != obs.end()) return score > it->second ? L_ADD : L_NOOP;
    auto mit = masked.find(id);
    if (mit != masked.end() && !(score > mit->second)) return L_NOOP;
    if ((i64)obs.size() < size || lb_cmp(LPair{id, score}, min)) return L_ADD;
    return L_ADD_R;
  }
  int downstream_ban(i64 id) const { return bans.count(id) ? L_NOOP : L_BAN; }
};

// ===================================================================
// topk   (src/antidote_ccrdt_topk.erl)
// ===================================================================
struct Topk {
  std::map<i64, i64> top;  // Id -> Score (last writer wins, unbounded: Q10)
  i64 size;
  explicit Topk(i64 k = 1000) : size(k) {}  // new/0 = new(1000) (:65-66, Q8)
  void add(i64 id, i64 score) { top[id] = score; }  // add/3 (:156-158)
  // add_map/2 (:160-161): maps:merge(TopK, Map) — Map's values win.
  void add_map(const std::map<i64, i64>& m) {
    for (const auto& [k, v] : m) top[k] = v;
  }
  // value/1 (:81-83): sort by Score desc, then Id desc.
  std::vector<std::pair<i64, i64>> value() const {
    std::vector<std::pair<i64, i64>> v(top.begin(), top.end());
    std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) {
      return a.second > b.second || (a.second == b.second && a.first > b.first);
    });
    return v;
  }
  // downstream/2 + changes_state/2 (:89-94, :164-166): add iff Score > Size (Q9)
  bool downstream_add(i64 score) const { return score > size; }
};

// ===================================================================
// average   (src/antidote_ccrdt_average.erl)
// ===================================================================
struct Average {
  i64 sum = 0, num = 0;  // new/0 (:56-57)
  // update/2 (:88-94): {add,{_,0}} is a no-op (Q14); N must be > 0.
  // Returns false for an op the reference would crash on (function_clause).
  bool add(i64 v, i64 n) {
    if (n == 0) return true;
    if (n < 0) return false;
    sum += v;
    num += n;
    return true;
  }
  // value/1 (:68-70): Sum / Num as IEEE doubles.
  double value() const { return (double)sum / (double)num; }
};

// ===================================================================
// wordcount / worddocumentcount
// (src/antidote_ccrdt_wordcount.erl, src/antidote_ccrdt_worddocumentcount.erl)
// ===================================================================
// binary:split(File, [<<"\n">>, <<" ">>], [global]) — every separator byte
// splits, empty tokens kept, <<>> -> [<<>>] (Q13).  (wordcount.erl:77)
inline std::vector<std::string> split_words(const std::string& f) {
  std::vector<std::string> out;
  size_t start = 0;
  for (size_t i = 0; i < f.size(); ++i) {
    if (f[i] == '\n' || f[i] == ' ') {
      out.emplace_back(f.substr(start, i - start));
      start = i + 1;
    }
  }
  out.emplace_back(f.substr(start));
  return out;
}
struct Wordcount {
  std::map<std::string, i64> counts;
  // add/2 (wordcount.erl:76-85): +1 per token.
  void add(const std::string& file) {
    for (auto& w : split_words(file)) counts[w] += 1;
  }
};
struct WordDocCount {
  std::map<std::string, i64> counts;
  // add/2 (worddocumentcount.erl:76-86): +1 per distinct token of the doc.
  void add(const std::string& file) {
    auto ws = split_words(file);
    std::set<std::string> d(ws.begin(), ws.end());
    for (auto& w : d) counts[w] += 1;
  }
};

}  // namespace ccrdt_oracle
