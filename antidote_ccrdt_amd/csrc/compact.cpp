// compact.cpp — host log compaction of a batch before upload:
// per key, the reference's can_compact/2 + compact_ops/2 folded over adjacent
// effects in stream order.  The fold keeps a list L; an incoming effect x is
// tried once against L's last effect: if can_compact(last, x), the pair is
// replaced by compact_ops(last, x) ({noop} halves dropped), else x is
// appended.  Only the rewrite rules come from the reference; the fold is this
// pipeline's (Antidote's caller drives them, outside the reference).
//   topk_rmv     src/antidote_ccrdt_topk_rmv.erl:178-223
//   leaderboard  src/antidote_ccrdt_leaderboard.erl:163-205
//   average      src/antidote_ccrdt_average.erl:122-127
// Keys are independent: two passes over key ranges on host threads (count,
// prefix, write), so the output is CSR by key like the input.
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "common.hpp"

namespace ccrdt {
namespace {

int host_threads(uint64_t n_keys) {
  const unsigned hw = std::thread::hardware_concurrency();
  uint64_t t = hw ? hw : 4;
  if (t > 32) t = 32;
  if (t > n_keys / 1024 + 1) t = n_keys / 1024 + 1;
  return (int)(t ? t : 1);
}

// f(k0, k1) over [0, n_keys) split into contiguous ranges, one thread each;
// returns the first non-OK code.
template <class F>
int for_key_ranges(uint64_t n_keys, F f) {
  const int nt = host_threads(n_keys);
  std::vector<int> rc(nt, CCRDT_OK);
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; ++t) {
    const uint64_t k0 = n_keys * t / nt, k1 = n_keys * (t + 1) / nt;
    if (t == nt - 1) {
      rc[t] = f(k0, k1);
    } else {
      pool.emplace_back([&, t, k0, k1] { rc[t] = f(k0, k1); });
    }
  }
  for (auto& th : pool) th.join();
  for (int r : rc)
    if (r != CCRDT_OK) return r;
  return CCRDT_OK;
}

// ------------------------------------------------------------- topk_rmv
struct TOp {
  uint8_t kind;
  int64_t id, score, ts;  // rmv: ts unused
  uint8_t dc;
  int64_t vc[CCRDT_TRMV_MAX_DC];  // rmv: VcRmv (0 = DC absent)
};

bool trmv_is_add(uint8_t k) { return k == CCRDT_TRMV_ADD || k == CCRDT_TRMV_ADD_R; }
bool trmv_is_rmv(uint8_t k) { return k == CCRDT_TRMV_RMV || k == CCRDT_TRMV_RMV_R; }

// can_compact/2 (:178-194)
bool trmv_can(const TOp& a, const TOp& b) {
  if (trmv_is_add(a.kind) && b.kind == CCRDT_TRMV_ADD) return a.id == b.id;
  if ((a.kind == CCRDT_TRMV_ADD_R && trmv_is_rmv(b.kind)) ||
      (a.kind == CCRDT_TRMV_ADD && b.kind == CCRDT_TRMV_RMV))
    return a.id == b.id && b.vc[a.dc] >= a.ts;  // vc_get_timestamp(Vc, DcId) >= Ts
  if (trmv_is_rmv(a.kind) && trmv_is_rmv(b.kind)) return a.id == b.id;
  return false;
}

// The fold over one key's effects; `L` is the compacted list.
void trmv_fold(const ccrdt_trmv_ops* in, int D, uint64_t o0, uint64_t o1, std::vector<TOp>& L) {
  L.clear();
  for (uint64_t i = o0; i < o1; ++i) {
    TOp x{};
    x.kind = in->kind[i];
    x.id = in->id[i];
    if (trmv_is_add(x.kind)) {
      x.score = in->score[i];
      x.dc = in->dc[i];
      x.ts = in->ts[i];
    } else {
      const int64_t* row = in->rmv_vc + (uint64_t)in->ts[i] * D;
      for (int d = 0; d < D; ++d) x.vc[d] = row[d];
    }
    if (!L.empty() && trmv_can(L.back(), x)) {  // compact_ops/2 (:197-223)
      TOp a = L.back();
      L.pop_back();
      if (a.kind == CCRDT_TRMV_ADD && x.kind == CCRDT_TRMV_ADD) {
        // the lower score is retagged add_r (Q20): both stay
        if (a.score > x.score) {
          x.kind = CCRDT_TRMV_ADD_R;
        } else {
          a.kind = CCRDT_TRMV_ADD_R;
        }
        L.push_back(a);
      } else if (a.kind == CCRDT_TRMV_ADD_R && x.kind == CCRDT_TRMV_ADD) {
        if (!(a.score == x.score && a.dc == x.dc && a.ts == x.ts)) L.push_back(a);  // else {noop}
      } else if (trmv_is_add(a.kind)) {
        // add* then a rmv that covers it: {noop}, rmv
      } else {
        // rmv* then rmv*: {noop}, merged Vc; rmv_r only if both are
        for (int d = 0; d < D; ++d) x.vc[d] = std::max(x.vc[d], a.vc[d]);
        x.kind = (a.kind == CCRDT_TRMV_RMV_R && x.kind == CCRDT_TRMV_RMV_R) ? CCRDT_TRMV_RMV_R
                                                                              : CCRDT_TRMV_RMV;
      }
    }
    L.push_back(x);
  }
}

// ---------------------------------------------------------- leaderboard
struct LOp {
  uint8_t kind;
  int64_t id, score;
};
bool lb_is_add(uint8_t k) { return k == CCRDT_LB_ADD || k == CCRDT_LB_ADD_R; }

void lb_fold(const ccrdt_lb_ops* in, uint64_t o0, uint64_t o1, std::vector<LOp>& L) {
  L.clear();
  for (uint64_t i = o0; i < o1; ++i) {
    LOp x{in->kind[i], in->id[i], lb_is_add(in->kind[i]) ? in->score[i] : 0};
    if (!L.empty()) {
      const LOp a = L.back();
      // can_compact/2 (:163-171)
      const bool can = (lb_is_add(a.kind) && lb_is_add(x.kind) && a.id == x.id) ||
                       ((lb_is_add(a.kind) || a.kind == CCRDT_LB_BAN) && x.kind == CCRDT_LB_BAN && a.id == x.id);
      if (can) {  // compact_ops/2 (:174-205)
        L.pop_back();
        if (lb_is_add(x.kind)) {
          if (a.score > x.score) {  // the higher score survives, the other is {noop}
            L.push_back(a);
            continue;
          }
        }
        // an add absorbed by a later ban, or two bans: {noop}, {ban, Id}
      }
    }
    L.push_back(x);
  }
}

}  // namespace
}  // namespace ccrdt

using namespace ccrdt;

extern "C" int ccrdt_trmv_compact(int n_dc, int64_t n_keys, const ccrdt_trmv_ops* in, ccrdt_trmv_batch* out) {
  if (!in || !out || n_keys < 0 || n_dc < 1 || n_dc > CCRDT_TRMV_MAX_DC || !in->key_ptr || !out->key_ptr ||
      (in->n_ops && (!in->kind || !in->id || !in->score || !in->dc || !in->ts)) ||
      (in->n_ops && (!out->kind || !out->id || !out->score || !out->dc || !out->ts || !out->rmv_vc))) {
    set_error("trmv_compact: null arrays or bad n_dc");
    return CCRDT_EINVAL;
  }
  const uint64_t nk = (uint64_t)n_keys;
  if (in->key_ptr[nk] != (uint64_t)in->n_ops) {
    set_error("trmv_compact: key_ptr[n_keys] != n_ops");
    return CCRDT_EINVAL;
  }
  for (int64_t i = 0; i < in->n_ops; ++i) {
    if (in->kind[i] > CCRDT_TRMV_RMV_R) {
      set_error("trmv_compact: effect kind > 3 (no function clause)");
      return CCRDT_EINVAL;
    }
    if (trmv_is_rmv(in->kind[i]) && (in->ts[i] < 0 || in->ts[i] >= in->n_rmv_rows || !in->rmv_vc)) {
      set_error("trmv_compact: rmv clock row out of range");
      return CCRDT_EINVAL;
    }
    if (trmv_is_add(in->kind[i]) && in->dc[i] >= n_dc) {
      set_error("trmv_compact: add DC rank >= n_dc");
      return CCRDT_EINVAL;
    }
  }
  // pass 1: compacted op and rmv counts per key
  std::vector<uint64_t> nops(nk + 1, 0), nrm(nk + 1, 0);
  int rc = for_key_ranges(nk, [&](uint64_t k0, uint64_t k1) {
    std::vector<TOp> L;
    for (uint64_t k = k0; k < k1; ++k) {
      trmv_fold(in, n_dc, in->key_ptr[k], in->key_ptr[k + 1], L);
      nops[k + 1] = L.size();
      for (const TOp& t : L) nrm[k + 1] += trmv_is_rmv(t.kind) ? 1u : 0u;
    }
    return CCRDT_OK;
  });
  if (rc != CCRDT_OK) return rc;
  for (uint64_t k = 0; k < nk; ++k) {
    nops[k + 1] += nops[k];
    nrm[k + 1] += nrm[k];
  }
  // pass 2: write (one clock row per output rmv, numbered in stream order)
  rc = for_key_ranges(nk, [&](uint64_t k0, uint64_t k1) {
    std::vector<TOp> L;
    for (uint64_t k = k0; k < k1; ++k) {
      trmv_fold(in, n_dc, in->key_ptr[k], in->key_ptr[k + 1], L);
      uint64_t o = nops[k], r = nrm[k];
      for (const TOp& t : L) {
        out->kind[o] = t.kind;
        out->id[o] = t.id;
        if (trmv_is_add(t.kind)) {
          out->score[o] = t.score;
          out->dc[o] = t.dc;
          out->ts[o] = t.ts;
        } else {
          out->score[o] = 0;
          out->dc[o] = 0;
          out->ts[o] = (int64_t)r;
          for (int d = 0; d < n_dc; ++d) out->rmv_vc[r * n_dc + d] = t.vc[d];
          ++r;
        }
        ++o;
      }
    }
    return CCRDT_OK;
  });
  if (rc != CCRDT_OK) return rc;
  for (uint64_t k = 0; k <= nk; ++k) out->key_ptr[k] = nops[k];
  out->n_ops = (int64_t)nops[nk];
  out->n_rmv_rows = (int64_t)nrm[nk];
  return CCRDT_OK;
}

extern "C" int ccrdt_lb_compact(int64_t n_keys, const ccrdt_lb_ops* in, ccrdt_lb_batch* out) {
  if (!in || !out || n_keys < 0 || !in->key_ptr || !out->key_ptr ||
      (in->n_ops && (!in->kind || !in->id || !in->score || !out->kind || !out->id || !out->score))) {
    set_error("lb_compact: null arrays");
    return CCRDT_EINVAL;
  }
  const uint64_t nk = (uint64_t)n_keys;
  if (in->key_ptr[nk] != (uint64_t)in->n_ops) {
    set_error("lb_compact: key_ptr[n_keys] != n_ops");
    return CCRDT_EINVAL;
  }
  for (int64_t i = 0; i < in->n_ops; ++i)
    if (in->kind[i] > CCRDT_LB_BAN) {
      set_error("lb_compact: effect kind > 2 (no function clause)");
      return CCRDT_EINVAL;
    }
  std::vector<uint64_t> nops(nk + 1, 0);
  int rc = for_key_ranges(nk, [&](uint64_t k0, uint64_t k1) {
    std::vector<LOp> L;
    for (uint64_t k = k0; k < k1; ++k) {
      lb_fold(in, in->key_ptr[k], in->key_ptr[k + 1], L);
      nops[k + 1] = L.size();
    }
    return CCRDT_OK;
  });
  if (rc != CCRDT_OK) return rc;
  for (uint64_t k = 0; k < nk; ++k) nops[k + 1] += nops[k];
  rc = for_key_ranges(nk, [&](uint64_t k0, uint64_t k1) {
    std::vector<LOp> L;
    for (uint64_t k = k0; k < k1; ++k) {
      lb_fold(in, in->key_ptr[k], in->key_ptr[k + 1], L);
      uint64_t o = nops[k];
      for (const LOp& t : L) {
        out->kind[o] = t.kind;
        out->id[o] = t.id;
        out->score[o] = t.score;
        ++o;
      }
    }
    return CCRDT_OK;
  });
  if (rc != CCRDT_OK) return rc;
  for (uint64_t k = 0; k <= nk; ++k) out->key_ptr[k] = nops[k];
  out->n_ops = (int64_t)nops[nk];
  return CCRDT_OK;
}

// average: every pair compacts (:122-127), so a key's effects fold into one
// {add, {Sum V, Sum N}}; a sum that leaves int64 is ERANGE (Erlang integers
// are unbounded).
extern "C" int ccrdt_avg_compact(int64_t n_keys, const ccrdt_avg_ops* in, ccrdt_avg_batch* out) {
  if (!in || !out || n_keys < 0 || !in->key_ptr || !out->key_ptr ||
      (in->n_ops && (!in->value || !in->n || !out->value || !out->n))) {
    set_error("avg_compact: null arrays");
    return CCRDT_EINVAL;
  }
  const uint64_t nk = (uint64_t)n_keys;
  if (in->key_ptr[nk] != (uint64_t)in->n_ops) {
    set_error("avg_compact: key_ptr[n_keys] != n_ops");
    return CCRDT_EINVAL;
  }
  std::vector<uint64_t> nops(nk + 1, 0);
  for (uint64_t k = 0; k < nk; ++k) nops[k + 1] = nops[k] + (in->key_ptr[k + 1] > in->key_ptr[k] ? 1u : 0u);
  const int rc = for_key_ranges(nk, [&](uint64_t k0, uint64_t k1) {
    for (uint64_t k = k0; k < k1; ++k) {
      if (in->key_ptr[k + 1] == in->key_ptr[k]) continue;
      int64_t v = 0, c = 0;
      for (uint64_t i = in->key_ptr[k]; i < in->key_ptr[k + 1]; ++i)
        if (__builtin_add_overflow(v, in->value[i], &v) || __builtin_add_overflow(c, in->n[i], &c))
          return CCRDT_ERANGE;
      out->value[nops[k]] = v;
      out->n[nops[k]] = c;
    }
    return CCRDT_OK;
  });
  if (rc != CCRDT_OK) {
    set_error("avg_compact: a compacted sum leaves int64");
    return rc;
  }
  for (uint64_t k = 0; k <= nk; ++k) out->key_ptr[k] = nops[k];
  out->n_ops = (int64_t)nops[nk];
  return CCRDT_OK;
}
