// etf_codec.cpp — to_binary/1 and from_binary/1 of topk_rmv states in native
// code: the Erlang external term format (ETF) of the
// reference's state 6-tuple {Observed, Masked, Removals, Vc, Min, Size}
// (src/antidote_ccrdt_topk_rmv.erl:67-74; to_binary = term_to_binary(State),
// :156-163), read from and written to the canonical state image of
// include/ccrdt.h (ccrdt_trmv_state), one key at a time.  A NIF shim hands
// these bytes to enif_binary_to_term / takes them from enif_term_to_binary, so
// a state crosses the boundary without a term walk per element on the BEAM
// side.
//
// Writer (byte-identical to antidote_ccrdt_amd/etf.py, the Python codec the
// behaviour mirror uses): elements are pair_internal() = {Score, Id, {DcId,
// Ts}}; Observed maps Id -> element; Masked maps Id -> gb_sets set, written as
// the balanced {Size, Tree} of gb_sets:from_ordset/1 (balance_list/2); Removals
// maps Id -> vc(), a vc() maps DcId -> Ts (entries that are 0 are absent:
// vc_get_timestamp/2 :350-355); Min is an element or {nil, nil, nil}.  Map
// keys are written in term order (any order decodes); integers as SMALL_INT /
// INT / SMALL_BIG; atoms as SMALL_ATOM_UTF8.  DcIds are the caller's terms:
// rank d (the engine's DC ranks preserve term order) is written as
// the bytes dc_term[dc_off[d] .. dc_off[d + 1]).
//
// Reader: whatever ERTS produced -- maps in any order, every integer and atom
// tag, tuples of any arity tag, gb_sets trees of any shape (walked in order:
// gb_sets:insert/2 leaves unbalanced ones) -- into the image of one key; a
// DcId is matched by its canonical re-encoding against dc_term.
#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ccrdt.h"

namespace ccrdt {
void set_error(const std::string& msg);
}

namespace {

enum : uint8_t {
  E_VERSION = 131,
  E_NEW_FLOAT = 70,
  E_SMALL_INT = 97,
  E_INT = 98,
  E_ATOM = 100,
  E_SMALL_TUPLE = 104,
  E_LARGE_TUPLE = 105,
  E_NIL = 106,
  E_STRING = 107,
  E_LIST = 108,
  E_BINARY = 109,
  E_SMALL_BIG = 110,
  E_LARGE_BIG = 111,
  E_MAP = 116,
  E_SMALL_ATOM = 115,
  E_ATOM_UTF8 = 118,
  E_SMALL_ATOM_UTF8 = 119,
};

// ------------------------------------------------------------------ writer
struct Out {
  uint8_t* buf;
  uint64_t cap, n = 0;
  void b(uint8_t v) {
    if (n < cap) buf[n] = v;
    ++n;
  }
  void bytes(const uint8_t* p, uint64_t k) {
    for (uint64_t i = 0; i < k; ++i) b(p[i]);
  }
  void be32(uint32_t v) {
    b((uint8_t)(v >> 24));
    b((uint8_t)(v >> 16));
    b((uint8_t)(v >> 8));
    b((uint8_t)v);
  }
};

void w_int(Out& o, int64_t v) {
  if (v >= 0 && v <= 255) {
    o.b(E_SMALL_INT);
    o.b((uint8_t)v);
  } else if (v >= INT32_MIN && v <= INT32_MAX) {
    o.b(E_INT);
    o.be32((uint32_t)(int32_t)v);
  } else {  // SMALL_BIG: sign, magnitude little-endian in its fewest bytes
    const uint64_t mag = v < 0 ? 0 - (uint64_t)v : (uint64_t)v;
    uint8_t n = 0;
    for (uint64_t m = mag; m; m >>= 8) ++n;
    o.b(E_SMALL_BIG);
    o.b(n);
    o.b(v < 0 ? 1 : 0);
    for (uint8_t i = 0; i < n; ++i) o.b((uint8_t)(mag >> (8 * i)));
  }
}
void w_atom(Out& o, const char* s) {
  const size_t n = strlen(s);
  o.b(E_SMALL_ATOM_UTF8);
  o.b((uint8_t)n);
  o.bytes(reinterpret_cast<const uint8_t*>(s), n);
}
void w_tuple(Out& o, uint32_t n) {
  o.b(E_SMALL_TUPLE);
  o.b((uint8_t)n);
}
void w_map(Out& o, uint32_t n) {
  o.b(E_MAP);
  o.be32(n);
}

struct Dcs {
  const uint8_t* term;
  const uint64_t* off;
  int n;
  void w(Out& o, uint32_t d) const { o.bytes(term + off[d], off[d + 1] - off[d]); }
};

// {Score, Id, {DcId, Ts}}
void w_elem(Out& o, const Dcs& dc, int64_t sc, int64_t id, uint32_t d, int64_t ts) {
  w_tuple(o, 3);
  w_int(o, sc);
  w_int(o, id);
  w_tuple(o, 2);
  dc.w(o, d);
  w_int(o, ts);
}

// gb_sets:from_ordset/1 -> balance_list/2: the tree of n sorted elements
// starting at index i: {Key, Smaller, Bigger} | nil, the larger half on the
// smaller side (S1 = ceil((n-1)/2)).
void w_gb(Out& o, const Dcs& dc, const ccrdt_trmv_state* st, uint64_t i, uint64_t n) {
  if (n == 0) {
    w_atom(o, "nil");
    return;
  }
  const uint64_t m = n - 1, s2 = m / 2, s1 = m - s2;
  const uint64_t k = i + s1;
  w_tuple(o, 3);
  w_elem(o, dc, st->m_score[k], st->m_id[k], st->m_dc[k], st->m_ts[k]);
  w_gb(o, dc, st, i, s1);
  w_gb(o, dc, st, k + 1, s2);
}

void w_vc(Out& o, const Dcs& dc, const int64_t* row) {
  uint32_t n = 0;
  for (int d = 0; d < dc.n; ++d) n += row[d] != 0;
  w_map(o, n);
  for (int d = 0; d < dc.n; ++d)
    if (row[d]) {
      dc.w(o, (uint32_t)d);
      w_int(o, row[d]);
    }
}

// ------------------------------------------------------------------ reader
struct In {
  const uint8_t* p;
  uint64_t n, i = 0;
  bool ok = true;
  std::string why;
  bool fail(const char* w) {
    if (ok) why = w;
    ok = false;
    return false;
  }
  bool need(uint64_t k) { return i + k <= n ? true : fail("truncated term"); }
  uint8_t u8() { return need(1) ? p[i++] : 0; }
  uint32_t u16() {
    if (!need(2)) return 0;
    const uint32_t v = (uint32_t)p[i] << 8 | p[i + 1];
    i += 2;
    return v;
  }
  uint32_t u32() {
    if (!need(4)) return 0;
    const uint32_t v = (uint32_t)p[i] << 24 | (uint32_t)p[i + 1] << 16 | (uint32_t)p[i + 2] << 8 | p[i + 3];
    i += 4;
    return v;
  }
};

// An integer term (any tag) that fits int64.
bool r_int(In& r, int64_t& v) {
  const uint8_t t = r.u8();
  if (t == E_SMALL_INT) {
    v = r.u8();
    return r.ok;
  }
  if (t == E_INT) {
    v = (int32_t)r.u32();
    return r.ok;
  }
  if (t == E_SMALL_BIG || t == E_LARGE_BIG) {
    const uint32_t n = t == E_SMALL_BIG ? r.u8() : r.u32();
    const uint8_t sign = r.u8();
    if (!r.need(n)) return false;
    uint64_t mag = 0;
    for (uint32_t k = 0; k < n; ++k) {
      const uint8_t byte = r.p[r.i + k];
      if (k >= 8 && byte) return r.fail("integer outside int64");
      if (k < 8) mag |= (uint64_t)byte << (8 * k);
    }
    r.i += n;
    if (sign ? mag > (uint64_t)INT64_MAX + 1 : mag > (uint64_t)INT64_MAX) return r.fail("integer outside int64");
    v = sign ? (int64_t)(0 - mag) : (int64_t)mag;
    return true;
  }
  return r.fail("not an integer");
}

// An atom term (any of the four tags) -> its name.
bool r_atom(In& r, std::string& s) {
  const uint8_t t = r.u8();
  uint32_t n;
  if (t == E_ATOM || t == E_ATOM_UTF8) n = r.u16();
  else if (t == E_SMALL_ATOM || t == E_SMALL_ATOM_UTF8) n = r.u8();
  else return r.fail("not an atom");
  if (!r.need(n)) return false;
  s.assign(reinterpret_cast<const char*>(r.p + r.i), n);  // (latin-1 names of ATOM/SMALL_ATOM are ASCII here)
  r.i += n;
  return true;
}

bool r_tuple(In& r, uint32_t& n) {
  const uint8_t t = r.u8();
  if (t == E_SMALL_TUPLE) n = r.u8();
  else if (t == E_LARGE_TUPLE) n = r.u32();
  else return r.fail("not a tuple");
  return r.ok;
}

bool r_map(In& r, uint32_t& n) {
  if (r.u8() != E_MAP) return r.fail("not a map");
  n = r.u32();
  return r.ok;
}

// Any term, re-encoded canonically (the writer's tags) into `o`: how a DcId
// read back is matched against the caller's DcId terms.
bool r_canon(In& r, Out& o, int depth = 0) {
  if (depth > 64) return r.fail("term nested too deep");
  if (!r.need(1)) return false;
  const uint8_t t = r.p[r.i];
  switch (t) {
    case E_SMALL_INT:
    case E_INT:
    case E_SMALL_BIG:
    case E_LARGE_BIG: {
      int64_t v;
      if (!r_int(r, v)) return false;
      w_int(o, v);
      return true;
    }
    case E_ATOM:
    case E_ATOM_UTF8:
    case E_SMALL_ATOM:
    case E_SMALL_ATOM_UTF8: {
      std::string s;
      if (!r_atom(r, s)) return false;
      if (s.size() > 255) return r.fail("atom too long");
      o.b(E_SMALL_ATOM_UTF8);
      o.b((uint8_t)s.size());
      o.bytes(reinterpret_cast<const uint8_t*>(s.data()), s.size());
      return true;
    }
    case E_SMALL_TUPLE:
    case E_LARGE_TUPLE: {
      uint32_t n;
      if (!r_tuple(r, n)) return false;
      if (n > 255) return r.fail("DcId tuple too large");
      w_tuple(o, n);
      for (uint32_t k = 0; k < n; ++k)
        if (!r_canon(r, o, depth + 1)) return false;
      return true;
    }
    case E_NIL:
      r.i++;
      o.b(E_NIL);
      return true;
    case E_BINARY: {
      r.i++;
      const uint32_t n = r.u32();
      if (!r.need(n)) return false;
      o.b(E_BINARY);
      o.be32(n);
      o.bytes(r.p + r.i, n);
      r.i += n;
      return true;
    }
    default:
      return r.fail("unsupported DcId term");
  }
}

struct Reader {
  In r;
  Dcs dc;
  std::vector<std::vector<uint8_t>> canon;  // the caller's DcId terms
  uint8_t tmp[512];

  bool dcid(uint32_t& d) {
    Out o{tmp, sizeof(tmp)};
    if (!r_canon(r, o)) return false;
    if (o.n > sizeof(tmp)) return r.fail("DcId term too large");
    for (size_t k = 0; k < canon.size(); ++k)
      if (canon[k].size() == o.n && memcmp(canon[k].data(), tmp, o.n) == 0) {
        d = (uint32_t)k;
        return true;
      }
    return r.fail("DcId not among the engine's DCs");
  }
  // {Score, Id, {DcId, Ts}}
  bool elem(int64_t& sc, int64_t& id, uint32_t& d, int64_t& ts) {
    uint32_t n;
    if (!r_tuple(r, n) || n != 3) return r.fail("not a pair_internal() element");
    if (!r_int(r, sc) || !r_int(r, id)) return false;
    if (!r_tuple(r, n) || n != 2) return r.fail("not a {DcId, Ts} pair");
    return dcid(d) && r_int(r, ts);
  }
  bool vc(std::vector<int64_t>& row) {
    uint32_t n;
    if (!r_map(r, n)) return false;
    row.assign(dc.n, 0);
    for (uint32_t k = 0; k < n; ++k) {
      uint32_t d;
      int64_t t;
      if (!dcid(d) || !r_int(r, t)) return false;
      row[d] = t;
    }
    return true;
  }
  // a gb_sets tree node: {Key, Smaller, Bigger} | nil, walked in order
  bool gb_tree(std::vector<std::array<int64_t, 4>>& out, int depth) {
    if (depth > 4096) return r.fail("gb_sets tree too deep");
    if (!r.need(1)) return false;
    const uint8_t t = r.p[r.i];
    if (t == E_ATOM || t == E_ATOM_UTF8 || t == E_SMALL_ATOM || t == E_SMALL_ATOM_UTF8) {
      std::string s;
      if (!r_atom(r, s)) return false;
      return s == "nil" ? true : r.fail("not a gb_sets tree");
    }
    uint32_t n;
    if (!r_tuple(r, n) || n != 3) return r.fail("not a gb_sets tree node");
    // the key comes first in the bytes but sorts between the subtrees
    int64_t sc, id, ts;
    uint32_t d;
    if (!elem(sc, id, d, ts)) return false;
    std::vector<std::array<int64_t, 4>> left;
    if (!gb_tree(left, depth + 1)) return false;
    out.insert(out.end(), left.begin(), left.end());
    out.push_back({id, sc, (int64_t)d, ts});
    return gb_tree(out, depth + 1);
  }
};

struct Row {
  int64_t id, sc;
  int64_t d;
  int64_t ts;
};

}  // namespace

extern "C" int ccrdt_trmv_key_to_binary(const ccrdt_trmv_state* st, int n_dc, int64_t k, int64_t size,
                                        const uint8_t* dc_term, const uint64_t* dc_off, uint8_t* buf,
                                        uint64_t cap, uint64_t* len) {
  if (!st || !len || !dc_off || (!dc_term && dc_off[n_dc] != 0) || n_dc < 1 || n_dc > CCRDT_TRMV_MAX_DC ||
      k < 0 || size <= 0 || (cap && !buf)) {
    ccrdt::set_error("trmv_key_to_binary: bad argument");
    return CCRDT_EINVAL;
  }
  for (int d = 0; d < n_dc; ++d)
    if (dc_off[d + 1] <= dc_off[d]) {
      ccrdt::set_error("trmv_key_to_binary: empty DcId term");
      return CCRDT_EINVAL;
    }
  Out o{buf, cap};
  const Dcs dc{dc_term, dc_off, n_dc};
  o.b(E_VERSION);
  w_tuple(o, 6);
  // Observed: Id -> element (the image is sorted by Id)
  const uint64_t o0 = st->obs_ptr[k], o1 = st->obs_ptr[k + 1];
  w_map(o, (uint32_t)(o1 - o0));
  for (uint64_t i = o0; i < o1; ++i) {
    w_int(o, st->obs_id[i]);
    w_elem(o, dc, st->obs_score[i], st->obs_id[i], st->obs_dc[i], st->obs_ts[i]);
  }
  // Masked: Id -> gb_sets (elements sorted by (Id, Score, DcId, Ts) = term order within an Id)
  const uint64_t m0 = st->m_ptr[k], m1 = st->m_ptr[k + 1];
  uint32_t nid = 0;
  for (uint64_t i = m0; i < m1; ++i) nid += (i == m0 || st->m_id[i] != st->m_id[i - 1]);
  w_map(o, nid);
  for (uint64_t i = m0; i < m1;) {
    uint64_t j = i + 1;
    while (j < m1 && st->m_id[j] == st->m_id[i]) ++j;
    w_int(o, st->m_id[i]);
    w_tuple(o, 2);
    w_int(o, (int64_t)(j - i));
    w_gb(o, dc, st, i, j - i);
    i = j;
  }
  // Removals: Id -> vc()
  const uint64_t r0 = st->r_ptr[k], r1 = st->r_ptr[k + 1];
  w_map(o, (uint32_t)(r1 - r0));
  for (uint64_t i = r0; i < r1; ++i) {
    w_int(o, st->r_id[i]);
    w_vc(o, dc, st->r_vc + i * n_dc);
  }
  // Vc, Min, Size
  w_vc(o, dc, st->vc + (uint64_t)k * n_dc);
  if (st->min_valid[k]) {
    w_elem(o, dc, st->min_score[k], st->min_id[k], st->min_dc[k], st->min_ts[k]);
  } else {
    w_tuple(o, 3);
    for (int i = 0; i < 3; ++i) w_atom(o, "nil");
  }
  w_int(o, size);
  *len = o.n;
  if (o.n > cap) {
    ccrdt::set_error("trmv_key_to_binary: buffer too small (*len bytes needed)");
    return CCRDT_ENOMEM;
  }
  return CCRDT_OK;
}

extern "C" int ccrdt_trmv_key_from_binary(const uint8_t* buf, uint64_t len, int n_dc, const uint8_t* dc_term,
                                          const uint64_t* dc_off, ccrdt_trmv_state* out, const int64_t* caps,
                                          int64_t* counts, int64_t* size) {
  if (!buf || !dc_off || n_dc < 1 || n_dc > CCRDT_TRMV_MAX_DC || !counts || !size) {
    ccrdt::set_error("trmv_key_from_binary: bad argument");
    return CCRDT_EINVAL;
  }
  Reader R{In{buf, len}, Dcs{dc_term, dc_off, n_dc}, {}, {}};
  for (int d = 0; d < n_dc; ++d) R.canon.emplace_back(dc_term + dc_off[d], dc_term + dc_off[d + 1]);
  In& r = R.r;
  std::vector<Row> obs, msk;
  std::vector<std::pair<int64_t, std::vector<int64_t>>> rem;
  std::vector<int64_t> vc;
  int64_t mn[4] = {0, 0, 0, 0};
  bool has_min = false;
  uint32_t n = 0;
  auto parse = [&]() -> bool {
    if (r.u8() != E_VERSION) return r.fail("not an external term (version byte)");
    if (!r_tuple(r, n) || n != 6) return r.fail("not a topkrmv() 6-tuple");
    if (!r_map(r, n)) return false;  // Observed
    for (uint32_t i = 0; i < n; ++i) {
      int64_t key, sc, id, ts;
      uint32_t d;
      if (!r_int(r, key) || !R.elem(sc, id, d, ts)) return false;
      if (key != id) return r.fail("Observed key differs from its element's Id");
      obs.push_back({id, sc, d, ts});
    }
    if (!r_map(r, n)) return false;  // Masked
    for (uint32_t i = 0; i < n; ++i) {
      int64_t key, cnt;
      uint32_t t2;
      if (!r_int(r, key) || !r_tuple(r, t2) || t2 != 2 || !r_int(r, cnt)) return r.fail("not a gb_sets set");
      std::vector<std::array<int64_t, 4>> items;
      if (!R.gb_tree(items, 0)) return false;
      if ((int64_t)items.size() != cnt) return r.fail("gb_sets size does not match its tree");
      for (auto& e : items) {
        if (e[0] != key) return r.fail("Masked element under another Id");
        msk.push_back({e[0], e[1], e[2], e[3]});
      }
    }
    if (!r_map(r, n)) return false;  // Removals
    for (uint32_t i = 0; i < n; ++i) {
      int64_t key;
      std::vector<int64_t> row;
      if (!r_int(r, key) || !R.vc(row)) return false;
      rem.emplace_back(key, std::move(row));
    }
    if (!R.vc(vc)) return false;  // Vc
    {                              // Min: an element or {nil, nil, nil}
      const uint64_t at = r.i;
      uint32_t t3;
      if (!r_tuple(r, t3) || t3 != 3) return r.fail("Min is not a 3-tuple");
      if (r.need(1) && r.p[r.i] != E_SMALL_INT && r.p[r.i] != E_INT && r.p[r.i] != E_SMALL_BIG &&
          r.p[r.i] != E_LARGE_BIG) {
        for (int k = 0; k < 3; ++k) {
          std::string s;
          if (!r_atom(r, s) || s != "nil") return r.fail("Min is neither an element nor {nil, nil, nil}");
        }
      } else {
        r.i = at;
        uint32_t d;
        if (!R.elem(mn[1], mn[0], d, mn[3])) return false;
        mn[2] = d;
        has_min = true;
      }
    }
    if (!r_int(r, *size)) return false;
    if (*size <= 0) return r.fail("topkrmv() Size must be a positive integer");
    if (r.i != r.n) return r.fail("trailing bytes after the term");
    return r.ok;
  };
  if (!parse()) {
    ccrdt::set_error("trmv_key_from_binary: " + r.why);
    return r.why.find("int64") != std::string::npos ? CCRDT_ERANGE : CCRDT_EINVAL;
  }
  counts[0] = (int64_t)obs.size();
  counts[1] = (int64_t)msk.size();
  counts[2] = (int64_t)rem.size();
  if (!out || !caps) return CCRDT_OK;  // (sizing call)
  if (counts[0] > caps[0] || counts[1] > caps[1] || counts[2] > caps[2]) {
    ccrdt::set_error("trmv_key_from_binary: arrays too small (counts[] entries needed)");
    return CCRDT_ENOMEM;
  }
  // the canonical image of one key: Observed and Removals by Id, Masked by
  // (Id, Score, DcId, Ts)
  auto by = [](const Row& a, const Row& b) {
    return a.id != b.id ? a.id < b.id : a.sc != b.sc ? a.sc < b.sc : a.d != b.d ? a.d < b.d : a.ts < b.ts;
  };
  std::sort(obs.begin(), obs.end(), by);
  std::sort(msk.begin(), msk.end(), by);
  std::sort(rem.begin(), rem.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  out->obs_ptr[0] = out->m_ptr[0] = out->r_ptr[0] = 0;
  out->obs_ptr[1] = obs.size();
  out->m_ptr[1] = msk.size();
  out->r_ptr[1] = rem.size();
  for (size_t i = 0; i < obs.size(); ++i) {
    out->obs_id[i] = obs[i].id;
    out->obs_score[i] = obs[i].sc;
    out->obs_dc[i] = (uint8_t)obs[i].d;
    out->obs_ts[i] = obs[i].ts;
  }
  for (size_t i = 0; i < msk.size(); ++i) {
    out->m_id[i] = msk[i].id;
    out->m_score[i] = msk[i].sc;
    out->m_dc[i] = (uint8_t)msk[i].d;
    out->m_ts[i] = msk[i].ts;
  }
  for (size_t i = 0; i < rem.size(); ++i) {
    out->r_id[i] = rem[i].first;
    for (int d = 0; d < n_dc; ++d) out->r_vc[i * n_dc + d] = rem[i].second[d];
  }
  for (int d = 0; d < n_dc; ++d) out->vc[d] = vc[d];
  out->min_valid[0] = has_min ? 1 : 0;
  out->min_id[0] = has_min ? mn[0] : 0;
  out->min_score[0] = has_min ? mn[1] : 0;
  out->min_dc[0] = (uint8_t)(has_min ? mn[2] : 0);
  out->min_ts[0] = has_min ? mn[3] : 0;
  return CCRDT_OK;
}
