// trmv_kernels.hip — gfx950 kernels for antidote_ccrdt_topk_rmv update/2.
//
// One wavefront owns one key (one CCRDT object) and runs that key's effects in
// stream order: the per-key state machine of the reference is sequential
// (SURVEY §8a "path-dependent semantics"), while keys are independent, so the
// chip-level parallelism is 1M keys ≫ resident waves.  The key's whole state
// lives in VGPRs while its ops run: element e of a 64·S-entry table sits in
// lane e%64 of register slot e/64.  Lookups by Id are wave-wide compares +
// ballot; reads/writes of one element are v_readlane / v_writelane with a
// wave-uniform index; min/max over Observed or over Masked candidates are
// 64-lane shuffle reductions.  Nothing touches LDS except the staging of the
// removal vector clocks of the current 64-op chunk.
//
// Reference semantics (src/antidote_ccrdt_topk_rmv.erl):
//   update/2 :140-148 · add/4 :231-249 · rmv/3 :252-298
//   recompute_observed/5 :301-334 · cmp/2 :389-395 · min_observed/1 :398-406
//   vc_update/3 :358-366 · merge_vc/3 :369-375 · merge_vcs/2 :378-386
//   downstream/2 :102-124
#include "common.hpp"
#include "trmv_kernels.hpp"

namespace ccrdt {

// Strict cmp/2 of topk_rmv (:389-395): (Score, Id, Ts), DcId ignored.
__device__ __forceinline__ bool trmv_cmp(int64_t s1, int64_t i1, int64_t t1, int64_t s2, int64_t i2,
                                         int64_t t2) {
  return s1 > s2 || (s1 == s2 && i1 > i2) || (s1 == s2 && i1 == i2 && t1 > t2);
}

// --------------------------------------------------------------- slot access
// Register tables are clang ext_vector values (one element per 64-lane slot)
// so that they stay SSA values — never a private-memory alloca.
template <int N>
using V64 = int64_t __attribute__((ext_vector_type(N)));
template <int N>
using V32 = uint32_t __attribute__((ext_vector_type(N)));

template <int N>
__device__ __forceinline__ uint32_t slot_get(const V32<N>& a, uint32_t idx) {
  uint32_t r = 0;
#pragma unroll
  for (int s = 0; s < N; ++s)
    if ((idx >> 6) == (uint32_t)s) r = rl32(a[s], idx & 63);
  return r;
}
template <int N>
__device__ __forceinline__ int64_t slot_get(const V64<N>& a, uint32_t idx) {
  int64_t r = 0;
#pragma unroll
  for (int s = 0; s < N; ++s)
    if ((idx >> 6) == (uint32_t)s) r = rl64(a[s], idx & 63);
  return r;
}
template <int N>
__device__ __forceinline__ void slot_set(V32<N>& a, uint32_t idx, uint32_t v) {
#pragma unroll
  for (int s = 0; s < N; ++s)
    if ((idx >> 6) == (uint32_t)s) a[s] = wl32(a[s], idx & 63, v);
}
template <int N>
__device__ __forceinline__ void slot_set(V64<N>& a, uint32_t idx, int64_t v) {
#pragma unroll
  for (int s = 0; s < N; ++s)
    if ((idx >> 6) == (uint32_t)s) a[s] = wl64(a[s], idx & 63, v);
}
// Per-lane gather a[idx_lane] (idx differs per lane).
template <int N>
__device__ __forceinline__ int64_t slot_gather(const V64<N>& a, uint32_t idx) {
  int64_t r = 0;
#pragma unroll
  for (int s = 0; s < N; ++s) {
    int64_t v = shfl64(a[s], idx & 63);
    if ((idx >> 6) == (uint32_t)s) r = v;
  }
  return r;
}
template <int N>
__device__ __forceinline__ uint32_t slot_gather(const V32<N>& a, uint32_t idx) {
  uint32_t r = 0;
#pragma unroll
  for (int s = 0; s < N; ++s) {
    uint32_t v = shfl32(a[s], idx & 63);
    if ((idx >> 6) == (uint32_t)s) r = v;
  }
  return r;
}

// --------------------------------------------------------------- key state
template <int S>
struct KeyState {
  static constexpr uint32_t CAP = 64u * S;      // players and pool entries
  static constexpr uint32_t RSLOTS = 2 * S;     // removal-row register pairs
  static constexpr uint32_t RCAP = 8u * RSLOTS; // removal rows
  // players
  V64<S> qid;
  V32<S> qinfo;
  V64<S> qos;  // score of the player's Observed element (valid iff in Obs)
  // pool (Masked elements)
  V64<S> ps, pt;
  V32<S> pm;
  // removal rows: row r, dc d -> lane (r%8)*8+d of rv[r/8]
  V64<2 * S> rv;
  // replica Vc: lane d
  int64_t vcv;
  // uniforms
  uint32_t np, npool, nrows, nobs, minq;
  int64_t min_sc, min_id, min_ts;
  uint32_t nex;
  bool ovf;
};

template <int S>
__device__ __forceinline__ int find_player(const KeyState<S>& st, int64_t id) {
  const int lane = lane_id();
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if ((uint32_t)s * 64u < st.np) {
      uint64_t m = ballot(st.qid[s] == id && (uint32_t)(s * 64 + lane) < st.np);
      if (m) return s * 64 + __builtin_ctzll(m);
    }
  }
  return -1;
}

// Set / clear the INOBS flag of every pool element owned by player q.
template <int S>
__device__ __forceinline__ void mark_owner(KeyState<S>& st, uint32_t q, bool in) {
#pragma unroll
  for (int s = 0; s < S; ++s) {
    bool own = (st.pm[s] & 0xFFFFu) == q;
    if (own) st.pm[s] = in ? (st.pm[s] | PD_INOBS) : (st.pm[s] & ~PD_INOBS);
  }
}

template <int S>
__device__ __forceinline__ void set_obs(KeyState<S>& st, uint32_t q, uint32_t e, int64_t sc) {
  uint32_t info = slot_get<S>(st.qinfo, q);
  slot_set<S>(st.qinfo, q, (info & 0xFFFF0000u) | e);
  slot_set<S>(st.qos, q, sc);
  mark_owner<S>(st, q, true);
}
template <int S>
__device__ __forceinline__ void unset_obs(KeyState<S>& st, uint32_t q) {
  uint32_t info = slot_get<S>(st.qinfo, q);
  slot_set<S>(st.qinfo, q, info | 0xFFFFu);
  mark_owner<S>(st, q, false);
}

// min_observed/1 (:398-406): term-order smallest Observed value.  Ids are
// distinct inside Observed, so (Score, Id) decides.
template <int S>
__device__ __forceinline__ void recompute_min(KeyState<S>& st) {
  const int lane = lane_id();
  bool valid[S];
  bool any = false;
  int64_t best = INT64_MAX;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    valid[s] = (uint32_t)(s * 64 + lane) < st.np && (st.qinfo[s] & 0xFFFFu) != NONE16;
    if (valid[s] && st.qos[s] < best) best = st.qos[s];
    any |= ballot(valid[s]) != 0;
  }
  if (!any) {
    st.minq = NONE32;
    return;
  }
  const int64_t ms = wave_min_i64(best);
  int64_t bid = INT64_MAX;
#pragma unroll
  for (int s = 0; s < S; ++s)
    if (valid[s] && st.qos[s] == ms && st.qid[s] < bid) bid = st.qid[s];
  const int64_t mi = wave_min_i64(bid);
  uint32_t q = NONE32;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    uint64_t m = ballot(valid[s] && st.qos[s] == ms && st.qid[s] == mi);
    if (m && q == NONE32) q = s * 64 + __builtin_ctzll(m);
  }
  st.minq = q;
  const uint32_t o = slot_get<S>(st.qinfo, q) & 0xFFFFu;
  st.min_sc = ms;
  st.min_id = mi;
  st.min_ts = slot_get<S>(st.pt, o);
}

// recompute_observed/5 (:301-334) for element e = {sc, id, {dc, ts}} of
// player q.
template <int S>
__device__ __forceinline__ void recompute_observed(KeyState<S>& st, uint32_t k, uint32_t q,
                                                   uint32_t e, int64_t id, int64_t sc, int64_t ts) {
  const uint32_t o = slot_get<S>(st.qinfo, q) & 0xFFFFu;
  if (o != NONE16) {  // Id in Observed (:303-315)
    const int64_t os = slot_get<S>(st.qos, q);
    const int64_t ots = slot_get<S>(st.pt, o);
    if (trmv_cmp(sc, id, ts, os, id, ots)) {
      uint32_t info = slot_get<S>(st.qinfo, q);
      slot_set<S>(st.qinfo, q, (info & 0xFFFF0000u) | e);
      slot_set<S>(st.qos, q, sc);
      if (q == st.minq) recompute_min<S>(st);  // Old =:= Min
    }
    return;
  }
  if (st.nobs < k) {  // (:317-324)
    set_obs<S>(st, q, e, sc);
    st.nobs++;
    if (st.minq == NONE32 || trmv_cmp(st.min_sc, st.min_id, st.min_ts, sc, id, ts)) {
      st.minq = q;
      st.min_sc = sc;
      st.min_id = id;
      st.min_ts = ts;
    }
    return;
  }
  if (trmv_cmp(sc, id, ts, st.min_sc, st.min_id, st.min_ts)) {  // (:325-331)
    unset_obs<S>(st, st.minq);
    set_obs<S>(st, q, e, sc);
    recompute_min<S>(st);
  }
}

template <int S>
__device__ __forceinline__ void emit_add(const TrmvApplyArgs& a, KeyState<S>& st, uint64_t op0,
                                         uint64_t op, int64_t id, int64_t sc, uint32_t dc,
                                         int64_t ts) {
  if (lane_id() == 0) {
    TrmvExtraRec r;
    r.op = (uint32_t)op;
    r.kind = CCRDT_TRMV_ADD;
    r.dc = (uint8_t)dc;
    r.pad = 0;
    r.id = id;
    r.score = sc;
    r.ts = ts;
    a.ex[op0 + st.nex] = r;
  }
  st.nex++;
}

template <int S>
__device__ __forceinline__ void emit_rmv_echo(const TrmvApplyArgs& a, KeyState<S>& st, uint64_t op0,
                                              uint64_t op, int64_t id, uint32_t row) {
  const int lane = lane_id();
  const uint64_t pos = op0 + st.nex;
  if (lane == 0) {
    TrmvExtraRec r;
    r.op = (uint32_t)op;
    r.kind = CCRDT_TRMV_RMV;
    r.dc = 0;
    r.pad = 0;
    r.id = id;
    r.score = 0;
    r.ts = 0;
    a.ex[pos] = r;
  }
  // the row lives in lanes (row%8)*8 + d of rv[row/8]
  const int d = lane & 7;
  if ((uint32_t)(lane >> 3) == (row & 7) && d < a.n_dc) {
#pragma unroll
    for (int s = 0; s < (int)KeyState<S>::RSLOTS; ++s)
      if ((row >> 3) == (uint32_t)s) a.ex_vc[pos * a.n_dc + d] = st.rv[s];
  }
  st.nex++;
}

// add/4 (:231-249)
template <int S>
__device__ __forceinline__ void op_add(const TrmvApplyArgs& a, KeyState<S>& st, uint64_t op0,
                                       uint64_t op, int64_t id, int64_t sc, uint32_t dc,
                                       int64_t ts) {
  const int lane = lane_id();
  int q = find_player<S>(st, id);
  const int64_t oldvc = rl64(st.vcv, dc);
  if ((uint32_t)lane == dc) st.vcv = ts > st.vcv ? ts : st.vcv;  // vc_update (:233)
  if (q >= 0) {
    const uint32_t row = slot_get<S>(st.qinfo, (uint32_t)q) >> 16;
    if (row != NONE16) {
      int64_t rts = 0;
#pragma unroll
      for (int s = 0; s < (int)KeyState<S>::RSLOTS; ++s)
        if ((row >> 3) == (uint32_t)s) rts = rl64(st.rv[s], ((row & 7) << 3) + dc);
      if (rts >= ts) {  // dominated (:234-237)
        emit_rmv_echo<S>(a, st, op0, op, id, row);
        return;
      }
    }
  }
  if (q < 0) {
    if (st.np >= KeyState<S>::CAP) {
      st.ovf = true;
      return;
    }
    q = (int)st.np++;
    slot_set<S>(st.qid, (uint32_t)q, id);
    slot_set<S>(st.qinfo, (uint32_t)q, NONE32);
  }
  // Masked[Id] := add_element(Elem) (:240-246).  Every element of dc has
  // ts <= Vc[dc], so a duplicate is only possible when ts <= old Vc[dc].
  int e = -1;
  if (ts <= oldvc) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const bool hit = (uint32_t)(s * 64 + lane) < st.npool && (st.pm[s] & PD_ALIVE) &&
                       (st.pm[s] & 0xFFFFu) == (uint32_t)q && ((st.pm[s] >> 16) & 0xFFu) == dc &&
                       st.pt[s] == ts && st.ps[s] == sc;
      const uint64_t m = ballot(hit);
      if (m && e < 0) e = s * 64 + __builtin_ctzll(m);
    }
  }
  if (e < 0) {
    if (st.npool >= KeyState<S>::CAP) {
      st.ovf = true;
      return;
    }
    e = (int)st.npool++;
    const bool inobs = (slot_get<S>(st.qinfo, (uint32_t)q) & 0xFFFFu) != NONE16;
    slot_set<S>(st.ps, (uint32_t)e, sc);
    slot_set<S>(st.pt, (uint32_t)e, ts);
    slot_set<S>(st.pm, (uint32_t)e, (uint32_t)q | (dc << 16) | PD_ALIVE | (inobs ? PD_INOBS : 0u));
  }
  recompute_observed<S>(st, a.k, (uint32_t)q, (uint32_t)e, id, sc, ts);
}

// rmv/3 (:252-298).  VcRmv is in stage[0..n_dc) (LDS).
template <int S>
__device__ __forceinline__ void op_rmv(const TrmvApplyArgs& a, KeyState<S>& st, uint64_t op0,
                                       uint64_t op, int64_t id, const int64_t* stage) {
  const int lane = lane_id();
  const int d8 = lane & 7;
  const int64_t vcr = lane < a.n_dc ? stage[lane] : 0;         // VcRmv, lane d
  const int64_t vsh = d8 < a.n_dc ? stage[d8] : 0;             // VcRmv, lane (r%8)*8+d
  int q = find_player<S>(st, id);
  if (q < 0) {
    if (st.np >= KeyState<S>::CAP) {
      st.ovf = true;
      return;
    }
    q = (int)st.np++;
    slot_set<S>(st.qid, (uint32_t)q, id);
    slot_set<S>(st.qinfo, (uint32_t)q, NONE32);
  }
  // merge_vc (:254, :369-375)
  uint32_t info = slot_get<S>(st.qinfo, (uint32_t)q);
  uint32_t row = info >> 16;
  if (row == NONE16) {
    if (st.nrows >= KeyState<S>::RCAP) {
      st.ovf = true;
      return;
    }
    row = st.nrows++;
    slot_set<S>(st.qinfo, (uint32_t)q, (info & 0xFFFFu) | (row << 16));
#pragma unroll
    for (int s = 0; s < (int)KeyState<S>::RSLOTS; ++s)
      if ((row >> 3) == (uint32_t)s && (uint32_t)(lane >> 3) == (row & 7)) st.rv[s] = vsh;
  } else {
#pragma unroll
    for (int s = 0; s < (int)KeyState<S>::RSLOTS; ++s)
      if ((row >> 3) == (uint32_t)s && (uint32_t)(lane >> 3) == (row & 7))
        st.rv[s] = vsh > st.rv[s] ? vsh : st.rv[s];
  }
  // filter Masked[Id] by Ts > VcRmv[DcId] (:255-266)
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const uint32_t pmv = st.pm[s];
    const uint32_t edc = (pmv >> 16) & 0xFFu;
    const int64_t vr = stage[edc & 7];
    const bool kill = (uint32_t)(s * 64 + lane) < st.npool && (pmv & PD_ALIVE) &&
                      (pmv & 0xFFFFu) == (uint32_t)q && st.pt[s] <= vr;
    if (kill) st.pm[s] = pmv & ~PD_ALIVE;
  }
  // impacts Observed? (:267-272)
  const uint32_t o = info & 0xFFFFu;
  if (o == NONE16) return;
  const uint32_t odc = (slot_get<S>(st.pm, o) >> 16) & 0xFFu;
  const int64_t ots = slot_get<S>(st.pt, o);
  if (rl64(vcr, odc) < ots) return;
  const bool was_min = (uint32_t)q == st.minq;
  unset_obs<S>(st, (uint32_t)q);
  st.nobs--;
  // promotion candidate: term-order largest alive element whose owner is not
  // in TmpObserved (:276-281, :291) — largest of per-Id largest.
  bool cand[S];
  bool any = false;
  int64_t best = INT64_MIN;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    cand[s] = (uint32_t)(s * 64 + lane) < st.npool && (st.pm[s] & PD_ALIVE) && !(st.pm[s] & PD_INOBS);
    if (cand[s] && st.ps[s] > best) best = st.ps[s];
    any |= ballot(cand[s]) != 0;
  }
  if (!any) {  // (:283-289)
    if (was_min) recompute_min<S>(st);
    return;
  }
  const int64_t ms = wave_max_i64(best);
  // ties on Score: resolve (Id, DcId, Ts) sequentially over the tie set
  uint32_t be = NONE32;
  int64_t bid = 0, bts = 0;
  uint32_t bdc = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    uint64_t m = ballot(cand[s] && st.ps[s] == ms);
    while (m) {
      const int l = __builtin_ctzll(m);
      m &= m - 1;
      const uint32_t e = s * 64 + l;
      const uint32_t pmv = rl32(st.pm[s], l);
      const int64_t eid = slot_get<S>(st.qid, pmv & 0xFFFFu);
      const uint32_t edc = (pmv >> 16) & 0xFFu;
      const int64_t ets = rl64(st.pt[s], l);
      const bool better = be == NONE32 || eid > bid || (eid == bid && edc > bdc) ||
                          (eid == bid && edc == bdc && ets > bts);
      if (better) {
        be = e;
        bid = eid;
        bdc = edc;
        bts = ets;
      }
    }
  }
  const uint32_t nq = slot_get<S>(st.pm, be) & 0xFFFFu;
  set_obs<S>(st, nq, be, ms);
  st.nobs++;
  recompute_min<S>(st);
  emit_add<S>(a, st, op0, op, bid, ms, bdc, bts);  // {add, {I, S, T}} (:295)
}

template <int S>
struct SeqLds {
  int64_t stage[64 * TRMV_DPAD];  // removal clocks of the current 64-op chunk
  uint16_t own[64 * S];           // load: owner player of flat pool entry e
  uint16_t src[64 * S];           // load: slab-relative index of entry e
};

template <int S>
__device__ __forceinline__ void trmv_process_key(const TrmvApplyArgs& a, uint32_t key,
                                                 SeqLds<S>& L) {
  const int lane = lane_id();
  const int D = a.n_dc;
  KeyState<S> st;
  const KeyMeta nmeta = a.new_s.meta[key];
  KeyMeta om;
  if (a.fresh) {
    om.p_off = om.m_off = om.r_off = 0;
    om.np = om.nm = om.nr = om.nobs = 0;
    om.minq = NONE32;
  } else {
    om = a.old_s.meta[key];
  }
  const uint64_t op0 = a.key_ptr[key];
  const uint64_t op1 = a.key_ptr[key + 1];
  st.ovf = om.np > KeyState<S>::CAP || om.nm > KeyState<S>::CAP || om.nr > KeyState<S>::RCAP;
  if (st.ovf) goto overflow;

  // ---- load the key's state into registers
  st.np = om.np;
  st.npool = om.nm;
  st.nrows = om.nr;
  st.nobs = om.nobs;
  st.minq = om.minq;
  st.nex = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    st.qid[s] = 0;
    st.qinfo[s] = NONE32;
    st.qos[s] = 0;
    st.ps[s] = 0;
    st.pt[s] = 0;
    st.pm[s] = 0xFFFFu;
  }
#pragma unroll
  for (int s = 0; s < (int)KeyState<S>::RSLOTS; ++s) st.rv[s] = 0;
  st.vcv = 0;
  st.min_sc = st.min_id = st.min_ts = 0;
  if (!a.fresh) {  // wave-uniform: fresh keys read nothing
    // players, and the flat position of every player's Masked slab
    V32<S> fs;
    uint32_t base = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const uint32_t p = s * 64 + lane;
      uint32_t slab = 0;
      if (p < st.np) {
        st.qid[s] = a.old_s.pl_id[om.p_off + p];
        st.qinfo[s] = a.old_s.pl_info[om.p_off + p];
        slab = a.old_s.pl_slab[om.p_off + p];
      }
      uint32_t tot;
      fs[s] = base + wave_excl_scan_u32(slab >> 16, tot);
      base += tot;
      // scatter owner / slab index of each of this player's elements
      for (uint32_t j = 0; j < (slab >> 16); ++j) {
        L.own[fs[s] + j] = (uint16_t)p;
        L.src[fs[s] + j] = (uint16_t)((slab & 0xFFFFu) + j);
      }
      // Observed index: slab-relative -> flat
      const uint32_t o = st.qinfo[s] & 0xFFFFu;
      if (p < st.np && o != NONE16) st.qinfo[s] = (st.qinfo[s] & 0xFFFF0000u) | (fs[s] + o);
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const uint32_t e = s * 64 + lane;
      if (e < st.npool) {
        const uint32_t q = L.own[e];
        const uint64_t g = (uint64_t)om.m_off + L.src[e];
        st.ps[s] = a.old_s.m_score[g];
        st.pt[s] = a.old_s.m_ts[g];
        st.pm[s] = q | ((uint32_t)a.old_s.m_dc[g] << 16) | PD_ALIVE;
      }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < S; ++s) {  // INOBS: owner is in Observed
      const uint32_t q = st.pm[s] & 0xFFFFu;
      const uint32_t qi = slot_gather<S>(st.qinfo, q == 0xFFFFu ? 0u : q);
      if (q != 0xFFFFu && (qi & 0xFFFFu) != NONE16) st.pm[s] |= PD_INOBS;
    }
#pragma unroll
    for (int s = 0; s < (int)KeyState<S>::RSLOTS; ++s) {
      const uint32_t r = s * 8 + (lane >> 3);
      const int d = lane & 7;
      if (r < st.nrows && d < D) st.rv[s] = a.old_s.r_vc[(uint64_t)(om.r_off + r) * D + d];
    }
    if (lane < D) st.vcv = a.old_s.vc[(uint64_t)key * D + lane];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const uint32_t o = st.qinfo[s] & 0xFFFFu;
      const int64_t v = slot_gather<S>(st.ps, o == NONE16 ? 0u : o);
      st.qos[s] = v;
    }
    if (st.minq != NONE32) {
      const uint32_t o = slot_get<S>(st.qinfo, st.minq) & 0xFFFFu;
      st.min_sc = slot_get<S>(st.ps, o);
      st.min_id = slot_get<S>(st.qid, st.minq);
      st.min_ts = slot_get<S>(st.pt, o);
    }
  }

  // ---- run the key's effects in stream order, 64 ops per chunk
  for (uint64_t base = op0; base < op1 && !st.ovf; base += 64) {
    const uint64_t i = base + lane;
    const bool v = i < op1;
    const uint32_t kd = v ? ((uint32_t)a.kind[i] | ((uint32_t)a.dc[i] << 8)) : 0u;
    const int64_t oid = v ? a.id[i] : 0;
    const int64_t osc = v ? a.score[i] : 0;
    const int64_t ots = v ? a.ts[i] : 0;
    // validate (reference: function_clause / engine range)
    uint32_t err = 0;
    if (v) {
      const uint32_t kk = kd & 0xFFu;
      if (kk > 3) err |= TRMV_ERR_KIND;
      else if (kk < 2) {
        if ((int)(kd >> 8) >= D) err |= TRMV_ERR_DC;
        if (ots < 1) err |= TRMV_ERR_TS;
      } else if (ots < 0 || ots >= a.n_rmv_rows) {
        err |= TRMV_ERR_ROW;
      }
    }
    // stage the removal clocks of this chunk's rmv ops in LDS
    const bool isr = v && !err && (kd & 0xFFu) >= 2 && (kd & 0xFFu) <= 3;
    if (isr) {
      for (int d = 0; d < D; ++d) {
        const int64_t x = a.rmv_vc[(uint64_t)ots * D + d];
        if (x < 0) err |= TRMV_ERR_VC;
        L.stage[lane * TRMV_DPAD + d] = x;
      }
    }
    const uint64_t em = ballot(err != 0);
    if (em) {
      if (err) atomicOr(&a.status[1], err);
      return;  // state of the whole batch is discarded by the host
    }
    __syncthreads();
    const int n = (int)((op1 - base) < 64 ? (op1 - base) : 64);
    for (int j = 0; j < n && !st.ovf; ++j) {
      const uint32_t k = rl32(kd, j);
      const int64_t id = rl64(oid, j);
      if ((k & 0xFFu) < 2) {
        op_add<S>(a, st, op0, base + j, id, rl64(osc, j), k >> 8, rl64(ots, j));
      } else {
        op_rmv<S>(a, st, op0, base + j, id, L.stage + j * TRMV_DPAD);
      }
    }
    __syncthreads();
  }
  if (st.ovf) goto overflow;

  // ---- write the new state: Masked elements grouped into one slab per
  // player (flat order inside a slab), removed elements dropped
  {
    V32<S> npos;
    V32<S> qslab;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      npos[s] = 0;
      qslab[s] = 0;
    }
    uint32_t base = 0;
    for (uint32_t q = 0; q < st.np; ++q) {
      uint32_t c = 0;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const bool mine = (uint32_t)(s * 64 + lane) < st.npool && (st.pm[s] & PD_ALIVE) &&
                          (st.pm[s] & 0xFFFFu) == q;
        const uint64_t m = ballot(mine);
        if (mine) npos[s] = base + c + mbcnt(m);
        c += __builtin_popcountll(m);
      }
      slot_set<S>(qslab, q, base | (c << 16));
      base += c;
    }
    const uint32_t nm = base;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const bool al = (uint32_t)(s * 64 + lane) < st.npool && (st.pm[s] & PD_ALIVE);
      if (al) {
        const uint64_t dst = (uint64_t)nmeta.m_off + npos[s];
        a.new_s.m_score[dst] = st.ps[s];
        a.new_s.m_ts[dst] = st.pt[s];
        a.new_s.m_dc[dst] = (uint8_t)((st.pm[s] >> 16) & 0xFFu);
      }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const uint32_t p = s * 64 + lane;
      const uint32_t o = st.qinfo[s] & 0xFFFFu;
      const uint32_t no = slot_gather<S>(npos, o == NONE16 ? 0u : o);
      if (p < st.np) {
        a.new_s.pl_id[nmeta.p_off + p] = st.qid[s];
        const uint32_t rel = o == NONE16 ? NONE16 : no - (qslab[s] & 0xFFFFu);
        a.new_s.pl_info[nmeta.p_off + p] = (st.qinfo[s] & 0xFFFF0000u) | rel;
        a.new_s.pl_slab[nmeta.p_off + p] = qslab[s];
      }
    }
#pragma unroll
    for (int s = 0; s < (int)KeyState<S>::RSLOTS; ++s) {
      const uint32_t r = s * 8 + (lane >> 3);
      const int d = lane & 7;
      if (r < st.nrows && d < D) a.new_s.r_vc[(uint64_t)(nmeta.r_off + r) * D + d] = st.rv[s];
    }
    if (lane < D) a.new_s.vc[(uint64_t)key * D + lane] = st.vcv;
    if (lane == 0) {
      KeyMeta out = nmeta;
      out.np = st.np;
      out.nm = nm;
      out.nr = st.nrows;
      out.nobs = st.nobs;
      out.minq = st.minq;
      a.new_s.meta[key] = out;
      a.ex_cnt[key] = st.nex;
    }
  }
  return;

overflow:
  if (lane == 0) {
    const uint32_t pos = atomicAdd(&a.status[0], 1u);
    a.ovf_list[pos] = key;
  }
}

// S = 4 is held to 128 VGPRs (4 waves per SIMD; it spills ~200 B per lane):
// it runs beside tier 0 on the side chain, and a wave that needs more
// registers than one retiring tier-0 wave frees is not dispatched until
// tier 0 has drained (unbounded, 184 VGPRs: the side chain's class 4 took
// ~1.9 ms instead of 0.22 ms)
template <int S>
__global__ __launch_bounds__(64, S == 4 ? 4 : 1) void trmv_apply_kernel(TrmvApplyArgs a) {
  __shared__ SeqLds<S> lds;
  const uint32_t n = a.n_list_dev ? *a.n_list_dev : a.n_list;
  for (uint32_t w = blockIdx.x; w < n; w += gridDim.x) {
    const uint32_t key = a.key_list ? a.key_list[w] : w;
    trmv_process_key<S>(a, key, lds);
    __syncthreads();  // LDS is reused by the next key
  }
}

// ------------------------------------------------------------- capacity scan
// New segment capacities per key: old counts + this batch's ops on the key.
// Three exclusive scans (players, pool, rows) over n_keys, block = 256 x 4.
constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 4;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

__device__ __forceinline__ void caps_of(const TrmvApplyArgs& a, uint64_t k, uint64_t c[3]) {
  const uint64_t nops = a.key_ptr[k + 1] - a.key_ptr[k];
  if (a.fresh) {
    c[0] = c[1] = c[2] = nops;
  } else {
    const KeyMeta m = a.old_s.meta[k];
    c[0] = m.np + nops;
    c[1] = m.nm + nops;
    c[2] = m.nr + nops;
  }
  if (c[1] > TRMV_SEG_MAX) atomicOr(&a.status[1], TRMV_ERR_SEG);  // u16 slab offsets
}

__device__ __forceinline__ void block_scan3(uint64_t v[3], uint64_t total[3]) {
  // inclusive wave scan then cross-wave via LDS
  __shared__ uint64_t wsum[SCAN_BLOCK / 64][3];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t inc[3] = {v[0], v[1], v[2]};
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      uint64_t o = (uint64_t)shfl64((int64_t)inc[c], lane - off < 0 ? 0 : lane - off);
      if (lane >= off) inc[c] += o;
    }
  }
  if (lane == 63)
    for (int c = 0; c < 3; ++c) wsum[w][c] = inc[c];
  __syncthreads();
  for (int c = 0; c < 3; ++c) {
    uint64_t pre = 0, tot = 0;
    for (int j = 0; j < SCAN_BLOCK / 64; ++j) {
      if (j < w) pre += wsum[j][c];
      tot += wsum[j][c];
    }
    v[c] = pre + inc[c] - v[c];  // exclusive
    total[c] = tot;
  }
  __syncthreads();
}

__global__ __launch_bounds__(SCAN_BLOCK) void trmv_scan_partials(TrmvApplyArgs a, uint64_t* partials) {
  uint64_t sum[3] = {0, 0, 0};
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    const uint64_t k = base + j;
    if (k < (uint64_t)a.n_keys) {
      uint64_t c[3];
      caps_of(a, k, c);
      for (int x = 0; x < 3; ++x) sum[x] += c[x];
    }
  }
  uint64_t tot[3];
  block_scan3(sum, tot);
  if (threadIdx.x == 0)
    for (int x = 0; x < 3; ++x) partials[(uint64_t)blockIdx.x * 3 + x] = tot[x];
}

// Single block: exclusive scan of the per-tile partials; totals at [nb*3..].
__global__ __launch_bounds__(SCAN_BLOCK) void trmv_scan_tops(uint64_t* partials, uint64_t nb) {
  __shared__ uint64_t carry[3];
  if (threadIdx.x < 3) carry[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t b0 = 0; b0 < nb; b0 += SCAN_BLOCK) {
    const uint64_t b = b0 + threadIdx.x;
    uint64_t v[3] = {0, 0, 0};
    if (b < nb)
      for (int x = 0; x < 3; ++x) v[x] = partials[b * 3 + x];
    uint64_t tot[3];
    block_scan3(v, tot);
    if (b < nb)
      for (int x = 0; x < 3; ++x) partials[b * 3 + x] = v[x] + carry[x];
    __syncthreads();
    if (threadIdx.x < 3) carry[threadIdx.x] += tot[threadIdx.x];
    __syncthreads();
  }
  if (threadIdx.x < 3) partials[nb * 3 + threadIdx.x] = carry[threadIdx.x];
}

__global__ __launch_bounds__(SCAN_BLOCK) void trmv_scan_apply(TrmvApplyArgs a, const uint64_t* partials) {
  uint64_t c[SCAN_ITEMS][3];
  uint64_t sum[3] = {0, 0, 0};
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    const uint64_t k = base + j;
    if (k < (uint64_t)a.n_keys) caps_of(a, k, c[j]);
    else c[j][0] = c[j][1] = c[j][2] = 0;
    for (int x = 0; x < 3; ++x) sum[x] += c[j][x];
  }
  uint64_t tot[3];
  block_scan3(sum, tot);
  uint64_t run[3];
  for (int x = 0; x < 3; ++x) run[x] = partials[(uint64_t)blockIdx.x * 3 + x] + sum[x];
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    const uint64_t k = base + j;
    if (k < (uint64_t)a.n_keys) {
      KeyMeta m;
      m.p_off = (uint32_t)run[0];
      m.m_off = (uint32_t)run[1];
      m.r_off = (uint32_t)run[2];
      m.np = m.nm = m.nr = m.nobs = 0;
      m.minq = NONE32;
      a.new_s.meta[k] = m;
    }
    for (int x = 0; x < 3; ++x) run[x] += c[j][x];
  }
}

// ----------------------------------------------------------- downstream/2
// One wave per request, read-only probe of the resident state (:102-124).
__global__ __launch_bounds__(64) void trmv_downstream_kernel(TrmvDownArgs a) {
  const int lane = lane_id();
  const uint64_t r = blockIdx.x;
  const uint64_t key = a.key[r];
  const int D = a.n_dc;
  KeyMeta m;
  if (a.fresh) {
    m.p_off = m.m_off = m.r_off = 0;
    m.np = m.nm = m.nr = m.nobs = 0;
    m.minq = NONE32;
  } else {
    m = a.s.meta[key];
  }
  const int64_t id = a.id[r];
  // find player
  uint32_t q = NONE32;
  for (uint32_t b = 0; b < m.np && q == NONE32; b += 64) {
    const uint32_t p = b + lane;
    const uint64_t hit = ballot(p < m.np && a.s.pl_id[m.p_off + p] == id);
    if (hit) q = b + __builtin_ctzll(hit);
  }
  const uint32_t info = q == NONE32 ? NONE32 : a.s.pl_info[m.p_off + q];
  const uint32_t slab = q == NONE32 ? 0u : a.s.pl_slab[m.p_off + q];
  const uint32_t o = info & 0xFFFFu;
  uint8_t kind;
  if (a.op[r] == 0) {
    const int64_t sc = a.score[r], ts = a.ts[r];
    bool changes;
    if (o != NONE16) {
      const uint64_t g = (uint64_t)m.m_off + (slab & 0xFFFFu) + o;
      changes = trmv_cmp(sc, id, ts, a.s.m_score[g], id, a.s.m_ts[g]);
    } else if (m.minq == NONE32) {
      changes = true;  // cmp(_, nil) = true
    } else {
      const uint32_t mi = a.s.pl_info[m.p_off + m.minq] & 0xFFFFu;
      const uint32_t ms = a.s.pl_slab[m.p_off + m.minq];
      const uint64_t g = (uint64_t)m.m_off + (ms & 0xFFFFu) + mi;
      changes = trmv_cmp(sc, id, ts, a.s.m_score[g], a.s.pl_id[m.p_off + m.minq], a.s.m_ts[g]);
    }
    kind = changes ? CCRDT_TRMV_ADD : CCRDT_TRMV_ADD_R;
  } else {
    const bool in_masked = (slab >> 16) != 0;  // Id in Masked
    kind = !in_masked ? (uint8_t)CCRDT_NOOP : (o != NONE16 ? CCRDT_TRMV_RMV : CCRDT_TRMV_RMV_R);
    if (a.out_vc && lane < D)
      a.out_vc[r * D + lane] = a.fresh ? 0 : a.s.vc[key * D + lane];
  }
  if (lane == 0) a.out_kind[r] = kind;
}

// ------------------------------------------------------------- launchers
int trmv_launch_scan(const TrmvApplyArgs& a, uint64_t* partials, hipStream_t st) {
  const uint64_t nb = ((uint64_t)a.n_keys + SCAN_TILE - 1) / SCAN_TILE;
  if (nb == 0) return CCRDT_OK;
  hipLaunchKernelGGL(trmv_scan_partials, dim3((unsigned)nb), dim3(SCAN_BLOCK), 0, st, a, partials);
  hipLaunchKernelGGL(trmv_scan_tops, dim3(1), dim3(SCAN_BLOCK), 0, st, partials, nb);
  hipLaunchKernelGGL(trmv_scan_apply, dim3((unsigned)nb), dim3(SCAN_BLOCK), 0, st, a, partials);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

int trmv_launch_apply(const TrmvApplyArgs& a, int slots, uint64_t n_work, hipStream_t st) {
  if (n_work == 0) return CCRDT_OK;
  const dim3 grid((unsigned)n_work), block(64);
  switch (slots) {
    case 2: hipLaunchKernelGGL(trmv_apply_kernel<2>, grid, block, 0, st, a); break;
    case 4: hipLaunchKernelGGL(trmv_apply_kernel<4>, grid, block, 0, st, a); break;
    case 8: hipLaunchKernelGGL(trmv_apply_kernel<8>, grid, block, 0, st, a); break;
    case 16: hipLaunchKernelGGL(trmv_apply_kernel<16>, grid, block, 0, st, a); break;
    default: set_error("bad slot class"); return CCRDT_EINVAL;
  }
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

int trmv_launch_downstream(const TrmvDownArgs& a, hipStream_t st) {
  if (a.n == 0) return CCRDT_OK;
  hipLaunchKernelGGL(trmv_downstream_kernel, dim3((unsigned)a.n), dim3(64), 0, st, a);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

}  // namespace ccrdt
