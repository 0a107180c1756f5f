// trmv_fast.hip — per-player-parallel topk_rmv apply (the common case).
//
// Why it is exact.  Let P be the number of distinct Ids a key has ever seen
// (its player table: every Id with a Masked or Removals entry).  If P <= K,
// Observed can never be full when an add arrives (|Observed| <= players
// with Masked elements <= P - 1 < K for a new player), so
//   * recompute_observed/5 (topk_rmv.erl:301-334) never evicts: an add
//     inserts its player, or improves Obs[Id] by cmp/2 (:389-395);
//   * every player with Masked elements is in Observed, so the promotion
//     candidates of rmv/3 (:276-281) are only the removed player's own
//     surviving elements, and the promoted one is their gb_sets:largest;
//   * Min only feeds later evictions, which cannot happen; at the end
//     Min = min_observed(Observed) (:398-406), an invariant of the reference.
// So the key's state decomposes into independent per-player histories: each
// lane of the wave owns one player and replays that player's effects in
// stream order; only the replica Vc (elementwise max, order-free) and the
// final Min are shared.  Keys with P > K go to the sequential kernel
// (trmv_kernels.hip) through the overflow list.
//
// Per key (one wavefront):
//   1. hash the key's old players into LDS (id -> player index);
//   2. op lanes load their op (coalesced), look up / claim their Id (parallel
//      open addressing, new players numbered in claim order), count ops per
//      player;
//   3. counting sort of the key's ops by player (each player's list is then
//      re-sorted by op index, so replay order = stream order);
//   4. player lanes replay their ops against their own Masked slab, Removals
//      row (registers) and Obs element;
//   5. Vc (LDS atomic max), Min (wave reduction), metadata.
// Two tiers: SMALL keeps the op fields, the removal clocks and the Masked
// slabs in LDS (every replay access is an LDS access; the slabs go to HBM in
// one coalesced pass); LARGE has 2x the caps and works on the slabs in HBM.
#include "common.hpp"
#include "trmv_kernels.hpp"

namespace ccrdt {

constexpr uint32_t F_CLAIM = 1u << 31;

template <bool SMALL>
struct FastCfg;
template <>
struct FastCfg<true> {
  static constexpr int HCAP = 256, PCAP = 128, OCAP = 192, MCAP = 192, RCAP = 16;
};
template <>
struct FastCfg<false> {
  static constexpr int HCAP = 512, PCAP = 256, OCAP = 512, MCAP = 1, RCAP = 1;
};

template <bool SMALL>
struct FastLds {
  using C = FastCfg<SMALL>;
  uint32_t hslot[C::HCAP];  // 0 empty | player+1 | F_CLAIM|lane (claim in flight)
  int64_t pid[C::PCAP];     // player ids
  unsigned long long vc[TRMV_DPAD];  // replica Vc (values >= 0)
  uint32_t kd[C::OCAP];     // player << 16 | dc << 8 | kind
  uint16_t sorted[C::OCAP]; // ops grouped by player
  uint32_t pcnt[C::PCAP];   // ops per player in this batch
  uint32_t pfill[C::PCAP];
  uint32_t pstart[C::PCAP];
  uint32_t nex;             // extra effects emitted by this key
  uint32_t nrmv;            // staged removal clocks
  // SMALL only: op fields, removal clocks, working Masked slabs
  int64_t osc[SMALL ? C::OCAP : 1];  // score (rmv: staged clock slot or -1)
  int64_t ots[SMALL ? C::OCAP : 1];  // ts (rmv: row of rmv_vc)
  int64_t rvc[SMALL ? C::RCAP * TRMV_DPAD : 1];
  int64_t msc[SMALL ? C::MCAP : 64];  // (LARGE: claim ids)
  int64_t mts[SMALL ? C::MCAP : 1];
  uint8_t mdc[SMALL ? C::MCAP : 1];
};

__device__ __forceinline__ uint32_t hash_id(int64_t id) {
  const uint64_t x = (uint64_t)id * 0x9E3779B97F4A7C15ull;
  return (uint32_t)(x >> 40);
}

// Removal clocks live in registers as an 8-wide vector (never in scratch).
typedef int64_t Row8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int64_t pick8(const Row8& v, uint32_t d) {
  int64_t r = v[0];
#pragma unroll
  for (int k = 1; k < TRMV_DPAD; ++k) r = d == (uint32_t)k ? v[k] : r;
  return r;
}

template <bool SMALL>
__device__ __forceinline__ void emit_extra(const TrmvApplyArgs& a, FastLds<SMALL>& L, uint64_t op0,
                                           uint64_t op, uint8_t kind, int64_t id, int64_t sc,
                                           uint32_t dc, int64_t ts, const Row8& row) {
  const uint32_t pos = atomicAdd(&L.nex, 1u);
  TrmvExtraRec r;
  r.op = (uint32_t)op;
  r.kind = kind;
  r.dc = (uint8_t)dc;
  r.pad = 0;
  r.id = id;
  r.score = sc;
  r.ts = ts;
  a.ex[op0 + pos] = r;
  if (kind == CCRDT_TRMV_RMV)
#pragma unroll
    for (int d = 0; d < TRMV_DPAD; ++d)
      if (d < a.n_dc) a.ex_vc[(op0 + pos) * a.n_dc + d] = row[d];
}

// Masked slab of one player: LDS (SMALL) or the new pool in HBM (LARGE).
template <bool SMALL>
struct Slab {
  FastLds<SMALL>& L;
  const TrmvSide& s;
  uint64_t g;  // SMALL: LDS index; LARGE: pool index
  __device__ __forceinline__ int64_t sc(uint32_t j) const { return SMALL ? L.msc[g + j] : s.m_score[g + j]; }
  __device__ __forceinline__ int64_t ts(uint32_t j) const { return SMALL ? L.mts[g + j] : s.m_ts[g + j]; }
  __device__ __forceinline__ uint32_t dc(uint32_t j) const { return SMALL ? L.mdc[g + j] : s.m_dc[g + j]; }
  __device__ __forceinline__ void set(uint32_t j, int64_t v, int64_t t, uint32_t d) const {
    if (SMALL) {
      L.msc[g + j] = v;
      L.mts[g + j] = t;
      L.mdc[g + j] = (uint8_t)d;
    } else {
      s.m_score[g + j] = v;
      s.m_ts[g + j] = t;
      s.m_dc[g + j] = (uint8_t)d;
    }
  }
};

// Returns false (having written nothing to HBM) if the key must take the
// next tier.
template <bool SMALL>
__device__ __forceinline__ bool trmv_fast_key(const TrmvApplyArgs& a, uint32_t key,
                                              FastLds<SMALL>& L) {
  using C = FastCfg<SMALL>;
  const int lane = lane_id();
  const int D = a.n_dc;
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
  const uint32_t nops = (uint32_t)(op1 - op0);
  const uint32_t pmax = a.k < (uint32_t)C::PCAP ? a.k : (uint32_t)C::PCAP;
  if (nops > (uint32_t)C::OCAP || om.np > pmax) return false;
  if (SMALL && om.nm + nops > (uint32_t)C::MCAP) return false;

  // ---- 1. clear LDS, hash the old players
  for (int i = lane; i < C::HCAP; i += 64) L.hslot[i] = 0;
  for (int i = lane; i < C::PCAP; i += 64) {
    L.pcnt[i] = 0;
    L.pfill[i] = 0;
  }
  if (lane < TRMV_DPAD)
    L.vc[lane] = (!a.fresh && lane < D) ? (unsigned long long)a.old_s.vc[(uint64_t)key * D + lane] : 0ull;
  if (lane == 0) {
    L.nex = 0;
    L.nrmv = 0;
  }
  __syncthreads();
  bool bad = false;
  for (uint32_t b = 0; b < om.np; b += 64) {
    const uint32_t p = b + lane;
    if (p < om.np) {
      const int64_t id = a.old_s.pl_id[om.p_off + p];
      L.pid[p] = id;
      uint32_t h = hash_id(id) & (C::HCAP - 1);
      while (atomicCAS(&L.hslot[h], 0u, p + 1) != 0u) h = (h + 1) & (C::HCAP - 1);
      // every player with Masked elements must be in Observed (true for any
      // state with P <= K that the reference's transitions can reach)
      const bool has_m = (a.old_s.pl_slab[om.p_off + p] >> 16) != 0;
      const bool in_o = (a.old_s.pl_info[om.p_off + p] & 0xFFFFu) != NONE16;
      bad |= has_m != in_o;
    }
  }
  if (ballot(bad)) return false;
  __syncthreads();

  // ---- 2. load ops, player of every op (new Ids claimed in lane order)
  int64_t* claim_id = SMALL ? L.msc : L.msc;  // LDS scratch, 64 entries
  uint32_t np = om.np;
  uint32_t err = 0;
  for (uint32_t b = 0; b < nops; b += 64) {
    const uint32_t l = b + lane;
    const bool valid = l < nops;
    const uint64_t i = op0 + l;
    const int64_t id = valid ? a.id[i] : 0;
    uint32_t kd = 0;
    if (SMALL && valid) {
      const uint32_t kind = a.kind[i], dc = a.dc[i];
      const int64_t sc = a.score[i], t = a.ts[i];
      kd = kind | (dc << 8);
      int64_t slot = -1;
      if (kind > 3) {
        err |= TRMV_ERR_KIND;
      } else if (kind < 2) {
        if ((int)dc >= D) err |= TRMV_ERR_DC;
        if (t < 1) err |= TRMV_ERR_TS;
      } else if (t < 0 || t >= a.n_rmv_rows) {
        err |= TRMV_ERR_ROW;
      } else {
        const uint32_t r = atomicAdd(&L.nrmv, 1u);
        if (r < (uint32_t)C::RCAP) {
          slot = r;
#pragma unroll
          for (int d = 0; d < TRMV_DPAD; ++d) {
            const int64_t x = d < D ? a.rmv_vc[(uint64_t)t * D + d] : 0;
            if (x < 0) err |= TRMV_ERR_VC;
            L.rvc[r * TRMV_DPAD + d] = x;
          }
        }
      }
      L.osc[l] = kind < 2 ? sc : slot;
      L.ots[l] = t;
    }
    claim_id[lane] = id;
    __syncthreads();
    uint32_t h = hash_id(id) & (C::HCAP - 1);
    bool resolved = !valid, claimed = false;
    int follow = -1;
    uint32_t p = 0;
    while (ballot(!resolved)) {
      if (!resolved) {
        const uint32_t s = L.hslot[h];
        if (s == 0u) {
          if (atomicCAS(&L.hslot[h], 0u, F_CLAIM | (uint32_t)lane) == 0u) {
            claimed = true;
            resolved = true;
          }  // lost the race: re-read the slot next round
        } else if (s & F_CLAIM) {
          const int c = (int)(s & 63u);
          if (claim_id[c] == id) {
            follow = c;
            resolved = true;
          } else {
            h = (h + 1) & (C::HCAP - 1);
          }
        } else if (L.pid[s - 1] == id) {
          p = s - 1;
          resolved = true;
        } else {
          h = (h + 1) & (C::HCAP - 1);
        }
      }
    }
    const uint64_t cm = ballot(claimed);
    if (claimed) {
      p = np + mbcnt(cm);
      if (p < (uint32_t)C::PCAP) L.pid[p] = id;
      L.hslot[h] = p + 1;
    }
    np += (uint32_t)__builtin_popcountll(cm);
    const uint32_t fp = shfl32(p, follow >= 0 ? follow : lane);
    if (follow >= 0) p = fp;
    if (np > pmax) return false;  // Observed could fill: next tier
    if (valid) {
      L.kd[l] = kd | (p << 16);
      atomicAdd(&L.pcnt[p], 1u);
    }
    __syncthreads();
  }
  if (SMALL && ballot(err != 0)) {
    if (err) atomicOr(&a.status[1], err);
    return true;  // the host rejects the batch
  }

  // ---- 3. counting sort of ops by player
  {
    uint32_t base = 0;
    for (uint32_t b = 0; b < np; b += 64) {
      const uint32_t p = b + lane;
      const uint32_t c = p < np ? L.pcnt[p] : 0u;
      uint32_t tot;
      const uint32_t ex = wave_excl_scan_u32(c, tot);
      if (p < np) L.pstart[p] = base + ex;
      base += tot;
    }
  }
  __syncthreads();
  for (uint32_t l = lane; l < nops; l += 64) {
    const uint32_t p = L.kd[l] >> 16;
    const uint32_t pos = atomicAdd(&L.pfill[p], 1u);
    L.sorted[L.pstart[p] + pos] = (uint16_t)l;
  }
  __syncthreads();

  // ---- 4. replay each player's ops (lane = player)
  uint32_t slab_base = 0, row_base = 0, nm = 0, nobs = 0;
  int64_t best_sc = 0, best_id = 0;
  uint32_t best_q = NONE32;
  for (uint32_t b = 0; b < np; b += 64) {
    const uint32_t p = b + lane;
    const bool act = p < np;
    const uint32_t cnt_ops = act ? L.pcnt[p] : 0u;
    const uint32_t st0 = act ? L.pstart[p] : 0u;
    // stable order: insertion sort of this player's op list
    for (uint32_t x = 1; x < cnt_ops; ++x) {
      const uint16_t v = L.sorted[st0 + x];
      uint32_t y = x;
      while (y > 0 && L.sorted[st0 + y - 1] > v) {
        L.sorted[st0 + y] = L.sorted[st0 + y - 1];
        --y;
      }
      L.sorted[st0 + y] = v;
    }
    uint32_t info = NONE32, slab_old = 0;
    if (act && p < om.np) {
      info = a.old_s.pl_info[om.p_off + p];
      slab_old = a.old_s.pl_slab[om.p_off + p];
    }
    const uint32_t cnt_old = slab_old >> 16;
    uint32_t tot;
    const uint32_t moff = slab_base + wave_excl_scan_u32(act ? cnt_old + cnt_ops : 0u, tot);
    slab_base += tot;
    const Slab<SMALL> sl{L, a.new_s, SMALL ? (uint64_t)moff : (uint64_t)nmeta.m_off + moff};
    // maxts bounds the ts of every element ever in the slab: an add with a
    // larger ts cannot duplicate one (skips the set-membership scan)
    int64_t maxts = 0;
    for (uint32_t j = 0; j < cnt_old; ++j) {  // copy the old slab
      const uint64_t go = (uint64_t)om.m_off + (slab_old & 0xFFFFu) + j;
      const int64_t t = a.old_s.m_ts[go];
      maxts = t > maxts ? t : maxts;
      sl.set(j, a.old_s.m_score[go], t, a.old_s.m_dc[go]);
    }
    uint32_t cnt = cnt_old;
    uint32_t o = info & 0xFFFFu;  // Obs[Id] as slab index
    int64_t osc = 0, ots = 0;
    if (act && o != NONE16) {
      osc = sl.sc(o);
      ots = sl.ts(o);
    }
    bool has_row = false;
    Row8 row = (Row8)(0);
    if (act && (info >> 16) != NONE16) {
      has_row = true;
      const uint64_t r0 = ((uint64_t)om.r_off + (info >> 16)) * D;
#pragma unroll
      for (int d = 0; d < TRMV_DPAD; ++d)
        if (d < D) row[d] = a.old_s.r_vc[r0 + d];
    }
    const int64_t id = act ? L.pid[p] : 0;
    for (uint32_t x = 0; x < cnt_ops; ++x) {
      const uint32_t l = L.sorted[st0 + x];
      const uint64_t i = op0 + l;
      uint32_t kind, dc;
      int64_t sc, tsf;
      if (SMALL) {
        kind = L.kd[l] & 0xFFu;
        dc = (L.kd[l] >> 8) & 0xFFu;
        sc = L.osc[l];
        tsf = L.ots[l];
      } else {
        kind = a.kind[i];
        dc = a.dc[i];
        sc = a.score[i];
        tsf = a.ts[i];
        if (kind > 3) {
          err |= TRMV_ERR_KIND;
          break;
        }
        if (kind < 2 && ((int)dc >= D || tsf < 1)) {
          err |= ((int)dc >= D ? TRMV_ERR_DC : 0u) | (tsf < 1 ? TRMV_ERR_TS : 0u);
          break;
        }
        if (kind >= 2 && (tsf < 0 || tsf >= a.n_rmv_rows)) {
          err |= TRMV_ERR_ROW;
          break;
        }
      }
      if (kind < 2) {  // add/4 (:231-249)
        atomicMax(&L.vc[dc], (unsigned long long)tsf);  // vc_update (:233)
        if (has_row && pick8(row, dc) >= tsf) {          // dominated (:234-237)
          emit_extra<SMALL>(a, L, op0, i, CCRDT_TRMV_RMV, id, 0, 0, 0, row);
          continue;
        }
        uint32_t e = NONE32;  // gb_sets:add_element (set semantics)
        if (tsf <= maxts)
          for (uint32_t j = 0; j < cnt && e == NONE32; ++j)
            if (sl.ts(j) == tsf && sl.dc(j) == dc && sl.sc(j) == sc) e = j;
        maxts = tsf > maxts ? tsf : maxts;
        if (e == NONE32) {
          e = cnt++;
          sl.set(e, sc, tsf, dc);
        }
        // recompute_observed (:301-324; never full here)
        if (o == NONE16 || sc > osc || (sc == osc && tsf > ots)) {
          o = e;
          osc = sc;
          ots = tsf;
        }
      } else {  // rmv/3 (:252-298)
        Row8 vr = (Row8)(0);
        const bool staged = SMALL && sc >= 0;
#pragma unroll
        for (int d = 0; d < TRMV_DPAD; ++d) {
          if (staged) {
            vr[d] = L.rvc[sc * TRMV_DPAD + d];
          } else {
            vr[d] = d < D ? a.rmv_vc[(uint64_t)tsf * D + d] : 0;
            if (vr[d] < 0) err |= TRMV_ERR_VC;
          }
          row[d] = has_row ? (vr[d] > row[d] ? vr[d] : row[d]) : vr[d];  // merge_vc
        }
        has_row = true;
        // filter Masked[Id]: keep Ts > VcRmv[DcId] (:255-266)
        uint32_t w = 0, no = NONE16;
        for (uint32_t j = 0; j < cnt; ++j) {
          const int64_t t = sl.ts(j);
          const uint32_t edc = sl.dc(j);
          if (t > pick8(vr, edc)) {
            if (w != j) sl.set(w, sl.sc(j), t, edc);
            if (j == o) no = w;
            ++w;
          }
        }
        cnt = w;
        if (o != NONE16 && no == NONE16) {  // impacts Observed (:267-272)
          if (cnt == 0) {
            o = NONE16;
          } else {  // promote gb_sets:largest of the survivors (:291-295)
            uint32_t bj = 0;
            int64_t bsc = sl.sc(0), bts = sl.ts(0);
            uint32_t bdc = sl.dc(0);
            for (uint32_t j = 1; j < cnt; ++j) {
              const int64_t s2 = sl.sc(j), t2 = sl.ts(j);
              const uint32_t d2 = sl.dc(j);
              if (s2 > bsc || (s2 == bsc && (d2 > bdc || (d2 == bdc && t2 > bts)))) {
                bj = j;
                bsc = s2;
                bts = t2;
                bdc = d2;
              }
            }
            o = bj;
            osc = bsc;
            ots = bts;
            emit_extra<SMALL>(a, L, op0, i, CCRDT_TRMV_ADD, id, bsc, bdc, bts, row);
          }
        } else {
          o = no;
        }
      }
    }
    if (SMALL)  // mark the unused tail of the slab as a hole
      for (uint32_t j = cnt; j < cnt_old + cnt_ops; ++j) L.mdc[moff + j] = 0xFF;
    // removal row index (player order) and the player record
    const uint64_t rm = ballot(act && has_row);
    const uint32_t rix = row_base + mbcnt(rm);
    row_base += (uint32_t)__builtin_popcountll(rm);
    if (act) {
      a.new_s.pl_id[nmeta.p_off + p] = id;
      a.new_s.pl_info[nmeta.p_off + p] = (o == NONE16 ? NONE16 : o) | ((has_row ? rix : NONE16) << 16);
      a.new_s.pl_slab[nmeta.p_off + p] = moff | (cnt << 16);
      if (has_row) {
        const uint64_t r0 = ((uint64_t)nmeta.r_off + rix) * D;
#pragma unroll
        for (int d = 0; d < TRMV_DPAD; ++d)
          if (d < D) a.new_s.r_vc[r0 + d] = row[d];
      }
    }
    // lane-local counts and Min candidate (reduced once per key below)
    const bool inobs = act && o != NONE16;
    nobs += (uint32_t)__builtin_popcountll(ballot(inobs));
    nm += act ? cnt : 0u;
    if (inobs && (best_q == NONE32 || osc < best_sc || (osc == best_sc && id < best_id))) {
      best_q = p;
      best_sc = osc;
      best_id = id;
    }
  }
  // Min = min_observed(Observed) by (Score, Id) — Ids are distinct
  {
    const bool has = best_q != NONE32;
    if (ballot(has)) {
      const int64_t ms = wave_min_i64(has ? best_sc : INT64_MAX);
      const int64_t mi = wave_min_i64(has && best_sc == ms ? best_id : INT64_MAX);
      const uint64_t hit = ballot(has && best_sc == ms && best_id == mi);
      best_q = shfl32(best_q, (int)__builtin_ctzll(hit));
      best_q = rl32(best_q, 0);
    } else {
      best_q = NONE32;
    }
    uint32_t tot;
    (void)wave_excl_scan_u32(nm, tot);
    nm = tot;
  }
  if (ballot(err != 0)) {
    if (err) atomicOr(&a.status[1], err);
    return true;  // the host rejects the batch
  }
  __syncthreads();
  // ---- 5. Masked slabs to HBM (SMALL), Vc, metadata
  if (SMALL) {
    for (uint32_t j = lane; j < slab_base; j += 64) {
      const uint32_t d = L.mdc[j];
      if (d != 0xFFu) {
        const uint64_t gj = (uint64_t)nmeta.m_off + j;
        a.new_s.m_score[gj] = L.msc[j];
        a.new_s.m_ts[gj] = L.mts[j];
        a.new_s.m_dc[gj] = (uint8_t)d;
      }
    }
  }
  if (lane < D) a.new_s.vc[(uint64_t)key * D + lane] = (int64_t)L.vc[lane];
  if (lane == 0) {
    KeyMeta out = nmeta;
    out.np = np;
    out.nm = nm;
    out.nr = row_base;
    out.nobs = nobs;
    out.minq = best_q;
    a.new_s.meta[key] = out;
    a.ex_cnt[key] = L.nex;
  }
  return true;
}

template <bool SMALL>
__global__ __launch_bounds__(64) void trmv_fast_kernel(TrmvApplyArgs a) {
  __shared__ FastLds<SMALL> lds;
  // grid-stride over the work list; its length may only be known on the
  // device (overflow count of the previous tier), so the host never waits
  const uint32_t n = a.n_list_dev ? *a.n_list_dev : a.n_list;
  for (uint32_t w = blockIdx.x; w < n; w += gridDim.x) {
    const uint32_t key = a.key_list ? a.key_list[w] : w;
    if (!trmv_fast_key<SMALL>(a, key, lds)) {
      if (lane_id() == 0) {
        const uint32_t pos = atomicAdd(&a.status[0], 1u);
        a.ovf_list[pos] = key;
      }
    }
    __syncthreads();  // LDS is reused by the next key
  }
}

// tier 0 = SMALL (all-LDS), tier 1 = LARGE (slabs in HBM)
int trmv_launch_fast(const TrmvApplyArgs& a, int tier, uint64_t n_work, hipStream_t st) {
  if (n_work == 0) return CCRDT_OK;
  // tier 0 is trmv_wave.hip; this file's LDS variant is kept only as the
  // reference formulation the wave kernel was derived from (not launched)
  if (tier != 1) {
    set_error("trmv_launch_fast: only the HBM-slab tier (1) is launched from here");
    return CCRDT_EINVAL;
  }
  hipLaunchKernelGGL(trmv_fast_kernel<false>, dim3((unsigned)n_work), dim3(64), 0, st, a);
  // (n_work is the grid: all keys for the first tier, a bound for later ones)
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

}  // namespace ccrdt

