// trmv_steady.hip — tier S of the topk_rmv apply: any key, fresh or resident,
// any number of ops, Masked slabs of any size inside the key's segment, and
// Observed full with more players than K (evictions, promotions).  One
// wavefront per key.  Tier 0 (trmv_wave.hip) takes the keys whose history
// decomposes per player; everything else ends here.
//
// Why the sequential part is small.  The reference state machine
// (src/antidote_ccrdt_topk_rmv.erl:231-334) keeps this invariant after every
// op (proof in DESIGN.md §4.1):
//   * Obs[Id] has the largest Score in Masked[Id] (Q2: Obs[Id] ∈ Masked[Id]);
//   * if |Observed| = K, every Id outside Observed ranks below Min by
//     (max Score of Masked[Id], Id); if |Observed| < K, every Id with Masked
//     elements is in Observed.
// So Observed is the top K players by (max Score, Id), and only three things
// depend on the order of ops across players: which element of a player is
// Obs[Id] when Scores tie inside Masked[Id] (cmp/2 keeps the first arrival,
// :389-395; a promotion takes gb_sets:largest, :291), Min, and the extra
// effects.  Everything per player — Removals[Id] merges, the rmv filters of
// Masked[Id], dominated adds (:234) and set semantics (:240-246) — is decided
// per player, off the sequential path:
//   K1  old players -> LDS (Id hash, old slab, Obs[Id] and gb_sets:largest
//       elements gathered from the pool);
//   K2  every op's player (new Ids numbered in claim order), ops per player,
//       new slab offsets (old count + ops: the key's new segment), new
//       Removals rows;
//   K3  old Masked slabs and Removals rows -> the new side, position-parallel
//       (coalesced), except the slabs of players with a rmv in the batch;
//   K4  per chunk of <= 64 ops (<= 16 rmvs): ops sorted by player (wave radix
//       sort); players without a rmv append their non-dominated adds
//       op-parallel; players with a rmv (or a possibly duplicated element) are
//       replayed by one lane each over their own slab and Removals row
//       (Masked filter, merge_vc, dominance, set semantics, the largest
//       survivor after each rmv); then one uniform pass over the chunk's ops
//       in stream order does recompute_observed/5 and the Observed half of
//       rmv/3 (impact, promotion, Min) with per-player LDS state;
//   K5  Obs/largest positions of replayed players, player records, Vc, meta.
#include <algorithm>
#include <type_traits>

#include "common.hpp"
#include "trmv_kernels.hpp"

// Diagnostic build only (-DTRMV_PROF): per-phase s_memtime stamps summed over
// a sample of keys; read with ccrdt_debug_steady_prof().
#ifdef TRMV_PROF
__device__ unsigned long long g_steady_prof[16];
#define SPROF_STAMP(v)                                                        \
  do {                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                        \
  } while (0)
#define SPROF(i)                                                                              \
  do {                                                                                        \
    unsigned long long _t;                                                                    \
    SPROF_STAMP(_t);                                                                          \
    if (lane_id() == 0 && (key & 63u) == 3) atomicAdd(&g_steady_prof[i], _t - prof_t);      \
    prof_t = _t;                                                                              \
  } while (0)
#define SCOUNT(i, v)                                                             \
  do {                                                                           \
    if (lane_id() == 0 && (key & 63u) == 3) atomicAdd(&g_steady_prof[i], (unsigned long long)(v)); \
  } while (0)
#else
#define SPROF_STAMP(v) (void)0
#define SPROF(i) (void)0
#define SCOUNT(i, v) (void)0
#endif

namespace ccrdt {

namespace {

#define KA trmv_kargs()  // (trmv_kernels.hpp)

constexpr int S_CH = 64;    // ops per chunk
constexpr int S_CHR = 16;   // rmvs per chunk (rows of the clock table)
constexpr uint32_t S_NONE = 0xFFFFFFFFu;
// opd[p] = flags (8) | Obs[Id] dc (8) | Obs[Id] slab position (16)
constexpr uint32_t F_OBS = 1u;    // Id in Observed
constexpr uint32_t F_HASM = 2u;   // Masked[Id] is not empty
constexpr uint32_t F_RMV = 4u;    // a rmv of Id in this batch: slab and row replayed by one lane
constexpr uint32_t F_MAT = 8u;    // (F_RMV) old slab already copied to the new region
constexpr uint32_t F_ROWV = 16u;  // the player's Removals row holds an entry
constexpr uint32_t F_WALK = 32u;  // slab compacted by a replay: positions restated at the end
constexpr uint32_t R_DOM = 1u;    // cres: dominated add (:234-237)

enum : int { S_DONE = 0, S_NEXT = 1, S_REJECT = 2 };

template <int N>
struct Log2 {
  static constexpr int v = 1 + Log2<N / 2>::v;
};
template <>
struct Log2<1> {
  static constexpr int v = 0;
};

// Hash slots hold a player index, a claim (CLAIM | lane) or NONE; u16 for
// up to 256 players (LDS is what bounds the waves per CU), u32 above.
template <int PCAP>
struct HSlot {
  using T = typename std::conditional<(PCAP <= 256), uint16_t, uint32_t>::type;
  static constexpr uint32_t NONE = (uint32_t)(T)~(T)0;
  static constexpr uint32_t CLAIM = (uint32_t)1 << (8 * sizeof(T) - 1);
};

// RANKED (K <= 128): Obs[Id]'s Score / Ts live with Observed's sorted entries
// (tsc/tts by rank, ork = a player's rank), not per player, which keeps the
// 256-player class at 4 workgroups (8 waves) per CU.
template <int PCAP, bool RANKED>
struct alignas(16) SLds {
  static constexpr int HS = 2 * PCAP;
  static constexpr int NP = RANKED ? 0 : PCAP + 1;  // per-player Obs[Id] arrays (unranked only)
  static constexpr int NR = RANKED ? 128 : 0;       // Observed entries (ranked only)
  typename HSlot<PCAP>::T hs[HS];        // Id hash: player | CLAIM|lane | NONE
  int64_t pid[PCAP + 1];                 // player Ids
  int64_t osc[NP], ots[NP];              // Obs[Id]: Score, Ts (unranked)
  int64_t gsc[PCAP + 1], gts[PCAP + 1];  // gb_sets:largest(Masked[Id]): Score, Ts
  uint32_t opd[PCAP + 1];                // flags | Obs dc << 8 | Obs position << 16
  uint32_t gpd[PCAP + 1];                // largest: dc << 8 | position << 16
  uint32_t oslab[PCAP + 1];              // old slab: offset | count << 16
  uint32_t orow[PCAP + 1];               // old Obs index | Removals row << 16 (new side)
  uint32_t nslab[PCAP + 1];              // new slab: offset | current count << 16
  struct Chunk {                         // the current chunk (stream order unless noted)
    int64_t csc[S_CH + 1], cts[S_CH + 1];
    uint32_t ckd[S_CH + 1];              // kind | dc << 2 | dup candidate << 5 | player << 8
    uint32_t cres[S_CH + 1];             // add: R_DOM | slab position << 16; rmv: its rank
    uint32_t crow[S_CHR + 1];            // rmv_vc row of the chunk's rmvs
    int64_t vtab[S_CHR][TRMV_DPAD];      // their clocks
    int64_t rgsc[S_CHR], rgts[S_CHR];    // Masked[Id]'s largest survivor after each rmv
    uint32_t rgd[S_CHR];                 // non-empty | dc << 8 | position << 16
    uint8_t csrt[S_CH];                  // sorted (player, stream) order -> stream index
    uint16_t cwp[S_CH];                  // replayed players of the chunk
    uint8_t cws[S_CH], cwe[S_CH];        // and their sorted ranges
    uint32_t mark[S_CH];                 // K3: player (+1) whose slab starts at a position
  };
  struct K2 {
    uint32_t nops[PCAP + 1];             // ops of each player in the batch
    int64_t claim[S_CH];                 // Ids being claimed
  };
  union {
    K2 k;
    Chunk c;
  } u;
  int64_t tsc[NR], tid[NR], tts[NR];     // Observed, sorted by (Score, Id): Score, Id, Ts
  uint16_t tp[NR];                       // and player
  uint8_t ork[RANKED ? PCAP + 1 : 0];    // rank of an observed player's entry
  unsigned long long vc[TRMV_DPAD + 1];  // replica Vc; [TRMV_DPAD] sink
  uint32_t nex;
  uint32_t nob;                          // K1: old Observed entries gathered
};

// The HBM class (PCAP > 1024) keeps SLds in a per-wave global scratch
// instead of LDS.  A wave's lanes hand values to each other through it, and
// atomics execute in L2 while plain loads may hit this CU's L1: every sync
// point waits for the wave's stores and invalidates the L1 (agent acquire),
// so the next loads see what every lane wrote.  Slow, and only for keys past
// the LDS classes.
constexpr int PCAP_HBM = 16384;
template <int PCAP, bool RK>
__device__ __forceinline__ void lsync(const SLds<PCAP, RK>&) {
  if constexpr (PCAP > 1024) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    __builtin_amdgcn_s_waitcnt(0x0F70);
  }
  wave_lds_sync();
}

template <int PCAP>
__device__ __forceinline__ uint32_t shash(int64_t id) {
  constexpr int B = Log2<2 * PCAP>::v;
  return (uint32_t)(((uint64_t)id * 0x9E3779B97F4A7C15ull) >> (64 - B));
}

// Compare-and-swap on one hash slot (u16 slots: on their 32-bit word);
// returns the slot's value before (== expect on success).
template <int PCAP, bool RK>
__device__ __forceinline__ uint32_t hs_cas(SLds<PCAP, RK>& L, uint32_t h, uint32_t expect, uint32_t val) {
  if constexpr (sizeof(L.hs[0]) == 4) {
    return atomicCAS(reinterpret_cast<uint32_t*>(&L.hs[h]), expect, val);
  } else {
    uint32_t* w = reinterpret_cast<uint32_t*>(&L.hs[h & ~1u]);
    const uint32_t sh = (h & 1u) * 16u;
    uint32_t old = *w;
    for (;;) {
      const uint32_t cur = (old >> sh) & 0xFFFFu;
      if (cur != expect) return cur;
      const uint32_t prev = atomicCAS(w, old, (old & ~(0xFFFFu << sh)) | (val << sh));
      if (prev == old) return expect;
      old = prev;
    }
  }
}

__device__ __forceinline__ uint32_t ufl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int64_t ufl64(int64_t v) {
  const uint32_t lo = ufl((uint32_t)v), hi = ufl((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Forward permute: lane i's v goes to lane dst (ds_permute).
__device__ __forceinline__ uint32_t perm32(uint32_t v, uint32_t dst) {
  return (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)v);
}

// Inclusive max-scan over the 64 lanes (DPP; identity 0).
__device__ __forceinline__ uint32_t wave_incl_max_dpp(uint32_t v) {
  uint32_t o;
  o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v = o > v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  v = o > v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
  v = o > v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
  v = o > v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v = o > v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  v = o > v ? o : v;
  return v;
}

// Stable sort of the wave by key bits [6, 6 + BITS) of kv (payload: low 6
// bits); one ballot split per bit.
template <int BITS>
__device__ __forceinline__ uint32_t wave_radix_sort(uint32_t kv) {
#pragma unroll
  for (int b = 0; b < BITS; ++b) {
    const bool bit = (kv >> (6 + b)) & 1u;
    const uint64_t ones = ballot(bit);
    const uint32_t nz = 64u - (uint32_t)__builtin_popcountll(ones);
    const uint32_t dst = bit ? nz + mbcnt(ones) : mbcnt(~ones);
    kv = perm32(kv, dst);
  }
  return kv;
}

typedef int64_t Row8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int64_t pick8(const Row8& v, uint32_t d) {
  int64_t r = v[0];
#pragma unroll
  for (int k = 1; k < TRMV_DPAD; ++k) r = d == (uint32_t)k ? v[k] : r;
  return r;
}

// gb_sets term order of two elements of one Id: (Score, DcId, Ts).
__device__ __forceinline__ bool gb_gt(int64_t s1, uint32_t d1, int64_t t1, int64_t s2, uint32_t d2,
                                      int64_t t2) {
  return s1 > s2 || (s1 == s2 && (d1 > d2 || (d1 == d2 && t1 > t2)));
}

template <int PCAP, bool RK>
__device__ __forceinline__ void s_emit(const TrmvApplyArgs& a, SLds<PCAP, RK>& L, uint64_t op0, uint64_t op,
                                       uint8_t kind, int64_t id, int64_t sc, uint32_t dc, int64_t ts,
                                       const Row8* vc) {
  const uint32_t pos = atomicAdd(&L.nex, 1u);
  TrmvExtraRec r;
  r.op = (uint32_t)op;
  r.kind = kind;
  r.dc = (uint8_t)dc;
  r.pad = 0;
  r.id = id;
  r.score = sc;
  r.ts = ts;
  KA->ex[op0 + pos] = r;
  if (vc)
    for (int d = 0; d < KA->n_dc; ++d) KA->ex_vc[(op0 + pos) * KA->n_dc + d] = pick8(*vc, (uint32_t)d);
}

// Player of each lane's Id (v lanes); new Ids are claimed and numbered
// np, np+1, ... in lane order.  Returns false if the key outgrows PCAP.
template <int PCAP, bool RK>
__device__ __forceinline__ bool s_resolve(SLds<PCAP, RK>& L, int64_t id, bool v, uint32_t& np, uint32_t& p) {
  constexpr int HS = SLds<PCAP, RK>::HS;
  const int lane = lane_id();
  L.u.k.claim[lane] = id;
  lsync(L);
  uint32_t h = shash<PCAP>(id);
  bool resolved = !v, claimed = false;
  int follow = -1;
  p = 0;
  constexpr uint32_t HNONE = HSlot<PCAP>::NONE, HCLAIM = HSlot<PCAP>::CLAIM;
  uint32_t rounds = 0;
  (void)rounds;
  while (ballot(!resolved)) {
    if constexpr (PCAP > 1024) {  // HBM class: fresh slot reads each round, and a bound
      lsync(L);
      if (++rounds > 4u * HS) return false;
    }
    if (!resolved) {
      const uint32_t s = L.hs[h];
      if (s == HNONE) {
        if (hs_cas(L, h, HNONE, HCLAIM | (uint32_t)lane) == HNONE) {
          claimed = true;
          resolved = true;
        }  // lost the race: read the slot again
      } else if (s & HCLAIM) {
        const int c = (int)(s & 63u);
        if (L.u.k.claim[c] == id) {
          follow = c;
          resolved = true;
        } else {
          h = (h + 1) & (HS - 1);
        }
      } else if (L.pid[s] == id) {
        p = s;
        resolved = true;
      } else {
        h = (h + 1) & (HS - 1);
      }
    }
  }
  lsync(L);
  const uint64_t cm = ballot(claimed);
  const uint32_t nn = np + (uint32_t)__builtin_popcountll(cm);
  if (nn > (uint32_t)PCAP) return false;
  if (claimed) {
    p = np + mbcnt(cm);
    L.pid[p] = id;
    L.hs[h] = (typename HSlot<PCAP>::T)p;
    L.oslab[p] = 0u;
    L.orow[p] = S_NONE;
    L.u.k.nops[p] = 0u;
    L.opd[p] = NONE16 << 16;
    L.gpd[p] = 0u;
    L.gsc[p] = L.gts[p] = 0;
    if constexpr (!RK) L.osc[p] = L.ots[p] = 0;
  }
  const uint32_t fp = shfl32(p, follow >= 0 ? follow : lane);
  if (follow >= 0) p = fp;
  np = nn;
  lsync(L);
  return true;
}

template <int PCAP, bool RK>
__device__ __forceinline__ uint32_t s_lookup(const SLds<PCAP, RK>& L, int64_t id, bool v) {
  constexpr int HS = SLds<PCAP, RK>::HS;
  uint32_t h = shash<PCAP>(id), p = (uint32_t)PCAP;
  if (v) {
    for (uint32_t probe = 0; probe < (uint32_t)HS; ++probe) {
      const uint32_t s = L.hs[h];
      if (s == HSlot<PCAP>::NONE) break;  // cannot happen: K2 resolved every Id
      if (L.pid[s] == id) {
        p = s;
        break;
      }
      h = (h + 1) & (HS - 1);
    }
  }
  return p;
}

struct SMin {
  uint32_t p;  // player of Min, S_NONE = {nil, nil, nil}
  int64_t sc, id, ts;
};

// min_observed/1 (:398-406): term-order smallest Observed value; Ids are
// distinct, so (Score, Id) decides.
template <int PCAP, bool RK>
__device__ __forceinline__ void s_min(const SLds<PCAP, RK>& L, uint32_t np, SMin& m) {
  const int lane = lane_id();
  uint32_t bp = S_NONE;
  int64_t bs = INT64_MAX, bi = INT64_MAX;
  for (uint32_t b = 0; b < np; b += 64) {
    const uint32_t p = b + lane;
    const uint32_t q = p < np ? p : (uint32_t)PCAP;
    const bool ok = p < np && (L.opd[q] & F_OBS);
    const int64_t sc = L.osc[q], id = L.pid[q];
    if (ok && (bp == S_NONE || sc < bs || (sc == bs && id < bi))) {
      bp = p;
      bs = sc;
      bi = id;
    }
  }
  const bool has = bp != S_NONE;
  if (!ballot(has)) {
    m.p = S_NONE;
    return;
  }
  const int64_t ms = wave_min_i64_dpp(has ? bs : INT64_MAX);
  const int64_t mi = wave_min_i64_dpp(has && bs == ms ? bi : INT64_MAX);
  const uint64_t hit = ballot(has && bs == ms && bi == mi);
  m.p = rl32(bp, (int)__builtin_ctzll(hit));
  m.sc = ms;
  m.id = mi;
  m.ts = ufl64(L.ots[m.p]);
}

// Promotion candidate of rmv/3 (:276-281, :291): the Id outside Observed
// whose largest Masked element is the term-order largest, i.e. the largest
// (max Score, Id); S_NONE if no Id outside Observed has Masked elements.
template <int PCAP, bool RK>
__device__ __forceinline__ uint32_t s_promote(const SLds<PCAP, RK>& L, uint32_t np) {
  const int lane = lane_id();
  uint32_t bp = S_NONE;
  int64_t bs = INT64_MIN, bi = INT64_MIN;
  // four slots of players per round, their loads issued together (one LDS
  // round trip per round instead of one per slot)
  for (uint32_t b0 = 0; b0 < np; b0 += 256) {
    uint32_t f[4];
    int64_t sc[4], id[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t p = b0 + 64 * u + lane;
      const uint32_t q = p < np ? p : (uint32_t)PCAP;
      f[u] = L.opd[q];
      sc[u] = L.gsc[q];
      id[u] = L.pid[q];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t p = b0 + 64 * u + lane;
      const bool ok = p < np && !(f[u] & F_OBS) && (f[u] & F_HASM);
      if (ok && (bp == S_NONE || sc[u] > bs || (sc[u] == bs && id[u] > bi))) {
        bp = p;
        bs = sc[u];
        bi = id[u];
      }
    }
  }
  const bool has = bp != S_NONE;
  if (!ballot(has)) return S_NONE;
  const int64_t ms = wave_max_i64_dpp(has ? bs : INT64_MIN);
  const int64_t mi = wave_max_i64_dpp(has && bs == ms ? bi : INT64_MIN);
  const uint64_t hit = ballot(has && bs == ms && bi == mi);
  return rl32(bp, (int)__builtin_ctzll(hit));
}

// Observed as a register table (K <= 128), kept sorted ascending by
// (Score, Id) -- min_observed/1's order (:398-406; Ids are distinct, so
// (Score, Id) decides): entry r in lane r % 64 of slot r / 64, entries >= n
// hold the sentinel (INT64_MAX, INT64_MAX, PCAP).  Min is entry 0.  Obs[Id]'s
// Ts / dc / slab position live in LDS (ots, opd), written on every change.
struct ObsTab {
  int64_t sc[2], id[2];  // Obs[Id] score, Id
  int64_t ts[2];         // Obs[Id] Ts
  uint32_t p[2];         // player
  uint32_t n;            // |Observed|
  uint32_t mi;           // entry of Min: 0, or S_NONE ({nil, nil, nil}) when empty
  int64_t msc, mid;      // Min's score and Id
};

__device__ __forceinline__ uint32_t ot_find(const ObsTab& o, uint32_t q) {
  const int lane = lane_id();
  const uint64_t m0 = ballot((uint32_t)lane < o.n && o.p[0] == q);
  const uint64_t m1 = ballot((uint32_t)(64 + lane) < o.n && o.p[1] == q);
  return m0 ? (uint32_t)__builtin_ctzll(m0) : (m1 ? 64u + (uint32_t)__builtin_ctzll(m1) : S_NONE);
}
__device__ __forceinline__ int64_t ot_get64(const int64_t f[2], uint32_t i) {
  const int64_t a = rl64(f[0], (int)(i & 63u)), b = rl64(f[1], (int)(i & 63u));
  return i < 64 ? a : b;
}
__device__ __forceinline__ uint32_t ot_get32(const uint32_t f[2], uint32_t i) {
  const uint32_t a = rl32(f[0], (int)(i & 63u)), b = rl32(f[1], (int)(i & 63u));
  return i < 64 ? a : b;
}
__device__ __forceinline__ bool key_lt(int64_t s1, int64_t i1, int64_t s2, int64_t i2) {
  return s1 < s2 || (s1 == s2 && i1 < i2);
}
__device__ __forceinline__ void ot_set_min(ObsTab& o) {
  o.mi = o.n ? 0u : S_NONE;
  o.msc = rl64(o.sc[0], 0);
  o.mid = rl64(o.id[0], 0);
}

// One merge step of Observed: drop the entries whose rank the `del` lanes
// hold in dr, add the `ins` lanes' (is, iid, ip) entries, and keep the K
// largest by (Score, Id).  For an add run this is exact: Observed at the end
// of a run of adds is the top K players by (max Score, Id) (invariant in the
// header), so the order of the run's adds across players does not matter;
// within a player the caller applies its adds one merge step each.  Players
// of evicted old entries lose F_OBS here; returns each `ins` lane's new rank,
// -1 if evicted (and -1 on the other lanes).
template <int PCAP, bool RK>
__device__ __forceinline__ int32_t ot_merge(ObsTab& o, SLds<PCAP, RK>& L, uint32_t K, bool del, uint32_t dr,
                                            bool ins, int64_t is, int64_t iid, int64_t its, uint32_t ip) {
  const int lane = lane_id();
  bool d0 = false, d1 = false;
  uint64_t dm = ballot(del);
  const uint32_t nd = (uint32_t)__builtin_popcountll(dm);
  while (dm) {
    const int x = (int)__builtin_ctzll(dm);
    dm &= dm - 1;
    const uint32_t r = rl32(dr, x);
    d0 |= r == (uint32_t)lane;
    d1 |= r == (uint32_t)(64 + lane);
  }
  const bool v0 = (uint32_t)lane < o.n && !d0, v1 = (uint32_t)(64 + lane) < o.n && !d1;
  uint64_t im = ballot(ins);
  const uint32_t ni = (uint32_t)__builtin_popcountll(im);
  uint32_t li0 = 0, li1 = 0, ri = 0, lo = 0;
  while (im) {
    const int x = (int)__builtin_ctzll(im);
    im &= im - 1;
    const int64_t xs = rl64(is, x), xi = rl64(iid, x);
    const bool lt0 = key_lt(xs, xi, o.sc[0], o.id[0]), lt1 = key_lt(xs, xi, o.sc[1], o.id[1]);
    li0 += lt0 ? 1u : 0u;
    li1 += lt1 ? 1u : 0u;
    ri += (ins && key_lt(xs, xi, is, iid)) ? 1u : 0u;
    // table entries below the insert: the kept entries have other Ids than
    // the inserted ones, so their keys differ and "below" is "not above"
    const uint32_t c = (uint32_t)__builtin_popcountll(ballot(v0 && !lt0)) +
                       (uint32_t)__builtin_popcountll(ballot(v1 && !lt1));
    lo = lane == x ? c : lo;
  }
  const uint64_t dm0 = ballot(d0), dm1 = ballot(d1);
  const uint32_t db0 = mbcnt(dm0), db1 = (uint32_t)__builtin_popcountll(dm0) + mbcnt(dm1);
  const uint32_t tot = o.n - nd + ni;
  const int32_t m = tot > K ? (int32_t)(tot - K) : 0;
  const int32_t pos0 = (int32_t)((uint32_t)lane - db0 + li0) - m;
  const int32_t pos1 = (int32_t)((uint32_t)(64 + lane) - db1 + li1) - m;
  const int32_t posi = (int32_t)(ri + lo) - m;
  if (v0 && pos0 >= 0) {
    L.tsc[pos0] = o.sc[0];
    L.tid[pos0] = o.id[0];
    L.tts[pos0] = o.ts[0];
    L.tp[pos0] = (uint16_t)o.p[0];
    L.ork[o.p[0]] = (uint8_t)pos0;
  }
  if (v1 && pos1 >= 0) {
    L.tsc[pos1] = o.sc[1];
    L.tid[pos1] = o.id[1];
    L.tts[pos1] = o.ts[1];
    L.tp[pos1] = (uint16_t)o.p[1];
    L.ork[o.p[1]] = (uint8_t)pos1;
  }
  if (ins && posi >= 0) {
    L.tsc[posi] = is;
    L.tid[posi] = iid;
    L.tts[posi] = its;
    L.tp[posi] = (uint16_t)ip;
    L.ork[ip] = (uint8_t)posi;
  }
  if (v0 && pos0 < 0) atomicAnd(&L.opd[o.p[0]], ~F_OBS);  // evicted (:325-331)
  if (v1 && pos1 < 0) atomicAnd(&L.opd[o.p[1]], ~F_OBS);
  lsync(L);
  o.n = tot - (uint32_t)m;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const uint32_t k = (uint32_t)(t * 64 + lane);
    const bool ok = k < o.n;
    const uint32_t kk = ok ? k : 0u;
    const int64_t sv = L.tsc[kk], iv = L.tid[kk], tv = L.tts[kk];
    const uint32_t pv = L.tp[kk];
    o.sc[t] = ok ? sv : INT64_MAX;
    o.id[t] = ok ? iv : INT64_MAX;
    o.ts[t] = ok ? tv : 0;
    o.p[t] = ok ? pv : (uint32_t)PCAP;
  }
  lsync(L);
  ot_set_min(o);
  return ins ? posi : -1;
}

// Deferred maintenance of each player's gb_sets:largest(Masked[Id]) (LDS
// gsc/gts/gpd): for the ops [lo, hi) of the chunk, the last op of each player
// in the range writes the running largest of the player's non-dominated adds
// since its last rmv (rok/rsc/rts/rd, computed in the sorted view; a rmv
// resets it, and the rmv itself sets the player's largest from its replay).
// One writer per player, so no two lanes race.  Called before a promotion
// reads the players' largest elements, and at the end of a chunk.
template <int PCAP, bool RK>
__device__ __forceinline__ void s_catch_up(SLds<PCAP, RK>& L, uint32_t lo, uint32_t hi, uint32_t kd, uint32_t nxt,
                                           bool rok, int64_t rsc, int64_t rts, uint32_t rd) {
  const uint32_t l = (uint32_t)lane_id();
  if (l >= lo && l < hi && nxt >= hi && rok) {
    const uint32_t p = kd >> 8, rdc = rd & 0xFFu;
    const uint32_t f = L.opd[p];
    const int64_t gs = L.gsc[p], gt = L.gts[p];
    const uint32_t gd = (L.gpd[p] >> 8) & 0xFFu;
    if (!(f & F_HASM) || gb_gt(rsc, rdc, rts, gs, gd, gt)) {
      L.gsc[p] = rsc;
      L.gts[p] = rts;
      L.gpd[p] = (rdc << 8) | ((rd >> 8) << 16);
      atomicOr(&L.opd[p], F_HASM);
    }
  }
  lsync(L);
}

// One key.  Writes nothing to the new side before its last early return
// that hands the key on (S_NEXT).
template <int PCAP, bool RANKED>
__device__ int trmv_steady_key(const TrmvApplyArgs& a, uint32_t key, SLds<PCAP, RANKED>& L) {
  constexpr int HS = SLds<PCAP, RANKED>::HS;
  const int lane = lane_id();
  const int D = KA->n_dc;
#ifdef TRMV_PROF
  unsigned long long prof_t;
  SPROF_STAMP(prof_t);
#endif
  const uint64_t op0 = KA->key_ptr[key];
  // (a key whose ops an earlier pass applied is only rewritten: no ops)
  const bool done = KA->key_done && KA->key_done[key];
  const uint32_t nops = done ? 0u : (uint32_t)(KA->key_ptr[key + 1] - op0);
  const KeyMeta nm = trmv_new_meta(a, key);
  KeyMeta om;
  if (KA->fresh) {
    om.p_off = om.m_off = om.r_off = 0;
    om.np = om.nm = om.nr = om.nobs = 0;
    om.minq = NONE32;
  } else {
    om = KA->old_s.meta[key];
  }
  if (om.np > (uint32_t)PCAP) return S_NEXT;

  for (int i = lane; i < HS; i += 64) L.hs[i] = (typename HSlot<PCAP>::T)HSlot<PCAP>::NONE;
  if (lane <= TRMV_DPAD)
    L.vc[lane] = (!KA->fresh && lane < D) ? (unsigned long long)KA->old_s.vc[(uint64_t)key * D + lane] : 0ull;
  if (lane == 0) {
    L.nex = 0u;
    L.nob = 0u;
  }
  // sinks (PCAP) read by lanes without a player
  if (lane == 0) {
    L.opd[PCAP] = 0u;
    L.gsc[PCAP] = L.pid[PCAP] = 0;
    if constexpr (RANKED) L.ork[PCAP] = 0u;
    else L.osc[PCAP] = L.ots[PCAP] = 0;
  }
  lsync(L);

  // ---- K1. old players: four slots per round, each round's HBM loads
  // issued together (records, then the Obs[Id] / largest elements they name)
  uint32_t span = 0;
  for (uint32_t b0 = 0; b0 < om.np; b0 += 256) {
    int64_t id[4];
    uint32_t info[4], slab[4], gb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t p = b0 + 64 * u + lane;
      const uint64_t pp = (uint64_t)om.p_off + (p < om.np ? p : 0u);
      const bool v = p < om.np;
      id[u] = v ? KA->old_s.pl_id[pp] : 0;
      info[u] = v ? KA->old_s.pl_info[pp] : NONE32;
      slab[u] = v ? KA->old_s.pl_slab[pp] : 0u;
      gb[u] = (v && (slab[u] >> 16) > 1) ? (uint32_t)KA->old_s.pl_gb[pp] : 0u;
    }
    int64_t os[4], ot[4], gs[4], gt[4];
    uint32_t od[4], gd[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t off = slab[u] & 0xFFFFu, cnt = slab[u] >> 16, obx = info[u] & 0xFFFFu;
      const uint64_t g0 = (uint64_t)om.m_off + off;
      const bool ho = obx != NONE16, hg = cnt != 0;
      os[u] = ho ? KA->old_s.m_score[g0 + obx] : 0;
      ot[u] = ho ? KA->old_s.m_ts[g0 + obx] : 0;
      od[u] = ho ? (uint32_t)KA->old_s.m_dc[g0 + obx] : 0u;
      gs[u] = hg ? KA->old_s.m_score[g0 + gb[u]] : 0;
      gt[u] = hg ? KA->old_s.m_ts[g0 + gb[u]] : 0;
      gd[u] = hg ? (uint32_t)KA->old_s.m_dc[g0 + gb[u]] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t p = b0 + 64 * u + lane;
      if (p < om.np) {
        const uint32_t off = slab[u] & 0xFFFFu, cnt = slab[u] >> 16, obx = info[u] & 0xFFFFu;
        L.pid[p] = id[u];
        L.oslab[p] = slab[u];
        L.orow[p] = info[u];
        L.u.k.nops[p] = 0u;
        if constexpr (RANKED) {  // Observed's entries, gathered for the build
          if (obx != NONE16) {
            const uint32_t k = atomicAdd(&L.nob, 1u);
            L.tsc[k] = os[u];
            L.tid[k] = id[u];
            L.tts[k] = ot[u];
            L.tp[k] = (uint16_t)p;
          }
        } else {
          L.osc[p] = os[u];
          L.ots[p] = ot[u];
        }
        L.gsc[p] = gs[u];
        L.gts[p] = gt[u];
        L.opd[p] = (obx != NONE16 ? F_OBS : 0u) | (cnt ? F_HASM : 0u) |
                   ((info[u] >> 16) != NONE16 ? F_ROWV : 0u) | (od[u] << 8) | (obx << 16);
        L.gpd[p] = (gd[u] << 8) | (gb[u] << 16);
        span = off + cnt > span ? off + cnt : span;
        uint32_t h = shash<PCAP>(id[u]);
        while (hs_cas(L, h, HSlot<PCAP>::NONE, p) != HSlot<PCAP>::NONE) h = (h + 1) & (HS - 1);
      }
    }
  }
  span = wave_max_u32_dpp(span);
  lsync(L);
  SPROF(0);

  // ---- K2. the player of every op, ops per player, players with a rmv
  uint32_t np = om.np;
  for (uint32_t c0 = 0; c0 < nops; c0 += 64) {
    const uint32_t l = c0 + lane;
    const bool v = l < nops;
    const int64_t id = v ? KA->id[op0 + l] : 0;
    const uint32_t kind = v ? (uint32_t)KA->kind[op0 + l] : 0u;
    uint32_t p;
    if (!s_resolve<PCAP, RANKED>(L, id, v, np, p)) return S_NEXT;
    if (v) {
      atomicAdd(&L.u.k.nops[p], 1u);
      if (kind == 2 || kind == 3) atomicOr(&L.opd[p], F_RMV);
    }
  }
  lsync(L);
  // new Removals rows, new slab offsets (old count + ops: the new segment)
  uint32_t nr = om.nr, mtot = 0;
  for (uint32_t b = 0; b < np; b += 64) {
    const uint32_t p = b + lane;
    const bool act = p < np;
    const uint32_t q = act ? p : (uint32_t)PCAP;
    const uint32_t info = L.orow[q], f = L.opd[q];
    const bool newrow = act && (f & F_RMV) && (info >> 16) == NONE16;
    const uint64_t m = ballot(newrow);
    if (newrow) L.orow[p] = (info & 0xFFFFu) | ((nr + mbcnt(m)) << 16);
    nr += (uint32_t)__builtin_popcountll(m);
    const uint32_t ocnt = act ? (L.oslab[q] >> 16) : 0u;
    const uint32_t cap = act ? ocnt + L.u.k.nops[q] : 0u;
    uint32_t tot;
    const uint32_t ex = wave_excl_scan_dpp(cap, tot);
    if (act) L.nslab[p] = (mtot + ex) | (ocnt << 16);
    mtot += tot;
  }
  if (nr >= NONE16 || mtot > TRMV_SEG_MAX) return S_NEXT;  // over the per-key capacity
  lsync(L);
  SPROF(1);

  // ---- K3. old slabs (except replayed players') and old Removals rows
  if (PCAP > 1024 && !KA->fresh && span && om.np > 64) {
    // The HBM class with many players: one lane per old player copies its
    // slab (O(np + span); the position windows below would sweep every
    // player for every 64 positions)
    for (uint32_t j0 = 0; j0 < om.np; j0 += 64) {
      const uint32_t j = j0 + lane;
      const bool act = j < om.np;
      const uint32_t sl = act ? L.oslab[j] : 0u;
      const uint32_t cnt = (act && !(L.opd[j] & F_RMV)) ? (sl >> 16) : 0u;
      const uint64_t src = (uint64_t)om.m_off + (sl & 0xFFFFu);
      const uint64_t dst = (uint64_t)nm.m_off + (act ? (L.nslab[j] & 0xFFFFu) : 0u);
      for (uint32_t e = 0; e < cnt; ++e) {
        KA->new_s.m_score[dst + e] = KA->old_s.m_score[src + e];
        KA->new_s.m_ts[dst + e] = KA->old_s.m_ts[src + e];
        KA->new_s.m_dc[dst + e] = KA->old_s.m_dc[src + e];
      }
    }
  } else if (!KA->fresh && span) {
    int32_t prev = -1;  // owner of the position before the window
    // the next window's elements load while this one is placed
    int64_t nsc = 0, nts = 0;
    uint32_t ndc = 0;
    if ((uint32_t)lane < span) {
      nsc = KA->old_s.m_score[(uint64_t)om.m_off + lane];
      nts = KA->old_s.m_ts[(uint64_t)om.m_off + lane];
      ndc = KA->old_s.m_dc[(uint64_t)om.m_off + lane];
    }
    for (uint32_t q0 = 0; q0 < span; q0 += 64) {
      const uint32_t q = q0 + lane;
      const int64_t sc = nsc, ts = nts;
      const uint32_t dc = ndc;
      if (q + 64 < span) {
        const uint64_t src = (uint64_t)om.m_off + q + 64;
        nsc = KA->old_s.m_score[src];
        nts = KA->old_s.m_ts[src];
        ndc = KA->old_s.m_dc[src];
      }
      // The owner of a position is the player whose slab starts last at or
      // before it.  Slabs are not in player order (tier R writes players in
      // Observed order), so every player marks its slab start if it falls in
      // the window; (position, player) pairs, max-scanned by position.
      L.u.c.mark[lane] = 0u;
      lsync(L);
      for (uint32_t j0 = 0; j0 < om.np; j0 += 64) {
        const uint32_t j = j0 + lane;
        const uint32_t sl = j < om.np ? L.oslab[j] : 0u;
        const uint32_t off = sl & 0xFFFFu;
        if ((sl >> 16) && off >= q0 && off < q0 + 64) L.u.c.mark[off - q0] = j + 1;
      }
      lsync(L);
      const uint32_t mk = L.u.c.mark[lane];
      const uint32_t own = wave_incl_max_dpp(mk ? (((uint32_t)lane + 1) << 16) | mk : 0u) & 0xFFFFu;
      const int32_t o = own ? (int32_t)own - 1 : prev;
      prev = (int32_t)rl32((uint32_t)o, 63);
      if (q < span && o >= 0) {
        const uint32_t sl = L.oslab[o];
        const uint32_t off = sl & 0xFFFFu, cnt = sl >> 16;
        if (q < off + cnt && !(L.opd[o] & F_RMV)) {
          const uint64_t dst = (uint64_t)nm.m_off + (L.nslab[o] & 0xFFFFu) + (q - off);
          KA->new_s.m_score[dst] = sc;
          KA->new_s.m_ts[dst] = ts;
          KA->new_s.m_dc[dst] = (uint8_t)dc;
        }
      }
      lsync(L);
    }
  }
  for (uint32_t r0 = 0; r0 < om.nr; r0 += 8) {
    const uint32_t r = r0 + (lane >> 3), d = lane & 7;
    if (r < om.nr && (int)d < D)
      KA->new_s.r_vc[((uint64_t)nm.r_off + r) * D + d] = KA->old_s.r_vc[((uint64_t)om.r_off + r) * D + d];
  }
  // the replays read rows written here: retire the stores first
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  SPROF(2);

  // ---- K4. chunks of the key's ops
  const uint32_t K = KA->k;
  SMin mn;  // !RANKED: Min and |Observed|
  uint32_t nobs = om.nobs;
  ObsTab ob;  // RANKED: Observed in registers
  if (!RANKED) {
    mn.p = om.minq;
    mn.sc = mn.id = mn.ts = 0;
    if (mn.p != NONE32) {
      mn.sc = ufl64(L.osc[mn.p]);
      mn.id = ufl64(L.pid[mn.p]);
      mn.ts = ufl64(L.ots[mn.p]);
    }
  } else {
    // the old Observed (gathered by K1) -> sorted by (Score, Id): each
    // entry's rank is the number of entries below it (broadcast LDS reads,
    // independent across j)
    const uint32_t c = ufl(L.nob);
    int64_t es[2], ei[2], et[2];
    uint32_t ep[2], rk[2] = {0u, 0u};
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint32_t k = (uint32_t)(t * 64 + lane);
      const uint32_t kk = k < c ? k : 0u;
      es[t] = L.tsc[kk];
      ei[t] = L.tid[kk];
      et[t] = L.tts[kk];
      ep[t] = L.tp[kk];
    }
    for (uint32_t j = 0; j < c; ++j) {
      const int64_t js = L.tsc[j], ji = L.tid[j];
      rk[0] += key_lt(js, ji, es[0], ei[0]) ? 1u : 0u;
      rk[1] += key_lt(js, ji, es[1], ei[1]) ? 1u : 0u;
    }
    lsync(L);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if ((uint32_t)(t * 64 + lane) < c) {
        L.tsc[rk[t]] = es[t];
        L.tid[rk[t]] = ei[t];
        L.tts[rk[t]] = et[t];
        L.tp[rk[t]] = (uint16_t)ep[t];
        L.ork[ep[t]] = (uint8_t)rk[t];
      }
    }
    lsync(L);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint32_t k = (uint32_t)(t * 64 + lane);
      const bool ok = k < c;
      const uint32_t kk = ok ? k : 0u;
      ob.sc[t] = ok ? L.tsc[kk] : INT64_MAX;
      ob.id[t] = ok ? L.tid[kk] : INT64_MAX;
      ob.ts[t] = ok ? L.tts[kk] : 0;
      ob.p[t] = ok ? (uint32_t)L.tp[kk] : (uint32_t)PCAP;
    }
    ob.n = c;
    ot_set_min(ob);
    lsync(L);
  }
  for (uint32_t c0 = 0; c0 < nops;) {
    uint32_t n = nops - c0 < (uint32_t)S_CH ? nops - c0 : (uint32_t)S_CH;
    bool v = (uint32_t)lane < n;
    const uint64_t gi = op0 + c0 + lane;
    const uint32_t kind = v ? (uint32_t)KA->kind[gi] : 0u;
    const int64_t id = v ? KA->id[gi] : 0;
    const int64_t sc = v ? KA->score[gi] : 0;
    const int64_t ts = v ? KA->ts[gi] : 0;
    const uint32_t dc = v ? (uint32_t)KA->dc[gi] : 0u;
    bool isr = v && (kind == 2 || kind == 3);
    uint64_t rm = ballot(isr);
    if (__builtin_popcountll(rm) > S_CHR) {  // cut before the chunk's 17th rmv
      uint64_t m = rm;
      for (int k = 0; k < S_CHR; ++k) m &= m - 1;
      n = (uint32_t)__builtin_ctzll(m);
      v = (uint32_t)lane < n;
      isr = isr && v;
      rm = ballot(isr);
    }
    const bool add = v && kind < 2;
    uint32_t err = 0;
    err |= (v && kind > 3) ? TRMV_ERR_KIND : 0u;
    err |= (add && (int)dc >= D) ? TRMV_ERR_DC : 0u;
    err |= (add && ts < 1) ? TRMV_ERR_TS : 0u;
    err |= (isr && (ts < 0 || ts >= KA->n_rmv_rows)) ? TRMV_ERR_ROW : 0u;
    if (ballot(err != 0)) {
      if (err) atomicOr(&KA->status[1], err);
      return S_REJECT;
    }
    const uint32_t p = s_lookup<PCAP, RANKED>(L, id, v);
    // the rmvs' clocks (8 lanes per row)
    const uint32_t rk = mbcnt(rm), nrm = (uint32_t)__builtin_popcountll(rm);
    if (isr) L.u.c.crow[rk] = (uint32_t)ts;
    lsync(L);
    for (uint32_t r0 = 0; r0 < nrm; r0 += 8) {
      const uint32_t r = r0 + (lane >> 3), d = lane & 7;
      if (r < nrm) {
        const int64_t x = (int)d < D ? KA->rmv_vc[(uint64_t)L.u.c.crow[r] * D + d] : 0;
        err |= x < 0 ? TRMV_ERR_VC : 0u;
        L.u.c.vtab[r][d] = x;
      }
    }
    if (ballot(err != 0)) {
      if (err) atomicOr(&KA->status[1], err);
      return S_REJECT;
    }
    SPROF(3);
    // Elements that may already be in Masked[Id] (gb_sets:add_element, :240-246):
    // every element of dc in the key has Ts <= Vc[dc], so an add whose Ts is
    // above the key's Vc[dc] before it is new.  Exact when the chunk's adds of
    // each dc have rising Ts (then the previous one holds the maximum);
    // otherwise every add of that dc after the first fall is a candidate.
    bool dupc;
    {
      const int64_t vcs = (int64_t)L.vc[add ? dc : (uint32_t)TRMV_DPAD];
      const uint32_t kv = wave_radix_sort<4>(((add ? dc : 8u) << 6) | (uint32_t)lane);
      const uint32_t src = kv & 63u, sdc = kv >> 6;
      const int64_t sts = shfl64(ts, (int)src);
      const uint32_t lkv = shfl32(kv, lane ? lane - 1 : 0);
      const int64_t lts = shfl64(sts, lane ? lane - 1 : 0);
      const bool fall = lane > 0 && sdc < 8u && (lkv >> 6) == sdc && lts >= sts;
      const uint64_t fm = ballot(fall);
      // a fall taints the rest of its dc run (sorted lanes, stream order inside)
      bool taint = false;
      if (fm) {
        const uint64_t below = lane == 63 ? ~0ull : ((2ull << lane) - 1);
        const uint64_t f = fm & below;
        const uint32_t hi = f ? 63u - (uint32_t)__builtin_clzll(f) : (uint32_t)lane;
        const uint32_t fkv = shfl32(kv, (int)hi);
        taint = f != 0 && (fkv >> 6) == sdc;
      }
      const bool taint_src = perm32(taint ? 1u : 0u, src) != 0;  // back to stream lanes
      dupc = add && (ts <= vcs || taint_src);
    }
    lsync(L);
    if (add) atomicMax(&L.vc[dc], (unsigned long long)ts);  // vc_update (:233)
    L.u.c.csc[lane] = sc;
    L.u.c.cts[lane] = ts;
    L.u.c.ckd[lane] = v ? (kind | (dc << 2) | ((dupc ? 1u : 0u) << 5) | (p << 8)) : ((uint32_t)PCAP << 8);
    L.u.c.cres[lane] = isr ? rk : 0u;
    lsync(L);

    SPROF(4);
    // ---- ops in (player, stream) order
    const uint32_t kvs = wave_radix_sort<Log2<PCAP>::v + 1>(((v ? p : (uint32_t)PCAP) << 6) | (uint32_t)lane);
    const uint32_t sp = kvs >> 6, so = kvs & 63u;
    const bool sv = sp < (uint32_t)PCAP;
    const uint32_t lkvs = shfl32(kvs, lane ? lane - 1 : 0);
    const bool start = sv && (lane == 0 || (lkvs >> 6) != sp);
    L.u.c.csrt[lane] = (uint8_t)so;
    const uint64_t ss = ballot(start);
    const uint64_t incl = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const uint64_t sb = ss & incl;
    const uint32_t slo = sb ? 63u - (uint32_t)__builtin_clzll(sb) : 0u;
    const uint64_t above = ss & ~incl;
    const uint32_t shi = above ? (uint32_t)__builtin_ctzll(above) : n;
    const uint64_t segm = (shi >= 64 ? ~0ull : ((1ull << shi) - 1)) & ~((1ull << slo) - 1);
    const uint32_t skd = L.u.c.ckd[so];
    const int64_t ssc = L.u.c.csc[so], sts = L.u.c.cts[so];
    const uint32_t sdc = (skd >> 2) & 7u;
    const uint32_t pf = L.opd[sv ? sp : (uint32_t)PCAP];
    const uint64_t dm = ballot(sv && ((skd >> 5) & 1u));
    const bool walk = sv && ((pf & F_RMV) || (dm & segm));
    // players without a rmv: append their non-dominated adds (op-parallel);
    // their Removals row is the old one for the whole batch
    bool dom = false;
    uint32_t orw = NONE16;
    if (sv && !walk && (pf & F_ROWV)) {
      orw = L.orow[sp] >> 16;
      dom = KA->old_s.r_vc[((uint64_t)om.r_off + orw) * D + sdc] >= sts;
    }
    const bool app = sv && !walk && !dom;
    const uint64_t nd = ballot(app);
    if (app) {
      const uint32_t ns = L.nslab[sp];
      const uint32_t pos = (ns >> 16) + (uint32_t)__builtin_popcountll(nd & segm & ((1ull << lane) - 1));
      const uint64_t dst = (uint64_t)nm.m_off + (ns & 0xFFFFu) + pos;
      KA->new_s.m_score[dst] = ssc;
      KA->new_s.m_ts[dst] = sts;
      KA->new_s.m_dc[dst] = (uint8_t)sdc;
      L.u.c.cres[so] = pos << 16;
    }
    if (dom) {  // {rmv, {Id, Removals[Id]}} (:236-237)
      Row8 rv = (Row8)(0);
      for (int d = 0; d < D; ++d) rv[d] = KA->old_s.r_vc[((uint64_t)om.r_off + orw) * D + d];
      L.u.c.cres[so] = R_DOM;
      s_emit<PCAP, RANKED>(a, L, op0, op0 + c0 + so, CCRDT_TRMV_RMV, L.pid[sp], 0, 0, 0, &rv);
    }
    lsync(L);
    if (sv && !walk && lane + 1 == (int)shi) {
      const uint32_t ns = L.nslab[sp];
      L.nslab[sp] = ns + ((uint32_t)__builtin_popcountll(nd & segm) << 16);
    }
    SPROF(5);
    // players with a rmv, or a possibly duplicated element: one lane each
    const uint64_t wm = ballot(start && walk);
    if (start && walk) {
      const uint32_t k = mbcnt(wm);
      L.u.c.cwp[k] = (uint16_t)sp;
      L.u.c.cws[k] = (uint8_t)lane;
      L.u.c.cwe[k] = (uint8_t)shi;
    }
    lsync(L);
    if ((uint32_t)lane < (uint32_t)__builtin_popcountll(wm)) {
      const uint32_t wp = L.u.c.cwp[lane], ws = L.u.c.cws[lane], we = L.u.c.cwe[lane];
      uint32_t f = L.opd[wp];
      const uint32_t ns = L.nslab[wp];
      const uint64_t base = (uint64_t)nm.m_off + (ns & 0xFFFFu);
      uint32_t cnt = ns >> 16;
      const uint32_t row = L.orow[wp] >> 16;
      if ((f & F_RMV) && !(f & F_MAT)) {  // its old slab, copied by itself
        const uint32_t os = L.oslab[wp];
        const uint64_t g0 = (uint64_t)om.m_off + (os & 0xFFFFu);
        for (uint32_t j = 0; j < (os >> 16); ++j) {
          KA->new_s.m_score[base + j] = KA->old_s.m_score[g0 + j];
          KA->new_s.m_ts[base + j] = KA->old_s.m_ts[g0 + j];
          KA->new_s.m_dc[base + j] = KA->old_s.m_dc[g0 + j];
        }
        f |= F_MAT;
      }
      bool has_row = (f & F_ROWV) != 0;
      Row8 R = (Row8)(0);
      const uint64_t rbase = ((uint64_t)nm.r_off + row) * D;
      if (has_row)
        for (int d = 0; d < D; ++d) R[d] = KA->new_s.r_vc[rbase + d];
      const int64_t wid = L.pid[wp];
      bool moved = false;
      for (uint32_t x = ws; x < we; ++x) {
        const uint32_t o = L.u.c.csrt[x];
        const uint32_t kd = L.u.c.ckd[o];
        const int64_t esc = L.u.c.csc[o], ets = L.u.c.cts[o];
        const uint32_t edc = (kd >> 2) & 7u;
        if ((kd & 3u) < 2) {  // add/4
          if (has_row && pick8(R, edc) >= ets) {  // dominated (:234-237)
            L.u.c.cres[o] = R_DOM;
            s_emit<PCAP, RANKED>(a, L, op0, op0 + c0 + o, CCRDT_TRMV_RMV, wid, 0, 0, 0, &R);
            continue;
          }
          uint32_t pos = S_NONE;
          if ((kd >> 5) & 1u)  // set semantics: the element may be there
            for (uint32_t j = 0; j < cnt; ++j)
              if (KA->new_s.m_ts[base + j] == ets && KA->new_s.m_dc[base + j] == edc &&
                  KA->new_s.m_score[base + j] == esc) {
                pos = j;
                break;
              }
          if (pos == S_NONE) {
            pos = cnt++;
            KA->new_s.m_score[base + pos] = esc;
            KA->new_s.m_ts[base + pos] = ets;
            KA->new_s.m_dc[base + pos] = (uint8_t)edc;
          }
          L.u.c.cres[o] = pos << 16;
        } else {  // rmv/3: merge_vc (:254, :369-386), filter Masked[Id] (:255-266)
          const uint32_t r = L.u.c.cres[o];
          Row8 V;
#pragma unroll
          for (int d = 0; d < TRMV_DPAD; ++d) V[d] = L.u.c.vtab[r][d];
#pragma unroll
          for (int d = 0; d < TRMV_DPAD; ++d) R[d] = has_row ? (V[d] > R[d] ? V[d] : R[d]) : V[d];
          has_row = true;
          uint32_t w = 0, bpos = 0, bdc = 0;
          int64_t bsc = 0, bts = 0;
          for (uint32_t j = 0; j < cnt; ++j) {
            const int64_t s2 = KA->new_s.m_score[base + j], t2 = KA->new_s.m_ts[base + j];
            const uint32_t d2 = KA->new_s.m_dc[base + j];
            if (t2 > pick8(V, d2)) {
              if (w != j) {
                KA->new_s.m_score[base + w] = s2;
                KA->new_s.m_ts[base + w] = t2;
                KA->new_s.m_dc[base + w] = (uint8_t)d2;
              }
              if (w == 0 || gb_gt(s2, d2, t2, bsc, bdc, bts)) {
                bsc = s2;
                bdc = d2;
                bts = t2;
                bpos = w;
              }
              ++w;
            }
          }
          moved |= w != cnt;
          cnt = w;
          L.u.c.rgsc[r] = bsc;
          L.u.c.rgts[r] = bts;
          L.u.c.rgd[r] = (w ? 1u : 0u) | (bdc << 8) | (bpos << 16);
        }
      }
      L.nslab[wp] = (ns & 0xFFFFu) | (cnt << 16);
      if (has_row) {
        for (int d = 0; d < D; ++d) KA->new_s.r_vc[rbase + d] = pick8(R, (uint32_t)d);
        f |= F_ROWV;
      }
      if (moved) f |= F_WALK;
      L.opd[wp] = f;
    }
    lsync(L);
    // the next chunk's replays read this chunk's stores
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    SPROF(6);

    // ---- the running largest element of each player's adds since its last
    // rmv (sorted view, segmented max-scan), for the deferred catch-up
    bool rok;
    int64_t rsc, rts;
    uint32_t rd, nxt;
    {
      const uint32_t scres = L.u.c.cres[so];
      const bool srmv = sv && (skd & 3u) >= 2;
      bool ok = sv && !srmv && !(scres & R_DOM);
      int64_t vs = ssc, vt = sts;
      uint32_t vd = sdc | ((scres >> 16) << 8);
      bool hf = start || srmv;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int src = lane >= d ? lane - d : lane;
        const bool yok = shfl32(ok ? 1u : 0u, src) != 0;
        const int64_t ys = shfl64(vs, src), yt = shfl64(vt, src);
        const uint32_t yd = shfl32(vd, src);
        const bool yhf = shfl32(hf ? 1u : 0u, src) != 0;
        if (lane >= d && !hf) {
          if (yok && (!ok || gb_gt(ys, yd & 0xFFu, yt, vs, vd & 0xFFu, vt))) {
            vs = ys;
            vt = yt;
            vd = yd;
            ok = true;
          }
          hf = yhf;
        }
      }
      // stream index of the player's next op in the chunk (0xFF: none)
      const uint32_t nso = shfl32(so, lane < 63 ? lane + 1 : lane);
      const uint64_t nb = lane < 63 ? (1ull << (lane + 1)) : 0ull;
      const bool has_next = lane < 63 && (uint32_t)(lane + 1) < n && !(ss & nb);
      const uint32_t nx = has_next ? nso : 0xFFu;
      // back to stream order (so is a permutation of the lanes)
      rok = perm32(ok ? 1u : 0u, so) != 0;
      rsc = (int64_t)(((uint64_t)perm32((uint32_t)((uint64_t)vs >> 32), so) << 32) | perm32((uint32_t)vs, so));
      rts = (int64_t)(((uint64_t)perm32((uint32_t)((uint64_t)vt >> 32), so) << 32) | perm32((uint32_t)vt, so));
      rd = perm32(vd, so);
      nxt = perm32(nx, so);
    }

    // ---- the Observed half, in stream order (recompute_observed/5 :301-334;
    // rmv/3 :267-298).  Per run of adds between two rmvs, a lane-parallel
    // filter drops the adds that cannot change Observed given the state at
    // the run's start (inside a run Min and every Obs[Id] only rise, so an add
    // below them stays below them); the others run one by one.
    const uint32_t kdr = L.u.c.ckd[lane], crr = L.u.c.cres[lane];
    const int64_t scr = L.u.c.csc[lane], tsr = L.u.c.cts[lane];
    const uint32_t rl = (uint32_t)lane < (uint32_t)S_CHR ? (uint32_t)lane : 0u;
    const int64_t rgs = L.u.c.rgsc[rl], rgt = L.u.c.rgts[rl];
    const uint32_t rgdv = L.u.c.rgd[rl];
    const int64_t vt0 = L.u.c.vtab[lane >> 3][lane & 7], vt1 = L.u.c.vtab[8 + (lane >> 3)][lane & 7];
    const bool ladd = (uint32_t)lane < n && (kdr & 3u) < 2 && !(crr & R_DOM);
    uint32_t last = 0;
    for (uint32_t j = 0; j < n;) {
      const uint64_t nr = j < 64 ? rm & (~0ull << j) : 0ull;
      const uint32_t hi = nr ? (uint32_t)__builtin_ctzll(nr) : n;
      if (hi > j) {
        const bool inr = ladd && (uint32_t)lane >= j && (uint32_t)lane < hi;
        bool rel = inr;
        if (RANKED) {
          lsync(L);
          const uint32_t pq = inr ? (kdr >> 8) : (uint32_t)PCAP;
          const uint32_t f = L.opd[pq];
          const uint32_t rq = L.ork[pq];  // meaningful with F_OBS
          const int64_t os = L.tsc[rq], ot = L.tts[rq];
          rel = inr && ((f & F_OBS) ? (scr > os || (scr == os && tsr > ot))
                                    : (ob.n < K || scr > ob.msc || (scr == ob.msc && id > ob.mid)));
        }
        uint64_t relm = ballot(rel);
        SPROF(13);
        if (RANKED) {
          // The run's relevant adds in merge steps: step g takes the g-th
          // add of each player (so a player's adds keep their stream order);
          // usually one step per run.
          const uint32_t q = kdr >> 8;
          while (relm) {
            bool later = false;  // an earlier remaining add of the same player
            for (uint64_t t = relm; t; t &= t - 1) {
              const int x = (int)__builtin_ctzll(t);
              later |= lane > x && q == (rl32(kdr, x) >> 8);
            }
            const bool mine = ((relm >> lane) & 1ull) && !later;
            relm &= ~ballot(mine);
            lsync(L);
            const uint32_t qq = mine ? q : (uint32_t)PCAP;
            const uint32_t f = L.opd[qq];
            const uint32_t rq = L.ork[qq];  // meaningful with F_OBS
            const int64_t os = L.tsc[rq], ot = L.tts[rq];
            // Id in Observed: a better element replaces Obs[Id] (:303-315);
            // else it competes for a place (:317-331)
            const bool up = mine && (f & F_OBS) && (scr > os || (scr == os && tsr > ot));
            const bool en = mine && !(f & F_OBS);
            const uint32_t dr = rq;  // an Observed player's rank (ork)
            SPROF(14);
            const int32_t pos = ot_merge<PCAP, RANKED>(ob, L, K, up, dr, up || en, scr, id, tsr, q);
            SPROF(15);
            const uint32_t obits = (((kdr >> 2) & 7u) << 8) | ((crr >> 16) << 16);
            if ((up || en) && pos >= 0) {
              L.opd[q] = (f & 0xFFu) | F_OBS | obits;
            } else if (up) {
              atomicAnd(&L.opd[q], ~F_OBS);
            }
            lsync(L);
          }
        }
        while (!RANKED && relm) {
          const uint32_t x = (uint32_t)__builtin_ctzll(relm);
          relm &= relm - 1;
          const uint32_t kd = rl32(kdr, (int)x), cr = rl32(crr, (int)x);
          const uint32_t q = kd >> 8;
          const int64_t s = rl64(scr, (int)x), t = rl64(tsr, (int)x), qid = rl64(id, (int)x);
          const uint32_t edc = (kd >> 2) & 7u, pos = cr >> 16;
          const uint32_t obits = (edc << 8) | (pos << 16);
          {
            uint32_t f = ufl(L.opd[q]);
            const uint32_t fobs = (f & 0xFFu) | F_OBS | obits;
            bool need_min = false;
            if (f & F_OBS) {  // Id in Observed (:303-315)
              const int64_t os = ufl64(L.osc[q]), ot = ufl64(L.ots[q]);
              if (s > os || (s == os && t > ot)) {
                if (lane == 0) {
                  L.osc[q] = s;
                  L.ots[q] = t;
                }
                f = fobs;
                need_min = q == mn.p;  // Old =:= Min
              }
            } else if (nobs < K) {  // (:317-324)
              if (lane == 0) {
                L.osc[q] = s;
                L.ots[q] = t;
              }
              f = fobs;
              ++nobs;
              if (mn.p == S_NONE || mn.sc > s || (mn.sc == s && (mn.id > qid || (mn.id == qid && mn.ts > t)))) {
                mn.p = q;
                mn.sc = s;
                mn.id = qid;
                mn.ts = t;
              }
            } else {  // full: evict Min if cmp(Elem, Min) (:325-331)
              if (s > mn.sc || (s == mn.sc && (qid > mn.id || (qid == mn.id && t > mn.ts)))) {
                if (lane == 0) {
                  atomicAnd(&L.opd[mn.p], ~F_OBS);
                  L.osc[q] = s;
                  L.ots[q] = t;
                }
                f = fobs;
                need_min = true;
              }
            }
            if (lane == 0) L.opd[q] = (L.opd[q] & F_HASM) | (f & ~F_HASM);
            lsync(L);
            if (need_min) s_min<PCAP, RANKED>(L, np, mn);
          }
        }
      }
      SPROF(9);
      if (hi >= n) break;
      // ---- the rmv at hi
      const uint32_t jr = hi;
      j = hi + 1;
      const uint32_t kd = rl32(kdr, (int)jr), r = rl32(crr, (int)jr);
      const uint32_t q = kd >> 8;
      const uint32_t g = rl32(rgdv, (int)r);
      const int64_t gsv = rl64(rgs, (int)r), gtv = rl64(rgt, (int)r);
      if (lane == 0) {  // Masked[Id] after the filter (:255-266): its largest
        if (g & 1u) {
          L.gsc[q] = gsv;
          L.gts[q] = gtv;
          L.gpd[q] = g & 0xFFFFFF00u;
          atomicOr(&L.opd[q], F_HASM);
        } else {
          atomicAnd(&L.opd[q], ~F_HASM);
        }
      }
      lsync(L);
      SPROF(10);
      // impacts Observed?  VcRmv[ObsDc] >= Obs[Id].Ts (:267-272)
      uint32_t ix = S_NONE;
      {
        const uint32_t f = ufl(L.opd[q]);
        if (RANKED) ix = ot_find(ob, q);
        else ix = (f & F_OBS) ? 0u : S_NONE;
        if (ix == S_NONE) continue;
        const uint32_t odc = (f >> 8) & 7u;
        int64_t ot;
        if constexpr (RANKED) ot = ot_get64(ob.ts, ix);
        else ot = ufl64(L.ots[q]);
        const int vl = (int)(((r & 7u) << 3) | odc);
        const int64_t va = rl64(vt0, vl), vb = rl64(vt1, vl);
        if ((r < 8 ? va : vb) < ot) continue;
      }
      bool was_min = false;
      if (!RANKED) {
        was_min = q == mn.p;
        --nobs;
      }
      if (lane == 0) atomicAnd(&L.opd[q], ~F_OBS);
      s_catch_up<PCAP, RANKED>(L, last, jr + 1, kdr, nxt, rok, rsc, rts, rd);
      last = jr + 1;
      SPROF(11);
      const uint32_t w = s_promote<PCAP, RANKED>(L, np);
      if (w == S_NONE) {  // (:283-289): Obs[Id] dropped, Min of the rest
        if (RANKED) (void)ot_merge<PCAP, RANKED>(ob, L, K, lane == 0, ix, false, 0, 0, 0, 0u);
        else if (was_min) s_min<PCAP, RANKED>(L, np, mn);
      } else {  // promote the largest (:290-295)
        const int64_t gs = ufl64(L.gsc[w]), gt = ufl64(L.gts[w]), wid = ufl64(L.pid[w]);
        const uint32_t gd = ufl(L.gpd[w]);
        if (lane == 0) {
          if constexpr (!RANKED) {
            L.osc[w] = gs;
            L.ots[w] = gt;
          }
          L.opd[w] = (L.opd[w] & 0xFFu) | F_OBS | (gd & 0xFFFFFF00u);
        }
        if (RANKED) {  // Obs[Id] dropped and the promoted entry placed in one step
          lsync(L);
          (void)ot_merge<PCAP, RANKED>(ob, L, K, lane == 0, ix, lane == 0, gs, wid, gt, w);
        } else {
          ++nobs;
          lsync(L);
          s_min<PCAP, RANKED>(L, np, mn);
        }
        if (lane == 0)
          s_emit<PCAP, RANKED>(a, L, op0, op0 + c0 + jr, CCRDT_TRMV_ADD, wid, gs, (gd >> 8) & 0xFFu, gt, nullptr);
      }
      lsync(L);
      SPROF(12);
    }
    s_catch_up<PCAP, RANKED>(L, last, n, kdr, nxt, rok, rsc, rts, rd);
    lsync(L);
    c0 += n;
    SPROF(7);
  }

  // ---- K5. positions of compacted slabs; player records; Vc; meta
  if (RANKED) {
    nobs = ob.n;
    mn.p = ob.mi == S_NONE ? S_NONE : ot_get32(ob.p, ob.mi);
  }
  uint32_t mcount = 0;
  for (uint32_t b = 0; b < np; b += 64) {
    const uint32_t p = b + lane;
    if (p < np) {
      uint32_t f = L.opd[p], g = L.gpd[p];
      const uint32_t ns = L.nslab[p], cnt = ns >> 16;
      if ((f & F_WALK) && cnt) {
        const uint64_t base = (uint64_t)nm.m_off + (ns & 0xFFFFu);
        int64_t os, ot;
        if constexpr (RANKED) {
          const uint32_t r = L.ork[p];  // meaningful with F_OBS
          os = L.tsc[r];
          ot = L.tts[r];
        } else {
          os = L.osc[p];
          ot = L.ots[p];
        }
        const uint32_t od = (f >> 8) & 0xFFu;
        uint32_t opos = NONE16, bpos = 0, bdc = 0;
        int64_t bsc = 0, bts = 0;
        for (uint32_t j = 0; j < cnt; ++j) {
          const int64_t s2 = KA->new_s.m_score[base + j], t2 = KA->new_s.m_ts[base + j];
          const uint32_t d2 = KA->new_s.m_dc[base + j];
          if (s2 == os && t2 == ot && d2 == od) opos = j;
          if (j == 0 || gb_gt(s2, d2, t2, bsc, bdc, bts)) {
            bsc = s2;
            bdc = d2;
            bts = t2;
            bpos = j;
          }
        }
        if (f & F_OBS) f = (f & 0xFFFFu) | (opos << 16);
        g = (bdc << 8) | (bpos << 16);
      }
      const uint64_t pp = (uint64_t)nm.p_off + p;
      KA->new_s.pl_id[pp] = L.pid[p];
      KA->new_s.pl_slab[pp] = ns;
      KA->new_s.pl_info[pp] = ((f & F_OBS) ? (f >> 16) : NONE16) | (L.orow[p] & 0xFFFF0000u);
      KA->new_s.pl_gb[pp] = (uint16_t)(cnt ? (g >> 16) : 0u);
      mcount += cnt;
    }
  }
  uint32_t mtotal;
  (void)wave_excl_scan_dpp(mcount, mtotal);
  if (lane < D) KA->new_s.vc[(uint64_t)key * D + lane] = (int64_t)L.vc[lane];
  if (lane == 0) {
    KeyMeta out = nm;
    out.np = np;
    out.nm = mtotal;
    out.nr = nr;
    out.nobs = nobs;
    out.minq = mn.p;
    KA->new_s.meta[key] = out;
    if (!done) KA->ex_cnt[key] = L.nex;
    KA->new_s.cap[key].flags = 0;  // (tier S's layout has no room recorded: tier R relocates the key)
  }
  SPROF(8);
  return S_DONE;
}

}  // namespace

template <int PCAP, int WAVES, bool RANKED>
__global__ __launch_bounds__(64 * WAVES) void trmv_steady_kernel(TrmvApplyArgs a) {
  __shared__ SLds<PCAP, RANKED> lds[WAVES];
  const uint32_t wv = ufl(threadIdx.x >> 6);
  SLds<PCAP, RANKED>& L = lds[wv];
  const uint32_t n = a.n_list_dev ? *a.n_list_dev : a.n_list;
  for (uint32_t w = blockIdx.x * WAVES + wv; w < n; w += gridDim.x * WAVES) {
    const uint32_t key = ufl(a.key_list ? a.key_list[w] : w);
    const int r = trmv_steady_key<PCAP, RANKED>(a, key, L);
    if (r == S_NEXT && lane_id() == 0) {
      const uint32_t pos = atomicAdd(&a.status[0], 1u);
      a.ovf_list[pos] = key;
    }
    lsync(L);
  }
}

// cls 0: up to 256 players per key, two keys per workgroup; cls 1: up to 1024
// players.  grid_keys bounds the work list (its length may live on the device).
void trmv_steady_preload() {
  preload_kernels(trmv_steady_kernel<256, 2, true>, trmv_steady_kernel<256, 2, false>, trmv_steady_kernel<1024, 1, true>,
                  trmv_steady_kernel<1024, 1, false>);
}

int trmv_launch_steady(const TrmvApplyArgs& a, int cls, uint64_t grid_keys, hipStream_t st) {
  if (grid_keys == 0) return CCRDT_OK;
  // Observed in registers when K <= 128 (ObsTab), else in LDS
  const bool ranked = a.k <= 128;
  if (cls == 0) {
    const uint64_t blocks = std::min<uint64_t>((grid_keys + 1) / 2, 16384);
    if (ranked)
      hipLaunchKernelGGL((trmv_steady_kernel<256, 2, true>), dim3((unsigned)blocks), dim3(128), 0, st, a);
    else
      hipLaunchKernelGGL((trmv_steady_kernel<256, 2, false>), dim3((unsigned)blocks), dim3(128), 0, st, a);
  } else {
    const uint64_t blocks = std::min<uint64_t>(grid_keys, 4096);
    if (ranked)
      hipLaunchKernelGGL((trmv_steady_kernel<1024, 1, true>), dim3((unsigned)blocks), dim3(64), 0, st, a);
    else
      hipLaunchKernelGGL((trmv_steady_kernel<1024, 1, false>), dim3((unsigned)blocks), dim3(64), 0, st, a);
  }
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

// The HBM class: up to PCAP_HBM players per key, SLds in a per-wave global
// scratch (`scratch` holds gridDim.x of them), one wave per workgroup.  Run
// on the keys the 1024-player class handed on.
template <bool RANKED>
__global__ __launch_bounds__(64) void trmv_steady_hbm_kernel(TrmvApplyArgs a, SLds<PCAP_HBM, RANKED>* scratch) {
  SLds<PCAP_HBM, RANKED>& L = scratch[blockIdx.x];
  const uint32_t n = a.n_list_dev ? *a.n_list_dev : a.n_list;
  for (uint32_t w = blockIdx.x; w < n; w += gridDim.x) {
    const uint32_t key = ufl(a.key_list ? a.key_list[w] : w);
    const int r = trmv_steady_key<PCAP_HBM, RANKED>(a, key, L);
    if (r == S_NEXT && lane_id() == 0) {
      const uint32_t pos = atomicAdd(&a.status[0], 1u);
      a.ovf_list[pos] = key;
    }
    lsync(L);
  }
}

uint64_t trmv_steady_hbm_bytes(bool ranked) {
  return ranked ? sizeof(SLds<PCAP_HBM, true>) : sizeof(SLds<PCAP_HBM, false>);
}
uint32_t trmv_steady_hbm_players() { return (uint32_t)PCAP_HBM; }

// `waves` workgroups, each with its scratch slot in `scratch` (waves *
// trmv_steady_hbm_bytes(K <= 128)).
int trmv_launch_steady_hbm(const TrmvApplyArgs& a, uint32_t waves, void* scratch, hipStream_t st) {
  if (waves == 0) return CCRDT_OK;
  if (a.k <= 128)
    hipLaunchKernelGGL((trmv_steady_hbm_kernel<true>), dim3(waves), dim3(64), 0, st, a,
                       reinterpret_cast<SLds<PCAP_HBM, true>*>(scratch));
  else
    hipLaunchKernelGGL((trmv_steady_hbm_kernel<false>), dim3(waves), dim3(64), 0, st, a,
                       reinterpret_cast<SLds<PCAP_HBM, false>*>(scratch));
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

}  // namespace ccrdt

#ifdef TRMV_PROF
extern "C" int ccrdt_debug_steady_prof(unsigned long long* out16, int reset) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_steady_prof), 16 * 8) != hipSuccess) return 4;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_steady_prof), z, sizeof(z)) != hipSuccess) return 4;
  }
  return 0;
}
#endif
