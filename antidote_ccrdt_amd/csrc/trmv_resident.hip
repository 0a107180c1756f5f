// trmv_resident.hip — tier R of the topk_rmv apply: a batch onto RESIDENT
// keys (the steady state Antidote drives: the same keys receive batch after
// batch, Observed full, more players than K, evictions and promotions).  One
// wavefront per key; the class: at most 256 players, K <= 128, Ids and Scores
// that fit in 32 bits.  A key outside it is handed on to tier S
// (trmv_steady.hip), which redoes it from the old side.
//
// The reference state machine (src/antidote_ccrdt_topk_rmv.erl:231-334) keeps
// two invariants after every op: Obs[Id] has the largest
// Score of Masked[Id], and Observed is the top K players by (largest Score,
// Id).  Every per-player effect — Removals merges, rmv filters, dominated adds
// (:234-237), set semantics (:240-246), gb_sets:largest — depends on the
// player's own ops only and is decided per player (op-parallel, or one lane
// per replayed player).  What depends on the order of ops ACROSS players is
// Observed: which element Obs[Id] holds, Min, and the promotions of rmv/3.
// Tier R keeps Observed as an array SORTED ascending by (Score, Id) in two
// register slots (entry r in lane r % 64 of slot r / 64, one packed 64-bit key
// per entry): Min is entry 0 (min_observed/1, :398-406; Ids are distinct), an
// eviction (:325-331), an upgrade (:303-315) or a promotion (:276-295) is one
// shift of a range of entries (DPP wave shifts).  Per run of adds between two
// rmvs, a lane-parallel filter keeps only the adds that can change Observed
// given the state at the run's start (inside a run Min and every Obs[Id] only
// rise); those run one by one in stream order on the register array alone.
// gb_sets:largest of every player — what a promotion needs — is brought up to
// date lane-parallel at each rmv (one segmented scan per chunk).  Players are
// written back with Observed first, in sorted order, so the next batch starts
// from the sorted array as it is (a key last written by tier 0 or tier S is
// sorted once, in registers).
//
// Phases per key:
//   P1  old players -> LDS / registers, the Id hash, the sorted Observed;
//   P2  every op's player (new Ids numbered in claim order; recorded per op),
//       ops per player, new slab offsets (old count + ops) and Removals rows;
//   P3  old Masked slabs and Removals rows -> the new side, position-parallel;
//   per chunk of <= 64 ops (<= 16 rmvs):
//     P3c validation, clocks, dominance and appends of the players without a
//         rmv (op-parallel), replays of the players with one (a lane each);
//     P4  the Observed half in stream order;
//   P5  player records (Observed first, sorted), positions, Vc, meta.
#include "common.hpp"
#include "trmv_kernels.hpp"

// Diagnostic build only (-DTRMV_PROF): per-phase s_memtime stamps summed over
// a sample of keys; read with ccrdt_debug_resident_prof().
#ifdef TRMV_PROF
__device__ unsigned long long g_resident_prof[32];
#define RPROF_STAMP(v)                                                        \
  do {                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                        \
  } while (0)
// (stamped keys: key & RPROF_MASK == 3 & RPROF_MASK; -DRPROF_MASK=0u stamps every key)
#ifndef RPROF_MASK
#define RPROF_MASK 63u
#endif
#define RPROF(i)                                                                         \
  do {                                                                                   \
    unsigned long long _t;                                                               \
    RPROF_STAMP(_t);                                                                     \
    if (lane_id() == 0 && (key & RPROF_MASK) == (3u & RPROF_MASK)) atomicAdd(&g_resident_prof[i], _t - prof_t); \
    prof_t = _t;                                                                         \
  } while (0)
#define RCOUNT(i, v)                                                                              \
  do {                                                                                            \
    if (lane_id() == 0 && (key & RPROF_MASK) == (3u & RPROF_MASK)) atomicAdd(&g_resident_prof[i], (unsigned long long)(v)); \
  } while (0)
#else
#define RPROF(i) (void)0
#define RCOUNT(i, v) (void)0
#endif

namespace ccrdt {

namespace {

#define KA trmv_kargs()  // (trmv_kernels.hpp)

constexpr int RP = 256;        // players per key
constexpr int RSL = RP / 64;   // player slots per lane
constexpr int RCH = 64;        // ops per chunk
constexpr int RCHR = 16;       // rmvs per chunk (rows of the clock table)
constexpr uint32_t RNONE = 0xFFFFFFFFu;
constexpr int RFBLK = 4;           // replays: slab elements per block of loads in a rmv's filter
constexpr uint32_t MBALLOT = 3;    // merges of up to this many candidates ranked by ballot pairs; more: LDS list + histogram
constexpr uint32_t RH_NONE = 0xFFFFu, RH_CLAIM = 0x8000u;  // hash slots: player | CLAIM|lane | NONE
enum : int { R_DONE = 0, R_NEXT = 1, R_REJECT = 2 };
enum : int { LAY_TIGHT = 0, LAY_APPEND = 1, LAY_COMPACT = 2 };

// pf[p] flags
constexpr uint32_t Q_OBS = 1u;   // Id in Observed
constexpr uint32_t Q_HASM = 2u;  // Masked[Id] is not empty
constexpr uint32_t Q_ROWV = 4u;  // Removals[Id] exists
constexpr uint32_t Q_RMV = 8u;   // a rmv of Id in this batch: its slab is replayed by one lane
constexpr uint32_t Q_WALK = 16u; // a replay compacted the slab: positions restated in P5
constexpr uint32_t Q_DUP = 32u;  // a possibly duplicated element: replayed too
constexpr uint32_t Q_UPG = 64u;  // (inside a merge) an Observed player whose entry the run upgrades
constexpr uint32_t Q_DIRTY = 128u;  // the player's record changes (ops, a moved slab, a promotion): written in P5
constexpr uint32_t R_DOM = 1u;   // cres: dominated add (:234-237)

__device__ __forceinline__ uint32_t ufl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int64_t ufl64(int64_t v) {
  const uint32_t lo = ufl((uint32_t)v), hi = ufl((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t perm32(uint32_t v, uint32_t dst) {
  return (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)v);
}
// Lane i <- v of lane i + 1 (lane 63 <- fill): DPP wave_shl:1.
__device__ __forceinline__ uint32_t wshl1(uint32_t v, uint32_t fill) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x130, 0xf, 0xf, false);
}
// Lane i <- v of lane i - 1 (lane 0 <- fill): DPP wave_shr:1.
__device__ __forceinline__ uint32_t wshr1(uint32_t v, uint32_t fill) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t lo32(int64_t v) { return (uint32_t)v; }
__device__ __forceinline__ uint32_t hi32(int64_t v) { return (uint32_t)((uint64_t)v >> 32); }
__device__ __forceinline__ int64_t mk64(uint32_t lo, uint32_t hi) { return (int64_t)(((uint64_t)hi << 32) | lo); }
__device__ __forceinline__ bool fits32(int64_t v) { return v == (int64_t)(int32_t)v; }

// (Score, Id) of 32-bit values as one signed 64-bit key: comparing keys
// compares Score, then Id (the Id's sign bit flipped so it orders unsigned).
__device__ __forceinline__ int64_t mkkey(int64_t score, int64_t id) {
  return (int64_t)(((uint64_t)(uint32_t)(int32_t)score << 32) | ((uint32_t)(int32_t)id ^ 0x80000000u));
}
__device__ __forceinline__ int64_t key_score(int64_t k) { return (int64_t)(int32_t)(uint32_t)((uint64_t)k >> 32); }
__device__ __forceinline__ int64_t key_id(int64_t k) { return (int64_t)(int32_t)((uint32_t)k ^ 0x80000000u); }

// gb_sets term order of two elements of one Id: (Score, DcId, Ts).
__device__ __forceinline__ bool gb_gt(int64_t s1, uint32_t d1, int64_t t1, int64_t s2, uint32_t d2, int64_t t2) {
  return s1 > s2 || (s1 == s2 && (d1 > d2 || (d1 == d2 && t1 > t2)));
}

// One step of P4's segmented scan over the sorted chunk (DPP: row_shr 1, 2,
// 4, 8 inside rows of 16, then row_bcast 15 and 31 across rows -- the
// inclusive-scan pattern, valid for any associative operator).  A lane whose
// source lies outside its row (or whose row the step skips) reads 0: flags
// 0, no source, the step leaves it as it is.  Per lane: v = the gb_sets-largest
// (Score, DcId, Ts) of the segment so far, w = its cmp/2-largest (Score, Ts;
// the earlier of equals); vd = DcId | slab position << 8 | ok << 30 | head << 31.
template <int C, int RM>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, C, RM, 0xf, false);
}
template <int C, int RM>
__device__ __forceinline__ int64_t dpp0_64(int64_t x) {
  return (int64_t)(((uint64_t)dpp0<C, RM>((uint32_t)((uint64_t)x >> 32)) << 32) | dpp0<C, RM>((uint32_t)x));
}
template <int C, int RM>
__device__ __forceinline__ void seg_step(int32_t& vs, int64_t& vt, uint32_t& vd, int32_t& ws, int64_t& wt,
                                         uint32_t& wd) {
  const uint32_t yd = dpp0<C, RM>(vd), zd = dpp0<C, RM>(wd);
  const int32_t ys = (int32_t)dpp0<C, RM>((uint32_t)vs), zs = (int32_t)dpp0<C, RM>((uint32_t)ws);
  const int64_t yt = dpp0_64<C, RM>(vt), zt = dpp0_64<C, RM>(wt);
  const bool ok = (vd >> 30) & 1u, hf = (vd >> 31) != 0u, yok = (yd >> 30) & 1u, yhf = (yd >> 31) != 0u;
  if (!hf) {
    if (yok) {
      if (!ok || gb_gt(ys, yd & 0xFFu, yt, vs, vd & 0xFFu, vt)) {
        vs = ys;
        vt = yt;
        vd = (vd & 0xC0000000u) | (yd & 0x3FFFFFFFu);
      }
      if (!ok || !(ws > zs || (ws == zs && wt > zt))) {  // the earlier one wins ties
        ws = zs;
        wt = zt;
        wd = zd;
      }
    }
    vd = (vd & 0x3FFFFFFFu) | ((ok || yok) ? (1u << 30) : 0u) | (yhf ? (1u << 31) : 0u);
  }
}

// Inclusive max-scan over the wave (DPP row shifts, then row broadcasts):
// each lane gets the largest value at or below it.
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

typedef int64_t Row8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ int64_t pick8(const Row8& v, uint32_t d) {
  int64_t r = v[0];
#pragma unroll
  for (int k = 1; k < TRMV_DPAD; ++k) r = d == (uint32_t)k ? v[k] : r;
  return r;
}

template <int BITS>
__device__ __forceinline__ uint32_t wave_radix_sort(uint32_t kv) {  // by bits [6, 6 + BITS); payload 6 bits
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

// One stable counting pass over a 4-bit digit (bits [6 + SHIFT, 10 + SHIFT))
// of kv (payload: the low 6 bits): the sixteen digit masks by ballot, each
// lane's destination = the lanes of smaller digits + its rank among its own,
// one permute.  Two passes sort by 8 bits with two LDS-crossbar round trips
// (a bit per pass took eight).
template <int SHIFT>
__device__ __forceinline__ uint32_t radix16_pass(uint32_t kv) {
  const uint32_t dg = (kv >> (6 + SHIFT)) & 15u;
  uint64_t mine = 0;
  uint32_t base = 0, acc = 0;
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    const bool me = dg == (uint32_t)d;
    const uint64_t m = ballot(me);
    mine = me ? m : mine;
    base = me ? acc : base;
    acc += (uint32_t)__builtin_popcountll(m);
  }
  return perm32(kv, base + mbcnt(mine));
}

// Position of the k-th (0-based) set bit of m (k < popcount(m)).
__device__ __forceinline__ uint32_t kth_bit(uint64_t m, uint32_t k) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t s = 32; s >= 1; s >>= 1) {
    const uint64_t low = pos + s >= 64 ? ~0ull : ((1ull << (pos + s)) - 1);
    if ((uint32_t)__builtin_popcountll(m & low) <= k) pos += s;
  }
  return pos;
}

__device__ __forceinline__ uint32_t rhash(int64_t id) {
  return (uint32_t)(((uint64_t)id * 0x9E3779B97F4A7C15ull) >> (64 - 9));  // 512 slots
}

// One key's LDS: 12,112 bytes (6 two-key workgroups per CU).  Ids and Scores are 32-bit in
// this class; Obs[Id]'s DcId lives in the sorted Observed array (Obs.pl).
struct alignas(16) RLds {
  int64_t gts[RP];     // gb_sets:largest(Masked[Id]): Ts
  int64_t ots[RP];     // Obs[Id]'s Ts (valid while the player is in Observed)
  int32_t msc[RP];     // largest Score of Masked[Id] (= Obs[Id]'s Score in Observed, or below it mid-run)
  uint32_t nslab[RP];  // new slab: offset | current count << 16
  uint16_t prow[RP];   // Removals row (new side), NONE16
  uint16_t opos[RP];   // Obs[Id]'s position in the new slab
  uint16_t gpos[RP];   // the largest's position in the new slab
  uint8_t pf[RP];      // flags (atomics: pf_or / pf_and on the containing word)
  uint8_t gdc[RP];     // the largest: DcId
  uint32_t obs0[RP / 32];  // players in Observed when the batch starts (P5 writes the records that change)
  union {
    struct {  // P1 / P2 (P3: hs..claim hold the start map; nops (the slab need) and oslab stay)
      uint16_t hs[2 * RP];
      int32_t pid[RP];
      int32_t claim[64];
      uint16_t nops[RP];   // P2: adds per player; from the plan on: the slab's need (old count + adds)
      uint32_t oslab[RP];  // old slab: offset | count << 16
    } r;
    struct {  // chunks
      int32_t csc[RCH];
      int64_t cts[RCH];
      int32_t cid[RCH];    // Ids, (player, stream) order
      uint32_t ckd[RCH];   // kind | dc << 2 | dup candidate << 5 | player << 8
      uint32_t cres[RCH];  // add: R_DOM | slab position << 16; rmv: its rank in the chunk
      int64_t vtab[RCHR][TRMV_DPAD];
      uint32_t crow[RCHR];
      int64_t rgs[RCHR], rgt[RCHR];  // Masked[Id]'s largest survivor after each rmv
      uint32_t rgd[RCHR];            // non-empty | dc << 8 | position << 16
      uint16_t cwp[RCH];
      uint8_t cws[RCH], cwe[RCH], csrt[RCH];
    } c;
    struct {  // P5
      uint8_t odc[RP];  // Obs[Id]'s DcId by player
    } f;
  } u;
  unsigned long long vc[TRMV_DPAD + 1];  // replica Vc; [TRMV_DPAD] sink
  uint32_t nex;
};

__device__ __forceinline__ void pf_or(RLds& L, uint32_t p, uint32_t m) {
  atomicOr(reinterpret_cast<uint32_t*>(&L.pf[p & ~3u]), m << (8u * (p & 3u)));
}
__device__ __forceinline__ void pf_and(RLds& L, uint32_t p, uint32_t m) {  // clears m
  atomicAnd(reinterpret_cast<uint32_t*>(&L.pf[p & ~3u]), ~(m << (8u * (p & 3u))));
}

// --------------------------------------------------- the sorted Observed
// Entry r = lane r % 64 of slot r / 64, ascending by key = (Score, Id);
// pl = player | Obs[Id]'s DcId << 16; entries >= n hold (INT64_MAX, RNONE).
// (Obs[Id]'s Ts lives per player in LDS, RLds::ots: an entry is three dwords.)
struct Obs {
  int64_t key[2];
  uint32_t pl[2];
  uint32_t n;
};

__device__ __forceinline__ void ob_clear_tail(Obs& o) {
  const uint32_t l = (uint32_t)lane_id();
#pragma unroll
  for (int t = 0; t < 2; ++t)
    if (64u * t + l >= o.n) {
      o.key[t] = INT64_MAX;
      o.pl[t] = RNONE;
    }
}

// Entries i in [lo, hi) take entry i + 1 (down) or entries i in [lo, hi]
// take entry i - 1 (up); both slots always shift (no branches on the range).
template <bool DOWN>
__device__ __forceinline__ void ob_shift(Obs& o, uint32_t lo, uint32_t hi) {
  const uint32_t l = (uint32_t)lane_id();
  const bool in0 = DOWN ? (l >= lo && l < hi) : (l >= lo && l <= hi);
  const bool in1 = DOWN ? (64u + l >= lo && 64u + l < hi) : (64u + l >= lo && 64u + l <= hi);
  uint32_t w0[3] = {lo32(o.key[0]), hi32(o.key[0]), o.pl[0]};
  uint32_t w1[3] = {lo32(o.key[1]), hi32(o.key[1]), o.pl[1]};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    uint32_t n0, n1;
    if (DOWN) {
      n0 = wshl1(w0[k], rl32(w1[k], 0));
      n1 = wshl1(w1[k], 0u);
    } else {
      n0 = wshr1(w0[k], 0u);
      n1 = wshr1(w1[k], rl32(w0[k], 63));
    }
    w0[k] = in0 ? n0 : w0[k];
    w1[k] = in1 ? n1 : w1[k];
  }
  o.key[0] = mk64(w0[0], w0[1]);
  o.pl[0] = w0[2];
  o.key[1] = mk64(w1[0], w1[1]);
  o.pl[1] = w1[2];
}

__device__ __forceinline__ void ob_put(Obs& o, uint32_t q, int64_t key, uint32_t pl) {
  const uint32_t l = (uint32_t)lane_id();
  if (l == (q & 63u)) {
    if (q < 64u) {
      o.key[0] = key;
      o.pl[0] = pl;
    } else {
      o.key[1] = key;
      o.pl[1] = pl;
    }
  }
}

// Entries below key, skipping entry `skip` (RNONE: none).
__device__ __forceinline__ uint32_t ob_rank(const Obs& o, int64_t key, uint32_t skip) {
  const uint32_t l = (uint32_t)lane_id();
  const bool b0 = l < o.n && l != skip && o.key[0] < key;
  const bool b1 = 64u + l < o.n && 64u + l != skip && o.key[1] < key;
  return (uint32_t)__builtin_popcountll(ballot(b0)) + (uint32_t)__builtin_popcountll(ballot(b1));
}

__device__ __forceinline__ uint32_t ob_find(const Obs& o, uint32_t p) {
  const uint64_t m0 = ballot((o.pl[0] & 0xFFFFu) == p), m1 = ballot((o.pl[1] & 0xFFFFu) == p);
  return m0 ? (uint32_t)__builtin_ctzll(m0) : (m1 ? 64u + (uint32_t)__builtin_ctzll(m1) : RNONE);
}
__device__ __forceinline__ int64_t ob_get64(const int64_t f[2], uint32_t i) {
  const int64_t a = rl64(f[0], (int)(i & 63u)), b = rl64(f[1], (int)(i & 63u));
  return i < 64u ? a : b;
}
__device__ __forceinline__ uint32_t ob_get32(const uint32_t f[2], uint32_t i) {
  const uint32_t a = rl32(f[0], (int)(i & 63u)), b = rl32(f[1], (int)(i & 63u));
  return i < 64u ? a : b;
}

// Entry r removed and (key, pl) inserted, in one range shift.
__device__ __forceinline__ void ob_replace(Obs& o, uint32_t r, int64_t key, uint32_t pl) {
  const uint32_t q = ob_rank(o, key, r);
  if (q >= r) ob_shift<true>(o, r, q);
  else ob_shift<false>(o, q + 1, r);
  ob_put(o, q, key, pl);
}
__device__ __forceinline__ void ob_insert(Obs& o, int64_t key, uint32_t pl) {
  const uint32_t q = ob_rank(o, key, RNONE);
  ob_shift<false>(o, q + 1, o.n);
  ob_put(o, q, key, pl);
  ++o.n;
}
__device__ __forceinline__ void ob_remove(Obs& o, uint32_t r) {
  ob_shift<true>(o, r, o.n - 1);
  --o.n;
  ob_clear_tail(o);
}

__device__ __forceinline__ void r_emit(const TrmvApplyArgs& a, RLds& L, uint64_t op0, uint64_t op, uint8_t kind,
                                       int64_t id, int64_t sc, uint32_t dc, int64_t ts, const Row8* vc) {
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

// A dominated add's {rmv, {Id, Removals[Id]}} with the row read from memory.
__device__ __forceinline__ void r_emit_row(const TrmvApplyArgs& a, RLds& L, uint64_t op0, uint64_t op, int64_t id,
                                           const int64_t* row) {
  const uint32_t pos = atomicAdd(&L.nex, 1u);
  TrmvExtraRec r;
  r.op = (uint32_t)op;
  r.kind = CCRDT_TRMV_RMV;
  r.dc = 0;
  r.pad = 0;
  r.id = id;
  r.score = 0;
  r.ts = 0;
  KA->ex[op0 + pos] = r;
  for (int d = 0; d < KA->n_dc; ++d) KA->ex_vc[(op0 + pos) * KA->n_dc + d] = row[d];
}

// P2: the player of each lane's Id; new Ids claimed and numbered np, np+1,
// ... in lane order.  False if the key outgrows RP players.
__device__ __forceinline__ bool r_resolve(RLds& L, int64_t id, bool v, uint32_t& np, uint32_t& p) {
  const int lane = lane_id();
  L.u.r.claim[lane] = id;
  wave_lds_sync();
  uint32_t h = rhash(id);
  bool resolved = !v, claimed = false;
  int follow = -1;
  p = 0;
  while (ballot(!resolved)) {
    if (!resolved) {
      uint32_t* w = reinterpret_cast<uint32_t*>(&L.u.r.hs[h & ~1u]);
      const uint32_t sh = (h & 1u) * 16u;
      const uint32_t s = (*w >> sh) & 0xFFFFu;
      if (s == RH_NONE) {
        uint32_t old = *w;
        bool won = false;
        for (;;) {
          if (((old >> sh) & 0xFFFFu) != RH_NONE) break;
          const uint32_t prev = atomicCAS(w, old, (old & ~(0xFFFFu << sh)) | ((RH_CLAIM | (uint32_t)lane) << sh));
          if (prev == old) {
            won = true;
            break;
          }
          old = prev;
        }
        if (won) {
          claimed = true;
          resolved = true;
        }  // else: read the slot again
      } else if (s & RH_CLAIM) {
        const int c = (int)(s & 63u);
        if (L.u.r.claim[c] == id) {
          follow = c;
          resolved = true;
        } else {
          h = (h + 1) & (2 * RP - 1);
        }
      } else if (L.u.r.pid[s] == id) {
        p = s;
        resolved = true;
      } else {
        h = (h + 1) & (2 * RP - 1);
      }
    }
  }
  wave_lds_sync();
  const uint64_t cm = ballot(claimed);
  const uint32_t nn = np + (uint32_t)__builtin_popcountll(cm);
  if (nn > (uint32_t)RP) return false;
  if (claimed) {
    p = np + mbcnt(cm);
    L.u.r.pid[p] = id;
    L.u.r.hs[h] = (uint16_t)p;
    L.u.r.nops[p] = 0;
    L.u.r.oslab[p] = 0u;
    L.prow[p] = (uint16_t)NONE16;
    L.pf[p] = 0u;
    L.msc[p] = 0;
    L.gts[p] = 0;
    L.opos[p] = (uint16_t)NONE16;
    L.gpos[p] = 0;
    L.gdc[p] = 0;
  }
  const uint32_t fp = shfl32(p, follow >= 0 ? follow : lane);
  if (follow >= 0) p = fp;
  np = nn;
  wave_lds_sync();
  return true;
}

// Promotion candidate of rmv/3 (:276-281, :291): the player outside Observed
// with Masked elements whose (largest Score, Id) is largest; RNONE if none.
// Its key in `wk`, its largest element's Ts / DcId / slab position in `wt`,
// `wd`, `wp` (read with the slots' flags and Scores, one LDS round trip).
__device__ __forceinline__ uint32_t r_promote(const RLds& L, const int64_t pid[RSL], uint32_t np, int64_t& wk,
                                             int64_t& wt, uint32_t& wd, uint32_t& wp) {
  const uint32_t l = (uint32_t)lane_id();
  uint32_t bp = RNONE;
  int64_t best = INT64_MIN;
  // flags and Scores of the lane's four slots, then the largest element's
  // Ts / DcId / position of its best slot only (4 + 3 LDS reads, not 20)
  uint32_t f[RSL];
  int32_t sc[RSL];
#pragma unroll
  for (int u = 0; u < RSL; ++u) {
    const uint32_t p = 64u * u + l;
    f[u] = p < np ? L.pf[p] : 0u;
    sc[u] = L.msc[p];
  }
#pragma unroll
  for (int u = 0; u < RSL; ++u) {
    const int64_t k = mkkey(sc[u], pid[u]);
    if ((f[u] & (Q_OBS | Q_HASM)) == Q_HASM && (bp == RNONE || k > best)) {
      bp = 64u * u + l;
      best = k;
    }
  }
  const uint32_t bq = bp != RNONE ? bp : 0u;
  const int64_t bt = L.gts[bq];
  const uint32_t bd = L.gdc[bq], bg = L.gpos[bq];
  if (!ballot(bp != RNONE)) return RNONE;
  const int64_t m = wave_max_i64_dpp(bp != RNONE ? best : INT64_MIN);
  const int src = (int)__builtin_ctzll(ballot(bp != RNONE && best == m));
  wk = m;
  wt = rl64(bt, src);
  wd = rl32(bd, src);
  wp = rl32(bg, src);
  return rl32(bp, src);
}

// One key.  Returns R_NEXT for a key outside the class: the next tier redoes
// it from the old side (whatever this one wrote of it is rewritten).  In
// place (KA->inplace) every R_NEXT is decided before the key's first store,
// so the key is left as it was.
template <bool INPL>
__device__ int trmv_resident_key(const TrmvApplyArgs& a, uint32_t key, uint32_t nkey, RLds& L) {
  const uint32_t lane = (uint32_t)lane_id();
  const int D = KA->n_dc;
#ifdef TRMV_PROF
  unsigned long long prof_t;
  RPROF_STAMP(prof_t);
#endif
  constexpr bool inpl = INPL;  // (KA->inplace: one instantiation per mode)
  // in place: an invalid op anywhere in the batch (the validation pass ran
  // before this kernel) means nothing is written
  if (inpl && *KA->verr) return R_REJECT;
  const uint64_t op0 = KA->key_ptr[key];
  // (a key whose ops an earlier pass applied is only rewritten: no ops)
  const bool done = KA->key_done && KA->key_done[key];
  const uint32_t nops = done ? 0u : (uint32_t)(KA->key_ptr[key + 1] - op0);
  // (a fresh batch: the keys tier 0 handed on, with no old state)
  const bool fresh = KA->fresh != 0;
  KeyMeta om;
  KeyCap oc;
  if (fresh) {
    om.p_off = om.m_off = om.r_off = 0;
    om.np = om.nm = om.nr = om.nobs = 0;
    om.minq = NONE32;
    oc.p_cap = oc.m_cap = oc.r_cap = 0;
    oc.m_top = oc.flags = 0;
  } else {
    om = KA->old_s.meta[key];
    if (inpl) oc = KA->old_s.cap[key];
  }
  // (per-player op counts are 16-bit here)
  if (om.np > (uint32_t)RP || om.nobs > 128u || nops > 0xFFFFu) return R_NEXT;
  const uint32_t K = KA->k;

  for (uint32_t i = lane; i < (uint32_t)RP; i += 64) reinterpret_cast<uint32_t*>(L.u.r.hs)[i] = 0xFFFFFFFFu;
  if (lane <= (uint32_t)TRMV_DPAD)
    L.vc[lane] = (!fresh && lane < (uint32_t)D) ? (unsigned long long)KA->old_s.vc[(uint64_t)key * D + lane] : 0ull;
  if (lane == 0) L.nex = 0u;
  wave_lds_sync();

  // P2's first round of op Ids and kinds, loaded now: their latency runs
  // under P1's own load chains instead of after them
  int64_t pre_id[2], pre_sc[2];
  uint32_t pre_kd[2], pre_ord[2];
  {
    // (and the Observed order tier R recorded, which P1 checks)
    const __amdgpu_buffer_rsrc_t bor = bsrc(KA->obs_ord + (uint64_t)key * TRMV_ORD, om.nobs * 2u);
#pragma unroll
    for (int h = 0; h < 2; ++h) pre_ord[h] = bld16(bor, (64u * h + lane) * 2u);
    const __amdgpu_buffer_rsrc_t bid0 = bsrc(KA->id + op0, nops * 8u);
    const __amdgpu_buffer_rsrc_t bsc0 = bsrc(KA->score + op0, nops * 8u);
    const __amdgpu_buffer_rsrc_t bkd0 = bsrc(KA->kind + op0, nops);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      pre_id[h] = bld64(bid0, (64u * h + lane) * 8u);
      pre_sc[h] = bld64(bsc0, (64u * h + lane) * 8u);
      pre_kd[h] = bld8(bkd0, 64u * h + lane);
    }
  }
  // ---- P1. old players: records of all four slots, then the Obs[Id] /
  // largest elements they name (two rounds of loads in flight), then LDS and
  // the Id hash (the four slots' probes interleaved).
  // Observed comes sorted from the order tier R recorded (obs_ord, checked),
  // else it is gathered and sorted here.
  int64_t pid[RSL];
  uint32_t span = 0, inobs = 0;  // inobs: bit u = player of slot u in Observed
  uint32_t odr[RSL];             // Obs[Id]'s DcId by slot
  bool wide = false;
  {
    uint32_t info[RSL], slab[RSL], gb[RSL];
    {
      // (the four arrays' bases once, and pl_gb read whatever the slab's
      // count: a load conditional on another load's value waited for it, slot
      // by slot)
      // (bounds-checked buffer loads: the slots past np read 0, every load
      // of the four slots goes out back to back)
      const __amdgpu_buffer_rsrc_t rid = bsrc(KA->old_s.pl_id + om.p_off, om.np * 8u);
      const __amdgpu_buffer_rsrc_t rinfo = bsrc(KA->old_s.pl_info + om.p_off, om.np * 4u);
      const __amdgpu_buffer_rsrc_t rslab = bsrc(KA->old_s.pl_slab + om.p_off, om.np * 4u);
      const __amdgpu_buffer_rsrc_t rgb = bsrc(KA->old_s.pl_gb + om.p_off, om.np * 2u);
#pragma unroll
      for (int u = 0; u < RSL; ++u) {
        const uint32_t p = 64u * u + lane;
        const bool v = p < om.np;
        pid[u] = bld64(rid, p * 8u);
        const uint32_t in = bld32(rinfo, p * 4u);
        info[u] = v ? in : RNONE;
        slab[u] = bld32(rslab, p * 4u);
        gb[u] = bld16(rgb, p * 2u);
      }
#pragma unroll
      for (int u = 0; u < RSL; ++u) gb[u] = (slab[u] >> 16) > 1 ? gb[u] : 0u;  // (readers take 0 below 2)
    }
    int64_t os[RSL], ot[RSL], gs[RSL], gt[RSL];
    uint32_t gd[RSL];
    {
      // (slabs may leave holes, so a key's pool segment is not [0, nm): the
      // range is open-ended and only the lanes with nothing to read are sent
      // past it; the others read exactly what the plain loads read)
      const __amdgpu_buffer_rsrc_t rsc = bsrc(KA->old_s.m_score + om.m_off, BOOB);
      const __amdgpu_buffer_rsrc_t rts = bsrc(KA->old_s.m_ts + om.m_off, BOOB);
      const __amdgpu_buffer_rsrc_t rdc = bsrc(KA->old_s.m_dc + om.m_off, BOOB);
#pragma unroll
      for (int u = 0; u < RSL; ++u) {
        const uint32_t off = slab[u] & 0xFFFFu, cnt = slab[u] >> 16, obx = info[u] & 0xFFFFu;
        const bool ho = obx != NONE16, hg = cnt != 0;
        const uint32_t qo = off + (ho ? obx : 0u), qg = off + gb[u];
        os[u] = bld64(rsc, ho ? qo * 8u : BOOB);
        ot[u] = bld64(rts, ho ? qo * 8u : BOOB);
        odr[u] = bld8(rdc, ho ? qo : BOOB);
        gs[u] = bld64(rsc, hg ? qg * 8u : BOOB);
        gt[u] = bld64(rts, hg ? qg * 8u : BOOB);
        gd[u] = bld8(rdc, hg ? qg : BOOB);
      }
    }
    {
      // the Id hash (16-bit slots: CAS on the containing word) while the
      // element loads above are in flight; each round reads every pending
      // slot's word, then claims the free ones
      uint32_t hh[RSL];
      bool pend[RSL];
#pragma unroll
      for (int u = 0; u < RSL; ++u) {
        pend[u] = 64u * u + lane < om.np;
        hh[u] = rhash(pid[u]);
      }
      for (;;) {
        bool any = false;
#pragma unroll
        for (int u = 0; u < RSL; ++u) any |= pend[u];
        if (!ballot(any)) break;
        uint32_t cur[RSL];
#pragma unroll
        for (int u = 0; u < RSL; ++u)
          cur[u] = pend[u] ? *reinterpret_cast<const uint32_t*>(&L.u.r.hs[hh[u] & ~1u]) : 0u;
#pragma unroll
        for (int u = 0; u < RSL; ++u) {
          if (!pend[u]) continue;
          const uint32_t sh = (hh[u] & 1u) * 16u;
          if (((cur[u] >> sh) & 0xFFFFu) == RH_NONE) {
            const uint32_t p = 64u * u + lane;
            uint32_t* w = reinterpret_cast<uint32_t*>(&L.u.r.hs[hh[u] & ~1u]);
            if (atomicCAS(w, cur[u], (cur[u] & ~(0xFFFFu << sh)) | (p << sh)) == cur[u]) pend[u] = false;
          } else {
            hh[u] = (hh[u] + 1) & (2 * RP - 1);
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < RSL; ++u) {
      const uint32_t p = 64u * u + lane;
      const uint32_t off = slab[u] & 0xFFFFu, cnt = slab[u] >> 16, obx = info[u] & 0xFFFFu;
      const bool ho = obx != NONE16;
      if (p < om.np) {
        wide |= !fits32(pid[u]) || !fits32(os[u]) || !fits32(gs[u]);
        L.msc[p] = (int32_t)gs[u];
        L.gts[p] = gt[u];
        L.ots[p] = ot[u];  // (meaningful for players in Observed)
        L.pf[p] = (ho ? Q_OBS : 0u) | (cnt ? Q_HASM : 0u) | ((info[u] >> 16) != NONE16 ? Q_ROWV : 0u);
        L.gdc[p] = (uint8_t)gd[u];
        L.opos[p] = (uint16_t)obx;
        L.gpos[p] = (uint16_t)gb[u];
        L.u.r.oslab[p] = slab[u];
        L.prow[p] = (uint16_t)(info[u] >> 16);
        L.u.r.pid[p] = pid[u];
        L.u.r.nops[p] = 0;
        span = off + cnt > span ? off + cnt : span;
      }
      inobs |= (ho ? 1u : 0u) << u;
    }
  }
  if (ballot(wide)) return R_NEXT;  // a wide Id or Score: tier S
  span = wave_max_u32_dpp(span);
#pragma unroll
  for (int u = 0; u < RSL; ++u) {  // the players in Observed at the start
    const uint64_t m = ballot((inobs >> u) & 1u);
    if (lane == 0) {
      L.obs0[2 * u] = (uint32_t)m;
      L.obs0[2 * u + 1] = (uint32_t)(m >> 32);
    }
  }
  wave_lds_sync();
  Obs ob;
  ob.n = om.nobs;
  {
    // entry r = the player obs_ord[r]: its key (Obs[Id]'s Score is the
    // largest, I1) from LDS, its DcId from the lane that holds its slot.
    // Accepted when every entry is an Observed player and the keys rise
    // strictly: then the nobs entries are exactly Observed, sorted (the
    // record can be stale: a key other tiers wrote since, or never written)
    bool bad = false;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint32_t i = 64u * t + lane;
      const bool in = i < ob.n;
      const uint32_t q0 = in ? pre_ord[t] : 0u;
      const bool qok = in && q0 < om.np;
      const uint32_t q = qok ? q0 : 0u;
      const uint32_t qf = L.pf[q];
      uint32_t d = 0;
#pragma unroll
      for (int u = 0; u < RSL; ++u) {
        const uint32_t v = shfl32(odr[u], (int)(q & 63u));
        d = (q >> 6) == (uint32_t)u ? v : d;
      }
      ob.key[t] = in ? mkkey(L.msc[q], L.u.r.pid[q]) : INT64_MAX;
      ob.pl[t] = in ? (q | (d << 16)) : RNONE;
      bad |= in && (!qok || !(qf & Q_OBS));
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint32_t i = 64u * t + lane;
      const uint32_t nlo = t == 0 ? wshl1(lo32(ob.key[0]), rl32(lo32(ob.key[1]), 0)) : wshl1(lo32(ob.key[1]), 0u);
      const uint32_t nhi = t == 0 ? wshl1(hi32(ob.key[0]), rl32(hi32(ob.key[1]), 0)) : wshl1(hi32(ob.key[1]), 0u);
      if (i + 1 < ob.n) bad |= !(ob.key[t] < mk64(nlo, nhi));
    }
    if (ballot(bad)) {
      // the r-th Observed player in player order is pulled by entry r; then sort
      uint64_t mk[RSL];
      uint32_t base[RSL + 1];
      base[0] = 0;
#pragma unroll
      for (int u = 0; u < RSL; ++u) {
        mk[u] = ballot((inobs >> u) & 1u);
        base[u + 1] = base[u] + (uint32_t)__builtin_popcountll(mk[u]);
      }
      ob.n = base[RSL];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const uint32_t r = 64u * t + lane;
        ob.key[t] = INT64_MAX;
        ob.pl[t] = RNONE;
#pragma unroll
        for (int u = 0; u < RSL; ++u) {
          const bool here = r >= base[u] && r < base[u + 1];
          const uint32_t src = here ? kth_bit(mk[u], r - base[u]) : lane;
          const int64_t vi = shfl64(pid[u], (int)src);
          const uint32_t vd = shfl32(odr[u], (int)src);
          if (here) {
            const uint32_t p = 64u * u + src;
            ob.key[t] = mkkey(L.msc[p], vi);  // Obs[Id]'s Score = the largest (I1)
            ob.pl[t] = p | (vd << 16);
          }
        }
      }
      // sorted by rank: each entry counts the keys below it (distinct Ids,
      // so distinct keys), every key broadcast from its lane, one round per
      // entry; then each entry goes to its rank through LDS (nslab is first
      // written in P2) and its key is made again from its player.  (A bitonic
      // sort on LDS-crossbar shuffles took ~18k cycles per key here.)
      uint32_t rk[2] = {0u, 0u};
      for (uint32_t i = 0; i < ob.n; ++i) {
        const int64_t ki = i < 64u ? rl64(ob.key[0], (int)i) : rl64(ob.key[1], (int)(i - 64u));
        rk[0] += ki < ob.key[0] ? 1u : 0u;
        rk[1] += ki < ob.key[1] ? 1u : 0u;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
        if (64u * t + lane < ob.n) L.nslab[rk[t]] = ob.pl[t];
      wave_lds_sync();
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (64u * t + lane < ob.n) {
          const uint32_t pl = L.nslab[64u * t + lane], p = pl & 0xFFFFu;
          ob.pl[t] = pl;
          ob.key[t] = mkkey(L.msc[p], L.u.r.pid[p]);
        }
      }
      wave_lds_sync();
    }
  }
  ob_clear_tail(ob);
  wave_lds_sync();
  RPROF(0);
  {
    // ---- P2. every op's player; adds per player; rmv players
    uint32_t np = om.np;
    // 128 ops per round: both halves' Ids, Scores and kinds load together,
    // then each half is resolved (one 64-lane claim table).  A wide Id or add
    // Score hands the key on here, before anything is written.
    // (the key's op columns through bounds-checked descriptors: past nops reads 0)
    const __amdgpu_buffer_rsrc_t bid = bsrc(KA->id + op0, nops * 8u);
    const __amdgpu_buffer_rsrc_t bsc = bsrc(KA->score + op0, nops * 8u);
    const __amdgpu_buffer_rsrc_t bkd = bsrc(KA->kind + op0, nops);
    for (uint32_t c0 = 0; c0 < nops; c0 += 128) {
      int64_t idh[2], sch[2];
      uint32_t kh[2];
      bool vh[2], wide = false;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t l = c0 + 64u * h + lane;
        vh[h] = l < nops;
        if (c0 == 0) {
          idh[h] = pre_id[h];
          sch[h] = pre_sc[h];
          kh[h] = pre_kd[h];
        } else
        {
          idh[h] = bld64(bid, l * 8u);
          sch[h] = bld64(bsc, l * 8u);
          kh[h] = bld8(bkd, l);
        }
        wide |= vh[h] && (!fits32(idh[h]) || (kh[h] < 2 && !fits32(sch[h])));
      }
      if (ballot(wide)) return R_NEXT;  // a wide Id or Score: tier S
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (c0 + 64u * h >= nops) break;
        const uint32_t l = c0 + 64u * h + lane;
        uint32_t p;
        if (!r_resolve(L, idh[h], vh[h], np, p)) return R_NEXT;
        if (vh[h]) {
          KA->op_pl[op0 + l] = (uint8_t)p;
          if (kh[h] < 2) atomicAdd(reinterpret_cast<uint32_t*>(&L.u.r.nops[p & ~1u]), 1u << ((p & 1u) * 16u));
          pf_or(L, p, (kh[h] == 2 || kh[h] == 3) ? (Q_RMV | Q_DIRTY) : Q_DIRTY);
        }
      }
    }
    wave_lds_sync();
#pragma unroll
    for (int u = 0; u < RSL; ++u) {
      const uint32_t p = 64u * u + lane;
      if (p >= om.np && p < np) pid[u] = L.u.r.pid[p];
    }
    // new Removals rows; each player's slab need (old count + adds), kept in
    // nops; mtot = the whole pool's need, grow = the need of the players
    // with adds (the slabs that move in place)
    uint32_t nr = om.nr, mtot = 0, grow = 0;
#pragma unroll
    for (int u = 0; u < RSL; ++u) {
      const uint32_t p = 64u * u + lane;
      const bool act = p < np;
      const uint32_t q = act ? p : 0u;
      const uint32_t f = act ? L.pf[q] : 0u;
      const uint32_t row = L.prow[q];
      const bool newrow = act && (f & Q_RMV) && row == NONE16;
      const uint64_t m = ballot(newrow);
      if (newrow) L.prow[p] = (uint16_t)(nr + mbcnt(m));
      nr += (uint32_t)__builtin_popcountll(m);
      const uint32_t ocnt = act ? (L.u.r.oslab[q] >> 16) : 0u;
      const uint32_t adds = act ? (uint32_t)L.u.r.nops[q] : 0u;
      const uint32_t need = ocnt + adds;
      if (act) L.u.r.nops[p] = (uint16_t)(need > 0xFFFFu ? 0xFFFFu : need);
      uint32_t t1, t2;
      (void)wave_excl_scan_dpp(need, t1);
      (void)wave_excl_scan_dpp(adds ? need : 0u, t2);
      mtot += t1;
      grow += t2;
    }
    if (nr >= NONE16 || mtot > TRMV_SEG_MAX) return R_NEXT;  // over the per-key capacity
    // The new state's segments.  TIGHT: every slab laid out again, in player
    // order, in a new segment (a fresh key: its op range; a full rewrite: the
    // capacity scan's; in place: a relocation to the arena's top).  In place,
    // APPEND: the slabs of the players with adds move to the pool's top, the
    // rest stay; COMPACT: the pool is first compacted inside the segment.
    int lay = LAY_TIGHT;
    uint32_t mbase = 0;
    KeyMeta nm;
    KeyCap nc;
    if (fresh) {
      nm = trmv_new_meta(a, key);
      nc.p_cap = trmv_fresh_cap(a.slack != 0, 0, nops);
      nc.m_cap = trmv_fresh_cap(a.slack != 0, 1, nops);
      nc.r_cap = trmv_fresh_cap(a.slack != 0, 2, nops);
    } else if (!inpl) {
      nm = KA->new_s.meta[key];
      nc = KA->new_s.cap[key];
    } else {
      // (pool positions stay below 2^16: slab offsets are 16-bit)
      const uint32_t mcap = oc.m_cap < TRMV_SEG_MAX ? oc.m_cap : TRMV_SEG_MAX;
      const bool fitpr = (oc.flags & TRMV_CAP_VALID) && np <= oc.p_cap && nr <= oc.r_cap;
      if (fitpr && (uint32_t)oc.m_top + grow <= mcap) {
        lay = LAY_APPEND;
        mbase = oc.m_top;
      } else if (fitpr && om.nm + grow <= mcap) {
        lay = LAY_COMPACT;
        mbase = om.nm;
      }
      if (lay != LAY_TIGHT) {
        nm = om;
        nc = oc;
      } else {
        // a new segment at the top of the workgroup's sub-arena, with room
        // to grow in place
        const uint32_t pc = np + np / 2u + 8u, rc = nr + nr / 2u + 16u;
        const uint32_t mc0 = (uint32_t)KA->slack * mtot + 32u, mc = mc0 > TRMV_SEG_MAX ? TRMV_SEG_MAX : mc0;
        const uint32_t sub = 3u * (blockIdx.x % (uint32_t)TRMV_NSUB);
        unsigned long long b0 = 0, b1 = 0, b2 = 0;
        if (lane == 0) {
          b0 = atomicAdd(&KA->arena[sub], (unsigned long long)pc);
          b1 = atomicAdd(&KA->arena[sub + 1], (unsigned long long)mc);
          b2 = atomicAdd(&KA->arena[sub + 2], (unsigned long long)rc);
        }
        b0 = (unsigned long long)ufl64((int64_t)b0);
        b1 = (unsigned long long)ufl64((int64_t)b1);
        b2 = (unsigned long long)ufl64((int64_t)b2);
        if (b0 + pc > KA->arena_lim[sub] || b1 + mc > KA->arena_lim[sub + 1] || b2 + rc > KA->arena_lim[sub + 2])
        {
          RCOUNT(13, 1);
          return R_NEXT;  // the sub-arena is full: the batch is finished by a full rewrite
        }
        nm = om;
        nm.p_off = (uint32_t)b0;
        nm.m_off = (uint32_t)b1;
        nm.r_off = (uint32_t)b2;
        nc.p_cap = pc;
        nc.m_cap = mc;
        nc.r_cap = rc;
      }
    }
    nc.flags = TRMV_CAP_VALID;
    nc.m_top = (uint16_t)(lay == LAY_TIGHT ? mtot : mbase + grow);
    // (the capacity record is final here: written now, not held to P5; a
    // relocated key that hands on later leaves a record nothing reads -- the
    // finishing pass rewrites every key)
    if (lane == 0) KA->new_s.cap[key] = nc;
    RCOUNT(10 + lay, inpl ? 1 : 0);  // (diagnostic: in-place layouts, TIGHT = relocated)
    if (inpl && lane == 0) atomicAdd(&KA->lay_cnt[4u * (blockIdx.x % (uint32_t)TRMV_NSUB) + (uint32_t)lay], 1u);
    if (lay == LAY_TIGHT) {
      // every slab re-laid in player order: offset = the needs before it
      uint32_t run = 0;
#pragma unroll
      for (int u = 0; u < RSL; ++u) {
        const uint32_t p = 64u * u + lane;
        const bool act = p < np;
        const uint32_t need = act ? (uint32_t)L.u.r.nops[p] : 0u;
        const uint32_t ocnt = act ? (L.u.r.oslab[p] >> 16) : 0u;
        uint32_t tot;
        const uint32_t ex = wave_excl_scan_dpp(need, tot);
        if (act) L.nslab[p] = (run + ex) | (ocnt << 16);
        run += tot;
      }
    } else if (lay == LAY_COMPACT) {
#pragma unroll
      for (int u = 0; u < RSL; ++u) {  // (the compaction sets the players with elements)
        const uint32_t p = 64u * u + lane;
        if (p < np) L.nslab[p] = 0u;
        if (p < np) pf_or(L, p, Q_DIRTY);  // (slabs move: every record is rewritten)
      }
    } else {
#pragma unroll
      for (int u = 0; u < RSL; ++u) {
        const uint32_t p = 64u * u + lane;
        if (p < np) L.nslab[p] = L.u.r.oslab[p];
      }
    }
    wave_lds_sync();
    RPROF(1);

    // ---- P3. TIGHT: old slabs and old Removals rows -> the new segment,
    // position-parallel.  COMPACT: the pool compacted inside the segment
    // (slabs in old-offset order, so every element moves down: a window's
    // stores never reach a position not yet read).  Then, in place, the slabs
    // of the players with adds move to the pool's top.
    // (start map: u16 per pool position of the span, player + 1 at each slab
    // start, in the P1/P2 union up to nops, which with oslab stays)
    constexpr uint32_t SMAP = (uint32_t)(offsetof(decltype(L.u.r), nops) / 2);
    uint16_t* smap16 = reinterpret_cast<uint16_t*>(&L.u.r);
    const bool smap = span <= SMAP;
    const bool copy = lay == LAY_TIGHT || lay == LAY_COMPACT;
    if (copy && span && smap) {
      for (uint32_t i = lane; i < (span + 1) / 2; i += 64) reinterpret_cast<uint32_t*>(smap16)[i] = 0u;
      wave_lds_sync();
#pragma unroll
      for (int u = 0; u < RSL; ++u) {
        const uint32_t p = 64u * u + lane;
        const uint32_t sl = p < om.np ? L.u.r.oslab[p] : 0u;
        if (sl >> 16) smap16[sl & 0xFFFFu] = (uint16_t)(p + 1);
      }
      wave_lds_sync();
    }
    bool wide = false;
    if (copy && span) {
      const bool cmp = lay == LAY_COMPACT;
      int32_t prev = -1;
      uint32_t carry = 0;  // COMPACT: elements of the slabs that start before the window
      // (the old pool through bounds-checked descriptors over the key's span,
      // the destination's bases read once: the window's loads and stores issue
      // without a branch or a scalar wait each)
      const __amdgpu_buffer_rsrc_t qsc = bsrc(KA->old_s.m_score + om.m_off, span * 8u);
      const __amdgpu_buffer_rsrc_t qts = bsrc(KA->old_s.m_ts + om.m_off, span * 8u);
      const __amdgpu_buffer_rsrc_t qdc = bsrc(KA->old_s.m_dc + om.m_off, span);
      int64_t* const Nsc = KA->new_s.m_score + nm.m_off;
      int64_t* const Nts = KA->new_s.m_ts + nm.m_off;
      uint8_t* const Ndc = KA->new_s.m_dc + nm.m_off;
      // four windows of 64 positions per round: their loads go out together
      for (uint32_t g0 = 0; g0 < span; g0 += 256) {
        int64_t wsc[4], wts[4];
        uint32_t wdc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t q = g0 + 64u * i + lane;
          wsc[i] = bld64(qsc, q * 8u);  // (past the span: 0)
          wts[i] = bld64(qts, q * 8u);
          wdc[i] = bld8(qdc, q);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t q0 = g0 + 64u * i;
          if (q0 >= span) break;
          const uint32_t q = q0 + lane;
          const int64_t sc = wsc[i], ts = wts[i];
          const uint32_t dc = wdc[i];
          // the owner of a position is the player whose slab starts last at
          // or before it (slabs are in no particular order); starts come from
          // the start map, or for a span past its size from a sweep of every
          // player
          uint32_t st = 0;
          if (smap) {
            st = q < span ? (uint32_t)smap16[q] : 0u;
          } else {
            uint32_t* const mark = reinterpret_cast<uint32_t*>(smap16);  // (the map is unused here)
            mark[lane] = 0u;
            wave_lds_sync();
            for (uint32_t j0 = 0; j0 < om.np; j0 += 64) {
              const uint32_t j = j0 + lane;
              const uint32_t sl = j < om.np ? L.u.r.oslab[j] : 0u;
              const uint32_t off = sl & 0xFFFFu;
              if ((sl >> 16) && off >= q0 && off < q0 + 64) mark[off - q0] = j + 1;
            }
            wave_lds_sync();
            st = mark[lane];
          }
          if (cmp) {
            // a slab starting here moves to the elements of the slabs before it
            const uint32_t c = st ? (L.u.r.oslab[st - 1] >> 16) : 0u;
            uint32_t tot;
            const uint32_t ex = wave_excl_scan_dpp(c, tot);
            if (st) L.nslab[st - 1] = (carry + ex) | (c << 16);
            carry += tot;
            wave_lds_sync();
          }
          // (inclusive max-scan: the last start at or before the lane)
          uint32_t own = wave_incl_max_dpp(st ? ((lane + 1) << 16) | st : 0u);
          own &= 0xFFFFu;
          const int32_t o = own ? (int32_t)own - 1 : prev;
          prev = (int32_t)rl32((uint32_t)o, 63);
          if (q < span && o >= 0) {
            const uint32_t sl = L.u.r.oslab[o];
            const uint32_t off = sl & 0xFFFFu, cnt = sl >> 16;
            if (q < off + cnt) {
              wide |= !fits32(sc);
              const uint32_t dst = (L.nslab[o] & 0xFFFFu) + (q - off);
              if (!cmp || dst != q) {
                Nsc[dst] = sc;
                Nts[dst] = ts;
                Ndc[dst] = (uint8_t)dc;
              }
            }
          }
          wave_lds_sync();
        }
      }
    }
    if (lay == LAY_TIGHT && ballot(wide)) return R_NEXT;  // a wide Score in Masked (a new segment only): tier S
    if (lay == LAY_TIGHT) {
      // old Removals rows, 32 per round: the round's loads, then its stores
      const __amdgpu_buffer_rsrc_t qr = bsrc(KA->old_s.r_vc + (uint64_t)om.r_off * D, om.nr * (uint32_t)D * 8u);
      int64_t* const Nr = KA->new_s.r_vc + (uint64_t)nm.r_off * D;
      const uint32_t d = lane & 7u;
      for (uint32_t r0 = 0; r0 < om.nr; r0 += 32) {
        int64_t rv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t r = r0 + 8u * i + (lane >> 3);
          rv[i] = bld64(qr, (int)d < D ? (r * (uint32_t)D + d) * 8u : BOOB);  // (past nr: 0)
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t r = r0 + 8u * i + (lane >> 3);
          if (r < om.nr && (int)d < D) Nr[r * (uint32_t)D + d] = rv[i];
        }
      }
    } else {
      // in place: the slabs of the players with adds move to the pool's top
      // (the slab's appends follow in the chunks).  Their old elements are
      // numbered in one copy stream and copied position-parallel: an LDS map
      // marks where each mover's elements start in the stream.
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): a compacted slab is read back here
      uint16_t* const emap = reinterpret_cast<uint16_t*>(&L.u.r);  // (the start map's region, free here)
      const uint32_t eclr = om.nm < SMAP ? om.nm : SMAP;
      for (uint32_t i = lane; i < (eclr + 1) / 2; i += 64) reinterpret_cast<uint32_t*>(emap)[i] = 0u;
      wave_lds_sync();
      uint32_t run = mbase, ecnt = 0;
#pragma unroll
      for (int u = 0; u < RSL; ++u) {
        const uint32_t p = 64u * u + lane;
        const bool act = p < np;
        const uint32_t need = act ? (uint32_t)L.u.r.nops[p] : 0u;
        const uint32_t sl = act ? L.nslab[p] : 0u;
        const uint32_t ocnt = sl >> 16;
        const bool mv = need > ocnt;
        uint32_t t1, t2;
        const uint32_t ex = wave_excl_scan_dpp(mv ? need : 0u, t1);
        const uint32_t ey = wave_excl_scan_dpp(mv ? ocnt : 0u, t2);
        if (act) L.u.r.oslab[p] = sl;              // the source (a player that stays: the same)
        if (mv) {
          L.nslab[p] = (run + ex) | (ocnt << 16);  // the destination
          L.u.r.nops[p] = (uint16_t)(ecnt + ey);   // its first element's number in the stream
          if (ocnt && ecnt + ey < SMAP) emap[ecnt + ey] = (uint16_t)(p + 1);
        }
        run += t1;
        ecnt += t2;
      }
      wave_lds_sync();
      int64_t* const Psc = KA->new_s.m_score + nm.m_off;
      int64_t* const Pts = KA->new_s.m_ts + nm.m_off;
      uint8_t* const Pdc = KA->new_s.m_dc + nm.m_off;
      if (ecnt <= SMAP) {
        int32_t prev = -1;
        for (uint32_t k0 = 0; k0 < ecnt; k0 += 64) {
          const uint32_t k = k0 + lane;
          const uint32_t st = k < ecnt ? (uint32_t)emap[k] : 0u;
          const uint32_t own = wave_incl_max_dpp(st ? ((lane + 1) << 16) | st : 0u) & 0xFFFFu;
          const int32_t o = own ? (int32_t)own - 1 : prev;
          prev = (int32_t)rl32((uint32_t)o, 63);
          if (k < ecnt && o >= 0) {
            const uint32_t j = k - (uint32_t)L.u.r.nops[o];
            const uint32_t src = (L.u.r.oslab[o] & 0xFFFFu) + j, dst = (L.nslab[o] & 0xFFFFu) + j;
            const int64_t s1 = Psc[src], t1 = Pts[src];
            const uint8_t d1 = Pdc[src];
            Psc[dst] = s1;
            Pts[dst] = t1;
            Pdc[dst] = d1;
          }
        }
      } else {
        // (a stream past the map: one lane per mover)
#pragma unroll
        for (int u = 0; u < RSL; ++u) {
          const uint32_t p = 64u * u + lane;
          const bool act = p < np;
          const uint32_t dl = act ? L.nslab[p] : 0u;
          const bool mv = act && dl != L.u.r.oslab[p];
          if (mv) {
            const uint32_t src = L.u.r.oslab[p] & 0xFFFFu, dst = dl & 0xFFFFu;
            for (uint32_t j = 0; j < (dl >> 16); ++j) {
              const int64_t s1 = Psc[src + j], t1 = Pts[src + j];
              const uint8_t d1 = Pdc[src + j];
              Psc[dst + j] = s1;
              Pts[dst + j] = t1;
              Pdc[dst + j] = d1;
            }
          }
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the replays read these stores
    RPROF(2);

    // ---- chunks
    for (uint32_t c0 = 0; c0 < nops;) {
      // this chunk's lane-indexed LDS addresses are made from a lane the
      // compiler cannot see through, so they are computed here and not held
      // in VGPRs across the whole kernel
      uint32_t lane_o = lane;
      asm volatile("" : "+v"(lane_o));
      const uint32_t lane = lane_o;
      uint32_t n = nops - c0 < (uint32_t)RCH ? nops - c0 : (uint32_t)RCH;
      bool v = lane < n;
      [[maybe_unused]] const uint64_t gi = op0 + c0 + lane;
      // (bounds-checked loads over the key's ops: no branch around them)
      uint32_t kind, dc, p;
      int64_t id, sc, ts;
      {
        uint32_t kb, db, pb;
        int64_t ib, sb, tb;
        {
          const uint32_t o = c0 + lane;
          kb = bld8(bsrc(KA->kind + op0, nops), o);
          ib = bld64(bsrc(KA->id + op0, nops * 8u), o * 8u);
          sb = bld64(bsrc(KA->score + op0, nops * 8u), o * 8u);
          tb = bld64(bsrc(KA->ts + op0, nops * 8u), o * 8u);
          db = bld8(bsrc(KA->dc + op0, nops), o);
          pb = bld8(bsrc(KA->op_pl + op0, nops), o);
        }
        kind = v ? kb : 0u;
        id = v ? ib : 0;
        sc = v ? sb : 0;
        ts = v ? tb : 0;
        dc = v ? db : 0u;
        p = v ? pb : (uint32_t)RP;
      }
      bool isr = v && (kind == 2 || kind == 3);
      uint64_t rm = ballot(isr);
      if (__builtin_popcountll(rm) > RCHR) {  // cut before the chunk's 17th rmv
        uint64_t m = rm;
        for (int k = 0; k < RCHR; ++k) m &= m - 1;
        n = (uint32_t)__builtin_ctzll(m);
        v = lane < n;
        isr = isr && v;
        rm = ballot(isr);
      }
      const bool add = v && kind < 2;
      // the Removals-row entry a non-replayed add is checked against (:234),
      // loaded here and read after the sort: a player without a rmv in the
      // batch keeps its row unchanged through the batch's replays
      int64_t rte;
      {
        const uint32_t pq = add ? p : 0u;
        const uint32_t pfe = L.pf[pq];
        const bool need = add && (pfe & Q_ROWV) && !(pfe & Q_RMV);
        const uint32_t orwe = L.prow[pq];
        rte = bld64(bsrc(KA->new_s.r_vc + (uint64_t)nm.r_off * D, nr * (uint32_t)D * 8u),
                    need ? (orwe * (uint32_t)D + dc) * 8u : BOOB);
      }
      uint32_t err = 0;
      err |= (v && kind > 3) ? TRMV_ERR_KIND : 0u;
      err |= (add && (int)dc >= D) ? TRMV_ERR_DC : 0u;
      err |= (add && ts < 1) ? TRMV_ERR_TS : 0u;
      err |= (isr && (ts < 0 || ts >= KA->n_rmv_rows)) ? TRMV_ERR_ROW : 0u;
      if (ballot(err != 0)) {
        if (err) atomicOr(&KA->status[1], err);
        return R_REJECT;
      }
      if (ballot(v && (!fits32(id) || (add && !fits32(sc))))) return R_NEXT;  // wide values: tier S
      const uint32_t rk = mbcnt(rm), nrm = (uint32_t)__builtin_popcountll(rm);
      if (isr) L.u.c.crow[rk] = (uint32_t)ts;
      wave_lds_sync();
      {
        // (<= 16 rows: both halves' loads go out before either is stored)
        static_assert(RCHR <= 16, "two rounds of 8 clock rows");
        const uint32_t d = lane & 7u, ra = lane >> 3, rb = 8u + (lane >> 3);
        const bool va = ra < nrm && (int)d < D, vb = rb < nrm && (int)d < D;
        const uint32_t ca = L.u.c.crow[ra < nrm ? ra : 0u], cb = L.u.c.crow[rb < nrm ? rb : 0u];
        const int64_t* const rv = KA->rmv_vc;
        const int64_t xa = va ? rv[(uint64_t)ca * D + d] : 0;
        const int64_t xb = vb ? rv[(uint64_t)cb * D + d] : 0;
        err |= (xa < 0 || xb < 0) ? TRMV_ERR_VC : 0u;
        if (ra < nrm) L.u.c.vtab[ra][d] = xa;
        if (rb < nrm) L.u.c.vtab[rb][d] = xb;
      }
      if (ballot(err != 0)) {
        if (err) atomicOr(&KA->status[1], err);
        return R_REJECT;
      }
      // Elements that may already be in Masked[Id] (:240-246): every element
      // of dc in the key has Ts <= Vc[dc], so an add above the key's Vc[dc]
      // before it is new.  Exact when the chunk's adds of each dc have rising
      // Ts; otherwise every add of that dc after the first fall is a candidate.
      bool dupc;
      {
        const int64_t vcs = (int64_t)L.vc[add ? dc : (uint32_t)TRMV_DPAD];
        // per dc, the adds of the chunk as a lane mask (lane order = stream
        // order): a fall is an add whose previous add of its dc has a Ts as
        // large; every add of that dc from the first fall on is a candidate
        uint64_t md = 0;
#pragma unroll
        for (int d = 0; d < TRMV_DPAD; ++d) {
          const bool in = add && dc == (uint32_t)d;
          const uint64_t m = ballot(in);
          md = in ? m : md;
        }
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));  // (lane masks made here, not held across keys)
        const uint64_t below = ln ? (~0ull >> (64u - ln)) : 0ull;
        const uint64_t pm = md & below;
        const int prv = pm ? 63 - (int)__builtin_clzll(pm) : (int)ln;
        const int64_t pts = shfl64(ts, prv);
        const uint64_t fm = ballot(add && pm != 0 && pts >= ts);
        const bool taint = (fm & md & (below | (1ull << ln))) != 0;
        dupc = add && (ts <= vcs || taint);
      }
      wave_lds_sync();
      if (add) atomicMax(&L.vc[dc], (unsigned long long)ts);  // vc_update (:233)
      if (dupc) pf_or(L, p, Q_DUP);
      L.u.c.csc[lane] = sc;
      L.u.c.cts[lane] = ts;
      L.u.c.ckd[lane] = v ? (kind | (dc << 2) | ((dupc ? 1u : 0u) << 5) | (p << 8)) : ((uint32_t)RP << 8);
      L.u.c.cres[lane] = isr ? rk : 0u;
      wave_lds_sync();
      RPROF(3);

      // ---- P3c. ops in (player, stream) order: appends of players without
      // a rmv or duplicate candidate (op-parallel), replays of the others
      // (player, stream) order: a stable sort by the 8-bit player, lanes past
      // the chunk keyed 255 (they follow any real player 255: stable, and
      // told apart by their source lane)
      const uint32_t kvs = radix16_pass<4>(radix16_pass<0>(((v ? p : 255u) << 6) | lane));
      const uint32_t so = kvs & 63u;
      const bool sv = so < n;
      const uint32_t sp = sv ? (kvs >> 6) : (uint32_t)RP;
      const uint32_t lkvs = shfl32(kvs, lane ? (int)lane - 1 : 0);
      const bool start = sv && (lane == 0 || (lkvs >> 6) != sp);
      L.u.c.csrt[lane] = (uint8_t)so;
      const uint64_t ss = ballot(start);
      uint32_t ol = lane;
      asm volatile("" : "+v"(ol));  // (lane masks made here, not held across keys)
      const uint64_t incl = ol == 63 ? ~0ull : ((2ull << ol) - 1);
      const uint64_t sb = ss & incl;
      const uint32_t slo = sb ? 63u - (uint32_t)__builtin_clzll(sb) : 0u;
      const uint64_t above = ss & ~incl;
      const uint32_t shi = above ? (uint32_t)__builtin_ctzll(above) : n;
      const uint64_t segm = (shi >= 64 ? ~0ull : ((1ull << shi) - 1)) & ~((1ull << slo) - 1);
      const uint32_t skd = L.u.c.ckd[so];
      const int64_t ssc = L.u.c.csc[so], sts = L.u.c.cts[so];
      const uint32_t sdc = (skd >> 2) & 7u;
      const int64_t sid = shfl64(id, (int)so);
      L.u.c.cid[lane] = sid;
      const uint32_t pf0 = L.pf[sv ? sp : 0u];
      const bool walk = sv && (pf0 & (Q_RMV | Q_DUP));
      bool dom = false;
      uint32_t orw = NONE16;
      const int64_t rts = shfl64(rte, (int)so);
      if (sv && !walk && (pf0 & Q_ROWV)) {
        orw = L.prow[sp];
        dom = rts >= sts;
      }
      const bool app = sv && !walk && !dom;
      const uint64_t nd = ballot(app);
      if (app) {
        const uint32_t ns = L.nslab[sp];
        const uint32_t pos = (ns >> 16) + (uint32_t)__builtin_popcountll(nd & segm & ((1ull << ol) - 1));
        const uint64_t dst = (uint64_t)nm.m_off + (ns & 0xFFFFu) + pos;
        KA->new_s.m_score[dst] = ssc;
        KA->new_s.m_ts[dst] = sts;
        KA->new_s.m_dc[dst] = (uint8_t)sdc;
        L.u.c.cres[so] = pos << 16;
      }
      if (dom) {  // {rmv, {Id, Removals[Id]}} (:236-237)
        L.u.c.cres[so] = R_DOM;
        r_emit_row(a, L, op0, op0 + c0 + so, sid, KA->new_s.r_vc + ((uint64_t)nm.r_off + orw) * D);
      }
      wave_lds_sync();
      if (sv && !walk && lane + 1 == shi) {
        const uint32_t ns = L.nslab[sp];
        L.nslab[sp] = ns + ((uint32_t)__builtin_popcountll(nd & segm) << 16);
      }
      RPROF(4);
      const uint64_t wm = ballot(start && walk);
      if (start && walk) {
        const uint32_t k = mbcnt(wm);
        L.u.c.cwp[k] = (uint16_t)sp;
        L.u.c.cws[k] = (uint8_t)lane;
        L.u.c.cwe[k] = (uint8_t)shi;
      }
      wave_lds_sync();
      if (lane < (uint32_t)__builtin_popcountll(wm)) {
#define Msc KA->new_s.m_score
#define Mts KA->new_s.m_ts
#define Mdc KA->new_s.m_dc
        const uint32_t wp = L.u.c.cwp[lane], ws = L.u.c.cws[lane], we = L.u.c.cwe[lane];
        uint32_t f = L.pf[wp];
        const uint32_t ns = L.nslab[wp];
        const uint64_t base = (uint64_t)nm.m_off + (ns & 0xFFFFu);
        uint32_t cnt = ns >> 16;
        const uint32_t row = L.prow[wp];
        bool has_row = (f & Q_ROWV) != 0;
        Row8 R = (Row8)(0);
        const uint64_t rbase = ((uint64_t)nm.r_off + row) * D;
        {
          const int dn = KA->n_dc;  // (re-read here: no per-d masks held across the key)
#pragma unroll
          for (int d = 0; d < TRMV_DPAD; ++d) R[d] = (has_row && d < dn) ? KA->new_s.r_vc[rbase + d] : 0;
        }
        const int64_t wid = L.u.c.cid[ws];
        bool moved = false;
        for (uint32_t x = ws; x < we; ++x) {
          const uint32_t o = L.u.c.csrt[x];
          const uint32_t kd = L.u.c.ckd[o];
          const int64_t esc = L.u.c.csc[o], ets = L.u.c.cts[o];
          const uint32_t edc = (kd >> 2) & 7u;
          if ((kd & 3u) < 2) {  // add/4
            if (has_row && pick8(R, edc) >= ets) {  // dominated (:234-237)
              L.u.c.cres[o] = R_DOM;
              r_emit(a, L, op0, op0 + c0 + o, CCRDT_TRMV_RMV, wid, 0, 0, 0, &R);
              continue;
            }
            uint32_t pos = RNONE;
            if ((kd >> 5) & 1u) {  // set semantics: the element may be there
              // four elements per trip, their loads together (one round trip
              // per four elements, not one or three per element)
              for (uint32_t j0 = 0; j0 < cnt && pos == RNONE; j0 += 4) {
                int64_t t4[4], s4[4];
                uint32_t d4[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const uint32_t j = j0 + e < cnt ? j0 + e : j0;
                  t4[e] = Mts[base + j];
                  s4[e] = Msc[base + j];
                  d4[e] = Mdc[base + j];
                }
#pragma unroll
                for (int e = 3; e >= 0; --e)
                  if (j0 + e < cnt && t4[e] == ets && d4[e] == edc && s4[e] == esc) pos = j0 + e;
              }
            }
            if (pos == RNONE) {
              pos = cnt++;
              Msc[base + pos] = esc;
              Mts[base + pos] = ets;
              Mdc[base + pos] = (uint8_t)edc;
            }
            L.u.c.cres[o] = pos << 16;
          } else {  // rmv/3: merge_vc (:254, :369-386), filter Masked[Id] (:255-266)
            const uint32_t r = L.u.c.cres[o];
            const int64_t* V = L.u.c.vtab[r];  // (read from LDS where used: no second row in registers)
#pragma unroll
            for (int d = 0; d < TRMV_DPAD; ++d) {
              const int64_t v = V[d];
              R[d] = has_row ? (v > R[d] ? v : R[d]) : v;
            }
            has_row = true;
            uint32_t w = 0, bpos = 0, bdc = 0;
            int64_t bsc = 0, bts = 0;
            // the slab in blocks of 4 elements, each block's loads issued
            // together (the compaction only writes positions already read)
            constexpr int RFB = INPL ? 1 : RFBLK;  // (in place one: blocks of 2 spilled two VGPRs and ran slower)
            for (uint32_t j0 = 0; j0 < cnt; j0 += RFB) {
              int64_t s4[RFB], t4[RFB];
              uint32_t d4[RFB];
#pragma unroll
              for (int e = 0; e < RFB; ++e) {
                const uint32_t j = j0 + e < cnt ? j0 + e : j0;
                s4[e] = Msc[base + j];
                t4[e] = Mts[base + j];
                d4[e] = Mdc[base + j];
              }
#pragma unroll
              for (int e = 0; e < RFB; ++e) {
                const uint32_t j = j0 + e;
                if (j < cnt && t4[e] > V[d4[e]]) {
                  if (w != j) {
                    Msc[base + w] = s4[e];
                    Mts[base + w] = t4[e];
                    Mdc[base + w] = (uint8_t)d4[e];
                  }
                  if (w == 0 || gb_gt(s4[e], d4[e], t4[e], bsc, bdc, bts)) {
                    bsc = s4[e];
                    bdc = d4[e];
                    bts = t4[e];
                    bpos = w;
                  }
                  ++w;
                }
              }
            }
            moved |= w != cnt;
            cnt = w;
            L.u.c.rgs[r] = bsc;
            L.u.c.rgt[r] = bts;
            L.u.c.rgd[r] = (w ? 1u : 0u) | (bdc << 8) | (bpos << 16);
          }
        }
#undef Msc
#undef Mts
#undef Mdc
        L.nslab[wp] = (ns & 0xFFFFu) | (cnt << 16);
        if (has_row) {
          for (int d = 0, dn = KA->n_dc; d < dn; ++d) KA->new_s.r_vc[rbase + d] = pick8(R, (uint32_t)d);
          f |= Q_ROWV;
        }
        if (moved) f |= Q_WALK;
        L.pf[wp] = f;
      }
      wave_lds_sync();
      // vmcnt(0): the next chunk's replays read these stores.  After the last
      // chunk nothing reads them before P5, which waits there: the Observed
      // half runs while they drain.
      if (c0 + n < nops) __builtin_amdgcn_s_waitcnt(0x0F70);
      RPROF(5);

      // ---- P4. the Observed half, in stream order (recompute_observed/5
      // :301-334; rmv/3 :267-298)
      const uint32_t kdr = L.u.c.ckd[lane], crr = L.u.c.cres[lane];
      const uint32_t rl = lane < (uint32_t)RCHR ? lane : 0u;
      const int64_t rgs = L.u.c.rgs[rl], rgt = L.u.c.rgt[rl];
      const uint32_t rgdv = L.u.c.rgd[rl];
      const int64_t vt0 = L.u.c.vtab[lane >> 3][lane & 7], vt1 = L.u.c.vtab[8 + (lane >> 3)][lane & 7];
      // Per (player, run) segment of the sorted order -- a run = the adds
      // between two rmvs -- two segmented scans over its non-dominated adds:
      // gb_sets:largest (Score, DcId, Ts), which brings the player's largest
      // up to date at the run's end (catch_up), and the cmp/2-largest (Score,
      // Ts; the first of equals), which is Obs[Id] after the run whenever the
      // player is in Observed then and had a relevant add (the
      // state after a run of adds is the top K players by (largest Score,
      // Id), whatever the order of the run's adds across players).
      bool cu_ok;
      int64_t cu_s, cu_t, cm_s, cm_t;
      uint32_t cu_d, cu_pos, cu_run, cm_d, cm_pos;
      {
        const uint32_t scres = L.u.c.cres[so];
        const bool sadd = sv && (skd & 3u) < 2 && !(scres & R_DOM);
        const uint32_t srun = sv ? (uint32_t)__builtin_popcountll(rm & ((1ull << so) - 1)) : 0xFFu;
        const uint32_t seg = (sp << 8) | srun;
        const uint32_t pseg = shfl32(seg, lane ? (int)lane - 1 : 0);
        const bool hf0 = lane == 0 || pseg != seg;
        int32_t vs = (int32_t)ssc, ws = (int32_t)ssc;  // (Scores of adds fit 32 bits here)
        int64_t vt = sts, wt = sts;
        uint32_t vd = sdc | ((scres >> 16) << 8) | (sadd ? (1u << 30) : 0u) | (hf0 ? (1u << 31) : 0u);
        uint32_t wd = sdc | ((scres >> 16) << 8);
        seg_step<0x111, 0xf>(vs, vt, vd, ws, wt, wd);
        seg_step<0x112, 0xf>(vs, vt, vd, ws, wt, wd);
        seg_step<0x114, 0xf>(vs, vt, vd, ws, wt, wd);
        seg_step<0x118, 0xf>(vs, vt, vd, ws, wt, wd);
        seg_step<0x142, 0xa>(vs, vt, vd, ws, wt, wd);
        seg_step<0x143, 0xc>(vs, vt, vd, ws, wt, wd);
        const bool ok = (vd >> 30) & 1u;
        vd &= 0x3FFFFFFFu;
        const uint32_t nseg = shfl32(seg, lane < 63 ? (int)lane + 1 : (int)lane);
        const bool last = sv && (lane == 63 || nseg != seg);
        cu_ok = last && ok;
        cu_s = vs;
        cu_t = vt;
        cu_d = vd & 0xFFu;
        cu_pos = vd >> 8;
        cu_run = srun;
        cm_s = ws;
        cm_t = wt;
        cm_d = wd & 0xFFu;
        cm_pos = wd >> 8;
      }
      const uint32_t cu_p = sp;
      const int64_t cm_k = mkkey(cm_s, sid);
      wave_lds_sync();  // the chunk region is free from here on: merge staging
      // merge staging (K <= 128 entries), the candidate list, its histogram
      int64_t* stk = reinterpret_cast<int64_t*>(&L.u);
      uint32_t* stp = reinterpret_cast<uint32_t*>(stk + 128);
      int64_t* ck = reinterpret_cast<int64_t*>(stp + 128);
      uint32_t* hist = reinterpret_cast<uint32_t*>(ck + 64);
      static_assert(sizeof(L.u) >= 128 * 8 + 128 * 4 + 64 * 8 + 72 * 4, "merge staging in the chunk union");
      auto catch_up = [&](uint32_t run) {
        if (cu_ok && cu_run == run) {  // one lane per player
          const uint32_t f = L.pf[cu_p];
          const int64_t cs = L.msc[cu_p], ct = L.gts[cu_p];
          const uint32_t cd = L.gdc[cu_p];
          if (!(f & Q_HASM) || gb_gt(cu_s, cu_d, cu_t, cs, cd, ct)) {
            L.msc[cu_p] = (int32_t)cu_s;
            L.gts[cu_p] = cu_t;
            L.gdc[cu_p] = (uint8_t)cu_d;
            L.gpos[cu_p] = (uint16_t)cu_pos;
            if (!(f & Q_HASM)) pf_or(L, cu_p, Q_HASM);
          }
        }
        wave_lds_sync();
      };
      // A run's effect on Observed in one merge: the players whose run can
      // change it (an Observed player whose cmp-largest beats Obs[Id]; any
      // other whose key beats Min -- state at the run's start, where L.msc /
      // L.msc is exact), their old entries out, their cmp-largest in, the
      // smallest dropped to K.
      auto run_merge = [&](uint32_t run) {
        const bool seg_r = cu_ok && cu_run == run;
        uint32_t f = 0;
        int64_t ms = 0, ot = 0;
        if (seg_r) {
          f = L.pf[cu_p];
          ms = L.msc[cu_p];
          ot = L.ots[cu_p];  // (meaningful when in Observed)
        }
        const bool inobs = (f & Q_OBS) != 0;
        const int64_t mk = rl64(ob.key[0], 0);
        const bool rel = seg_r && (inobs ? (cm_s > ms || (cm_s == ms && cm_t > ot)) : (ob.n < K || cm_k > mk));
        const uint64_t relm = ballot(rel);
        RCOUNT(27, __builtin_popcountll(relm));
        RCOUNT(29, 1);
        if (!relm) return;
        RPROF(16);
        const uint32_t m = (uint32_t)__builtin_popcountll(relm);
        // The merge's ranks.  Up to three candidates: a ballot pair per
        // candidate.  More: no loop over the candidates -- their keys are
        // listed in LDS (upgraded players flagged Q_UPG); every kept entry and
        // every candidate counts the candidates below it from the list
        // (broadcast reads); a histogram of the kept entries by that count,
        // prefix-summed, gives each candidate the kept entries below it:
        // entry < candidate c  <=>  (candidates below the entry) <= (c's rank
        // among the candidates), keys being distinct.
        bool rem0, rem1;
        uint32_t cb0 = 0, cb1 = 0, cbc = 0, abc = 0;
        if (m <= MBALLOT) {
          // few candidates: one ballot pair per candidate
          rem0 = rem1 = false;
          for (uint64_t t = ballot(rel && inobs); t; t &= t - 1) {  // upgraded players' old entries
            const uint32_t xp = rl32(cu_p, (int)__builtin_ctzll(t));
            rem0 |= lane < ob.n && (ob.pl[0] & 0xFFFFu) == xp;
            rem1 |= 64u + lane < ob.n && (ob.pl[1] & 0xFFFFu) == xp;
          }
          const bool v0 = lane < ob.n && !rem0, v1 = 64u + lane < ob.n && !rem1;
          for (uint64_t t = relm; t; t &= t - 1) {
            const int x = (int)__builtin_ctzll(t);
            const int64_t kx = rl64(cm_k, x);
            cb0 += (v0 && kx < ob.key[0]) ? 1u : 0u;
            cb1 += (v1 && kx < ob.key[1]) ? 1u : 0u;
            cbc += (rel && kx < cm_k) ? 1u : 0u;
            const uint32_t ab = (uint32_t)__builtin_popcountll(ballot(v0 && ob.key[0] < kx)) +
                                (uint32_t)__builtin_popcountll(ballot(v1 && ob.key[1] < kx));
            abc = (int)lane == x ? ab : abc;
          }
        } else {
          if (rel) {
            ck[mbcnt(relm)] = cm_k;
            if (inobs) pf_or(L, cu_p, Q_UPG);
          }
          if (lane <= m) hist[lane] = 0u;
          wave_lds_sync();
          rem0 = lane < ob.n && (L.pf[lane < ob.n ? (ob.pl[0] & 0xFFFFu) : 0u] & Q_UPG);
          rem1 = 64u + lane < ob.n && (L.pf[64u + lane < ob.n ? (ob.pl[1] & 0xFFFFu) : 0u] & Q_UPG);
#pragma unroll 4
          for (uint32_t j = 0; j < m; ++j) {
            const int64_t kj = ck[j];
            cb0 += kj < ob.key[0] ? 1u : 0u;
            cb1 += kj < ob.key[1] ? 1u : 0u;
            cbc += kj < cm_k ? 1u : 0u;
          }
          const bool v0 = lane < ob.n && !rem0, v1 = 64u + lane < ob.n && !rem1;
          if (v0) atomicAdd(&hist[cb0], 1u);
          if (v1) atomicAdd(&hist[cb1], 1u);
          wave_lds_sync();
          const uint32_t hinc = wave_incl_scan_dpp(lane <= m ? hist[lane] : 0u);
          abc = shfl32(hinc, rel ? (int)cbc : (int)lane);
          if (rel && inobs) pf_and(L, cu_p, Q_UPG);
        }
        const bool v0 = lane < ob.n && !rem0, v1 = 64u + lane < ob.n && !rem1;
        RPROF(17);
        const uint64_t rm0 = ballot(rem0), rm1 = ballot(rem1);
        const uint32_t nrem = (uint32_t)__builtin_popcountll(rm0) + (uint32_t)__builtin_popcountll(rm1);
        const uint32_t T = ob.n - nrem + m, drop = T > K ? T - K : 0u;
        const int32_t i0 = (int32_t)(lane - mbcnt(rm0) + cb0) - (int32_t)drop;
        const int32_t i1 = (int32_t)(64u + lane - (uint32_t)__builtin_popcountll(rm0) - mbcnt(rm1) + cb1) - (int32_t)drop;
        const int32_t ic = (int32_t)(abc + cbc) - (int32_t)drop;
        if (v0) {
          if (i0 >= 0) {
            stk[i0] = ob.key[0];
            stp[i0] = ob.pl[0];
          } else {
            pf_and(L, ob.pl[0] & 0xFFFFu, Q_OBS);  // evicted (:325-331)
          }
        }
        if (v1) {
          if (i1 >= 0) {
            stk[i1] = ob.key[1];
            stp[i1] = ob.pl[1];
          } else {
            pf_and(L, ob.pl[1] & 0xFFFFu, Q_OBS);
          }
        }
        if (rel) {
          if (ic >= 0) {  // Obs[Id] := its cmp-largest (:303-331)
            stk[ic] = cm_k;
            stp[ic] = cu_p | (cm_d << 16);
            if (!inobs) pf_or(L, cu_p, Q_OBS);
            L.opos[cu_p] = (uint16_t)cm_pos;
            L.ots[cu_p] = cm_t;
          } else if (inobs) {
            pf_and(L, cu_p, Q_OBS);
          }
        }
        wave_lds_sync();
        RPROF(18);
        ob.n = T - drop;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const uint32_t i = 64u * t + lane;
          const uint32_t ii = i < ob.n ? i : 0u;
          const int64_t kk = stk[ii];
          const uint32_t pp = stp[ii];
          ob.key[t] = i < ob.n ? kk : INT64_MAX;
          ob.pl[t] = i < ob.n ? pp : RNONE;
        }
        wave_lds_sync();
      };
      RPROF(6);
      uint32_t nexs = ufl(L.nex);  // (the replays' extras are counted)
      for (uint32_t j = 0;;) {
        const uint64_t nxr = j < 64 ? rm & (~0ull << j) : 0ull;
        const uint32_t hi = nxr ? (uint32_t)__builtin_ctzll(nxr) : n;
        const uint32_t run = (uint32_t)__builtin_popcountll(rm & (hi >= 64 ? ~0ull : ((1ull << hi) - 1)));
        run_merge(run);
        RPROF(7);
        if (hi >= n) break;
        // ---- the rmv at hi: the run's largest elements, then Masked[Id]
        // after the filter (:255-266), then Observed (:267-298)
        catch_up(run);
        RPROF(20);
        const uint32_t kd = rl32(kdr, (int)hi);
        const uint32_t X = kd >> 8;
        const int64_t xots = L.ots[X];  // Obs[Id]'s Ts (kept per player; read early)
        const uint32_t r = rl32(crr, (int)hi);
        const uint32_t g = rl32(rgdv, (int)r);
        if (lane == 0) {
          if (g & 1u) {
            L.msc[X] = (int32_t)rl64(rgs, (int)r);
            L.gts[X] = rl64(rgt, (int)r);
            L.gdc[X] = (uint8_t)((g >> 8) & 7u);
            L.gpos[X] = (uint16_t)(g >> 16);
            pf_or(L, X, Q_HASM);
          } else {
            pf_and(L, X, Q_HASM);
          }
        }
        const uint32_t ix = ob_find(ob, X);
        if (ix != RNONE) {  // impacts Observed?  VcRmv[ObsDc] >= Obs[Id].Ts (:267-272)
          const uint32_t odc = ob_get32(ob.pl, ix) >> 16;
          const int vl = (int)(((r & 7u) << 3) | odc);
          const int64_t va = rl64(vt0, vl), vb = rl64(vt1, vl);
          if ((r < 8 ? va : vb) >= ufl64(xots)) {
            if (lane == 0) pf_and(L, X, Q_OBS);
            wave_lds_sync();
            int64_t wk = 0, gt = 0;
            uint32_t gd = 0, gp = 0;
            RCOUNT(31, 1);
            RPROF(21);
            const uint32_t w = r_promote(L, pid, np, wk, gt, gd, gp);
            RPROF(22);
            if (w == RNONE) {  // (:283-289): Obs[Id] dropped, Min of the rest
              ob_remove(ob, ix);
            } else {  // promote the largest (:290-295)
              ob_replace(ob, ix, wk, w | (gd << 16));
              // the extra effect's slot: P4 emits from one lane at a time, so
              // the key's count is a wave-uniform register here (nexs)
              const uint32_t pos = nexs++;
              if (lane == 0) {
                pf_or(L, w, Q_OBS | Q_DIRTY);
                L.opos[w] = (uint16_t)gp;
                L.ots[w] = gt;
                TrmvExtraRec e;
                e.op = (uint32_t)(op0 + c0 + hi);
                e.kind = CCRDT_TRMV_ADD;
                e.dc = (uint8_t)gd;
                e.pad = 0;
                e.id = key_id(wk);
                e.score = key_score(wk);
                e.ts = gt;
                KA->ex[op0 + pos] = e;
              }
            }
          }
        }
        wave_lds_sync();
        RPROF(8);
        j = hi + 1;
      }
      catch_up((uint32_t)__builtin_popcountll(rm & (n >= 64 ? ~0ull : ((1ull << n) - 1))));
      if (lane == 0) L.nex = nexs;
      wave_lds_sync();
      c0 += n;
    }

    // ---- P5. player records (a player's record sits at its index): TIGHT
    // writes every record, in place only the ones that change (a player with
    // ops, a moved slab, a change of Observed membership); positions of
    // slabs a replay compacted; the Observed order (obs_ord, read back by
    // the next batch's P1); Vc; meta; capacity.  (The re-find of a compacted
    // slab reads the last chunk's stores: they must have landed.)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint32_t i = 64u * t + lane;
      if (i < ob.n) L.u.f.odc[ob.pl[t] & 0xFFFFu] = (uint8_t)(ob.pl[t] >> 16);
    }
    wave_lds_sync();
    const bool all = lay == LAY_TIGHT;
    uint32_t mcount = 0;
#pragma unroll
    for (int u = 0; u < RSL; ++u) {
      const uint32_t p = 64u * u + lane;
      const bool act = p < np;
      const uint32_t f = act ? L.pf[p] : 0u;
      const bool ino = act && (f & Q_OBS);
      const bool was = (L.obs0[p >> 5] >> (p & 31u)) & 1u;
      const uint32_t ns = act ? L.nslab[p] : 0u, cnt = ns >> 16;
      mcount += cnt;
      if (act && (all || (f & Q_DIRTY) || ino != was)) {
        uint32_t opos = L.opos[p], gpos = L.gpos[p];
        if ((f & Q_WALK) && cnt) {  // a replay compacted the slab: find the elements again
          const int64_t msv = L.msc[p], otv = ino ? L.ots[p] : 0, gtv = L.gts[p];
          const uint32_t od = L.u.f.odc[p], gd = L.gdc[p];
          const uint64_t base = (uint64_t)nm.m_off + (ns & 0xFFFFu);
          for (uint32_t j = 0; j < cnt; ++j) {
            const int64_t s2 = KA->new_s.m_score[base + j], t2 = KA->new_s.m_ts[base + j];
            const uint32_t d2 = KA->new_s.m_dc[base + j];
            if (s2 == msv && t2 == otv && d2 == od) opos = j;
            if (s2 == msv && t2 == gtv && d2 == gd) gpos = j;
          }
        }
        const uint64_t pq = (uint64_t)nm.p_off + p;
        if (all || p >= om.np) KA->new_s.pl_id[pq] = pid[u];
        KA->new_s.pl_slab[pq] = ns;
        KA->new_s.pl_info[pq] = (ino ? (opos & 0xFFFFu) : NONE16) | ((uint32_t)L.prow[p] << 16);
        KA->new_s.pl_gb[pq] = (uint16_t)(cnt > 1 ? gpos : 0u);
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint32_t i = 64u * t + lane;
      if (i < ob.n) KA->obs_ord[(uint64_t)key * TRMV_ORD + i] = (uint16_t)(ob.pl[t] & 0xFFFFu);
    }
    uint32_t mtotal;
    (void)wave_excl_scan_dpp(mcount, mtotal);
    const uint32_t minp = rl32(ob.pl[0], 0) & 0xFFFFu;  // Min = entry 0
    if (lane < (uint32_t)D) KA->new_s.vc[(uint64_t)key * D + lane] = (int64_t)L.vc[lane];
    if (lane == 0) {
      KeyMeta out = nm;
      out.np = np;
      out.nm = mtotal;
      out.nr = nr;
      out.nobs = ob.n;
      out.minq = ob.n ? minp : NONE32;
      KA->new_s.meta[key] = out;
      if (!done) KA->ex_cnt[key] = L.nex;
    }
    RPROF(9);
  }
  return R_DONE;
}

}  // namespace

// (TRMV_R_WAVES: build knob, the minimum waves per SIMD the register
// allocation must allow; TRMV_R_WG: keys (waves) per workgroup)
#ifndef TRMV_R_WAVES
#define TRMV_R_WAVES 3
#endif
#ifndef TRMV_R_WG
#define TRMV_R_WG 1
#endif
template <bool INPL>
__global__ __launch_bounds__(64 * TRMV_R_WG, TRMV_R_WAVES) void trmv_resident_kernel(TrmvApplyArgs a) {
  __shared__ RLds lds[TRMV_R_WG];
  const uint32_t wv = ufl(threadIdx.x >> 6);
  RLds& L = lds[wv];
  const uint32_t n = a.n_list_dev ? *a.n_list_dev : a.n_list;
  for (uint32_t w = blockIdx.x * TRMV_R_WG + wv; w < n; w += gridDim.x * TRMV_R_WG) {
    const uint32_t key = ufl(KA->key_list ? KA->key_list[w] : w);
    const uint32_t w2 = w + gridDim.x * TRMV_R_WG;
    const uint32_t nkey = w2 < n ? ufl(KA->key_list ? KA->key_list[w2] : w2) : RNONE;
    const int r = trmv_resident_key<INPL>(a, key, nkey, L);
    if (r == R_NEXT && lane_id() == 0) {
      const uint32_t pos = atomicAdd(&KA->status[0], 1u);
      KA->ovf_list[pos] = key;
      // in place the key is as it was: its record carries over, and the pass
      // that finishes the batch applies its ops
      if (INPL) {
        KA->new_s.meta[key] = KA->old_s.meta[key];
        KA->new_s.cap[key] = KA->old_s.cap[key];
      }
    }
    wave_lds_sync();
  }
}

// Tier R over a fresh batch's hand-ons WHILE tier 0 runs (the overlapped
// hand-on): each wave claims the next index of tier 0's hand-on
// list, waits until tier 0 has published that entry (a.pub[idx] = key + 1),
// and applies the key; it leaves when tier 0 is finished (its done words sum
// to a.prod_waves) and the index is past tier 0's final count
// (*a.n_list_dev).  Every access the two kernels share is a device-scope
// atomic (the XCDs' L2s are not coherent with each other).  A wave that has
// waited ~2 s sets TRMV_ERR_STALL and leaves; the host then re-runs tier R
// over the whole list (a fresh key's tier R is idempotent).  Launched after
// tier 0 on a high-priority stream: if the two do not run side by side, this
// one runs after tier 0 and takes the list as the chain would.
__device__ __forceinline__ uint32_t r_atomic_read(uint32_t* p) { return atomicOr(p, 0u); }

__global__ __launch_bounds__(64, TRMV_R_WAVES) void trmv_resident_consume_kernel(TrmvApplyArgs a) {
  __shared__ RLds L;
  uint32_t* const cnt = const_cast<uint32_t*>(a.n_list_dev);
  const uint32_t lane = (uint32_t)lane_id();
  for (;;) {
    uint32_t idx = 0;
    if (lane == 0) idx = atomicAdd(a.claim, 1u);
    idx = ufl(idx);
    uint32_t key = RNONE;
    bool fin = idx >= a.n_pub;  // (n_pub covers every key: no hand-on lies past it)
    for (uint32_t spin = 0; !fin; ++spin) {
      uint32_t v = 0;
      if (lane == 0) v = r_atomic_read(&a.pub[idx]);
      v = ufl(v);
      if (v != 0u) {
        key = v - 1u;
        break;
      }
      // tier 0 finished?  (its waves' done words, one per lane; looking at
      // them only every fourth poll measured no faster for tier 0 and a
      // longer tail, profiles/r06/ab_overlap_waves.txt)
      const uint32_t dn = lane < (uint32_t)TRMV_NDONE ? r_atomic_read(&a.done[lane]) : 0u;
      uint32_t tot;
      (void)wave_excl_scan_dpp(dn, tot);
      if (ufl(tot) >= a.prod_waves) {  // its count is final, every entry below it published
        uint32_t c = 0;
        if (lane == 0) c = r_atomic_read(cnt);
        if (idx >= ufl(c)) {
          fin = true;
          break;
        }
        continue;  // (published before its wave's done add: the next read finds it)
      }
      if (spin >= a.spin_limit) {  // (~2 s: tier 0 is not running beside this kernel as it should)
        if (lane == 0) atomicOr(&a.status[1], TRMV_ERR_STALL);
        fin = true;
        break;
      }
      __builtin_amdgcn_s_sleep(127);  // (~4 us between polls)
    }
    if (fin) break;
    const int r = trmv_resident_key<false>(a, key, RNONE, L);
    if (r == R_NEXT && lane == 0) {
      const uint32_t pos = atomicAdd(&KA->status[0], 1u);
      KA->ovf_list[pos] = key;
    }
    wave_lds_sync();
  }
}

void trmv_resident_preload() {
  preload_kernels(trmv_resident_kernel<true>, trmv_resident_kernel<false>, trmv_resident_consume_kernel);
}

int trmv_launch_resident_consume(const TrmvApplyArgs& a, uint32_t waves, hipStream_t st) {
  if (waves == 0) return CCRDT_OK;
  hipLaunchKernelGGL(trmv_resident_consume_kernel, dim3(waves), dim3(64), 0, st, a);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

int trmv_launch_resident(const TrmvApplyArgs& a, uint64_t grid_keys, hipStream_t st) {
  if (grid_keys == 0) return CCRDT_OK;
  const uint64_t blocks = std::min<uint64_t>((grid_keys + TRMV_R_WG - 1) / TRMV_R_WG, 65536 / TRMV_R_WG);
  if (a.inplace)
    hipLaunchKernelGGL(trmv_resident_kernel<true>, dim3((unsigned)blocks), dim3(64 * TRMV_R_WG), 0, st, a);
  else
    hipLaunchKernelGGL(trmv_resident_kernel<false>, dim3((unsigned)blocks), dim3(64 * TRMV_R_WG), 0, st, a);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

}  // namespace ccrdt

#ifdef TRMV_PROF
extern "C" int ccrdt_debug_resident_prof(unsigned long long* out16, int reset) {  // (32 entries)
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_resident_prof), 32 * 8) != hipSuccess) return 4;
  if (reset) {
    unsigned long long z[32] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_resident_prof), z, sizeof(z)) != hipSuccess) return 4;
  }
  return 0;
}
#endif
