// trmv_kernels.hpp — device layout of GPU-resident topk_rmv state and the
// kernel argument blocks shared by the trmv kernels and engine.cpp.
//
// Per key, the reference state {Observed, Masked, Removals, Vc, Min, Size}
// (src/antidote_ccrdt_topk_rmv.erl:67-74) is held in HBM as variable-length
// segments addressed through one 32-byte KeyMeta:
//   players  pl_id[i64]   one per distinct Id the key has seen (Masked or
//                         Removals entry; players are never dropped)
//            pl_info[u32] obs (low 16): index of Obs[Id] inside the player's
//                         Masked slab, 0xFFFF = Id not in Observed;
//                         row (high 16): Removals row, 0xFFFF = none
//            pl_slab[u32] Masked slab of the player inside the key's pool
//                         segment: offset (low 16) | element count (high 16)
//            pl_gb[u16]   gb_sets:largest(Masked[Id]) as an index into the
//                         slab (term order (Score, DcId, Ts) inside one Id;
//                         the promotion candidate of rmv/3, :279,291); only
//                         meaningful for slabs of 2+ elements (readers take 0
//                         otherwise, whatever is stored)
//   pool     m_score[i64], m_ts[i64], m_dc[u8]   the Masked elements, one
//                         slab per player (slabs may leave holes)
//   rows     r_vc[n_dc x i64]   Removals[Id] (0 = DC absent)
//   vc       vc[n_dc x i64]     replica Vc (0 = DC absent)
//   meta     segment offsets, counts, |Observed| and Min (a player index)
// Observed is implicit (Observed ⊆ Masked) and Min is always
// Obs[minq] (Min == min_observed(Observed) is an invariant of the reference).
//
// Segments and sides.  The data arrays (players, pool, rows, vc) form ARENAS:
// a key's segments lie anywhere in them, and a KeyCap per key records how
// much each segment holds.  meta and cap ping-pong every batch; the data
// arrays ping-pong only on a full rewrite (a fresh batch, a batch that lays
// every key out again with the capacity scan, or a compaction).  In between,
// tier R updates resident keys IN PLACE (TrmvApplyArgs::inplace): a batch
// reads and writes only the records, slabs and rows of the players its ops
// name, plus every key's meta / Vc / Observed order; a player whose slab must
// grow moves it to the pool's top (m_top), a pool that runs out is compacted
// inside its segment, and a key whose segment is too small moves to the
// arena's top (a device bump allocator).  Keys that cannot be updated in
// place are handed on and the batch is finished by a full rewrite.
#pragma once
#include <cstdint>

namespace ccrdt {

constexpr uint32_t NONE16 = 0xFFFFu;
constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr int TRMV_DPAD = 8;             // lanes per removal row (n_dc <= 8)
constexpr uint32_t TRMV_SEG_MAX = 0xFFFFu;  // pool elements addressable per key

struct alignas(32) KeyMeta {
  uint32_t p_off, m_off, r_off;  // segment starts (players / pool elements / rows)
  uint32_t np;                   // players
  uint32_t nm;                   // Masked elements (sum of slab counts)
  uint32_t nr;                   // Removals rows
  uint32_t nobs;                 // |Observed|
  uint32_t minq;                 // player index of Min, NONE32 = nil
};
static_assert(sizeof(KeyMeta) == 32, "KeyMeta is one 32-byte record");

// The capacity of a key's segments (ping-pongs with meta).  Written by the
// capacity scan (flags 0) and by tier R (TRMV_CAP_VALID); tier R's in-place
// path reads it and relocates a key whose record is not VALID.
struct alignas(16) KeyCap {
  uint32_t p_cap, m_cap, r_cap;  // players / pool positions / Removals rows the segments hold
  uint16_t m_top;                // pool positions in use: every slab lies in [0, m_top)
  uint16_t flags;                // TRMV_CAP_VALID
};
static_assert(sizeof(KeyCap) == 16, "KeyCap is one 16-byte record");
constexpr uint16_t TRMV_CAP_VALID = 1u;
constexpr int TRMV_ORD = 128;  // Observed-order slots per key (tier R's class: K <= 128)
// The arena's free space is cut into sub-arenas, one bump counter each (a
// workgroup allocates from sub-arena blockIdx % TRMV_NSUB): one counter for
// every relocation of a batch serialised hundreds of thousands of atomics.
constexpr int TRMV_NSUB = 64;

// One side of the resident state: meta + cap of one ping-pong index, the
// data arrays of one (possibly the same) data index.
struct TrmvSide {
  KeyMeta* meta;
  KeyCap* cap;
  int64_t* pl_id;
  uint32_t* pl_info;
  uint32_t* pl_slab;
  uint16_t* pl_gb;
  int64_t* m_score;
  int64_t* m_ts;
  uint8_t* m_dc;
  int64_t* r_vc;
  int64_t* vc;
};

// Extra effect record; a key's records sit inside the key's op range, in any
// order (the host orders them by `op`).
struct alignas(16) TrmvExtraRec {
  uint32_t op;    // global op index
  uint8_t kind;   // CCRDT_TRMV_ADD or CCRDT_TRMV_RMV
  uint8_t dc;
  uint16_t pad;
  int64_t id;
  int64_t score;
  int64_t ts;
};

struct TrmvApplyArgs {
  int64_t n_keys;
  int32_t n_dc;
  uint32_t k;  // Size (clamped)
  // ops (device)
  const uint64_t* key_ptr;
  const uint8_t* kind;
  const int64_t* id;
  const int64_t* score;
  const uint8_t* dc;
  const int64_t* ts;
  const int64_t* rmv_vc;
  int64_t n_rmv_rows;
  // state
  TrmvSide old_s;  // ignored when fresh
  TrmvSide new_s;  // new_s.meta offsets precomputed by the scan
  int32_t fresh;
  // extra effects
  uint32_t* ex_cnt;       // [n_keys]
  TrmvExtraRec* ex;       // [n_ops]
  int64_t* ex_vc;         // [n_ops * n_dc]
  // work list (nullptr = all keys) and overflow list
  const uint32_t* key_list;
  uint32_t n_list;
  const uint32_t* n_list_dev;  // non-null: the list length lives on the device
                               // (the previous tier's overflow count)
  uint32_t* ovf_list;
  uint32_t* status;  // [0] overflow count, [1] error flags
  uint8_t* op_pl;    // [n_ops] tier R scratch: each op's player index in its key
  // in-place updates (tier R) and the passes that finish them
  int32_t inplace;                  // old_s and new_s share the data arrays; keys are updated in place
  unsigned long long* arena;            // [TRMV_NSUB][3] next free player / pool / row position of each sub-arena
  const unsigned long long* arena_lim;  // [TRMV_NSUB][3] each sub-arena's end
  uint32_t* lay_cnt;                    // [TRMV_NSUB][4] in-place keys by layout: TIGHT (relocated), APPEND, COMPACT
  uint16_t* obs_ord;                // [n_keys * TRMV_ORD] each key's Observed players, ascending (tier R)
  const uint8_t* key_done;          // non-null: 1 = the key's ops were applied already (it is rewritten, no ops)
  const uint32_t* verr;             // in place: the batch validation's error flags (non-zero: nothing is written)
  int32_t slack;                    // > 0: segments laid out with room for in-place growth, the pool's
                                    // capacity slack x (its elements + the batch's ops) + 32
  // The overlapped hand-on of a fresh batch: tier 0 takes the
  // keys of first_list (count *n_first: the keys with more than first_thresh
  // ops, the likely hand-ons) before every other key in key order (those with
  // more than first_thresh ops skipped), publishes each hand-on also as key + 1
  // in pub[pos] (pos < n_pub; 0 = not yet) with a device-scope atomic, and
  // each of its waves adds one to done[wave % TRMV_NDONE] when it is finished
  // (TRMV_NDONE words: 131k adds on one word, polled by the consumers, had
  // made tier 0 1.8x slower).  Tier R, on a second stream, takes the keys as
  // they are published (claim: the consumers' next list index) until the done
  // words sum to prod_waves and its index is past tier 0's final count.
  const uint32_t* first_list;
  const uint32_t* n_first;
  uint32_t first_thresh;
  uint32_t n_pub;
  uint32_t prod_waves;              // tier 0's waves (what the done words sum to when it is finished)
  uint32_t spin_limit;              // tier R's polls (~4 us each) before it gives up waiting for tier 0
  uint32_t* pub;
  uint32_t* done;
  uint32_t* claim;
};
constexpr int TRMV_NDONE = 64;
// (tier R's consumer gave up waiting for tier 0: the host re-runs tier R
// over the whole hand-on list)
constexpr uint32_t TRMV_ERR_STALL = 1u << 30;

// The ops of key k in this pass (a key whose ops an earlier pass applied has
// none: it is only rewritten).
__device__ __forceinline__ uint32_t trmv_key_nops(const TrmvApplyArgs& a, uint64_t k, uint64_t op0) {
  return (a.key_done && a.key_done[k]) ? 0u : (uint32_t)(a.key_ptr[k + 1] - op0);
}

// The kernel's TrmvApplyArgs re-read at the point of use (kernarg_as,
// common.hpp): valid in kernels whose FIRST parameter is the TrmvApplyArgs.
__device__ __forceinline__ const __attribute__((address_space(4))) TrmvApplyArgs* trmv_kargs() {
  return kernarg_as<TrmvApplyArgs>();
}

// The fresh layout (no capacity scan): array x's segment of key k (x = 0
// players, 1 pool, 2 rows) starts at F_x * o + C_x * k, o = key_ptr[k] (the
// key's op offset), and holds F_x * ops + C_x.  With a.slack (later batches
// may grow the keys in place) F = 3 / 6 / 1, C = 16 / 32 / 8: room for the
// players, slabs and rows of the next batches without a relocation, and the
// first resident batch runs in place; without, exactly the ops (F = 1, C = 0).
__host__ __device__ __forceinline__ uint64_t trmv_fresh_off(bool room, int x, uint64_t k, uint64_t o) {
  return room ? (x == 0 ? 3 * o + 16 * k : (x == 1 ? 6 * o + 32 * k : o + 8 * k)) : o;
}
__host__ __device__ __forceinline__ uint32_t trmv_fresh_cap(bool room, int x, uint32_t nops) {
  return room ? (x == 0 ? 3 * nops + 16 : (x == 1 ? 6 * nops + 32 : nops + 8)) : nops;
}

// New-side metadata of key k before its tier writes it: a fresh batch's from
// the fresh layout, otherwise what the capacity scan laid out in new_s.meta.
__device__ __forceinline__ KeyMeta trmv_new_meta(const TrmvApplyArgs& a, uint64_t k) {
  if (a.fresh) {
    KeyMeta m;
    const uint64_t o = a.key_ptr[k];
    m.p_off = (uint32_t)trmv_fresh_off(a.slack != 0, 0, k, o);
    m.m_off = (uint32_t)trmv_fresh_off(a.slack != 0, 1, k, o);
    m.r_off = (uint32_t)trmv_fresh_off(a.slack != 0, 2, k, o);
    m.np = m.nm = m.nr = m.nobs = 0;
    m.minq = NONE32;
    return m;
  }
  return a.new_s.meta[k];
}

enum : uint32_t {
  TRMV_ERR_KIND = 1u,
  TRMV_ERR_DC = 2u,
  TRMV_ERR_TS = 4u,
  TRMV_ERR_ROW = 8u,
  TRMV_ERR_VC = 16u,
};

struct TrmvDownArgs {
  int64_t n;
  int32_t n_dc;
  uint32_t k;
  const uint64_t* key;
  const uint8_t* op;
  const int64_t* id;
  const int64_t* score;
  const uint8_t* dc;
  const int64_t* ts;
  uint8_t* out_kind;
  int64_t* out_vc;
  TrmvSide s;
  int32_t fresh;
};

}  // namespace ccrdt
