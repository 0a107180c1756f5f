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

// One ping-pong side of the resident state.
struct TrmvSide {
  KeyMeta* meta;
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
};

// The kernel's TrmvApplyArgs re-read at the point of use (kernarg_as,
// common.hpp): valid in kernels whose FIRST parameter is the TrmvApplyArgs.
__device__ __forceinline__ const __attribute__((address_space(4))) TrmvApplyArgs* trmv_kargs() {
  return kernarg_as<TrmvApplyArgs>();
}

// New-side metadata of key k before its tier writes it.  A fresh batch's
// segments hold exactly the key's ops (capacity = ops for players, pool and
// rows), so their offsets are the key's op offset and the capacity scan is
// skipped; otherwise the scan laid them out in new_s.meta.
__device__ __forceinline__ KeyMeta trmv_new_meta(const TrmvApplyArgs& a, uint64_t k) {
  if (a.fresh) {
    KeyMeta m;
    m.p_off = m.m_off = m.r_off = (uint32_t)a.key_ptr[k];
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
