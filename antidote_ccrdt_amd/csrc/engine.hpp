// engine.hpp — the opaque ccrdt_engine of include/ccrdt.h.
#pragma once
#include <cstdint>
#include <map>

#include "common.hpp"
#include "trmv_kernels.hpp"

namespace ccrdt {

// One ping-pong side of GPU-resident topk_rmv state (trmv_kernels.hpp): the
// meta + cap arrays of meta index s and the data arrays of data index s
// (the two indices move apart when tier R updates keys in place).
struct TrmvBufs {
  DevBuf meta, cap, pl_id, pl_info, pl_slab, pl_gb, m_score, m_ts, m_dc, r_vc, vc;
};

// Per-type resident state of the other CCRDTs (types_kernels.hip); [2] =
// ping-pong sides, tcur = side holding the current state.
struct TypeBufs {
  int tcur = 0;
  // average: sum[n_keys], num[n_keys]
  DevBuf avg_sum[2], avg_num[2];
  // topk: per key a segment (off[k], cnt[k]) of (id, score) entries
  DevBuf tk_off[2], tk_cnt[2], tk_id[2], tk_score[2];
  // leaderboard: per board LbMeta + a segment of (id, score, status)
  DevBuf lb_meta[2], lb_id[2], lb_score[2], lb_st[2];
  // wordcount / worddocumentcount: word table (open addressing on the
  // 64-bit word hash) + byte arena of the words
  DevBuf t_tab[2], t_meta[2], t_cnt[2];  // word table: WcSlot[t_slots], WcMeta[t_slots], counts[t_slots]
  uint64_t t_slots[2] = {0, 0};
  DevBuf arena, arena_top, d_hash, chk;  // chk: the insert kernel's check list (WcChk)
  // the dedupe table (d_hash): slots cleared since its last reset, the last
  // launch's document tags end there (WcArgs::d_base)
  uint64_t d_clean = 0, d_base = 0;
  DevBuf dl, dl_pre, dl_cur;  // worddocumentcount's document lists (WcArgs::dl)
  DevBuf cl, cl_bcnt, fl, bkt, cl_small;  // the count list (WcArgs::cl) and its bucket sums
  uint64_t arena_cap = 0;
  uint64_t wc_seed = 0;   // word-hash seed; a batch that meets a collision is re-run once with a new one
  int64_t wc_checks = 0;  // the last batch's check-list records (-1: verified token by token)
  // scratch shared by the types
  DevBuf caps, part, ovf_a, ovf_b, status, ex_cnt, ex, kp, stage[8];
  // HBM class of topk / leaderboard (keys beyond the LDS classes)
  DevBuf hb_off, hb_cap, hb_a, hb_b, hb_c, hb_d;
};

}  // namespace ccrdt

struct ccrdt_engine {
  int type = 0;
  int64_t k = 0;
  int64_t n_keys = 0;
  int n_dc = 0;
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t evk0 = nullptr, evk1 = nullptr;  // around the main apply kernel
  hipEvent_t evt[8] = {};                      // topk_rmv tier boundaries
  bool create_tier_events() {
    for (hipEvent_t& v : evt)
      if (hipEventCreate(&v) != hipSuccess) return false;
    return true;
  }
  void destroy_tier_events() {
    for (hipEvent_t& v : evt)
      if (v) (void)hipEventDestroy(v);
  }
  float last_kernel_ms = 0.f;
  void* h_status = nullptr;  // pinned, 256 bytes
  bool fresh = true;         // every key == new(k); resident arrays ignored

  // topk_rmv
  ccrdt::TrmvBufs trmv[2];
  int cur = 0;   // data arrays holding the current state
  int mcur = 0;  // meta + cap arrays holding the current state
  // In-place updates (tier R): possible once a full rewrite laid every key
  // out with room to grow (inplace_ready); relocations take space from the
  // data arrays' arena (device bump counters, capacities in elements).
  bool inplace_ready = false;
  bool arena_pending = false;  // arena_sub not yet copied to the device (the next in-place pass does it)
  bool fresh_room = false;     // fresh batches laid out with room to grow in place (ccrdt_trmv_set_fresh_room)
  uint64_t arena_cap[3] = {0, 0, 0};
  uint64_t arena_sub[2][ccrdt::TRMV_NSUB][3] = {};  // each sub-arena's start and end (host copy)
  uint64_t arena_used[3] = {0, 0, 0};               // elements the in-place passes took since the rewrite
  uint64_t arena_rate[3] = {0, 0, 0};               // the most one in-place pass took (sizes the next rewrite's room)
  void* h_arena = nullptr;                          // pinned: the sub-arena counters read back
  ccrdt::DevBuf arena, obs_ord, key_done;
  ccrdt::DevBuf partials, ex_cnt, ex, ex_vc, ex_key_ptr, status, op_pl;
  ccrdt::DevBuf tier_ovf[5];    // keys each topk_rmv tier handed on (last batch)
  // the overlapped hand-on of fresh batches: tier R on a second stream beside
  // tier 0 (created on first use); first_list = the likely hand-ons, taken
  // first; ovl = [tier 0 waves finished, consumer claim counter, first_list count]
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_ovl = nullptr;
  ccrdt::DevBuf first_list, ovl;
  ccrdt::DevBuf hbm_scratch;    // tier 4's per-wave working sets
  int trmv_first_tier = 0;
  uint64_t last_n_ops = 0;
  uint64_t trmv_tot[2][3] = {};  // per side: bound on (players, pool, rows) held
  std::map<int, uint32_t> trmv_overflow_keys;  // per tier / slot class, last apply
  std::map<int, float> trmv_tier_ms;
  // host-API staging
  ccrdt::DevBuf st_kp, st_kind, st_id, st_score, st_dc, st_ts, st_rvc, st_out_kind, st_out_vc;
  void* pin[16] = {};          // pinned upload slots (staging.cpp), allocated on first use
  void* pin_base = nullptr;    // pinned chunk bases of the narrow column uploads (staging.cpp)
  hipEvent_t pin_bev[3] = {};  // each base region's last DMA
  ccrdt::DevBuf st_n32[3], st_nbase[3];  // narrow upload scratch: int32 column, chunk bases
  hipEvent_t pin_ev[16] = {};  // each slot's last DMA
  int pin_n = 0;

  // other types
  ccrdt::TypeBufs tb;

  ccrdt::TrmvSide trmv_side(int ms, int ds) const;
  ccrdt::TrmvSide trmv_cur() const { return trmv_side(mcur, cur); }
  void release_all();
  int init_type();
  int reset_type();
  void release_types();
  int clone_from(const ccrdt_engine& src);
};

namespace ccrdt {
using Engine = ccrdt_engine;
// Host -> device copy of pageable caller memory through the engine's pinned
// staging slots, parallel host threads (staging.cpp); queued on E.stream.
void host_fill(void* dst, int v, uint64_t bytes);
int h2d_staged(Engine& E, void* dst, const void* src, uint64_t bytes);
// An int64 column through the staging slots as int32 (staging.cpp).
int h2d_staged_i64(Engine& E, int64_t* dst, const int64_t* src, uint64_t n, const uint8_t* kind,
                   const uint8_t* kind_dev, int slot, DevBuf& scratch, DevBuf& dbase, bool based = false);
int h2d_trmv_ops(Engine& E, uint64_t n, const uint8_t* kind, const int64_t* id, const int64_t* score,
                 const uint8_t* dc, const int64_t* ts, uint8_t* kind_d, uint8_t* dc_d, int64_t* id_d,
                 int64_t* score_d, int64_t* ts_d, DevBuf& scratch, DevBuf& dbase);
void stage_release(Engine& E);
}
