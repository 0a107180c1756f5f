// engine.hpp — the opaque ccrdt_engine of include/ccrdt.h.
#pragma once
#include <cstdint>
#include <map>

#include "common.hpp"
#include "trmv_kernels.hpp"

namespace ccrdt {

// One ping-pong side of GPU-resident topk_rmv state (trmv_kernels.hpp).
struct TrmvBufs {
  DevBuf meta, pl_id, pl_info, pl_slab, m_score, m_ts, m_dc, r_vc, vc;
};

// Per-type resident state of the simpler CCRDTs (types.hip).
struct TypeBufs {
  // average: sum[n_keys], num[n_keys]
  DevBuf avg_sum, avg_num;
  // topk: per-key open-addressing table (id, score, used flag), capacity per
  // key in tk_cap (power of two), plus the sorted value/1 output.
  DevBuf tk_id, tk_score, tk_cnt, tk_off, tk_scratch;
  uint64_t tk_slots = 0;
  // leaderboard: per-key register-resident board image (lb_* in types.hip)
  DevBuf lb_meta, lb_id, lb_score, lb_flag;
  DevBuf lb_meta2, lb_id2, lb_score2, lb_flag2;
  uint64_t lb_cap_total = 0;
  // wordcount / worddocumentcount: global hash table of words
  DevBuf wc_hash, wc_off, wc_len, wc_cnt, wc_bytes, wc_used, wc_status;
  uint64_t wc_slots = 0, wc_byte_cap = 0;
  // scratch
  DevBuf scratch0, scratch1, scratch2, scratch3;
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
  float last_kernel_ms = 0.f;
  void* h_status = nullptr;  // pinned, 64 bytes
  bool fresh = true;         // every key == new(k); resident arrays ignored

  // topk_rmv
  ccrdt::TrmvBufs trmv[2];
  int cur = 0;
  ccrdt::DevBuf partials, ex_cnt, ex, ex_vc, ex_key_ptr, ovf_a, ovf_b, status;
  uint64_t last_n_ops = 0;
  std::map<int, uint32_t> trmv_overflow_keys;  // per tier / slot class, last apply
  std::map<int, float> trmv_tier_ms;
  // host-API staging
  ccrdt::DevBuf st_kp, st_kind, st_id, st_score, st_dc, st_ts, st_rvc, st_out_kind, st_out_vc;

  // other types
  ccrdt::TypeBufs tb;

  ccrdt::TrmvSide trmv_side(int s) const;
  void release_all();
  int init_type();
  int reset_type();
  void release_types();
  int clone_from(const ccrdt_engine& src);
};

namespace ccrdt {
using Engine = ccrdt_engine;
}
