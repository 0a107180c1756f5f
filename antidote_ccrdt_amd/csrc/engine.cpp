// engine.cpp — libccrdt engine runtime + the topk_rmv C-ABI (include/ccrdt.h).
//
// The engine keeps every key's CCRDT state resident in HBM and applies a
// batch of effect ops (update/2 of the reference behaviour,
// src/antidote_ccrdt.erl:50) with one pass of hand-written gfx950 kernels.
// Host code here only sizes buffers, launches, and converts between the
// canonical state image and the device layout.  There is no CPU compute path:
// if the HIP runtime or the device is missing, calls fail with CCRDT_EDEVICE.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "common.hpp"
#include "engine.hpp"
#include "trmv_kernels.hpp"

namespace ccrdt {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

int trmv_launch_scan(const TrmvApplyArgs& a, uint64_t* partials, uint32_t* key_rmv, hipStream_t st);
void trmv_kernels_preload();
void trmv_wave_preload();
void trmv_resident_preload();
void trmv_steady_preload();
int trmv_launch_validate(const TrmvApplyArgs& a, uint64_t n_ops, uint32_t* err, unsigned long long* scratch,
                         hipStream_t st);
int trmv_launch_mark_done(uint8_t* done, uint64_t n_keys, const uint32_t* list, uint32_t n_list, const uint32_t* n_dev,
                          uint32_t* ex_cnt, hipStream_t st);
int trmv_launch_keep(const TrmvApplyArgs& a, uint32_t grid, hipStream_t st);
int trmv_launch_downstream(const TrmvDownArgs& a, hipStream_t st);
int trmv_launch_wave(const TrmvApplyArgs& a, uint64_t grid_keys, hipStream_t st);
int trmv_launch_first_list(const uint64_t* key_ptr, uint64_t n_keys, uint32_t thresh, uint32_t* list,
                           uint32_t* count, hipStream_t st);
uint32_t trmv_wave_waves(uint64_t grid_keys);
int trmv_launch_resident_consume(const TrmvApplyArgs& a, uint32_t waves, hipStream_t st);
int trmv_launch_steady(const TrmvApplyArgs& a, int cls, uint64_t grid_keys, hipStream_t st);
int trmv_launch_resident(const TrmvApplyArgs& a, uint64_t grid_keys, hipStream_t st);
int trmv_launch_steady_hbm(const TrmvApplyArgs& a, uint32_t waves, void* scratch, hipStream_t st);
uint64_t trmv_steady_hbm_bytes(bool ranked);
uint32_t trmv_steady_hbm_players();
int trmv_launch_replica_vc(const int64_t* vc, uint64_t n_keys, int n_dc, int64_t* out,
                           hipStream_t st);
int trmv_launch_pack_extras(const uint64_t* key_ptr, const uint32_t* ex_cnt, const TrmvExtraRec* ex,
                            const int64_t* ex_vc, uint64_t n_keys, int n_dc, int64_t* rows,
                            int64_t cap, uint32_t* count, hipStream_t st);
int trmv_launch_exchange_pack(const int64_t* vc, const uint64_t* key_ptr, const uint32_t* ex_cnt,
                              const TrmvExtraRec* ex, const int64_t* ex_vc, uint64_t n_keys, int n_dc, int64_t* pack,
                              int64_t cap, const int64_t* op_map, int64_t n_map, uint32_t host_word, hipStream_t st);
int trmv_launch_exchange_reduce(const int64_t* g, int world, int64_t len, int n_dc, int64_t* hdr, int64_t* out,
                                hipStream_t st);

// Tiers of the apply chain: 0 = trmv_wave (tier 0), 1 / 2 = trmv_steady with
// up to 256 / 1024 players per key (tier S, LDS), 3 = trmv_resident (tier R),
// 4 = trmv_steady's HBM class (up to trmv_steady_hbm_players() players).  A
// batch queues one chain: onto fresh keys 0 -> 1 -> 2, onto resident keys
// 3 -> 1 -> 2 (tier R needs K <= 128; else 1 -> 2); only when tier 2 handed
// keys on does the host launch tier 4 on them, after the chain's status read.
// Tier 4 is last: the keys it hands on are over the per-key capacity
// (CCRDT_EKEYCAP, ccrdt_engine_handed_on(e, 4)).
static constexpr int TRMV_N_TIERS = 5;
static constexpr int TRMV_TIER_LAST = 4;
static constexpr uint32_t TRMV_HBM_WAVES = 128;  // workgroups (scratch slots) of tier 4
static constexpr int TRMV_STATUS_WORDS = 2 + 2 * TRMV_N_TIERS;  // [0,2) scan, [2+2t, 4+2t) tier t
static constexpr uint32_t TRMV_LATER_GRID = 4096;  // keys the grids of the later tiers cover

// f(k0, k1) over [0, n) in contiguous ranges on up to 16 host threads (the
// host-side passes over a whole state: export).
template <class F>
void for_key_ranges_host(uint64_t n, F f) {
  const unsigned hw = std::thread::hardware_concurrency();
  uint64_t nt = std::min<uint64_t>(16, hw ? hw : 1);
  nt = std::min<uint64_t>(nt, n / 4096 + 1);
  std::vector<std::thread> pool;
  for (uint64_t t = 1; t < nt; ++t) pool.emplace_back([&, t] { f(n * t / nt, n * (t + 1) / nt); });
  f(0, n / nt);
  for (auto& th : pool) th.join();
}

}  // namespace ccrdt

using namespace ccrdt;

TrmvSide ccrdt_engine::trmv_side(int ms, int ds) const {
  const TrmvBufs& b = trmv[ds];
  TrmvSide t;
  t.meta = trmv[ms].meta.as<KeyMeta>();
  t.cap = trmv[ms].cap.as<KeyCap>();
  t.pl_id = b.pl_id.as<int64_t>();
  t.pl_info = b.pl_info.as<uint32_t>();
  t.m_score = b.m_score.as<int64_t>();
  t.m_ts = b.m_ts.as<int64_t>();
  t.m_dc = b.m_dc.as<uint8_t>();
  t.pl_slab = b.pl_slab.as<uint32_t>();
  t.pl_gb = b.pl_gb.as<uint16_t>();
  t.r_vc = b.r_vc.as<int64_t>();
  t.vc = b.vc.as<int64_t>();
  return t;
}

void ccrdt_engine::release_all() {
  for (auto& b : trmv) {
    b.meta.release();
    b.cap.release();
    b.pl_id.release();
    b.pl_info.release();
    b.m_score.release();
    b.m_ts.release();
    b.m_dc.release();
    b.pl_slab.release();
    b.pl_gb.release();
    b.r_vc.release();
    b.vc.release();
  }
  for (DevBuf& d : tier_ovf) d.release();
  for (DevBuf& d : st_n32) d.release();
  for (DevBuf& d : st_nbase) d.release();
  for (DevBuf* d : {&arena, &obs_ord, &key_done, &partials, &ex_cnt, &ex, &ex_vc, &ex_key_ptr, &status, &op_pl,
                    &first_list, &ovl,
                    &hbm_scratch, &st_kp,
                    &st_kind, &st_id, &st_score, &st_dc, &st_ts, &st_rvc, &st_out_kind, &st_out_vc})
    d->release();
  release_types();
}

// ===================================================================== C-ABI
extern "C" {

const char* ccrdt_strerror(int code) {
  switch (code) {
    case CCRDT_OK: return "ok";
    case CCRDT_EINVAL: return "invalid argument or operation";
    case CCRDT_ERANGE: return "integer outside engine range";
    case CCRDT_ENOMEM: return "out of device memory or per-key capacity";
    case CCRDT_EKEYCAP: return "keys over the per-key capacity were left out of the batch";
    case CCRDT_EPARTIAL: return "the batch committed except for the keys whose finishing pass failed";
    case CCRDT_EDEVICE: return "HIP device error";
    case CCRDT_ENOSYS: return "operation not supported for this CCRDT type";
    default: return "unknown error";
  }
}
const char* ccrdt_last_error(void) { return g_last_error.c_str(); }

int ccrdt_is_type(int type) { return type >= CCRDT_AVERAGE && type <= CCRDT_WORDDOCUMENTCOUNT; }
int ccrdt_generates_extra_operations(int type) {
  return type == CCRDT_TOPK_RMV || type == CCRDT_LEADERBOARD;
}

int ccrdt_device_count(int* n) {
  CCRDT_HIP(hipGetDeviceCount(n));
  return CCRDT_OK;
}
int ccrdt_set_device(int device) {
  CCRDT_HIP(hipSetDevice(device));
  return CCRDT_OK;
}
int ccrdt_device_alloc(void** p, uint64_t bytes) {
  CCRDT_HIP(hipMalloc(p, bytes ? bytes : 1));
  return CCRDT_OK;
}
int ccrdt_device_free(void* p) {
  CCRDT_HIP(hipFree(p));
  return CCRDT_OK;
}
int ccrdt_memcpy_h2d(void* dst, const void* src, uint64_t bytes) {
  CCRDT_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return CCRDT_OK;
}
int ccrdt_memcpy_d2h(void* dst, const void* src, uint64_t bytes) {
  CCRDT_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return CCRDT_OK;
}
int ccrdt_device_synchronize(void) {
  CCRDT_HIP(hipDeviceSynchronize());
  return CCRDT_OK;
}

int ccrdt_engine_create(int type, int64_t k, int64_t n_keys, int n_dc, int device,
                        ccrdt_engine** out) {
  if (!out || !ccrdt_is_type(type) || n_keys < 0 || k <= 0) {
    set_error("engine_create: bad type / k / n_keys");
    return CCRDT_EINVAL;
  }
  if (type == CCRDT_TOPK_RMV && (n_dc < 1 || n_dc > CCRDT_TRMV_MAX_DC)) {
    set_error("engine_create: topk_rmv needs 1 <= n_dc <= 8");
    return CCRDT_EINVAL;
  }
  if (n_keys > 0xFFFFFFFFll) {
    set_error("engine_create: n_keys must fit in 32 bits");
    return CCRDT_EINVAL;
  }
  int ndev = 0;
  CCRDT_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    set_error("engine_create: no such HIP device");
    return CCRDT_EDEVICE;
  }
  CCRDT_HIP(hipSetDevice(device));
  Engine* e = new Engine();
  e->type = type;
  e->k = k;
  e->n_keys = n_keys;
  e->n_dc = n_dc;
  e->device = device;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&e->ev0) != hipSuccess || hipEventCreate(&e->ev1) != hipSuccess ||
      hipEventCreate(&e->evk0) != hipSuccess || hipEventCreate(&e->evk1) != hipSuccess ||
      !e->create_tier_events() ||
      hipHostMalloc((void**)&e->h_status, 256, hipHostMallocDefault) != hipSuccess) {
    set_error("engine_create: stream/event/pinned allocation failed");
    delete e;
    return CCRDT_EDEVICE;
  }
  if (type == CCRDT_TOPK_RMV) {  // the apply chain's kernels set up now, not in the first batches
    trmv_kernels_preload();
    trmv_wave_preload();
    trmv_resident_preload();
    trmv_steady_preload();
  }
  int rc = e->init_type();
  if (rc != CCRDT_OK) {
    ccrdt_engine_destroy(e);
    return rc;
  }
  *out = e;
  return CCRDT_OK;
}

int ccrdt_engine_destroy(ccrdt_engine* e) {
  if (!e) return CCRDT_OK;
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  e->release_all();
  ccrdt::stage_release(*e);
  if (e->h_status) (void)hipHostFree(e->h_status);
  if (e->h_arena) (void)hipHostFree(e->h_arena);
  if (e->ev0) (void)hipEventDestroy(e->ev0);
  if (e->ev1) (void)hipEventDestroy(e->ev1);
  if (e->evk0) (void)hipEventDestroy(e->evk0);
  if (e->evk1) (void)hipEventDestroy(e->evk1);
  e->destroy_tier_events();
  if (e->ev_ovl) (void)hipEventDestroy(e->ev_ovl);
  if (e->stream2) {
    (void)hipStreamSynchronize(e->stream2);
    (void)hipStreamDestroy(e->stream2);
  }
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
  return CCRDT_OK;
}

int ccrdt_engine_reset(ccrdt_engine* e) {
  if (!e) return CCRDT_EINVAL;
  e->fresh = true;
  e->inplace_ready = false;
  e->arena_pending = false;
  return e->reset_type();
}

int ccrdt_engine_sync(ccrdt_engine* e) {
  if (!e) return CCRDT_EINVAL;
  CCRDT_HIP(hipStreamSynchronize(e->stream));
  return CCRDT_OK;
}
void* ccrdt_engine_stream(ccrdt_engine* e) { return e ? (void*)e->stream : nullptr; }

int ccrdt_timer_start(ccrdt_engine* e) {
  if (!e) return CCRDT_EINVAL;
  CCRDT_HIP(hipSetDevice(e->device));
  CCRDT_HIP(hipEventRecord(e->ev0, e->stream));
  return CCRDT_OK;
}
int ccrdt_timer_stop(ccrdt_engine* e, float* ms) {
  if (!e || !ms) return CCRDT_EINVAL;
  CCRDT_HIP(hipEventRecord(e->ev1, e->stream));
  CCRDT_HIP(hipEventSynchronize(e->ev1));
  CCRDT_HIP(hipEventElapsedTime(ms, e->ev0, e->ev1));
  return CCRDT_OK;
}

int ccrdt_engine_last_kernel_ms(ccrdt_engine* e, float* ms) {
  if (!e || !ms) return CCRDT_EINVAL;
  *ms = e->last_kernel_ms;
  return CCRDT_OK;
}

int ccrdt_engine_tier_ms(ccrdt_engine* e, int tier, float* ms) {
  if (!e || !ms) return CCRDT_EINVAL;
  auto it = e->trmv_tier_ms.find(tier);
  *ms = it == e->trmv_tier_ms.end() ? 0.f : it->second;
  return CCRDT_OK;
}

int ccrdt_engine_overflow_keys(ccrdt_engine* e, int slot_class, int64_t* n) {
  if (!e || !n) return CCRDT_EINVAL;
  auto it = e->trmv_overflow_keys.find(slot_class);
  *n = it == e->trmv_overflow_keys.end() ? 0 : it->second;
  return CCRDT_OK;
}

// ------------------------------------------------------------------ topk_rmv

static int check_trmv(ccrdt_engine* e) {
  if (!e) {
    set_error("null engine");
    return CCRDT_EINVAL;
  }
  if (e->type != CCRDT_TOPK_RMV) {
    set_error("engine is not topk_rmv");
    return CCRDT_ENOSYS;
  }
  if (hipSetDevice(e->device) != hipSuccess) {
    set_error("hipSetDevice failed");
    return CCRDT_EDEVICE;
  }
  return CCRDT_OK;
}

namespace {

// The error bits the kernels OR-ed into a status word -> the C-ABI code.
int trmv_err_code(uint32_t err) {
  std::string m = "trmv_apply: invalid op in batch:";
  if (err & TRMV_ERR_KIND) m += " kind>3";
  if (err & TRMV_ERR_DC) m += " dc>=n_dc";
  if (err & TRMV_ERR_TS) m += " add ts<1";
  if (err & TRMV_ERR_ROW) m += " rmv row out of range";
  if (err & TRMV_ERR_VC) m += " negative VcRmv entry";
  set_error(m);
  return (err & (TRMV_ERR_TS | TRMV_ERR_VC)) && !(err & (TRMV_ERR_KIND | TRMV_ERR_DC | TRMV_ERR_ROW)) ? CCRDT_ERANGE
                                                                                                  : CCRDT_EINVAL;
}

// The pool's capacity factor of segments laid out for in-place growth
// (a.slack): capacity = factor x (elements + the batch's ops) + 32, so later
// batches append slabs in place (CCRDT_TRMV_POOL_SLACK = 2..8, tuning knob).
int trmv_pool_slack() {
  static const int v = [] {
    const char* e = getenv("CCRDT_TRMV_POOL_SLACK");
    const int x = e ? atoi(e) : 2;
    return x < 2 ? 2 : (x > 8 ? 8 : x);
  }();
  return v;
}

// Capacities (elements) of a data side's arrays.
void trmv_side_caps(const Engine& E, int ds, uint64_t cap[3]) {
  const TrmvBufs& b = E.trmv[ds];
  cap[0] = std::min(b.pl_id.bytes / 8, std::min(b.pl_info.bytes / 4, std::min(b.pl_slab.bytes / 4, b.pl_gb.bytes / 2)));
  cap[1] = std::min(b.m_score.bytes / 8, std::min(b.m_ts.bytes / 8, b.m_dc.bytes));
  cap[2] = E.n_dc ? b.r_vc.bytes / (8 * (uint64_t)E.n_dc) : 0;
}

// In place (tier R alone): the batch validated, then every key updated in
// the data arrays it lives in (meta / cap ping-pong).  Keys that cannot be
// updated in place (outside tier R's class, or the arena is full) are left
// as they were and listed in tier_ovf[3]; *handed = their number.
int trmv_pass_inplace(Engine& E, TrmvApplyArgs a, uint64_t n_ops, uint32_t* status, uint32_t& handed) {
  const uint64_t nk = (uint64_t)E.n_keys;
  const int D = E.n_dc;
  CCRDT_TRY(E.trmv[1 - E.mcur].meta.ensure(nk * sizeof(KeyMeta)));
  CCRDT_TRY(E.trmv[1 - E.mcur].cap.ensure(nk * sizeof(KeyCap)));
  constexpr size_t ARENA_RB = sizeof(E.arena_sub[0]);  // (the counters; the layout counts follow the ends)
  // the readback's pinned buffer before anything is queued: a failure here
  // leaves the state untouched
  if (!E.h_arena && hipHostMalloc(&E.h_arena, 2 * ARENA_RB + 16 * TRMV_NSUB, hipHostMallocDefault) != hipSuccess) {
    E.h_arena = nullptr;
    set_error("trmv_apply: pinned allocation failed");
    return CCRDT_EDEVICE;
  }
  a.inplace = 1;
  a.slack = trmv_pool_slack();  // (relocations' pool capacity)
  a.old_s = E.trmv_side(E.mcur, E.cur);
  a.new_s = E.trmv_side(1 - E.mcur, E.cur);
  if (E.arena_pending) {  // the sub-arena table the last full pass laid out
    CCRDT_HIP(hipMemcpyAsync(E.arena.p, E.arena_sub, sizeof(E.arena_sub), hipMemcpyHostToDevice, E.stream));
    E.arena_pending = false;
  }
  a.arena = E.arena.as<unsigned long long>();
  a.arena_lim = E.arena.as<unsigned long long>() + 3 * TRMV_NSUB;
  a.lay_cnt = reinterpret_cast<uint32_t*>(E.arena.as<unsigned long long>() + 6 * TRMV_NSUB);
  CCRDT_HIP(hipMemsetAsync(a.lay_cnt, 0, 4 * TRMV_NSUB * sizeof(uint32_t), E.stream));
  a.key_done = nullptr;
  a.key_list = nullptr;
  a.n_list = (uint32_t)nk;
  a.n_list_dev = nullptr;
  a.ovf_list = E.tier_ovf[3].as<uint32_t>();
  a.status = status + 2 + 2 * 3;
  a.verr = status + 2 + 2 * 3 + 1;  // (tier R's error word: the validation writes it)
  CCRDT_HIP(hipEventRecord(E.evt[0], E.stream));
  CCRDT_TRY(trmv_launch_validate(a, n_ops, status + 2 + 2 * 3 + 1,
                                 reinterpret_cast<unsigned long long*>(status + TRMV_STATUS_WORDS), E.stream));
  CCRDT_HIP(hipEventRecord(E.evt[1], E.stream));
  CCRDT_TRY(trmv_launch_resident(a, nk, E.stream));
  CCRDT_HIP(hipEventRecord(E.evt[2], E.stream));
  CCRDT_HIP(hipMemcpyAsync(E.h_status, status, TRMV_STATUS_WORDS * 4, hipMemcpyDeviceToHost, E.stream));
  CCRDT_HIP(hipMemcpyAsync(E.h_arena, E.arena.p, ARENA_RB, hipMemcpyDeviceToHost, E.stream));
  CCRDT_HIP(hipMemcpyAsync(static_cast<char*>(E.h_arena) + 2 * ARENA_RB, a.lay_cnt, 16 * TRMV_NSUB,
                           hipMemcpyDeviceToHost, E.stream));
  CCRDT_HIP(hipStreamSynchronize(E.stream));
  const uint32_t* hs = (const uint32_t*)E.h_status;
  if (hs[3 + 2 * 3]) return trmv_err_code(hs[3 + 2 * 3]);
  {
    // the arena's use: what this pass took, what is left; the next batch
    // runs in place only while the room left covers twice this pass's take
    const uint64_t(*cnt)[3] = reinterpret_cast<const uint64_t(*)[3]>(E.h_arena);
    bool roomy = true;
    for (int x = 0; x < 3; ++x) {
      uint64_t used = 0, room = 0;
      for (int i = 0; i < TRMV_NSUB; ++i) {
        const uint64_t c = std::min(cnt[i][x], E.arena_sub[1][i][x]);
        used += c - E.arena_sub[0][i][x];
        room += E.arena_sub[1][i][x] - c;
      }
      const uint64_t take = used - std::min(used, E.arena_used[x]);
      E.arena_used[x] = used;
      E.arena_rate[x] = std::max(E.arena_rate[x], take);
      roomy &= room >= 2 * take;
    }
    E.inplace_ready = roomy;
    // keys by layout (ccrdt_engine_overflow_keys slots 6, 7, 8: relocated, appended, compacted)
    const uint32_t* lc = reinterpret_cast<const uint32_t*>(static_cast<const char*>(E.h_arena) + 2 * ARENA_RB);
    for (int l = 0; l < 3; ++l) {
      uint32_t n = 0;
      for (int i = 0; i < TRMV_NSUB; ++i) n += lc[4 * i + l];
      E.trmv_overflow_keys[6 + l] = n;
    }
  }
  float mv = 0.f, mr = 0.f;
  CCRDT_HIP(hipEventElapsedTime(&mv, E.evt[0], E.evt[1]));
  CCRDT_HIP(hipEventElapsedTime(&mr, E.evt[1], E.evt[2]));
  E.trmv_tier_ms[5] += mv;  // (the validation pass)
  E.trmv_tier_ms[3] += mr;
  handed = hs[2 + 2 * 3];
  E.trmv_overflow_keys[5] = handed;  // (keys the in-place pass left to the full rewrite)
  (void)D;
  return CCRDT_OK;
}

// A full rewrite: the capacity scan lays every key out in the other data
// arrays (with room for in-place growth when tier R can take the keys), then
// the tier chain.  With a.key_done the keys an in-place pass completed are
// only copied (no ops).
int trmv_pass_full(Engine& E, TrmvApplyArgs a, uint64_t n_ops, uint32_t* status, int& first_tier, int& n_over) {
  const int D = E.n_dc;
  const uint64_t nk = (uint64_t)E.n_keys;
  const int out = 1 - E.cur, mout = 1 - E.mcur;
  a.inplace = 0;
  a.fresh = E.fresh ? 1 : 0;
  // CCRDT_TRMV_FAIL_FINISH=1 (tests): the full rewrite that finishes an
  // in-place batch fails as an allocation would (CCRDT_EPARTIAL's path)
  if (a.key_done) {
    const char* ff = getenv("CCRDT_TRMV_FAIL_FINISH");
    if (ff && ff[0] == '1') {
      set_error("trmv_apply: injected failure of the finishing pass (CCRDT_TRMV_FAIL_FINISH)");
      return CCRDT_ENOMEM;
    }
  }
  // room for in-place growth when tier R can take the keys (K <= 128): the
  // capacity scan's slack, or a fresh batch's roomy layout while its offsets
  // fit 32 bits
  a.slack = E.k <= 128 ? trmv_pool_slack() : 0;
  if (E.fresh && !E.fresh_room) a.slack = 0;  // (ccrdt_trmv_set_fresh_room)
  if (E.fresh && a.slack)
    for (int x = 0; x < 3; ++x)
      if (trmv_fresh_off(true, x, nk, n_ops) >= 0xFFFFFFFFull) a.slack = 0;
  a.old_s = E.trmv_side(E.mcur, E.cur);
  CCRDT_TRY(E.trmv[mout].meta.ensure(nk * sizeof(KeyMeta)));
  CCRDT_TRY(E.trmv[mout].cap.ensure(nk * sizeof(KeyCap)));
  a.new_s = E.trmv_side(mout, out);
  const uint64_t nb = (nk + 1023) / 1024;
  // partials: per-tile sums and totals, then each key's rmv-op count (u32)
  CCRDT_TRY(E.partials.ensure((nb * 3 + 3) * sizeof(uint64_t) + nk * sizeof(uint32_t)));
  // 1) capacities -> segment offsets of the new state (a fresh batch's
  //    offsets are the keys' op offsets: trmv_new_meta, no scan)
  uint64_t tot[3];
  for (int x = 0; x < 3; ++x) tot[x] = trmv_fresh_off(a.slack != 0, x, nk, n_ops);  // (fresh: no scan)
  if (!E.fresh && nk) {
    CCRDT_TRY(trmv_launch_scan(a, E.partials.as<uint64_t>(),
                               reinterpret_cast<uint32_t*>(E.partials.as<uint64_t>() + nb * 3 + 3), E.stream));
    // (the exact totals size the new side)
    CCRDT_HIP(hipMemcpyAsync(E.h_status, E.partials.as<uint64_t>() + nb * 3, 3 * sizeof(uint64_t),
                             hipMemcpyDeviceToHost, E.stream));
    CCRDT_HIP(hipStreamSynchronize(E.stream));
    memcpy(tot, E.h_status, sizeof(tot));
  }
  if (tot[0] >= 0xFFFFFFFFull || tot[1] >= 0xFFFFFFFFull || tot[2] >= 0xFFFFFFFFull) {
    set_error("trmv_apply: resident state would exceed 2^32 elements");
    return CCRDT_ENOMEM;
  }
  // Sizes of the new side: the totals, and with room to grow in place a
  // quarter more for the keys later batches relocate (the arena)
  auto grow = [&](TrmvBufs& b, bool room) -> int {
    // (room: for the keys later in-place batches relocate -- three passes'
    // worth of the most one pass took so far, a quarter of the totals at least)
    uint64_t t[3];
    for (int x = 0; x < 3; ++x) t[x] = room ? tot[x] + std::max(tot[x] / 4, 3 * E.arena_rate[x]) : tot[x];
    CCRDT_TRY(b.pl_id.ensure_grow(t[0] * 8));
    CCRDT_TRY(b.pl_info.ensure_grow(t[0] * 4));
    CCRDT_TRY(b.pl_slab.ensure_grow(t[0] * 4));
    CCRDT_TRY(b.pl_gb.ensure_grow(t[0] * 2));
    CCRDT_TRY(b.m_score.ensure_grow(t[1] * 8));
    CCRDT_TRY(b.m_ts.ensure_grow(t[1] * 8));
    CCRDT_TRY(b.m_dc.ensure_grow(t[1]));
    CCRDT_TRY(b.r_vc.ensure_grow(t[2] * 8 * D));
    CCRDT_TRY(b.vc.ensure(nk * 8 * D));
    return CCRDT_OK;
  };
  CCRDT_TRY(grow(E.trmv[out], a.slack != 0));
  // The current side holds nothing live after reset(): size it too, so the
  // next batch (which writes it) does not allocate.
  if (E.fresh) CCRDT_TRY(grow(E.trmv[E.cur], false));
  a.new_s = E.trmv_side(mout, out);
  // 2) the chain: its first tier over every key, then each later tier over
  //    the keys the one before handed on.  Every later tier reads its list
  //    length from the device, so the whole chain is queued without a host
  //    round trip; one sync at the end reads the status.
  // CCRDT_TRMV_FIRST_TIER (tuning knob): -1 = the default chain, 0 = tier 0
  // first (fresh batches only), 1 = tier S first, 3 = tier R first (resident
  // batches only).
  static const int first_env = [] {
    const char* v = getenv("CCRDT_TRMV_FIRST_TIER");
    return v ? atoi(v) : -1;
  }();
  int chain[4], n_chain = 0;
  {
    int first = E.fresh ? 0 : (E.k <= 128 ? 3 : 1);
    if (first_env == 1 || (first_env == 0 && E.fresh) || (first_env == 3 && !E.fresh && E.k <= 128)) first = first_env;
    chain[n_chain++] = first;
    // a fresh batch: tier 0's hand-ons (P > K) go to tier R first, whose
    // per-key latency is about half of tier S's
    if (first == 0 && E.k <= 128) chain[n_chain++] = 3;
    chain[n_chain++] = 1;
    chain[n_chain++] = 2;
    if (first == 1) n_chain = 2, chain[1] = 2;
  }
  first_tier = chain[0];
  for (int ci = 0; ci < n_chain; ++ci) E.trmv_overflow_keys[chain[ci]] = 0;
  // The chain's head -- tier 0 and / or tier R, which take every key of the
  // bench streams -- is queued in one go; its tier S tail only when the
  // status read after the head says the head handed keys on (a chain that
  // starts at tier S, K > 128, is all head).  Each segment's kernels read
  // their list lengths from the device.
  int n_head = 0;
  while (n_head < n_chain && (chain[n_head] == 0 || chain[n_head] == 3)) ++n_head;
  if (n_head == 0) n_head = n_chain;
  const uint32_t later_grid = (uint32_t)std::min<uint64_t>(nk, TRMV_LATER_GRID);
  DevBuf* work = nullptr;
  const uint32_t* n_dev = nullptr;
  int ev = 0;
  const uint32_t* hs = (const uint32_t*)E.h_status;
  // chain[c0, c1): launches, one status read, the tiers' errors, times and hand-on counts
  auto segment = [&](int c0, int c1) -> int {
    const int e0 = ev;
    CCRDT_HIP(hipEventRecord(E.evt[ev++], E.stream));
    for (int ci = c0; ci < c1 && nk; ++ci) {
      const int t = chain[ci];
      DevBuf* ovf = &E.tier_ovf[t];
      a.key_list = work ? work->as<uint32_t>() : nullptr;
      a.n_list = work ? 0u : (uint32_t)nk;
      a.n_list_dev = n_dev;
      a.ovf_list = ovf->as<uint32_t>();
      a.status = status + 2 + 2 * t;
      const uint64_t grid = work ? later_grid : nk;
      if (t == 0) CCRDT_TRY(trmv_launch_wave(a, grid, E.stream));
      else if (t == 3) CCRDT_TRY(trmv_launch_resident(a, grid, E.stream));
      else CCRDT_TRY(trmv_launch_steady(a, t - 1, grid, E.stream));
      CCRDT_HIP(hipEventRecord(E.evt[ev++], E.stream));
      work = ovf;
      n_dev = a.status;
    }
    CCRDT_HIP(hipMemcpyAsync(E.h_status, status, TRMV_STATUS_WORDS * 4, hipMemcpyDeviceToHost, E.stream));
    CCRDT_HIP(hipStreamSynchronize(E.stream));
    uint32_t err = 0;
    for (int ci = c0; ci < c1; ++ci) err |= hs[3 + 2 * chain[ci]];
    if (err) return trmv_err_code(err);
    for (int ci = c0; ci < c1 && nk; ++ci) {
      const int t = chain[ci];
      float ms = 0.f;
      CCRDT_HIP(hipEventElapsedTime(&ms, E.evt[e0 + ci - c0], E.evt[e0 + ci - c0 + 1]));
      E.trmv_tier_ms[t] += ms;
      E.trmv_overflow_keys[t] = hs[2 + 2 * t];
    }
    return CCRDT_OK;
  };
  // The overlapped hand-on: a fresh batch's head [tier 0,
  // tier R] with tier R on a second, high-priority stream beside tier 0,
  // taking the keys tier 0 hands on while it runs; tier 0 takes the likely
  // hand-ons (more than min(128, 1.2 pmax) ops) first, so tier R's per-key
  // latency is spent while tier 0 still works instead of after it.  On for
  // engines of at most CCRDT_TRMV_OVERLAP_KEYS keys (default 2^18: a rank of
  // the strong line at N >= 4): the tail it hides is one key's latency, a
  // larger share of a smaller shard's step, and tier 0 runs ~5 % slower beside
  // it (profiles/r06/ab_overlap_waves.txt: 2^17 keys, step 0.404 -> 0.374 ms;
  // 2^20 keys, 2.29 -> 2.34 ms, so off there).
  // CCRDT_TRMV_OVERLAP=0: never; CCRDT_TRMV_OVERLAP_WAVES: tier R's waves
  // (32: 16 could not keep up with the hand-ons, 48 and 64 slowed tier 0).
  static const bool overlap_env = [] {
    const char* v = getenv("CCRDT_TRMV_OVERLAP");
    return !(v && v[0] == '0');
  }();
  static const uint64_t overlap_keys = [] {
    const char* v = getenv("CCRDT_TRMV_OVERLAP_KEYS");
    return v ? strtoull(v, nullptr, 10) : (1ull << 18);
  }();
  static const uint32_t overlap_waves = [] {
    const char* v = getenv("CCRDT_TRMV_OVERLAP_WAVES");
    const int x = v ? atoi(v) : 32;
    return (uint32_t)(x < 1 ? 1 : (x > 4096 ? 4096 : x));
  }();
  auto head_overlapped = [&]() -> int {
    if (!E.stream2) {
      // (created through the priority API at the highest priority: a plain
      // second stream shared a hardware queue with the engine's and ran after it)
      int lo = 0, hi = 0;
      CCRDT_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
      CCRDT_HIP(hipStreamCreateWithPriority(&E.stream2, hipStreamNonBlocking, hi));
      CCRDT_HIP(hipEventCreateWithFlags(&E.ev_ovl, hipEventDisableTiming));
    }
    // ovl: [done words | claim | first_list count | pad | published hand-ons (key + 1), one per key]
    constexpr uint32_t O_CLAIM = TRMV_NDONE, O_NFIRST = TRMV_NDONE + 1, O_PUB = TRMV_NDONE + 4;
    CCRDT_TRY(E.first_list.ensure(nk * 4));
    CCRDT_TRY(E.ovl.ensure((O_PUB + nk) * 4));
    uint32_t* ov = E.ovl.as<uint32_t>();
    CCRDT_HIP(hipMemsetAsync(ov, 0, (O_PUB + nk) * 4, E.stream));
    const uint32_t pmax = (uint32_t)std::min<int64_t>(E.k, 128);
    const uint32_t thresh = std::min<uint32_t>(128u, pmax + pmax / 5);
    CCRDT_TRY(trmv_launch_first_list(a.key_ptr, nk, thresh, E.first_list.as<uint32_t>(), ov + O_NFIRST, E.stream));
    const int e0 = ev;
    CCRDT_HIP(hipEventRecord(E.evt[ev++], E.stream));
    TrmvApplyArgs a0 = a;
    a0.key_list = nullptr;
    a0.n_list = (uint32_t)nk;
    a0.n_list_dev = nullptr;
    a0.ovf_list = E.tier_ovf[0].as<uint32_t>();
    a0.status = status + 2;
    a0.first_list = E.first_list.as<uint32_t>();
    a0.n_first = ov + O_NFIRST;
    a0.first_thresh = thresh;
    a0.pub = ov + O_PUB;
    a0.n_pub = (uint32_t)nk;
    a0.done = ov;
    CCRDT_TRY(trmv_launch_wave(a0, nk, E.stream));
    CCRDT_HIP(hipEventRecord(E.evt[ev++], E.stream));
    CCRDT_HIP(hipStreamWaitEvent(E.stream2, E.evt[e0], 0));
    TrmvApplyArgs a3 = a;
    a3.key_list = E.tier_ovf[0].as<uint32_t>();
    a3.n_list = 0;
    a3.n_list_dev = status + 2;
    a3.ovf_list = E.tier_ovf[3].as<uint32_t>();
    a3.status = status + 2 + 2 * 3;
    a3.pub = ov + O_PUB;
    a3.n_pub = (uint32_t)nk;
    a3.done = ov;
    a3.prod_waves = trmv_wave_waves(nk);
    a3.claim = ov + O_CLAIM;
    // CCRDT_TRMV_OVERLAP_STALL=1 (tests): the consumers give up at once when
    // no hand-on is there yet, and the host's fallback runs
    const char* stall_env = getenv("CCRDT_TRMV_OVERLAP_STALL");
    const bool force_stall = stall_env && stall_env[0] == '1';
    a3.spin_limit = force_stall ? 0u : (1u << 19);  // (~2 s)
    CCRDT_TRY(trmv_launch_resident_consume(a3, overlap_waves, E.stream2));
    CCRDT_HIP(hipEventRecord(E.ev_ovl, E.stream2));
    CCRDT_HIP(hipStreamWaitEvent(E.stream, E.ev_ovl, 0));
    CCRDT_HIP(hipEventRecord(E.evt[ev++], E.stream));
    CCRDT_HIP(hipMemcpyAsync(E.h_status, status, TRMV_STATUS_WORDS * 4, hipMemcpyDeviceToHost, E.stream));
    CCRDT_HIP(hipStreamSynchronize(E.stream));
    if ((hs[3 + 2 * 3] & TRMV_ERR_STALL) || force_stall) {
      // tier 0 did not run beside the consumers: tier R over the whole list
      // after it (a fresh key's tier R rewrites the same result)
      CCRDT_HIP(hipMemsetAsync(status + 2 + 2 * 3, 0, 8, E.stream));
      a3.pub = nullptr;
      a3.done = nullptr;
      CCRDT_TRY(trmv_launch_resident(a3, later_grid, E.stream));
      CCRDT_HIP(hipEventRecord(E.evt[ev - 1], E.stream));
      CCRDT_HIP(hipMemcpyAsync(E.h_status, status, TRMV_STATUS_WORDS * 4, hipMemcpyDeviceToHost, E.stream));
      CCRDT_HIP(hipStreamSynchronize(E.stream));
      E.trmv_overflow_keys[9] = 1;  // (diagnostic: the stall fallback ran)
    }
    const uint32_t err = hs[3] | hs[3 + 2 * 3];
    if (err) return trmv_err_code(err);
    float m0 = 0.f, m3 = 0.f;
    CCRDT_HIP(hipEventElapsedTime(&m0, E.evt[e0], E.evt[e0 + 1]));
    CCRDT_HIP(hipEventElapsedTime(&m3, E.evt[e0 + 1], E.evt[e0 + 2]));
    E.trmv_tier_ms[0] += m0;
    E.trmv_tier_ms[3] += m3;  // (tier R's tail past tier 0: the rest ran beside it)
    E.trmv_overflow_keys[0] = hs[2];
    E.trmv_overflow_keys[3] = hs[2 + 2 * 3];
    work = &E.tier_ovf[3];
    n_dev = status + 2 + 2 * 3;
    return CCRDT_OK;
  };
  const bool overlap = overlap_env && E.fresh && nk && nk <= overlap_keys && n_head == 2 && chain[0] == 0 &&
                       chain[1] == 3;
  if (overlap) CCRDT_TRY(head_overlapped());
  else CCRDT_TRY(segment(0, n_head));
  if (n_head < n_chain && nk && hs[2 + 2 * chain[n_head - 1]] != 0) CCRDT_TRY(segment(n_head, n_chain));
  // Keys past the 1024-player class: tier 4 (HBM scratch), on the host-known
  // list tier 2 handed on.
  const uint32_t n_big = nk ? hs[2 + 2 * 2] : 0u;
  if (n_big) {
    const uint32_t waves = std::min<uint32_t>(n_big, TRMV_HBM_WAVES);
    CCRDT_TRY(E.hbm_scratch.ensure((uint64_t)TRMV_HBM_WAVES * trmv_steady_hbm_bytes(E.k <= 128)));
    a.key_list = E.tier_ovf[2].as<uint32_t>();
    a.n_list = n_big;
    a.n_list_dev = nullptr;
    a.ovf_list = E.tier_ovf[4].as<uint32_t>();
    a.status = status + 2 + 2 * 4;
    CCRDT_HIP(hipEventRecord(E.evt[ev++], E.stream));
    CCRDT_TRY(trmv_launch_steady_hbm(a, waves, E.hbm_scratch.p, E.stream));
    CCRDT_HIP(hipEventRecord(E.evt[ev++], E.stream));
    CCRDT_HIP(hipMemcpyAsync(E.h_status, status, TRMV_STATUS_WORDS * 4, hipMemcpyDeviceToHost, E.stream));
    CCRDT_HIP(hipStreamSynchronize(E.stream));
    const uint32_t e4 = hs[3 + 2 * 4];
    if (e4) return trmv_err_code(e4);
    float ms = 0.f;
    CCRDT_HIP(hipEventElapsedTime(&ms, E.evt[ev - 2], E.evt[ev - 1]));
    E.trmv_tier_ms[4] += ms;
  }
  E.trmv_overflow_keys[4] = n_big ? hs[2 + 2 * 4] : 0u;
  // Keys over the per-key capacity (tier 4's hand-ons) keep their old state;
  // every other key commits.
  n_over = (int)E.trmv_overflow_keys[4];
  if (n_over) {
    a.key_list = E.tier_ovf[TRMV_TIER_LAST].as<uint32_t>();
    a.n_list = 0;
    a.n_list_dev = status + 2 + 2 * TRMV_TIER_LAST;  // (trmv_keep_kernel reads the count here)
    CCRDT_TRY(trmv_launch_keep(a, std::min<uint32_t>((uint32_t)n_over, TRMV_LATER_GRID), E.stream));
  }
  // the arena of the new data arrays (only when in-place batches may
  // follow: tier 0 / tier R wrote the keys with room): its top = the
  // layout's totals, its free space cut into TRMV_NSUB sub-arenas.  The
  // device copy of the table is made by the next in-place pass (arena_pending),
  // so a fresh batch that no resident batch follows pays no round trip for it.
  const bool roomy = a.slack != 0 && (first_tier == 3 || first_tier == 0);
  if (roomy) {
    trmv_side_caps(E, out, E.arena_cap);
    // CCRDT_TRMV_ARENA_ROOM=n (tests): at most n free elements past the top,
    // so relocations run out and the full rewrite that finishes a batch runs
    if (const char* v = getenv("CCRDT_TRMV_ARENA_ROOM"))
      for (int x = 0; x < 3; ++x) E.arena_cap[x] = std::min<uint64_t>(E.arena_cap[x], tot[x] + strtoull(v, nullptr, 10));
    auto& sub = E.arena_sub;
    for (int x = 0; x < 3; ++x) {
      const uint64_t room = E.arena_cap[x] > tot[x] ? E.arena_cap[x] - tot[x] : 0;
      for (int i = 0; i < TRMV_NSUB; ++i) {
        sub[0][i][x] = tot[x] + room * i / TRMV_NSUB;
        sub[1][i][x] = tot[x] + room * (i + 1) / TRMV_NSUB;
      }
      E.arena_used[x] = 0;
    }
    CCRDT_TRY(E.arena.ensure(sizeof(sub) + 16 * TRMV_NSUB));
    E.arena_pending = true;
    // what the next (in-place) pass writes and reads back, allocated now: its
    // first use made the first in-place batch after a fresh one 2.4 ms slower
    // in wall time than its kernels (meta / cap of the other side, 48 B per
    // key, and the pinned read-back)
    CCRDT_TRY(E.trmv[1 - mout].meta.ensure(nk * sizeof(KeyMeta)));
    CCRDT_TRY(E.trmv[1 - mout].cap.ensure(nk * sizeof(KeyCap)));
    if (!E.h_arena && hipHostMalloc(&E.h_arena, 2 * sizeof(E.arena_sub[0]) + 16 * TRMV_NSUB,
                                    hipHostMallocDefault) != hipSuccess)
      E.h_arena = nullptr;  // (the in-place pass allocates it, or fails cleanly)
  }
  for (int x = 0; x < 3; ++x) E.trmv_tot[out][x] = tot[x];
  E.cur = out;
  E.mcur = mout;
  E.inplace_ready = roomy;
  return CCRDT_OK;
}

}  // namespace

int ccrdt_trmv_apply_device(ccrdt_engine* e, const ccrdt_trmv_ops* ops) {
  CCRDT_TRY(check_trmv(e));
  if (!ops || !ops->key_ptr || (ops->n_ops > 0 && (!ops->kind || !ops->id || !ops->score ||
                                                   !ops->dc || !ops->ts))) {
    set_error("trmv_apply: null op array");
    return CCRDT_EINVAL;
  }
  if (ops->n_ops >= (int64_t)0xFFFFFFFFll) {
    set_error("trmv_apply: batch too large (n_ops must fit in 32 bits)");
    return CCRDT_EINVAL;
  }
  Engine& E = *e;
  const int D = E.n_dc;
  const uint64_t nk = (uint64_t)E.n_keys;
  const uint64_t n_ops = (uint64_t)ops->n_ops;
  TrmvApplyArgs a{};
  a.n_keys = E.n_keys;
  a.n_dc = D;
  a.k = (uint32_t)std::min<int64_t>(E.k, 0xFFFFFFFFll);
  a.key_ptr = ops->key_ptr;
  a.kind = ops->kind;
  a.id = ops->id;
  a.score = ops->score;
  a.dc = ops->dc;
  a.ts = ops->ts;
  a.rmv_vc = ops->rmv_vc;
  a.n_rmv_rows = ops->rmv_vc ? ops->n_rmv_rows : 0;
  a.fresh = E.fresh ? 1 : 0;
  // status words: [0..1] scan, [2+2t, 3+2t] tier t (overflow count, errors)
  CCRDT_TRY(E.status.ensure(TRMV_STATUS_WORDS * 4 + 16));  // (+ the validation's scratch flag)
  uint32_t* status = E.status.as<uint32_t>();
  CCRDT_HIP(hipMemsetAsync(E.status.p, 0, TRMV_STATUS_WORDS * 4, E.stream));
  a.status = status;
  CCRDT_TRY(E.ex_cnt.ensure(nk * 4));
  CCRDT_TRY(E.ex.ensure(n_ops * sizeof(TrmvExtraRec)));
  CCRDT_TRY(E.ex_vc.ensure(n_ops * 8 * D));
  CCRDT_TRY(E.ex_key_ptr.ensure((nk + 1) * 8));
  for (DevBuf& d : E.tier_ovf) CCRDT_TRY(d.ensure(nk * 4));
  if (E.k <= 128) {  // tier R's per-op scratch and each key's Observed order
    CCRDT_TRY(E.op_pl.ensure(n_ops + 1));
    CCRDT_TRY(E.obs_ord.ensure(nk * TRMV_ORD * 2));
  }
  a.op_pl = E.op_pl.as<uint8_t>();
  a.obs_ord = E.obs_ord.as<uint16_t>();
  a.ex_cnt = E.ex_cnt.as<uint32_t>();
  a.ex = E.ex.as<TrmvExtraRec>();
  a.ex_vc = E.ex_vc.as<int64_t>();
  E.trmv_overflow_keys.clear();
  E.trmv_tier_ms.clear();
  // CCRDT_TRMV_INPLACE=0: every resident batch is a full rewrite (A/B knob)
  static const bool inplace_env = [] {
    const char* v = getenv("CCRDT_TRMV_INPLACE");
    return !(v && v[0] == '0');
  }();
  int first_tier = 3, n_over = 0;
  int partial = CCRDT_OK;
  if (nk && !E.fresh && E.k <= 128 && E.inplace_ready && inplace_env) {
    uint32_t handed = 0;
    CCRDT_TRY(trmv_pass_inplace(E, a, n_ops, status, handed));
    E.mcur = 1 - E.mcur;  // (meta / cap now hold the batch, except the handed-on keys)
    if (handed) {
      // the handed-on keys' ops in a full rewrite of every key (the others
      // only copied): it also compacts the arena.  Until it commits, the live
      // state (meta[mcur] over data side cur) is the batch applied to every
      // key but the handed-on ones, which kept theirs; the rewrite writes only
      // the other sides, so when it fails that state stands: a partial commit
      // (CCRDT_EPARTIAL), not a rollback -- the in-place pass already changed
      // the data arrays of the keys it completed.
      // (the list, host-side: the rewrite's own tier R overwrites tier_ovf[3])
      std::vector<uint32_t> hkeys(handed);
      CCRDT_HIP(hipMemcpy(hkeys.data(), E.tier_ovf[3].p, (size_t)handed * 4, hipMemcpyDeviceToHost));
      int rc = E.key_done.ensure(nk);
      if (rc == CCRDT_OK)
        rc = trmv_launch_mark_done(E.key_done.as<uint8_t>(), nk, E.tier_ovf[3].as<uint32_t>(), handed, nullptr,
                                   nullptr, E.stream);
      if (rc == CCRDT_OK && hipMemsetAsync(E.status.p, 0, TRMV_STATUS_WORDS * 4, E.stream) != hipSuccess)
        rc = CCRDT_EDEVICE;
      if (rc == CCRDT_OK) {
        a.key_done = E.key_done.as<uint8_t>();
        rc = trmv_pass_full(E, a, n_ops, status, first_tier, n_over);
      }
      if (rc != CCRDT_OK) {
        const std::string why = g_last_error;
        E.inplace_ready = false;  // (the next batch lays every key out again)
        // the handed-on keys listed again and their extra counts zeroed (a
        // failed rewrite may have written some): they produce no extras
        CCRDT_HIP(hipStreamSynchronize(E.stream));  // (whatever the failed rewrite queued)
        CCRDT_HIP(hipMemcpy(E.tier_ovf[3].p, hkeys.data(), (size_t)handed * 4, hipMemcpyHostToDevice));
        CCRDT_TRY(trmv_launch_mark_done(E.key_done.as<uint8_t>(), nk, E.tier_ovf[3].as<uint32_t>(), handed, nullptr,
                                        a.ex_cnt, E.stream));
        CCRDT_HIP(hipStreamSynchronize(E.stream));
        E.trmv_overflow_keys[3] = handed;
        set_error("trmv_apply: the batch committed except for " + std::to_string(handed) +
                  " key(s) the in-place pass handed on (ccrdt_engine_handed_on(e, 3)); they keep their previous "
                  "state: the full rewrite that applies their ops failed: " + why);
        partial = CCRDT_EPARTIAL;
        first_tier = 3;
        n_over = 0;
      }
    }
  } else {
    CCRDT_TRY(trmv_pass_full(E, a, n_ops, status, first_tier, n_over));
  }
  // the sum of the tiers' own intervals (tier 4 starts after a host round
  // trip, whose gap is not kernel time)
  float kernel_ms = 0.f;
  for (const auto& tm : E.trmv_tier_ms) kernel_ms += tm.second;
  CCRDT_HIP(hipMemcpyAsync(E.ex_key_ptr.p, ops->key_ptr, (nk + 1) * 8, hipMemcpyDeviceToDevice,
                           E.stream));
  E.trmv_first_tier = first_tier;
  E.fresh = false;
  E.last_n_ops = n_ops;
  E.last_kernel_ms = kernel_ms;
  if (partial != CCRDT_OK) return partial;
  if (n_over) {
    set_error("trmv_apply: " + std::to_string(n_over) +
              " key(s) would exceed the per-key capacity (" + std::to_string(trmv_steady_hbm_players()) +
              " players, 65535 Masked elements, 65534 Removals rows): they keep their previous "
              "state, the other keys committed; ccrdt_engine_handed_on(e, 4) lists them");
    return CCRDT_EKEYCAP;
  }
  return CCRDT_OK;
}

int ccrdt_trmv_set_fresh_room(ccrdt_engine* e, int on) {
  CCRDT_TRY(check_trmv(e));
  e->fresh_room = on != 0;
  return CCRDT_OK;
}

int ccrdt_trmv_replica_vc_device(ccrdt_engine* e, int64_t* d_out) {
  CCRDT_TRY(check_trmv(e));
  if (!d_out) return CCRDT_EINVAL;
  const TrmvBufs& b = e->trmv[e->cur];  // (vc lives with the data arrays)
  return trmv_launch_replica_vc(e->fresh ? nullptr : b.vc.as<int64_t>(), (uint64_t)e->n_keys,
                                e->n_dc, d_out, e->stream);
}

int ccrdt_trmv_extras_device(ccrdt_engine* e, int64_t* d_rows, int64_t cap_rows, uint32_t* d_count) {
  CCRDT_TRY(check_trmv(e));
  if (!d_rows || !d_count || cap_rows < 0) return CCRDT_EINVAL;
  const bool have = e->last_n_ops > 0 && e->ex_cnt.p;
  return trmv_launch_pack_extras(e->ex_key_ptr.as<uint64_t>(), have ? e->ex_cnt.as<uint32_t>() : nullptr,
                                 e->ex.as<TrmvExtraRec>(), e->ex_vc.as<int64_t>(),
                                 (uint64_t)e->n_keys, e->n_dc, d_rows, cap_rows, d_count, e->stream);
}

int ccrdt_trmv_exchange_pack(ccrdt_engine* e, int64_t* d_pack, int64_t cap_rows, const int64_t* d_op_map,
                             int64_t n_map, uint32_t host_word) {
  CCRDT_TRY(check_trmv(e));
  if (!d_pack || cap_rows < 0 || n_map < 0) return CCRDT_EINVAL;
  const bool have = e->last_n_ops > 0 && e->ex_cnt.p;
  const TrmvBufs& b = e->trmv[e->cur];
  return trmv_launch_exchange_pack(e->fresh ? nullptr : b.vc.as<int64_t>(), e->ex_key_ptr.as<uint64_t>(),
                                   have ? e->ex_cnt.as<uint32_t>() : nullptr, e->ex.as<TrmvExtraRec>(),
                                   e->ex_vc.as<int64_t>(), (uint64_t)e->n_keys, e->n_dc, d_pack, cap_rows, d_op_map,
                                   n_map, host_word, e->stream);
}

int ccrdt_trmv_exchange_reduce(ccrdt_engine* e, const int64_t* d_gathered, int world, int64_t len, int64_t* d_hdr,
                               int64_t* d_rows) {
  CCRDT_TRY(check_trmv(e));
  const int D = e->n_dc;
  const int64_t per = (len - 1 - D) / (6 + D);
  if (!d_gathered || !d_hdr || !d_rows || world < 1 || world > 64 || per < 0 || (int64_t)world * per > 2048) {
    set_error("trmv_exchange_reduce: bad arguments (at most 2048 gathered rows)");
    return CCRDT_EINVAL;
  }
  return trmv_launch_exchange_reduce(d_gathered, world, len, D, d_hdr, d_rows, e->stream);
}

int ccrdt_trmv_extra_count(ccrdt_engine* e, int64_t* n) {
  CCRDT_TRY(check_trmv(e));
  if (!n) return CCRDT_EINVAL;
  std::vector<uint32_t> cnt(e->n_keys);
  if (e->n_keys && e->ex_cnt.p) {
    CCRDT_HIP(hipStreamSynchronize(e->stream));
    CCRDT_HIP(hipMemcpy(cnt.data(), e->ex_cnt.p, cnt.size() * 4, hipMemcpyDeviceToHost));
  }
  int64_t s = 0;
  for (uint32_t c : cnt) s += c;
  *n = s;
  return CCRDT_OK;
}

int ccrdt_trmv_fetch_extra(ccrdt_engine* e, ccrdt_trmv_extra* x) {
  CCRDT_TRY(check_trmv(e));
  if (!x) return CCRDT_EINVAL;
  Engine& E = *e;
  const uint64_t n_ops = E.last_n_ops, nk = (uint64_t)E.n_keys;
  const int D = E.n_dc;
  if (x->kind && n_ops) host_fill(x->kind, CCRDT_NOOP, n_ops);
  if (!n_ops || !nk || !E.ex_cnt.p) return CCRDT_OK;
  // The extras are packed on the device into rows [op, kind, id, score, dc,
  // ts, vc...] (the exchange's pack kernel) and only those rows cross PCIe:
  // a batch's extras are a few per million ops, its op-indexed extra
  // buffers are n_ops records.
  const uint64_t w = 6 + (uint64_t)D;
  uint64_t cap = std::max<uint64_t>(E.st_out_vc.bytes / (w * 8), 4096);
  uint32_t cnt = 0;
  for (int pass = 0; pass < 2; ++pass) {
    CCRDT_TRY(E.st_out_vc.ensure(cap * w * 8));
    CCRDT_TRY(E.st_out_kind.ensure(4));
    CCRDT_TRY(trmv_launch_pack_extras(E.ex_key_ptr.as<uint64_t>(), E.ex_cnt.as<uint32_t>(),
                                      E.ex.as<TrmvExtraRec>(), E.ex_vc.as<int64_t>(), nk, D,
                                      E.st_out_vc.as<int64_t>(), (int64_t)cap,
                                      E.st_out_kind.as<uint32_t>(), E.stream));
    CCRDT_HIP(hipMemcpyAsync(E.h_status, E.st_out_kind.p, 4, hipMemcpyDeviceToHost, E.stream));
    CCRDT_HIP(hipStreamSynchronize(E.stream));
    memcpy(&cnt, E.h_status, 4);
    if (cnt <= cap) break;
    cap = cnt;  // (a second pass packs them all)
  }
  if (!cnt) return CCRDT_OK;
  std::vector<int64_t> rows((size_t)cnt * w);
  CCRDT_HIP(hipMemcpy(rows.data(), E.st_out_vc.p, rows.size() * 8, hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < cnt; ++i) {
    const int64_t* r = &rows[i * w];
    const uint64_t op = (uint64_t)r[0];
    if (op >= n_ops) continue;
    if (x->kind) x->kind[op] = (uint8_t)r[1];
    if (x->id) x->id[op] = r[2];
    if (x->score) x->score[op] = r[3];
    if (x->dc) x->dc[op] = (uint8_t)r[4];
    if (x->ts) x->ts[op] = r[5];
    if (x->vc && r[1] == CCRDT_TRMV_RMV)
      for (int d = 0; d < D; ++d) x->vc[op * D + d] = r[6 + d];
  }
  return CCRDT_OK;
}

int ccrdt_trmv_apply(ccrdt_engine* e, const ccrdt_trmv_ops* ops, ccrdt_trmv_extra* extra) {
  CCRDT_TRY(check_trmv(e));
  if (!ops || !ops->key_ptr) {
    set_error("trmv_apply: null ops");
    return CCRDT_EINVAL;
  }
  Engine& E = *e;
  const uint64_t nk = (uint64_t)E.n_keys, n = (uint64_t)ops->n_ops;
  const int D = E.n_dc;
  // CCRDT_STAGE_TRACE=1: host-side phase times of this call on stderr
  static const bool trace = std::getenv("CCRDT_STAGE_TRACE") != nullptr;
  double tp[6] = {};
  int ti = 0;
  const auto t0 = std::chrono::steady_clock::now();
  auto mark = [&] {
    if (trace) tp[ti++] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  };
  // CSR shape checks (host side; values are validated by the kernel)
  if (ops->key_ptr[0] != 0 || ops->key_ptr[nk] != n) {
    set_error("trmv_apply: key_ptr must start at 0 and end at n_ops");
    return CCRDT_EINVAL;
  }
  for (uint64_t k = 0; k < nk; ++k)
    if (ops->key_ptr[k + 1] < ops->key_ptr[k]) {
      set_error("trmv_apply: key_ptr not monotone");
      return CCRDT_EINVAL;
    }
  const uint64_t nr = ops->rmv_vc ? (uint64_t)ops->n_rmv_rows : 0;
  CCRDT_TRY(E.st_kp.ensure((nk + 1) * 8));
  CCRDT_TRY(E.st_kind.ensure(n));
  CCRDT_TRY(E.st_id.ensure(n * 8));
  CCRDT_TRY(E.st_score.ensure(n * 8));
  CCRDT_TRY(E.st_dc.ensure(n));
  CCRDT_TRY(E.st_ts.ensure(n * 8));
  CCRDT_TRY(E.st_rvc.ensure(nr * D * 8));
  // (pageable caller memory: through the pinned staging slots, staging.cpp)
  mark();
  CCRDT_TRY(h2d_staged(E, E.st_kp.p, ops->key_ptr, (nk + 1) * 8));
  int up = n ? h2d_trmv_ops(E, n, ops->kind, ops->id, ops->score, ops->dc, ops->ts, E.st_kind.as<uint8_t>(),
                            E.st_dc.as<uint8_t>(), E.st_id.as<int64_t>(), E.st_score.as<int64_t>(),
                            E.st_ts.as<int64_t>(), E.st_n32[0], E.st_nbase[2])
               : CCRDT_OK;
  if (up != CCRDT_OK && up != CCRDT_ERANGE) return up;
  if (up == CCRDT_ERANGE) {  // a value leaves int32: column by column
    CCRDT_TRY(h2d_staged(E, E.st_kind.p, ops->kind, n));
    // Ids, Scores and Ts cross as int32 when they fit (Ts relative to a
    // per-chunk base), widened on the device; else as they are
    CCRDT_TRY(h2d_staged_i64(E, E.st_id.as<int64_t>(), ops->id, n, nullptr, nullptr, 0, E.st_n32[0], E.st_nbase[0]));
    CCRDT_TRY(h2d_staged_i64(E, E.st_score.as<int64_t>(), ops->score, n, nullptr, nullptr, 1, E.st_n32[1],
                             E.st_nbase[1]));
    CCRDT_TRY(h2d_staged(E, E.st_dc.p, ops->dc, n));
    CCRDT_TRY(h2d_staged_i64(E, E.st_ts.as<int64_t>(), ops->ts, n, ops->kind, E.st_kind.as<uint8_t>(), 2, E.st_n32[2],
                             E.st_nbase[2]));
  }
  mark();
  // removal clocks as int32 relative to a per-chunk base when they fit
  if (nr)
    CCRDT_TRY(h2d_staged_i64(E, E.st_rvc.as<int64_t>(), ops->rmv_vc, nr * D, nullptr, nullptr, 1, E.st_n32[1],
                             E.st_nbase[1], true));
  ccrdt_trmv_ops d = *ops;
  d.key_ptr = E.st_kp.as<uint64_t>();
  d.kind = E.st_kind.as<uint8_t>();
  d.id = E.st_id.as<int64_t>();
  d.score = E.st_score.as<int64_t>();
  d.dc = E.st_dc.as<uint8_t>();
  d.ts = E.st_ts.as<int64_t>();
  d.rmv_vc = nr ? E.st_rvc.as<int64_t>() : nullptr;
  d.n_rmv_rows = (int64_t)nr;
  mark();
  const int rc = ccrdt_trmv_apply_device(e, &d);
  mark();
  if (rc != CCRDT_OK && rc != CCRDT_EKEYCAP && rc != CCRDT_EPARTIAL) return rc;
  if (extra) {  // EKEYCAP / EPARTIAL: the batch committed (but for some keys); its extras are fetched too
    const std::string msg = g_last_error;
    CCRDT_TRY(ccrdt_trmv_fetch_extra(e, extra));
    if (rc != CCRDT_OK) set_error(msg);
  }
  mark();
  if (trace)
    std::fprintf(stderr, "trmv_apply: checks %.2f | key_ptr + ops staged %.2f | rmv clocks staged %.2f | "
                 "apply (waits the DMAs) %.2f | extras %.2f ms\n", tp[0], tp[1] - tp[0], tp[2] - tp[1],
                 tp[3] - tp[2], tp[4] - tp[3]);
  return rc;
}

// ---- state image conversion

namespace {
struct HostTrmv {
  std::vector<KeyMeta> meta;
  std::vector<int64_t> pl_id, m_score, m_ts, r_vc, vc;
  std::vector<uint32_t> pl_info, pl_slab;
  std::vector<uint16_t> pl_gb;
  std::vector<uint8_t> m_dc;
};

// Keys [k0, k1) of the resident state -> host, offsets rebased to the range
// (segments of consecutive keys are consecutive: the capacity scan and the
// import lay them out in key order).
int download_trmv(Engine& E, HostTrmv& h, uint64_t k0, uint64_t k1) {
  const uint64_t n = k1 - k0;
  const int D = E.n_dc;
  h.meta.assign(n, KeyMeta{0, 0, 0, 0, 0, 0, 0, NONE32});
  h.vc.assign(n * D, 0);
  h.pl_id.clear();
  h.pl_info.clear();
  h.pl_slab.clear();
  h.m_score.clear();
  h.m_ts.clear();
  h.m_dc.clear();
  h.r_vc.clear();
  if (E.fresh || !n) return CCRDT_OK;
  CCRDT_HIP(hipStreamSynchronize(E.stream));
  const TrmvBufs& b = E.trmv[E.cur];
  CCRDT_HIP(hipMemcpy(h.meta.data(), E.trmv[E.mcur].meta.as<KeyMeta>() + k0, n * sizeof(KeyMeta),
                      hipMemcpyDeviceToHost));
  CCRDT_HIP(hipMemcpy(h.vc.data(), b.vc.as<int64_t>() + k0 * D, n * D * 8, hipMemcpyDeviceToHost));
  // (segments lie anywhere in the arena: the range's extent is min..max)
  uint64_t p0 = UINT64_MAX, r0 = UINT64_MAX, m0 = UINT64_MAX, p1 = 0, r1 = 0;
  for (const KeyMeta& m : h.meta) {
    if (m.np) p0 = std::min<uint64_t>(p0, m.p_off), p1 = std::max<uint64_t>(p1, (uint64_t)m.p_off + m.np);
    if (m.nr) r0 = std::min<uint64_t>(r0, m.r_off), r1 = std::max<uint64_t>(r1, (uint64_t)m.r_off + m.nr);
    if (m.np) m0 = std::min<uint64_t>(m0, m.m_off);
  }
  if (p0 == UINT64_MAX) p0 = p1 = 0;
  if (r0 == UINT64_MAX) r0 = r1 = 0;
  if (m0 == UINT64_MAX) m0 = 0;
  const uint64_t np = p1 - p0, nr = r1 - r0;
  h.pl_id.resize(np);
  h.pl_info.resize(np);
  h.pl_slab.resize(np);
  if (np) {
    CCRDT_HIP(hipMemcpy(h.pl_id.data(), b.pl_id.as<int64_t>() + p0, np * 8, hipMemcpyDeviceToHost));
    CCRDT_HIP(hipMemcpy(h.pl_info.data(), b.pl_info.as<uint32_t>() + p0, np * 4, hipMemcpyDeviceToHost));
    CCRDT_HIP(hipMemcpy(h.pl_slab.data(), b.pl_slab.as<uint32_t>() + p0, np * 4, hipMemcpyDeviceToHost));
  }
  uint64_t m1 = m0;
  for (const KeyMeta& m : h.meta)
    for (uint32_t p = 0; p < m.np; ++p) {
      const uint32_t sl = h.pl_slab[m.p_off - p0 + p];
      m1 = std::max<uint64_t>(m1, (uint64_t)m.m_off + (sl & 0xFFFFu) + (sl >> 16));
    }
  const uint64_t nm = m1 - m0;
  h.m_score.resize(nm);
  h.m_ts.resize(nm);
  h.m_dc.resize(nm);
  h.r_vc.resize(nr * D);
  if (nm) {
    CCRDT_HIP(hipMemcpy(h.m_score.data(), b.m_score.as<int64_t>() + m0, nm * 8, hipMemcpyDeviceToHost));
    CCRDT_HIP(hipMemcpy(h.m_ts.data(), b.m_ts.as<int64_t>() + m0, nm * 8, hipMemcpyDeviceToHost));
    CCRDT_HIP(hipMemcpy(h.m_dc.data(), b.m_dc.as<uint8_t>() + m0, nm, hipMemcpyDeviceToHost));
  }
  if (nr)
    CCRDT_HIP(hipMemcpy(h.r_vc.data(), b.r_vc.as<int64_t>() + r0 * D, nr * D * 8, hipMemcpyDeviceToHost));
  for (KeyMeta& m : h.meta) {  // (keys without players / rows keep offsets nothing reads)
    m.p_off = m.np ? m.p_off - (uint32_t)p0 : 0u;
    m.m_off = m.np ? m.m_off - (uint32_t)m0 : 0u;
    m.r_off = m.nr ? m.r_off - (uint32_t)r0 : 0u;
  }
  return CCRDT_OK;
}
}  // namespace

int ccrdt_trmv_state_sizes(ccrdt_engine* e, int64_t* n_obs, int64_t* n_masked, int64_t* n_rows) {
  CCRDT_TRY(check_trmv(e));
  return ccrdt_trmv_range_sizes(e, 0, e->n_keys, n_obs, n_masked, n_rows);
}

int ccrdt_trmv_key_sizes(ccrdt_engine* e, uint32_t* np, uint32_t* nm, uint32_t* nr, uint32_t* nobs) {
  CCRDT_TRY(check_trmv(e));
  const uint64_t nk = (uint64_t)e->n_keys;
  std::vector<KeyMeta> meta(nk);
  if (!e->fresh && nk) {
    CCRDT_HIP(hipStreamSynchronize(e->stream));
    CCRDT_HIP(hipMemcpy(meta.data(), e->trmv[e->mcur].meta.p, nk * sizeof(KeyMeta),
                        hipMemcpyDeviceToHost));
  }
  for (uint64_t k = 0; k < nk; ++k) {
    const KeyMeta m = e->fresh ? KeyMeta{} : meta[k];
    if (np) np[k] = m.np;
    if (nm) nm[k] = m.nm;
    if (nr) nr[k] = m.nr;
    if (nobs) nobs[k] = m.nobs;
  }
  return CCRDT_OK;
}

int ccrdt_engine_handed_on(ccrdt_engine* e, int t, uint32_t* keys, int64_t cap, int64_t* n) {
  if (!e || !n || cap < 0) return CCRDT_EINVAL;
  const int ti = t >= 0 && t < TRMV_N_TIERS ? t : -1;
  auto it = e->trmv_overflow_keys.find(t);
  if (ti < 0 || e->type != CCRDT_TOPK_RMV || it == e->trmv_overflow_keys.end()) {
    *n = 0;
    return ti < 0 ? CCRDT_EINVAL : CCRDT_OK;
  }
  *n = it->second;
  const int64_t m = std::min<int64_t>(cap, *n);
  if (m > 0 && keys) {
    const DevBuf& src = e->tier_ovf[ti];
    CCRDT_HIP(hipStreamSynchronize(e->stream));
    CCRDT_HIP(hipMemcpy(keys, src.p, (size_t)m * 4, hipMemcpyDeviceToHost));
  }
  return CCRDT_OK;
}

int ccrdt_trmv_export(ccrdt_engine* e, ccrdt_trmv_state* out) {
  CCRDT_TRY(check_trmv(e));
  return ccrdt_trmv_export_range(e, 0, e->n_keys, out);
}

int ccrdt_trmv_range_sizes(ccrdt_engine* e, int64_t k0, int64_t k1, int64_t* n_obs, int64_t* n_masked,
                           int64_t* n_rows) {
  CCRDT_TRY(check_trmv(e));
  if (k0 < 0 || k1 < k0 || k1 > e->n_keys) {
    set_error("trmv_range_sizes: bad key range");
    return CCRDT_EINVAL;
  }
  int64_t o = 0, m = 0, r = 0;
  if (!e->fresh && k1 > k0) {
    std::vector<KeyMeta> meta(k1 - k0);
    CCRDT_HIP(hipStreamSynchronize(e->stream));
    CCRDT_HIP(hipMemcpy(meta.data(), e->trmv[e->mcur].meta.as<KeyMeta>() + k0, meta.size() * sizeof(KeyMeta),
                        hipMemcpyDeviceToHost));
    for (const KeyMeta& k : meta) {
      o += k.nobs;
      m += k.nm;
      r += k.nr;
    }
  }
  if (n_obs) *n_obs = o;
  if (n_masked) *n_masked = m;
  if (n_rows) *n_rows = r;
  return CCRDT_OK;
}

int ccrdt_trmv_export_range(ccrdt_engine* e, int64_t k0, int64_t k1, ccrdt_trmv_state* out) {
  CCRDT_TRY(check_trmv(e));
  if (!out || k0 < 0 || k1 < k0 || k1 > e->n_keys) {
    set_error("trmv_export_range: bad arguments");
    return CCRDT_EINVAL;
  }
  HostTrmv h;
  CCRDT_TRY(download_trmv(*e, h, (uint64_t)k0, (uint64_t)k1));
  const uint64_t nk = (uint64_t)(k1 - k0);
  const int D = e->n_dc;
  // per key: |Observed|, |Masked|, |Removals| -> the output offsets; then every
  // key sorted into the canonical order and written, key ranges on host
  // threads (a 2^20-key state of 370M Masked elements took ~40 s on one)
  std::vector<uint64_t> po(nk + 1, 0), pm(nk + 1, 0), pr(nk + 1, 0);
  for_key_ranges_host(nk, [&](uint64_t b, uint64_t e2) {
    for (uint64_t k = b; k < e2; ++k) {
      const KeyMeta& m = h.meta[k];
      uint64_t o = 0, ms = 0, r = 0;
      for (uint32_t p = 0; p < m.np; ++p) {
        const uint64_t pp = (uint64_t)m.p_off + p;
        const uint32_t info = h.pl_info[pp];
        ms += h.pl_slab[pp] >> 16;
        o += (info & 0xFFFFu) != NONE16 ? 1u : 0u;
        r += (info >> 16) != NONE16 ? 1u : 0u;
      }
      po[k + 1] = o;
      pm[k + 1] = ms;
      pr[k + 1] = r;
    }
  });
  for (uint64_t k = 0; k < nk; ++k) {
    po[k + 1] += po[k];
    pm[k + 1] += pm[k];
    pr[k + 1] += pr[k];
  }
  for (uint64_t k = 0; k <= nk; ++k) {
    if (out->obs_ptr) out->obs_ptr[k] = po[k];
    if (out->m_ptr) out->m_ptr[k] = pm[k];
    if (out->r_ptr) out->r_ptr[k] = pr[k];
  }
  struct E4 {
    int64_t id, score;
    uint8_t dc;
    int64_t ts;
  };
  for_key_ranges_host(nk, [&](uint64_t b, uint64_t e2) {
    std::vector<E4> obs, msk;
    std::vector<std::pair<int64_t, uint32_t>> rows;
    for (uint64_t k = b; k < e2; ++k) {
      const KeyMeta& m = h.meta[k];
      if (out->vc)
        for (int d = 0; d < D; ++d) out->vc[k * D + d] = h.vc[k * D + d];
      obs.clear();
      msk.clear();
      rows.clear();
      int64_t mid = 0, msc = 0, mts = 0;
      uint8_t mdc = 0;
      for (uint32_t p = 0; p < m.np; ++p) {
        const uint64_t pp = (uint64_t)m.p_off + p;
        const uint32_t info = h.pl_info[pp], slab = h.pl_slab[pp];
        const int64_t id = h.pl_id[pp];
        const uint64_t g0 = (uint64_t)m.m_off + (slab & 0xFFFFu);
        for (uint32_t j = 0; j < (slab >> 16); ++j)
          msk.push_back({id, h.m_score[g0 + j], h.m_dc[g0 + j], h.m_ts[g0 + j]});
        const uint32_t o = info & 0xFFFFu, r = info >> 16;
        if (o != NONE16) {
          obs.push_back({id, h.m_score[g0 + o], h.m_dc[g0 + o], h.m_ts[g0 + o]});
          if (p == m.minq) {
            mid = id;
            msc = h.m_score[g0 + o];
            mts = h.m_ts[g0 + o];
            mdc = h.m_dc[g0 + o];
          }
        }
        if (r != NONE16) rows.push_back({id, r});
      }
      std::sort(obs.begin(), obs.end(), [](const E4& a, const E4& c) { return a.id < c.id; });
      std::sort(msk.begin(), msk.end(), [](const E4& a, const E4& c) {
        return std::tie(a.id, a.score, a.dc, a.ts) < std::tie(c.id, c.score, c.dc, c.ts);
      });
      std::sort(rows.begin(), rows.end());
      uint64_t qo = po[k], qm = pm[k], qr = pr[k];
      for (const E4& x : obs) {
        if (out->obs_id) out->obs_id[qo] = x.id;
        if (out->obs_score) out->obs_score[qo] = x.score;
        if (out->obs_dc) out->obs_dc[qo] = x.dc;
        if (out->obs_ts) out->obs_ts[qo] = x.ts;
        ++qo;
      }
      for (const E4& x : msk) {
        if (out->m_id) out->m_id[qm] = x.id;
        if (out->m_score) out->m_score[qm] = x.score;
        if (out->m_dc) out->m_dc[qm] = x.dc;
        if (out->m_ts) out->m_ts[qm] = x.ts;
        ++qm;
      }
      for (const auto& [id, r] : rows) {
        if (out->r_id) out->r_id[qr] = id;
        if (out->r_vc)
          for (int d = 0; d < D; ++d) out->r_vc[qr * D + d] = h.r_vc[((uint64_t)m.r_off + r) * D + d];
        ++qr;
      }
      const bool mv = m.minq != NONE32;
      if (out->min_valid) out->min_valid[k] = mv ? 1 : 0;
      if (out->min_id) out->min_id[k] = mid;
      if (out->min_score) out->min_score[k] = msc;
      if (out->min_ts) out->min_ts[k] = mts;
      if (out->min_dc) out->min_dc[k] = mdc;
    }
  });
  return CCRDT_OK;
}

int ccrdt_trmv_import(ccrdt_engine* e, const ccrdt_trmv_state* in) {
  CCRDT_TRY(check_trmv(e));
  if (!in || !in->vc || !in->obs_ptr || !in->m_ptr || !in->r_ptr || !in->min_valid) {
    set_error("trmv_import: missing arrays");
    return CCRDT_EINVAL;
  }
  Engine& E = *e;
  const uint64_t nk = (uint64_t)E.n_keys;
  const int D = E.n_dc;
  HostTrmv h;
  h.meta.resize(nk);
  h.vc.assign(in->vc, in->vc + nk * D);
  for (int64_t v : h.vc)
    if (v < 0) {
      set_error("trmv_import: negative Vc entry");
      return CCRDT_ERANGE;
    }
  struct E3 {
    int64_t score;
    uint8_t dc;
    int64_t ts;
  };
  std::vector<int64_t> ids;
  std::vector<std::vector<E3>> per;
  for (uint64_t k = 0; k < nk; ++k) {
    KeyMeta m{};
    m.p_off = (uint32_t)h.pl_id.size();
    m.m_off = (uint32_t)h.m_score.size();
    m.r_off = (uint32_t)(h.r_vc.size() / D);
    ids.clear();
    for (uint64_t i = in->m_ptr[k]; i < in->m_ptr[k + 1]; ++i) ids.push_back(in->m_id[i]);
    for (uint64_t i = in->r_ptr[k]; i < in->r_ptr[k + 1]; ++i) ids.push_back(in->r_id[i]);
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    const uint64_t nmk = in->m_ptr[k + 1] - in->m_ptr[k], nrk = in->r_ptr[k + 1] - in->r_ptr[k];
    if (ids.size() > trmv_steady_hbm_players() || nmk > TRMV_SEG_MAX || nrk >= NONE16) {
      set_error("trmv_import: key exceeds per-key capacity (players, 65535 Masked elements, 65534 Removals rows)");
      return CCRDT_ENOMEM;
    }
    auto pidx = [&](int64_t id) -> uint32_t {
      auto it = std::lower_bound(ids.begin(), ids.end(), id);
      return (it != ids.end() && *it == id) ? (uint32_t)(it - ids.begin()) : NONE32;
    };
    per.assign(ids.size(), {});
    for (uint64_t i = in->m_ptr[k]; i < in->m_ptr[k + 1]; ++i) {
      if (in->m_dc[i] >= D || in->m_ts[i] < 1) {
        set_error("trmv_import: Masked element with bad dc or ts < 1");
        return CCRDT_ERANGE;
      }
      per[pidx(in->m_id[i])].push_back({in->m_score[i], in->m_dc[i], in->m_ts[i]});
    }
    std::vector<uint32_t> info(ids.size(), NONE32), slab(ids.size(), 0);
    std::vector<uint16_t> gb(ids.size(), 0);
    uint32_t off = 0;
    for (size_t q = 0; q < ids.size(); ++q) {
      slab[q] = off | ((uint32_t)per[q].size() << 16);
      for (size_t j = 1; j < per[q].size(); ++j) {  // gb_sets:largest: (Score, DcId, Ts)
        const E3& x = per[q][j];
        const E3& y = per[q][gb[q]];
        if (std::tie(x.score, x.dc, x.ts) > std::tie(y.score, y.dc, y.ts)) gb[q] = (uint16_t)j;
      }
      for (const E3& x : per[q]) {
        h.m_score.push_back(x.score);
        h.m_dc.push_back(x.dc);
        h.m_ts.push_back(x.ts);
      }
      off += (uint32_t)per[q].size();
    }
    for (uint64_t i = in->r_ptr[k]; i < in->r_ptr[k + 1]; ++i) {
      const uint32_t q = pidx(in->r_id[i]);
      if ((info[q] >> 16) != NONE16) {
        set_error("trmv_import: duplicate Removals Id");
        return CCRDT_EINVAL;
      }
      info[q] = (info[q] & 0xFFFFu) | ((uint32_t)(i - in->r_ptr[k]) << 16);
      for (int d = 0; d < D; ++d) {
        const int64_t v = in->r_vc[i * D + d];
        if (v < 0) {
          set_error("trmv_import: negative Removals entry");
          return CCRDT_ERANGE;
        }
        h.r_vc.push_back(v);
      }
    }
    uint32_t nobs = 0;
    for (uint64_t i = in->obs_ptr[k]; i < in->obs_ptr[k + 1]; ++i) {
      // Observed ⊆ Masked: find the element in the player's slab
      const uint32_t q = pidx(in->obs_id[i]);
      uint32_t found = NONE32;
      for (size_t j = 0; q != NONE32 && j < per[q].size(); ++j)
        if (per[q][j].score == in->obs_score[i] && per[q][j].ts == in->obs_ts[i] &&
            per[q][j].dc == in->obs_dc[i]) {
          found = (uint32_t)j;
          break;
        }
      if (found == NONE32) {
        set_error("trmv_import: Observed element not in Masked");
        return CCRDT_EINVAL;
      }
      if ((info[q] & 0xFFFFu) != NONE16) {
        set_error("trmv_import: duplicate Observed Id");
        return CCRDT_EINVAL;
      }
      info[q] = (info[q] & 0xFFFF0000u) | found;
      ++nobs;
    }
    if ((int64_t)nobs > E.k) {
      set_error("trmv_import: |Observed| > Size");
      return CCRDT_EINVAL;
    }
    m.minq = NONE32;
    if (in->min_valid[k]) {
      const uint32_t q = pidx(in->min_id[k]);
      const uint32_t o = q != NONE32 ? (info[q] & 0xFFFFu) : NONE16;
      if (o == NONE16 || per[q][o].score != in->min_score[k] || per[q][o].ts != in->min_ts[k]) {
        set_error("trmv_import: Min is not an Observed element");
        return CCRDT_EINVAL;
      }
      m.minq = q;
    } else if (nobs) {
      set_error("trmv_import: Min is nil but Observed is not empty");
      return CCRDT_EINVAL;
    }
    for (size_t q = 0; q < ids.size(); ++q) {
      h.pl_id.push_back(ids[q]);
      h.pl_info.push_back(info[q]);
      h.pl_slab.push_back(slab[q]);
      h.pl_gb.push_back(gb[q]);
    }
    m.np = (uint32_t)ids.size();
    m.nm = (uint32_t)nmk;
    m.nr = (uint32_t)nrk;
    m.nobs = nobs;
    h.meta[k] = m;
  }
  TrmvBufs& b = E.trmv[E.cur];
  DevBuf& bmeta = E.trmv[E.mcur].meta;
  CCRDT_TRY(bmeta.ensure(nk * sizeof(KeyMeta)));
  CCRDT_TRY(b.vc.ensure(nk * D * 8));
  CCRDT_TRY(b.pl_id.ensure(h.pl_id.size() * 8));
  CCRDT_TRY(b.pl_info.ensure(h.pl_info.size() * 4));
  CCRDT_TRY(b.pl_slab.ensure(h.pl_slab.size() * 4));
  CCRDT_TRY(b.pl_gb.ensure(h.pl_gb.size() * 2));
  CCRDT_TRY(b.m_score.ensure(h.m_score.size() * 8));
  CCRDT_TRY(b.m_ts.ensure(h.m_ts.size() * 8));
  CCRDT_TRY(b.m_dc.ensure(h.m_dc.size()));
  CCRDT_TRY(b.r_vc.ensure(h.r_vc.size() * 8));
  CCRDT_HIP(hipStreamSynchronize(E.stream));
  if (nk) {
    CCRDT_HIP(hipMemcpy(bmeta.p, h.meta.data(), nk * sizeof(KeyMeta), hipMemcpyHostToDevice));
    CCRDT_HIP(hipMemcpy(b.vc.p, h.vc.data(), nk * D * 8, hipMemcpyHostToDevice));
  }
  if (!h.pl_id.empty()) {
    CCRDT_HIP(hipMemcpy(b.pl_id.p, h.pl_id.data(), h.pl_id.size() * 8, hipMemcpyHostToDevice));
    CCRDT_HIP(hipMemcpy(b.pl_info.p, h.pl_info.data(), h.pl_info.size() * 4, hipMemcpyHostToDevice));
    CCRDT_HIP(hipMemcpy(b.pl_slab.p, h.pl_slab.data(), h.pl_slab.size() * 4, hipMemcpyHostToDevice));
    CCRDT_HIP(hipMemcpy(b.pl_gb.p, h.pl_gb.data(), h.pl_gb.size() * 2, hipMemcpyHostToDevice));
  }
  if (!h.m_score.empty()) {
    CCRDT_HIP(hipMemcpy(b.m_score.p, h.m_score.data(), h.m_score.size() * 8, hipMemcpyHostToDevice));
    CCRDT_HIP(hipMemcpy(b.m_ts.p, h.m_ts.data(), h.m_ts.size() * 8, hipMemcpyHostToDevice));
    CCRDT_HIP(hipMemcpy(b.m_dc.p, h.m_dc.data(), h.m_dc.size(), hipMemcpyHostToDevice));
  }
  if (!h.r_vc.empty())
    CCRDT_HIP(hipMemcpy(b.r_vc.p, h.r_vc.data(), h.r_vc.size() * 8, hipMemcpyHostToDevice));
  E.trmv_tot[E.cur][0] = h.pl_id.size();
  E.trmv_tot[E.cur][1] = h.m_score.size();
  E.trmv_tot[E.cur][2] = h.r_vc.size() / D;
  E.fresh = false;
  E.inplace_ready = false;  // (the imported layout has no room to grow: the next batch rewrites every key)
  return CCRDT_OK;
}

int ccrdt_trmv_import_range(ccrdt_engine* e, int64_t k0, int64_t k1, const ccrdt_trmv_state* in) {
  CCRDT_TRY(check_trmv(e));
  if (!in || !in->vc || !in->obs_ptr || !in->m_ptr || !in->r_ptr || !in->min_valid || k0 < 0 || k1 < k0 ||
      k1 > e->n_keys) {
    set_error("trmv_import_range: bad arguments");
    return CCRDT_EINVAL;
  }
  // the whole image with keys [k0, k1) replaced, imported at once (the
  // import validates and lays out every key); O(n_keys) host work
  const uint64_t nk = (uint64_t)e->n_keys, n = (uint64_t)(k1 - k0);
  const int D = e->n_dc;
  int64_t no = 0, nm = 0, nr = 0;
  CCRDT_TRY(ccrdt_trmv_state_sizes(e, &no, &nm, &nr));
  struct Img {
    std::vector<int64_t> vc, obs_id, obs_score, obs_ts, m_id, m_score, m_ts, r_id, r_vc, min_id, min_score,
        min_ts;
    std::vector<uint64_t> obs_ptr, m_ptr, r_ptr;
    std::vector<uint8_t> obs_dc, m_dc, min_valid, min_dc;
    ccrdt_trmv_state view() {
      return ccrdt_trmv_state{vc.data(), obs_ptr.data(), obs_id.data(), obs_score.data(), obs_ts.data(),
                              obs_dc.data(), m_ptr.data(), m_id.data(), m_score.data(), m_ts.data(),
                              m_dc.data(), r_ptr.data(), r_id.data(), r_vc.data(), min_valid.data(),
                              min_id.data(), min_score.data(), min_ts.data(), min_dc.data()};
    }
    void size(uint64_t k, uint64_t o, uint64_t m, uint64_t r, int d) {
      vc.resize(k * d);
      obs_ptr.resize(k + 1);
      m_ptr.resize(k + 1);
      r_ptr.resize(k + 1);
      obs_id.resize(o), obs_score.resize(o), obs_ts.resize(o), obs_dc.resize(o);
      m_id.resize(m), m_score.resize(m), m_ts.resize(m), m_dc.resize(m);
      r_id.resize(r), r_vc.resize(r * d);
      min_valid.resize(k), min_id.resize(k), min_score.resize(k), min_ts.resize(k), min_dc.resize(k);
    }
  } cur, out;
  cur.size(nk, (uint64_t)no, (uint64_t)nm, (uint64_t)nr, D);
  ccrdt_trmv_state cv = cur.view();
  CCRDT_TRY(ccrdt_trmv_export(e, &cv));
  const uint64_t io = in->obs_ptr[n], im = in->m_ptr[n], ir = in->r_ptr[n];
  const uint64_t ro = cur.obs_ptr[k1] - cur.obs_ptr[k0], rm = cur.m_ptr[k1] - cur.m_ptr[k0],
                 rr = cur.r_ptr[k1] - cur.r_ptr[k0];
  out.size(nk, no - ro + io, nm - rm + im, nr - rr + ir, D);
  uint64_t po = 0, pm = 0, pr = 0;
  out.obs_ptr[0] = out.m_ptr[0] = out.r_ptr[0] = 0;
  for (uint64_t k = 0; k < nk; ++k) {
    const bool mine = k >= (uint64_t)k0 && k < (uint64_t)k1;
    const uint64_t j = mine ? k - k0 : k;
    auto take = [&](const uint64_t* sp, const int64_t* id, const int64_t* sc, const int64_t* ts,
                    const uint8_t* dc, std::vector<int64_t>& oid, std::vector<int64_t>& osc,
                    std::vector<int64_t>& ots, std::vector<uint8_t>& odc, uint64_t& p) {
      for (uint64_t i = sp[j]; i < sp[j + 1]; ++i, ++p) {
        oid[p] = id[i];
        osc[p] = sc[i];
        ots[p] = ts[i];
        odc[p] = dc[i];
      }
    };
    if (mine) {
      take(in->obs_ptr, in->obs_id, in->obs_score, in->obs_ts, in->obs_dc, out.obs_id, out.obs_score,
           out.obs_ts, out.obs_dc, po);
      take(in->m_ptr, in->m_id, in->m_score, in->m_ts, in->m_dc, out.m_id, out.m_score, out.m_ts, out.m_dc,
           pm);
      for (uint64_t i = in->r_ptr[j]; i < in->r_ptr[j + 1]; ++i, ++pr) {
        out.r_id[pr] = in->r_id[i];
        for (int d = 0; d < D; ++d) out.r_vc[pr * D + d] = in->r_vc[i * D + d];
      }
      for (int d = 0; d < D; ++d) out.vc[k * D + d] = in->vc[j * D + d];
      out.min_valid[k] = in->min_valid[j];
      out.min_id[k] = in->min_id ? in->min_id[j] : 0;
      out.min_score[k] = in->min_score ? in->min_score[j] : 0;
      out.min_ts[k] = in->min_ts ? in->min_ts[j] : 0;
      out.min_dc[k] = in->min_dc ? in->min_dc[j] : 0;
    } else {
      take(cur.obs_ptr.data(), cur.obs_id.data(), cur.obs_score.data(), cur.obs_ts.data(), cur.obs_dc.data(),
           out.obs_id, out.obs_score, out.obs_ts, out.obs_dc, po);
      take(cur.m_ptr.data(), cur.m_id.data(), cur.m_score.data(), cur.m_ts.data(), cur.m_dc.data(), out.m_id,
           out.m_score, out.m_ts, out.m_dc, pm);
      for (uint64_t i = cur.r_ptr[k]; i < cur.r_ptr[k + 1]; ++i, ++pr) {
        out.r_id[pr] = cur.r_id[i];
        for (int d = 0; d < D; ++d) out.r_vc[pr * D + d] = cur.r_vc[i * D + d];
      }
      for (int d = 0; d < D; ++d) out.vc[k * D + d] = cur.vc[k * D + d];
      out.min_valid[k] = cur.min_valid[k];
      out.min_id[k] = cur.min_id[k];
      out.min_score[k] = cur.min_score[k];
      out.min_ts[k] = cur.min_ts[k];
      out.min_dc[k] = cur.min_dc[k];
    }
    out.obs_ptr[k + 1] = po;
    out.m_ptr[k + 1] = pm;
    out.r_ptr[k + 1] = pr;
  }
  const ccrdt_trmv_state ov = out.view();
  return ccrdt_trmv_import(e, &ov);
}

int ccrdt_trmv_downstream(ccrdt_engine* e, int64_t n, const uint64_t* key, const uint8_t* op,
                          const int64_t* id, const int64_t* score, const uint8_t* dc,
                          const int64_t* ts, uint8_t* out_kind, int64_t* out_vc) {
  CCRDT_TRY(check_trmv(e));
  if (n < 0 || (n > 0 && (!key || !op || !id || !score || !dc || !ts || !out_kind))) {
    set_error("trmv_downstream: null arrays");
    return CCRDT_EINVAL;
  }
  Engine& E = *e;
  const int D = E.n_dc;
  for (int64_t i = 0; i < n; ++i) {
    if (key[i] >= (uint64_t)E.n_keys || op[i] > 1 || (op[i] == 0 && (dc[i] >= D || ts[i] < 1))) {
      set_error("trmv_downstream: bad request (key, op, dc or ts)");
      return CCRDT_EINVAL;
    }
  }
  if (n == 0) return CCRDT_OK;
  const uint64_t un = (uint64_t)n;
  CCRDT_TRY(E.st_kp.ensure(un * 8));
  CCRDT_TRY(E.st_kind.ensure(un));
  CCRDT_TRY(E.st_id.ensure(un * 8));
  CCRDT_TRY(E.st_score.ensure(un * 8));
  CCRDT_TRY(E.st_dc.ensure(un));
  CCRDT_TRY(E.st_ts.ensure(un * 8));
  CCRDT_TRY(E.st_out_kind.ensure(un));
  CCRDT_TRY(E.st_out_vc.ensure(un * D * 8));
  CCRDT_HIP(hipMemcpyAsync(E.st_kp.p, key, un * 8, hipMemcpyHostToDevice, E.stream));
  CCRDT_HIP(hipMemcpyAsync(E.st_kind.p, op, un, hipMemcpyHostToDevice, E.stream));
  CCRDT_HIP(hipMemcpyAsync(E.st_id.p, id, un * 8, hipMemcpyHostToDevice, E.stream));
  CCRDT_HIP(hipMemcpyAsync(E.st_score.p, score, un * 8, hipMemcpyHostToDevice, E.stream));
  CCRDT_HIP(hipMemcpyAsync(E.st_dc.p, dc, un, hipMemcpyHostToDevice, E.stream));
  CCRDT_HIP(hipMemcpyAsync(E.st_ts.p, ts, un * 8, hipMemcpyHostToDevice, E.stream));
  TrmvDownArgs a{};
  a.n = n;
  a.n_dc = D;
  a.k = (uint32_t)std::min<int64_t>(E.k, 0xFFFFFFFFll);
  a.key = E.st_kp.as<uint64_t>();
  a.op = E.st_kind.as<uint8_t>();
  a.id = E.st_id.as<int64_t>();
  a.score = E.st_score.as<int64_t>();
  a.dc = E.st_dc.as<uint8_t>();
  a.ts = E.st_ts.as<int64_t>();
  a.out_kind = E.st_out_kind.as<uint8_t>();
  a.out_vc = E.st_out_vc.as<int64_t>();
  a.s = E.trmv_cur();
  a.fresh = E.fresh ? 1 : 0;
  CCRDT_TRY(trmv_launch_downstream(a, E.stream));
  CCRDT_HIP(hipMemcpyAsync(out_kind, E.st_out_kind.p, un, hipMemcpyDeviceToHost, E.stream));
  if (out_vc)
    CCRDT_HIP(hipMemcpyAsync(out_vc, E.st_out_vc.p, un * D * 8, hipMemcpyDeviceToHost, E.stream));
  CCRDT_HIP(hipStreamSynchronize(E.stream));
  return CCRDT_OK;
}

int ccrdt_engine_clone(const ccrdt_engine* src, ccrdt_engine** out) {
  if (!src || !out) return CCRDT_EINVAL;
  ccrdt_engine* e = nullptr;
  CCRDT_TRY(ccrdt_engine_create(src->type, src->k, src->n_keys, src->n_dc, src->device, &e));
  int rc = e->clone_from(*src);
  if (rc != CCRDT_OK) {
    ccrdt_engine_destroy(e);
    return rc;
  }
  *out = e;
  return CCRDT_OK;
}

}  // extern "C"
