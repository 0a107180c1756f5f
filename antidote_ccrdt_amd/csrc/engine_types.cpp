// engine_types.cpp — per-type engine lifecycle and the C-ABI of average,
// topk, leaderboard and wordcount/worddocumentcount (include/ccrdt.h).
// Host code only sizes buffers, launches kernels (types_kernels.hip) and
// converts canonical images; every update/2 runs on the GPU.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <tuple>
#include <vector>

#include "common.hpp"
#include "engine.hpp"
#include "types_kernels.hpp"

namespace ccrdt {
int avg_launch_apply(const AvgArgs& a, hipStream_t st);
int avg_launch_value(const int64_t* sum, const int64_t* num, int64_t n_keys, int fresh, double* out,
                     uint8_t* defined, hipStream_t st);
int topk_launch_apply(const TopkArgs& a, int cls, uint64_t n_work, hipStream_t st);
int topk_launch_value(const TopkValueArgs& a, int cls, uint64_t n_work, hipStream_t st);
int lb_launch_apply(const LbArgs& a, int cls, uint64_t n_work, hipStream_t st);
int lb_launch_downstream(const LbDownArgs& a, hipStream_t st);
int lb_launch_pack_extras(const uint64_t* key_ptr, const uint32_t* ex_cnt, const LbExtraRec* ex, uint64_t n_keys,
                          int64_t* rows, int64_t cap, uint32_t* count, hipStream_t st);
int launch_ovf_need(const uint32_t* list, uint64_t n, const uint64_t* key_ptr, const uint32_t* cnt,
                    uint32_t stride, uint64_t* need, hipStream_t st);
int launch_caps_scan(const uint64_t* key_ptr, const uint32_t* cnt, uint32_t stride, uint64_t n,
                     uint64_t* caps, uint64_t* off, uint64_t* part, hipStream_t st);
int wc_launch_count(const uint64_t* doc_off, const uint8_t* bytes, uint64_t n_docs, uint64_t* ntok,
                    hipStream_t st);
int wc_launch_doc_key(const uint64_t* key_ptr, uint64_t n_keys, uint64_t n_docs, uint64_t* doc_key,
                     hipStream_t st);
int wc_launch_insert(const WcArgs& a, uint64_t n_tiles, hipStream_t st);
int wc_launch_verify(const WcArgs& a, uint64_t n_tiles, hipStream_t st);
int wc_launch_persist(const WcArgs& a, uint8_t* arena, unsigned long long* top, hipStream_t st);
int wc_launch_owner_count(const WcArgs& a, uint32_t world, uint32_t* owner, unsigned long long* cur, hipStream_t st);
int wc_launch_owner_scatter(const WcArgs& a, const uint32_t* owner, unsigned long long* cur, int64_t* meta,
                            uint8_t* out, uint32_t world, hipStream_t st);
int wc_launch_meta_split(const int64_t* meta, uint64_t n, uint64_t* wkey, int64_t* wcnt, uint32_t* wlen,
                         hipStream_t st);
int wc_launch_merge(const WcArgs& a, const uint64_t* wkey, const uint64_t* woff, const int64_t* cnt, uint64_t n,
                    int verify, hipStream_t st);
int wc_launch_check(const WcArgs& a, uint32_t n, hipStream_t st);
int wc_launch_dl(const WcArgs& a, uint64_t n_docs, uint32_t passes, hipStream_t st);
int wc_launch_cl_count(const WcClArgs& c, hipStream_t st);
int wc_launch_cl_sum(const WcClArgs& c, hipStream_t st);
int wc_launch_rehash(const WcSlot* old, const WcMeta* oldm, const unsigned long long* ocnt, uint64_t on, const WcArgs& a,
                     hipStream_t st);
}  // namespace ccrdt

using namespace ccrdt;

static int copy_buf(DevBuf& dst, const DevBuf& src, hipStream_t st) {
  if (!src.p) return CCRDT_OK;
  CCRDT_TRY(dst.ensure(src.bytes));
  CCRDT_HIP(hipMemcpyAsync(dst.p, src.p, src.bytes, hipMemcpyDeviceToDevice, st));
  return CCRDT_OK;
}

// (host memory of the caller: large copies go through the engine's pinned
// staging slots, staging.cpp)
static int h2d(Engine& E, DevBuf& d, const void* src, uint64_t bytes) {
  CCRDT_TRY(d.ensure(bytes));
  return h2d_staged(E, d.p, src, bytes);
}

template <class T>
static int d2h(std::vector<T>& v, const DevBuf& d, uint64_t n, hipStream_t st) {
  v.resize(n);
  if (n) {
    CCRDT_HIP(hipMemcpyAsync(v.data(), d.p, n * sizeof(T), hipMemcpyDeviceToHost, st));
    CCRDT_HIP(hipStreamSynchronize(st));
  }
  return CCRDT_OK;
}

template <class T>
static int d2h_at(std::vector<T>& v, const DevBuf& d, uint64_t at, uint64_t n, hipStream_t st) {
  v.resize(n);
  if (n) {
    CCRDT_HIP(hipMemcpyAsync(v.data(), (const T*)d.p + at, n * sizeof(T), hipMemcpyDeviceToHost, st));
    CCRDT_HIP(hipStreamSynchronize(st));
  }
  return CCRDT_OK;
}

// CSR splice: keys [k0, k1) of (fp, fv...) replaced by the range image (ip, iv...).
template <class T>
static void splice_csr(const std::vector<uint64_t>& fp, const std::vector<T>& fv, const uint64_t* ip,
                       const T* iv, uint64_t k0, uint64_t k1, std::vector<uint64_t>& op, std::vector<T>& ov,
                       size_t width = 1) {
  const uint64_t nk = fp.size() - 1;
  op.assign(nk + 1, 0);
  ov.clear();
  for (uint64_t k = 0; k < nk; ++k) {
    if (k >= k0 && k < k1)
      ov.insert(ov.end(), iv + ip[k - k0] * width, iv + ip[k - k0 + 1] * width);
    else
      ov.insert(ov.end(), fv.begin() + fp[k] * width, fv.begin() + fp[k + 1] * width);
    op[k + 1] = ov.size() / width;
  }
}

int ccrdt_engine::init_type() {
  fresh = true;
  return CCRDT_OK;
}

int ccrdt_engine::reset_type() { return CCRDT_OK; }

void ccrdt_engine::release_types() {
  for (int s = 0; s < 2; ++s) {
    for (DevBuf* d : {&tb.avg_sum[s], &tb.avg_num[s], &tb.tk_off[s], &tb.tk_cnt[s], &tb.tk_id[s],
                      &tb.tk_score[s], &tb.lb_meta[s], &tb.lb_id[s], &tb.lb_score[s], &tb.lb_st[s],
                      &tb.t_tab[s], &tb.t_meta[s], &tb.t_cnt[s]})
      d->release();
  }
  for (DevBuf* d : {&tb.hb_off, &tb.hb_cap, &tb.hb_a, &tb.hb_b, &tb.hb_c, &tb.hb_d})
    d->release();
  for (DevBuf* d : {&tb.arena, &tb.arena_top, &tb.d_hash, &tb.dl, &tb.dl_pre, &tb.dl_cur, &tb.chk, &tb.cl, &tb.cl_bcnt, &tb.fl, &tb.bkt, &tb.cl_small, &tb.caps, &tb.part, &tb.ovf_a, &tb.ovf_b,
                    &tb.status, &tb.ex_cnt, &tb.ex, &tb.kp})
    d->release();
  for (auto& d : tb.stage) d.release();
}

int ccrdt_engine::clone_from(const ccrdt_engine& src) {
  CCRDT_HIP(hipStreamSynchronize(src.stream));
  fresh = src.fresh;
  if (type == CCRDT_TOPK_RMV) {
    cur = src.cur;
    mcur = src.mcur;
    inplace_ready = src.inplace_ready;
    arena_pending = src.arena_pending;
    fresh_room = src.fresh_room;
    for (int x = 0; x < 3; ++x) trmv_tot[cur][x] = src.trmv_tot[src.cur][x];
    for (int x = 0; x < 3; ++x) {
      arena_cap[x] = src.arena_cap[x];
      arena_used[x] = src.arena_used[x];
      arena_rate[x] = src.arena_rate[x];
    }
    memcpy(arena_sub, src.arena_sub, sizeof(arena_sub));
    const TrmvBufs& s = src.trmv[src.cur];
    TrmvBufs& d = trmv[cur];
    CCRDT_TRY(copy_buf(trmv[mcur].meta, src.trmv[src.mcur].meta, stream));
    CCRDT_TRY(copy_buf(trmv[mcur].cap, src.trmv[src.mcur].cap, stream));
    CCRDT_TRY(copy_buf(arena, src.arena, stream));
    CCRDT_TRY(copy_buf(obs_ord, src.obs_ord, stream));
    CCRDT_TRY(copy_buf(d.pl_id, s.pl_id, stream));
    CCRDT_TRY(copy_buf(d.pl_info, s.pl_info, stream));
    CCRDT_TRY(copy_buf(d.pl_slab, s.pl_slab, stream));
    CCRDT_TRY(copy_buf(d.pl_gb, s.pl_gb, stream));
    CCRDT_TRY(copy_buf(d.m_score, s.m_score, stream));
    CCRDT_TRY(copy_buf(d.m_ts, s.m_ts, stream));
    CCRDT_TRY(copy_buf(d.m_dc, s.m_dc, stream));
    CCRDT_TRY(copy_buf(d.r_vc, s.r_vc, stream));
    CCRDT_TRY(copy_buf(d.vc, s.vc, stream));
  } else {
    const int c = src.tb.tcur;
    tb.tcur = c;
    const TypeBufs& s = src.tb;
    for (auto [dd, ss] : {std::pair<DevBuf*, const DevBuf*>{&tb.avg_sum[c], &s.avg_sum[c]},
                          {&tb.avg_num[c], &s.avg_num[c]}, {&tb.tk_off[c], &s.tk_off[c]},
                          {&tb.tk_cnt[c], &s.tk_cnt[c]}, {&tb.tk_id[c], &s.tk_id[c]},
                          {&tb.tk_score[c], &s.tk_score[c]}, {&tb.lb_meta[c], &s.lb_meta[c]},
                          {&tb.lb_id[c], &s.lb_id[c]}, {&tb.lb_score[c], &s.lb_score[c]},
                          {&tb.lb_st[c], &s.lb_st[c]}, {&tb.t_tab[c], &s.t_tab[c]}, {&tb.t_meta[c], &s.t_meta[c]},
                          {&tb.t_cnt[c], &s.t_cnt[c]},
                          {&tb.arena, &s.arena},
                          {&tb.arena_top, &s.arena_top}})
      CCRDT_TRY(copy_buf(*dd, *ss, stream));
    tb.t_slots[c] = s.t_slots[c];
    tb.arena_cap = s.arena_cap;
  }
  CCRDT_HIP(hipStreamSynchronize(stream));
  return CCRDT_OK;
}

static int check_type(ccrdt_engine* e, int type) {
  if (!e) {
    set_error("null engine");
    return CCRDT_EINVAL;
  }
  if (e->type != type &&
      !(type == CCRDT_WORDCOUNT && e->type == CCRDT_WORDDOCUMENTCOUNT)) {
    set_error("operation does not match the engine's CCRDT type");
    return CCRDT_ENOSYS;
  }
  if (hipSetDevice(e->device) != hipSuccess) {
    set_error("hipSetDevice failed");
    return CCRDT_EDEVICE;
  }
  return CCRDT_OK;
}

static int check_csr(const uint64_t* key_ptr, uint64_t nk, uint64_t n) {
  if (key_ptr[0] != 0 || key_ptr[nk] != n) {
    set_error("key_ptr must start at 0 and end at the op count");
    return CCRDT_EINVAL;
  }
  for (uint64_t k = 0; k < nk; ++k)
    if (key_ptr[k + 1] < key_ptr[k]) {
      set_error("key_ptr not monotone");
      return CCRDT_EINVAL;
    }
  return CCRDT_OK;
}

static int read_status(ccrdt_engine* e, uint32_t* out2) {
  CCRDT_HIP(hipMemcpyAsync(e->h_status, e->tb.status.p, 8, hipMemcpyDeviceToHost, e->stream));
  CCRDT_HIP(hipStreamSynchronize(e->stream));
  memcpy(out2, e->h_status, 8);
  return CCRDT_OK;
}
static int read_status3(ccrdt_engine* e, uint32_t* out3) {
  CCRDT_HIP(hipMemcpyAsync(e->h_status, e->tb.status.p, 12, hipMemcpyDeviceToHost, e->stream));
  CCRDT_HIP(hipStreamSynchronize(e->stream));
  memcpy(out3, e->h_status, 12);
  return CCRDT_OK;
}

// segment offsets off[0..nk] of the new side: caps = cnt (stride) + ops
static int scan_caps(ccrdt_engine* e, const uint64_t* key_ptr, const uint32_t* cnt, uint32_t stride,
                     DevBuf& off, uint64_t* total) {
  const uint64_t nk = (uint64_t)e->n_keys;
  CCRDT_TRY(e->tb.caps.ensure((nk + 1) * 8));
  CCRDT_TRY(e->tb.part.ensure(((nk + 255) / 256 + 2) * 8));
  CCRDT_TRY(off.ensure((nk + 1) * 8));
  CCRDT_TRY(launch_caps_scan(key_ptr, cnt, stride, nk, e->tb.caps.as<uint64_t>(), off.as<uint64_t>(),
                             e->tb.part.as<uint64_t>(), e->stream));
  CCRDT_HIP(hipMemcpyAsync(e->h_status, off.as<uint64_t>() + nk, 8, hipMemcpyDeviceToHost, e->stream));
  CCRDT_HIP(hipStreamSynchronize(e->stream));
  memcpy(total, e->h_status, 8);
  return CCRDT_OK;
}

// HBM class for the n keys left in `list`: per key a scratch region of
// cap = the power of two >= max(64, mult * need) slots, need = ops of the key
// + cnt[k * stride]; offsets (exclusive scan of the caps) and caps go to
// tb.hb_off / tb.hb_cap.  *total = sum of the caps.
static int hbm_regions(ccrdt_engine* e, const uint32_t* list, uint64_t n, const uint64_t* key_ptr,
                       const uint32_t* cnt, uint32_t stride, uint64_t mult, uint64_t* total) {
  TypeBufs& T = e->tb;
  CCRDT_TRY(T.caps.ensure(n * 8));
  CCRDT_TRY(launch_ovf_need(list, n, key_ptr, cnt, stride, T.caps.as<uint64_t>(), e->stream));
  std::vector<uint64_t> need;
  CCRDT_TRY(d2h(need, T.caps, n, e->stream));
  std::vector<uint64_t> off(n);
  std::vector<uint32_t> cap(n);
  uint64_t t = 0;
  for (uint64_t w = 0; w < n; ++w) {
    uint64_t c = 64;
    while (c < mult * need[w]) c <<= 1;
    if (c > (1ull << 31)) {
      set_error("a key needs more than 2^31 slots in one batch");
      return CCRDT_ENOMEM;
    }
    off[w] = t;
    cap[w] = (uint32_t)c;
    t += c;
  }
  CCRDT_TRY(h2d(*e, T.hb_off, off.data(), n * 8));
  CCRDT_TRY(h2d(*e, T.hb_cap, cap.data(), n * 4));
  *total = t;
  return CCRDT_OK;
}

extern "C" {

// ======================================================================= average
int ccrdt_avg_apply_device(ccrdt_engine* e, const ccrdt_avg_ops* ops) {
  CCRDT_TRY(check_type(e, CCRDT_AVERAGE));
  if (!ops || !ops->key_ptr || (ops->n_ops && (!ops->value || !ops->n))) {
    set_error("avg_apply: null arrays");
    return CCRDT_EINVAL;
  }
  TypeBufs& T = e->tb;
  const int in = T.tcur, out = 1 - T.tcur;
  const uint64_t nk = (uint64_t)e->n_keys;
  CCRDT_TRY(T.avg_sum[out].ensure(nk * 8));
  CCRDT_TRY(T.avg_num[out].ensure(nk * 8));
  CCRDT_TRY(T.status.ensure(64));
  CCRDT_HIP(hipMemsetAsync(T.status.p, 0, 8, e->stream));
  AvgArgs a{};
  a.n_keys = e->n_keys;
  a.key_ptr = ops->key_ptr;
  a.v = ops->value;
  a.n = ops->n;
  a.sum_in = T.avg_sum[in].as<int64_t>();
  a.num_in = T.avg_num[in].as<int64_t>();
  a.sum_out = T.avg_sum[out].as<int64_t>();
  a.num_out = T.avg_num[out].as<int64_t>();
  a.fresh = e->fresh ? 1 : 0;
  a.status = T.status.as<uint32_t>();
  CCRDT_HIP(hipEventRecord(e->evk0, e->stream));
  CCRDT_TRY(avg_launch_apply(a, e->stream));
  CCRDT_HIP(hipEventRecord(e->evk1, e->stream));
  uint32_t st[2];
  CCRDT_TRY(read_status(e, st));
  CCRDT_HIP(hipEventElapsedTime(&e->last_kernel_ms, e->evk0, e->evk1));
  if (st[0] & AVG_ERR_NEG) {
    set_error("avg_apply: {add, {V, N}} with N < 0 (no function clause)");
    return CCRDT_EINVAL;
  }
  if (st[0] & AVG_ERR_RANGE) {
    set_error("avg_apply: Sum or Num leaves int64");
    return CCRDT_ERANGE;
  }
  T.tcur = out;
  e->fresh = false;
  return CCRDT_OK;
}

int ccrdt_avg_apply(ccrdt_engine* e, const ccrdt_avg_ops* ops) {
  CCRDT_TRY(check_type(e, CCRDT_AVERAGE));
  if (!ops || !ops->key_ptr) return CCRDT_EINVAL;
  const uint64_t nk = (uint64_t)e->n_keys, n = (uint64_t)ops->n_ops;
  CCRDT_TRY(check_csr(ops->key_ptr, nk, n));
  TypeBufs& T = e->tb;
  CCRDT_TRY(h2d(*e, T.kp, ops->key_ptr, (nk + 1) * 8));
  CCRDT_TRY(h2d(*e, T.stage[0], ops->value, n * 8));
  CCRDT_TRY(h2d(*e, T.stage[1], ops->n, n * 8));
  ccrdt_avg_ops d{ops->n_ops, T.kp.as<uint64_t>(), T.stage[0].as<int64_t>(), T.stage[1].as<int64_t>()};
  return ccrdt_avg_apply_device(e, &d);
}

int ccrdt_avg_export(ccrdt_engine* e, int64_t* sum, int64_t* num) {
  CCRDT_TRY(check_type(e, CCRDT_AVERAGE));
  const uint64_t nk = (uint64_t)e->n_keys;
  if (e->fresh) {
    if (sum) memset(sum, 0, nk * 8);
    if (num) memset(num, 0, nk * 8);
    return CCRDT_OK;
  }
  CCRDT_HIP(hipStreamSynchronize(e->stream));
  if (sum && nk) CCRDT_HIP(hipMemcpy(sum, e->tb.avg_sum[e->tb.tcur].p, nk * 8, hipMemcpyDeviceToHost));
  if (num && nk) CCRDT_HIP(hipMemcpy(num, e->tb.avg_num[e->tb.tcur].p, nk * 8, hipMemcpyDeviceToHost));
  return CCRDT_OK;
}

int ccrdt_avg_import(ccrdt_engine* e, const int64_t* sum, const int64_t* num) {
  CCRDT_TRY(check_type(e, CCRDT_AVERAGE));
  if (!sum || !num) return CCRDT_EINVAL;
  const uint64_t nk = (uint64_t)e->n_keys;
  TypeBufs& T = e->tb;
  CCRDT_TRY(h2d(*e, T.avg_sum[T.tcur], sum, nk * 8));
  CCRDT_TRY(h2d(*e, T.avg_num[T.tcur], num, nk * 8));
  CCRDT_HIP(hipStreamSynchronize(e->stream));
  e->fresh = false;
  return CCRDT_OK;
}

int ccrdt_avg_value(ccrdt_engine* e, double* value, uint8_t* defined) {
  CCRDT_TRY(check_type(e, CCRDT_AVERAGE));
  if (!value || !defined) return CCRDT_EINVAL;
  const uint64_t nk = (uint64_t)e->n_keys;
  TypeBufs& T = e->tb;
  CCRDT_TRY(T.stage[2].ensure(nk * 8));
  CCRDT_TRY(T.stage[3].ensure(nk));
  CCRDT_TRY(T.avg_sum[T.tcur].ensure(8));
  CCRDT_TRY(T.avg_num[T.tcur].ensure(8));
  CCRDT_TRY(avg_launch_value(T.avg_sum[T.tcur].as<int64_t>(), T.avg_num[T.tcur].as<int64_t>(), e->n_keys,
                             e->fresh ? 1 : 0, T.stage[2].as<double>(), T.stage[3].as<uint8_t>(),
                             e->stream));
  CCRDT_HIP(hipStreamSynchronize(e->stream));
  if (nk) {
    CCRDT_HIP(hipMemcpy(value, T.stage[2].p, nk * 8, hipMemcpyDeviceToHost));
    CCRDT_HIP(hipMemcpy(defined, T.stage[3].p, nk, hipMemcpyDeviceToHost));
  }
  return CCRDT_OK;
}

// ========================================================================== topk
int ccrdt_topk_apply_device(ccrdt_engine* e, const ccrdt_topk_ops* ops) {
  CCRDT_TRY(check_type(e, CCRDT_TOPK));
  if (!ops || !ops->key_ptr || (ops->n_ops && (!ops->id || !ops->score))) {
    set_error("topk_apply: null arrays");
    return CCRDT_EINVAL;
  }
  TypeBufs& T = e->tb;
  const int in = T.tcur, out = 1 - T.tcur;
  const uint64_t nk = (uint64_t)e->n_keys;
  uint64_t total = 0;
  CCRDT_TRY(scan_caps(e, ops->key_ptr, e->fresh ? nullptr : T.tk_cnt[in].as<uint32_t>(), 1,
                      T.tk_off[out], &total));
  CCRDT_TRY(T.tk_cnt[out].ensure(nk * 4));
  CCRDT_TRY(T.tk_id[out].ensure(total * 8));
  CCRDT_TRY(T.tk_score[out].ensure(total * 8));
  CCRDT_TRY(T.ovf_a.ensure(nk * 4));
  CCRDT_TRY(T.ovf_b.ensure(nk * 4));
  CCRDT_TRY(T.status.ensure(64));
  TopkArgs a{};
  a.n_keys = e->n_keys;
  a.key_ptr = ops->key_ptr;
  a.op_id = ops->id;
  a.op_score = ops->score;
  a.off_in = T.tk_off[in].as<uint64_t>();
  a.cnt_in = T.tk_cnt[in].as<uint32_t>();
  a.id_in = T.tk_id[in].as<int64_t>();
  a.score_in = T.tk_score[in].as<int64_t>();
  a.off_out = T.tk_off[out].as<uint64_t>();
  a.cnt_out = T.tk_cnt[out].as<uint32_t>();
  a.id_out = T.tk_id[out].as<int64_t>();
  a.score_out = T.tk_score[out].as<int64_t>();
  a.fresh = e->fresh ? 1 : 0;
  a.status = T.status.as<uint32_t>();
  uint64_t n_work = nk;
  const uint32_t* list = nullptr;
  float total_ms = 0.f;
  for (int cls = 0; cls < 4 && n_work; ++cls) {
    DevBuf* ovf = (list == T.ovf_a.as<uint32_t>()) ? &T.ovf_b : &T.ovf_a;
    a.key_list = list;
    a.ovf_list = ovf->as<uint32_t>();
    if (cls == 3) {  // HBM hash: cap + 1 slots per key
      uint64_t slots = 0;
      CCRDT_TRY(hbm_regions(e, list, n_work, ops->key_ptr, e->fresh ? nullptr : a.cnt_in, 1, 2, &slots));
      slots += n_work;
      CCRDT_TRY(T.hb_a.ensure(slots * 8));
      CCRDT_TRY(T.hb_b.ensure(slots * 4));
      a.tab_off = T.hb_off.as<uint64_t>();
      a.tab_cap = T.hb_cap.as<uint32_t>();
      a.g_id = T.hb_a.as<int64_t>();
      a.g_seq = T.hb_b.as<int32_t>();
    }
    CCRDT_HIP(hipMemsetAsync(T.status.p, 0, 8, e->stream));
    CCRDT_HIP(hipEventRecord(e->evk0, e->stream));
    CCRDT_TRY(topk_launch_apply(a, cls, n_work, e->stream));
    CCRDT_HIP(hipEventRecord(e->evk1, e->stream));
    uint32_t st[2];
    CCRDT_TRY(read_status(e, st));
    float ms = 0.f;
    CCRDT_HIP(hipEventElapsedTime(&ms, e->evk0, e->evk1));
    total_ms += ms;
    n_work = st[0];
    list = ovf->as<uint32_t>();
  }
  e->last_kernel_ms = total_ms;
  T.tcur = out;
  e->fresh = false;
  return CCRDT_OK;
}

int ccrdt_topk_apply(ccrdt_engine* e, const ccrdt_topk_ops* ops) {
  CCRDT_TRY(check_type(e, CCRDT_TOPK));
  if (!ops || !ops->key_ptr) return CCRDT_EINVAL;
  const uint64_t nk = (uint64_t)e->n_keys, n = (uint64_t)ops->n_ops;
  CCRDT_TRY(check_csr(ops->key_ptr, nk, n));
  TypeBufs& T = e->tb;
  CCRDT_TRY(h2d(*e, T.kp, ops->key_ptr, (nk + 1) * 8));
  CCRDT_TRY(h2d(*e, T.stage[0], ops->id, n * 8));
  CCRDT_TRY(h2d(*e, T.stage[1], ops->score, n * 8));
  ccrdt_topk_ops d{ops->n_ops, T.kp.as<uint64_t>(), T.stage[0].as<int64_t>(), T.stage[1].as<int64_t>()};
  return ccrdt_topk_apply_device(e, &d);
}

namespace {
struct TopkHost {
  std::vector<uint64_t> off;
  std::vector<uint32_t> cnt;
  std::vector<int64_t> id, score;
};
// Keys [k0, k1) only (offsets rebased to the downloaded slice).
int topk_download(ccrdt_engine* e, TopkHost& h, uint64_t k0, uint64_t k1) {
  const uint64_t nk = k1 - k0;
  h.cnt.assign(nk, 0);
  h.off.assign(nk + 1, 0);
  if (e->fresh || !nk) return CCRDT_OK;
  TypeBufs& T = e->tb;
  const int c = T.tcur;
  CCRDT_TRY(d2h_at(h.off, T.tk_off[c], k0, nk + 1, e->stream));
  CCRDT_TRY(d2h_at(h.cnt, T.tk_cnt[c], k0, nk, e->stream));
  const uint64_t b = h.off[0], n = h.off[nk] - b;
  for (uint64_t& o : h.off) o -= b;
  CCRDT_TRY(d2h_at(h.id, T.tk_id[c], b, n, e->stream));
  CCRDT_TRY(d2h_at(h.score, T.tk_score[c], b, n, e->stream));
  return CCRDT_OK;
}
void topk_export_host(const TopkHost& h, uint64_t nk, uint64_t* ptr, int64_t* id, int64_t* score) {
  std::vector<std::pair<int64_t, int64_t>> v;
  uint64_t p = 0;
  ptr[0] = 0;
  for (uint64_t k = 0; k < nk; ++k) {
    v.clear();
    for (uint32_t j = 0; j < h.cnt[k]; ++j) v.push_back({h.id[h.off[k] + j], h.score[h.off[k] + j]});
    std::sort(v.begin(), v.end());
    for (auto& [i, s] : v) {
      id[p] = i;
      score[p++] = s;
    }
    ptr[k + 1] = p;
  }
}
}  // namespace

int ccrdt_topk_size(ccrdt_engine* e, int64_t* n_entries) {
  CCRDT_TRY(check_type(e, CCRDT_TOPK));
  const uint64_t nk = (uint64_t)e->n_keys;
  int64_t s = 0;
  if (!e->fresh && nk) {
    std::vector<uint32_t> cnt;
    CCRDT_TRY(d2h(cnt, e->tb.tk_cnt[e->tb.tcur], nk, e->stream));
    for (uint32_t c : cnt) s += c;
  }
  *n_entries = s;
  return CCRDT_OK;
}

int ccrdt_topk_export(ccrdt_engine* e, uint64_t* ptr, int64_t* id, int64_t* score) {
  return ccrdt_topk_export_range(e, 0, e ? e->n_keys : 0, ptr, id, score);
}

static int key_range(ccrdt_engine* e, int64_t k0, int64_t k1, const char* where) {
  if (k0 < 0 || k1 < k0 || k1 > e->n_keys) {
    set_error(std::string(where) + ": key range outside [0, n_keys]");
    return CCRDT_EINVAL;
  }
  return CCRDT_OK;
}

int ccrdt_topk_range_size(ccrdt_engine* e, int64_t k0, int64_t k1, int64_t* n_entries) {
  CCRDT_TRY(check_type(e, CCRDT_TOPK));
  CCRDT_TRY(key_range(e, k0, k1, "topk_range_size"));
  int64_t s = 0;
  if (!e->fresh && k1 > k0) {
    std::vector<uint32_t> cnt;
    CCRDT_TRY(d2h_at(cnt, e->tb.tk_cnt[e->tb.tcur], (uint64_t)k0, (uint64_t)(k1 - k0), e->stream));
    for (uint32_t c : cnt) s += c;
  }
  *n_entries = s;
  return CCRDT_OK;
}

int ccrdt_topk_export_range(ccrdt_engine* e, int64_t k0, int64_t k1, uint64_t* ptr, int64_t* id,
                            int64_t* score) {
  CCRDT_TRY(check_type(e, CCRDT_TOPK));
  CCRDT_TRY(key_range(e, k0, k1, "topk_export_range"));
  TopkHost h;
  CCRDT_TRY(topk_download(e, h, (uint64_t)k0, (uint64_t)k1));
  topk_export_host(h, (uint64_t)(k1 - k0), ptr, id, score);
  return CCRDT_OK;
}

int ccrdt_topk_import_range(ccrdt_engine* e, int64_t k0, int64_t k1, const uint64_t* ptr, const int64_t* id,
                            const int64_t* score) {
  CCRDT_TRY(check_type(e, CCRDT_TOPK));
  CCRDT_TRY(key_range(e, k0, k1, "topk_import_range"));
  const uint64_t nk = (uint64_t)e->n_keys;
  int64_t n = 0;
  CCRDT_TRY(ccrdt_topk_size(e, &n));
  std::vector<uint64_t> fp(nk + 1), op, op2;
  std::vector<int64_t> fi((size_t)n + 1), fs((size_t)n + 1), oi, os;
  CCRDT_TRY(ccrdt_topk_export(e, fp.data(), fi.data(), fs.data()));
  splice_csr(fp, fi, ptr, id, (uint64_t)k0, (uint64_t)k1, op, oi);
  splice_csr(fp, fs, ptr, score, (uint64_t)k0, (uint64_t)k1, op2, os);
  oi.push_back(0);
  os.push_back(0);
  return ccrdt_topk_import(e, op.data(), oi.data(), os.data());
}

int ccrdt_topk_import(ccrdt_engine* e, const uint64_t* ptr, const int64_t* id, const int64_t* score) {
  CCRDT_TRY(check_type(e, CCRDT_TOPK));
  const uint64_t nk = (uint64_t)e->n_keys;
  TypeBufs& T = e->tb;
  std::vector<uint32_t> cnt(nk);
  for (uint64_t k = 0; k < nk; ++k) {
    cnt[k] = (uint32_t)(ptr[k + 1] - ptr[k]);
    std::vector<int64_t> ids(id + ptr[k], id + ptr[k + 1]);
    std::sort(ids.begin(), ids.end());
    if (std::adjacent_find(ids.begin(), ids.end()) != ids.end()) {
      set_error("topk_import: duplicate Id in a key");
      return CCRDT_EINVAL;
    }
  }
  const int c = T.tcur;
  CCRDT_TRY(h2d(*e, T.tk_off[c], ptr, (nk + 1) * 8));
  CCRDT_TRY(h2d(*e, T.tk_cnt[c], cnt.data(), nk * 4));
  CCRDT_TRY(h2d(*e, T.tk_id[c], id, ptr[nk] * 8));
  CCRDT_TRY(h2d(*e, T.tk_score[c], score, ptr[nk] * 8));
  CCRDT_HIP(hipStreamSynchronize(e->stream));
  e->fresh = false;
  return CCRDT_OK;
}

int ccrdt_topk_value(ccrdt_engine* e, uint64_t* ptr, int64_t* id, int64_t* score) {
  CCRDT_TRY(check_type(e, CCRDT_TOPK));
  const uint64_t nk = (uint64_t)e->n_keys;
  TypeBufs& T = e->tb;
  const int c = T.tcur;
  if (e->fresh || !nk) {
    for (uint64_t k = 0; k <= nk; ++k) ptr[k] = 0;
    return CCRDT_OK;
  }
  uint64_t total = 0;
  CCRDT_TRY(scan_caps(e, nullptr, T.tk_cnt[c].as<uint32_t>(), 1, T.stage[4], &total));
  CCRDT_TRY(T.stage[2].ensure(total * 8 + 8));
  CCRDT_TRY(T.stage[3].ensure(total * 8 + 8));
  CCRDT_TRY(T.ovf_a.ensure(nk * 4));
  CCRDT_TRY(T.ovf_b.ensure(nk * 4));
  CCRDT_TRY(T.status.ensure(64));
  TopkValueArgs a{};
  a.off = T.tk_off[c].as<uint64_t>();
  a.cnt = T.tk_cnt[c].as<uint32_t>();
  a.id = T.tk_id[c].as<int64_t>();
  a.score = T.tk_score[c].as<int64_t>();
  a.out_ptr = T.stage[4].as<uint64_t>();
  a.out_id = T.stage[2].as<int64_t>();
  a.out_score = T.stage[3].as<int64_t>();
  a.status = T.status.as<uint32_t>();
  uint64_t n_work = nk;
  const uint32_t* list = nullptr;
  for (int cls = 0; cls < 3 && n_work; ++cls) {
    DevBuf* ovf = (list == T.ovf_a.as<uint32_t>()) ? &T.ovf_b : &T.ovf_a;
    a.key_list = list;
    a.ovf_list = ovf->as<uint32_t>();
    if (cls == 2) {  // HBM bitonic sort regions
      uint64_t slots = 0;
      CCRDT_TRY(hbm_regions(e, list, n_work, nullptr, a.cnt, 1, 1, &slots));
      CCRDT_TRY(T.hb_a.ensure(slots * 8));
      CCRDT_TRY(T.hb_b.ensure(slots * 8));
      a.tab_off = T.hb_off.as<uint64_t>();
      a.tab_cap = T.hb_cap.as<uint32_t>();
      a.g_id = T.hb_a.as<int64_t>();
      a.g_score = T.hb_b.as<int64_t>();
    }
    CCRDT_HIP(hipMemsetAsync(T.status.p, 0, 8, e->stream));
    CCRDT_TRY(topk_launch_value(a, cls, n_work, e->stream));
    uint32_t st[2];
    CCRDT_TRY(read_status(e, st));
    n_work = st[0];
    list = ovf->as<uint32_t>();
  }
  CCRDT_HIP(hipMemcpy(ptr, T.stage[4].p, (nk + 1) * 8, hipMemcpyDeviceToHost));
  if (total) {
    CCRDT_HIP(hipMemcpy(id, T.stage[2].p, total * 8, hipMemcpyDeviceToHost));
    CCRDT_HIP(hipMemcpy(score, T.stage[3].p, total * 8, hipMemcpyDeviceToHost));
  }
  return CCRDT_OK;
}

int ccrdt_topk_downstream(ccrdt_engine* e, int64_t n, const int64_t* score, uint8_t* out_kind) {
  CCRDT_TRY(check_type(e, CCRDT_TOPK));
  // changes_state/2 (topk.erl:164-166) compares the op's Score with Size
  // only; no state is read.
  for (int64_t i = 0; i < n; ++i) out_kind[i] = score[i] > e->k ? 0 : CCRDT_NOOP;
  return CCRDT_OK;
}

// =================================================================== leaderboard
int ccrdt_lb_apply_device(ccrdt_engine* e, const ccrdt_lb_ops* ops) {
  CCRDT_TRY(check_type(e, CCRDT_LEADERBOARD));
  if (!ops || !ops->key_ptr || (ops->n_ops && (!ops->kind || !ops->id || !ops->score))) {
    set_error("lb_apply: null arrays");
    return CCRDT_EINVAL;
  }
  TypeBufs& T = e->tb;
  const int in = T.tcur, out = 1 - T.tcur;
  const uint64_t nk = (uint64_t)e->n_keys, n_ops = (uint64_t)ops->n_ops;
  uint64_t total = 0;
  CCRDT_TRY(T.stage[5].ensure((nk + 1) * 8));
  CCRDT_TRY(scan_caps(e, ops->key_ptr,
                      e->fresh ? nullptr : (const uint32_t*)T.lb_meta[in].as<LbMeta>() + 1, 4,
                      T.stage[5], &total));
  if (total >= 0xFFFFFFFFull) {
    set_error("lb_apply: resident entries would exceed 2^32");
    return CCRDT_ENOMEM;
  }
  CCRDT_TRY(T.lb_meta[out].ensure(nk * sizeof(LbMeta)));
  CCRDT_TRY(T.lb_id[out].ensure(total * 8));
  CCRDT_TRY(T.lb_score[out].ensure(total * 8));
  CCRDT_TRY(T.lb_st[out].ensure(total));
  CCRDT_TRY(T.ex_cnt.ensure(nk * 4));
  CCRDT_TRY(T.ex.ensure(n_ops * sizeof(LbExtraRec)));
  CCRDT_TRY(T.ovf_a.ensure(nk * 4));
  CCRDT_TRY(T.ovf_b.ensure(nk * 4));
  CCRDT_TRY(T.status.ensure(64));
  CCRDT_TRY(T.kp.ensure((nk + 1) * 8));
  LbArgs a{};
  a.n_keys = e->n_keys;
  a.k = (uint32_t)std::min<int64_t>(e->k, 0xFFFFFFFFll);
  a.key_ptr = ops->key_ptr;
  a.kind = ops->kind;
  a.id = ops->id;
  a.score = ops->score;
  a.meta_in = T.lb_meta[in].as<LbMeta>();
  a.id_in = T.lb_id[in].as<int64_t>();
  a.score_in = T.lb_score[in].as<int64_t>();
  a.st_in = T.lb_st[in].as<uint8_t>();
  a.meta_out = T.lb_meta[out].as<LbMeta>();
  a.off_out = T.stage[5].as<uint64_t>();
  a.id_out = T.lb_id[out].as<int64_t>();
  a.score_out = T.lb_score[out].as<int64_t>();
  a.st_out = T.lb_st[out].as<uint8_t>();
  a.fresh = e->fresh ? 1 : 0;
  a.ex_cnt = T.ex_cnt.as<uint32_t>();
  a.ex = T.ex.as<LbExtraRec>();
  a.status = T.status.as<uint32_t>();
  {
    const char* sq = getenv("CCRDT_LB_SEQ");
    a.seq = (sq && sq[0] == '1') ? 1 : 0;
  }
  uint64_t n_work = nk;
  const uint32_t* list = nullptr;
  float total_ms = 0.f;
  // LDS classes: 512 / 640 / 1024 entries for boards whose Ids and Scores fit
  // 32 bits, then 512 / 640 / 1024 / 2048 entries of 64-bit values, then HBM
  // boards (lb_launch_apply)
  for (int cls = 0; cls < 8 && n_work; ++cls) {
    DevBuf* ovf = (list == T.ovf_a.as<uint32_t>()) ? &T.ovf_b : &T.ovf_a;
    a.key_list = list;
    a.ovf_list = ovf->as<uint32_t>();
    if (cls == 7) {  // HBM boards: entries + a 2x hash per board
      uint64_t slots = 0;
      CCRDT_TRY(hbm_regions(e, list, n_work, ops->key_ptr,
                            e->fresh ? nullptr : (const uint32_t*)a.meta_in + 1, 4, 1, &slots));
      CCRDT_TRY(T.hb_a.ensure(slots * 8));
      CCRDT_TRY(T.hb_b.ensure(slots * 8));
      CCRDT_TRY(T.hb_c.ensure(slots));
      CCRDT_TRY(T.hb_d.ensure(slots * 8));
      a.tab_off = T.hb_off.as<uint64_t>();
      a.tab_cap = T.hb_cap.as<uint32_t>();
      a.g_eid = T.hb_a.as<int64_t>();
      a.g_esc = T.hb_b.as<int64_t>();
      a.g_est = T.hb_c.as<uint8_t>();
      a.g_hslot = T.hb_d.as<uint32_t>();
    }
    CCRDT_HIP(hipMemsetAsync(T.status.p, 0, 8, e->stream));
    CCRDT_HIP(hipEventRecord(e->evk0, e->stream));
    CCRDT_TRY(lb_launch_apply(a, cls, n_work, e->stream));
    CCRDT_HIP(hipEventRecord(e->evk1, e->stream));
    uint32_t st[2];
    CCRDT_TRY(read_status(e, st));
    float ms = 0.f;
    CCRDT_HIP(hipEventElapsedTime(&ms, e->evk0, e->evk1));
    total_ms += ms;
    if (st[1]) {
      set_error("lb_apply: effect kind > 2 (no function clause)");
      return CCRDT_EINVAL;
    }
    n_work = st[0];
    list = ovf->as<uint32_t>();
  }
  CCRDT_HIP(hipMemcpyAsync(T.kp.p, ops->key_ptr, (nk + 1) * 8, hipMemcpyDeviceToDevice, e->stream));
  e->last_kernel_ms = total_ms;
  e->last_n_ops = n_ops;
  T.tcur = out;
  e->fresh = false;
  return CCRDT_OK;
}

int ccrdt_lb_extras_device(ccrdt_engine* e, int64_t* d_rows, int64_t cap_rows, uint32_t* d_count) {
  CCRDT_TRY(check_type(e, CCRDT_LEADERBOARD));
  if (!d_rows || !d_count || cap_rows < 0) return CCRDT_EINVAL;
  const bool have = e->last_n_ops > 0 && e->tb.ex_cnt.p;
  return lb_launch_pack_extras(e->tb.kp.as<uint64_t>(), have ? e->tb.ex_cnt.as<uint32_t>() : nullptr,
                               e->tb.ex.as<LbExtraRec>(), (uint64_t)e->n_keys, d_rows, cap_rows, d_count,
                               e->stream);
}

int ccrdt_lb_fetch_extra(ccrdt_engine* e, ccrdt_lb_extra* x) {
  CCRDT_TRY(check_type(e, CCRDT_LEADERBOARD));
  if (!x) return CCRDT_EINVAL;
  const uint64_t nk = (uint64_t)e->n_keys, n = e->last_n_ops;
  if (x->kind && n) memset(x->kind, CCRDT_NOOP, n);
  if (!n || !nk || !e->tb.ex_cnt.p) return CCRDT_OK;
  // packed on the device ([key, op, id, score] rows, the replication
  // exchange's pack kernel); only those rows cross PCIe
  TypeBufs& T = e->tb;
  uint64_t cap = std::max<uint64_t>(T.stage[7].bytes / 32, 4096);
  uint32_t cnt = 0;
  for (int pass = 0; pass < 2; ++pass) {
    CCRDT_TRY(T.stage[7].ensure(cap * 32));
    CCRDT_TRY(T.status.ensure(64));
    CCRDT_TRY(lb_launch_pack_extras(T.kp.as<uint64_t>(), T.ex_cnt.as<uint32_t>(), T.ex.as<LbExtraRec>(), nk,
                                    T.stage[7].as<int64_t>(), (int64_t)cap, T.status.as<uint32_t>() + 8,
                                    e->stream));
    CCRDT_HIP(hipMemcpyAsync(e->h_status, T.status.as<uint32_t>() + 8, 4, hipMemcpyDeviceToHost, e->stream));
    CCRDT_HIP(hipStreamSynchronize(e->stream));
    memcpy(&cnt, e->h_status, 4);
    if (cnt <= cap) break;
    cap = cnt;
  }
  std::vector<int64_t> rows;
  CCRDT_TRY(d2h(rows, T.stage[7], (uint64_t)cnt * 4, e->stream));
  for (uint64_t i = 0; i < cnt; ++i) {
    const int64_t* r = &rows[i * 4];
    const uint64_t op = (uint64_t)r[1];
    if (op >= n) continue;
    if (x->kind) x->kind[op] = CCRDT_LB_ADD;
    if (x->id) x->id[op] = r[2];
    if (x->score) x->score[op] = r[3];
  }
  return CCRDT_OK;
}

int ccrdt_lb_apply(ccrdt_engine* e, const ccrdt_lb_ops* ops, ccrdt_lb_extra* extra) {
  CCRDT_TRY(check_type(e, CCRDT_LEADERBOARD));
  if (!ops || !ops->key_ptr) return CCRDT_EINVAL;
  const uint64_t nk = (uint64_t)e->n_keys, n = (uint64_t)ops->n_ops;
  CCRDT_TRY(check_csr(ops->key_ptr, nk, n));
  TypeBufs& T = e->tb;
  CCRDT_TRY(h2d(*e, T.stage[0], ops->key_ptr, (nk + 1) * 8));
  CCRDT_TRY(h2d(*e, T.stage[1], ops->kind, n));
  CCRDT_TRY(h2d(*e, T.stage[2], ops->id, n * 8));
  CCRDT_TRY(h2d(*e, T.stage[3], ops->score, n * 8));
  ccrdt_lb_ops d{ops->n_ops, T.stage[0].as<uint64_t>(), T.stage[1].as<uint8_t>(), T.stage[2].as<int64_t>(),
                 T.stage[3].as<int64_t>()};
  CCRDT_TRY(ccrdt_lb_apply_device(e, &d));
  if (extra) CCRDT_TRY(ccrdt_lb_fetch_extra(e, extra));
  return CCRDT_OK;
}

namespace {
struct LbHost {
  std::vector<LbMeta> meta;
  std::vector<int64_t> id, score;
  std::vector<uint8_t> st;
};
// Keys [k0, k1) only (board offsets rebased to the downloaded slice).
int lb_download(ccrdt_engine* e, LbHost& h, uint64_t k0, uint64_t k1) {
  const uint64_t nk = k1 - k0;
  h.meta.assign(nk, LbMeta{0, 0, 0, 0xFFFFFFFFu});
  if (e->fresh || !nk) return CCRDT_OK;
  TypeBufs& T = e->tb;
  const int c = T.tcur;
  CCRDT_TRY(d2h_at(h.meta, T.lb_meta[c], k0, nk, e->stream));
  uint64_t b = ~0ull, t = 0;
  for (const LbMeta& m : h.meta) {
    b = std::min<uint64_t>(b, m.off);
    t = std::max<uint64_t>(t, (uint64_t)m.off + m.n);
  }
  if (t <= b) b = t = 0;
  for (LbMeta& m : h.meta) m.off = (uint32_t)(m.off - b);
  CCRDT_TRY(d2h_at(h.id, T.lb_id[c], b, t - b, e->stream));
  CCRDT_TRY(d2h_at(h.score, T.lb_score[c], b, t - b, e->stream));
  CCRDT_TRY(d2h_at(h.st, T.lb_st[c], b, t - b, e->stream));
  return CCRDT_OK;
}

}  // namespace

int ccrdt_lb_state_sizes(ccrdt_engine* e, int64_t* n_obs, int64_t* n_masked, int64_t* n_bans) {
  CCRDT_TRY(check_type(e, CCRDT_LEADERBOARD));
  LbHost h;
  CCRDT_TRY(lb_download(e, h, 0, (uint64_t)e->n_keys));
  int64_t o = 0, m = 0, b = 0;
  for (const LbMeta& mt : h.meta)
    for (uint32_t j = 0; j < mt.n; ++j) {
      const uint8_t s = h.st[mt.off + j];
      o += s == LB_OBS;
      m += s == LB_MASKED;
      b += s == LB_BANNED;
    }
  *n_obs = o;
  *n_masked = m;
  *n_bans = b;
  return CCRDT_OK;
}

int ccrdt_lb_export(ccrdt_engine* e, ccrdt_lb_state* out) {
  return ccrdt_lb_export_range(e, 0, e ? e->n_keys : 0, out);
}

int ccrdt_lb_range_sizes(ccrdt_engine* e, int64_t k0, int64_t k1, int64_t* n_obs, int64_t* n_masked,
                         int64_t* n_bans) {
  CCRDT_TRY(check_type(e, CCRDT_LEADERBOARD));
  CCRDT_TRY(key_range(e, k0, k1, "lb_range_sizes"));
  LbHost h;
  CCRDT_TRY(lb_download(e, h, (uint64_t)k0, (uint64_t)k1));
  int64_t o = 0, m = 0, b = 0;
  for (const LbMeta& mt : h.meta)
    for (uint32_t j = 0; j < mt.n; ++j) {
      const uint8_t s = h.st[mt.off + j];
      o += s == LB_OBS;
      m += s == LB_MASKED;
      b += s == LB_BANNED;
    }
  *n_obs = o;
  *n_masked = m;
  *n_bans = b;
  return CCRDT_OK;
}

int ccrdt_lb_export_range(ccrdt_engine* e, int64_t k0, int64_t k1, ccrdt_lb_state* out) {
  CCRDT_TRY(check_type(e, CCRDT_LEADERBOARD));
  CCRDT_TRY(key_range(e, k0, k1, "lb_export_range"));
  LbHost h;
  CCRDT_TRY(lb_download(e, h, (uint64_t)k0, (uint64_t)k1));
  const uint64_t nk = (uint64_t)(k1 - k0);
  uint64_t po = 0, pm = 0, pb = 0;
  out->obs_ptr[0] = out->m_ptr[0] = out->b_ptr[0] = 0;
  std::vector<std::pair<int64_t, int64_t>> o, m;
  std::vector<int64_t> b;
  for (uint64_t k = 0; k < nk; ++k) {
    const LbMeta& mt = h.meta[k];
    o.clear();
    m.clear();
    b.clear();
    for (uint32_t j = 0; j < mt.n; ++j) {
      const uint64_t g = (uint64_t)mt.off + j;
      if (h.st[g] == LB_OBS) o.push_back({h.id[g], h.score[g]});
      else if (h.st[g] == LB_MASKED) m.push_back({h.id[g], h.score[g]});
      else b.push_back(h.id[g]);
    }
    std::sort(o.begin(), o.end());
    std::sort(m.begin(), m.end());
    std::sort(b.begin(), b.end());
    for (auto& [i, s] : o) {
      out->obs_id[po] = i;
      out->obs_score[po++] = s;
    }
    for (auto& [i, s] : m) {
      out->m_id[pm] = i;
      out->m_score[pm++] = s;
    }
    for (int64_t i : b) out->b_id[pb++] = i;
    out->obs_ptr[k + 1] = po;
    out->m_ptr[k + 1] = pm;
    out->b_ptr[k + 1] = pb;
    const bool mv = mt.minq != 0xFFFFFFFFu;
    out->min_valid[k] = mv;
    out->min_id[k] = mv ? h.id[mt.off + mt.minq] : 0;
    out->min_score[k] = mv ? h.score[mt.off + mt.minq] : 0;
  }
  return CCRDT_OK;
}

int ccrdt_lb_import(ccrdt_engine* e, const ccrdt_lb_state* in) {
  CCRDT_TRY(check_type(e, CCRDT_LEADERBOARD));
  const uint64_t nk = (uint64_t)e->n_keys;
  std::vector<LbMeta> meta(nk);
  std::vector<int64_t> id, score;
  std::vector<uint8_t> st;
  for (uint64_t k = 0; k < nk; ++k) {
    LbMeta m{(uint32_t)id.size(), 0, 0, 0xFFFFFFFFu};
    std::vector<int64_t> all;
    auto put = [&](int64_t i, int64_t s, uint8_t t) {
      id.push_back(i);
      score.push_back(s);
      st.push_back(t);
      all.push_back(i);
    };
    for (uint64_t j = in->obs_ptr[k]; j < in->obs_ptr[k + 1]; ++j) put(in->obs_id[j], in->obs_score[j], LB_OBS);
    for (uint64_t j = in->m_ptr[k]; j < in->m_ptr[k + 1]; ++j) put(in->m_id[j], in->m_score[j], LB_MASKED);
    for (uint64_t j = in->b_ptr[k]; j < in->b_ptr[k + 1]; ++j) put(in->b_id[j], 0, LB_BANNED);
    std::sort(all.begin(), all.end());
    if (std::adjacent_find(all.begin(), all.end()) != all.end()) {
      set_error("lb_import: Observed, Masked and Bans must be disjoint by Id");
      return CCRDT_EINVAL;
    }
    const uint64_t nobs = in->obs_ptr[k + 1] - in->obs_ptr[k];
    const uint64_t nmask = in->m_ptr[k + 1] - in->m_ptr[k];
    if ((int64_t)nobs > e->k || (nmask && (int64_t)nobs != e->k)) {
      set_error("lb_import: |Observed| > Size, or Masked non-empty with Observed not full");
      return CCRDT_EINVAL;
    }
    m.n = (uint32_t)(id.size() - m.off);
    m.nobs = (uint32_t)nobs;
    if (in->min_valid[k]) {
      for (uint32_t j = 0; j < nobs; ++j)
        if (id[m.off + j] == in->min_id[k] && score[m.off + j] == in->min_score[k]) m.minq = j;
      if (m.minq == 0xFFFFFFFFu) {
        set_error("lb_import: Min is not an Observed pair");
        return CCRDT_EINVAL;
      }
    } else if (nobs) {
      set_error("lb_import: Min is nil but Observed is not empty");
      return CCRDT_EINVAL;
    }
    meta[k] = m;
  }
  TypeBufs& T = e->tb;
  const int c = T.tcur;
  CCRDT_TRY(h2d(*e, T.lb_meta[c], meta.data(), nk * sizeof(LbMeta)));
  CCRDT_TRY(h2d(*e, T.lb_id[c], id.data(), id.size() * 8));
  CCRDT_TRY(h2d(*e, T.lb_score[c], score.data(), score.size() * 8));
  CCRDT_TRY(h2d(*e, T.lb_st[c], st.data(), st.size()));
  CCRDT_HIP(hipStreamSynchronize(e->stream));
  e->fresh = false;
  return CCRDT_OK;
}

int ccrdt_lb_import_range(ccrdt_engine* e, int64_t k0, int64_t k1, const ccrdt_lb_state* in) {
  CCRDT_TRY(check_type(e, CCRDT_LEADERBOARD));
  CCRDT_TRY(key_range(e, k0, k1, "lb_import_range"));
  if (!in) return CCRDT_EINVAL;
  const uint64_t nk = (uint64_t)e->n_keys, a = (uint64_t)k0, b = (uint64_t)k1;
  int64_t no = 0, nm = 0, nb = 0;
  CCRDT_TRY(ccrdt_lb_state_sizes(e, &no, &nm, &nb));
  std::vector<uint64_t> op(nk + 1), mp(nk + 1), bp(nk + 1);
  std::vector<int64_t> oi(no + 1), os(no + 1), mi(nm + 1), ms(nm + 1), bi(nb + 1), mid(nk), msc(nk);
  std::vector<uint8_t> mv(nk);
  ccrdt_lb_state f{op.data(), oi.data(), os.data(), mp.data(), mi.data(), ms.data(), bp.data(),
                   bi.data(), mv.data(), mid.data(), msc.data()};
  CCRDT_TRY(ccrdt_lb_export(e, &f));
  oi.resize(no);
  os.resize(no);
  mi.resize(nm);
  ms.resize(nm);
  bi.resize(nb);
  std::vector<uint64_t> op2, mp2, bp2, tmp;
  std::vector<int64_t> oi2, os2, mi2, ms2, bi2;
  splice_csr(op, oi, in->obs_ptr, in->obs_id, a, b, op2, oi2);
  splice_csr(op, os, in->obs_ptr, in->obs_score, a, b, tmp, os2);
  splice_csr(mp, mi, in->m_ptr, in->m_id, a, b, mp2, mi2);
  splice_csr(mp, ms, in->m_ptr, in->m_score, a, b, tmp, ms2);
  splice_csr(bp, bi, in->b_ptr, in->b_id, a, b, bp2, bi2);
  for (uint64_t k = a; k < b; ++k) {
    mv[k] = in->min_valid[k - a];
    mid[k] = in->min_id[k - a];
    msc[k] = in->min_score[k - a];
  }
  for (auto* v : {&oi2, &os2, &mi2, &ms2, &bi2}) v->push_back(0);
  ccrdt_lb_state g{op2.data(), oi2.data(), os2.data(), mp2.data(), mi2.data(), ms2.data(), bp2.data(),
                   bi2.data(), mv.data(), mid.data(), msc.data()};
  return ccrdt_lb_import(e, &g);
}

int ccrdt_lb_downstream(ccrdt_engine* e, int64_t n, const uint64_t* key, const uint8_t* op,
                        const int64_t* id, const int64_t* score, uint8_t* out_kind) {
  CCRDT_TRY(check_type(e, CCRDT_LEADERBOARD));
  if (n <= 0) return CCRDT_OK;
  for (int64_t i = 0; i < n; ++i)
    if (key[i] >= (uint64_t)e->n_keys || op[i] > 1) {
      set_error("lb_downstream: bad key or op");
      return CCRDT_EINVAL;
    }
  TypeBufs& T = e->tb;
  const uint64_t un = (uint64_t)n;
  CCRDT_TRY(h2d(*e, T.stage[0], key, un * 8));
  CCRDT_TRY(h2d(*e, T.stage[1], op, un));
  CCRDT_TRY(h2d(*e, T.stage[2], id, un * 8));
  CCRDT_TRY(h2d(*e, T.stage[3], score, un * 8));
  CCRDT_TRY(T.stage[4].ensure(un));
  const int c = T.tcur;
  for (DevBuf* d : {&T.lb_meta[c], &T.lb_id[c], &T.lb_score[c], &T.lb_st[c]}) CCRDT_TRY(d->ensure(8));
  LbDownArgs a{};
  a.n = n;
  a.k = (uint32_t)std::min<int64_t>(e->k, 0xFFFFFFFFll);
  a.key = T.stage[0].as<uint64_t>();
  a.op = T.stage[1].as<uint8_t>();
  a.id = T.stage[2].as<int64_t>();
  a.score = T.stage[3].as<int64_t>();
  a.out = T.stage[4].as<uint8_t>();
  a.meta = T.lb_meta[c].as<LbMeta>();
  a.eid = T.lb_id[c].as<int64_t>();
  a.escore = T.lb_score[c].as<int64_t>();
  a.est = T.lb_st[c].as<uint8_t>();
  a.fresh = e->fresh ? 1 : 0;
  CCRDT_TRY(lb_launch_downstream(a, e->stream));
  CCRDT_HIP(hipMemcpyAsync(out_kind, T.stage[4].p, un, hipMemcpyDeviceToHost, e->stream));
  CCRDT_HIP(hipStreamSynchronize(e->stream));
  return CCRDT_OK;
}

// ============================================== wordcount / worddocumentcount
static uint64_t pow2_at_least(uint64_t x) {
  uint64_t p = 1024;
  while (p < x) p <<= 1;
  return p;
}

static uint64_t wc_next_seed(uint64_t z) {  // splitmix64 step
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static WcArgs wc_table_args(ccrdt_engine* e, int side) {
  TypeBufs& T = e->tb;
  WcArgs a{};
  a.n_keys = e->n_keys;
  a.wdc = e->type == CCRDT_WORDDOCUMENTCOUNT;
  a.t = T.t_tab[side].as<WcSlot>();
  a.tm = T.t_meta[side].as<WcMeta>();
  a.t_cnt = T.t_cnt[side].as<unsigned long long>();
  a.t_mask = T.t_slots[side] ? T.t_slots[side] - 1 : 0;
  a.seed = T.wc_seed;
  a.weak0 = getenv("CCRDT_WC_WEAK0") ? 1 : 0;
  a.arena = T.arena.as<uint8_t>();
  a.status = T.status.as<uint32_t>();
  return a;
}

static int wc_alloc_table(ccrdt_engine* e, int side, uint64_t slots) {
  TypeBufs& T = e->tb;
  if (slots > (1ull << 32)) {  // (check records hold 32-bit slot indices)
    set_error("wc: word table above 2^32 slots");
    return CCRDT_ENOMEM;
  }
  CCRDT_TRY(T.t_tab[side].ensure(slots * sizeof(WcSlot)));
  CCRDT_TRY(T.t_meta[side].ensure(slots * sizeof(WcMeta)));
  CCRDT_TRY(T.t_cnt[side].ensure(slots * 8));
  CCRDT_HIP(hipMemsetAsync(T.t_tab[side].p, 0, slots * sizeof(WcSlot), e->stream));
  CCRDT_HIP(hipMemsetAsync(T.t_cnt[side].p, 0, slots * 8, e->stream));
  T.t_slots[side] = slots;
  return CCRDT_OK;
}

int ccrdt_wc_apply_device(ccrdt_engine* e, const ccrdt_wc_docs* docs) {
  CCRDT_TRY(check_type(e, CCRDT_WORDCOUNT));
  if (!docs || !docs->key_ptr || !docs->doc_off || (docs->n_bytes && !docs->bytes)) {
    set_error("wc_apply: null arrays");
    return CCRDT_EINVAL;
  }
  if (e->n_keys > 0xFFFFFFFFll) return CCRDT_EINVAL;
  TypeBufs& T = e->tb;
  const uint64_t nd = (uint64_t)docs->n_docs, nk = (uint64_t)e->n_keys;
  CCRDT_TRY(T.status.ensure(64));
  CCRDT_TRY(T.arena_top.ensure(16));
  if (e->fresh) {
    CCRDT_HIP(hipMemsetAsync(T.arena_top.p, 0, 16, e->stream));
    T.t_slots[T.tcur] = 0;
  }
  // document keys and token counts
  CCRDT_TRY(T.stage[0].ensure(nd * 8 + 8));
  CCRDT_TRY(T.stage[1].ensure(nd * 8 + 8));
  CCRDT_TRY(wc_launch_doc_key(docs->key_ptr, nk, nd, T.stage[0].as<uint64_t>(), e->stream));
  // tokens per document: worddocumentcount sizes its (document, word) dedupe
  // table by them; wordcount only sizes its word table, for which the bound
  // bytes + documents will do (the table regrows if a batch overflows it)
  std::vector<uint64_t> ntok;
  uint64_t tokens = 0;
  if (e->type == CCRDT_WORDDOCUMENTCOUNT) {
    CCRDT_TRY(wc_launch_count(docs->doc_off, docs->bytes, nd, T.stage[1].as<uint64_t>(), e->stream));
    CCRDT_TRY(d2h(ntok, T.stage[1], nd, e->stream));
    for (uint64_t t : ntok) tokens += t;
  } else {
    ntok.assign(nd, 0);
    tokens = docs->n_bytes + nd;
  }
  // documents -> chunks of WC_TPW tiles of WC_TILE bytes (one wave each)
  std::vector<uint64_t> doff(nd + 1), tptr(nd + 1);
  if (nd) {
    CCRDT_HIP(hipMemcpyAsync(doff.data(), docs->doc_off, (nd + 1) * 8, hipMemcpyDeviceToHost, e->stream));
    CCRDT_HIP(hipStreamSynchronize(e->stream));
  }
  tptr[0] = 0;
  for (uint64_t d = 0; d < nd; ++d)
    tptr[d + 1] = tptr[d] + ((doff[d + 1] - doff[d]) / WC_TILE + WC_TPW) / WC_TPW;
  CCRDT_TRY(h2d(*e, T.stage[4], tptr.data(), (nd + 1) * 8));
  if (nd > 0xFFFFFFFFull) {
    set_error("wc_apply: more than 2^32 documents in one batch");
    return CCRDT_EINVAL;
  }
  std::vector<uint32_t> cdoc(tptr[nd] + 1, 0u);  // chunk -> document (lives until the batch is done)
  for (uint64_t d = 0; d < nd; ++d)
    for (uint64_t c = tptr[d]; c < tptr[d + 1]; ++c) cdoc[c] = (uint32_t)d;
  CCRDT_TRY(h2d(*e, T.stage[5], cdoc.data(), cdoc.size() * 4));
  // worddocumentcount: groups of WC_WAVES_WDC chunks of one document (one workgroup each)
  std::vector<uint64_t> gptr(nd + 1, 0);
  std::vector<uint32_t> gdoc;
  if (e->type == CCRDT_WORDDOCUMENTCOUNT) {
    for (uint64_t d = 0; d < nd; ++d) gptr[d + 1] = gptr[d] + (tptr[d + 1] - tptr[d] + WC_WAVES_WDC - 1) / WC_WAVES_WDC;
    gdoc.resize(gptr[nd] + 1, 0u);
    for (uint64_t d = 0; d < nd; ++d)
      for (uint64_t g = gptr[d]; g < gptr[d + 1]; ++g) gdoc[g] = (uint32_t)d;
    CCRDT_TRY(h2d(*e, T.stage[6], gptr.data(), (nd + 1) * 8));
    CCRDT_TRY(h2d(*e, T.stage[7], gdoc.data(), gdoc.size() * 4));
  }
  std::vector<uint64_t> top;
  CCRDT_TRY(d2h(top, T.arena_top, 2, e->stream));
  const uint64_t words_old = e->fresh ? 0 : top[1], arena_used = e->fresh ? 0 : top[0];
  // arena: room for every byte of the batch (upper bound of new word bytes)
  // (+32: the verify pass reads three aligned 8-byte words around a word)
  if (arena_used + docs->n_bytes + 32 > T.arena_cap) {
    DevBuf grown;
    const uint64_t cap = std::max<uint64_t>(2 * (arena_used + docs->n_bytes) + 32, 4096);
    CCRDT_TRY(grown.ensure(cap));
    if (arena_used)
      CCRDT_HIP(hipMemcpyAsync(grown.p, T.arena.p, arena_used, hipMemcpyDeviceToDevice, e->stream));
    CCRDT_HIP(hipStreamSynchronize(e->stream));
    T.arena.release();
    T.arena = grown;
    grown.p = nullptr;
    T.arena_cap = cap;
  }
  const int in = T.tcur, out = 1 - T.tcur;
  // (a batch's new words are guessed at <= 2^20: the table then stays
  // resident in the 256 MiB Infinity Cache; a batch with more overflows it and
  // is re-run on a table four times larger)
  uint64_t slots = pow2_at_least(2 * (words_old + std::min<uint64_t>(tokens, 1ull << 20)));
  bool reseeded = false;
  uint64_t dmul = 1;  // worddocumentcount dedupe table: multiple of its first size
  if (getenv("CCRDT_WC_SLOTS")) slots = strtoull(getenv("CCRDT_WC_SLOTS"), nullptr, 0);
  // the check list: tokens whose identity the insert kernel leaves open
  // (words of more than WC_SHORT bytes; slots whose identity was not yet
  // visible); a batch that fills it is verified token by token instead
  // (CCRDT_WC_CHK_CAP: test hook for the list's capacity)
  uint64_t chk_cap = std::min<uint64_t>(docs->n_bytes / 128 + 65536, 1ull << 27);
  if (getenv("CCRDT_WC_CHK_CAP")) chk_cap = strtoull(getenv("CCRDT_WC_CHK_CAP"), nullptr, 0);
  CCRDT_TRY(T.chk.ensure(std::max<uint64_t>(chk_cap, 1) * sizeof(WcChk)));
  // the count list (WcArgs::cl): token blocks for the LDS misses' counts
  // (room for a sixteenth of the bytes plus a block per chunk), one flush
  // region per insert workgroup; CCRDT_WC_NOLIST=1 keeps the device adds
  const uint64_t n_chunks = tptr[nd];
  const bool wdc = e->type == CCRDT_WORDDOCUMENTCOUNT;
  bool use_cl = !(getenv("CCRDT_WC_NOLIST") && atoi(getenv("CCRDT_WC_NOLIST")));
  // worddocumentcount: document lists instead of the dedupe table
  // (CCRDT_WC_DLIST=0: the dedupe table; also when the word table needs more
  // than WC_DL_MAXPASS bitmap passes, or a document's list overflows)
  bool use_dl = wdc && !(getenv("CCRDT_WC_DLIST") && !atoi(getenv("CCRDT_WC_DLIST")));
  // region of a document: twice its tokens + a block per wave (wc_dl_push)
  std::vector<uint64_t> dl_rn(use_dl ? nd : 0);
  if (use_dl && nd) {
    std::vector<uint64_t> pre(nd + 1, 0);
    for (uint64_t d = 0; d < nd; ++d) {
      dl_rn[d] = 2 * ntok[d] + (gptr[d + 1] - gptr[d]) * WC_WAVES_WDC * WC_DL_BLK;
      pre[d + 1] = pre[d] + dl_rn[d];
    }
    CCRDT_TRY(h2d(*e, T.dl_pre, pre.data(), (nd + 1) * 8));
  }
  const uint64_t cl_entries = docs->n_bytes / 16 + n_chunks * WC_BLK;
  uint32_t shard_blocks = (uint32_t)std::min<uint64_t>((cl_entries / WC_BLK + WC_NSHARD - 1) / WC_NSHARD + 1,
                                                       0xFFFFFFFFull / WC_BLK / WC_NSHARD);
  if (getenv("CCRDT_WC_CL_BLOCKS")) shard_blocks = (uint32_t)strtoul(getenv("CCRDT_WC_CL_BLOCKS"), nullptr, 0);  // test hook
  const uint64_t n_tb = (uint64_t)WC_NSHARD * shard_blocks;
  const uint32_t fl_tab = wdc ? WC_TAB_WDC : WC_TAB_WC;
  const uint64_t n_fl = wdc ? gptr[nd] : (n_chunks + WC_WAVES_WC - 1) / WC_WAVES_WC;
  for (int attempt = 0;; ++attempt) {
    // new table (rehash of the current words), then the batch
    CCRDT_TRY(wc_alloc_table(e, out, slots));
    WcArgs a = wc_table_args(e, out);
    if (!e->fresh && T.t_slots[in])
      CCRDT_TRY(wc_launch_rehash(T.t_tab[in].as<WcSlot>(), T.t_meta[in].as<WcMeta>(), T.t_cnt[in].as<unsigned long long>(),
                                 T.t_slots[in], a, e->stream));
    CCRDT_HIP(hipMemsetAsync(T.status.p, 0, 16, e->stream));
    a.chk = T.chk.as<WcChk>();
    a.chk_cap = (uint32_t)std::min<uint64_t>(chk_cap, 0xFFFFFFFFull);
    // (bucket sums: buckets of 2^WC_CL_MAXSH slots -- few buckets, so the
    // scatter pass writes long runs -- at most WC_CL_NB of them)
    uint32_t lg = 0;
    while ((1ull << lg) < slots) ++lg;
    const uint32_t bsh = std::min<uint32_t>(lg, WC_CL_MAXSH);
    const bool cl_on = use_cl && (slots >> bsh) <= WC_CL_NB && n_tb * WC_BLK + n_fl * fl_tab < (1ull << 32);
    const uint32_t dl_passes = (uint32_t)((slots + WC_DL_BITS - 1) / WC_DL_BITS);
    const bool dl_on = use_dl && dl_passes <= WC_DL_MAXPASS;
    if (cl_on) {
      CCRDT_TRY(T.cl.ensure(n_tb * WC_BLK * 4));
      CCRDT_TRY(T.cl_bcnt.ensure(n_tb * 4));
      CCRDT_TRY(T.fl.ensure(std::max<uint64_t>(n_fl * fl_tab, 1) * 8));
      CCRDT_TRY(T.cl_small.ensure((WC_NSHARD + 2 * WC_CL_NB) * 4 + (WC_CL_NB + 1) * 8));
      CCRDT_HIP(hipMemsetAsync(T.cl_small.p, 0, (WC_NSHARD + 2 * WC_CL_NB) * 4, e->stream));
      a.cl = T.cl.as<uint32_t>();
      a.cl_bcnt = T.cl_bcnt.as<uint32_t>();
      a.cl_cur = T.cl_small.as<uint32_t>();
      a.cl_shard_blocks = shard_blocks;
      a.fl = dl_on ? nullptr : T.fl.as<uint64_t>();  // (document lists: the flush appends pairs instead)
    }
    a.doc_off = docs->doc_off;
    a.bytes = docs->bytes;
    a.n_bytes = docs->n_bytes;
    CCRDT_HIP(hipEventRecord(e->evk0, e->stream));
    // worddocumentcount: the (document, word) dedupe table is sized by the
    // chunk's tokens; documents are processed in chunks of <= 2^28 tokens
    // (wordcount: one launch)
    // (test hooks: CCRDT_WC_LAUNCH_TOKENS, the tokens per launch;
    // CCRDT_WC_DTAGS, the document tags before the dedupe table is cleared)
    const uint64_t launch_tok = getenv("CCRDT_WC_LAUNCH_TOKENS") ? strtoull(getenv("CCRDT_WC_LAUNCH_TOKENS"), nullptr, 0) : (1ull << 28);
    const uint64_t dtags = getenv("CCRDT_WC_DTAGS") ? strtoull(getenv("CCRDT_WC_DTAGS"), nullptr, 0) : (1ull << 24);
    // (worddocumentcount dedupe entries hold a document tag in 24 bits: at
    // most 2^23 documents per launch)
    auto launch_end = [&](uint64_t x0, uint64_t& tk) {
      uint64_t x1 = x0;
      tk = 0;
      while (x1 < nd && (x1 == x0 || !a.wdc || (tk + ntok[x1] <= launch_tok && x1 - x0 < (1ull << 23))))
        tk += ntok[x1++];
      return x1;
    };
    uint64_t max_rn = 0, max_docs = 0;  // (the document lists are sized once for every launch)
    for (uint64_t x0 = 0, tk = 0; x0 < nd;) {
      const uint64_t x1 = launch_end(x0, tk);
      uint64_t rn = 0;
      for (uint64_t x = x0; x < x1 && use_dl; ++x) rn += dl_rn[x];
      max_rn = std::max(max_rn, rn);
      max_docs = std::max(max_docs, x1 - x0);
      x0 = x1;
    }
    uint64_t d0 = 0;
    while (d0 < nd) {
      uint64_t tk = 0;
      const uint64_t d1 = launch_end(d0, tk);
      a.n_docs = (int64_t)(d1 - d0);
      a.doc_key = T.stage[0].as<uint64_t>() + d0;
      a.doc_off = docs->doc_off + d0;
      a.tile_ptr = T.stage[4].as<uint64_t>() + d0;
      a.tile0 = tptr[d0];
      a.chunk_doc = T.stage[5].as<uint32_t>();
      a.doc0 = d0;
      if (a.wdc) {
        a.group_doc = T.stage[7].as<uint32_t>();
        a.group_ptr = T.stage[6].as<uint64_t>() + d0;
        a.group0 = gptr[d0];
        a.n_groups = gptr[d1] - gptr[d0];
      }
      if (a.wdc && dl_on) {
        CCRDT_TRY(T.dl.ensure(std::max<uint64_t>(max_rn, 1) * 4));
        CCRDT_TRY(T.dl_cur.ensure(std::max<uint64_t>(max_docs, 1) * 4));
        CCRDT_HIP(hipMemsetAsync(T.dl_cur.p, 0, (d1 - d0) * 4, e->stream));
        a.dl = T.dl.as<uint32_t>();
        a.dl_pre = T.dl_pre.as<uint64_t>() + d0;
        a.dl_cur = T.dl_cur.as<uint32_t>();
        a.d_hash = nullptr;
      } else if (a.wdc) {
        a.dl = nullptr;
        // two slots per token (measured: half a slot per token overflowed on
        // the Zipf corpus and the re-run cost 13 ms); an overflow re-runs the
        // batch with four times the slots
        const uint64_t ds = pow2_at_least(std::max<uint64_t>(2 * tk, 1024) * dmul);
        // not cleared per launch: the launch's document tags lie above every
        // earlier launch's (WcArgs::d_base), so the old pairs read as free;
        // only a new buffer, slots never cleared, or spent tags (2^24) clear
        const uint64_t b0 = T.d_hash.bytes;
        CCRDT_TRY(T.d_hash.ensure(ds * 8));
        if (T.d_hash.bytes != b0) T.d_clean = T.d_base = 0;
        if (T.d_base + (d1 - d0) >= dtags || getenv("CCRDT_WC_DCLEAR")) {  // (diagnostic: every launch)
          T.d_clean = std::max(T.d_clean, ds);
          CCRDT_HIP(hipMemsetAsync(T.d_hash.p, 0, T.d_clean * 8, e->stream));
          T.d_base = 0;
        } else if (ds > T.d_clean) {
          CCRDT_HIP(hipMemsetAsync(T.d_hash.as<uint64_t>() + T.d_clean, 0, (ds - T.d_clean) * 8, e->stream));
          T.d_clean = ds;
        }
        a.d_hash = T.d_hash.as<uint64_t>();
        a.d_mask = ds - 1;
        a.d_base = T.d_base;
        T.d_base += d1 - d0;
      }
      a.fl_base = a.wdc ? a.group0 : 0;  // (wordcount: one launch)
      a.dbg = getenv("CCRDT_WC_IDBG") ? atoi(getenv("CCRDT_WC_IDBG")) : 0;
      CCRDT_TRY(wc_launch_insert(a, tptr[d1] - tptr[d0], e->stream));
      a.dbg = 0;
      if (a.wdc && dl_on) CCRDT_TRY(wc_launch_dl(a, d1 - d0, dl_passes, e->stream));
      d0 = d1;
    }
    CCRDT_HIP(hipEventRecord(e->evk1, e->stream));
    uint32_t st[3];
    CCRDT_TRY(read_status3(e, st));
    CCRDT_HIP(hipEventElapsedTime(&e->last_kernel_ms, e->evk0, e->evk1));
    if (st[0] && attempt < 4) {  // table (or dedupe table) too small, count list full
      if (st[0] & 1u) slots *= 4;
      if (st[0] & 2u) dmul *= 4;
      if (st[0] & 4u) use_cl = false;
      if (st[0] & 8u) use_dl = false;
      continue;
    }
    if (st[0]) {
      set_error("wc_apply: word table overflow");
      return CCRDT_ENOMEM;
    }
    // the count list summed into the counts, per bucket of slots
    if (cl_on) {
      WcClArgs c{};
      c.cl = T.cl.as<uint32_t>();
      c.bcnt = T.cl_bcnt.as<uint32_t>();
      c.cur = T.cl_small.as<uint32_t>();
      c.shard_blocks = shard_blocks;
      c.fl = T.fl.as<uint64_t>();
      c.tab = fl_tab;
      c.n_tb = n_tb;
      c.n_fl = dl_on ? 0 : n_fl;
      c.bsh = bsh;
      c.nb = (uint32_t)(slots >> bsh);
      c.bkt_cnt = T.cl_small.as<uint32_t>() + WC_NSHARD;
      c.bkt_cur = c.bkt_cnt + WC_CL_NB;
      c.bkt_off = reinterpret_cast<uint64_t*>(c.bkt_cur + WC_CL_NB);
      c.t_cnt = a.t_cnt;
      c.status = a.status;
      CCRDT_TRY(wc_launch_cl_count(c, e->stream));
      std::vector<uint64_t> tot;
      CCRDT_TRY(d2h_at(tot, T.cl_small, (WC_NSHARD + 2 * WC_CL_NB) / 2 + c.nb, 1, e->stream));
      CCRDT_TRY(T.bkt.ensure(std::max<uint64_t>(tot[0], 1) * 4));
      c.bkt = T.bkt.as<uint32_t>();
      CCRDT_TRY(wc_launch_cl_sum(c, e->stream));
    }
    // the batch's new words into the arena first (the check list's long
    // words are compared against a compact, cache-resident copy)
    a.doc_key = T.stage[0].as<uint64_t>();
    a.doc_off = docs->doc_off;
    a.n_docs = (int64_t)nd;
    a.tile_ptr = T.stage[4].as<uint64_t>();
    a.tile0 = 0;
    a.chunk_doc = T.stage[5].as<uint32_t>();
    a.doc0 = 0;
    a.group_doc = nullptr;
    a.arena = T.arena.as<uint8_t>();
    CCRDT_HIP(hipMemsetAsync((uint64_t*)T.arena_top.p + 1, 0, 8, e->stream));
    CCRDT_TRY(wc_launch_persist(a, T.arena.as<uint8_t>(), T.arena_top.as<unsigned long long>(), e->stream));
    // exactness: every token equals its word's identity -- the insert kernel
    // compared all but the check list's tokens (a full list: every token
    // again; CCRDT_WC_VERIFY=1 forces that pass)
    const bool full = (st[1] & 16u) || (getenv("CCRDT_WC_VERIFY") && atoi(getenv("CCRDT_WC_VERIFY")));
    T.wc_checks = full ? -1 : (int64_t)st[2];
    if (full) CCRDT_TRY(wc_launch_verify(a, tptr[nd], e->stream));
    else CCRDT_TRY(wc_launch_check(a, st[2], e->stream));
    CCRDT_TRY(read_status(e, st));
    st[1] &= ~16u;
    if (st[1]) {
      // the state is unchanged: the new table side is dropped, the arena
      // top goes back to the words it held
      const uint64_t back[2] = {arena_used, words_old};
      CCRDT_TRY(h2d(*e, T.arena_top, back, 16));
      CCRDT_HIP(hipStreamSynchronize(e->stream));
      if ((st[1] & 1) && !reseeded) {
        // two distinct words met on one 64-bit hash: the collision depends on
        // the bytes and the seed only, so the batch is re-run once under a
        // new seed (the rehash recomputes every old word's hash)
        reseeded = true;
        T.wc_seed = wc_next_seed(T.wc_seed);
        continue;
      }
      set_error(st[1] & 1 ? "wc_apply: 64-bit word hash collision between distinct words (also under a second seed)"
                          : "wc_apply: token lost (table overflow)");
      return CCRDT_ERANGE;
    }
    CCRDT_HIP(hipStreamSynchronize(e->stream));
    break;
  }
  T.tcur = out;
  e->fresh = false;
  return CCRDT_OK;
}

int ccrdt_wc_apply(ccrdt_engine* e, const ccrdt_wc_docs* docs) {
  CCRDT_TRY(check_type(e, CCRDT_WORDCOUNT));
  if (!docs || !docs->key_ptr || !docs->doc_off) return CCRDT_EINVAL;
  const uint64_t nk = (uint64_t)e->n_keys, nd = (uint64_t)docs->n_docs;
  CCRDT_TRY(check_csr(docs->key_ptr, nk, nd));
  if (docs->doc_off[0] != 0 || docs->doc_off[nd] != docs->n_bytes) {
    set_error("wc_apply: doc_off must start at 0 and end at n_bytes");
    return CCRDT_EINVAL;
  }
  TypeBufs& T = e->tb;
  CCRDT_TRY(h2d(*e, T.kp, docs->key_ptr, (nk + 1) * 8));
  CCRDT_TRY(h2d(*e, T.stage[2], docs->doc_off, (nd + 1) * 8));
  CCRDT_TRY(h2d(*e, T.stage[3], docs->bytes, docs->n_bytes));
  CCRDT_TRY(T.stage[3].ensure(8));
  ccrdt_wc_docs d{docs->n_docs, T.kp.as<uint64_t>(), T.stage[2].as<uint64_t>(), T.stage[3].as<uint8_t>(),
                  docs->n_bytes};
  return ccrdt_wc_apply_device(e, &d);
}

static int wc_merge_core(ccrdt_engine* e, uint64_t nw, const uint64_t* wk, const uint64_t* wo, const int64_t* wc,
                         const uint8_t* bytes, uint64_t nb, bool replace);

static int wc_merge_words(ccrdt_engine* e, int64_t n_words, const uint64_t* key_ptr,
                          const uint64_t* word_off, const uint8_t* bytes, const int64_t* count,
                          bool replace) {
  if (n_words < 0 || !key_ptr || !word_off || (n_words && !count)) {
    set_error("wc_merge: null arrays");
    return CCRDT_EINVAL;
  }
  const uint64_t nk = (uint64_t)e->n_keys, nw = (uint64_t)n_words;
  CCRDT_TRY(check_csr(key_ptr, nk, nw));
  if (word_off[0] != 0) {
    set_error("wc_merge: word_off must start at 0");
    return CCRDT_EINVAL;
  }
  for (uint64_t i = 0; i < nw; ++i) {
    if (word_off[i + 1] < word_off[i] || word_off[i + 1] - word_off[i] > 0xFFFFFFFFull) {
      set_error("wc_merge: word_off not monotone");
      return CCRDT_EINVAL;
    }
    if (count[i] < 1) {  // a map entry counts at least one token (wordcount.erl:57-58)
      set_error("wc_merge: counts must be >= 1");
      return CCRDT_EINVAL;
    }
  }
  const uint64_t nb = word_off[nw];
  if (nb && !bytes) {
    set_error("wc_merge: null bytes");
    return CCRDT_EINVAL;
  }
  TypeBufs& T = e->tb;
  // words -> device: keys, offsets, bytes, counts
  CCRDT_TRY(h2d(*e, T.kp, key_ptr, (nk + 1) * 8));
  CCRDT_TRY(h2d(*e, T.stage[2], word_off, (nw + 1) * 8));
  CCRDT_TRY(h2d(*e, T.stage[3], bytes, nb));
  CCRDT_TRY(T.stage[3].ensure(8));
  CCRDT_TRY(h2d(*e, T.stage[1], count, nw * 8));
  CCRDT_TRY(T.stage[0].ensure(nw * 8 + 8));
  CCRDT_TRY(wc_launch_doc_key(T.kp.as<uint64_t>(), nk, nw, T.stage[0].as<uint64_t>(), e->stream));
  return wc_merge_core(e, nw, T.stage[0].as<uint64_t>(), T.stage[2].as<uint64_t>(), T.stage[1].as<int64_t>(),
                       T.stage[3].as<uint8_t>(), nb, replace);
}

// The words (device arrays: key, offsets, counts, bytes) added into the maps,
// or replacing them.
static int wc_merge_core(ccrdt_engine* e, uint64_t nw, const uint64_t* wk, const uint64_t* wo, const int64_t* wc,
                         const uint8_t* bytes, uint64_t nb, bool replace) {
  TypeBufs& T = e->tb;
  CCRDT_TRY(T.status.ensure(64));
  CCRDT_TRY(T.arena_top.ensure(16));
  // replace: the maps := the words (ccrdt_wc_import); the old state stays
  // intact until the new table has been verified.
  const bool start_empty = e->fresh || replace;
  std::vector<uint64_t> top{0, 0};
  if (!e->fresh) CCRDT_TRY(d2h(top, T.arena_top, 2, e->stream));
  const uint64_t words_old = start_empty ? 0 : top[1], arena_used = top[0];
  if (arena_used + nb > T.arena_cap) {
    DevBuf grown;
    const uint64_t cap = std::max<uint64_t>(2 * (arena_used + nb), 4096);
    CCRDT_TRY(grown.ensure(cap));
    if (arena_used)
      CCRDT_HIP(hipMemcpyAsync(grown.p, T.arena.p, arena_used, hipMemcpyDeviceToDevice, e->stream));
    CCRDT_HIP(hipStreamSynchronize(e->stream));
    T.arena.release();
    T.arena = grown;
    grown.p = nullptr;
    T.arena_cap = cap;
  }
  const int in = T.tcur, out = 1 - T.tcur;
  const uint64_t slots = pow2_at_least(2 * (words_old + nw));
  WcArgs a;
  uint32_t st[2];
  for (int attempt = 0;; ++attempt) {
    CCRDT_TRY(wc_alloc_table(e, out, slots));
    a = wc_table_args(e, out);
    if (!start_empty && T.t_slots[in])
      CCRDT_TRY(wc_launch_rehash(T.t_tab[in].as<WcSlot>(), T.t_meta[in].as<WcMeta>(), T.t_cnt[in].as<unsigned long long>(),
                                 T.t_slots[in], a, e->stream));
    CCRDT_HIP(hipMemsetAsync(T.status.p, 0, 8, e->stream));
    a.bytes = bytes;
    a.n_bytes = nb;
    CCRDT_TRY(wc_launch_merge(a, wk, wo, wc, nw, 0, e->stream));
    CCRDT_TRY(wc_launch_merge(a, wk, wo, wc, nw, 1, e->stream));
    CCRDT_TRY(read_status(e, st));
    if (st[1] == 1u && attempt == 0) {  // a hash collision alone: once more under a new seed
      T.wc_seed = wc_next_seed(T.wc_seed);
      continue;
    }
    break;
  }
  if (st[0] || st[1]) {
    set_error(st[1] & 8   ? "wc_merge: a count < 1 or a key outside [0, n_keys)"
              : st[1] & 1 ? "wc_merge: 64-bit word hash collision between distinct words"
              : st[1] & 4 ? "wc_merge: a count would leave int64"
                          : "wc_merge: word table overflow");
    return st[1] & 8 ? CCRDT_EINVAL : st[1] & 5 ? CCRDT_ERANGE : CCRDT_ENOMEM;
  }
  // persist appends the new words' bytes at arena_top[0] and counts words in
  // arena_top[1]; a replaced state starts both from zero
  CCRDT_HIP(hipMemsetAsync((uint64_t*)T.arena_top.p + (start_empty ? 0 : 1), 0, start_empty ? 16 : 8,
                           e->stream));
  CCRDT_TRY(wc_launch_persist(a, T.arena.as<uint8_t>(), T.arena_top.as<unsigned long long>(), e->stream));
  CCRDT_HIP(hipStreamSynchronize(e->stream));
  T.tcur = out;
  e->fresh = false;
  return CCRDT_OK;
}

static uint64_t owner_mix(uint64_t z) {  // splitmix64 (cluster.splitmix64)
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int ccrdt_wc_owner(int64_t n_keys, int64_t n_words, const uint64_t* key_ptr, const uint64_t* word_off,
                   const uint8_t* bytes, int world, int32_t* owner) {
  if (n_keys < 0 || n_words < 0 || world < 1 || !key_ptr || (n_words && (!word_off || !owner))) {
    set_error("wc_owner: bad arguments");
    return CCRDT_EINVAL;
  }
  if (key_ptr[0] != 0 || key_ptr[n_keys] != (uint64_t)n_words) {
    set_error("wc_owner: key_ptr must run from 0 to n_words");
    return CCRDT_EINVAL;
  }
  for (int64_t k = 0; k < n_keys; ++k) {
    if (key_ptr[k + 1] < key_ptr[k]) {
      set_error("wc_owner: key_ptr not monotone");
      return CCRDT_EINVAL;
    }
    for (uint64_t i = key_ptr[k]; i < key_ptr[k + 1]; ++i) {
      uint64_t f = 0xCBF29CE484222325ull;
      for (uint64_t j = word_off[i]; j < word_off[i + 1]; ++j) f = (f ^ bytes[j]) * 0x100000001B3ull;
      owner[i] = (int32_t)(owner_mix(f ^ ((uint64_t)k * 0x9E3779B97F4A7C15ull)) % (uint64_t)world);
    }
  }
  return CCRDT_OK;
}

int ccrdt_wc_merge(ccrdt_engine* e, int64_t n_words, const uint64_t* key_ptr, const uint64_t* word_off,
                   const uint8_t* bytes, const int64_t* count) {
  CCRDT_TRY(check_type(e, CCRDT_WORDCOUNT));
  return wc_merge_words(e, n_words, key_ptr, word_off, bytes, count, false);
}

int ccrdt_wc_import(ccrdt_engine* e, int64_t n_words, const uint64_t* key_ptr, const uint64_t* word_off,
                    const uint8_t* bytes, const int64_t* count) {
  CCRDT_TRY(check_type(e, CCRDT_WORDCOUNT));
  return wc_merge_words(e, n_words, key_ptr, word_off, bytes, count, true);
}

int ccrdt_wc_partition_device(ccrdt_engine* e, int world, int64_t* d_meta, uint8_t* d_bytes, int64_t cap_words,
                              int64_t cap_bytes, int64_t* owner_words, int64_t* owner_bytes) {
  CCRDT_TRY(check_type(e, CCRDT_WORDCOUNT));
  if (world < 1 || !owner_words || !owner_bytes || cap_words < 0 || cap_bytes < 0) return CCRDT_EINVAL;
  for (int o = 0; o < world; ++o) owner_words[o] = owner_bytes[o] = 0;
  int64_t nw = 0, nb = 0;
  CCRDT_TRY(ccrdt_wc_sizes(e, &nw, &nb));
  if (!nw) return CCRDT_OK;
  if (nw > cap_words || nb > cap_bytes || !d_meta || (nb && !d_bytes)) {
    set_error("wc_partition_device: output buffers smaller than ccrdt_wc_sizes");
    return CCRDT_EINVAL;
  }
  // the owner cursors pack (rows << 40 | bytes) into one 64-bit word, so the
  // rows of one table must stay below 2^24 and its bytes below 2^40
  // (test hook CCRDT_WC_PART_MAX_WORDS lowers the row limit)
  uint64_t max_words = 1ull << 24;
  if (const char* s = getenv("CCRDT_WC_PART_MAX_WORDS")) max_words = std::min<uint64_t>(max_words, strtoull(s, nullptr, 0));
  if ((uint64_t)nw >= max_words || (uint64_t)nb >= (1ull << 40)) {
    set_error("wc_partition_device: more than 2^24 - 1 words or 2^40 - 1 bytes in one table "
              "(export with ccrdt_wc_export and partition on the host)");
    return CCRDT_ERANGE;
  }
  TypeBufs& T = e->tb;
  const int c = T.tcur;
  WcArgs a = wc_table_args(e, c);
  CCRDT_TRY(T.caps.ensure(T.t_slots[c] * 4));
  CCRDT_TRY(T.part.ensure((size_t)world * 8));
  unsigned long long* cur = T.part.as<unsigned long long>();
  CCRDT_HIP(hipMemsetAsync(cur, 0, (size_t)world * 8, e->stream));
  CCRDT_TRY(wc_launch_owner_count(a, (uint32_t)world, T.caps.as<uint32_t>(), cur, e->stream));
  std::vector<uint64_t> cnt;
  CCRDT_TRY(d2h(cnt, T.part, (uint64_t)world, e->stream));
  std::vector<uint64_t> base(world);
  uint64_t w = 0, b = 0;
  for (int o = 0; o < world; ++o) {
    owner_words[o] = (int64_t)(cnt[o] >> 40);
    owner_bytes[o] = (int64_t)(cnt[o] & ((1ull << 40) - 1));
    base[o] = (w << 40) | b;
    w += (uint64_t)owner_words[o];
    b += (uint64_t)owner_bytes[o];
  }
  CCRDT_HIP(hipMemcpyAsync(cur, base.data(), (size_t)world * 8, hipMemcpyHostToDevice, e->stream));
  CCRDT_TRY(wc_launch_owner_scatter(a, T.caps.as<uint32_t>(), cur, d_meta, d_bytes, (uint32_t)world, e->stream));
  CCRDT_HIP(hipStreamSynchronize(e->stream));
  return CCRDT_OK;
}

int ccrdt_wc_merge_device(ccrdt_engine* e, int64_t n_words, const int64_t* d_meta, const uint8_t* d_bytes,
                          int64_t n_bytes) {
  CCRDT_TRY(check_type(e, CCRDT_WORDCOUNT));
  if (n_words < 0 || n_bytes < 0 || (n_words && !d_meta) || (n_bytes && !d_bytes)) return CCRDT_EINVAL;
  const uint64_t nw = (uint64_t)n_words;
  TypeBufs& T = e->tb;
  CCRDT_TRY(T.stage[0].ensure(nw * 8 + 8));
  CCRDT_TRY(T.stage[1].ensure(nw * 8 + 8));
  CCRDT_TRY(T.stage[2].ensure((nw + 1) * 8));
  CCRDT_TRY(T.caps.ensure((nw + 1) * 8));
  CCRDT_TRY(T.part.ensure(((nw + 255) / 256 + 2) * 8));
  CCRDT_TRY(wc_launch_meta_split(d_meta, nw, T.stage[0].as<uint64_t>(), T.stage[1].as<int64_t>(), nullptr,
                                 e->stream));
  // word offsets: exclusive scan of the lengths (the low words of column 1)
  CCRDT_TRY(launch_caps_scan(nullptr, nw ? (const uint32_t*)d_meta + 2 : nullptr, 6, nw, T.caps.as<uint64_t>(),
                             T.stage[2].as<uint64_t>(), T.part.as<uint64_t>(), e->stream));
  std::vector<uint64_t> tot;
  CCRDT_TRY(d2h_at(tot, T.stage[2], nw, 1, e->stream));
  if (tot[0] != (uint64_t)n_bytes) {
    set_error("wc_merge_device: the word lengths do not add up to n_bytes");
    return CCRDT_EINVAL;
  }
  return wc_merge_core(e, nw, T.stage[0].as<uint64_t>(), T.stage[2].as<uint64_t>(), T.stage[1].as<int64_t>(),
                       d_bytes, (uint64_t)n_bytes, false);
}

int ccrdt_wc_last_checks(ccrdt_engine* e, int64_t* n_checked) {
  CCRDT_TRY(check_type(e, CCRDT_WORDCOUNT));
  if (!n_checked) return CCRDT_EINVAL;
  *n_checked = e->tb.wc_checks;
  return CCRDT_OK;
}

int ccrdt_wc_sizes(ccrdt_engine* e, int64_t* n_words, int64_t* n_bytes) {
  CCRDT_TRY(check_type(e, CCRDT_WORDCOUNT));
  if (e->fresh) {
    *n_words = *n_bytes = 0;
    return CCRDT_OK;
  }
  std::vector<uint64_t> top;
  CCRDT_TRY(d2h(top, e->tb.arena_top, 2, e->stream));
  *n_words = (int64_t)top[1];
  *n_bytes = (int64_t)top[0];
  return CCRDT_OK;
}

int ccrdt_wc_export(ccrdt_engine* e, uint64_t* key_ptr, uint64_t* word_off, uint8_t* word_bytes,
                    int64_t* count) {
  CCRDT_TRY(check_type(e, CCRDT_WORDCOUNT));
  const uint64_t nk = (uint64_t)e->n_keys;
  key_ptr[0] = 0;
  word_off[0] = 0;
  if (e->fresh) {
    for (uint64_t k = 0; k < nk; ++k) key_ptr[k + 1] = 0;
    return CCRDT_OK;
  }
  TypeBufs& T = e->tb;
  const int c = T.tcur;
  const uint64_t n = T.t_slots[c];
  std::vector<WcSlot> tab;
  std::vector<WcMeta> meta;
  std::vector<unsigned long long> cnt;
  std::vector<uint64_t> top;
  std::vector<uint8_t> arena;
  CCRDT_TRY(d2h(tab, T.t_tab[c], n, e->stream));
  CCRDT_TRY(d2h(meta, T.t_meta[c], n, e->stream));
  CCRDT_TRY(d2h(cnt, T.t_cnt[c], n, e->stream));
  CCRDT_TRY(d2h(top, T.arena_top, 2, e->stream));
  CCRDT_TRY(d2h(arena, T.arena, top[0], e->stream));
  std::vector<std::tuple<uint32_t, std::string, uint64_t>> words;
  for (uint64_t i = 0; i < n; ++i)
    if (tab[i].h)
      words.emplace_back(meta[i].key, std::string((const char*)arena.data() + meta[i].ref, meta[i].len), cnt[i]);
  std::sort(words.begin(), words.end());
  uint64_t w = 0, b = 0, p = 0;
  for (uint64_t k = 0; k < nk; ++k) {
    while (p < words.size() && std::get<0>(words[p]) == k) {
      const std::string& s = std::get<1>(words[p]);
      memcpy(word_bytes + b, s.data(), s.size());
      b += s.size();
      count[w] = (int64_t)std::get<2>(words[p]);
      word_off[++w] = b;
      ++p;
    }
    key_ptr[k + 1] = w;
  }
  return CCRDT_OK;
}

}  // extern "C"
