// engine_types.cpp — per-type engine lifecycle (init / reset / clone).
#include "common.hpp"
#include "engine.hpp"

using namespace ccrdt;

static int copy_buf(DevBuf& dst, const DevBuf& src, hipStream_t st) {
  if (!src.p) return CCRDT_OK;
  CCRDT_TRY(dst.ensure(src.bytes));
  CCRDT_HIP(hipMemcpyAsync(dst.p, src.p, src.bytes, hipMemcpyDeviceToDevice, st));
  return CCRDT_OK;
}

int ccrdt_engine::init_type() {
  fresh = true;
  return CCRDT_OK;
}

int ccrdt_engine::reset_type() { return CCRDT_OK; }

void ccrdt_engine::release_types() {
  for (DevBuf* d : {&tb.avg_sum, &tb.avg_num, &tb.tk_id, &tb.tk_score, &tb.tk_cnt, &tb.tk_off,
                    &tb.tk_scratch, &tb.lb_meta, &tb.lb_id, &tb.lb_score, &tb.lb_flag, &tb.lb_meta2,
                    &tb.lb_id2, &tb.lb_score2, &tb.lb_flag2, &tb.wc_hash, &tb.wc_off, &tb.wc_len,
                    &tb.wc_cnt, &tb.wc_bytes, &tb.wc_used, &tb.wc_status, &tb.scratch0, &tb.scratch1,
                    &tb.scratch2, &tb.scratch3})
    d->release();
}

int ccrdt_engine::clone_from(const ccrdt_engine& src) {
  CCRDT_HIP(hipStreamSynchronize(src.stream));
  fresh = src.fresh;
  if (type == CCRDT_TOPK_RMV) {
    cur = src.cur;
    const TrmvBufs& s = src.trmv[src.cur];
    TrmvBufs& d = trmv[cur];
    CCRDT_TRY(copy_buf(d.meta, s.meta, stream));
    CCRDT_TRY(copy_buf(d.pl_id, s.pl_id, stream));
    CCRDT_TRY(copy_buf(d.pl_info, s.pl_info, stream));
    CCRDT_TRY(copy_buf(d.m_score, s.m_score, stream));
    CCRDT_TRY(copy_buf(d.m_ts, s.m_ts, stream));
    CCRDT_TRY(copy_buf(d.m_dc, s.m_dc, stream));
    CCRDT_TRY(copy_buf(d.pl_slab, s.pl_slab, stream));
    CCRDT_TRY(copy_buf(d.r_vc, s.r_vc, stream));
    CCRDT_TRY(copy_buf(d.vc, s.vc, stream));
  } else {
    const TypeBufs& s = src.tb;
    CCRDT_TRY(copy_buf(tb.avg_sum, s.avg_sum, stream));
    CCRDT_TRY(copy_buf(tb.avg_num, s.avg_num, stream));
    CCRDT_TRY(copy_buf(tb.tk_id, s.tk_id, stream));
    CCRDT_TRY(copy_buf(tb.tk_score, s.tk_score, stream));
    CCRDT_TRY(copy_buf(tb.tk_cnt, s.tk_cnt, stream));
    CCRDT_TRY(copy_buf(tb.tk_off, s.tk_off, stream));
    tb.tk_slots = s.tk_slots;
    CCRDT_TRY(copy_buf(tb.lb_meta, s.lb_meta, stream));
    CCRDT_TRY(copy_buf(tb.lb_id, s.lb_id, stream));
    CCRDT_TRY(copy_buf(tb.lb_score, s.lb_score, stream));
    CCRDT_TRY(copy_buf(tb.lb_flag, s.lb_flag, stream));
    tb.lb_cap_total = s.lb_cap_total;
    CCRDT_TRY(copy_buf(tb.wc_hash, s.wc_hash, stream));
    CCRDT_TRY(copy_buf(tb.wc_off, s.wc_off, stream));
    CCRDT_TRY(copy_buf(tb.wc_len, s.wc_len, stream));
    CCRDT_TRY(copy_buf(tb.wc_cnt, s.wc_cnt, stream));
    CCRDT_TRY(copy_buf(tb.wc_bytes, s.wc_bytes, stream));
    CCRDT_TRY(copy_buf(tb.wc_used, s.wc_used, stream));
    tb.wc_slots = s.wc_slots;
    tb.wc_byte_cap = s.wc_byte_cap;
  }
  CCRDT_HIP(hipStreamSynchronize(stream));
  return CCRDT_OK;
}
