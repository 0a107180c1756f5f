// trmv_kernels.hip — the pieces of the topk_rmv apply around its tiers (the
// tiers are trmv_wave.hip and trmv_steady.hip): the capacity scan that lays
// out the new side's per-key segments, and the batched read-only
// downstream/2 probe.
//
// Reference semantics (src/antidote_ccrdt_topk_rmv.erl):
//   cmp/2 :389-395 · downstream/2 :102-124
#include "common.hpp"
#include "trmv_kernels.hpp"

namespace ccrdt {

// Strict cmp/2 of topk_rmv (:389-395): (Score, Id, Ts), DcId ignored.
__device__ __forceinline__ bool trmv_cmp(int64_t s1, int64_t i1, int64_t t1, int64_t s2, int64_t i2,
                                         int64_t t2) {
  return s1 > s2 || (s1 == s2 && i1 > i2) || (s1 == s2 && i1 == i2 && t1 > t2);
}

// ------------------------------------------------------------- capacity scan
// New segment capacities per key: old counts + this batch's ops on the key.
// Three exclusive scans (players, pool, rows) over n_keys, block = 256 x 4.
constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 4;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

// Ops of kind 2/3 (rmv: the only ones that can add a Removals row) of the
// 64 keys [k0, k0 + 64) -- lane j: key k0 + j; keys past n_keys count 0 --
// with the wave reading their op range's kind bytes as coalesced aligned
// 8-byte words (bytes of the first and last word outside the range lie in
// the same aligned word, hence the same page, and are never counted).  A
// kind above 3 counts too (the batch is rejected anyway).  P(x) = rmv bytes
// in [aligned start, x): per 64-word round, each lane's word count, a DPP
// prefix sum, and each key lane picks the prefix of the word holding its end
// boundary; the key's count is P(end) - P(start), its start being the
// previous key's end.
__device__ __forceinline__ uint32_t wave_rmv_counts(const uint64_t* key_ptr, const uint8_t* kind, uint64_t k0,
                                                    uint64_t n_keys) {
  const uint32_t lane = (uint32_t)lane_id();
  const uint64_t kl = k0 + lane < n_keys ? k0 + lane : n_keys;
  const uint64_t hi = key_ptr[kl + (k0 + lane < n_keys ? 1 : 0)];  // this key's end (past n_keys: the last end)
  const uint64_t lo0 = key_ptr[k0 < n_keys ? k0 : n_keys];
  const uint64_t hi63 = (uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)hi, 63) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(hi >> 32), 63) << 32);
  if (hi63 <= lo0) return 0u;
  const uintptr_t ab = reinterpret_cast<uintptr_t>(kind + lo0) & ~(uintptr_t)7;
  const uint64_t nw = (reinterpret_cast<uintptr_t>(kind + hi63) - ab + 7) / 8;
  const uint64_t wx = (reinterpret_cast<uintptr_t>(kind + hi) - ab) / 8;  // word of the end boundary
  const uint32_t bx = (uint32_t)((reinterpret_cast<uintptr_t>(kind + hi) - ab) & 7);
  uint64_t P = 0, carry = 0;
  for (uint64_t w0 = 0; w0 < nw; w0 += 64) {
    const uint64_t w = w0 + lane;
    const uint64_t v = w < nw ? reinterpret_cast<const uint64_t*>(ab)[w] : 0ull;
    const uint64_t bits = (v >> 1) & 0x0101010101010101ull;
    const uint32_t c = (uint32_t)__builtin_popcountll(bits);
    const uint32_t incl = wave_incl_scan_dpp(c);
    const uint32_t tot = rl32(incl, 63);
    // the end boundary's word in this round: its exclusive prefix and its
    // bytes below the boundary
    const bool here = wx >= w0 && wx < w0 + 64;
    const int src = here ? (int)(wx - w0) : (int)lane;
    const uint32_t ex = shfl32(incl - c, src);
    const uint64_t wb = (uint64_t)shfl64((int64_t)bits, src);
    const uint64_t below = bx ? (wb & ((1ull << (8 * bx)) - 1)) : 0ull;
    if (here) P = carry + ex + (uint32_t)__builtin_popcountll(below);
    carry += tot;
  }
  if (wx >= nw) P = carry;
  // the start boundary of key 0: the bytes of [ab, lo0) are not in the range
  const uint64_t ps = (uint64_t)shfl64((int64_t)P, lane ? (int)lane - 1 : 0);
  uint64_t P0 = 0;
  {
    const uint32_t b0 = (uint32_t)((reinterpret_cast<uintptr_t>(kind + lo0) - ab) & 7);
    const uint64_t v0 = *reinterpret_cast<const uint64_t*>(ab);
    P0 = b0 ? (uint64_t)__builtin_popcountll((v0 >> 1) & 0x0101010101010101ull & ((1ull << (8 * b0)) - 1)) : 0ull;
  }
  return (uint32_t)(P - (lane ? ps : P0));
}

__device__ __forceinline__ void caps_of(const TrmvApplyArgs& a, uint64_t k, uint32_t nrmv, uint64_t c[3]) {
  const uint64_t nops = trmv_key_nops(a, k, a.key_ptr[k]);
  if (a.fresh) {
    c[0] = c[1] = c[2] = nops;
  } else if (a.slack) {
    // room for in-place growth (tier R writes the key: its later batches
    // append players, slabs and rows inside these segments)
    const KeyMeta m = a.old_s.meta[k];
    c[0] = (3 * ((uint64_t)m.np + nops)) / 2 + 8;
    c[1] = (uint64_t)a.slack * ((uint64_t)m.nm + nops) + 32;  // (a.slack: the pool's factor)
    c[2] = (3 * ((uint64_t)m.nr + nrmv)) / 2 + 16;
  } else {
    const KeyMeta m = a.old_s.meta[k];
    c[0] = m.np + nops;
    c[1] = m.nm + nops;
    c[2] = m.nr + nrmv;  // (rows: rmv ops only)
  }
  // No per-key limit here: a segment is address space only.  The tiers check
  // the key's real layout against the u16 slab offsets (TRMV_SEG_MAX) and hand
  // on a key that does not fit.
}

__device__ __forceinline__ void block_scan3(uint64_t v[3], uint64_t total[3]) {
  // inclusive wave scan then cross-wave via LDS
  __shared__ uint64_t wsum[SCAN_BLOCK / 64][3];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t inc[3] = {v[0], v[1], v[2]};
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      uint64_t o = (uint64_t)shfl64((int64_t)inc[c], lane - off < 0 ? 0 : lane - off);
      if (lane >= off) inc[c] += o;
    }
  }
  if (lane == 63)
    for (int c = 0; c < 3; ++c) wsum[w][c] = inc[c];
  __syncthreads();
  for (int c = 0; c < 3; ++c) {
    uint64_t pre = 0, tot = 0;
    for (int j = 0; j < SCAN_BLOCK / 64; ++j) {
      if (j < w) pre += wsum[j][c];
      tot += wsum[j][c];
    }
    v[c] = pre + inc[c] - v[c];  // exclusive
    total[c] = tot;
  }
  __syncthreads();
}

// Pass 1: each key's rmv-op count (every wave counts 256 consecutive keys,
// 64 at a time, coalesced; key_rmv keeps them for pass 2), then the tile sums.
__global__ __launch_bounds__(SCAN_BLOCK) void trmv_scan_partials(TrmvApplyArgs a, uint64_t* partials,
                                                                    uint32_t* key_rmv) {
  __shared__ uint32_t cnt[SCAN_TILE];
  const uint64_t tile0 = (uint64_t)blockIdx.x * SCAN_TILE;
  if (!a.fresh) {
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll 1
    for (int g = 0; g < 4; ++g) {
      const uint64_t k0 = tile0 + 256u * w + 64u * g;
      uint32_t r = k0 < (uint64_t)a.n_keys ? wave_rmv_counts(a.key_ptr, a.kind, k0, (uint64_t)a.n_keys) : 0u;
      if (a.key_done && k0 + lane < (uint64_t)a.n_keys && a.key_done[k0 + lane]) r = 0u;
      cnt[256u * w + 64u * g + lane] = r;
      if (k0 + lane < (uint64_t)a.n_keys) key_rmv[k0 + lane] = r;
    }
    __syncthreads();
  }
  uint64_t sum[3] = {0, 0, 0};
  const uint64_t base = tile0 + (uint64_t)threadIdx.x * SCAN_ITEMS;
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    const uint64_t k = base + j;
    if (k < (uint64_t)a.n_keys) {
      uint64_t c[3];
      caps_of(a, k, a.fresh ? 0u : cnt[threadIdx.x * SCAN_ITEMS + j], c);
      for (int x = 0; x < 3; ++x) sum[x] += c[x];
    }
  }
  uint64_t tot[3];
  block_scan3(sum, tot);
  if (threadIdx.x == 0)
    for (int x = 0; x < 3; ++x) partials[(uint64_t)blockIdx.x * 3 + x] = tot[x];
}

// Single block: exclusive scan of the per-tile partials; totals at [nb*3..].
__global__ __launch_bounds__(SCAN_BLOCK) void trmv_scan_tops(uint64_t* partials, uint64_t nb) {
  __shared__ uint64_t carry[3];
  if (threadIdx.x < 3) carry[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t b0 = 0; b0 < nb; b0 += SCAN_BLOCK) {
    const uint64_t b = b0 + threadIdx.x;
    uint64_t v[3] = {0, 0, 0};
    if (b < nb)
      for (int x = 0; x < 3; ++x) v[x] = partials[b * 3 + x];
    uint64_t tot[3];
    block_scan3(v, tot);
    if (b < nb)
      for (int x = 0; x < 3; ++x) partials[b * 3 + x] = v[x] + carry[x];
    __syncthreads();
    if (threadIdx.x < 3) carry[threadIdx.x] += tot[threadIdx.x];
    __syncthreads();
  }
  if (threadIdx.x < 3) partials[nb * 3 + threadIdx.x] = carry[threadIdx.x];
}

__global__ __launch_bounds__(SCAN_BLOCK) void trmv_scan_apply(TrmvApplyArgs a, const uint64_t* partials,
                                                                 const uint32_t* key_rmv) {
  uint64_t c[SCAN_ITEMS][3];
  uint64_t sum[3] = {0, 0, 0};
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    const uint64_t k = base + j;
    if (k < (uint64_t)a.n_keys) caps_of(a, k, a.fresh ? 0u : key_rmv[k], c[j]);
    else c[j][0] = c[j][1] = c[j][2] = 0;
    for (int x = 0; x < 3; ++x) sum[x] += c[j][x];
  }
  uint64_t tot[3];
  block_scan3(sum, tot);
  uint64_t run[3];
  for (int x = 0; x < 3; ++x) run[x] = partials[(uint64_t)blockIdx.x * 3 + x] + sum[x];
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    const uint64_t k = base + j;
    if (k < (uint64_t)a.n_keys) {
      KeyMeta m;
      m.p_off = (uint32_t)run[0];
      m.m_off = (uint32_t)run[1];
      m.r_off = (uint32_t)run[2];
      m.np = m.nm = m.nr = m.nobs = 0;
      m.minq = NONE32;
      a.new_s.meta[k] = m;
      if (a.new_s.cap) {
        KeyCap cp;
        cp.p_cap = (uint32_t)c[j][0];
        cp.m_cap = c[j][1] > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)c[j][1];
        cp.r_cap = (uint32_t)c[j][2];
        cp.m_top = 0;
        cp.flags = 0;
        a.new_s.cap[k] = cp;
      }
    }
    for (int x = 0; x < 3; ++x) run[x] += c[j][x];
  }
}

// ----------------------------------------------------------- downstream/2
// One wave per request, read-only probe of the resident state (:102-124).
__global__ __launch_bounds__(64) void trmv_downstream_kernel(TrmvDownArgs a) {
  const int lane = lane_id();
  const uint64_t r = blockIdx.x;
  const uint64_t key = a.key[r];
  const int D = a.n_dc;
  KeyMeta m;
  if (a.fresh) {
    m.p_off = m.m_off = m.r_off = 0;
    m.np = m.nm = m.nr = m.nobs = 0;
    m.minq = NONE32;
  } else {
    m = a.s.meta[key];
  }
  const int64_t id = a.id[r];
  // find player
  uint32_t q = NONE32;
  for (uint32_t b = 0; b < m.np && q == NONE32; b += 64) {
    const uint32_t p = b + lane;
    const uint64_t hit = ballot(p < m.np && a.s.pl_id[m.p_off + p] == id);
    if (hit) q = b + __builtin_ctzll(hit);
  }
  const uint32_t info = q == NONE32 ? NONE32 : a.s.pl_info[m.p_off + q];
  const uint32_t slab = q == NONE32 ? 0u : a.s.pl_slab[m.p_off + q];
  const uint32_t o = info & 0xFFFFu;
  uint8_t kind;
  if (a.op[r] == 0) {
    const int64_t sc = a.score[r], ts = a.ts[r];
    bool changes;
    if (o != NONE16) {
      const uint64_t g = (uint64_t)m.m_off + (slab & 0xFFFFu) + o;
      changes = trmv_cmp(sc, id, ts, a.s.m_score[g], id, a.s.m_ts[g]);
    } else if (m.minq == NONE32) {
      changes = true;  // cmp(_, nil) = true
    } else {
      const uint32_t mi = a.s.pl_info[m.p_off + m.minq] & 0xFFFFu;
      const uint32_t ms = a.s.pl_slab[m.p_off + m.minq];
      const uint64_t g = (uint64_t)m.m_off + (ms & 0xFFFFu) + mi;
      changes = trmv_cmp(sc, id, ts, a.s.m_score[g], a.s.pl_id[m.p_off + m.minq], a.s.m_ts[g]);
    }
    kind = changes ? CCRDT_TRMV_ADD : CCRDT_TRMV_ADD_R;
  } else {
    const bool in_masked = (slab >> 16) != 0;  // Id in Masked
    kind = !in_masked ? (uint8_t)CCRDT_NOOP : (o != NONE16 ? CCRDT_TRMV_RMV : CCRDT_TRMV_RMV_R);
    if (a.out_vc && lane < D)
      a.out_vc[r * D + lane] = a.fresh ? 0 : a.s.vc[key * D + lane];
  }
  if (lane == 0) a.out_kind[r] = kind;
}

// --------------------------------------------------- over-capacity keys
// The keys the last tier handed on (over the per-key capacity) keep their
// previous state: one wave per listed key copies it from the old side into
// the segments the scan laid out on the new side (which hold old counts +
// ops, so the old state fits), closing the holes between Masked slabs, and
// clears the key's extras.  A fresh engine's previous state is empty.
__global__ __launch_bounds__(64) void trmv_keep_kernel(TrmvApplyArgs a) {
  const uint32_t n = a.n_list_dev ? *a.n_list_dev : a.n_list;
  const int lane = lane_id();
  const int D = a.n_dc;
  for (uint32_t w = blockIdx.x; w < n; w += gridDim.x) {
    const uint32_t key = a.key_list[w];
    KeyMeta nm = trmv_new_meta(a, key);
    if (lane == 0) a.ex_cnt[key] = 0u;
    if (a.fresh) {
      if (lane < D) a.new_s.vc[(uint64_t)key * D + lane] = 0;
      if (lane == 0) {
        nm.np = nm.nm = nm.nr = nm.nobs = 0;
        nm.minq = NONE32;
        a.new_s.meta[key] = nm;
        a.new_s.cap[key].flags = 0;
      }
      continue;
    }
    const KeyMeta om = a.old_s.meta[key];
    const TrmvSide& o = a.old_s;
    const TrmvSide& d = a.new_s;
    uint32_t base = 0;
    for (uint32_t p0 = 0; p0 < om.np; p0 += 64) {
      const uint32_t p = p0 + lane;
      const bool v = p < om.np;
      const uint32_t slab = v ? o.pl_slab[om.p_off + p] : 0u;
      const uint32_t cnt = slab >> 16;
      uint32_t tot;
      const uint32_t off = base + wave_excl_scan_u32(cnt, tot);
      if (v) {
        d.pl_id[nm.p_off + p] = o.pl_id[om.p_off + p];
        d.pl_info[nm.p_off + p] = o.pl_info[om.p_off + p];
        d.pl_gb[nm.p_off + p] = o.pl_gb[om.p_off + p];
        d.pl_slab[nm.p_off + p] = off | (cnt << 16);
      }
      for (int j = 0; j < 64; ++j) {  // each player's elements, lanes over elements
        const uint32_t c = shfl32(cnt, j);
        const uint32_t so = shfl32(slab & 0xFFFFu, j);
        const uint32_t to = shfl32(off, j);
        for (uint32_t e = lane; e < c; e += 64) {
          const uint64_t src = (uint64_t)om.m_off + so + e, dst = (uint64_t)nm.m_off + to + e;
          d.m_score[dst] = o.m_score[src];
          d.m_ts[dst] = o.m_ts[src];
          d.m_dc[dst] = o.m_dc[src];
        }
      }
      base += tot;
    }
    for (uint32_t i = lane; i < om.nr * (uint32_t)D; i += 64)
      d.r_vc[(uint64_t)nm.r_off * D + i] = o.r_vc[(uint64_t)om.r_off * D + i];
    if (lane < D) d.vc[(uint64_t)key * D + lane] = o.vc[(uint64_t)key * D + lane];
    if (lane == 0) {
      nm.np = om.np;
      nm.nm = om.nm;
      nm.nr = om.nr;
      nm.nobs = om.nobs;
      nm.minq = om.minq;
      d.meta[key] = nm;
      d.cap[key].flags = 0;
    }
  }
}

// ------------------------------------------------------ batch validation
// Before an in-place pass nothing may be written when any op of the batch is
// invalid (the state must stay untouched, as the reference's update/2 crashes
// on such an op with function_clause): the checks tier R makes per chunk --
// kind <= 3; an add's DcId < n_dc and Ts >= 1; a rmv's clock row in range and
// its entries >= 0 -- over every op, the error bits OR-ed into *err.
// (kind, DcId and Ts of one op; a rmv's clock row only in range here)
__device__ __forceinline__ uint32_t trmv_check_op(const TrmvApplyArgs& a, uint32_t kind, uint32_t dc, int64_t ts) {
  uint32_t e = 0;
  if (kind > 3) {
    e |= TRMV_ERR_KIND;
  } else if (kind < 2) {
    e |= dc >= (uint32_t)a.n_dc ? TRMV_ERR_DC : 0u;
    e |= ts < 1 ? TRMV_ERR_TS : 0u;
  } else if (ts < 0 || ts >= a.n_rmv_rows) {
    e |= TRMV_ERR_ROW;
  }
  return e;
}

__device__ __forceinline__ void trmv_err_or(uint32_t e, uint32_t* err) {  // one atomic per wave
  uint32_t w = e;
  for (int s = 1; s < 64; s <<= 1) w |= (uint32_t)__shfl_xor((int)w, s);
  if (w && lane_id() == 0) atomicOr(err, w);
}

// Pass 1: every op's kind, DcId, Ts and clock-row range.  16 consecutive ops
// per thread: their kinds and DcIds in one 16-byte load each, their Ts in
// eight (when the columns are 16-byte aligned; else and for the tail, one op
// at a time).
__global__ __launch_bounds__(256) void trmv_validate_kernel(TrmvApplyArgs a, uint64_t n_ops, uint32_t* err) {
  uint32_t e = 0;
  const bool vec = ((reinterpret_cast<uintptr_t>(a.kind) | reinterpret_cast<uintptr_t>(a.dc) |
                     reinterpret_cast<uintptr_t>(a.ts)) & 15u) == 0;
  const uint64_t n16 = vec ? n_ops / 16 : 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n16; g += stride) {
    const uint4 kv = reinterpret_cast<const uint4*>(a.kind)[g];
    const uint4 dv = reinterpret_cast<const uint4*>(a.dc)[g];
    int64_t ts[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const longlong2 t2 = reinterpret_cast<const longlong2*>(a.ts + 16 * g)[i];
      ts[2 * i] = t2.x;
      ts[2 * i + 1] = t2.y;
    }
    const uint32_t kw[4] = {kv.x, kv.y, kv.z, kv.w}, dw[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
    for (int i = 0; i < 16; ++i)
      e |= trmv_check_op(a, (kw[i / 4] >> (8 * (i % 4))) & 0xFFu, (dw[i / 4] >> (8 * (i % 4))) & 0xFFu, ts[i]);
  }
  for (uint64_t i = 16 * n16 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_ops; i += stride)
    e |= trmv_check_op(a, a.kind[i], a.dc[i], a.ts[i]);
  trmv_err_or(e, err);
}

// Pass 2: is any entry of the clock table negative?  (Coalesced over the
// whole table: in a valid batch none is, and nothing more is read.)
__global__ __launch_bounds__(256) void trmv_validate_rows_any(TrmvApplyArgs a, unsigned long long* any) {
  const uint64_t n = (uint64_t)a.n_rmv_rows * a.n_dc;
  bool neg = false;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    neg |= a.rmv_vc[i] < 0;
  if (ballot(neg) && lane_id() == 0) atomicOr(any, 1ull);
}

// Pass 3, only when pass 2 found a negative entry: the rows the rmv ops
// name, as tier R checks them (a row no rmv names is not an error).
__global__ __launch_bounds__(256) void trmv_validate_rows_exact(TrmvApplyArgs a, uint64_t n_ops,
                                                                const unsigned long long* any, uint32_t* err) {
  if (!*any) return;
  uint32_t e = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_ops; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t kind = a.kind[i];
    const int64_t ts = a.ts[i];
    if ((kind == 2 || kind == 3) && ts >= 0 && ts < a.n_rmv_rows)
      for (int d = 0; d < a.n_dc; ++d) e |= a.rmv_vc[(uint64_t)ts * a.n_dc + d] < 0 ? TRMV_ERR_VC : 0u;
  }
  trmv_err_or(e, err);
}

// key_done for the pass that finishes an in-place batch: every key 1, then
// the keys the in-place pass handed on 0.
// done[k] = 0 for the listed keys (n_list: the device count, else n_host);
// with ex_cnt their extra counts are zeroed too
__global__ __launch_bounds__(256) void trmv_mark_done_kernel(uint8_t* done, uint64_t n_keys, const uint32_t* list,
                                                             const uint32_t* n_list, uint32_t n_host, uint32_t* ex_cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t n = n_list ? *n_list : n_host;
  if (i < n && list[i] < n_keys) {
    done[list[i]] = 0u;
    if (ex_cnt) ex_cnt[list[i]] = 0u;
  }
}

// The likely hand-ons of a fresh batch (keys with more than `thresh` ops) ->
// list (any order; *count = how many): tier 0 takes them first.
__global__ __launch_bounds__(256) void trmv_first_list_kernel(const uint64_t* key_ptr, uint64_t n_keys,
                                                              uint32_t thresh, uint32_t* list, uint32_t* count) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool f = k < n_keys && key_ptr[k + 1] - key_ptr[k] > thresh;
  const uint64_t m = ballot(f);
  if (!m) return;
  uint32_t base = 0;
  if (lane_id() == (int)__builtin_ctzll(m)) base = atomicAdd(count, (uint32_t)__builtin_popcountll(m));
  base = shfl32(base, (int)__builtin_ctzll(m));
  if (f) list[base + mbcnt(m)] = (uint32_t)k;
}

int trmv_launch_first_list(const uint64_t* key_ptr, uint64_t n_keys, uint32_t thresh, uint32_t* list,
                           uint32_t* count, hipStream_t st) {
  if (n_keys == 0) return CCRDT_OK;
  hipLaunchKernelGGL(trmv_first_list_kernel, dim3((unsigned)((n_keys + 255) / 256)), dim3(256), 0, st, key_ptr,
                     n_keys, thresh, list, count);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

// ------------------------------------------------------------- launchers
// (scratch: one u64 flag, zeroed here)
void trmv_kernels_preload() {
  preload_kernels(trmv_scan_partials, trmv_scan_tops, trmv_scan_apply, trmv_validate_kernel, trmv_validate_rows_any,
                  trmv_validate_rows_exact, trmv_keep_kernel, trmv_mark_done_kernel, trmv_first_list_kernel);
}

int trmv_launch_validate(const TrmvApplyArgs& a, uint64_t n_ops, uint32_t* err, unsigned long long* scratch,
                         hipStream_t st) {
  if (n_ops == 0) return CCRDT_OK;
  const uint64_t blocks = std::min<uint64_t>((n_ops / 16 + 255) / 256 + 1, 8192);
  hipLaunchKernelGGL(trmv_validate_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a, n_ops, err);
  const uint64_t nv = (uint64_t)a.n_rmv_rows * a.n_dc;
  if (nv && a.rmv_vc) {
    CCRDT_HIP(hipMemsetAsync(scratch, 0, sizeof(unsigned long long), st));
    hipLaunchKernelGGL(trmv_validate_rows_any, dim3((unsigned)std::min<uint64_t>((nv + 255) / 256, 4096)), dim3(256), 0,
                       st, a, scratch);
    hipLaunchKernelGGL(trmv_validate_rows_exact, dim3((unsigned)std::min<uint64_t>((n_ops + 255) / 256, 4096)),
                       dim3(256), 0, st, a, n_ops, scratch, err);
  }
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

int trmv_launch_mark_done(uint8_t* done, uint64_t n_keys, const uint32_t* list, uint32_t n_list, const uint32_t* n_dev,
                          uint32_t* ex_cnt, hipStream_t st) {
  CCRDT_HIP(hipMemsetAsync(done, 1, n_keys, st));
  if (n_list == 0) return CCRDT_OK;
  hipLaunchKernelGGL(trmv_mark_done_kernel, dim3((n_list + 255) / 256), dim3(256), 0, st, done, n_keys, list, n_dev,
                     n_list, ex_cnt);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

int trmv_launch_keep(const TrmvApplyArgs& a, uint32_t grid, hipStream_t st) {
  if (grid == 0) return CCRDT_OK;
  hipLaunchKernelGGL(trmv_keep_kernel, dim3(grid), dim3(64), 0, st, a);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

int trmv_launch_scan(const TrmvApplyArgs& a, uint64_t* partials, uint32_t* key_rmv, hipStream_t st) {
  const uint64_t nb = ((uint64_t)a.n_keys + SCAN_TILE - 1) / SCAN_TILE;
  if (nb == 0) return CCRDT_OK;
  hipLaunchKernelGGL(trmv_scan_partials, dim3((unsigned)nb), dim3(SCAN_BLOCK), 0, st, a, partials, key_rmv);
  hipLaunchKernelGGL(trmv_scan_tops, dim3(1), dim3(SCAN_BLOCK), 0, st, partials, nb);
  hipLaunchKernelGGL(trmv_scan_apply, dim3((unsigned)nb), dim3(SCAN_BLOCK), 0, st, a, partials, key_rmv);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

int trmv_launch_downstream(const TrmvDownArgs& a, hipStream_t st) {
  if (a.n == 0) return CCRDT_OK;
  hipLaunchKernelGGL(trmv_downstream_kernel, dim3((unsigned)a.n), dim3(64), 0, st, a);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

}  // namespace ccrdt
