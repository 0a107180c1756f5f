// trmv_wave.hip — tier 0 of the topk_rmv apply: one wavefront per key, one
// wave per 64-thread workgroup (W_WAVES), each wave taking W_KPW consecutive
// keys; one key's working set (WaveLds<true>) is ~8 KB of LDS.
//
// Exactness argument: the per-player decomposition (P <= K players =>
// recompute_observed/5 never evicts, and the promotion candidates of rmv/3
// are the removed player's own survivors; src/antidote_ccrdt_topk_rmv.erl
// :231-334).  Keys outside this tier's caps go to the next tier (tier R).
//
// The mapping onto gfx950:
//  * occupancy: elements are addressed by index, Masked slabs are u8 index
//    lists, removal clocks are one shared table of 24 rows, so a key's LDS
//    stays small and five waves fit per SIMD (__launch_bounds__);
//  * latency: every global load a key needs is issued before its first use:
//    a key's ops, and then its removal clocks (8 lanes per clock row,
//    coalesced), are loaded while the wave still works on the previous key;
//  * no workgroup barriers: each wave orders its own LDS accesses
//    (wave_lds_sync);
//  * grouping: 64-bit LDS compare-and-swap on the Id itself (one probe loop,
//    no claim protocol); players are numbered in hash-slot order (new ones
//    after the old ones), so the device layout is deterministic;
//  * scans are DPP (wave_excl_scan_dpp), not LDS-crossbar shuffles;
//  * each wave runs W_KPW consecutive keys and issues the next key's loads
//    (bounds, metadata, ops, clocks) before the current key's write-out, so
//    the first HBM round trip of a key overlaps the previous key's stores;
//  * op elements are stored at their position in player order, so every op
//    lane reads its player's ops with one LDS round trip each;
//  * players are decided op-parallel wherever the history allows it (step 5):
//    every op lane scans its player's positions once.
//    A player's rmvs cut its ops into segments.  When (a) no add is dominated
//    by an earlier rmv, (b) every add that has a later rmv is removed by the
//    first of them, and (c) the adds after the last rmv have strictly
//    increasing Ts, every rmv empties Masked[Id] and drops the Id from
//    Observed without a promotion, so Masked[Id] is the last segment, Obs[Id]
//    its first add with the largest (Score, Ts) (recompute_observed/5's
//    strict cmp/2 keeps the first arrival on a tie), Removals[Id] the
//    elementwise max of its rmv clocks, and the player emits no extra effect.
//    A player without rmvs is the case of one segment.  Only the players that
//    fail a test (and, outside FRESH, every player with old state or a rmv)
//    are replayed op by op, one lane per player.
//
// Element index space of a key: [0, nops) = this batch's ops, grouped by player
// (stream order inside a player), [nops, nops + old |Masked|) = the key's old
// Masked elements.
#include "common.hpp"
#include "trmv_kernels.hpp"

// Diagnostic build only (-DTRMV_PROF): per-phase s_memtime stamps summed
// over keys; read with ccrdt_debug_trmv_prof().  No stamp in the real build.
#ifdef TRMV_PROF
__device__ unsigned long long g_trmv_prof[16];
#define PROF_STAMP(v)                                                        \
  do {                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                       \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                       \
  } while (0)
#define PROF_MARK(i)                                                         \
  do {                                                                       \
    unsigned long long _t;                                                   \
    PROF_STAMP(_t);                                                          \
    if (lane_id() == 0 && (key & 63u) == 3) atomicAdd(&g_trmv_prof[i], _t - prof_t);             \
    prof_t = _t;                                                             \
  } while (0)
#else
#define PROF_STAMP(v) (void)0
#define PROF_MARK(i) (void)0
#endif

namespace ccrdt {

namespace {
constexpr int W_HCAP = 256;  // hash slots (Ids)
constexpr int W_ECAP = 128;  // elements: ops + old Masked elements
constexpr int W_PCAP = 128;  // players
constexpr int W_RCAP = 24;   // clock rows: old Removals rows + this batch's rmv clocks
constexpr int W_WAVES = 1;  // waves (keys in flight) per workgroup (4 before A/B r04 run 31)
#define ST_OUT(p, v) (*(p) = (v))
#define LD_IN(p) (*(p))
constexpr int W_KPW = 8;  // consecutive keys per wave chunk (1..64; A/B r03: 2/3/4/16 slower; r06 at 5 waves: 4/16 slower)
constexpr int W_MD = (W_KPW + 7) / 8;  // metadata registers of a chunk header
static_assert(W_KPW >= 1 && W_KPW <= 64, "1..64 keys per wave chunk");
constexpr unsigned long long W_EMPTY = 0x8000000000000000ull;  // an Id of INT64_MIN takes tier 1
constexpr uint32_t NONE8 = 0xFFu;
// Sink entries: a lane with nothing to read reads the extra entry of the
// array, so the hot phases issue their LDS reads back to back without
// per-lane branches.  (Stores and atomics stay exec-masked: many lanes on one
// sink address would serialize.)
constexpr uint32_t HSINK = W_HCAP, ESINK = W_ECAP, PSINK = W_PCAP;

// FRESH keys have no old state: the arrays only the steady-state path uses
// take no space in their instantiation (zero-length), which keeps the FRESH
// workgroup inside a fifth of the CU's LDS.
template <bool FRESH>
struct alignas(16) WaveLds {
  static constexpr int NS_ = FRESH ? 0 : 1;
  unsigned long long htab[W_HCAP + 2];   // Ids (W_EMPTY = free); [HSINK]
  int64_t esc[W_ECAP + 2];               // element score (rmv op: its clock row in `rows`)
  int64_t ets[W_ECAP + 2];               // element ts
  int64_t rows[W_RCAP][TRMV_DPAD];       // [0, old nr) old Removals rows, then rmv clocks
  unsigned long long vc[TRMV_DPAD + 2];  // replica Vc; [TRMV_DPAD] sink
  uint32_t pcnt2[W_PCAP / 2 + 4];        // ops per player (two u16 counters per word)
  uint32_t rsrc[W_RCAP];                 // rmv_vc row of each rmv op of the key being prefetched
  uint16_t ekd[W_ECAP + 8];              // kind | dc << 2 | player << 8
  uint8_t hp[W_HCAP];                    // hash slot -> player
  uint8_t sorted[W_ECAP + 8];            // op index (stream position) of every op element
  uint8_t slab[W_ECAP];                  // working Masked slabs (element indices)
  uint8_t fin[NS_ * (W_ECAP + 8)];       // final pool: element of every output position
  // Per-player bytes, packed four to a word so a pass over players reads
  // them with one LDS load each (byte stores still write single fields):
  //  pa: pstart (first position of the player's ops) | plr (FRESH: 1 +
  //      position of its last rmv, 0 = none) | pflag (1 = replayed op by op)
  //      | pcntf (replayed player: final |Masked[Id]|)
  //  pb: pobs (Obs[Id], an element; NONE8 = none) | prow (its clock row =
  //      Removals[Id], or NONE8) | pgb (gb_sets:largest(Masked[Id]): element;
  //      slab-relative + slab start for replayed players) | pslot (hash slot)
  uint32_t pa[W_PCAP + 8];
  uint32_t pb[W_PCAP + 8];
  uint8_t pmoff[NS_ * (W_PCAP + 8)];     // replayed player: its working slab in `slab`
  uint8_t peb[NS_ * (W_PCAP + 8)];       // old player: first element of its old slab
  uint8_t cpl[W_PCAP + 8];               // replayed players, packed
  uint8_t rl[W_RCAP + 8];                // clock row of each output Removals row
  uint32_t nex;                          // extra effects emitted by the key
  __device__ __forceinline__ uint8_t& fa(uint32_t p, int b) { return reinterpret_cast<uint8_t*>(pa)[4 * p + b]; }
  __device__ __forceinline__ uint8_t& fb(uint32_t p, int b) { return reinterpret_cast<uint8_t*>(pb)[4 * p + b]; }
};
#define PSTART(p) L.fa((p), 0)
#define PLR(p) L.fa((p), 1)
#define PFLAG(p) L.fa((p), 2)
#define PCNTF(p) L.fa((p), 3)
#define POBS(p) L.fb((p), 0)
#define PROW(p) L.fb((p), 1)
#define PGB(p) L.fb((p), 2)
#define PSLOT(p) L.fb((p), 3)

#define KA trmv_kargs()

__device__ __forceinline__ uint32_t whash(int64_t id) {
  const uint64_t x = (uint64_t)id * 0x9E3779B97F4A7C15ull;
  return (uint32_t)(x >> 56);  // 8 bits = W_HCAP slots
}

template <class W>
__device__ __forceinline__ uint32_t pcnt_of(const W& L, uint32_t p) {
  return (L.pcnt2[p >> 1] >> (16 * (p & 1))) & 0xFFFFu;
}

// One extra effect (the {ok, S, [Effect]} of topk_rmv.erl:236-237 / :294-295).
template <class W>
__device__ __forceinline__ void wave_emit(const TrmvApplyArgs& a, W& L, uint64_t op0,
                                          uint64_t op, uint8_t kind, int64_t id, int64_t sc,
                                          uint32_t dc, int64_t ts, uint32_t row) {
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
  if (kind == CCRDT_TRMV_RMV)
    for (int d = 0; d < KA->n_dc; ++d) KA->ex_vc[(op0 + pos) * KA->n_dc + d] = L.rows[row][d];
}

// What a key needs before anything else: bounds, new-side metadata, its ops,
// and the removal clocks of its rmv ops.
struct KeyIn {
  uint64_t op0;
  uint32_t nops;
  KeyMeta nmeta;
  int64_t id[2], sc[2], ts[2];
  uint32_t kind[2], dc[2];  // kept apart: combining them would force a wait at the load
  int64_t rv[W_RCAP / 8];   // clock of the (lane/8 + 8s)-th rmv op, entry lane%8
};

// Bounds and new-side metadata of a wave's W_KPW keys, loaded once per chunk
// into lanes (key j: lane j holds its key and op range; register i, lane
// 8(j%8) + d: dword d of the KeyMeta of key 8i + j/8... see wave_load_chunk),
// so a key's op loads never wait on a scalar load of its own bounds.
struct ChunkHdr {
  uint32_t key;         // lane j < n: key j
  uint64_t lo, hi;      // lane j < n: key_ptr[key j], key_ptr[key j + 1]
  uint32_t meta[W_MD];  // meta[i], lane 8m + d: dword d of new_s.meta[key 8i + m]
  uint64_t skip;        // bit j: key j was taken from first_list already (overlapped hand-on)
};

// Key at work-list position i: the list's entry, or (overlapped hand-on)
// first_list's entries first and then every key in order.
__device__ __forceinline__ uint32_t wave_list_key(uint32_t i, uint32_t n_first) {
  if (KA->first_list) return i < n_first ? KA->first_list[i] : i - n_first;
  return KA->key_list ? KA->key_list[i] : i;
}

__device__ __forceinline__ void wave_load_chunk(const TrmvApplyArgs& a, uint32_t c0, uint32_t n,
                                                uint32_t n_first, ChunkHdr& h) {
  const int lane = lane_id();
  const uint32_t j = (uint32_t)lane < n ? (uint32_t)lane : 0u;
  h.key = wave_list_key(c0 + j, n_first);
  h.lo = KA->key_ptr[h.key];
  h.hi = KA->key_ptr[h.key + 1];
  h.skip = KA->first_list ? ballot((uint32_t)lane < n && c0 + j >= n_first && h.hi - h.lo > KA->first_thresh) : 0ull;
#pragma unroll
  for (int i = 0; i < W_MD; ++i) {
    const uint32_t m = 8 * i + (lane >> 3);
    const uint32_t jm = m < n ? m : 0u;
    const uint32_t km = shfl32(h.key, (int)jm);
    if (KA->fresh) {  // trmv_new_meta: the fresh layout's offsets, counts 0, Min nil
      const uint32_t d = lane & 7;
      h.meta[i] = d < 3 ? (uint32_t)trmv_fresh_off(KA->slack != 0, (int)d, km, KA->key_ptr[km])
                        : (d == 7 ? NONE32 : 0u);
    } else {
      h.meta[i] = reinterpret_cast<const uint32_t*>(a.new_s.meta + km)[lane & 7];
    }
  }
}

__device__ __forceinline__ void wave_load_key(const TrmvApplyArgs& a, const ChunkHdr& h, uint32_t j,
                                              KeyIn& in) {
  const int lane = lane_id();
  in.op0 = (uint64_t)rl64((int64_t)h.lo, (int)j);
  in.nops = (uint32_t)((uint64_t)rl64((int64_t)h.hi, (int)j) - in.op0);
  uint32_t* m = reinterpret_cast<uint32_t*>(&in.nmeta);
#pragma unroll
  for (int d = 0; d < 8; ++d) {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < W_MD; ++i)
      if ((j >> 3) == (uint32_t)i) v = rl32(h.meta[i], (int)(8 * (j & 7) + d));
    m[d] = v;
  }
  // wave-uniform bases + 32-bit lane offsets (saddr addressing, no 64-bit
  // per-lane address arithmetic)
  const int64_t* idp = KA->id + in.op0;
  const int64_t* scp = KA->score + in.op0;
  const int64_t* tsp = KA->ts + in.op0;
  const uint8_t* kp = KA->kind + in.op0;
  const uint8_t* dp = KA->dc + in.op0;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const uint32_t l = s * 64 + lane;
    const bool v = l < in.nops;
    in.id[s] = v ? LD_IN(idp + l) : 0;
    in.sc[s] = v ? LD_IN(scp + l) : 0;
    in.ts[s] = v ? LD_IN(tsp + l) : 0;
    in.kind[s] = v ? (uint32_t)LD_IN(kp + l) : 0u;
    in.dc[s] = v ? (uint32_t)LD_IN(dp + l) : 0u;
  }
}

// Issue the loads of a key's removal clocks (rmv ops in stream order, 8 lanes
// per clock row, coalesced) once its ops are in registers; they are consumed
// after the key's hash build.  A row outside [0, n_rmv_rows) reads row 0: the
// key's validation rejects the batch before any value is used.
template <class W>
__device__ __forceinline__ void wave_load_rows(const TrmvApplyArgs& a, W& L, KeyIn& in) {
  const int lane = lane_id();
#pragma unroll
  for (int s = 0; s < W_RCAP / 8; ++s) in.rv[s] = 0;
  bool r[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
    r[s] = (uint32_t)(s * 64 + lane) < in.nops && (in.kind[s] == 2 || in.kind[s] == 3);
  const uint64_t b0 = ballot(r[0]), b1 = ballot(r[1]);
  const uint32_t n0 = (uint32_t)__builtin_popcountll(b0);
  const uint32_t n = n0 + (uint32_t)__builtin_popcountll(b1);
  if (n == 0 || KA->n_rmv_rows <= 0) return;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const uint32_t k = s ? n0 + mbcnt(b1) : mbcnt(b0);
    if (r[s] && k < (uint32_t)W_RCAP)
      L.rsrc[k] = (in.ts[s] >= 0 && in.ts[s] < KA->n_rmv_rows) ? (uint32_t)in.ts[s] : 0u;
  }
  wave_lds_sync();
  const uint32_t d = (lane & 7) < KA->n_dc ? (lane & 7) : 0u;
#pragma unroll
  for (int s = 0; s < W_RCAP / 8; ++s) {
    const uint32_t k = s * 8 + (lane >> 3);
    const uint32_t row = k < n ? L.rsrc[k] : 0u;
    in.rv[s] = KA->rmv_vc[(uint64_t)row * KA->n_dc + d];
  }
  wave_lds_sync();  // rsrc is rewritten for the next key
}

// Outcome of one key.  Only W_DONE has already issued the loads of the wave's
// next key; the rare other paths leave that to the caller.
enum : int { W_DONE = 0, W_NEXT_TIER = 1, W_REJECT = 2 };

template <bool FRESH>
__device__ __forceinline__ int trmv_wave_key(const TrmvApplyArgs& a, uint32_t key, const KeyIn& in,
                                              WaveLds<FRESH>& L, bool has_next, const ChunkHdr& hdr,
                                              uint32_t nj, KeyIn& nxt) {
  // opaque per key: lane-derived addresses are formed where they are used
  // instead of being hoisted out of the key loop into VGPR pairs that live
  // (and spill) across every key
  int lane = lane_id();
  asm volatile("" : "+v"(lane));
  const int D = KA->n_dc;
#ifdef TRMV_PROF
  unsigned long long prof_t;
  PROF_STAMP(prof_t);
#endif
  const uint64_t op0 = in.op0;
  const uint32_t nops = in.nops;
  // the new-side offsets are wave-uniform: SGPRs, so every output address is
  // a scalar base plus a 32-bit lane offset (no 64-bit VGPR bases to spill)
  KeyMeta nmeta = in.nmeta;
  nmeta.p_off = __builtin_amdgcn_readfirstlane(nmeta.p_off);
  nmeta.m_off = __builtin_amdgcn_readfirstlane(nmeta.m_off);
  nmeta.r_off = __builtin_amdgcn_readfirstlane(nmeta.r_off);
  KeyMeta om;
  if (FRESH) {
    om.p_off = om.m_off = om.r_off = 0;
    om.np = om.nm = om.nr = om.nobs = 0;
    om.minq = NONE32;
  } else {
    om = a.old_s.meta[key];
  }
  const uint32_t pmax = KA->k < (uint32_t)W_PCAP ? KA->k : (uint32_t)W_PCAP;
  if (nops > (uint32_t)W_ECAP || om.np > pmax || om.nm + nops > (uint32_t)W_ECAP ||
      om.nr > (uint32_t)W_RCAP)
    return W_NEXT_TIER;

  // ---- 1. the ops are in `in`; issue the old-state loads
  int64_t xsc[2] = {in.sc[0], in.sc[1]};
  const int64_t xts[2] = {in.ts[0], in.ts[1]};
  const uint32_t xkind[2] = {in.kind[0], in.kind[1]};
  const uint32_t xdc[2] = {in.dc[0], in.dc[1]};
  const bool xv[2] = {(uint32_t)lane < nops, (uint32_t)(64 + lane) < nops};
  int64_t pid[2] = {0, 0};
  uint32_t pinfo[2] = {NONE32, NONE32}, pslab[2] = {0u, 0u};
  if (!FRESH) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t p = s * 64 + lane;
      if (p < om.np) {
        pid[s] = (a.old_s.pl_id + om.p_off)[p];
        pinfo[s] = (a.old_s.pl_info + om.p_off)[p];
        pslab[s] = (a.old_s.pl_slab + om.p_off)[p];
      }
    }
  }
  // LDS init (overlaps the loads)
#pragma unroll
  for (int i = 0; i < W_HCAP / 64; ++i) L.htab[i * 64 + lane] = W_EMPTY;
  if (lane == 0) {
    L.htab[HSINK] = W_EMPTY;
    L.nex = 0u;
  }
  reinterpret_cast<uint32_t*>(L.hp)[lane] = 0xFFFFFFFFu;  // 256 B
  L.pcnt2[lane] = 0u;
  // pflag, plr = 0; pobs, prow = NONE8 (the sink entries included)
  L.pa[lane] = 0u;
  L.pa[64 + lane] = 0u;
  L.pb[lane] = 0xFFFFFFFFu;
  L.pb[64 + lane] = 0xFFFFFFFFu;
  if (lane < 8) {
    L.pa[128 + lane] = 0u;
    L.pb[128 + lane] = 0xFFFFFFFFu;
  }
  if (lane < TRMV_DPAD)
    L.vc[lane] = (!FRESH && lane < D) ? (unsigned long long)a.old_s.vc[(uint64_t)key * D + lane] : 0ull;
  if (!FRESH) {  // old Removals rows -> clock rows [0, om.nr)
    for (uint32_t r0 = 0; r0 < om.nr; r0 += 8) {
      const uint32_t r = r0 + (lane >> 3), d = lane & 7;
      if (r < om.nr)
        L.rows[r][d] = (int)d < D ? (a.old_s.r_vc + (uint64_t)om.r_off * D)[r * D + d] : 0;
    }
  }

  PROF_MARK(0);
  // ---- 2. validate ops (predicated), rank the rmv ops
  uint32_t err = 0;
  bool xr[2], xa[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    xa[s] = xv[s] && xkind[s] < 2;
    xr[s] = xv[s] && (xkind[s] == 2 || xkind[s] == 3);
    err |= (xv[s] && xkind[s] > 3) ? TRMV_ERR_KIND : 0u;
    err |= (xa[s] && (int)xdc[s] >= D) ? TRMV_ERR_DC : 0u;
    err |= (xa[s] && xts[s] < 1) ? TRMV_ERR_TS : 0u;
    err |= (xr[s] && (xts[s] < 0 || xts[s] >= KA->n_rmv_rows)) ? TRMV_ERR_ROW : 0u;
  }
  if (ballot(err != 0)) {
    if (err) atomicOr(&KA->status[1], err);
    return W_REJECT;  // the host rejects the batch
  }
  const uint64_t rb0 = ballot(xr[0]), rb1 = ballot(xr[1]);
  const uint32_t nr0 = (uint32_t)__builtin_popcountll(rb0);
  const uint32_t nrmv = nr0 + (uint32_t)__builtin_popcountll(rb1);
  if (om.nr + nrmv > (uint32_t)W_RCAP) return W_NEXT_TIER;
  {
    // a rmv's "score": its clock row (the order wave_load_rows staged them in)
    const uint32_t r0 = mbcnt(rb0), r1 = nr0 + mbcnt(rb1);
    xsc[0] = xr[0] ? (int64_t)(om.nr + r0) : xsc[0];
    xsc[1] = xr[1] ? (int64_t)(om.nr + r1) : xsc[1];
  }
  wave_lds_sync();
  // ---- 3 (set-up). hash slots; an Id equal to the empty marker takes tier 1
  constexpr int NS = FRESH ? 2 : 4;
  uint32_t hs[4];
  bool pend[4];
  const int64_t hid[4] = {in.id[0], in.id[1], pid[0], pid[1]};
  pend[0] = xv[0];
  pend[1] = xv[1];
  pend[2] = !FRESH && (uint32_t)lane < om.np;
  pend[3] = !FRESH && (uint32_t)(64 + lane) < om.np;
  bool bad = false;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    hs[j] = whash(hid[j]);
    bad |= pend[j] && (unsigned long long)hid[j] == W_EMPTY;
  }
  if (ballot(bad)) return W_NEXT_TIER;

  PROF_MARK(1);
  // ---- 3. hash build: ops, then old players (64-bit CAS on the Id)
  for (;;) {
    bool any = false;
#pragma unroll
    for (int j = 0; j < NS; ++j) any |= pend[j];
    if (!ballot(any)) break;
    unsigned long long prev[4];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      prev[j] = W_EMPTY;
      if (pend[j]) prev[j] = atomicCAS(&L.htab[hs[j]], W_EMPTY, (unsigned long long)hid[j]);
    }
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const bool done = prev[j] == W_EMPTY || prev[j] == (unsigned long long)hid[j];
      hs[j] = (pend[j] && !done) ? ((hs[j] + 1) & (W_HCAP - 1)) : hs[j];
      pend[j] = pend[j] && !done;
    }
  }
  PROF_MARK(8);
  // write the rmv clocks (their loads were issued with the key's ops)
  {
#pragma unroll
    for (int s = 0; s < W_RCAP / 8; ++s) {
      const uint32_t r = s * 8 + (lane >> 3), d = lane & 7;
      const int64_t v = (int)d < D ? in.rv[s] : 0;
      err |= (r < nrmv && v < 0) ? TRMV_ERR_VC : 0u;
      if (r < nrmv) L.rows[om.nr + r][d] = v;
    }
    if (ballot(err != 0)) {
      if (err) atomicOr(&KA->status[1], err);
      return W_REJECT;
    }
  }
  PROF_MARK(9);
  // old players keep their index
  if (!FRESH) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t p = s * 64 + lane;
      if (p < om.np) {
        L.hp[hs[2 + s]] = (uint8_t)p;
        PSLOT(p) = (uint8_t)hs[2 + s];
        // every player with Masked elements must be in Observed (P <= K states)
        bad |= ((pslab[s] >> 16) != 0) != ((pinfo[s] & 0xFFFFu) != NONE16);
      }
    }
    if (ballot(bad)) return W_NEXT_TIER;
  }
  wave_lds_sync();
  // new players numbered after the old ones, in hash-slot order (branch-free:
  // each lane owns four consecutive slots)
  uint32_t np;
  {
    const unsigned long long* h4 = &L.htab[lane * 4];
    const unsigned long long t0 = h4[0], t1 = h4[1], t2 = h4[2], t3 = h4[3];
    const uint32_t hp4 = reinterpret_cast<const uint32_t*>(L.hp)[lane];
    const uint32_t n0 = (t0 != W_EMPTY && (hp4 & 0xFFu) == NONE8) ? 1u : 0u;
    const uint32_t n1 = (t1 != W_EMPTY && ((hp4 >> 8) & 0xFFu) == NONE8) ? 1u : 0u;
    const uint32_t n2 = (t2 != W_EMPTY && ((hp4 >> 16) & 0xFFu) == NONE8) ? 1u : 0u;
    const uint32_t n3 = (t3 != W_EMPTY && (hp4 >> 24) == NONE8) ? 1u : 0u;
    const uint32_t c = n0 + n1 + n2 + n3;
    const uint64_t b0 = ballot(c & 1), b1 = ballot(c & 2), b2 = ballot(c & 4);
    const uint32_t base = om.np + mbcnt(b0) + 2 * mbcnt(b1) + 4 * mbcnt(b2);
    np = om.np + (uint32_t)__builtin_popcountll(b0) + 2 * (uint32_t)__builtin_popcountll(b1) +
         4 * (uint32_t)__builtin_popcountll(b2);
    if (np > pmax) return W_NEXT_TIER;  // Observed could fill: next tier
    const uint32_t i0 = base, i1 = i0 + n0, i2 = i1 + n1, i3 = i2 + n2;
    const uint32_t nhp = (n0 ? i0 : (hp4 & 0xFFu)) | ((n1 ? i1 : ((hp4 >> 8) & 0xFFu)) << 8) |
                         ((n2 ? i2 : ((hp4 >> 16) & 0xFFu)) << 16) |
                         ((n3 ? i3 : (hp4 >> 24)) << 24);
    reinterpret_cast<uint32_t*>(L.hp)[lane] = nhp;
    if (n0) PSLOT(i0) = (uint8_t)(lane * 4 + 0);
    if (n1) PSLOT(i1) = (uint8_t)(lane * 4 + 1);
    if (n2) PSLOT(i2) = (uint8_t)(lane * 4 + 2);
    if (n3) PSLOT(i3) = (uint8_t)(lane * 4 + 3);
  }
  wave_lds_sync();
  // the next key's op loads go out here, after the last early return: they
  // land during steps 4-5; the explicit wait before this key's stores
  // retires them, so the next key never waits on (and its vmcnt never
  // counts) this key's stores.  (Non-FRESH keys keep more registers live
  // through step 4: their next key's loads go out at step 5.)
  if (FRESH && has_next) wave_load_key(a, hdr, nj, nxt);

  PROF_MARK(2);
  // ---- 4. player of every op, Vc, op elements in player order
  uint32_t xrank[2], xp[2];
  {
    // every lane reads its slots' player bytes and adds to a counter word
    // (a lane without an op adds 0 to the word of its own lane index), so
    // both slots' LDS round trips go out together instead of one after the
    // other behind exec-masked branches
    uint32_t hpv[2], cr[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) hpv[s] = L.hp[hs[s]];  // hs[s] < W_HCAP for every lane
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t p = xv[s] ? hpv[s] : PSINK;
      xp[s] = p;
      if (xa[s]) atomicMax(&L.vc[xdc[s]], (unsigned long long)xts[s]);  // vc_update (:233)
      if (!FRESH && xr[s]) PFLAG(p) = 1;                              // a rmv: replayed
      cr[s] = atomicAdd(&L.pcnt2[(xv[s] ? p : (uint32_t)lane) >> 1], xv[s] ? 1u << (16 * (p & 1)) : 0u);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) xrank[s] = xv[s] ? (cr[s] >> (16 * (xp[s] & 1))) & 0xFFFFu : 0u;
  }
  wave_lds_sync();
  // per player (lane, lane + 64): first position of its ops
  {
    uint32_t tot0, tot1;
    const uint32_t c0 = (uint32_t)lane < np ? pcnt_of(L, lane) : 0u;
    const uint32_t c1 = (uint32_t)(64 + lane) < np ? pcnt_of(L, 64 + lane) : 0u;
    const uint32_t st0 = wave_excl_scan_dpp(c0, tot0);
    const uint32_t st1 = wave_excl_scan_dpp(c1, tot1);
    PSTART(lane) = (uint8_t)st0;
    PSTART(64 + lane) = (uint8_t)(tot0 + st1);
  }
  wave_lds_sync();
  uint32_t xq[2], xst[2], xc[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    xst[s] = PSTART(xp[s]);
    xc[s] = pcnt_of(L, xp[s]);
    xq[s] = xv[s] ? xst[s] + xrank[s] : ESINK;
    if (xv[s]) {
      L.esc[xq[s]] = xsc[s];
      L.ets[xq[s]] = xts[s];
      L.ekd[xq[s]] = (uint16_t)(xkind[s] | (xdc[s] << 2) | (xp[s] << 8));
      L.sorted[xq[s]] = (uint8_t)(s * 64 + lane);
    }
  }
  wave_lds_sync();
  // The ranks came from LDS atomics, whose order inside one instruction is
  // not specified: check that every player's ops are in stream order, and
  // restore it (insertion sort per player) where they are not.
  {
    bool bad_order = false;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bool has_prev = xv[s] && xq[s] > xst[s];
      bad_order |= has_prev && L.sorted[has_prev ? xq[s] - 1 : ESINK] > (uint32_t)(s * 64 + lane);
    }
    if (ballot(bad_order)) {
#pragma unroll 1
      for (int s = 0; s < 2; ++s) {
        const uint32_t p = s * 64 + lane;
        const uint32_t c = p < np ? pcnt_of(L, p) : 0u, st = p < np ? PSTART(p) : 0u;
        for (uint32_t x = 1; x < c; ++x) {
          const uint32_t v = L.sorted[st + x];
          const int64_t vs = L.esc[st + x], vt = L.ets[st + x];
          const uint16_t vk = L.ekd[st + x];
          uint32_t y = x;
          while (y > 0 && L.sorted[st + y - 1] > v) {
            L.sorted[st + y] = L.sorted[st + y - 1];
            L.esc[st + y] = L.esc[st + y - 1];
            L.ets[st + y] = L.ets[st + y - 1];
            L.ekd[st + y] = L.ekd[st + y - 1];
            --y;
          }
          L.sorted[st + y] = (uint8_t)v;
          L.esc[st + y] = vs;
          L.ets[st + y] = vt;
          L.ekd[st + y] = vk;
        }
      }
      wave_lds_sync();
      // positions moved: every op lane finds its own again
#pragma unroll
      for (int s = 0; s < 2; ++s)
        if (xv[s])
          for (uint32_t x = 0; x < xc[s]; ++x)
            if (L.sorted[xst[s] + x] == (uint32_t)(s * 64 + lane)) xq[s] = xst[s] + x;
    }
  }
  // old Masked elements -> elements [nops, nops + om.nm), player by player
  if (!FRESH) {
    uint32_t ebase = nops;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t p = s * 64 + lane;
      const uint32_t oc = p < om.np ? (pslab[s] >> 16) : 0u;
      uint32_t tot;
      const uint32_t eb = ebase + wave_excl_scan_dpp(oc, tot);
      ebase += tot;
      if (p < om.np) {
        L.peb[p] = (uint8_t)eb;
        PFLAG(p) = 1;  // old state: replayed
      }
      for (uint32_t j = 0; j < oc; ++j) {
        const uint32_t go = (pslab[s] & 0xFFFFu) + j;
        const uint32_t e = eb + j;
        L.esc[e] = (a.old_s.m_score + om.m_off)[go];
        L.ets[e] = (a.old_s.m_ts + om.m_off)[go];
        L.ekd[e] = (uint16_t)(((uint32_t)(a.old_s.m_dc + om.m_off)[go] << 2) | (p << 8));
      }
    }
  }
  wave_lds_sync();

  PROF_MARK(3);
  if (!FRESH && has_next) wave_load_key(a, hdr, nj, nxt);
  if (!FRESH) {
    // ---- 5a. players without rmv or old state, op-parallel: each add
    // decides whether it is its player's Obs[Id] and whether its Ts rises
    // over every earlier add's
    bool simple[2], beaten[2] = {false, false}, gbeaten[2] = {false, false}, risk[2] = {false, false};
    uint32_t me[2], cl[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      simple[s] = xa[s] && !PFLAG(xp[s]);
      me[s] = xq[s] - xst[s];
      cl[s] = simple[s] ? xc[s] : 0u;
    }
    const uint32_t maxc = wave_max_u32_dpp(cl[0] > cl[1] ? cl[0] : cl[1]);
    for (uint32_t x = 0; x < maxc; ++x) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bool valid = x < cl[s] && x != me[s];
        const uint32_t pos = x < cl[s] ? xst[s] + x : (uint32_t)ESINK;
        const int64_t sx = L.esc[pos], tx = L.ets[pos];
        const uint32_t dx = (L.ekd[pos] >> 2) & 7u;
        const int64_t sm = xsc[s], tm = xts[s];
        const bool before = x < me[s];
        risk[s] |= valid && before && tx >= tm;
        beaten[s] |= valid && (sx > sm || (sx == sm && (before ? tx >= tm : tx > tm)));
        gbeaten[s] |= valid && (sx > sm || (sx == sm && (dx > xdc[s] || (dx == xdc[s] && tx > tm))));
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (risk[s]) PFLAG(xp[s]) = 1;
      if (simple[s] && !beaten[s]) POBS(xp[s]) = (uint8_t)xq[s];
      if (simple[s] && !gbeaten[s]) PGB(xp[s]) = (uint8_t)xq[s];
    }
    wave_lds_sync();
  } else {
    // ---- 5. players decided op-parallel (header: tests (a)-(c)).  A player
    // with one op is decided by it.  The ops of the other players are packed
    // into as few 64-lane passes as they fill (one, in practice) and each
    // scans its player's positions once; a rmv at a position ends the
    // segments before it, so the Obs/Ts bookkeeping restarts there and ends
    // with the last segment's.  (slab and cpl, used by the replay only after
    // this step, hold the packed positions and the pending Removals merges.)
    uint8_t* const cq = L.slab;
    uint8_t* const mrg = L.cpl;
    uint32_t mn0, mn;
    {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bool single = xv[s] && xc[s] == 1;
        if (single && xa[s]) POBS(xp[s]) = (uint8_t)xq[s];
        if (single && xr[s]) {
          PROW(xp[s]) = (uint8_t)xsc[s];
          PLR(xp[s]) = (uint8_t)(xq[s] + 1);
        }
      }
      const bool mu0 = xv[0] && xc[0] > 1, mu1 = xv[1] && xc[1] > 1;
      const uint64_t mb0 = ballot(mu0), mb1 = ballot(mu1);
      mn0 = (uint32_t)__builtin_popcountll(mb0);
      mn = mn0 + (uint32_t)__builtin_popcountll(mb1);
      if (mu0) cq[mbcnt(mb0)] = (uint8_t)xq[0];
      if (mu1) cq[mn0 + mbcnt(mb1)] = (uint8_t)xq[1];
    }
    wave_lds_sync();
    bool any_merge = false;
#pragma unroll 1
    for (uint32_t b = 0; b < mn; b += 64) {
      const uint32_t k = b + lane;
      const bool act = k < mn;
      const uint32_t q = act ? (uint32_t)cq[k] : ESINK;
      const int64_t sm = L.esc[q], tm = L.ets[q];
      const uint32_t kd = L.ekd[q];
      const uint32_t p = act ? (kd >> 8) : PSINK;
      const bool ya = act && (kd & 2u) == 0, yr = act && (kd & 2u) != 0;
      const uint32_t adc = ya ? ((kd >> 2) & 7u) : 0u;
      const uint32_t st = PSTART(p), c = act ? pcnt_of(L, p) : 0u;
      const uint32_t me = q - st;
      const uint32_t maxc = wave_max_u32_dpp(c);
      // software-pipelined: position x+1 is read while position x's clock
      // entry (its address depends on x's element) is in flight.  The flags
      // are wave lane masks combined on the scalar unit: each condition is
      // one compare (a VALU instruction writing a mask), everything else
      // SALU (as per-lane bools under short-circuits the compiler made
      // divergent branches and kept the flags in VGPRs, four VALU
      // instructions per flag per position)
      const uint64_t Mya = ballot(ya);
      uint64_t Mfb = 0, Mbeaten = 0, Mrisk = 0, Mseen = 0, Mfirst = ~0ull, Mgbeaten = 0, Mgtie = 0;
      const uint32_t p0 = c ? st : (uint32_t)ESINK;
      int64_t sxn = L.esc[p0], txn = L.ets[p0];
      uint32_t kxn = L.ekd[p0];
      for (uint32_t x = 0; x < maxc; ++x) {
        const int64_t sx = sxn, tx = txn;
        const uint64_t Mvalid = ballot(x < c) & ballot(x != me);
        const uint64_t Misr = Mvalid & ballot((kxn & 2u) != 0u);
        const uint64_t Mbefore = ballot(x < me);
        // an add against a rmv of its player: dominated by an earlier one
        // (:234), or kept by the first later one (:255-266) -> replay
        const uint64_t Mneed = Mya & Misr & (Mbefore | ~Mseen);
        const bool need = (Mneed >> lane) & 1u;
        const int64_t rt = L.rows[need ? (uint32_t)sx : 0u][adc];
        const uint32_t pn = x + 1 < c ? st + x + 1 : (uint32_t)ESINK;
        sxn = L.esc[pn];
        txn = L.ets[pn];
        kxn = L.ekd[pn];
        const uint64_t Msgt = ballot(sx > sm), Mseq = ballot(sx == sm);
        const uint64_t Mtge = ballot(tx >= tm), Mtgt = ballot(tx > tm);
        const uint64_t Mrge = ballot(rt >= tm);
        Mfb |= Mneed & ~(Mbefore ^ Mrge);  // before ? rt >= tm : rt < tm
        Mseen |= Misr & ~Mbefore;
        Mfirst &= ~(Misr & Mbefore);
        const uint64_t Mboth = Mya & Mvalid & ~Misr;
        Mrisk = (Mrisk & ~Misr) | (Mboth & Mbefore & Mtge);
        Mbeaten = (Mbeaten & ~Misr) | (Mboth & (Msgt | (Mseq & ((Mbefore & Mtge) | (~Mbefore & Mtgt)))));
        Mgbeaten = (Mgbeaten & ~Misr) | (Mboth & Msgt);
        Mgtie = (Mgtie & ~Misr) | (Mboth & Mseq);
      }
      const bool fb = (Mfb >> lane) & 1u, beaten = (Mbeaten >> lane) & 1u, risk = (Mrisk >> lane) & 1u;
      const bool seen = (Mseen >> lane) & 1u, first = (Mfirst >> lane) & 1u;
      const bool gbeaten = (Mgbeaten >> lane) & 1u, gtie = (Mgtie >> lane) & 1u;
      // equal Scores in the last segment: gb_sets order goes on to DcId and
      // Ts, which the replay settles
      if (act && (fb || risk || (ya && !seen && gtie))) PFLAG(p) = 1;
      if (ya && !seen && !beaten) POBS(p) = (uint8_t)q;
      if (ya && !seen && !gbeaten) PGB(p) = (uint8_t)q;  // largest of the last segment (by Score)
      if (yr && first) PROW(p) = (uint8_t)sm;  // a rmv's "score" is its clock row
      if (yr && !seen) PLR(p) = (uint8_t)(q + 1);
      if (act) mrg[k] = (uint8_t)(yr && !first);
      any_merge |= ballot(yr && !first) != 0;
    }
    wave_lds_sync();
    // Removals[Id]: the player's later rmv clocks merge into its first rmv's
    // row (merge_vc, :369-386); replayed players merge their own
    if (any_merge) {
#pragma unroll 1
      for (uint32_t b = 0; b < mn; b += 64) {
        const uint32_t k = b + lane;
        const uint32_t q = k < mn && mrg[k] ? (uint32_t)cq[k] : ESINK;
        const uint32_t p = q != ESINK ? (uint32_t)(L.ekd[q] >> 8) : PSINK;
        if (q != ESINK && !PFLAG(p)) {
          unsigned long long* dst = reinterpret_cast<unsigned long long*>(L.rows[PROW(p)]);
          const int64_t* src = L.rows[(uint32_t)L.esc[q]];
          for (int d = 0; d < D; ++d) atomicMax(dst + d, (unsigned long long)src[d]);
        }
      }
    }
    wave_lds_sync();
  }

  PROF_MARK(6);
  // ---- 5b. replayed players, one lane per player, op by op
  uint32_t ncx;
  {
    const bool c0 = (uint32_t)lane < np && PFLAG(lane);
    const bool c1 = (uint32_t)(64 + lane) < np && PFLAG(64 + lane);
    const uint64_t m0 = ballot(c0), m1 = ballot(c1);
    const uint32_t n0 = (uint32_t)__builtin_popcountll(m0);
    ncx = n0 + (uint32_t)__builtin_popcountll(m1);
    if (c0) L.cpl[mbcnt(m0)] = (uint8_t)lane;
    if (c1) L.cpl[n0 + mbcnt(m1)] = (uint8_t)(64 + lane);
  }
  wave_lds_sync();
  // The next key's ops are retired before this key's first store, so the
  // next key never waits on (and its vmcnt never counts) these stores.
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  // the next key's clock loads go out before this key's first store: a
  // load's data waits for every older vector-memory op, stores included
  if (FRESH && has_next) wave_load_rows(a, L, nxt);
  PROF_MARK(7);
  uint32_t best_q = NONE32;                      // Min candidate of this lane
  int64_t best_sc = INT64_MAX, best_id = INT64_MAX;
  auto min_cand = [&](bool has, int64_t sc, int64_t id, uint32_t p) {
    const bool better = has && (best_q == NONE32 || sc < best_sc || (sc == best_sc && id < best_id));
    best_q = better ? p : best_q;
    best_sc = better ? sc : best_sc;
    best_id = better ? id : best_id;
  };
  if (FRESH) {
    // FRESH: every player's Masked slab lives inside its own op positions
    // [pstart, pstart + ops) of the key's pool segment (|Masked[Id]| <= its
    // adds), so no pool order has to be built: the op positions of a decided
    // player's last segment (its slab) are written as their ops' elements
    // (coalesced).  Every op position is written, rmv ops and filtered adds
    // included (writing only the surviving positions measured slower: the
    // per-element lookup costs more than the bytes it saves, A/B r04);
    // replayed players' positions are rewritten below
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t q = s * 64 + lane;
      const uint32_t qq = q < nops ? q : (uint32_t)ESINK;
      const int64_t sc = L.esc[qq], ts = L.ets[qq];
      const uint32_t kd = L.ekd[qq];
      if (q < nops) {
        ST_OUT((KA->new_s.m_score + nmeta.m_off) + (q), sc);
        ST_OUT((KA->new_s.m_ts + nmeta.m_off) + (q), ts);
        ST_OUT((KA->new_s.m_dc + nmeta.m_off) + (q), (uint8_t)((kd >> 2) & 7u));
      }
    }
  }
  uint32_t mbase = 0;
#pragma unroll 1
  for (uint32_t b = 0; b < ncx; b += 64) {
    const uint32_t k = b + lane;
    const bool act = k < ncx;
    const uint32_t p = act ? L.cpl[k] : 0u;
    uint32_t ocnt = 0, pinfo_p = NONE32, eb = 0;
    if (!FRESH && act && p < om.np) {
      pinfo_p = (a.old_s.pl_info + om.p_off)[p];
      ocnt = (a.old_s.pl_slab + om.p_off)[p] >> 16;
      eb = L.peb[p];
    }
    const uint32_t c = act ? pcnt_of(L, p) : 0u;
    const uint32_t st = act ? PSTART(p) : 0u;
    uint32_t tot;
    const uint32_t moff = mbase + wave_excl_scan_dpp(c + ocnt, tot);  // slab capacity
    mbase += tot;
    // initial player state
    uint32_t cnt = ocnt;
    int64_t maxts = 0;
    for (uint32_t j = 0; j < cnt; ++j) {
      L.slab[moff + j] = (uint8_t)(eb + j);
      const int64_t t = L.ets[eb + j];
      maxts = t > maxts ? t : maxts;
    }
    uint32_t o = NONE8, prow = NONE8;
    int64_t osc = 0, ots = 0;
    if (!FRESH && act && p < om.np) {
      const uint32_t oi = pinfo_p & 0xFFFFu, ri = pinfo_p >> 16;
      if (oi != NONE16) {
        o = eb + oi;
        osc = L.esc[o];
        ots = L.ets[o];
      }
      if (ri != NONE16) prow = ri;
    }
    const int64_t id = act ? (int64_t)L.htab[PSLOT(p)] : 0;
    for (uint32_t x = 0; x < c; ++x) {
      const uint32_t e = st + x;  // op element (player order)
      const uint32_t kd = L.ekd[e];
      const int64_t sc = L.esc[e];
      const int64_t t = L.ets[e];
      const uint32_t kind = kd & 3u, dc = (kd >> 2) & 7u;
      if (kind < 2) {  // add/4 (:231-249)
        if (prow != NONE8 && L.rows[prow][dc] >= t) {  // dominated (:234-237)
          wave_emit(a, L, op0, op0 + L.sorted[e], CCRDT_TRMV_RMV, id, 0, 0, 0, prow);
          continue;
        }
        // gb_sets:add_element: set semantics (a ts above every ts ever in the
        // slab cannot duplicate an element)
        uint32_t ee = e;
        if (t <= maxts) {
          for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t e2 = L.slab[moff + j];
            if (L.ets[e2] == t && ((L.ekd[e2] >> 2) & 7u) == dc && L.esc[e2] == sc) {
              ee = e2;
              break;
            }
          }
        }
        maxts = t > maxts ? t : maxts;
        if (ee == e) L.slab[moff + cnt++] = (uint8_t)e;
        // recompute_observed (:301-324; never full in this tier)
        if (o == NONE8 || sc > osc || (sc == osc && t > ots)) {
          o = ee;
          osc = sc;
          ots = t;
        }
      } else {  // rmv/3 (:252-298)
        const uint32_t vs = (uint32_t)sc;  // this rmv's clock row
        if (prow == NONE8) {
          prow = vs;  // Removals[Id] := VcRmv
        } else {
          for (int d = 0; d < D; ++d) {  // merge_vc (:369-386)
            const int64_t u = L.rows[vs][d], w0 = L.rows[prow][d];
            L.rows[prow][d] = u > w0 ? u : w0;
          }
        }
        // keep Masked[Id] elements with Ts > VcRmv[DcId] (:255-266)
        uint32_t w = 0, be = NONE8, bdc = 0;
        bool alive = false;
        int64_t bsc = 0, bts = 0;
        for (uint32_t j = 0; j < cnt; ++j) {
          const uint32_t e2 = L.slab[moff + j];
          const int64_t t2 = L.ets[e2];
          const uint32_t d2 = (L.ekd[e2] >> 2) & 7u;
          if (t2 > L.rows[vs][d2]) {
            L.slab[moff + w++] = (uint8_t)e2;
            alive |= e2 == o;
            const int64_t s2 = L.esc[e2];
            if (be == NONE8 || s2 > bsc || (s2 == bsc && (d2 > bdc || (d2 == bdc && t2 > bts)))) {
              be = e2;
              bsc = s2;
              bdc = d2;
              bts = t2;
            }
          }
        }
        cnt = w;
        if (o != NONE8 && !alive) {  // impacts Observed (:267-272)
          if (cnt == 0) {
            o = NONE8;
          } else {  // promote gb_sets:largest of the survivors (:291-295)
            o = be;
            osc = bsc;
            ots = bts;
            wave_emit(a, L, op0, op0 + L.sorted[e], CCRDT_TRMV_ADD, id, bsc, bdc, bts, prow);
          }
        }
      }
    }
    if (FRESH) {
      // the player's slab at [pstart, pstart + cnt); its record is written
      // with every other player's below
      uint32_t opos = NONE16, gj = 0;
      for (uint32_t j = 0; j < cnt; ++j) {
        const uint32_t e2 = L.slab[moff + j];
        const int64_t s2 = L.esc[e2], t2 = L.ets[e2];
        const uint32_t d2 = (L.ekd[e2] >> 2) & 7u;
        ST_OUT((KA->new_s.m_score + nmeta.m_off) + (st + j), s2);
        ST_OUT((KA->new_s.m_ts + nmeta.m_off) + (st + j), t2);
        ST_OUT((KA->new_s.m_dc + nmeta.m_off) + (st + j), (uint8_t)d2);
        opos = e2 == o ? j : opos;
        // gb_sets:largest so far (re-read from LDS: no registers held across)
        const uint32_t eb = L.slab[moff + gj];
        const int64_t bs = L.esc[eb], bt = L.ets[eb];
        const uint32_t bd = (L.ekd[eb] >> 2) & 7u;
        if (s2 > bs || (s2 == bs && (d2 > bd || (d2 == bd && t2 > bt)))) gj = j;
      }
      if (act) {
        POBS(p) = (uint8_t)(o == NONE8 ? NONE8 : st + opos);
        PGB(p) = (uint8_t)(st + gj);
        PCNTF(p) = (uint8_t)cnt;
        PROW(p) = (uint8_t)prow;
      }
      min_cand(act && o != NONE8, osc, id, p);
    } else if (act) {
      POBS(p) = (uint8_t)o;
      PCNTF(p) = (uint8_t)cnt;
      L.pmoff[p] = (uint8_t)moff;
      PROW(p) = (uint8_t)prow;
    }
  }
  wave_lds_sync();
  // non-FRESH keys: the next key's clock loads after the replay (registers)
  if (!FRESH && has_next) wave_load_rows(a, L, nxt);

  PROF_MARK(4);
  // ---- 6. player records, final pool order, Removals rows
  uint32_t fbase = 0, rbase = 0, nobs = 0;
  uint32_t po[2] = {NONE8, NONE8};
  if (FRESH) {
    // slab of a decided player: its last segment (every op if it has no
    // rmv); of a replayed player: [pstart, pstart + final count)
    uint32_t csum = 0;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t p = s * 64 + lane;
      const bool act = p < np;
      const uint32_t pp = act ? p : (uint32_t)PSINK;
      const uint32_t wa = L.pa[pp], wb = L.pb[pp];  // (packed fields: WaveLds)
      const uint32_t st = wa & 0xFFu, c = pcnt_of(L, pp), lrp = (wa >> 8) & 0xFFu;
      const bool replayed = ((wa >> 16) & 0xFFu) != 0;
      const uint32_t off = (replayed || lrp == 0) ? st : lrp;
      const uint32_t cnt = act ? (replayed ? (wa >> 24) : st + c - off) : 0u;
      const uint32_t o = act ? (wb & 0xFFu) : NONE8;
      const uint32_t prow = act ? ((wb >> 8) & 0xFFu) : NONE8;
      const uint64_t rm = ballot(prow != NONE8);
      const uint32_t rix = rbase + mbcnt(rm);
      rbase += (uint32_t)__builtin_popcountll(rm);
      if (prow != NONE8) L.rl[rix] = (uint8_t)prow;
      const int64_t id = (int64_t)L.htab[wb >> 24];
      // gb_sets:largest of the slab: step 5 (a decided player: its last
      // segment, strictly rising Ts, so no two elements tie) or 5b (replayed)
      const uint32_t gb = (replayed || cnt > 1) ? ((wb >> 16) & 0xFFu) - off : 0u;
      if (act) {
        ST_OUT((KA->new_s.pl_id + nmeta.p_off) + (p), id);
        ST_OUT((KA->new_s.pl_slab + nmeta.p_off) + (p), off | (cnt << 16));
        if (cnt > 1) ST_OUT((KA->new_s.pl_gb + nmeta.p_off) + (p), (uint16_t)gb);  // readers take 0 for cnt <= 1
        ST_OUT(KA->new_s.pl_info + nmeta.p_off + p, (o == NONE8 ? NONE16 : o - off) |
                                             ((prow != NONE8 ? rix : NONE16) << 16));
      }
      csum += cnt;
      nobs += (uint32_t)__builtin_popcountll(ballot(o != NONE8));
      min_cand(!replayed && o != NONE8, L.esc[o != NONE8 ? o : (uint32_t)ESINK], id, p);
    }
    (void)wave_excl_scan_dpp(csum, fbase);  // |Masked| of the key
    wave_lds_sync();
  } else {
  {
    uint32_t cnt[2], st[2], moff[2], goff[2], prow[2], opos[2], gbj[2], gbd[2];
    int64_t gbs[2], gbt[2];
    bool act[2], cx[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t p = s * 64 + lane;
      act[s] = p < np;
      const uint32_t pp = act[s] ? p : PSINK;
      cx[s] = act[s] && PFLAG(pp);
      const uint32_t c = pcnt_of(L, pp);
      st[s] = PSTART(pp);
      po[s] = act[s] ? POBS(pp) : NONE8;
      cnt[s] = act[s] ? (cx[s] ? (uint32_t)PCNTF(pp) : c) : 0u;  // simple: every add is in Masked[Id]
      prow[s] = cx[s] ? PROW(pp) : NONE8;
      moff[s] = cx[s] ? L.pmoff[pp] : 0u;
      uint32_t ftot;
      goff[s] = fbase + wave_excl_scan_dpp(cnt[s], ftot);
      fbase += ftot;
      opos[s] = (act[s] && !cx[s]) ? po[s] - st[s] : NONE16;
      gbj[s] = (act[s] && !cx[s]) ? (uint32_t)PGB(pp) - st[s] : 0u;
      gbd[s] = 0u;
      gbs[s] = gbt[s] = 0;
    }
    // final pool order: replayed players' slabs, simple players' op runs
    const uint32_t maxcnt = wave_max_u32_dpp(cnt[0] > cnt[1] ? cnt[0] : cnt[1]);
    for (uint32_t j = 0; j < maxcnt; ++j) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bool in = j < cnt[s];
        const uint32_t e = cx[s] ? (uint32_t)L.slab[in ? moff[s] + j : 0u] : st[s] + j;
        if (in) L.fin[goff[s] + j] = (uint8_t)e;
        opos[s] = (cx[s] && in && e == po[s]) ? j : opos[s];
        if (cx[s] && in) {  // gb_sets:largest of a replayed player's slab
          const int64_t s2 = L.esc[e], t2 = L.ets[e];
          const uint32_t d2 = (L.ekd[e] >> 2) & 7u;
          if (j == 0 || s2 > gbs[s] || (s2 == gbs[s] && (d2 > gbd[s] || (d2 == gbd[s] && t2 > gbt[s])))) {
            gbj[s] = j;
            gbs[s] = s2;
            gbd[s] = d2;
            gbt[s] = t2;
          }
        }
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t p = s * 64 + lane;
      const uint64_t rm = ballot(prow[s] != NONE8);
      const uint32_t rix = rbase + mbcnt(rm);
      rbase += (uint32_t)__builtin_popcountll(rm);
      if (prow[s] != NONE8) L.rl[rix] = (uint8_t)prow[s];
      const int64_t id = (int64_t)L.htab[PSLOT(act[s] ? p : PSINK)];
      if (act[s]) {
        (KA->new_s.pl_id + nmeta.p_off)[p] = id;
        (KA->new_s.pl_info + nmeta.p_off)[p] = (po[s] == NONE8 ? NONE16 : opos[s]) |
                                             ((prow[s] != NONE8 ? rix : NONE16) << 16);
        (KA->new_s.pl_slab + nmeta.p_off)[p] = goff[s] | (cnt[s] << 16);
        (KA->new_s.pl_gb + nmeta.p_off)[p] = (uint16_t)(cnt[s] ? gbj[s] : 0u);
      }
      nobs += (uint32_t)__builtin_popcountll(ballot(act[s] && po[s] != NONE8));
    }
  }
  wave_lds_sync();

  // ---- 7. Masked pool (the FRESH pool is already written)
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const uint32_t q = s * 64 + lane;
    const uint32_t e0 = L.fin[q < fbase ? q : (uint32_t)ESINK];
    const uint32_t e = e0 < (uint32_t)W_ECAP ? e0 : (uint32_t)ESINK;
    const int64_t sc = L.esc[e], ts = L.ets[e];
    const uint8_t dc = (uint8_t)((L.ekd[e] >> 2) & 7u);
    if (q < fbase) {
      (KA->new_s.m_score + nmeta.m_off)[q] = sc;
      (KA->new_s.m_ts + nmeta.m_off)[q] = ts;
      (KA->new_s.m_dc + nmeta.m_off)[q] = dc;
    }
  }
  }  // !FRESH
  PROF_MARK(10);
  // Removals rows (8 lanes per row), Vc, Min, metadata
  for (uint32_t r0 = 0; r0 < rbase; r0 += 8) {
    const uint32_t r = r0 + (lane >> 3), d = lane & 7;
    const int64_t v = L.rows[L.rl[r < rbase ? r : 0u]][d];
    if (r < rbase && (int)d < D) (KA->new_s.r_vc + (uint64_t)nmeta.r_off * D)[r * D + d] = v;
  }
  if (lane < D) KA->new_s.vc[(uint64_t)key * D + lane] = (int64_t)L.vc[lane];
  PROF_MARK(11);
  // Min = min_observed(Observed) by (Score, Id) — Ids are distinct (:398-406)
  {
    if (!FRESH) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t p = s * 64 + lane;
        const uint32_t o = po[s];
        const int64_t sc = L.esc[o != NONE8 ? o : (uint32_t)ESINK];
        const int64_t id = (int64_t)L.htab[PSLOT(o != NONE8 ? p : (uint32_t)PSINK)];
        min_cand(o != NONE8, sc, id, p);
      }
    }
    const bool has = best_q != NONE32;
    const bool narrow = best_sc == (int64_t)(int32_t)best_sc && best_id == (int64_t)(int32_t)best_id;
    if (!ballot(has)) {
      best_q = NONE32;
    } else if (!ballot(has && !narrow)) {
      // 32-bit Scores and Ids (sign bits flipped: unsigned order): the least
      // Score, then the least Id among the lanes holding it -- two 32-bit DPP
      // reductions (fused min per step) instead of one over 64-bit keys
      const uint32_t us = has ? (uint32_t)(int32_t)best_sc ^ 0x80000000u : 0xFFFFFFFFu;
      const uint32_t ms = wave_min_u32_dpp(us);
      const bool at = has && us == ms;
      const uint32_t ui = at ? (uint32_t)(int32_t)best_id ^ 0x80000000u : 0xFFFFFFFFu;
      const uint32_t mi = wave_min_u32_dpp(ui);
      best_q = rl32(best_q, (int)__builtin_ctzll(ballot(at && ui == mi)));
    } else {
      const int64_t ms = wave_min_i64_dpp(has ? best_sc : INT64_MAX);
      const int64_t mi = wave_min_i64_dpp(has && best_sc == ms ? best_id : INT64_MAX);
      const uint64_t hit = ballot(has && best_sc == ms && best_id == mi);
      best_q = rl32(best_q, (int)__builtin_ctzll(hit));
    }
  }
  if (lane == 0) {
    KeyMeta out = nmeta;
    out.np = np;
    out.nm = fbase;
    out.nr = rbase;
    out.nobs = nobs;
    out.minq = best_q;
    KA->new_s.meta[key] = out;
    KA->ex_cnt[key] = L.nex;
    if (FRESH && KA->slack) {  // the fresh layout's room: later batches grow the key in place
      KeyCap c;
      c.p_cap = trmv_fresh_cap(true, 0, nops);
      c.m_cap = trmv_fresh_cap(true, 1, nops);
      c.r_cap = trmv_fresh_cap(true, 2, nops);
      c.m_top = (uint16_t)nops;  // (every slab lies in the key's op positions)
      c.flags = TRMV_CAP_VALID;
      KA->new_s.cap[key] = c;
    }
  }
  PROF_MARK(5);
  return W_DONE;
}
}  // namespace

// OCC waves per SIMD.  5 (96 VGPRs, 3 spilled on the FRESH path; 20 one-wave
// workgroups of 8 KB fill the CU's LDS): tier 0 2.206 -> 2.163 ms against 4
// (105 VGPRs), A/B round 6.  The overlapped hand-on launches the 4-wave
// build: at 5 waves tier 0 holds all of the LDS and the consumers beside it
// waited (one-eighth size: tail 0.013 -> 0.037 ms).
template <bool FRESH, int OCC>
__global__ __launch_bounds__(64 * W_WAVES, OCC) void trmv_wave_kernel(TrmvApplyArgs a) {
  __shared__ WaveLds<FRESH> lds[W_WAVES];
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  WaveLds<FRESH>& L = lds[wv];
  const uint32_t n_first = a.first_list ? *a.n_first : 0u;
  const uint32_t n = (a.n_list_dev ? *a.n_list_dev : a.n_list) + n_first;
  for (uint32_t c0 = (blockIdx.x * W_WAVES + wv) * W_KPW; c0 < n; c0 += gridDim.x * W_WAVES * W_KPW) {
    const uint32_t cn = c0 + W_KPW < n ? W_KPW : n - c0;
    ChunkHdr hdr;
    wave_load_chunk(a, c0, cn, n_first, hdr);
    KeyIn cur, nxt;
    wave_load_key(a, hdr, 0, cur);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the ops are in
    wave_load_rows(a, L, cur);
    for (uint32_t j = 0; j < cn; ++j) {
      const uint32_t key = rl32(hdr.key, (int)j);
      const bool has_next = j + 1 < cn;
      // a key first_list held is done already: only the next key's loads
      const int r = (hdr.skip >> j) & 1u ? W_REJECT + 1
                                         : trmv_wave_key<FRESH>(a, key, cur, L, has_next, hdr, j + 1, nxt);
      if (r != W_DONE) {
        if (r == W_NEXT_TIER && lane_id() == 0) {
          const uint32_t pos = atomicAdd(&KA->status[0], 1u);
          KA->ovf_list[pos] = key;
          // published for tier R beside this kernel: a device-scope atomic,
          // performed before the wave goes on (and before its done add)
          if (KA->pub && pos < KA->n_pub) {
            const uint32_t old = atomicExch(&KA->pub[pos], key + 1u);
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the exchange is done
            asm volatile("" ::"v"(old));
          }
        }
        if (has_next) wave_load_key(a, hdr, j + 1, nxt);
        // retire these loads here, as the common path does before its
        // stores: otherwise every key would wait on the previous key's stores
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        if (has_next) wave_load_rows(a, L, nxt);
      }
      wave_lds_sync();  // LDS is reused by the wave's next key
      cur = nxt;
    }
  }
  // this wave is finished (its hand-ons published above); relaxed: an
  // agent-scope release here would write the XCD's L2 back once per wave
  if (a.done && lane_id() == 0) atomicAdd(&KA->done[(blockIdx.x * W_WAVES + wv) % TRMV_NDONE], 1u);
}

// grid_keys = keys the grid covers (all keys for the first tier)
void trmv_wave_preload() {
  preload_kernels(trmv_wave_kernel<true, 5>, trmv_wave_kernel<false, 5>, trmv_wave_kernel<true, 4>);
}

// waves of the launch trmv_launch_wave makes for grid_keys keys
uint32_t trmv_wave_waves(uint64_t grid_keys) {
  const uint64_t per_block = (uint64_t)W_WAVES * W_KPW;
  return (uint32_t)((grid_keys + per_block - 1) / per_block) * W_WAVES;
}

int trmv_launch_wave(const TrmvApplyArgs& a, uint64_t grid_keys, hipStream_t st) {
  if (grid_keys == 0) return CCRDT_OK;
  const uint64_t per_block = (uint64_t)W_WAVES * W_KPW;
  const uint64_t blocks = (grid_keys + per_block - 1) / per_block;
  if (a.fresh)
    if (a.pub)  // overlapped hand-on: room for the consumers
      hipLaunchKernelGGL((trmv_wave_kernel<true, 4>), dim3((unsigned)blocks), dim3(64 * W_WAVES), 0, st, a);
    else
      hipLaunchKernelGGL((trmv_wave_kernel<true, 5>), dim3((unsigned)blocks), dim3(64 * W_WAVES), 0, st, a);
  else
    hipLaunchKernelGGL((trmv_wave_kernel<false, 5>), dim3((unsigned)blocks), dim3(64 * W_WAVES), 0, st, a);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

}  // namespace ccrdt

#ifdef TRMV_PROF
extern "C" int ccrdt_debug_trmv_prof(unsigned long long* out16, int reset) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_trmv_prof), 16 * 8) != hipSuccess) return 4;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_trmv_prof), z, sizeof(z)) != hipSuccess) return 4;
  }
  return 0;
}
#endif
