/* ccrdt.h — C-ABI of libccrdt, the MI355X batch engine for antidote_ccrdt.
 *
 * The reference is a pure-Erlang behaviour (src/antidote_ccrdt.erl:47-59):
 * every CCRDT module exports new/0, value/1, downstream/2, update/2, equal/2,
 * to_binary/1, from_binary/1, is_operation/1, is_replicate_tagged/1,
 * can_compact/2, compact_ops/2 and require_state_downstream/1.  Antidote
 * calls Mod:update(Effect, State) once per effect per replica.  This ABI is
 * what a NIF shim over that behaviour would bind: the host
 * batches effects per key (CSR by key, stream order inside a key) and one
 * call applies the whole batch on the GPU, with every key's state resident in
 * HBM.  Each entry point below names the reference function(s) it replaces.
 *
 * Conventions
 *  - Plain pointers and sizes only.  `host` pointers are read/written
 *    synchronously by the call; `_device` variants take device pointers and
 *    enqueue on the engine stream without synchronising.
 *  - Integers are int64 (Erlang integers are unbounded): values
 *    outside the engine's range are rejected with CCRDT_ERANGE so the caller
 *    can keep that key on its BEAM path.
 *  - DC ids are ranks 0..n_dc-1 that preserve Erlang term order between the
 *    DcIds.  Vector clocks are dense [n_dc] int64 rows where 0
 *    means "no entry" (vc_get_timestamp/2 default, topk_rmv.erl:350-355), so
 *    every stored timestamp must be >= 1.
 *  - Return codes are CCRDT_* below; ccrdt_last_error() gives a message for
 *    the calling thread.  Invalid ops (the reference crashes with
 *    function_clause, e.g. topk_rmv.erl:141-148) give CCRDT_EINVAL and leave
 *    the engine state unchanged.
 *  - Threading: one engine per GPU; calls on one engine must be serialised by
 *    the caller (a NIF would run them on a dirty scheduler).
 */
#ifndef CCRDT_H
#define CCRDT_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CCRDT_OK 0
#define CCRDT_EINVAL 1  /* malformed op / argument: reference would crash */
#define CCRDT_ERANGE 2  /* integer outside engine range (Q17) */
#define CCRDT_ENOMEM 3  /* device or per-key capacity exhausted */
#define CCRDT_EDEVICE 4 /* HIP / RCCL failure */
#define CCRDT_ENOSYS 5  /* operation not supported for this type */
#define CCRDT_EKEYCAP 6 /* topk_rmv: the batch COMMITTED except for the keys
                           that would exceed the per-key capacity
                           (CCRDT_TRMV_MAX_PLAYERS players, 65535 Masked
                           elements, 65534 Removals rows); those keep their
                           previous state, produce no extras, and are listed
                           by ccrdt_engine_handed_on(e, 4).  Their ops go to
                           the host (Erlang) path. */
#define CCRDT_EPARTIAL 7 /* topk_rmv: the batch COMMITTED except for the keys
                           listed by ccrdt_engine_handed_on(e, 3): the in-place
                           pass updated every other key, and the full rewrite
                           that applies these keys' ops failed (device memory,
                           2^32 elements, a HIP error: ccrdt_last_error says
                           which).  They keep their previous state and produce
                           no extras; the engine stays usable (the next batch
                           is a full rewrite).  Their ops may be re-applied in
                           a later batch. */

/* Registry: antidote_ccrdt:?CCRDTS (src/antidote_ccrdt.erl:28-35). */
#define CCRDT_AVERAGE 0
#define CCRDT_TOPK 1
#define CCRDT_TOPK_RMV 2
#define CCRDT_LEADERBOARD 3
#define CCRDT_WORDCOUNT 4
#define CCRDT_WORDDOCUMENTCOUNT 5

/* Effect kinds of topk_rmv (topk_rmv.erl:77-78) — also extra-effect kinds. */
#define CCRDT_TRMV_ADD 0
#define CCRDT_TRMV_ADD_R 1
#define CCRDT_TRMV_RMV 2
#define CCRDT_TRMV_RMV_R 3
#define CCRDT_NOOP 255 /* downstream result `noop` / "no extra effect" */

/* topk_rmv limits: DCs per engine; players per key (the HBM class of tier S,
 * tier 4 below, is the last one). */
#define CCRDT_TRMV_MAX_DC 8
#define CCRDT_TRMV_MAX_PLAYERS 16384

typedef struct ccrdt_engine ccrdt_engine;

/* ---------------------------------------------------------------- engine */

/* antidote_ccrdt:is_type/1 (src/antidote_ccrdt.erl:61-62) */
int ccrdt_is_type(int type);
/* antidote_ccrdt:generates_extra_operations/1 (src/antidote_ccrdt.erl:64-65) */
int ccrdt_generates_extra_operations(int type);

/* Create an engine holding `n_keys` CCRDT objects of `type`, each equal to
 * Mod:new(k) (topk_rmv.erl:86-88, leaderboard.erl:79-81, topk.erl:70-71;
 * average.erl:56-57 and wordcount.erl:44-45 ignore k), on HIP device
 * `device`.  n_dc is the number of DCs (topk_rmv only, <= CCRDT_TRMV_MAX_DC). */
int ccrdt_engine_create(int type, int64_t k, int64_t n_keys, int n_dc, int device,
                        ccrdt_engine** out);
int ccrdt_engine_destroy(ccrdt_engine* e);
/* Every key back to Mod:new(k).  O(1): marks the resident state empty. */
int ccrdt_engine_reset(ccrdt_engine* e);
/* Deep copy (used for the functional update/2 of the behaviour mirror). */
int ccrdt_engine_clone(const ccrdt_engine* src, ccrdt_engine** out);
int ccrdt_engine_sync(ccrdt_engine* e);
/* hipStream_t the engine enqueues on (for event timing by callers). */
void* ccrdt_engine_stream(ccrdt_engine* e);
const char* ccrdt_strerror(int code);
const char* ccrdt_last_error(void);

/* Device memory helpers so callers need no HIP headers. */
int ccrdt_device_count(int* n);
int ccrdt_set_device(int device);
int ccrdt_device_alloc(void** p, uint64_t bytes);
int ccrdt_device_free(void* p);
int ccrdt_memcpy_h2d(void* dst, const void* src, uint64_t bytes);
int ccrdt_memcpy_d2h(void* dst, const void* src, uint64_t bytes);
int ccrdt_device_synchronize(void);

/* Duration (HIP events on the engine stream) of the apply kernel launches of
 * the last batch (every tier of the chain) — what bench.py reports. */
int ccrdt_engine_last_kernel_ms(ccrdt_engine* e, float* ms);
/* topk_rmv tiers: 0 = trmv_wave (fresh keys, one wave per
 * key), 1 / 2 = trmv_steady with up to 256 / 1024 players per key in LDS,
 * 3 = trmv_resident (resident keys, K <= 128, Observed in registers),
 * 4 = trmv_steady's HBM class (up to CCRDT_TRMV_MAX_PLAYERS players, working
 * set in device scratch).  Chains: fresh 0 -> 3 -> 1 -> 2 (K <= 128),
 * resident 3 -> 1 -> 2;
 * tier 4 runs on tier 2's hand-ons.  Keys handed on by tier `t` in the last
 * batch: */
int ccrdt_engine_overflow_keys(ccrdt_engine* e, int t, int64_t* n);
/* Kernel time (HIP events) of tier `t` in the last topk_rmv batch. */
int ccrdt_engine_tier_ms(ccrdt_engine* e, int t, float* ms);
/* The keys tier `t` handed on in the last topk_rmv batch (up to `cap` of
 * them into `keys`; *n = how many there were).  Diagnostics / bench. */
int ccrdt_engine_handed_on(ccrdt_engine* e, int t, uint32_t* keys, int64_t cap, int64_t* n);

/* Event timing on the engine stream (for bench.py; HIP events). */
int ccrdt_timer_start(ccrdt_engine* e);
/* Milliseconds since ccrdt_timer_start, synchronising the stream. */
int ccrdt_timer_stop(ccrdt_engine* e, float* ms);

/* --------------------------------------------------------------- topk_rmv */

/* A batch of topk_rmv effects, CSR by key, stream order inside each key.
 * op i belongs to key k iff key_ptr[k] <= i < key_ptr[k+1].
 *   kind[i]  CCRDT_TRMV_ADD / _ADD_R  -> add/4   (topk_rmv.erl:141-144,231-249)
 *            CCRDT_TRMV_RMV / _RMV_R  -> rmv/3   (topk_rmv.erl:145-148,252-298)
 *   add:  id, score, dc (rank), ts (>= 1)        = {Id, Score, {DcId, Ts}}
 *   rmv:  id, and ts[i] = row r of rmv_vc: VcRmv = rmv_vc[r*n_dc .. +n_dc)
 *         (0 = DC absent from the Erlang map); score/dc ignored. */
typedef struct {
  int64_t n_ops;
  int64_t n_rmv_rows;
  const uint64_t* key_ptr; /* [n_keys+1] */
  const uint8_t* kind;     /* [n_ops] */
  const int64_t* id;       /* [n_ops] */
  const int64_t* score;    /* [n_ops] */
  const uint8_t* dc;       /* [n_ops] */
  const int64_t* ts;       /* [n_ops] */
  const int64_t* rmv_vc;   /* [n_rmv_rows * n_dc] */
} ccrdt_trmv_ops;

/* Host log compaction before upload: per key, can_compact/2
 * + compact_ops/2 (topk_rmv.erl:178-223) folded over adjacent effects in
 * stream order (an effect is tried once against the last kept one; {noop}
 * halves are dropped).  `out` arrays have the input's capacity (n_ops ops,
 * n_ops * n_dc clock values); out->key_ptr has n_keys + 1 entries.  Every
 * output rmv gets its own clock row (merged Vcs included), numbered in
 * stream order; out->n_ops / out->n_rmv_rows are set.  Host only. */
typedef struct {
  int64_t n_ops;
  int64_t n_rmv_rows;
  uint64_t* key_ptr;
  uint8_t* kind;
  int64_t* id;
  int64_t* score;
  uint8_t* dc;
  int64_t* ts;
  int64_t* rmv_vc;
} ccrdt_trmv_batch;
int ccrdt_trmv_compact(int n_dc, int64_t n_keys, const ccrdt_trmv_ops* in, ccrdt_trmv_batch* out);

/* Extra effects ({ok, State, [Effect]}, at most one per op — SURVEY Q3),
 * indexed by op.  kind[i] = CCRDT_NOOP when op i returned {ok, State}.
 *   CCRDT_TRMV_ADD -> {add, {Id, Score, {Dc, Ts}}}   promotion (topk_rmv.erl:295)
 *   CCRDT_TRMV_RMV -> {rmv, {Id, Vc}}, Vc in vc[i*n_dc..] (topk_rmv.erl:237)
 * Any pointer may be NULL (not wanted). */
typedef struct {
  uint8_t* kind;   /* [n_ops] */
  int64_t* id;     /* [n_ops] */
  int64_t* score;  /* [n_ops] */
  uint8_t* dc;     /* [n_ops] */
  int64_t* ts;     /* [n_ops] */
  int64_t* vc;     /* [n_ops * n_dc] */
} ccrdt_trmv_extra;

/* update/2 over a whole batch, host buffers (uploaded by the call). */
int ccrdt_trmv_apply(ccrdt_engine* e, const ccrdt_trmv_ops* ops, ccrdt_trmv_extra* extra);

/* update/2 over a batch already resident in HBM (device pointers, n_ops and
 * key_ptr in HBM too).  Enqueued on the engine stream; extra effects stay on
 * the device (ccrdt_trmv_extra_count / ccrdt_trmv_fetch_extra). */
int ccrdt_trmv_apply_device(ccrdt_engine* e, const ccrdt_trmv_ops* dev_ops);
/* Number of extra effects produced by the last apply. */
int ccrdt_trmv_extra_count(ccrdt_engine* e, int64_t* n);
/* Copy the last apply's extra effects into op-indexed host arrays. */
int ccrdt_trmv_fetch_extra(ccrdt_engine* e, ccrdt_trmv_extra* extra);

/* Layout of the next fresh batches (after ccrdt_engine_create / _reset):
 * on != 0 lays each key out with room to grow (players 3x its ops + 16,
 * Masked pool 6x + 32, Removals rows 1x + 8), so the resident batches that
 * follow update it in place from the first one on, instead of rewriting
 * every key once to give it room; 0 (the default) lays the fresh batch out
 * tight, which writes it about 3% faster.  Only with Size <= 128 (tier R's
 * class) and while the layout's offsets fit 32 bits; else ignored. */
int ccrdt_trmv_set_fresh_room(ccrdt_engine* e, int on);

/* Device side of the cluster's two exchange steps (the
 * collectives are the caller's, e.g. RCCL).  Both are enqueued on the engine
 * stream (ccrdt_engine_stream) and do not wait.
 * Replica Vc: d_out[n_dc] (device) := elementwise max of every key's Vc, the
 * dense form of merge_vcs/2 (topk_rmv.erl:378-386); a MAX all-reduce of it
 * over the shards is the replica-wide Vc. */
int ccrdt_trmv_replica_vc_device(ccrdt_engine* e, int64_t* d_out);
/* Extra effects of the last apply (topk_rmv.erl:236-237, :294-295) packed
 * into device rows d_rows[cap_rows][6 + n_dc] = {op, kind, id, score, dc, ts,
 * vc...}, grouped by key (order by op to get stream order); *d_count
 * (device) = how many there were (rows past cap_rows are not written). */
int ccrdt_trmv_extras_device(ccrdt_engine* e, int64_t* d_rows, int64_t cap_rows, uint32_t* d_count);
/* One rank's exchange pack in one call (both steps above, no host wait):
 * d_pack = [word | Vc[n_dc] | rows[cap_rows][6 + n_dc]] (int64, device), word
 * = extra-effect count (bits 0-31) | host_word << 32; a row's op is mapped
 * through d_op_map[n_map] (local op -> global op; NULL: as it is). */
int ccrdt_trmv_exchange_pack(ccrdt_engine* e, int64_t* d_pack, int64_t cap_rows, const int64_t* d_op_map,
                             int64_t n_map, uint32_t host_word);
/* The gathered packs of `world` ranks (d_gathered[world][len] int64, device,
 * each the first `len` words of a rank's pack: head + its first rows) ->
 * d_hdr (device int64[2 * world + 1 + n_dc]: per rank its count word's low
 * 32 bits, then per rank the word's high 32 bits, then the sum of the ranks'
 * bits 32-61, then the elementwise-max Vc) and d_rows (device, [world *
 * rows_per][6 + n_dc]): every rank's first min(count, rows_per) rows sorted by
 * op (ties: rank order), *then* d_hdr[...] is complete.  rows_per = (len - 1 -
 * n_dc) / (6 + n_dc).  Enqueued on the engine stream. */
int ccrdt_trmv_exchange_reduce(ccrdt_engine* e, const int64_t* d_gathered, int world, int64_t len, int64_t* d_hdr,
                               int64_t* d_rows);

/* Canonical state image (host arrays), used by export/import:
 *   vc[n_keys*n_dc]                                   replica Vc
 *   obs_ptr[n_keys+1], obs_{id,score,dc,ts}           Observed, sorted by id
 *   m_ptr[n_keys+1],  m_{id,score,dc,ts}              Masked elems, sorted by
 *                                                     (id, score, dc, ts)
 *   r_ptr[n_keys+1],  r_id, r_vc[*n_dc]               Removals, sorted by id
 *   min_valid[n_keys], min_{id,score,dc,ts}           Min ({nil,nil,nil} = 0)
 * (topkrmv() = {Observed, Masked, Removals, Vc, Min, Size}, topk_rmv.erl:67-74) */
typedef struct {
  int64_t* vc;
  uint64_t* obs_ptr;
  int64_t *obs_id, *obs_score, *obs_ts;
  uint8_t* obs_dc;
  uint64_t* m_ptr;
  int64_t *m_id, *m_score, *m_ts;
  uint8_t* m_dc;
  uint64_t* r_ptr;
  int64_t *r_id, *r_vc;
  uint8_t* min_valid;
  int64_t *min_id, *min_score, *min_ts;
  uint8_t* min_dc;
} ccrdt_trmv_state;

/* Totals for sizing a ccrdt_trmv_state. */
int ccrdt_trmv_state_sizes(ccrdt_engine* e, int64_t* n_obs, int64_t* n_masked, int64_t* n_rows);
/* The same for keys [k0, k1) only. */
int ccrdt_trmv_range_sizes(ccrdt_engine* e, int64_t k0, int64_t k1, int64_t* n_obs, int64_t* n_masked,
                           int64_t* n_rows);
/* Per-key counts of the resident state (players, Masked elements, Removals
 * rows, |Observed|); any output may be NULL.  For bench.py's byte accounting. */
int ccrdt_trmv_key_sizes(ccrdt_engine* e, uint32_t* np, uint32_t* nm, uint32_t* nr, uint32_t* nobs);
/* to_binary/1 analogue (topk_rmv.erl:156-158): canonical image of every key. */
int ccrdt_trmv_export(ccrdt_engine* e, ccrdt_trmv_state* out);
/* The canonical image of keys [k0, k1) only (value/1, to_binary/1 of a few
 * keys): downloads just their segments.  `out` is laid out as for an engine of
 * k1 - k0 keys (ptr arrays [k1-k0+1], vc / min arrays [k1-k0]). */
int ccrdt_trmv_export_range(ccrdt_engine* e, int64_t k0, int64_t k1, ccrdt_trmv_state* out);
/* from_binary/1 of keys [k0, k1): those keys take the given image (laid out
 * as for an engine of k1 - k0 keys); the other keys keep their state. */
int ccrdt_trmv_import_range(ccrdt_engine* e, int64_t k0, int64_t k1, const ccrdt_trmv_state* in);
/* from_binary/1 analogue (topk_rmv.erl:161-163).  Arrays as in export
 * (sorting not required); invariants of the reference are checked. */
int ccrdt_trmv_import(ccrdt_engine* e, const ccrdt_trmv_state* in);

/* to_binary/1 of one key of a state image (topk_rmv.erl:156-158: term_to_binary
 * of {Observed, Masked, Removals, Vc, Min, Size}) in native code: key k of `st`
 * (the ccrdt_trmv_state layout, n_dc clock columns) as Erlang external term
 * format -- elements {Score, Id, {DcId, Ts}}, Masked[Id] as the balanced
 * gb_sets {Size, Tree} of gb_sets:from_ordset/1, clocks as maps without their
 * 0 entries, Min {nil, nil, nil} when absent, map keys in term order.  DC rank
 * d is written as the ETF term dc_term[dc_off[d] .. dc_off[d+1]) (no version
 * byte; atoms as SMALL_ATOM_UTF8; ranks in term order, as the engine's are).
 * Writes at most `cap` bytes into buf; *len = the term's size in bytes
 * (CCRDT_ENOMEM when cap < *len: call with cap = 0 to size the buffer).  The
 * same bytes as the Python codec (antidote_ccrdt_amd/etf.py). */
int ccrdt_trmv_key_to_binary(const ccrdt_trmv_state* st, int n_dc, int64_t k, int64_t size,
                             const uint8_t* dc_term, const uint64_t* dc_off, uint8_t* buf, uint64_t cap,
                             uint64_t* len);
/* from_binary/1 (topk_rmv.erl:161-163): an ETF state 6-tuple as ERTS writes it
 * (maps in any order, any integer / atom / tuple tag, gb_sets trees of any
 * shape) -> the canonical image of ONE key in `out` (ptr arrays [2], vc /
 * min arrays [1]; sorted as ccrdt_trmv_export sorts).  DcIds are matched by
 * their canonical encoding against dc_term (as for to_binary).  counts[3] =
 * the key's |Observed|, Masked elements, Removals rows; *size = Size.  With
 * out or caps NULL only counts and size are set (the sizing call); a count
 * above caps[i] is CCRDT_ENOMEM.  A malformed term or unknown DcId is
 * CCRDT_EINVAL (binary_to_term badarg / a DC the engine does not hold), an
 * integer outside int64 CCRDT_ERANGE. */
int ccrdt_trmv_key_from_binary(const uint8_t* buf, uint64_t len, int n_dc, const uint8_t* dc_term,
                               const uint64_t* dc_off, ccrdt_trmv_state* out, const int64_t* caps,
                               int64_t* counts, int64_t* size);

/* downstream/2 (topk_rmv.erl:102-124) for n requests against the current
 * state (read-only).  op[i] 0 = {add, {Id, Score}}, 1 = {rmv, Id}.  For add,
 * dc[i]/ts[i] are the origin's DC rank and clock (?DC_META_DATA, ?TIME).
 * out_kind[i] = CCRDT_TRMV_ADD / _ADD_R / _RMV / _RMV_R / CCRDT_NOOP.  For rmv
 * the effect's Vc is the key's replica Vc, written to out_vc[i*n_dc..] if
 * out_vc is not NULL. */
int ccrdt_trmv_downstream(ccrdt_engine* e, int64_t n, const uint64_t* key, const uint8_t* op,
                          const int64_t* id, const int64_t* score, const uint8_t* dc,
                          const int64_t* ts, uint8_t* out_kind, int64_t* out_vc);


/* ---------------------------------------------------------------- average */

/* {add, {V, N}} effects (src/antidote_ccrdt_average.erl:88-94); {add, V} is
 * N = 1 (downstream/2 :77-81).  CSR by key. */
typedef struct {
  int64_t n_ops;
  const uint64_t* key_ptr; /* [n_keys+1] */
  const int64_t* value;    /* [n_ops] V */
  const int64_t* n;        /* [n_ops] N (0 = no-op, < 0 = EINVAL) */
} ccrdt_avg_ops;
/* update/2 over a batch (host arrays).  Sums that leave int64 give ERANGE. */
int ccrdt_avg_apply(ccrdt_engine* e, const ccrdt_avg_ops* ops);
/* Host log compaction (average.erl:122-127): every pair compacts, so each
 * key's effects become one {add, {Sum V, Sum N}}; ERANGE past int64. */
typedef struct {
  int64_t n_ops;
  uint64_t* key_ptr;
  int64_t* value;
  int64_t* n;
} ccrdt_avg_batch;
int ccrdt_avg_compact(int64_t n_keys, const ccrdt_avg_ops* in, ccrdt_avg_batch* out);
int ccrdt_avg_apply_device(ccrdt_engine* e, const ccrdt_avg_ops* dev_ops);
/* State {Sum, Num} of every key (to_binary/from_binary analogues). */
int ccrdt_avg_export(ccrdt_engine* e, int64_t* sum, int64_t* num);
int ccrdt_avg_import(ccrdt_engine* e, const int64_t* sum, const int64_t* num);
/* value/1 (:68-70): Sum / Num in IEEE double; defined[k] = 0 where Num = 0
 * (the reference raises badarith). */
int ccrdt_avg_value(ccrdt_engine* e, double* value, uint8_t* defined);

/* ------------------------------------------------------------------- topk */

/* {add, {Id, Score}} effects (src/antidote_ccrdt_topk.erl:100-104); an
 * {add_map, Map} effect is its entries in any order (maps:merge). */
typedef struct {
  int64_t n_ops;
  const uint64_t* key_ptr; /* [n_keys+1] */
  const int64_t* id;       /* [n_ops] (binary Ids interned by the host in term order) */
  const int64_t* score;    /* [n_ops] */
} ccrdt_topk_ops;
int ccrdt_topk_apply(ccrdt_engine* e, const ccrdt_topk_ops* ops);
int ccrdt_topk_apply_device(ccrdt_engine* e, const ccrdt_topk_ops* dev_ops);
int ccrdt_topk_size(ccrdt_engine* e, int64_t* n_entries);
/* The map of every key, sorted by Id: ptr[n_keys+1], id/score[n_entries]. */
int ccrdt_topk_export(ccrdt_engine* e, uint64_t* ptr, int64_t* id, int64_t* score);
int ccrdt_topk_import(ccrdt_engine* e, const uint64_t* ptr, const int64_t* id, const int64_t* score);
/* Keys [k0, k1) only (value/1, to_binary/from_binary of single objects
 * without a whole-engine round trip): entry count, the image laid out for
 * k1 - k0 keys (ptr[k1 - k0 + 1]), and its import over those keys. */
int ccrdt_topk_range_size(ccrdt_engine* e, int64_t k0, int64_t k1, int64_t* n_entries);
int ccrdt_topk_export_range(ccrdt_engine* e, int64_t k0, int64_t k1, uint64_t* ptr, int64_t* id,
                            int64_t* score);
int ccrdt_topk_import_range(ccrdt_engine* e, int64_t k0, int64_t k1, const uint64_t* ptr,
                            const int64_t* id, const int64_t* score);
/* value/1 (:81-83): every key's entries sorted by Score desc, Id desc (GPU
 * segmented sort). */
int ccrdt_topk_value(ccrdt_engine* e, uint64_t* ptr, int64_t* id, int64_t* score);
/* downstream/2 (:89-94, changes_state :164-166): out[i] = CCRDT_TRMV_ADD if
 * score[i] > Size else CCRDT_NOOP. */
int ccrdt_topk_downstream(ccrdt_engine* e, int64_t n, const int64_t* score, uint8_t* out_kind);

/* ------------------------------------------------------------ leaderboard */

#define CCRDT_LB_ADD 0
#define CCRDT_LB_ADD_R 1
#define CCRDT_LB_BAN 2
/* {add|add_r, {Id, Score}} and {ban, Id} effects
 * (src/antidote_ccrdt_leaderboard.erl:128-134). */
typedef struct {
  int64_t n_ops;
  const uint64_t* key_ptr; /* [n_keys+1] */
  const uint8_t* kind;     /* [n_ops] CCRDT_LB_* */
  const int64_t* id;       /* [n_ops] */
  const int64_t* score;    /* [n_ops] (ignored for ban) */
} ccrdt_lb_ops;
/* Host log compaction (leaderboard.erl:163-205), folded like
 * ccrdt_trmv_compact: of two adds of one Id the higher score survives, a ban
 * absorbs an earlier add or ban of its Id. */
typedef struct {
  int64_t n_ops;
  uint64_t* key_ptr;
  uint8_t* kind;
  int64_t* id;
  int64_t* score;
} ccrdt_lb_batch;
int ccrdt_lb_compact(int64_t n_keys, const ccrdt_lb_ops* in, ccrdt_lb_batch* out);
/* Extra effects, op-indexed: kind CCRDT_LB_ADD = {add, {Id, Score}} from a
 * ban that promoted a Masked player (:279-283), CCRDT_NOOP = none. */
typedef struct {
  uint8_t* kind;
  int64_t* id;
  int64_t* score;
} ccrdt_lb_extra;
int ccrdt_lb_apply(ccrdt_engine* e, const ccrdt_lb_ops* ops, ccrdt_lb_extra* extra);
int ccrdt_lb_apply_device(ccrdt_engine* e, const ccrdt_lb_ops* dev_ops);
int ccrdt_lb_fetch_extra(ccrdt_engine* e, ccrdt_lb_extra* extra);
/* The last apply's extra effects packed into device rows d_rows[cap_rows][4]
 * = {key, op, id, score} ({add, {Id, Score}}, leaderboard.erl:282-284), in
 * any order (op gives stream order); *d_count (device) = how many there were.
 * The replication step ships these without a host round trip. */
int ccrdt_lb_extras_device(ccrdt_engine* e, int64_t* d_rows, int64_t cap_rows, uint32_t* d_count);
/* leaderboard() = {Observed, Masked, Bans, Min, Size} (:62-68), canonical
 * (each list sorted by Id). */
typedef struct {
  uint64_t* obs_ptr;
  int64_t *obs_id, *obs_score;
  uint64_t* m_ptr;
  int64_t *m_id, *m_score;
  uint64_t* b_ptr;
  int64_t* b_id;
  uint8_t* min_valid;
  int64_t *min_id, *min_score;
} ccrdt_lb_state;
int ccrdt_lb_state_sizes(ccrdt_engine* e, int64_t* n_obs, int64_t* n_masked, int64_t* n_bans);
int ccrdt_lb_export(ccrdt_engine* e, ccrdt_lb_state* out);
int ccrdt_lb_import(ccrdt_engine* e, const ccrdt_lb_state* in);
/* Boards [k0, k1) only; the image is laid out for k1 - k0 boards. */
int ccrdt_lb_range_sizes(ccrdt_engine* e, int64_t k0, int64_t k1, int64_t* n_obs, int64_t* n_masked,
                         int64_t* n_bans);
int ccrdt_lb_export_range(ccrdt_engine* e, int64_t k0, int64_t k1, ccrdt_lb_state* out);
int ccrdt_lb_import_range(ccrdt_engine* e, int64_t k0, int64_t k1, const ccrdt_lb_state* in);
/* downstream/2 (:93-116): op 0 = {add, {Id, Score}}, 1 = {ban, Id};
 * out_kind CCRDT_LB_ADD / _ADD_R / _BAN / CCRDT_NOOP. */
int ccrdt_lb_downstream(ccrdt_engine* e, int64_t n, const uint64_t* key, const uint8_t* op,
                        const int64_t* id, const int64_t* score, uint8_t* out_kind);

/* ------------------------------------------- wordcount / worddocumentcount */

/* {add, File} effects (src/antidote_ccrdt_wordcount.erl:53-54,
 * worddocumentcount.erl:53-54): documents CSR by key. */
typedef struct {
  int64_t n_docs;
  const uint64_t* key_ptr; /* [n_keys+1] over documents */
  const uint64_t* doc_off; /* [n_docs+1] over bytes */
  const uint8_t* bytes;
  uint64_t n_bytes;
} ccrdt_wc_docs;
int ccrdt_wc_apply(ccrdt_engine* e, const ccrdt_wc_docs* docs);
int ccrdt_wc_apply_device(ccrdt_engine* e, const ccrdt_wc_docs* dev_docs);
int ccrdt_wc_sizes(ccrdt_engine* e, int64_t* n_words, int64_t* n_bytes);
/* Diagnostics of the last ccrdt_wc_apply(_device): the tokens the insert
 * kernel left to its check list (words of more than 14 bytes, slots whose
 * identity was not yet visible), or -1 when the batch was verified token by
 * token (the list filled up). */
int ccrdt_wc_last_checks(ccrdt_engine* e, int64_t* n_checked);
/* value/1 (:47-48) = the map word -> count; per key, words sorted by bytes
 * (Erlang binary order): key_ptr[n_keys+1] over words, word_off[n_words+1]
 * over word_bytes. */
int ccrdt_wc_export(ccrdt_engine* e, uint64_t* key_ptr, uint64_t* word_off, uint8_t* word_bytes,
                    int64_t* count);
/* The key-sharded histogram's exchange on the device (cluster.py): every
 * word of the maps, grouped by owner rank (the ccrdt_wc_owner function),
 * into device rows d_meta[n_words][3] = {key, length, count} and their bytes
 * d_bytes in the same order; owner_words / owner_bytes (host, [world]) get
 * each owner's share.  Buffers sized by ccrdt_wc_sizes.  CCRDT_ERANGE for a
 * table of 2^24 words or more (or 2^40 bytes): partition the export on the
 * host instead (cluster.ShardedWordcount.partition). */
int ccrdt_wc_partition_device(ccrdt_engine* e, int world, int64_t* d_meta, uint8_t* d_bytes, int64_t cap_words,
                              int64_t cap_bytes, int64_t* owner_words, int64_t* owner_bytes);
/* ccrdt_wc_merge of device rows {key, length, count} and their bytes (the
 * layout ccrdt_wc_partition_device writes; words in any order). */
int ccrdt_wc_merge_device(ccrdt_engine* e, int64_t n_words, const int64_t* d_meta, const uint8_t* d_bytes,
                          int64_t n_bytes);

/* Owner rank of every word of a CSR word list (the layout of ccrdt_wc_export):
 * splitmix64(FNV-1a64(bytes) ^ key * 0x9E3779B97F4A7C15) mod world.  The
 * key-sharded word histogram of the multi-GPU wordcount sends
 * each word to this rank, which merges it (ccrdt_wc_merge).  Host-only; no
 * engine needed. */
int ccrdt_wc_owner(int64_t n_keys, int64_t n_words, const uint64_t* key_ptr, const uint64_t* word_off,
                   const uint8_t* bytes, int world, int32_t* owner);

/* Merge word -> count pairs into the resident maps (host arrays, CSR by key:
 * key_ptr[n_keys+1] over words, word_off[n_words+1] over bytes): count is
 * added to the word's entry, created if absent.  The map union with summed
 * counts -- how a key-sharded histogram is merged after the all-to-all by word
 * owner; every word is byte-compared with its table entry
 * (ERANGE on a 64-bit hash collision). */
int ccrdt_wc_merge(ccrdt_engine* e, int64_t n_words, const uint64_t* key_ptr, const uint64_t* word_off,
                   const uint8_t* bytes, const int64_t* count);
/* from_binary/1 analogue (wordcount.erl:59-63, worddocumentcount.erl:59-63):
 * every key's map := the given words and counts (the layout of
 * ccrdt_wc_export), without replaying any text. */
int ccrdt_wc_import(ccrdt_engine* e, int64_t n_words, const uint64_t* key_ptr, const uint64_t* word_off,
                    const uint8_t* bytes, const int64_t* count);

#ifdef __cplusplus
}
#endif
#endif /* CCRDT_H */
