// types_kernels.hpp — argument blocks of the average / topk / leaderboard /
// wordcount kernels and the generic segment scan.
#pragma once
#include <cstdint>

namespace ccrdt {

enum : uint32_t { AVG_ERR_NEG = 1u, AVG_ERR_RANGE = 2u };

struct AvgArgs {
  int64_t n_keys;
  const uint64_t* key_ptr;
  const int64_t* v;
  const int64_t* n;
  const int64_t* sum_in;
  const int64_t* num_in;
  int64_t* sum_out;
  int64_t* num_out;
  int32_t fresh;
  uint32_t* status;
};

// topk: per key a segment of (id, score) entries (any order)
struct TopkArgs {
  int64_t n_keys;
  const uint64_t* key_ptr;
  const int64_t* op_id;
  const int64_t* op_score;
  const uint64_t* off_in;
  const uint32_t* cnt_in;
  const int64_t* id_in;
  const int64_t* score_in;
  const uint64_t* off_out;  // precomputed by the scan
  uint32_t* cnt_out;
  int64_t* id_out;
  int64_t* score_out;
  int32_t fresh;
  const uint32_t* key_list;
  uint32_t* ovf_list;
  uint32_t* status;
  // HBM class: per listed key a hash region at tab_off[w], tab_cap[w] slots
  const uint64_t* tab_off;
  const uint32_t* tab_cap;
  int64_t* g_id;
  int32_t* g_seq;
};

struct TopkValueArgs {
  const uint64_t* off;
  const uint32_t* cnt;
  const int64_t* id;
  const int64_t* score;
  const uint64_t* out_ptr;
  int64_t* out_id;
  int64_t* out_score;
  const uint32_t* key_list;
  uint32_t* ovf_list;
  uint32_t* status;
  // HBM class: per listed key a sort region at tab_off[w], tab_cap[w] slots
  const uint64_t* tab_off;
  const uint32_t* tab_cap;
  int64_t* g_id;
  int64_t* g_score;
};

// leaderboard: per board a segment of entries (id, score, status) + meta
enum : uint8_t { LB_OBS = 0, LB_MASKED = 1, LB_BANNED = 2 };
struct alignas(16) LbMeta {
  uint32_t off;    // segment start (entries)
  uint32_t n;      // entries
  uint32_t nobs;   // |Observed|
  uint32_t minq;   // entry index of Min, 0xFFFFFFFF = {nil,nil}
};
struct alignas(16) LbExtraRec {
  uint32_t op;
  uint32_t pad;
  int64_t id;
  int64_t score;
};
struct LbArgs {
  int64_t n_keys;
  uint32_t k;
  const uint64_t* key_ptr;
  const uint8_t* kind;
  const int64_t* id;
  const int64_t* score;
  const LbMeta* meta_in;
  const int64_t* id_in;
  const int64_t* score_in;
  const uint8_t* st_in;
  LbMeta* meta_out;
  const uint64_t* off_out;  // new segment starts (scan)
  int64_t* id_out;
  int64_t* score_out;
  uint8_t* st_out;
  int32_t fresh;
  uint32_t* ex_cnt;
  LbExtraRec* ex;
  const uint32_t* key_list;
  uint32_t* ovf_list;
  uint32_t* status;  // [0] overflow count, [1] error flags
  // HBM class: per listed board entries at tab_off[w] (tab_cap[w] of them),
  // hash slots at 2 * tab_off[w]
  const uint64_t* tab_off;
  const uint32_t* tab_cap;
  int64_t* g_eid;
  int64_t* g_esc;
  uint8_t* g_est;
  uint32_t* g_hslot;
  int32_t seq;  // 1: sequential replay only (diagnostic, CCRDT_LB_SEQ=1)
};
enum : uint32_t { LB_ERR_KIND = 1u };

struct LbDownArgs {
  int64_t n;
  uint32_t k;
  const uint64_t* key;
  const uint8_t* op;
  const int64_t* id;
  const int64_t* score;
  uint8_t* out;
  const LbMeta* meta;
  const int64_t* eid;
  const int64_t* escore;
  const uint8_t* est;
  int32_t fresh;
};

// wordcount / worddocumentcount
constexpr uint64_t WC_TILE = 4096;  // bytes of a document per wave step (64 per lane)
constexpr uint64_t WC_TPW = 8;  // tiles per wave (a chunk; measured 8 / 16 / 32: 8 best)

// A word-table slot: everything one probe or one identity compare needs lies
// in one 32-byte record (one cache sector): the hash and the word's identity
// (wc_ident: its length and up to WC_SHORT bytes, then its key), each word
// nonzero once written, so a reader that sees all three nonzero holds the
// final identity.  The counts live in their own array (the Zipf head's
// atomics would otherwise keep the lines every probe reads busy), the
// representative's bytes and the key / length as plain integers in WcMeta
// (read only by the passes after the insert kernel).
struct alignas(32) WcSlot {
  unsigned long long h;   // 0 = empty
  unsigned long long w0;  // WC_MARK | length << 56 | bytes 0..6 (a long word: WC_MARK | 0x7F << 56)
  unsigned long long w1;  // WC_MARK | bytes 7..13 (a long word: WC_MARK)
  unsigned long long w2;  // WC_MARK | key
};
static_assert(sizeof(WcSlot) == 32, "WcSlot is 32 bytes");
//   ref: the word's bytes, an arena offset once persisted, or
//        WC_REF_BATCH | the batch byte position of an occurrence (a word of
//        up to WC_SHORT bytes is persisted from its identity instead)
struct alignas(16) WcMeta {
  uint64_t ref;
  uint32_t key;
  uint32_t len;
};
constexpr uint64_t WC_REF_BATCH = 1ull << 63;
constexpr uint64_t WC_MARK = 1ull << 63;
constexpr uint32_t WC_SHORT = 14;  // words of up to 14 bytes are identified by their slot's words

// A token whose identity the insert kernel could not settle (a word of more
// than WC_SHORT bytes, or a slot whose identity words were not visible yet),
// checked after the kernel by wc_check_kernel: a = its identity w0 (WC_MARK
// set) or, for a long word, its batch position; b = w1 or its length.
struct WcChk {
  uint32_t slot;
  uint32_t key;
  uint64_t a;
  uint64_t b;
};

struct WcArgs {
  int64_t n_keys;
  int64_t n_docs;
  const uint64_t* doc_key;   // [n_docs] key of each document
  const uint64_t* doc_off;   // [n_docs+1] byte offsets
  const uint64_t* tile_ptr;  // [n_docs+1] first chunk (WC_TPW tiles) of each document, global index
  uint64_t tile0;            // first chunk of this launch (= tile_ptr[0])
  const uint32_t* chunk_doc; // [chunks of the batch] document of each chunk (batch index)
  uint64_t doc0;             // batch index of this launch's first document
  // worddocumentcount: workgroups of WAVES chunks of one document
  const uint32_t* group_doc; // [groups of the batch] document of each group (batch index), or nullptr
  const uint64_t* group_ptr; // [launch docs + 1] first group of each document (batch index)
  uint64_t group0;           // first group of this launch
  uint64_t n_groups;         // groups of this launch
  const uint8_t* bytes;
  uint64_t n_bytes;
  int32_t wdc;               // 1 = worddocumentcount (per-doc distinct)
  // word table (persistent across batches): one 32-byte slot per word
  WcSlot* t;
  WcMeta* tm;
  unsigned long long* t_cnt;
  uint64_t t_mask;
  uint64_t seed;             // word-hash seed of the table (every h of the table is under it)
  int32_t weak0;             // test hook (CCRDT_WC_WEAK0): a degenerate hash under seed 0
  const uint8_t* arena;
  // per-document dedupe table (worddocumentcount)
  uint64_t* d_hash;
  uint64_t d_mask;
  uint64_t d_base;           // document tags of this launch: d_base + 1 .. d_base + n_docs (< 2^24)
  // worddocumentcount's document lists (nullptr: the dedupe table above):
  // every (document, word) pair the insert kernel does not settle in LDS goes
  // to its document's region as the word's slot; wc_dl_kernel then counts each
  // document's distinct slots once (an LDS bitmap per document, no device
  // atomic per pair)
  uint32_t* dl;              // regions, one per document of the launch: its tokens' worth of entries
  const uint64_t* dl_pre;    // [launch docs + 1] token prefix: region of d = [dl_pre[d], dl_pre[d + 1]) - dl_pre[0]
  uint32_t* dl_cur;          // [launch docs] entries appended
  uint32_t* status;          // [0] table overflow (1) | dedupe table (2) | count list full (4) | document list full (8), [1] hash collision | token lost | check list full (16), [2] check records
  WcChk* chk;                // the check list (wc_check_kernel), chk_cap records
  uint32_t chk_cap;
  // The count list (wc_cl_*): the insert kernel's count adds, summed after
  // it by slot bucket instead of one device atomic per token.  nullptr: the
  // adds go to t_cnt directly (tables above 2^23 slots; a full list re-runs
  // the batch that way).
  uint32_t* cl;              // token entries (global slot), blocks of WC_BLK
  uint32_t* cl_bcnt;         // [blocks] entries of each block (written when the block is closed)
  uint32_t* cl_cur;          // [WC_NSHARD] blocks taken from each shard
  uint32_t cl_shard_blocks;  // blocks per shard
  uint64_t* fl;              // flush entries: per insert workgroup one per LDS entry (slot | count << 32; ~0 = none)
  uint64_t fl_base;          // flush region of this launch's first workgroup
  int32_t dbg;               // diagnostic (CCRDT_WC_IDBG): 5 = the insert kernel without its count adds
  uint64_t n_chunks;         // chunks of this insert launch
};

// The count list (types_kernels.hip wc_cl_*): blocks of WC_BLK token
// entries taken from WC_NSHARD shards; summed per bucket of 2^bsh slots
// (at most WC_CL_NB buckets, 2^WC_CL_MAXSH slots each).
constexpr uint32_t WC_BLK = 1024, WC_NSHARD = 64, WC_CL_NB = 1024, WC_CL_MAXSH = 13;
// insert workgroups: LDS entries x waves (wordcount, worddocumentcount)
// (A/B round 6: wordcount 3584 x 16 26.4 ms per step, 3072 x 16 27.5, 4096 x 12 28.9;
// worddocumentcount 1024 x 4 51.7, 3584 x 16 51.6, 1536 x 8 62.9)
constexpr uint32_t WC_TAB_WC = 3584, WC_WAVES_WC = 16, WC_TAB_WDC = 1024, WC_WAVES_WDC = 4;
static_assert(WC_TAB_WDC % 64 == 0, "the flush's document-list appends are wave-wide");
// wc_dl_kernel: slots per pass of its LDS bitmap (128 KiB), passes at most;
// the entries a wave reserves at once in its document's list
constexpr uint32_t WC_DL_BITS = 1u << 20, WC_DL_MAXPASS = 8, WC_DL_BLK = 256;
struct WcClArgs {
  const uint32_t* cl;
  const uint32_t* bcnt;
  const uint32_t* cur;
  uint32_t shard_blocks;
  const uint64_t* fl;
  uint32_t tab;
  uint64_t n_tb, n_fl;
  uint32_t bsh, nb;
  uint32_t* bkt_cnt;   // [nb] entries per bucket
  uint32_t* bkt_cur;   // [nb] scatter cursors (from the scan)
  uint64_t* bkt_off;   // [nb + 1] bucket offsets
  uint32_t* bkt;       // entries by bucket: slot within the bucket | count << bsh
  unsigned long long* t_cnt;
  uint32_t* status;
};

}  // namespace ccrdt
