/* ccrdt_gen.h — seeded synthetic effect streams for benchmarks and tests
 * (SURVEY §8d).  Not part of the drop-in boundary: a workload utility that
 * produces arrays in exactly the layout ccrdt_*_apply expects. */
#ifndef CCRDT_GEN_H
#define CCRDT_GEN_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

uint64_t ccrdt_splitmix64(uint64_t x);

/* Number of rmv ops (= rmv_vc rows) ccrdt_gen_trmv will produce. */
int64_t ccrdt_gen_trmv_count(int64_t n_ops, uint64_t seed, int rmv_pm);

/* topk_rmv effect stream, CSR by key (see gen.cpp for the distribution).
 * Every DC clock starts at clock0 (0 = a fresh stream; a later batch of the
 * same long stream passes a clock0 above every earlier timestamp).
 * Outputs: key_ptr[n_keys+1], kind/id/score/dc/ts[n_ops],
 * rmv_vc[ccrdt_gen_trmv_count(...) * n_dc]. */
int ccrdt_gen_trmv(int64_t n_ops, int64_t n_keys, int n_dc, int64_t n_players, int64_t score_max,
                   int rmv_pm, int lag_max, int dup_pm, int swap_pm, uint64_t seed,
                   int64_t clock0, uint64_t* key_ptr, uint8_t* kind, int64_t* id, int64_t* score, uint8_t* dc,
                   int64_t* ts, int64_t* rmv_vc);

/* Synthetic Zipf text corpus (wordcount / worddocumentcount):
 * a vocabulary of `vocab` lowercase words of length 1..12, word ranks drawn
 * with Zipf(s = 1) frequencies, ' ' between words, '\n' instead after ~1 in
 * 12 words, a doubled space after ~1 in 100 (empty tokens).  `n_docs`
 * documents of `doc_bytes` bytes each (the last word of a document is cut at
 * its end), written to bytes[n_docs * doc_bytes]; doc_off[n_docs + 1] gets
 * the document offsets.  Deterministic in `seed` for any thread count. */
int ccrdt_gen_corpus(int64_t n_docs, int64_t doc_bytes, int64_t vocab, uint64_t seed, int threads,
                     uint8_t* bytes, uint64_t* doc_off);

#ifdef __cplusplus
}
#endif
#endif
