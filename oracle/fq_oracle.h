/*
 * fq_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's per-read hot path (Wsc000123/fqtool,
 * src/peprocessor.cpp:261-508 and src/seprocessor.cpp:290-388 with the functions they call),
 * used as the parity checker for the HIP engine and as the "port" CPU baseline.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  It is pinned
 * against the compiled reference itself: per-function known-answer vectors produced by
 * oracle/harness/ref_kat.cpp (tests/golden/kat_*.tsv) and end-to-end outputs of
 * oracle/_ref/fqtool_ref on the reference's testdata (tests/golden/ref_*).
 *
 * It shares its types (fq_params, fq_batch, fq_read_result, accumulator layout) with the
 * engine's C-ABI (include/fqengine.h) so that both are run on identical inputs.
 */
#ifndef FQ_ORACLE_H
#define FQ_ORACLE_H

#include "../include/fqengine.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_overlap {
    int overlapped, offset, overlap_len, diff;
} orc_overlap;

/* Filter::passFilter (src/filter.cpp:3-52); is_null <=> Read* == NULL */
int orc_pass_filter(const fq_params* p, const uint8_t* seq, const uint8_t* qual, int len, int is_null);

/* Filter::trimAndCut (src/filter.cpp:69-189); returns 0 for NULL, else 1 with the surviving
 * window [*start, *start + *len) of the input */
int orc_trim_and_cut(const fq_params* p, const uint8_t* seq, const uint8_t* qual, int len,
                     int front, int tail, int* start, int* out_len);

/* PolyX::trimPolyG (src/polyx.cpp:14-38); returns the new length; *bases = recorded bases
 * (FilterResult::addPolyXTrimmed(3, bases)) or -1 when nothing was recorded */
int orc_trim_polyg(const uint8_t* seq, int len, int compare_req, int max_mismatch, int per,
                   int* bases);

/* PolyX::trimPolyX (src/polyx.cpp:45-101); *poly = base index (ATCGN) or -1 */
int orc_trim_polyx(const uint8_t* seq, int len, int mask, int compare_req, int max_mismatch,
                   int per, int* poly, int* bases);

/* OverlapAnalysis::analyze (src/overlapanalysis.cpp:7-72) */
orc_overlap orc_analyze(const uint8_t* s1, int len1, const uint8_t* s2, int len2, int diff_limit,
                        int require);

/* AdapterTrimmer::trimBySequence (src/adaptertrimmer.cpp:29-90): returns 1 if trimmed; *pos
 * is the matched position (may be negative); new length = pos < 0 ? 0 : pos */
int orc_trim_by_sequence(const uint8_t* seq, int len, const uint8_t* adapter, int alen, int* pos);

/* Stats::statRead (src/stats.cpp:237-295) into accumulator stats block `st` */
void orc_stat_read(uint64_t* st, int max_cycles, const uint8_t* seq, const uint8_t* qual, int len);

/* The whole loop body over one pack; results has n (SE) or 2n (PE) entries; acc is
 * fq_acc_words(p->insert_size_max, p->max_cycles) uint64 words and is accumulated into.
 * Returns FQ_OK, or FQ_E_TOO_LONG / FQ_E_INVALID. */
int orc_process_batch(const fq_params* p, const fq_batch* b, fq_read_result* results, uint64_t* acc);

/* Duplicate (src/duplicate.cpp:46-166): a table of 4^keylen (at most 2^32) keys; add_batch runs
 * statPair (PE) / statRead (SE) on every read of a pack in order (before any filter, as the
 * reference does); stat is statAll (hist / gc sums of hist_size bins, totals = reads, dups). */
typedef struct orc_dup orc_dup;
orc_dup* orc_dup_create(int keylen);
void orc_dup_destroy(orc_dup* d);
void orc_dup_add_batch(orc_dup* d, const fq_batch* b, int paired);
void orc_dup_stat(const orc_dup* d, int hist_size, uint64_t* hist, uint64_t* gc_sum, uint64_t* totals);

/* Evaluator::evaluateAdapterSeq's k-mer loops (src/evaluator.cpp:265-279, :392-405) with the
 * fq_kmer_* signatures (include/fqengine.h): the CPU suite's backend for fqh_set_kmer_backend. */
int orc_kmer_open(int device, const uint8_t* seq, const uint32_t* off, int32_t n, void** out);
int orc_kmer_close(void* set);
int orc_kmer_count(void* set, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t* counts);
int orc_kmer_find(void* set, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t seed, uint64_t* occ,
                  size_t cap, size_t* n_out);

/* Synthetic workload generator (host twin of fq_synth_fill_device, bit-identical output). */
void orc_synth_fill(const fq_batch* b, uint64_t seed, uint64_t first_index, int read_len);

#ifdef __cplusplus
}
#endif
#endif
