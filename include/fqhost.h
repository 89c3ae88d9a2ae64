/* fqhost.h -- C-ABI of the host side (libfqhost.so): the reference's CLI/Processor plumbing
 * around the engine of fqengine.h.
 *
 * fqh_run is the whole tool (the reference's main(), src/main.cpp:11-176, with the per-pack loop
 * bodies of src/peprocessor.cpp:276-441 / src/seprocessor.cpp:271-352 running on the GPU).
 *
 * The session calls expose the same pipeline one pack at a time with the engine call left to the
 * caller, so a host that keeps its own Processor threads can read packs, hand
 * them to fq_engine_process / fq_engine_process_device and get the reference's output text and
 * JSON back.  Tests drive it with the CPU oracle in the engine's place.
 */
#ifndef FQHOST_H
#define FQHOST_H

#include <stddef.h>
#include <stdint.h>

#include "fqengine.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The tool: same arguments, outputs, messages and exit codes as the reference binary. */
int fqh_run(int argc, char** argv);

/* nlohmann::json 3.5.0 number formatting of a double (Grisu2, src/json.hpp); returns length. */
int fqh_json_double(double v, char* buf, size_t n);
/* OverlapAnalysis::merge read name (src/overlapanalysis.cpp:93-101). */
int fqh_merged_name(const char* name, int len1, int len2, char* buf, size_t n);
/* Evaluator::evaluateReadLen / detectAdapter (src/evaluator.cpp:24-86, :88-260). */
int fqh_evaluate_read_len(const char* path);
int fqh_detect_adapter(const char* path, int trim_tail1, char* buf, size_t n);

/* JSON report from one accumulator block; argv_blob = argc NUL-terminated strings back to back;
 * side = lines "D1\tSEQ", "D2\tSEQ" (detected adapters), "1\tSEQ\tN", "2\tSEQ\tN" (adapter counts).
 * Returns a malloc'd string (free with fqh_free); starts with "ERROR: " on failure. */
char* fqh_report_json(int argc, const char* argv_blob, const uint64_t* acc, int max_cycles, const char* side);
void fqh_free(char* p);

typedef struct fqh_session fqh_session;
/* parses argv like the tool (incl. the Evaluator pre-pass) and opens the inputs; on failure
 * returns -1 with *out still set so fqh_session_error can be read (then close it) */
int fqh_session_open(int argc, char** argv, fqh_session** out);
const char* fqh_session_error(const fqh_session* s);
/* engine parameters for this command line at a given stats cycle capacity */
int fqh_session_params(fqh_session* s, int max_cycles, fq_params* out);
/* next pack (up to max_n records/pairs): 1 = got one, 0 = end of input, -1 = error.
 * The batch points into session memory valid until the next call. */
int fqh_session_next(fqh_session* s, int max_n, fq_batch* out);
/* per-read records of the current pack (fq_engine_process output) -> output files, written with
 * the tool's rules, and adapter string counts */
int fqh_session_consume(fqh_session* s, const fq_read_result* res, int max_cycles);
/* -d: whether the command line enables duplication analysis, its key length and histogram size;
 * the caller runs it (fq_dup_* on the engine's device) and hands statAll's result back
 * (hist_size bins, GC sums, totals = {reads counted, duplicates}) before fqh_session_finish */
int fqh_session_dup_params(fqh_session* s, int* enabled, int* keylen, int* hist_size);
int fqh_session_set_dup(fqh_session* s, const uint64_t* hist, const uint64_t* gc_sum, const uint64_t* totals);
/* adds an accumulator block (fq_engine_read_acc layout at max_cycles) */
int fqh_session_add_acc(fqh_session* s, const uint64_t* acc, int max_cycles);
/* closes the outputs, writes the JSON report file (-J) and returns its text (malloc'd, fqh_free) */
char* fqh_session_finish(fqh_session* s);
void fqh_session_close(fqh_session* s);

/* The adapter-detection pre-pass's k-mer work (fq_kmer_* signatures, include/fqengine.h).  By
 * default it runs on the GPU; a host without a device (the CPU test suite) registers another
 * implementation here (NULL restores the GPU). */
typedef struct fqh_kmer_backend {
    int (*open)(int device, const uint8_t* seq, const uint32_t* off, int32_t n, void** out);
    int (*close)(void* set);
    int (*count)(void* set, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t* counts);
    int (*find)(void* set, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t seed, uint64_t* occ, size_t cap,
                size_t* n_out);
} fqh_kmer_backend;
void fqh_set_kmer_backend(const fqh_kmer_backend* b);

/* Records of a FASTQ file as the tool's pack reader parses them (bulk = 1: the zero-copy pack
 * reader, packs of `pack_n` records; bulk = 0: the line-by-line FqReader), with read buffers of
 * `buf_size` bytes instead of the reference's 1 MiB (tests cross-check both readers on buffer
 * boundaries).  Returns a malloc'd listing: one "name\tseq\tstrand\tqual\n" line per record,
 * then the reader's error text, if any (fqh_free). */
char* fqh_debug_records(const char* path, int bulk, int buf_size, int pack_n, int phred64);

/* The decompressed stream of gzip file `path` as the tool's parallel single-stream inflater hands
 * it out (chunks of `chunk` compressed bytes, 0 = default; `threads` decoding threads), and as zlib's
 * gzread gives it in calls of `call` bytes (the reference's reader).  *out: malloc'd bytes (fqh_free),
 * *ok: 0 when the stream ended on corrupt data.  fqh_pargz_read_all returns 1 for the parallel
 * path, 2 when it handed the stream to zlib's reader (an anomaly or several members), 0 when it does
 * not apply (small file, not gzip), -1 on error; fqh_gzread_all returns 0, -1 on error. */
int fqh_pargz_read_all(const char* path, size_t call, int threads, size_t chunk, char** out, size_t* n, int* ok);
int fqh_gzread_all(const char* path, size_t call, char** out, size_t* n, int* ok);
/* Speed probe: the same streams read in `call`-byte calls into one reused buffer and discarded (the
 * tool's reader copies each call into its arena the same way).  threads > 0: the parallel inflater
 * (returns as fqh_pargz_read_all); threads == 0: zlib's gzread (returns 0).  *n: bytes read,
 * *seconds: wall time of the reads. */
int fqh_gz_drain(const char* path, size_t call, int threads, size_t chunk, size_t* n, int* ok, double* seconds);

#ifdef __cplusplus
}
#endif

#endif /* FQHOST_H */
