/*
 * fqengine.h -- C-ABI drop-in boundary of the MI355X FASTQ preprocessing engine.
 *
 * The reference (Wsc000123/fqtool, a fastp fork) has no plugin/FFI API; its hot path is the
 * per-pack worker call
 *     bool PairEndProcessor::processPairEnd(ReadPairPack*, ThreadConfig*)
 *         (reference src/peprocessor.h:61, body src/peprocessor.cpp:261-508)
 *     void SingleEndProcessor::processSingleEnd(ReadPack*, ThreadConfig*)
 *         (reference src/seprocessor.cpp:290-388)
 * which mutates the reads of one pack in place and accumulates into the worker's
 * ThreadConfig (Stats x4 + FilterResult, src/threadconfig.cpp:3-20) and the processor's
 * insert-size histogram (src/peprocessor.cpp:510-523).
 *
 * This header replaces that seam with plain pointers and sizes (no C++ / torch types):
 *   - fq_params       : POD snapshot of every derived Options field the loop body reads
 *                        (src/options.h:15-386 after Options::update, src/options.cpp:24-58)
 *   - fq_batch        : one pack of reads as SoA uint8 seq/qual planes (chunk-interleaved
 *                        tiles, see below) + uint16 lengths
 *                        (replaces ReadPairPack / ReadPack, src/peprocessor.h:28-31)
 *   - fq_read_result  : per-read trim window + filter code + adapter/merge descriptors, i.e.
 *                        everything the in-place std::string mutations of the loop body produce
 *   - accumulator     : flat uint64 block = Stats x4 + FilterResult counters + insert histogram,
 *                        sum-reducible (RCCL ncclSum/ncclUint64 across GPUs)
 * Every entry point returns 0 on success and a negative FQ_E* code on failure; nothing
 * throws across the ABI. The engine never falls back to a CPU path: without a usable gfx950
 * device fq_engine_create fails with FQ_E_NO_DEVICE.
 */
#ifndef FQENGINE_H
#define FQENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FQ_ABI_VERSION 3

/* ---- status codes ------------------------------------------------------------------- */
#define FQ_OK 0
#define FQ_E_INVALID (-1)    /* bad argument / unsupported parameter combination           */
#define FQ_E_NO_DEVICE (-2)  /* no HIP device, or not gfx950                                */
#define FQ_E_HIP (-3)        /* a HIP runtime call failed (message in fq_engine_last_error)  */
#define FQ_E_TOO_LONG (-4)   /* a read is longer than the engine's configured max_cycles     */
#define FQ_E_NOMEM (-5)

/* ---- filter result codes: reference src/common.h:9-30 -------------------------------- */
#define FQ_PASS_FILTER 0
#define FQ_FAIL_POLY_X 4
#define FQ_FAIL_OVERLAP 8
#define FQ_FAIL_N_BASE 12
#define FQ_FAIL_LENGTH 16
#define FQ_FAIL_TOO_LONG 17
#define FQ_FAIL_QUALITY 20
#define FQ_FAIL_COMPLEXITY 24
#define FQ_FILTER_RESULT_TYPES 32

#define FQ_MAX_ADAPTER 128 /* longest --adapter_of_read{1,2} accepted                       */

/*
 * Derived options, already in the form the reference's loop body consumes them.
 * The host (fqtool_amd/host/options.cpp) fills this exactly as Options::update does,
 * including the reference quirks:
 *   - low_qual_limit already has +33 added (src/options.cpp:26),
 *   - low_qual_base_limit = int(lowQualityRatio * 151) (src/options.cpp:44 runs before the
 *     read-length evaluation, src/main.cpp:124-129),
 *   - polyg_* are the EFFECTIVE (compareReq, maxMismatch, oneMismatchPer) triple: the PE call
 *     at src/peprocessor.cpp:297 passes (maxMismatch, allowedOneMismatchForEach, minLen) into
 *     PolyX::trimPolyG(r1, r2, compareReq, maxMismatch, allowedOneMismatchForEach, fr)
 *     (src/polyx.h:28), the SE call at src/seprocessor.cpp:317 passes them in order.
 */
typedef struct fq_params {
    int32_t paired; /* 1 = PairEndProcessor, 0 = SingleEndProcessor */

    /* Filter::trimAndCut, src/filter.cpp:69-189 */
    int32_t trim_front1, trim_tail1, trim_front2, trim_tail2; /* -f -t -F -T */
    int32_t cut_front, cut_right, cut_tail;                   /* enable flags */
    int32_t cut_front_window, cut_right_window, cut_tail_window;
    int32_t cut_front_quality, cut_right_quality, cut_tail_quality; /* mean quality, no +33 */

    /* PolyX::trimPolyG, src/polyx.cpp:14-38 (effective argument order, see above) */
    int32_t polyg_enabled;
    int32_t polyg_compare_req, polyg_max_mismatch, polyg_one_mismatch_per;

    /* PolyX::trimPolyX, src/polyx.cpp:45-101 */
    int32_t polyx_enabled;
    int32_t polyx_mask; /* bit b set <=> base "ATCGN"[b] is in --base_to_trim */
    int32_t polyx_compare_req, polyx_max_mismatch, polyx_one_mismatch_per;

    /* adapters: src/peprocessor.cpp:301-326, src/seprocessor.cpp:321-323 */
    int32_t adapter_trimming; /* -a */
    int32_t adapter1_len, adapter2_len; /* 0 = not provided (adapterSeqR{1,2}Provided) */
    uint8_t adapter1[FQ_MAX_ADAPTER];
    uint8_t adapter2[FQ_MAX_ADAPTER];

    /* OverlapAnalysis::analyze, src/overlapanalysis.cpp:7-72 */
    int32_t overlap_diff_limit; /* --max_diff_for_overlap, default 5 */
    int32_t overlap_require;    /* --min_overlap_len, default 30 */
    int32_t insert_size_max;    /* 512, src/options.cpp:17 */

    /* -b / -B, src/peprocessor.cpp:342-349 */
    int32_t max_len1, max_len2;

    /* -m, src/peprocessor.cpp:351-385 */
    int32_t merge_enabled, discard_unmerged;

    /* Filter::passFilter, src/filter.cpp:3-52 */
    int32_t qual_filter_enabled;
    int32_t low_qual_limit;      /* -Q + 33 */
    int32_t low_qual_base_limit; /* int(-U * 151) */
    int32_t n_base_limit;        /* -N */
    double avg_qual_limit;       /* -e */
    int32_t length_filter_enabled, min_len, max_len; /* -l --min_length --max_length */
    int32_t complexity_enabled;  /* -y */
    double complexity_threshold; /* -Y */

    /* engine sizing */
    int32_t max_cycles; /* per-cycle Stats buffer length; reads longer than this are rejected */

    /* -c: BaseCorrector::correctByOverlapAnalysis (src/basecorrector.cpp:14-70), PE only, run
     * between the insert-size statistics and adapter trimming (src/peprocessor.cpp:310-312).
     * The engine corrects the bases/qualities of the DEVICE batch planes in place. */
    int32_t correction_enabled;
    /* -u with the UMI in the read (UmiProcessor::process, src/umiprocessor.cpp:10-79): after the
     * pre-filter statistics each mate loses min(umi_front, len - 1) leading bases
     * (Read::trimFront, src/read.h:203-208); 0 = no UMI trim.  The UMI tag itself only changes
     * the read names and is the host's business. */
    int32_t umi_front1, umi_front2;
    int32_t reserved[4];
} fq_params;

/* One pack of reads.  Each plane (seq1, qual1, seq2, qual2) holds every read's row of `stride`
 * bytes in CHUNK-INTERLEAVED TILES: reads are grouped in tiles of FQ_TILE_READS consecutive reads,
 * and inside a tile the 16-byte chunk k of all its reads is stored together, so
 *     byte j of read i  is at  plane[fq_batch_offset(stride, i, j)]
 *                          =  (i / 32) * 32 * stride + (j / 16) * 512 + (i % 32) * 16 + j % 16.
 * One wave-wide load of chunk k of 32 (or 64) reads is then one (or two) 512-byte contiguous runs
 * instead of 64 rows touched 16 bytes at a time.  A plane spans fq_batch_bytes(n, stride) bytes
 * (whole tiles; the padding rows are never read as reads).  Bytes j >= len[i] of a row are
 * ignored.  Packers: fq_batch_offset / fq_batch_put_row below. */
#define FQ_TILE_READS 32
#define FQ_CHUNK 16
typedef struct fq_batch {
    int32_t n;      /* number of pairs (PE) or reads (SE) */
    int32_t stride; /* bytes per row, multiple of 16, >= every len */
    const uint8_t* seq1;
    const uint8_t* qual1;
    const uint16_t* len1;
    const uint8_t* seq2; /* PE only, else NULL */
    const uint8_t* qual2;
    const uint16_t* len2;
    /* optional per-pair (per-read in SE) FQ_BF_* flags, n bytes; NULL = all zero */
    const uint8_t* flags;
} fq_batch;

/* fq_batch.flags: the pair (read) was dropped by Filter::filterByIndex
 * (src/filter.cpp:209-232, called at src/peprocessor.cpp:283 / src/seprocessor.cpp:304): only the
 * pre-filter statistics count it, its record carries FQ_RF_INDEX_FILTERED and nothing else. */
#define FQ_BF_INDEX_FILTERED 0x01

static inline size_t fq_batch_offset(int32_t stride, int64_t i, int32_t j) {
    return (size_t)(i / FQ_TILE_READS) * FQ_TILE_READS * (size_t)stride +
           (size_t)(j / FQ_CHUNK) * (FQ_TILE_READS * FQ_CHUNK) + (size_t)(i % FQ_TILE_READS) * FQ_CHUNK +
           (size_t)(j % FQ_CHUNK);
}
static inline size_t fq_batch_bytes(int64_t n, int32_t stride) {
    return (size_t)((n + FQ_TILE_READS - 1) / FQ_TILE_READS) * FQ_TILE_READS * (size_t)stride;
}
/* copy `len` bytes of `src` into read i's row of a plane (len <= stride) */
static inline void fq_batch_put_row(uint8_t* plane, int32_t stride, int64_t i, const uint8_t* src, int32_t len) {
    int32_t j;
    for (j = 0; j < len; j += FQ_CHUNK) {
        const int32_t m = len - j < FQ_CHUNK ? len - j : FQ_CHUNK;
        const size_t o = fq_batch_offset(stride, i, j);
        int32_t k;
        for (k = 0; k < m; ++k) plane[o + k] = src[j + k];
    }
}
/* copy read i's first `len` row bytes out of a plane */
static inline void fq_batch_get_row(const uint8_t* plane, int32_t stride, int64_t i, uint8_t* dst, int32_t len) {
    int32_t j;
    for (j = 0; j < len; j += FQ_CHUNK) {
        const int32_t m = len - j < FQ_CHUNK ? len - j : FQ_CHUNK;
        const size_t o = fq_batch_offset(stride, i, j);
        int32_t k;
        for (k = 0; k < m; ++k) dst[j + k] = plane[o + k];
    }
}

/* fq_read_result.flags */
#define FQ_RF_NULL 0x01      /* trimAndCut returned NULL (src/filter.cpp:78,100,124,160,183) */
#define FQ_RF_AD_OVERLAP 0x02 /* trimmed by AdapterTrimmer::trimByOverlapAnalysis */
#define FQ_RF_AD_SEQ 0x04    /* trimmed by AdapterTrimmer::trimBySequence */
#define FQ_RF_AD_NEG 0x08    /* trimBySequence matched at pos<0: recorded adapter = adapter[ad_pos:] */
#define FQ_RF_MERGED 0x10    /* (read-1 record) pair was merged (-m) */
#define FQ_RF_OVERLAP 0x20   /* (read-1 record) OverlapAnalysis reported overlapped for this pair */
#define FQ_RF_CORRECTED 0x40 /* -c corrected bases of this read (see fq_read_result) */
#define FQ_RF_INDEX_FILTERED 0x80 /* the pair/read was dropped by the index filter (FQ_BF_INDEX_FILTERED) */

/*
 * Everything the loop body's in-place std::string edits leave behind, per read (16 bytes).
 * The surviving read is original[start .. start+len).  For adapter bookkeeping
 * (FilterResult::addAdapterTrimmed, src/filterresult.cpp:138-177) the host rebuilds the
 * recorded adapter string from (ad_pos, ad_len): original[ad_pos .. ad_pos+ad_len), or, with
 * FQ_RF_AD_NEG, adapter[ad_pos .. ad_pos+ad_len).  For a merged pair (FQ_RF_MERGED, read-1
 * record) the merged read is r1[0:m_len1] + revcomp(r2)[ol : ol+m_len2] with ol = len2 - m_len2
 * (src/overlapanalysis.cpp:74-104); the read-1 record's code is the merged read's code.
 * Base correction (-c, FQ_RF_CORRECTED on either mate's record): the read-2 record carries the
 * correcting overlap, m_len1 = (int16_t) offset, m_len2 = overlap length, reserved = read 2's length
 * at correction time; both reads' windows start at their final `start`.  The corrected bytes are
 * those BaseCorrector::correctByOverlapAnalysis rewrites for that overlap (src/basecorrector.cpp:
 * 14-70), which a host re-applies to its copy of the text (fq_correct_pair_text below).
 */
typedef struct fq_read_result {
    uint16_t start;
    uint16_t len;
    uint8_t code;  /* Filter::passFilter result, FQ_PASS_FILTER ... */
    uint8_t flags; /* FQ_RF_* */
    uint16_t ad_pos;
    uint16_t ad_len;
    uint16_t m_len1;
    uint16_t m_len2;
    uint16_t reserved;
} fq_read_result;

/* util::complement, reference src/util.h:438-451 */
static inline char fq_complement(char c) {
    switch (c) {
        case 'A': case 'a': return 'T';
        case 'T': case 't': return 'A';
        case 'C': case 'c': return 'G';
        case 'G': case 'g': return 'C';
        default: return 'N';
    }
}

/* Re-applies the edits of BaseCorrector::correctByOverlapAnalysis (src/basecorrector.cpp:14-70)
 * for a FQ_RF_CORRECTED pair to a host copy of its text: s1/q1 = read 1 from its record's start,
 * s2/q2 = read 2 from its record's start, (offset, ol, len2) from the read-2 record
 * ((int16_t) m_len1, m_len2, reserved).  The engine took the same decisions on the device. */
static inline void fq_correct_pair_text(char* s1, char* q1, char* s2, char* q2, int offset, int ol, int len2) {
    const int start1 = offset > 0 ? offset : 0;
    const int start2 = len2 - (offset < 0 ? -offset : 0) - 1;
    const char good = (char)(33 + 30), bad = (char)(33 + 14); /* util::num2qual(30), (14) */
    int i;
    for (i = 0; i < ol; ++i) {
        const int p1 = start1 + i, p2 = start2 - i;
        if (s1[p1] == fq_complement(s2[p2])) continue;
        if ((signed char)q1[p1] >= good && (signed char)q2[p2] <= bad) {
            s2[p2] = fq_complement(s1[p1]);
            q2[p2] = q1[p1];
        } else if ((signed char)q2[p2] >= good && (signed char)q1[p1] <= bad) {
            s1[p1] = fq_complement(s2[p2]);
            q1[p1] = q2[p2];
        }
    }
}

/*
 * Flat accumulator (uint64 words).  Layout (indices into the uint64 array):
 *   FQ_ACC_FILTER + code          FilterResult::mFilterReadStats[32]
 *   FQ_ACC_ADAPTER_READS/BASES    FilterResult::mTrimmedAdapterReads/Bases
 *   FQ_ACC_POLYX_READS + b        FilterResult::mTrimmedPolyXReads[5]  (b in A,T,C,G,N order)
 *   FQ_ACC_POLYX_BASES + b        FilterResult::mTrimmedPolyXBases[5]
 *   FQ_ACC_MERGED_PAIRS           ThreadConfig::addMergedPairs
 *   FQ_ACC_INSERT + isize         PairEndProcessor::mInsertSizeHist[insert_size_max + 1]
 *   fq_acc_stats_offset(k)        Stats block k in {0 pre-R1, 1 pre-R2, 2 post-R1, 3 post-R2}:
 *        +FQ_ST_READS, +FQ_ST_LENGTH_SUM, +FQ_ST_Q20, +FQ_ST_Q30 then, from +FQ_ST_CYCLES,
 *        [max_cycles][16] = per cycle 8 base-class counts (mCycleBaseContents[b][c], b = byte&7)
 *        followed by 8 base-class quality sums (mCycleBaseQuality[b][c]).
 *   fq_acc_tail_offset + FQ_ACC_TAIL_*  the -c counters.
 * All counters are sums, so N engines (GPUs) combine by element-wise uint64 addition.
 */
#define FQ_ACC_FILTER 0
#define FQ_ACC_ADAPTER_READS 32
#define FQ_ACC_ADAPTER_BASES 33
#define FQ_ACC_POLYX_READS 34
#define FQ_ACC_POLYX_BASES 39
#define FQ_ACC_MERGED_PAIRS 44
#define FQ_ACC_INSERT 48
/* after the four Stats blocks (fq_acc_tail_offset): -c counters */
#define FQ_ACC_TAIL_CORRECTED_READS 0 /* FilterResult::mCorrectedReads                        */
#define FQ_ACC_TAIL_CORRECTED_BASES 1 /* sum of FilterResult::mCorrectionMatrix (CorrectedBases) */
#define FQ_ACC_TAIL_WORDS 16
#define FQ_ST_READS 0
#define FQ_ST_LENGTH_SUM 1
#define FQ_ST_Q20 2
#define FQ_ST_Q30 3
#define FQ_ST_CYCLES 16
#define FQ_ST_PER_CYCLE 16

static inline size_t fq_acc_stats_words(int32_t max_cycles) {
    return (size_t)FQ_ST_CYCLES + (size_t)max_cycles * FQ_ST_PER_CYCLE;
}
static inline size_t fq_acc_stats_offset(int32_t insert_size_max, int32_t max_cycles, int k) {
    size_t base = (size_t)FQ_ACC_INSERT + (size_t)(insert_size_max + 1);
    base = (base + 15) & ~(size_t)15;
    return base + (size_t)k * fq_acc_stats_words(max_cycles);
}
static inline size_t fq_acc_tail_offset(int32_t insert_size_max, int32_t max_cycles) {
    return fq_acc_stats_offset(insert_size_max, max_cycles, 4);
}
static inline size_t fq_acc_words(int32_t insert_size_max, int32_t max_cycles) {
    return fq_acc_tail_offset(insert_size_max, max_cycles) + FQ_ACC_TAIL_WORDS;
}

/* ---- engine ------------------------------------------------------------------------- */
typedef struct fq_engine fq_engine;

/* fq_engine_create: validates params, selects `device` (hipSetDevice), allocates the device
 * accumulator and staging buffers for packs of up to max_batch reads/pairs with rows of up to
 * max_stride bytes.  Fails with FQ_E_NO_DEVICE when no gfx950 device is present. */
int fq_engine_create(const fq_params* params, int device, int32_t max_batch, int32_t max_stride,
                     fq_engine** out);
int fq_engine_destroy(fq_engine* e);

/* Host-memory pack (the CLI path): H2D copy, kernels, D2H of the per-read results.
 * `results` has n entries (SE) or 2n entries (PE: [2i] = read 1, [2i+1] = read 2).
 * Synchronous; replaces one call of processPairEnd / processSingleEnd. */
int fq_engine_process(fq_engine* e, const fq_batch* host_batch, fq_read_result* results);

/* Device-resident pack (inputs already in HBM): enqueues the kernels on `stream`
 * (a hipStream_t; NULL = the HIP default stream) and returns without synchronising.
 * `device_results` may be NULL when the caller needs only the accumulators.
 * The engine's hand-off list (pairs / reads the fast kernels pass to the general kernel) is
 * shared by these calls: use one stream at a time per engine (concurrent streams need one
 * engine each). */
int fq_engine_process_device(fq_engine* e, const fq_batch* device_batch,
                             fq_read_result* device_results, void* stream);

/* ---- asynchronous host-pack pipeline ---------------------------------------------------
 * Replaces the reference's concurrent workers over disjoint packs (consumePack on -w threads,
 * src/peprocessor.cpp:546-566) with an in-order device pipeline per engine:
 * fq_engine_submit enqueues one host pack -- H2D on a copy-in stream, the kernels on the compute
 * stream, D2H of its records into `results` on a copy-out stream -- and returns without waiting.
 * Up to 3 packs are in flight per engine (a further submit first waits for the oldest pack's
 * device slot to drain).  The host batch arrays and `results` must stay valid and untouched
 * until fq_engine_poll has reported `seq_no`.  With pinned host memory (fq_host_alloc) pack
 * k+1's H2D overlaps pack k's kernels and pack k-1's D2H.
 * fq_engine_poll reports packs in submission order: it returns 1 and sets *seq_no when the
 * oldest pending pack is complete (its records are in its `results`), 0 when nothing is pending
 * or (wait == 0) the oldest pack is still running, and a negative FQ_E_* code on failure.
 * One thread submits and polls a given engine; fq_engine_process must not be mixed with
 * packs still pending. */
int fq_engine_submit(fq_engine* e, const fq_batch* host_batch, fq_read_result* results, uint64_t seq_no);
int fq_engine_poll(fq_engine* e, int wait, uint64_t* seq_no);
int fq_engine_pending(const fq_engine* e); /* packs submitted and not yet reported */

/* ---- FASTQ-text packs: GPU-side ingest and egress ------------------------------------------
 * Replaces the host's tile packing and output formatting (Read::toString + the writers' input,
 * src/read.h:166-168, src/peprocessor.cpp:457-491, src/seprocessor.cpp:337-350) for the plain
 * output case: the pack's records go over as the bytes of the input FASTQ (a span of the mapped
 * file or of the read arena, pageable or pinned) plus one fq_text_rec per record; the device builds
 * the tiled batch planes from the text, runs the pack's kernels, and writes the output FASTQ text
 * of the records that pass (both mates of a pair for PE, to out1 / out2, in input order, each
 * record "name\nseq[start, start+len)\nstrand\nqual[start, start+len)\n" as the reference writes
 * it) into `out`.  With -m (merge_enabled, PE, no --discard_unmerged) every pair's output is the
 * merged stream (src/peprocessor.cpp:351-385: the merged read, name "_merged_<m1>_<m2>" spliced in
 * before the first space, when it merged and passes; otherwise each read that passes), written to
 * out->text[0] (which must then hold text_bytes[0] + text_bytes[1] + 24 * n + 16 bytes), and
 * out->bytes[1] is 0.  Only for options whose outputs are out1 (+ out2) or that merged stream: no
 * -c, UMI, index filter, phred64, split, failed or unpaired outputs, no --discard_unmerged; the
 * host routes everything else through fq_engine_submit.  Records and text must stay valid until fq_engine_poll reports the pack; then
 * `results` holds the records as from fq_engine_submit and out->bytes[m] the bytes of out->text[m].
 * out->text[m] must hold at least the mate's text_bytes + 16 (a record's output is never longer
 * than its input text, except by the final line terminator that the input may lack). */
typedef struct fq_text_rec {
    uint32_t name_off;   /* offsets from the mate's text pointer: the name line (without its terminator), */
    uint32_t seq_off;    /* the sequence, */
    uint32_t strand_off; /* the strand line, */
    uint32_t qual_off;   /* the quality line */
    uint16_t name_len, strand_len, len, pad;
} fq_text_rec;
typedef struct fq_text_batch {
    int32_t n;      /* records (PE: pairs) */
    int32_t stride; /* row stride of the planes the device builds (multiple of 16, >= every len) */
    const char* text[2];
    uint64_t text_bytes[2];
    const fq_text_rec* rec[2]; /* rec[1]: PE only */
} fq_text_batch;
typedef struct fq_text_out {
    char* text[2];      /* host buffers (pinned for full speed) of at least text_bytes[m] */
    uint64_t bytes[2];  /* set when the pack is reported by fq_engine_poll */
} fq_text_out;
int fq_engine_submit_text(fq_engine* e, const fq_text_batch* tb, fq_read_result* results, fq_text_out* out,
                          uint64_t seq_no);

/* ---- raw FASTQ streams: record indexing on the GPU ------------------------------------------
 * Replaces the reader too (FqReader::read over its 1 MiB buffers and FqReaderPair::read,
 * src/fqreader.cpp:90-195, :254-267) for the plain part of an input, on top of the text-pack
 * path above.  The caller hands each mate's input bytes over in consecutive windows of any size
 * (fq_engine_raw_enqueue; page-locked or registered host memory, fq_host_register, makes the copy
 * asynchronous).  On the device each window's text is the previous window's bytes after its last
 * taken record followed by the new bytes; the line terminators ('\n' and '\r') are indexed and
 * record i is lines 4i .. 4i+3 while records are "plain": all four lines end in '\n' and are
 * non-empty, the first starts with '@', quality and sequence are equally long, name/strand lines
 * are < 65536 bytes and the sequence <= the engine's max_stride and max_cycles.  On plain records
 * the reference reader is exactly "four lines per record" (no '@' search, no "\r\n" folding at its
 * buffer ends, no length error).  A window's pack is the leading plain records (PE: pairs, the
 * minimum over the mates), up to max_batch; fq_engine_raw_launch runs it as a text pack.
 *   fq_raw_result.stop != 0: a complete record that is not plain follows the pack (or the carry
 *   overflowed): the caller continues with its own reader at each mate's stream offset
 *   (end of the window's bytes) - carry[m].  The same applies when the input ended (every mate's
 *   last window enqueued) with carry left, or a window takes no pairs.
 * Protocol: fq_engine_raw_begin; enqueue window 0; then for k = 0, 1, ...: enqueue window k+1
 * (optional), fq_engine_raw_launch (window k: waits for its index), poll as for other packs.  At
 * most three windows are enqueued and not launched, and eight windows are in the engine (enqueued,
 * launched or not yet polled: a ninth enqueue waits for the oldest pack's copies); a window's
 * host bytes must stay valid until its pack is reported by fq_engine_poll.  Options as for text
 * packs (-m writes the merged stream into out->text.text[0], which must then hold both mates' window
 * and carry bytes + 28 * max_batch + 64; no -c, UMI, index filter, --discard_unmerged).
 * The trimmed-adapter strings (FilterResult::addAdapterTrimmed, src/filterresult.cpp:138-157) come
 * back after the output text, at out->text.text[m] + out->text.bytes[m], adapter_bytes[m] bytes of
 * entries "u16 ad_len (little endian), u8 neg, then ad_len bytes of the read (neg 0) or u16
 * ad_pos (neg 1: the string is adapter[ad_pos, ad_pos + ad_len) of the mate's adapter parameter)";
 * one copy back per mate, of the pack's text_bytes[m] + 3 * pairs + 16 bytes (a record's output
 * plus its entry is at most its input + 3 bytes).
 * Several engines on one GPU (one PCIe link): a window's host-to-device copies wait for the last
 * ones any other engine of the process enqueued on that device, and a pack's copies back likewise,
 * so copies run one after another in call order at the link's full rate; a caller dealing one
 * stream's windows over such engines enqueues (and launches) them in stream order.  Engines on
 * different GPUs never wait for each other. */
typedef struct fq_raw_window {
    const char* bytes[2]; /* mate m's next input bytes (bytes[1]: PE only) */
    uint64_t n[2];        /* their count, <= the window capacity given to fq_engine_raw_begin */
} fq_raw_window;
typedef struct fq_raw_result {
    int32_t pairs;      /* records (PE: pairs) in the window's pack */
    int32_t stop;       /* nonzero: the GPU path cannot continue after this pack (see above) */
    int32_t max_len;    /* longest sequence of the pack */
    int32_t pad;
    uint64_t carry[2];  /* mate m's bytes after the pack's last record (they stay on the device) */
    uint64_t text_bytes[2]; /* mate m's text bytes the pack's records span */
} fq_raw_result;
typedef struct fq_raw_out {
    fq_text_out text;          /* text[m]: >= carry capacity + window bytes + 4 * max_batch + 16 */
    uint64_t adapter_bytes[2]; /* set by fq_engine_poll: entries after the output text */
    /* Records-only egress (all set, or all null): instead of the output text the pack's records
     * come back -- results[2i + m] (PE) / results[i] as from fq_engine_submit, and rec[m][i] the
     * record's line offsets in the window buffer [carry capacity - carry | window bytes] (the
     * window's bytes at offset carry capacity, the previous pack's unconsumed bytes just before),
     * so a caller that kept its page-locked window bytes (and the carry in front of them) formats
     * the output itself; text.bytes and adapter_bytes are 0.  80 bytes per pair cross PCIe instead
     * of the ~input-sized text. */
    fq_read_result* results;   /* >= pairs * 2 (PE) / reads */
    fq_text_rec* rec[2];       /* >= max_batch each (rec[1]: PE) */
} fq_raw_out;
int fq_engine_raw_begin(fq_engine* e, uint64_t window_cap, uint64_t carry_cap);
int fq_engine_raw_enqueue(fq_engine* e, const fq_raw_window* w);
int fq_engine_raw_launch(fq_engine* e, fq_raw_result* r, fq_raw_out* out, uint64_t seq_no);
/* Waits until the oldest enqueued (not launched) window is indexed and reports its pack's pairs,
 * stop, carry and text bytes as fq_engine_raw_launch of it will (r may be null); that launch then
 * does not wait.  A caller ordering launches over several engines waits here, on each engine's own
 * thread, before it takes its turn (no counterpart in the reference: its reader is one thread). */
int fq_engine_raw_wait(fq_engine* e, fq_raw_result* r);
/* Leaves raw mode: waits for the copies and indexing of windows enqueued and never launched (their
 * host bytes may then be reused) and drops them; launched packs are polled as usual.  The engine
 * takes other packs, or a new fq_engine_raw_begin once nothing is in flight. */
int fq_engine_raw_end(fq_engine* e);

/* Page-locked host memory for packs and records (portable across devices; transparent huge
 * pages registered with the runtime, hipHostMalloc as fallback).  FQ_E_NO_DEVICE without a HIP
 * device: callers then use ordinary memory. */
int fq_host_alloc(size_t bytes, void** out);
int fq_host_free(void* p);
/* Page-lock an existing host range (e.g. of a read-only file mapping, page-aligned) so copies
 * from it are asynchronous DMA; fq_host_unregister releases it. */
int fq_host_register(const void* p, size_t bytes);
int fq_host_unregister(const void* p);

/* Accumulators */
size_t fq_engine_acc_words(const fq_engine* e);
int fq_engine_acc_device_ptr(fq_engine* e, uint64_t** dptr); /* for an RCCL all-reduce */
int fq_engine_read_acc(fq_engine* e, uint64_t* host_acc, size_t words);
/* Use a caller-owned, zero-initialised device buffer of fq_engine_acc_words() uint64 words as
 * the accumulator (e.g. a torch tensor that is then all-reduced over RCCL); NULL restores the
 * engine's own buffer. */
int fq_engine_set_acc_buffer(fq_engine* e, uint64_t* device_acc);
int fq_engine_reset_acc(fq_engine* e);
int fq_engine_sync(fq_engine* e);

/* Last error message of this engine (or of the last failed create when e == NULL). */
const char* fq_engine_last_error(const fq_engine* e);

/* Device id the engine runs on; gfx arch name of that device. */
int fq_engine_device_info(const fq_engine* e, int* device, char* arch, size_t arch_len);

/* ---- synthetic workload ------------------------------------------------ *
 * Fills a device-resident PE (seq2 != NULL) or SE batch with the seeded synthetic reads of
 * the benchmark configs: counter-based (splitmix64 keyed on seed and global read index), so
 * shards generate independently; `first_index` is the global index of the batch's first
 * pair/read.  Lengths are written too.  Asynchronous on `stream`. */
int fq_synth_fill_device(const fq_batch* device_batch, uint64_t seed, uint64_t first_index,
                         int32_t read_len, void* stream);

/* ---- duplication analysis (-d) ----------------------------------------------------------
 * Duplicate::statRead / statPair / statAll, reference src/duplicate.cpp:46-166.  A table lives
 * on one device and outlives engines (the tool re-creates engines when reads grow); an engine
 * with a table attached adds every later pack's reads to it, on its compute stream, in input
 * order (packs are ordered by their seq_no; fq_engine_process / process_device use a per-engine
 * call counter).  Tables of engines that processed interleaved packs of one input merge exactly
 * (fq_dup_merge), since each key remembers the order of its first read.  fq_dup_stat returns
 * statAll's histogram and GC sums (hist_size bins; a key seen more than hist_size times counts in
 * the last bin; exactly hist_size lands past the reference's array and is not reported) and
 * totals[0] = reads counted, totals[1] = duplicates (Rate = totals[1] / totals[0]). */
typedef struct fq_dup fq_dup;
int fq_dup_create(int device, int32_t keylen, fq_dup** out); /* keylen 1..31 (-dup_ana_key_len) */
int fq_dup_destroy(fq_dup* d);
int fq_dup_reset(fq_dup* d);
int fq_engine_set_dup(fq_engine* e, fq_dup* d); /* NULL detaches; d must be on the engine's device */
int fq_dup_merge(fq_dup* dst, const fq_dup* src);
int fq_dup_stat(fq_dup* d, int32_t hist_size, uint64_t* hist, uint64_t* gc_sum, uint64_t* totals);

/* ---- adapter-detection k-mers (Evaluator::evaluateAdapterSeq, src/evaluator.cpp:229-426) ------
 * A read set uploaded once (read i = seq[off[i] .. off[i+1]), n + 1 offsets).  For every read,
 * every window [pos, pos + keylen) of uppercase A/C/G/T bases with
 * first <= pos <= len - keylen - shift_tail is one k-mer (key = 2-bit codes A0 T1 C2 G3, first
 * base most significant, as Evaluator::seq2int).  fq_kmer_count fills counts[4^keylen];
 * fq_kmer_find lists where `seed` occurs as (read << 32 | pos), in no particular order, up to
 * cap entries (*n_out = all occurrences). */
typedef struct fq_kmer_set fq_kmer_set;
int fq_kmer_open(int device, const uint8_t* seq, const uint32_t* off, int32_t n, fq_kmer_set** out);
int fq_kmer_close(fq_kmer_set* s);
int fq_kmer_count(fq_kmer_set* s, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t* counts);
int fq_kmer_find(fq_kmer_set* s, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t seed, uint64_t* occ,
                 size_t cap, size_t* n_out);

/* Kernel timing of the engine's last process_device call (HIP events on the launch stream),
 * in milliseconds; 0 when unavailable. */
double fq_engine_last_kernel_ms(const fq_engine* e);

#ifdef __cplusplus
}
#endif
#endif /* FQENGINE_H */
