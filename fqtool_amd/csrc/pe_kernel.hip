// pe_kernel.hip -- the per-pack hot path on gfx950.
//
// One lane owns one pair (PE) or one read (SE) and runs the loop body of
// PairEndProcessor::processPairEnd (reference src/peprocessor.cpp:261-508) /
// SingleEndProcessor::processSingleEnd (src/seprocessor.cpp:290-388) on read *views* over the
// batch rows in HBM (chunk-interleaved tiles, include/fqengine.h); trimming only moves (start, len), nothing is copied.
//
// Accumulation (the ThreadConfig-owned Stats x4 + FilterResult and the insert histogram):
// every workgroup privatises all counters in LDS and flushes them once with 64-bit global
// atomics.  The per-cycle Stats histograms are [stats][cycle][17] u32 (8 base-class counts +
// 8 base-class quality sums biased by +128 so partial sums never go negative, padded to 17
// words so consecutive cycles land on different banks); each lane walks its read starting at a
// lane-dependent rotation, so the 64 lanes of a wave update 64 different cycles per step.
#include <hip/hip_runtime.h>

#include "device_ops.h"
#include "engine_internal.h"

using namespace fqdev;

namespace {

constexpr int kRec = 17;  // LDS words per (stats, cycle) record

struct Smem {
    uint32_t* hist;         // [4][clds][17]
    unsigned long long* c;  // small u64 counters, indexed like the global accumulator head
    unsigned long long* scal;  // [4][4] reads, length_sum, q20, q30
    unsigned long long* tail;  // [4] the accumulator's tail counters (-c)
    int clds;                  // cycles privatised in LDS; later cycles go to global atomics
    unsigned long long* gcyc;  // global per-cycle block of stats 0 (+ k * stats words)
    size_t gstride;            // u64 words between the stats blocks
};

// u32 LDS words of the small u64 counters: head (even count), 16 Stats scalars, 4 tail counters
__host__ __device__ inline int small_words(const fq_params& p) {
    const int nsmall = FQ_ACC_INSERT + p.insert_size_max + 1;
    return 2 * (((nsmall + 1) & ~1) + 16 + 4);
}

// cycles the LDS histograms can hold next to the small counters
__host__ __device__ inline int lds_cycles(const fq_params& p) {
    const int cap = (160 * 1024 / 4 - small_words(p)) / (4 * kRec);
    return p.max_cycles < cap ? p.max_cycles : cap;
}

__device__ __forceinline__ void lds_add64(unsigned long long* p, unsigned long long v) { atomicAdd(p, v); }

// Stats::statRead, reference src/stats.cpp:237-295, on a window of a row (cycle i = data[i]).
template <typename Fetch>
__device__ inline void stat_read(const Smem& sm, int k, int len, int skew, Fetch fetch) {
    uint32_t* hist = sm.hist + (size_t)k * sm.clds * kRec;
    unsigned long long* scal = sm.scal + 4 * k;
    if (len <= 0) {
        lds_add64(&scal[0], 1ull);
        return;
    }
    int rot = skew % len;
    uint32_t q20 = 0, q30 = 0;
    for (int i = 0; i < len; ++i) {
        int c = i + rot;
        if (c >= len) c -= len;
        uint8_t b;
        int q;
        fetch(c, b, q);
        const int cls = b & 7;
        q20 += q > '5';
        q30 += q > '?';
        if (c < sm.clds) {
            uint32_t* rec = hist + c * kRec;
            atomicAdd(&rec[cls], 1u);
            atomicAdd(&rec[8 + cls], (uint32_t)(q + 128));
        } else {  // reads longer than the LDS histograms (merged long reads): straight to HBM
            unsigned long long* g = sm.gcyc + k * sm.gstride + (size_t)c * FQ_ST_PER_CYCLE;
            atomicAdd(&g[cls], 1ull);
            atomicAdd(&g[8 + cls], (unsigned long long)(long long)(q - 33));
        }
    }
    lds_add64(&scal[0], 1ull);
    lds_add64(&scal[1], (unsigned long long)len);
    lds_add64(&scal[2], (unsigned long long)q20);
    lds_add64(&scal[3], (unsigned long long)q30);
}

__device__ __forceinline__ void row_stat(const Smem& sm, int k, int C, Row s, Row q, int len, int skew) {
    (void)C;
    stat_read(sm, k, len, skew, [&](int i, uint8_t& b, int& qq) {
        b = s[i];
        qq = qv(q, i);
    });
}

__device__ __forceinline__ void store_result(fq_read_result* out, const fq_read_result& r) {
    *reinterpret_cast<uint4*>(out) = *reinterpret_cast<const uint4*>(&r);
}

__device__ __forceinline__ fq_read_result make_result(bool nonnull, int start, int len) {
    fq_read_result r;
    r.start = nonnull ? (uint16_t)start : 0;
    r.len = nonnull ? (uint16_t)len : 0;
    r.code = 0;
    r.flags = nonnull ? 0 : FQ_RF_NULL;
    r.ad_pos = r.ad_len = r.m_len1 = r.m_len2 = r.reserved = 0;
    return r;
}

__device__ inline void apply_polyg(const fq_params& p, const Smem& sm, Row s, int st, int& n) {
    int bases;
    n = trim_polyg(s + st, n, p.polyg_compare_req, p.polyg_max_mismatch, p.polyg_one_mismatch_per, bases);
    if (bases >= 0) {
        lds_add64(&sm.c[FQ_ACC_POLYX_READS + 3], 1ull);
        lds_add64(&sm.c[FQ_ACC_POLYX_BASES + 3], (unsigned long long)(long long)bases);
    }
}

__device__ inline void apply_polyx(const fq_params& p, const Smem& sm, Row s, int st, int& n) {
    int poly, bases;
    n = trim_polyx(s + st, n, p.polyx_mask, p.polyx_compare_req, p.polyx_max_mismatch, p.polyx_one_mismatch_per,
                   poly, bases);
    if (poly >= 0) {
        lds_add64(&sm.c[FQ_ACC_POLYX_READS + poly], 1ull);
        lds_add64(&sm.c[FQ_ACC_POLYX_BASES + poly], (unsigned long long)(long long)bases);
    }
}

__device__ inline void apply_adapter_seq(const Smem& sm, Row s, int st, int& n, const uint8_t* ad,
                                         int alen, fq_read_result& rr) {
    int pos;
    if (!trim_by_sequence(s + st, n, ad, alen, pos)) return;
    int ad_len;
    if (pos < 0) {
        ad_len = alen + pos;
        rr.flags |= FQ_RF_AD_SEQ | FQ_RF_AD_NEG;
        rr.ad_pos = (uint16_t)(-pos);
        n = 0;
    } else {
        ad_len = n - pos;
        rr.flags |= FQ_RF_AD_SEQ;
        rr.ad_pos = (uint16_t)(st + pos);
        n = pos;
    }
    rr.ad_len = (uint16_t)ad_len;
    if (ad_len > 0) {  // FilterResult::addAdapterTrimmed(str, isR2), src/filterresult.cpp:138-157
        lds_add64(&sm.c[FQ_ACC_ADAPTER_READS], 1ull);
        lds_add64(&sm.c[FQ_ACC_ADAPTER_BASES], (unsigned long long)ad_len);
    }
}

// writable byte i of a batch row (the device planes are the engine's own copy; -c edits them)
__device__ __forceinline__ uint8_t* row_ptr(Row r, int i) {
    const int j = r.off + i;
    return const_cast<uint8_t*>(r.base) + (j >> 4) * (FQ_TILE_READS * FQ_CHUNK) + (j & 15);
}

// BaseCorrector::correctByOverlapAnalysis, reference src/basecorrector.cpp:14-70: mismatches of the
// overlap where one side is >= Q30 and the other <= Q14 take the good side's base (complemented)
// and quality.  Applied to the rows in place, so every later step (adapter by sequence, polyX,
// merge, passFilter, post statistics) sees the corrected read as the reference does.  The
// FilterResult correction matrix is reported only through its sum (CorrectedBases).
__device__ inline void correct_pair(const Smem& sm, Row s1, Row q1, Row s2, Row q2, int n2, const Overlap& ov,
                                    fq_read_result& r1, fq_read_result& r2) {
    if (ov.diff == 0 || ov.diff > 5) return;
    const int ol = ov.len;
    const int start1 = max(0, ov.offset);
    const int start2 = n2 - max(0, -ov.offset) - 1;
    const int good = 33 + 30, bad = 33 + 14;  // util::num2qual(30), util::num2qual(14)
    int corrected = 0;
    bool c1 = false, c2 = false;
    for (int i = 0; i < ol; ++i) {
        const int p1 = start1 + i, p2 = start2 - i;
        const uint8_t b1 = s1[p1], b2 = s2[p2];
        if (b1 == comp(b2)) continue;
        const int x1 = qv(q1, p1), x2 = qv(q2, p2);
        if (x1 >= good && x2 <= bad) {
            *row_ptr(s2, p2) = comp(b1);
            *row_ptr(q2, p2) = (uint8_t)x1;
            ++corrected;
            c2 = true;
        } else if (x2 >= good && x1 <= bad) {
            *row_ptr(s1, p1) = comp(b2);
            *row_ptr(q1, p1) = (uint8_t)x2;
            ++corrected;
            c1 = true;
        }
    }
    if (!corrected) return;
    lds_add64(&sm.tail[FQ_ACC_TAIL_CORRECTED_READS], (c1 && c2) ? 2ull : 1ull);
    lds_add64(&sm.tail[FQ_ACC_TAIL_CORRECTED_BASES], (unsigned long long)corrected);
    if (c1) r1.flags |= FQ_RF_CORRECTED;
    if (c2) r2.flags |= FQ_RF_CORRECTED;
    // (a signed 16-bit offset is exact: fq_engine_create caps max_cycles at 4096, and longer reads are
    // refused per pack with FQ_E_TOO_LONG before any kernel sees them as in range)
    static_assert(FQ_MAX_CYCLES_LIMIT <= 32767, "-c carries the overlap offset in 16 signed bits");
    r2.m_len1 = (uint16_t)(int16_t)ov.offset;
    r2.m_len2 = (uint16_t)ol;
    r2.reserved = (uint16_t)n2;
}

// Read::trimFront(umi length + skip) of UmiProcessor::process (src/umiprocessor.cpp:28-62,
// src/read.h:203-208): min(k, len - 1) bases (a read of length 0 is left alone)
__device__ __forceinline__ int umi_cut(int k, int len) { return (k > 0 && len > 0) ? min(k, len - 1) : 0; }

__device__ __forceinline__ fq_read_result index_filtered_result() {
    fq_read_result r = make_result(true, 0, 0);
    r.flags = FQ_RF_INDEX_FILTERED;
    return r;
}

template <bool PAIRED>
__global__ void __launch_bounds__(kPackThreads) fq_pack_kernel(fq_params p, fq_batch b, fq_read_result* __restrict__ res,
                                                      unsigned long long* __restrict__ acc, int* __restrict__ err,
                                                      const int* __restrict__ tiles, const int* __restrict__ ntiles) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int C = p.max_cycles;
    const int nsmall = FQ_ACC_INSERT + p.insert_size_max + 1;
    Smem sm;
    sm.c = reinterpret_cast<unsigned long long*>(lds);
    sm.scal = sm.c + ((nsmall + 1) & ~1);
    sm.tail = sm.scal + 16;
    sm.hist = reinterpret_cast<uint32_t*>(sm.tail + 4);
    sm.clds = lds_cycles(p);
    sm.gstride = acc_stats_words(C);
    sm.gcyc = acc + acc_stats_offset(p.insert_size_max, C, 0) + FQ_ST_CYCLES;
    const int total_words = small_words(p) + 4 * sm.clds * kRec;
    for (int i = threadIdx.x; i < total_words; i += blockDim.x) lds[i] = 0;
    __syncthreads();

    const int skew = threadIdx.x & 63;
    // all pairs of the pack, or (item-list mode) the pairs / single-end reads the fast kernel
    // handed over, one index each
    const int total = tiles ? *ntiles : b.n;
    for (int item = blockIdx.x * blockDim.x + threadIdx.x; item < total; item += gridDim.x * blockDim.x) {
        const int idx = tiles ? tiles[item] : item;
        if (idx >= b.n) continue;
        const Row s1 = batch_row(b.seq1, b.stride, idx);
        const Row q1 = batch_row(b.qual1, b.stride, idx);
        const int l1 = b.len1[idx];
        if (!PAIRED) {
            if (l1 > C || l1 > b.stride) {
                atomicOr(err, 1);
                continue;
            }
            row_stat(sm, 0, C, s1, q1, l1, skew);  // src/seprocessor.cpp:298
            if (b.flags && (b.flags[idx] & FQ_BF_INDEX_FILTERED)) {  // :304-307
                if (res) store_result(&res[idx], index_filtered_result());
                continue;
            }
            const int u = umi_cut(p.umi_front1, l1);  // :309-311
            int st = 0, n = 0;
            bool nn = trim_and_cut(p, s1 + u, q1 + u, l1 - u, p.trim_front1, p.trim_tail1, st, n);
            st += u;
            fq_read_result rr = make_result(nn, st, n);
            if (nn && p.polyg_enabled) apply_polyg(p, sm, s1, st, n);
            if (nn && p.adapter_trimming && p.adapter1_len > 0) apply_adapter_seq(sm, s1, st, n, p.adapter1, p.adapter1_len, rr);
            if (nn && p.polyx_enabled) apply_polyx(p, sm, s1, st, n);
            if (nn && p.max_len1 > 0 && p.max_len1 < n) n = p.max_len1;
            const int code = pass_filter(p, s1 + st, q1 + st, n, !nn);
            lds_add64(&sm.c[FQ_ACC_FILTER + code], 1ull);
            if (nn && code == FQ_PASS_FILTER) row_stat(sm, 2, C, s1 + st, q1 + st, n, skew);
            rr.start = nn ? (uint16_t)st : 0;
            rr.len = nn ? (uint16_t)n : 0;
            rr.code = (uint8_t)code;
            if (res) store_result(&res[idx], rr);
            continue;
        }
        const Row s2 = batch_row(b.seq2, b.stride, idx);
        const Row q2 = batch_row(b.qual2, b.stride, idx);
        const int l2 = b.len2[idx];
        if (l1 > C || l2 > C || l1 > b.stride || l2 > b.stride) {
            atomicOr(err, 1);
            continue;
        }
        row_stat(sm, 0, C, s1, q1, l1, skew);  // src/peprocessor.cpp:276-277
        row_stat(sm, 1, C, s2, q2, l2, skew);
        if (b.flags && (b.flags[idx] & FQ_BF_INDEX_FILTERED)) {  // :283-286
            if (res) {
                store_result(&res[2 * (size_t)idx], index_filtered_result());
                store_result(&res[2 * (size_t)idx + 1], index_filtered_result());
            }
            continue;
        }
        const int u1 = umi_cut(p.umi_front1, l1), u2 = umi_cut(p.umi_front2, l2);  // :288-290
        int st1 = 0, n1 = 0, st2 = 0, n2 = 0;  // :292-293
        const bool nn1 = trim_and_cut(p, s1 + u1, q1 + u1, l1 - u1, p.trim_front1, p.trim_tail1, st1, n1);
        const bool nn2 = trim_and_cut(p, s2 + u2, q2 + u2, l2 - u2, p.trim_front2, p.trim_tail2, st2, n2);
        st1 += u1;
        st2 += u2;
        fq_read_result r1 = make_result(nn1, st1, n1), r2 = make_result(nn2, st2, n2);
        const bool both = nn1 && nn2;
        if (both && p.polyg_enabled) {  // :295-299
            apply_polyg(p, sm, s1, st1, n1);
            apply_polyg(p, sm, s2, st2, n2);
        }
        if (both) {  // :302-333 -- insert size for every pair (reference with -w 1)
            Overlap ov = analyze(s1 + st1, n1, s2 + st2, n2, p.overlap_diff_limit, p.overlap_require);
            int isize = p.insert_size_max;  // :510-523
            if (ov.overlapped) isize = ov.offset > 0 ? n1 + n2 - ov.len : ov.len;
            if (isize > p.insert_size_max) isize = p.insert_size_max;
            lds_add64(&sm.c[FQ_ACC_INSERT + isize], 1ull);
            if (p.correction_enabled) correct_pair(sm, s1 + st1, q1 + st1, s2 + st2, q2 + st2, n2, ov, r1, r2);  // :310-312
            if (p.adapter_trimming) {
                const int ol = ov.len;  // AdapterTrimmer::trimByOverlapAnalysis, src/adaptertrimmer.cpp:14-27
                if (ov.diff <= 5 && ov.overlapped && ov.offset < 0 && ol > n1 / 3) {
                    r1.flags |= FQ_RF_AD_OVERLAP;
                    r1.ad_pos = (uint16_t)(st1 + ol);
                    r1.ad_len = (uint16_t)(n1 - ol);
                    r2.flags |= FQ_RF_AD_OVERLAP;
                    r2.ad_pos = (uint16_t)(st2 + ol);
                    r2.ad_len = (uint16_t)(n2 - ol);
                    lds_add64(&sm.c[FQ_ACC_ADAPTER_READS], 2ull);
                    lds_add64(&sm.c[FQ_ACC_ADAPTER_BASES], (unsigned long long)((n1 - ol) + (n2 - ol)));
                    n1 = ol;
                    n2 = ol;
                } else {
                    if (p.adapter1_len > 0) apply_adapter_seq(sm, s1, st1, n1, p.adapter1, p.adapter1_len, r1);
                    if (p.adapter2_len > 0) apply_adapter_seq(sm, s2, st2, n2, p.adapter2, p.adapter2_len, r2);
                }
            }
        }
        if (both && p.polyx_enabled) {  // :335-340
            apply_polyx(p, sm, s1, st1, n1);
            apply_polyx(p, sm, s2, st2, n2);
        }
        if (both) {  // :342-349
            if (p.max_len1 > 0 && p.max_len1 < n1) n1 = p.max_len1;
            if (p.max_len2 > 0 && p.max_len2 < n2) n2 = p.max_len2;
        }
        bool mergeProcessed = false;
        if (p.merge_enabled && both) {  // :351-385
            Overlap ov = analyze(s1 + st1, n1, s2 + st2, n2, p.overlap_diff_limit, p.overlap_require);
            if (ov.overlapped) {
                r1.flags |= FQ_RF_OVERLAP | FQ_RF_MERGED;
                int code = FQ_FAIL_LENGTH;  // OverlapAnalysis::merge returns NULL for overlapLen 0
                if (ov.len) {
                    const int ol = ov.len;
                    int m1 = min(ol + max(0, ov.offset), n1);
                    int m2 = ov.offset > 0 ? max(0, n2 - ol) : 0;
                    r1.m_len1 = (uint16_t)m1;
                    r1.m_len2 = (uint16_t)m2;
                    const int mlen = m1 + m2;
                    const Row a_s = s1 + st1;
                    const Row a_q = q1 + st1;
                    const Row b_s = s2 + st2;
                    const Row b_q = q2 + st2;
                    // merged base i: r1[i] for i < m1, else revcomp(r2)[ol + i - m1]
                    auto fetch = [&](int i, uint8_t& bb, int& qq) {
                        if (i < m1) {
                            bb = a_s[i];
                            qq = qv(a_q, i);
                        } else {
                            const int src = n2 - 1 - (ol + i - m1);
                            bb = comp(b_s[src]);
                            qq = qv(b_q, src);
                        }
                    };
                    // Filter::passFilter on the merged read
                    if (mlen == 0) {
                        code = FQ_FAIL_LENGTH;
                    } else {
                        int low = 0, nb = 0, tq = 0;
                        if (p.qual_filter_enabled || p.length_filter_enabled) {
                            for (int i = 0; i < mlen; ++i) {
                                uint8_t bb;
                                int qq;
                                fetch(i, bb, qq);
                                tq += qq - 33;
                                nb += bb == 'N';
                                low += qq < p.low_qual_limit;
                            }
                        }
                        code = FQ_PASS_FILTER;
                        if (p.qual_filter_enabled && low > p.low_qual_base_limit) code = FQ_FAIL_QUALITY;
                        else if (p.qual_filter_enabled && p.avg_qual_limit > 0 && p.avg_qual_limit > (double)tq / mlen)
                            code = FQ_FAIL_QUALITY;
                        else if (p.qual_filter_enabled && nb > p.n_base_limit) code = FQ_FAIL_N_BASE;
                        else if (p.length_filter_enabled && mlen < p.min_len) code = FQ_FAIL_LENGTH;
                        else if (p.length_filter_enabled && p.max_len > 0 && mlen > p.max_len) code = FQ_FAIL_TOO_LONG;
                        else if (p.complexity_enabled) {
                            bool ok = false;
                            if (mlen > 1) {
                                int diff = 0;
                                uint8_t prev;
                                int qq;
                                fetch(0, prev, qq);
                                for (int i = 1; i < mlen; ++i) {
                                    uint8_t cur;
                                    fetch(i, cur, qq);
                                    diff += cur != prev;
                                    prev = cur;
                                }
                                ok = (double)diff / (mlen - 1) >= p.complexity_threshold;
                            }
                            if (!ok) code = FQ_FAIL_COMPLEXITY;
                        }
                    }
                    if (code == FQ_PASS_FILTER) {
                        if (mlen > C) {
                            atomicOr(err, 1);
                        } else {
                            stat_read(sm, 2, mlen, skew, fetch);
                            lds_add64(&sm.c[FQ_ACC_MERGED_PAIRS], 1ull);
                        }
                    }
                }
                lds_add64(&sm.c[FQ_ACC_FILTER + code], 2ull);
                r1.code = r2.code = (uint8_t)code;
                mergeProcessed = true;
            } else if (!p.discard_unmerged) {
                const int c1 = pass_filter(p, s1 + st1, q1 + st1, n1, false);
                lds_add64(&sm.c[FQ_ACC_FILTER + c1], 1ull);
                if (c1 == FQ_PASS_FILTER) row_stat(sm, 2, C, s1 + st1, q1 + st1, n1, skew);
                const int c2 = pass_filter(p, s2 + st2, q2 + st2, n2, false);
                lds_add64(&sm.c[FQ_ACC_FILTER + c2], 1ull);
                if (c2 == FQ_PASS_FILTER) row_stat(sm, 3, C, s2 + st2, q2 + st2, n2, skew);
                r1.code = (uint8_t)c1;
                r2.code = (uint8_t)c2;
                mergeProcessed = true;
            }
        }
        if (!mergeProcessed) {  // :387-429
            const int c1 = pass_filter(p, s1 + st1, q1 + st1, n1, !nn1);
            const int c2 = pass_filter(p, s2 + st2, q2 + st2, n2, !nn2);
            lds_add64(&sm.c[FQ_ACC_FILTER + max(c1, c2)], 2ull);
            if (nn1 && c1 == FQ_PASS_FILTER && nn2 && c2 == FQ_PASS_FILTER && !p.merge_enabled) {
                row_stat(sm, 2, C, s1 + st1, q1 + st1, n1, skew);
                row_stat(sm, 3, C, s2 + st2, q2 + st2, n2, skew);
            }
            r1.code = (uint8_t)c1;
            r2.code = (uint8_t)c2;
        }
        r1.start = nn1 ? (uint16_t)st1 : 0;
        r1.len = nn1 ? (uint16_t)n1 : 0;
        r2.start = nn2 ? (uint16_t)st2 : 0;
        r2.len = nn2 ? (uint16_t)n2 : 0;
        if (res) {
            store_result(&res[2 * (size_t)idx], r1);
            store_result(&res[2 * (size_t)idx + 1], r2);
        }
    }
    __syncthreads();

    // flush: small counters, stats scalars, per-cycle histograms
    for (int i = threadIdx.x; i < nsmall; i += blockDim.x) {
        unsigned long long v = sm.c[i];
        if (v) atomicAdd(&acc[i], v);
    }
    const size_t st_base = acc_stats_offset(p.insert_size_max, C, 0);
    const size_t st_words = acc_stats_words(C);
    if (threadIdx.x < 4) {
        unsigned long long v = sm.tail[threadIdx.x];
        if (v) atomicAdd(&acc[st_base + 4 * st_words + threadIdx.x], v);
    }
    if (threadIdx.x < 16) {
        const int k = threadIdx.x >> 2, f = threadIdx.x & 3;
        unsigned long long v = sm.scal[threadIdx.x];
        if (v) atomicAdd(&acc[st_base + k * st_words + f], v);
    }
    for (int i = threadIdx.x; i < 4 * sm.clds; i += blockDim.x) {
        const int k = i / sm.clds, c = i - k * sm.clds;
        const uint32_t* rec = sm.hist + (size_t)i * kRec;
        unsigned long long* dst = acc + st_base + k * st_words + FQ_ST_CYCLES + (size_t)c * FQ_ST_PER_CYCLE;
#pragma unroll
        for (int f = 0; f < 8; ++f) {
            const uint32_t cnt = rec[f];
            if (cnt) {
                atomicAdd(&dst[f], (unsigned long long)cnt);
                const long long qsum = (long long)rec[8 + f] - 161ll * (long long)cnt;  // undo the +128 bias, -33
                atomicAdd(&dst[8 + f], (unsigned long long)qsum);
            }
        }
    }
}

}  // namespace

size_t fq_pack_kernel_lds_bytes(const fq_params& p) {
    return (size_t)(small_words(p) + 4 * lds_cycles(p) * kRec) * sizeof(uint32_t);
}

hipError_t fq_launch_pack_kernel(const fq_params& p, const fq_batch& b, fq_read_result* res, unsigned long long* acc,
                                 int* err, int grid, hipStream_t stream, const int* tiles, const int* ntiles) {
    const size_t lds = fq_pack_kernel_lds_bytes(p);
    if (p.paired)
        hipLaunchKernelGGL(fq_pack_kernel<true>, dim3(grid), dim3(kPackThreads), lds, stream, p, b, res, acc, err, tiles, ntiles);
    else
        hipLaunchKernelGGL(fq_pack_kernel<false>, dim3(grid), dim3(kPackThreads), lds, stream, p, b, res, acc, err, tiles,
                           ntiles);
    return hipGetLastError();
}

hipError_t fq_pack_kernel_set_lds(const fq_params& p) {
    const size_t lds = fq_pack_kernel_lds_bytes(p);
    hipError_t e = hipFuncSetAttribute((const void*)fq_pack_kernel<true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute((const void*)fq_pack_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds);
}
