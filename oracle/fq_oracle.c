/*
 * fq_oracle.c -- TEST INFRASTRUCTURE ONLY (see fq_oracle.h).
 *
 * A line-by-line behavioural restatement of the reference hot path in C99.  Every function
 * cites the reference file:line it follows.  Byte semantics follow the reference's
 * std::string/char usage on x86-64: bytes are compared raw, and quality bytes are read as
 * signed char.
 */
#include "fq_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ORC_MIN(a, b) ((a) < (b) ? (a) : (b))
#define ORC_MAX(a, b) ((a) > (b) ? (a) : (b))

static inline int qv(const uint8_t* q, int i) { return (int)(signed char)q[i]; }

/* The batch planes hold rows in chunk-interleaved tiles (include/fqengine.h); the restatement
 * below works on contiguous reads, gathered here one at a time. */
static _Thread_local uint8_t g_row[4][65536]; /* per thread: the checker runs chunks in parallel */
static const uint8_t* gather(int k, const uint8_t* plane, int stride, int i, int len) {
    fq_batch_get_row(plane, stride, i, g_row[k], len);
    return g_row[k];
}

/* src/filter.cpp:54-67 Filter::passLowComplexityFliter */
static int low_complexity_pass(const fq_params* p, const uint8_t* seq, int rlen) {
    if (rlen <= 1) return 0;
    int diff = 0;
    for (int i = 0; i < rlen - 1; ++i)
        if (seq[i] != seq[i + 1]) ++diff;
    return (double)diff / (rlen - 1) >= p->complexity_threshold;
}

/* src/filter.cpp:3-52 Filter::passFilter */
int orc_pass_filter(const fq_params* p, const uint8_t* seq, const uint8_t* qual, int rlen, int is_null) {
    if (is_null || rlen == 0) return FQ_FAIL_LENGTH;
    int lowQualNum = 0, nBaseNum = 0, totalQual = 0;
    if (p->qual_filter_enabled || p->length_filter_enabled) {
        for (int i = 0; i < rlen; ++i) {
            totalQual += qv(qual, i) - 33;
            if (seq[i] == 'N') ++nBaseNum;
            if (qv(qual, i) < p->low_qual_limit) ++lowQualNum;
        }
    }
    if (p->qual_filter_enabled) {
        if (lowQualNum > p->low_qual_base_limit) return FQ_FAIL_QUALITY;
        else if (p->avg_qual_limit > 0 && p->avg_qual_limit > (double)totalQual / rlen)
            return FQ_FAIL_QUALITY;
    }
    if (p->qual_filter_enabled && nBaseNum > p->n_base_limit) return FQ_FAIL_N_BASE;
    if (p->length_filter_enabled) {
        if (rlen < p->min_len) return FQ_FAIL_LENGTH;
        if (p->max_len > 0 && rlen > p->max_len) return FQ_FAIL_TOO_LONG;
    }
    if (p->complexity_enabled && !low_complexity_pass(p, seq, rlen)) return FQ_FAIL_COMPLEXITY;
    return FQ_PASS_FILTER;
}

/* src/filter.cpp:69-189 Filter::trimAndCut */
int orc_trim_and_cut(const fq_params* p, const uint8_t* seq, const uint8_t* qual, int l, int front,
                     int tail, int* out_start, int* out_len) {
    const int enF = p->cut_front, enR = p->cut_right, enT = p->cut_tail;
    if (front == 0 && tail == 0 && !enF && !enR && !enT) { /* :71-73 */
        *out_start = 0;
        *out_len = l;
        return 1;
    }
    int rlen = l - front - tail; /* :75-78 */
    if (rlen < 0) return 0;
    if (front == 0 && !enF && !enR && !enT) { /* :80-82 resize(rlen) */
        *out_start = 0;
        *out_len = rlen;
        return 1;
    } else if (!enF && !enR && !enT) { /* :83-87 substr(front, rlen) */
        *out_start = front;
        *out_len = rlen;
        return 1;
    }
    if (enF) { /* :94-123 */
        int w = p->cut_front_window;
        int s = front;
        if (l - front - tail - w <= 0) return 0;
        int totalQual = 0;
        for (int i = 0; i < w - 1; ++i) totalQual += qv(qual, s + i);
        for (s = front; s + w < l - tail; ++s) {
            totalQual += qv(qual, s + w - 1);
            if (s > front) totalQual -= qv(qual, s - 1);
            if ((double)totalQual / (double)w >= 33 + p->cut_front_quality) break;
        }
        if (s > 0) s = s + w - 1;
        while (s < l && seq[s] == 'N') ++s;
        front = s;
        rlen = l - front - tail;
    }
    if (enR) { /* :126-152 */
        int w = p->cut_right_window;
        int s = front;
        if (l - front - tail - w <= 0) return 0;
        int totalQual = 0, found = 0;
        for (int i = 0; i < w - 1; ++i) totalQual += qv(qual, s + i);
        for (s = front; s + w < l - tail; ++s) {
            totalQual += qv(qual, s + w - 1);
            if (s > front) totalQual -= qv(qual, s - 1);
            if ((double)totalQual / (double)w < 33 + p->cut_right_quality) {
                found = 1;
                break;
            }
        }
        if (found) {
            while (s < l - 1 && qv(qual, s) >= 33 + p->cut_right_quality) ++s;
            rlen = s - front;
        }
    }
    if (!enR && enT) { /* :155-181 */
        int w = p->cut_tail_window;
        if (l - front - tail - w <= 0) return 0;
        int totalQual = 0;
        int t = l - tail - 1;
        for (int i = 0; i < w - 1; ++i) totalQual += qv(qual, t - i);
        for (t = l - tail - 1; t - w >= front; --t) {
            totalQual += qv(qual, t - w + 1);
            if (t < l - tail - 1) totalQual -= qv(qual, t + 1);
            if ((double)totalQual / (double)w >= 33 + p->cut_tail_quality) break;
        }
        if (t < l - 1) t = t - w + 1;
        while (t >= 0 && seq[t] == 'N') --t;
        rlen = t - front + 1;
    }
    if (rlen <= 0 || front >= l - 1) return 0; /* :183-185 */
    *out_start = front;                       /* :186-187 substr(front, rlen) */
    *out_len = ORC_MIN(rlen, l - front);
    return 1;
}

/* src/polyx.cpp:14-38 PolyX::trimPolyG (single read) */
int orc_trim_polyg(const uint8_t* data, int rlen, int compareReq, int maxMismatch, int per, int* bases) {
    int mismatch = 0, i = 0, firstGpos = rlen - 1;
    for (i = 0; i < rlen; ++i) {
        if (data[rlen - i - 1] != 'G') ++mismatch;
        else firstGpos = rlen - i - 1;
        int allowed = ORC_MIN(maxMismatch, ORC_MAX(1, (i + 1) / per));
        if (mismatch > allowed) break;
    }
    *bases = -1;
    if (i + 1 >= compareReq) {
        int newlen = (firstGpos > rlen || firstGpos < 0) ? rlen : firstGpos; /* Read::resize, src/read.h:181-187 */
        *bases = rlen - firstGpos;
        return newlen;
    }
    return rlen;
}

/* src/polyx.cpp:45-101 PolyX::trimPolyX (single read) */
int orc_trim_polyx(const uint8_t* data, int rlen, int mask, int compareReq, int maxMismatch, int per,
                   int* poly_out, int* bases) {
    static const char bases_atcgn[5] = {'A', 'T', 'C', 'G', 'N'};
    int cnt[5] = {0, 0, 0, 0, 0};
    int pos = 0;
    for (pos = 0; pos < rlen; ++pos) {
        switch (data[rlen - 1 - pos]) {
            case 'A': ++cnt[0]; break;
            case 'T': ++cnt[1]; break;
            case 'C': ++cnt[2]; break;
            case 'G': ++cnt[3]; break;
            default: ++cnt[4]; break;
        }
        int cmp = pos + 1;
        int allowed = ORC_MIN(maxMismatch, ORC_MAX(1, cmp / per));
        int needToBreak = 1;
        for (int b = 0; b < 5; ++b)
            if ((mask >> b & 1) && cmp - cnt[b] <= allowed) needToBreak = 0;
        if (needToBreak) break;
    }
    *poly_out = -1;
    *bases = 0;
    if (pos + 1 >= compareReq) {
        int poly = 0, maxCount = -1;
        for (int b = 0; b < 5; ++b)
            if ((mask >> b & 1) && cnt[b] > maxCount) {
                maxCount = cnt[b];
                poly = b;
            }
        char polyBase = bases_atcgn[poly];
        pos = ORC_MIN(rlen - 1, pos);
        /* the reference tests data[...] before pos > 0; the value of the condition is the same */
        while (pos > 0 && data[rlen - pos - 1] != polyBase) --pos;
        int target = rlen - pos - 1;
        int newlen = (target > rlen || target < 0) ? rlen : target; /* Read::resize */
        *poly_out = poly;
        *bases = pos + 1;
        return newlen;
    }
    return rlen;
}

/* src/seq.h:24-48 Seq::reverseComplement */
static uint8_t complement_base(uint8_t c) {
    switch (c) {
        case 'A': case 'a': return 'T';
        case 'T': case 't': return 'A';
        case 'C': case 'c': return 'G';
        case 'G': case 'g': return 'C';
        default: return 'N';
    }
}

/* src/overlapanalysis.cpp:7-72 OverlapAnalysis::analyze */
orc_overlap orc_analyze(const uint8_t* pstr1, int len1, const uint8_t* s2, int len2, int overlapDiffLimit,
                        int overlapRequire) {
    uint8_t pstr2[65536];
    for (int i = 0; i < len2; ++i) pstr2[len2 - 1 - i] = complement_base(s2[i]);
    const int complete_compare_require = 50;
    int overlapLen = 0, offset = 0, diff = 0;
    orc_overlap ovr;
    while (offset < len1 - overlapRequire) { /* :20-41 */
        overlapLen = ORC_MIN(len1 - offset, len2);
        diff = 0;
        int i = 0;
        for (i = 0; i < overlapLen; ++i) {
            if (pstr1[offset + i] != pstr2[i]) {
                ++diff;
                if (diff >= overlapDiffLimit && i < complete_compare_require) break;
            }
        }
        if (diff < overlapDiffLimit || (diff >= overlapDiffLimit && i > complete_compare_require)) {
            ovr.overlapped = 1;
            ovr.offset = offset;
            ovr.overlap_len = overlapLen;
            ovr.diff = diff;
            return ovr;
        }
        ++offset;
    }
    offset = 0; /* :44-67 */
    while (offset > overlapRequire - len2) {
        overlapLen = ORC_MIN(len1, len2 - (offset < 0 ? -offset : offset));
        diff = 0;
        int i = 0;
        for (i = 0; i < overlapLen; ++i) {
            if (pstr1[i] != pstr2[-offset + i]) {
                ++diff;
                if (diff >= overlapDiffLimit && i < complete_compare_require) break;
            }
        }
        if (diff < overlapDiffLimit || (diff >= overlapDiffLimit && i > complete_compare_require)) {
            ovr.overlapped = 1;
            ovr.offset = offset;
            ovr.overlap_len = overlapLen;
            ovr.diff = diff;
            return ovr;
        }
        --offset;
    }
    ovr.overlapped = 0;
    ovr.offset = ovr.overlap_len = ovr.diff = 0;
    return ovr;
}

/* src/adaptertrimmer.cpp:29-90 AdapterTrimmer::trimBySequence (search part) */
int orc_trim_by_sequence(const uint8_t* rdata, int rlen, const uint8_t* adata, int alen, int* pos_out) {
    const int matchRequired = 4, allowOneMismatchForEach = 8;
    if (alen < matchRequired) return 0;
    int pos = 0, found = 0, start = 0;
    if (alen >= 16) start = -4;
    else if (alen >= 12) start -= 3;
    else if (alen >= 8) start = -2;
    for (pos = start; pos < rlen - matchRequired; ++pos) {
        int cmplen = ORC_MIN(rlen - pos, alen);
        int allowedMismatch = cmplen / allowOneMismatchForEach;
        int mismatch = 0, matched = 1;
        for (int i = ORC_MAX(0, -pos); i < cmplen; ++i) {
            if (adata[i] != rdata[i + pos]) {
                ++mismatch;
                if (mismatch > allowedMismatch) {
                    matched = 0;
                    break;
                }
            }
        }
        if (matched) {
            found = 1;
            break;
        }
    }
    *pos_out = pos;
    return found;
}

/* src/stats.cpp:237-295 Stats::statRead (k-mer / ORA parts are not enabled) */
void orc_stat_read(uint64_t* st, int max_cycles, const uint8_t* seq, const uint8_t* qual, int len) {
    (void)max_cycles;
    st[FQ_ST_LENGTH_SUM] += (uint64_t)len;
    for (int i = 0; i < len; ++i) {
        int b = seq[i] & 0x07;
        int q = qv(qual, i);
        if (q > '?') {
            st[FQ_ST_Q20] += 1;
            st[FQ_ST_Q30] += 1;
        } else if (q > '5') {
            st[FQ_ST_Q20] += 1;
        }
        uint64_t* cyc = st + FQ_ST_CYCLES + (size_t)i * FQ_ST_PER_CYCLE;
        cyc[b] += 1;
        cyc[8 + b] += (uint64_t)(int64_t)(q - 33);
    }
    st[FQ_ST_READS] += 1;
}

/* merged read bytes: src/overlapanalysis.cpp:74-104 (sequence / quality part) */
static int build_merged(const uint8_t* s1, const uint8_t* q1, const uint8_t* s2, const uint8_t* q2, int l2,
                        int len1, int len2, int ol, uint8_t* ms, uint8_t* mq) {
    memcpy(ms, s1, (size_t)len1);
    memcpy(mq, q1, (size_t)len1);
    for (int j = 0; j < len2; ++j) {
        int src = l2 - 1 - (ol + j); /* revcomp(r2)[ol + j] */
        ms[len1 + j] = complement_base(s2[src]);
        mq[len1 + j] = q2[src];
    }
    return len1 + len2;
}

static void set_result(fq_read_result* r, int is_null, int start, int len) {
    memset(r, 0, sizeof *r);
    r->flags = is_null ? FQ_RF_NULL : 0;
    r->start = (uint16_t)(is_null ? 0 : start);
    r->len = (uint16_t)(is_null ? 0 : len);
}

/* src/adaptertrimmer.cpp:29-90 applied to a read window: adapter bookkeeping + new length */
static void apply_trim_by_sequence(const fq_params* p, const uint8_t* seq, int start, int* len,
                                   const uint8_t* ad, int alen, fq_read_result* rr, uint64_t* acc) {
    int pos = 0;
    if (!orc_trim_by_sequence(seq + start, *len, ad, alen, &pos)) return;
    (void)p;
    int ad_len;
    if (pos < 0) {
        ad_len = alen + pos;
        rr->flags |= FQ_RF_AD_SEQ | FQ_RF_AD_NEG;
        rr->ad_pos = (uint16_t)(-pos);
        rr->ad_len = (uint16_t)ad_len;
        *len = 0;
    } else {
        ad_len = *len - pos;
        rr->flags |= FQ_RF_AD_SEQ;
        rr->ad_pos = (uint16_t)(start + pos);
        rr->ad_len = (uint16_t)ad_len;
        *len = pos;
    }
    if (ad_len > 0) { /* FilterResult::addAdapterTrimmed(str, isR2), src/filterresult.cpp:138-157 */
        acc[FQ_ACC_ADAPTER_READS] += 1;
        acc[FQ_ACC_ADAPTER_BASES] += (uint64_t)ad_len;
    }
}

static void apply_polyx(const fq_params* p, const uint8_t* seq, int start, int* len, uint64_t* acc) {
    int poly = -1, bases = 0;
    *len = orc_trim_polyx(seq + start, *len, p->polyx_mask, p->polyx_compare_req, p->polyx_max_mismatch,
                          p->polyx_one_mismatch_per, &poly, &bases);
    if (poly >= 0) { /* FilterResult::addPolyXTrimmed, src/filterresult.cpp:43-46 */
        acc[FQ_ACC_POLYX_READS + poly] += 1;
        acc[FQ_ACC_POLYX_BASES + poly] += (uint64_t)(int64_t)bases;
    }
}

static void apply_polyg(const fq_params* p, const uint8_t* seq, int start, int* len, uint64_t* acc) {
    int bases = -1;
    *len = orc_trim_polyg(seq + start, *len, p->polyg_compare_req, p->polyg_max_mismatch,
                          p->polyg_one_mismatch_per, &bases);
    if (bases >= 0) {
        acc[FQ_ACC_POLYX_READS + 3] += 1;
        acc[FQ_ACC_POLYX_BASES + 3] += (uint64_t)(int64_t)bases;
    }
}

/* Read::trimFront(umi length + skip) of UmiProcessor::process, src/umiprocessor.cpp:28-62 and
 * src/read.h:203-208: min(k, len - 1) leading bases go (a read of length 0 is left alone) */
static int umi_cut(int k, int len) { return (k > 0 && len > 0) ? ORC_MIN(k, len - 1) : 0; }

static int index_filtered(const fq_batch* b, int i) { return b->flags && (b->flags[i] & FQ_BF_INDEX_FILTERED); }

/* src/basecorrector.cpp:14-70 BaseCorrector::correctByOverlapAnalysis on the pair's windows (the
 * gathered row copies are edited in place, as the reference edits its strings) */
static void correct_by_overlap(uint8_t* s1, uint8_t* q1, uint8_t* s2, uint8_t* q2, int len2, orc_overlap ov,
                               fq_read_result* rr1, fq_read_result* rr2, uint64_t* tail) {
    if (ov.diff == 0 || ov.diff > 5) return;
    int ol = ov.overlap_len;
    int start1 = ORC_MAX(0, ov.offset);
    int start2 = len2 - ORC_MAX(0, -ov.offset) - 1;
    const int GOOD_QUAL = 33 + 30, BAD_QUAL = 33 + 14; /* util::num2qual */
    int corrected = 0, r1c = 0, r2c = 0;
    for (int i = 0; i < ol; ++i) {
        int p1 = start1 + i, p2 = start2 - i;
        if (s1[p1] != complement_base(s2[p2])) {
            if (qv(q1, p1) >= GOOD_QUAL && qv(q2, p2) <= BAD_QUAL) {
                s2[p2] = complement_base(s1[p1]);
                q2[p2] = q1[p1];
                ++corrected;
                r2c = 1;
            } else if (qv(q2, p2) >= GOOD_QUAL && qv(q1, p1) <= BAD_QUAL) {
                s1[p1] = complement_base(s2[p2]);
                q1[p1] = q2[p2];
                ++corrected;
                r1c = 1;
            }
        }
    }
    if (corrected > 0) {
        tail[FQ_ACC_TAIL_CORRECTED_READS] += (r1c && r2c) ? 2 : 1; /* incCorrectedReads */
        tail[FQ_ACC_TAIL_CORRECTED_BASES] += (uint64_t)corrected; /* one addCorrection per base */
        if (r1c) rr1->flags |= FQ_RF_CORRECTED;
        if (r2c) rr2->flags |= FQ_RF_CORRECTED;
        rr2->m_len1 = (uint16_t)(int16_t)ov.offset;
        rr2->m_len2 = (uint16_t)ol;
        rr2->reserved = (uint16_t)len2;
    }
}

static void set_index_filtered(fq_read_result* r) {
    memset(r, 0, sizeof *r);
    r->flags = FQ_RF_INDEX_FILTERED;
}

/* src/seprocessor.cpp:290-388 SingleEndProcessor::processSingleEnd, loop body */
static int process_se(const fq_params* p, const fq_batch* b, fq_read_result* res, uint64_t* acc) {
    uint64_t* pre = acc + fq_acc_stats_offset(p->insert_size_max, p->max_cycles, 0);
    uint64_t* post = acc + fq_acc_stats_offset(p->insert_size_max, p->max_cycles, 2);
    for (int i = 0; i < b->n; ++i) {
        int l = b->len1[i];
        const uint8_t* seq = gather(0, b->seq1, b->stride, i, l);
        const uint8_t* qual = gather(1, b->qual1, b->stride, i, l);
        if (l > p->max_cycles) return FQ_E_TOO_LONG;
        fq_read_result* rr = &res[i];
        orc_stat_read(pre, p->max_cycles, seq, qual, l); /* :298 */
        if (index_filtered(b, i)) { /* :304-307 */
            set_index_filtered(rr);
            continue;
        }
        int u = umi_cut(p->umi_front1, l); /* :309-311 */
        int s = 0, len = 0;
        int nonnull = orc_trim_and_cut(p, seq + u, qual + u, l - u, p->trim_front1, p->trim_tail1, &s, &len); /* :313 */
        s += u;
        set_result(rr, !nonnull, s, len);
        if (nonnull && p->polyg_enabled) apply_polyg(p, seq, s, &len, acc);          /* :315-319 */
        if (nonnull && p->adapter_trimming && p->adapter1_len > 0)                  /* :321-323 */
            apply_trim_by_sequence(p, seq, s, &len, p->adapter1, p->adapter1_len, rr, acc);
        if (nonnull && p->polyx_enabled) apply_polyx(p, seq, s, &len, acc);          /* :325-330 */
        if (nonnull && p->max_len1 > 0 && p->max_len1 < len) len = p->max_len1;     /* :332-336 */
        int code = orc_pass_filter(p, seq + s, qual + s, len, !nonnull);            /* :339 */
        acc[FQ_ACC_FILTER + code] += 1;                                               /* :340, mPaired=false */
        if (nonnull && code == FQ_PASS_FILTER) orc_stat_read(post, p->max_cycles, seq + s, qual + s, len);
        rr->start = (uint16_t)(nonnull ? s : 0);
        rr->len = (uint16_t)(nonnull ? len : 0);
        rr->code = (uint8_t)code;
    }
    return FQ_OK;
}

/* src/peprocessor.cpp:510-523 PairEndProcessor::statInsertSize */
static void stat_insert(const fq_params* p, uint64_t* acc, int len1, int len2, orc_overlap ov) {
    int isize = p->insert_size_max;
    if (ov.overlapped) isize = ov.offset > 0 ? len1 + len2 - ov.overlap_len : ov.overlap_len;
    if (isize > p->insert_size_max) isize = p->insert_size_max;
    acc[FQ_ACC_INSERT + isize] += 1;
}

/* src/peprocessor.cpp:261-508 PairEndProcessor::processPairEnd, loop body (outputs become records) */
static int process_pe(const fq_params* p, const fq_batch* b, fq_read_result* res, uint64_t* acc) {
    uint64_t* pre1 = acc + fq_acc_stats_offset(p->insert_size_max, p->max_cycles, 0);
    uint64_t* pre2 = acc + fq_acc_stats_offset(p->insert_size_max, p->max_cycles, 1);
    uint64_t* post1 = acc + fq_acc_stats_offset(p->insert_size_max, p->max_cycles, 2);
    uint64_t* post2 = acc + fq_acc_stats_offset(p->insert_size_max, p->max_cycles, 3);
    static _Thread_local uint8_t ms[131072], mq[131072];
    for (int i = 0; i < b->n; ++i) {
        int l1 = b->len1[i], l2 = b->len2[i];
        const uint8_t* s1 = gather(0, b->seq1, b->stride, i, l1);
        const uint8_t* q1 = gather(1, b->qual1, b->stride, i, l1);
        const uint8_t* s2 = gather(2, b->seq2, b->stride, i, l2);
        const uint8_t* q2 = gather(3, b->qual2, b->stride, i, l2);
        if (l1 > p->max_cycles || l2 > p->max_cycles) return FQ_E_TOO_LONG;
        fq_read_result* rr1 = &res[2 * i];
        fq_read_result* rr2 = &res[2 * i + 1];
        orc_stat_read(pre1, p->max_cycles, s1, q1, l1); /* :276-277 */
        orc_stat_read(pre2, p->max_cycles, s2, q2, l2);
        if (index_filtered(b, i)) { /* :283-286 */
            set_index_filtered(rr1);
            set_index_filtered(rr2);
            continue;
        }
        int u1 = umi_cut(p->umi_front1, l1), u2 = umi_cut(p->umi_front2, l2); /* :288-290 */
        int st1 = 0, n1 = 0, st2 = 0, n2 = 0; /* :292-293 */
        int nn1 = orc_trim_and_cut(p, s1 + u1, q1 + u1, l1 - u1, p->trim_front1, p->trim_tail1, &st1, &n1);
        int nn2 = orc_trim_and_cut(p, s2 + u2, q2 + u2, l2 - u2, p->trim_front2, p->trim_tail2, &st2, &n2);
        st1 += u1;
        st2 += u2;
        set_result(rr1, !nn1, st1, n1);
        set_result(rr2, !nn2, st2, n2);
        const int both = nn1 && nn2;
        if (both && p->polyg_enabled) { /* :295-299 */
            apply_polyg(p, s1, st1, &n1, acc);
            apply_polyg(p, s2, st2, &n2, acc);
        }
        if (both) { /* :302-333: overlap once per pair (every pair == reference -w 1) */
            orc_overlap ov = orc_analyze(s1 + st1, n1, s2 + st2, n2, p->overlap_diff_limit, p->overlap_require);
            stat_insert(p, acc, n1, n2, ov);
            if (p->correction_enabled) /* :310-312 */
                correct_by_overlap((uint8_t*)s1 + st1, (uint8_t*)q1 + st1, (uint8_t*)s2 + st2, (uint8_t*)q2 + st2, n2, ov,
                                   rr1, rr2, acc + fq_acc_tail_offset(p->insert_size_max, p->max_cycles));
            if (p->adapter_trimming) {
                /* AdapterTrimmer::trimByOverlapAnalysis, src/adaptertrimmer.cpp:14-27 */
                int ol = ov.overlap_len;
                if (ov.diff <= 5 && ov.overlapped && ov.offset < 0 && ol > n1 / 3) {
                    rr1->flags |= FQ_RF_AD_OVERLAP;
                    rr1->ad_pos = (uint16_t)(st1 + ol);
                    rr1->ad_len = (uint16_t)(n1 - ol);
                    rr2->flags |= FQ_RF_AD_OVERLAP;
                    rr2->ad_pos = (uint16_t)(st2 + ol);
                    rr2->ad_len = (uint16_t)(n2 - ol);
                    acc[FQ_ACC_ADAPTER_READS] += 2; /* src/filterresult.cpp:159-161 */
                    acc[FQ_ACC_ADAPTER_BASES] += (uint64_t)((n1 - ol) + (n2 - ol));
                    n1 = ol;
                    n2 = ol;
                } else {
                    if (p->adapter1_len > 0)
                        apply_trim_by_sequence(p, s1, st1, &n1, p->adapter1, p->adapter1_len, rr1, acc);
                    if (p->adapter2_len > 0)
                        apply_trim_by_sequence(p, s2, st2, &n2, p->adapter2, p->adapter2_len, rr2, acc);
                }
            }
        }
        if (both && p->polyx_enabled) { /* :335-340 */
            apply_polyx(p, s1, st1, &n1, acc);
            apply_polyx(p, s2, st2, &n2, acc);
        }
        if (both) { /* :342-349 */
            if (p->max_len1 > 0 && p->max_len1 < n1) n1 = p->max_len1;
            if (p->max_len2 > 0 && p->max_len2 < n2) n2 = p->max_len2;
        }
        int mergeProcessed = 0;
        if (p->merge_enabled && both) { /* :351-385 */
            orc_overlap ov = orc_analyze(s1 + st1, n1, s2 + st2, n2, p->overlap_diff_limit, p->overlap_require);
            if (ov.overlapped) {
                rr1->flags |= FQ_RF_OVERLAP | FQ_RF_MERGED;
                int code;
                if (!ov.overlap_len) { /* OverlapAnalysis::merge returns NULL */
                    code = orc_pass_filter(p, NULL, NULL, 0, 1);
                } else {
                    int ol = ov.overlap_len;
                    int ml1 = ol + ORC_MAX(0, ov.offset);
                    int ml2 = ov.offset > 0 ? n2 - ol : 0;
                    /* substr clamps: r1.substr(0, ml1), rr2.substr(ol, ml2) */
                    if (ml1 > n1) ml1 = n1;
                    if (ml2 > n2 - ol) ml2 = n2 - ol;
                    if (ml2 < 0) ml2 = 0;
                    rr1->m_len1 = (uint16_t)ml1;
                    rr1->m_len2 = (uint16_t)ml2;
                    int mlen = build_merged(s1 + st1, q1 + st1, s2 + st2, q2 + st2, n2, ml1, ml2, ol, ms, mq);
                    code = orc_pass_filter(p, ms, mq, mlen, 0);
                    if (code == FQ_PASS_FILTER) {
                        if (mlen > p->max_cycles) return FQ_E_TOO_LONG;
                        orc_stat_read(post1, p->max_cycles, ms, mq, mlen);
                        acc[FQ_ACC_MERGED_PAIRS] += 1;
                    }
                }
                acc[FQ_ACC_FILTER + code] += 2;
                rr1->code = (uint8_t)code;
                rr2->code = (uint8_t)code;
                mergeProcessed = 1;
            } else if (!p->discard_unmerged) {
                int c1 = orc_pass_filter(p, s1 + st1, q1 + st1, n1, 0);
                acc[FQ_ACC_FILTER + c1] += 1;
                if (c1 == FQ_PASS_FILTER) orc_stat_read(post1, p->max_cycles, s1 + st1, q1 + st1, n1);
                int c2 = orc_pass_filter(p, s2 + st2, q2 + st2, n2, 0);
                acc[FQ_ACC_FILTER + c2] += 1;
                if (c2 == FQ_PASS_FILTER) orc_stat_read(post2, p->max_cycles, s2 + st2, q2 + st2, n2);
                rr1->code = (uint8_t)c1;
                rr2->code = (uint8_t)c2;
                mergeProcessed = 1;
            }
        }
        if (!mergeProcessed) { /* :387-429 */
            int c1 = orc_pass_filter(p, s1 + st1, q1 + st1, n1, !nn1);
            int c2 = orc_pass_filter(p, s2 + st2, q2 + st2, n2, !nn2);
            acc[FQ_ACC_FILTER + ORC_MAX(c1, c2)] += 2; /* addFilterResult(result), paired: +2 */
            if (nn1 && c1 == FQ_PASS_FILTER && nn2 && c2 == FQ_PASS_FILTER && !p->merge_enabled) {
                orc_stat_read(post1, p->max_cycles, s1 + st1, q1 + st1, n1);
                orc_stat_read(post2, p->max_cycles, s2 + st2, q2 + st2, n2);
            }
            rr1->code = (uint8_t)c1;
            rr2->code = (uint8_t)c2;
        }
        rr1->start = (uint16_t)(nn1 ? st1 : 0);
        rr1->len = (uint16_t)(nn1 ? n1 : 0);
        rr2->start = (uint16_t)(nn2 ? st2 : 0);
        rr2->len = (uint16_t)(nn2 ? n2 : 0);
    }
    return FQ_OK;
}

int orc_process_batch(const fq_params* p, const fq_batch* b, fq_read_result* results, uint64_t* acc) {
    if (!p || !b || !results || !acc) return FQ_E_INVALID;
    return p->paired ? process_pe(p, b, results, acc) : process_se(p, b, results, acc);
}

/* ------------------------------------------------------------------------------------ *
 * Duplicate, src/duplicate.cpp:3-166
 * ------------------------------------------------------------------------------------ */
struct orc_dup {
    int keylen;
    uint64_t keys;
    uint64_t* dups;
    uint32_t* counts;
    uint8_t* gc;
};

orc_dup* orc_dup_create(int keylen) {
    orc_dup* d = (orc_dup*)calloc(1, sizeof *d);
    d->keylen = keylen;
    d->keys = keylen >= 16 ? (1ull << 32) : (1ull << (2 * keylen)); /* keys are (uint32_t) truncated */
    d->dups = (uint64_t*)calloc(d->keys, 8);
    d->counts = (uint32_t*)calloc(d->keys, 4);
    d->gc = (uint8_t*)calloc(d->keys, 1);
    return d;
}

void orc_dup_destroy(orc_dup* d) {
    if (!d) return;
    free(d->dups);
    free(d->counts);
    free(d->gc);
    free(d);
}

/* Duplicate::seq2int, src/duplicate.cpp:20-44 */
static uint64_t dup_seq2int(const uint8_t* s, int start, int keylen, int* valid) {
    uint64_t ret = 0;
    for (int i = 0; i < keylen; ++i) {
        ret <<= 2;
        switch (s[start + i]) {
            case 'A': ret += 0; break;
            case 'T': ret += 1; break;
            case 'C': ret += 2; break;
            case 'G': ret += 3; break;
            default: *valid = 0; return 0;
        }
    }
    return ret;
}

/* Duplicate::addRecord, src/duplicate.cpp:46-69 */
static void dup_add_record(orc_dup* d, uint32_t key, uint64_t kmer32, uint8_t gc) {
    if (d->counts[key] == 0) {
        d->counts[key] = 1;
        d->dups[key] = kmer32;
        d->gc[key] = gc;
    } else if (d->dups[key] == kmer32) {
        ++d->counts[key];
    } else if (d->dups[key] > kmer32) {
        d->dups[key] = kmer32;
        d->counts[key] = 1;
        d->gc[key] = gc;
    }
}

void orc_dup_add_batch(orc_dup* d, const fq_batch* b, int paired) {
    for (int i = 0; i < b->n; ++i) {
        int l1 = b->len1[i];
        const uint8_t* s1 = gather(0, b->seq1, b->stride, i, l1);
        int valid = 1;
        uint8_t gc = 0; /* uint8_t counter, as the reference's */
        if (paired) { /* Duplicate::statPair, src/duplicate.cpp:101-130 */
            int l2 = b->len2[i];
            const uint8_t* s2 = gather(2, b->seq2, b->stride, i, l2);
            if (l1 < 32 || l2 < 32) continue;
            uint32_t key = (uint32_t)dup_seq2int(s1, 0, d->keylen, &valid);
            if (!valid) continue;
            uint64_t kmer32 = dup_seq2int(s2, 0, 32, &valid);
            if (!valid) continue;
            if (d->counts[key] == 0) {
                for (int k = 0; k < l1; ++k) gc += s1[k] == 'C' || s1[k] == 'G';
                for (int k = 0; k < l2; ++k) gc += s2[k] == 'C' || s2[k] == 'G';
            }
            gc = (uint8_t)round(255.0 * (double)gc / (double)(l1 + l2));
            dup_add_record(d, key, kmer32, gc);
        } else { /* Duplicate::statRead, src/duplicate.cpp:71-99 */
            if (l1 < 32) continue;
            int start2 = ORC_MAX(0, l1 - 32 - 5);
            uint32_t key = (uint32_t)dup_seq2int(s1, 0, d->keylen, &valid);
            if (!valid) continue;
            uint64_t kmer32 = dup_seq2int(s1, start2, 32, &valid);
            if (!valid) continue;
            if (d->counts[key] == 0)
                for (int k = 0; k < l1; ++k) gc += s1[k] == 'C' || s1[k] == 'G';
            gc = (uint8_t)round(255.0 * (double)gc / (double)l1);
            dup_add_record(d, key, kmer32, gc);
        }
    }
}

/* Duplicate::statAll, src/duplicate.cpp:132-166 (counts == hist_size land past the reference's
 * arrays and are not reported) */
void orc_dup_stat(const orc_dup* d, int hist_size, uint64_t* hist, uint64_t* gc_sum, uint64_t* totals) {
    memset(hist, 0, (size_t)hist_size * 8);
    memset(gc_sum, 0, (size_t)hist_size * 8);
    totals[0] = totals[1] = 0;
    for (uint64_t key = 0; key < d->keys; ++key) {
        uint32_t count = d->counts[key];
        if (count == 0) continue;
        totals[0] += count;
        totals[1] += count - 1;
        int bin = count > (uint32_t)hist_size ? hist_size - 1 : (int)count;
        if (bin >= hist_size) continue;
        hist[bin] += 1;
        gc_sum[bin] += d->gc[key];
    }
}

/* ------------------------------------------------------------------------------------ *
 * Adapter-detection k-mers, src/evaluator.cpp:3-47 (seq2int), :265-279, :392-405
 * ------------------------------------------------------------------------------------ */
typedef struct orc_kmer_set {
    const uint8_t* seq;
    const uint32_t* off;
    int32_t n;
} orc_kmer_set;

/* Evaluator::seq2int: the key of [pos, pos + keylen) from the previous window's key, or -1 */
static int kmer_seq2int(const uint8_t* s, int pos, int keylen, int last) {
    if (last >= 0) {
        const int mask = (1 << (keylen * 2)) - 1;
        int key = (last << 2) & mask;
        switch (s[pos + keylen - 1]) {
            case 'A': return key + 0;
            case 'T': return key + 1;
            case 'C': return key + 2;
            case 'G': return key + 3;
            default: return -1;
        }
    }
    int key = 0;
    for (int i = pos; i < pos + keylen; ++i) {
        key <<= 2;
        switch (s[i]) {
            case 'A': break;
            case 'T': key += 1; break;
            case 'C': key += 2; break;
            case 'G': key += 3; break;
            default: return -1;
        }
    }
    return key;
}

int orc_kmer_open(int device, const uint8_t* seq, const uint32_t* off, int32_t n, void** out) {
    (void)device;
    orc_kmer_set* k = (orc_kmer_set*)calloc(1, sizeof *k);
    k->seq = seq; /* the caller keeps the reads alive while the set is open */
    k->off = off;
    k->n = n;
    *out = k;
    return FQ_OK;
}

int orc_kmer_close(void* set) {
    free(set);
    return FQ_OK;
}

int orc_kmer_count(void* set, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t* counts) {
    const orc_kmer_set* k = (const orc_kmer_set*)set;
    memset(counts, 0, ((size_t)1 << (2 * keylen)) * 4);
    for (int r = 0; r < k->n; ++r) {
        const uint8_t* s = k->seq + k->off[r];
        const int len = (int)(k->off[r + 1] - k->off[r]);
        int key = -1;
        for (int pos = first; pos <= len - keylen - shift_tail; ++pos) {
            key = kmer_seq2int(s, pos, keylen, key);
            if (key >= 0) ++counts[key];
        }
    }
    return FQ_OK;
}

int orc_kmer_find(void* set, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t seed, uint64_t* occ,
                  size_t cap, size_t* n_out) {
    const orc_kmer_set* k = (const orc_kmer_set*)set;
    size_t n = 0;
    for (int r = 0; r < k->n; ++r) {
        const uint8_t* s = k->seq + k->off[r];
        const int len = (int)(k->off[r + 1] - k->off[r]);
        int key = -1;
        for (int pos = first; pos <= len - keylen - shift_tail; ++pos) {
            key = kmer_seq2int(s, pos, keylen, key);
            if (key >= 0 && (uint32_t)key == seed) {
                if (n < cap) occ[n] = ((uint64_t)r << 32) | (uint32_t)pos;
                ++n;
            }
        }
    }
    *n_out = n;
    return FQ_OK;
}

/* ------------------------------------------------------------------------------------ *
 * Synthetic workload, host twin of the engine's fq_synth_fill_device.
 * Integer-only (no libm) so host and device agree bit for bit.
 * ------------------------------------------------------------------------------------ */
static const char SYN_AD1[] = "AGATCGGAAGAGCACACGTCTGAACTCCAGTCA"; /* TruSeq R1 */
static const char SYN_AD2[] = "AGATCGGAAGAGCGTCGTGTAGGGAAAGAGTGT"; /* TruSeq R2 */
static const char SYN_ACGT[] = "ACGT";

static uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static uint8_t syn_comp(uint8_t c) {
    return c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : c == 'T' ? 'A' : 'N';
}

static void synth_read(uint64_t key, int mate, int L, int ins, uint8_t* seq, uint8_t* qual) {
    const char* ad = mate ? SYN_AD2 : SYN_AD1;
    const int alen = 33;
    uint64_t rm = sm64(key + 2 + (uint64_t)mate);
    int polyg = ((rm & 0xFFFF) % 100 < 5) ? 10 + (int)(((rm >> 16) & 0xFFFF) % 51) : 0;
    int lowq = (((rm >> 32) & 0xFFFF) % 100 < 2) ? 100 + (int)((rm >> 48) % 51) : L;
    for (int i = 0; i < L; ++i) {
        uint8_t b;
        if (i < ins) {
            int k = mate ? ins - 1 - i : i;
            uint8_t f = (uint8_t)SYN_ACGT[sm64((key ^ 0x5BD1E9955BD1E995ull) + (uint64_t)k) & 3];
            b = mate ? syn_comp(f) : f;
        } else {
            int j = i - ins;
            b = j < alen ? (uint8_t)ad[j] : (uint8_t)'G';
        }
        if (i >= L - polyg) b = 'G';
        uint64_t hm = sm64((key ^ (0xA5A5A5A5A5A5A5A5ull * (uint64_t)(2 + mate))) + (uint64_t)i);
        int q;
        if ((hm & 0x3FF) < 1) {
            b = 'N';
        } else if (((hm >> 10) & 0x3FF) < 3) {
            int idx = b == 'A' ? 0 : b == 'C' ? 1 : b == 'G' ? 2 : 3;
            b = (uint8_t)SYN_ACGT[(idx + 1 + (int)((hm >> 20) % 3)) & 3];
        }
        int n = (int)((hm >> 24) & 0xFF) + (int)((hm >> 32) & 0xFF) + (int)((hm >> 40) & 0xFF) - 382;
        q = (3600 - 6 * i + n * 300 / 128) / 100;
        if (q < 2) q = 2;
        if (q > 41) q = 41;
        if (i >= lowq) q = 2 + (int)((hm >> 48) % 11);
        if (b == 'N') q = 2;
        seq[i] = b;
        qual[i] = (uint8_t)(q + 33);
    }
}

void orc_synth_fill(const fq_batch* b, uint64_t seed, uint64_t first_index, int L) {
    for (int p = 0; p < b->n; ++p) {
        uint64_t idx = first_index + (uint64_t)p;
        uint64_t key = sm64(seed ^ (idx * 0xD1B54A32D192ED03ull));
        uint64_t r0 = sm64(key + 1);
        int64_t S = (int64_t)(r0 & 0xFFFF) + (int64_t)((r0 >> 16) & 0xFFFF) + (int64_t)((r0 >> 32) & 0xFFFF) +
                    (int64_t)((r0 >> 48) & 0xFFFF);
        int64_t ins = 220 + (S - 131070) * 60 / 37837;
        if (ins < 60) ins = 60;
        if (ins > 600) ins = 600;
        synth_read(key, 0, L, (int)ins, g_row[0], g_row[1]);
        fq_batch_put_row((uint8_t*)b->seq1, b->stride, p, g_row[0], L);
        fq_batch_put_row((uint8_t*)b->qual1, b->stride, p, g_row[1], L);
        ((uint16_t*)b->len1)[p] = (uint16_t)L;
        if (b->seq2) {
            synth_read(key, 1, L, (int)ins, g_row[0], g_row[1]);
            fq_batch_put_row((uint8_t*)b->seq2, b->stride, p, g_row[0], L);
            fq_batch_put_row((uint8_t*)b->qual2, b->stride, p, g_row[1], L);
            ((uint16_t*)b->len2)[p] = (uint16_t)L;
        }
    }
}

size_t orc_sizeof_params(void) { return sizeof(fq_params); }
size_t orc_sizeof_result(void) { return sizeof(fq_read_result); }
