// device_ops.h -- per-read operations of the hot path as gfx950 device functions.
//
// Each function restates one reference function (file:line cited) on a read *view*: the
// read's bytes stay where they are in HBM (fq_batch rows) and trimming only moves
// (start, len).  Quality bytes are signed char, as std::string's char on x86-64.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fqengine.h"

namespace fqdev {

// A read's row in a batch plane (chunk-interleaved tiles, include/fqengine.h): byte j sits at
// base[(j / 16) * 512 + j % 16], base = the read's chunk 0.  Indexable and offsettable like a
// pointer, so the restatements below run on it unchanged.
struct Row {
    const uint8_t* base;
    int off;
    __device__ __forceinline__ uint8_t operator[](int i) const {
        const int j = off + i;
        return base[(j >> 4) * (FQ_TILE_READS * FQ_CHUNK) + (j & 15)];
    }
    __device__ __forceinline__ Row operator+(int k) const { return Row{base, off + k}; }
};
__device__ __forceinline__ Row batch_row(const uint8_t* plane, int stride, int idx) {
    return Row{plane + (size_t)(idx / FQ_TILE_READS) * FQ_TILE_READS * stride + (idx % FQ_TILE_READS) * FQ_CHUNK, 0};
}


// Accumulator layout of include/fqengine.h, usable in device code.
__device__ __forceinline__ size_t acc_stats_words(int max_cycles) {
    return (size_t)FQ_ST_CYCLES + (size_t)max_cycles * FQ_ST_PER_CYCLE;
}
__device__ __forceinline__ size_t acc_stats_offset(int insert_size_max, int max_cycles, int k) {
    size_t base = (size_t)FQ_ACC_INSERT + (size_t)(insert_size_max + 1);
    base = (base + 15) & ~(size_t)15;
    return base + (size_t)k * acc_stats_words(max_cycles);
}

template <class P>
__device__ __forceinline__ int qv(P q, int i) { return (int)(int8_t)q[i]; }

__device__ __forceinline__ uint8_t comp(uint8_t c) {
    // Seq::reverseComplement, reference src/seq.h:24-48
    switch (c) {
        case 'A': case 'a': return 'T';
        case 'T': case 't': return 'A';
        case 'C': case 'c': return 'G';
        case 'G': case 'g': return 'C';
        default: return 'N';
    }
}

// The decision part of Filter::passFilter (reference src/filter.cpp:29-51) from the three
// counts of its scan; `diffs` lazily counts seq[i] != seq[i+1] for the complexity filter
// (Filter::passLowComplexityFliter, src/filter.cpp:54-67).
template <class Diffs>
__device__ inline int filter_verdict(const fq_params& p, int rlen, int low, int nb, int tq, Diffs diffs) {
    if (p.qual_filter_enabled) {
        if (low > p.low_qual_base_limit) return FQ_FAIL_QUALITY;
        if (p.avg_qual_limit > 0 && p.avg_qual_limit > (double)tq / rlen) return FQ_FAIL_QUALITY;
    }
    if (p.qual_filter_enabled && nb > p.n_base_limit) return FQ_FAIL_N_BASE;
    if (p.length_filter_enabled) {
        if (rlen < p.min_len) return FQ_FAIL_LENGTH;
        if (p.max_len > 0 && rlen > p.max_len) return FQ_FAIL_TOO_LONG;
    }
    if (p.complexity_enabled) {
        bool ok = false;
        if (rlen > 1) ok = (double)diffs() / (rlen - 1) >= p.complexity_threshold;
        if (!ok) return FQ_FAIL_COMPLEXITY;
    }
    return FQ_PASS_FILTER;
}

// Accessors: every operation below reads bytes through functors seq(i) -> uint8_t and
// qual(i) -> int (signed char value), so the same restatement runs on HBM rows (v1 kernel)
// and on LDS-staged columns (v2 kernel).
template <class P>
struct PtrQual {
    P p;
    __device__ __forceinline__ int operator()(int i) const { return (int)(int8_t)p[i]; }
};
struct LdsQual {  // quality byte i (signed, as the reference's char) of a row packed 4 per LDS word
    const uint32_t* row;
    __device__ __forceinline__ int operator()(int i) const { return (int)(int8_t)(row[i >> 2] >> ((i & 3) * 8)); }
    __device__ __forceinline__ uint32_t word(int wi) const { return row[wi]; }
};
// Quality byte i of a batch row read straight from HBM/L2 (chunk-interleaved tile layout), with
// dword access for the word-wise window scan; words past the row's stride are clamped.
struct RowQual {
    const uint8_t* q;  // the row's chunk 0
    int nwords;        // stride / 4
    __device__ __forceinline__ int operator()(int i) const {
        return (int)(int8_t)q[(i >> 4) * (FQ_TILE_READS * FQ_CHUNK) + (i & 15)];
    }
    __device__ __forceinline__ uint32_t word(int wi) const {
        wi = min(wi, nwords - 1);
        return *reinterpret_cast<const uint32_t*>(q + (wi >> 2) * (FQ_TILE_READS * FQ_CHUNK) + 4 * (wi & 3));
    }
};
template <class P>
struct Bytes {
    P p;
    __device__ __forceinline__ uint8_t operator()(int i) const { return p[i]; }
};
template <class A>
struct Offset {  // window view: a(off + i)
    A a;
    int off;
    __device__ __forceinline__ auto operator()(int i) const { return a(off + i); }
};
template <class A>
__device__ __forceinline__ Offset<A> at(A a, int off) { return Offset<A>{a, off}; }

// Filter::passFilter, reference src/filter.cpp:3-52
template <class SQ, class QQ>
__device__ inline int pass_filter_t(const fq_params& p, SQ seq, QQ qual, int rlen, bool is_null) {
    if (is_null || rlen == 0) return FQ_FAIL_LENGTH;
    int low = 0, nb = 0, tq = 0;
    if (p.qual_filter_enabled || p.length_filter_enabled) {
        for (int i = 0; i < rlen; ++i) {
            int q = qual(i);
            tq += q - 33;
            nb += seq(i) == 'N';
            low += q < p.low_qual_limit;
        }
    }
    return filter_verdict(p, rlen, low, nb, tq, [&]() {
        int diff = 0;
        for (int i = 0; i < rlen - 1; ++i) diff += seq(i) != seq(i + 1);
        return diff;
    });
}

// (double)T/(double)w >= X  <=>  T >= X*w for integer T, X and 1 <= w <= 1000 (the quotient is
// correctly rounded and X - 1/w is never rounded up to X), so the sliding windows of
// Filter::trimAndCut are evaluated exactly in integers.
__device__ __forceinline__ bool win_ge(int total, int w, int x) { return total >= x * w; }

// The forward sliding-window scans of Filter::trimAndCut (cut_front src/filter.cpp:93-122, cut_right
// :124-152): the first s in [s0, send) whose window sum q[s..s+w-1] satisfies (sum >= T) == WANT,
// or send when there is none.
template <bool WANT, class QQ>
__device__ inline int window_scan(QQ qual, int s0, int send, int w, int T) {
    int tot = 0;
    for (int i = 0; i < w - 1; ++i) tot += qual(s0 + i);
    int s = s0;
    for (; s < send; ++s) {
        tot += qual(s + w - 1);
        if (s > s0) tot -= qual(s - 1);
        if (win_ge(tot, w, T) == WANT) break;
    }
    return s;
}

// The same scan over an LDS row, 4 positions per step: the added (q[s+w-1]) and removed (q[s-1])
// bytes arrive as words realigned with v_alignbyte, one LDS word per stream per step, prefetched
// one step ahead (the byte loop waits out the LDS latency at every position).
// (the row's dwords: LdsQual from its LDS row, RowQual from HBM/L2)
template <bool WANT, class WQ>
__device__ inline int window_scan_words(WQ qual, int s0, int send, int w, int T) {
    if (s0 >= send) return send;
    const int TW = T * w;
    int tot = 0;
    for (int i = 0; i < w; ++i) tot += qual(s0 + i);
    if ((tot >= TW) == WANT) return s0;
    int oa = s0 + w, orr = s0;  // byte offsets of q[s+w-1] and q[s-1] for s = s0 + 1
    const uint32_t sha = oa & 3, shr = orr & 3;
    int pa = oa >> 2, pr = orr >> 2;  // dword indices
    uint32_t alo = qual.word(pa), ahi = qual.word(pa + 1), rlo = qual.word(pr), rhi = qual.word(pr + 1);
    for (int s = s0 + 1; s < send; s += 4) {
        const uint32_t an = qual.word(pa + 2), rn = qual.word(pr + 2);
        const uint32_t aw = __builtin_amdgcn_alignbyte(ahi, alo, sha);
        const uint32_t rw = __builtin_amdgcn_alignbyte(rhi, rlo, shr);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            tot += ((int)(aw << (24 - 8 * k)) >> 24) - ((int)(rw << (24 - 8 * k)) >> 24);
            if (s + k < send && (tot >= TW) == WANT) return s + k;
        }
        alo = ahi;
        ahi = an;
        rlo = rhi;
        rhi = rn;
        ++pa;
        ++pr;
    }
    return send;
}
template <bool WANT>
__device__ inline int window_scan(LdsQual qual, int s0, int send, int w, int T) {
    return window_scan_words<WANT>(qual, s0, send, w, T);
}
template <bool WANT>
__device__ inline int window_scan(RowQual qual, int s0, int send, int w, int T) {
    return window_scan_words<WANT>(qual, s0, send, w, T);
}

// cut_right's scan (src/filter.cpp:124-152) restricted to the windows that can be low: a window
// whose mean is below T holds at least one base below T, so only windows overlapping a 16-position
// chunk with such a base (bit c of low_chunks) are scanned, in order; the others are skipped.
// The first low window in [s0, send) is the same as window_scan<false>'s (send if none).
template <class QQ>
__device__ inline int low_window_scan(QQ qual, int s0, int send, int w, int T, uint32_t low_chunks) {
    int from = s0;
    while (low_chunks) {
        const int c = __builtin_ctz(low_chunks);
        low_chunks &= low_chunks - 1;
        const int a = max(from, 16 * c - w + 1), b = min(send, 16 * c + 16);  // windows overlapping chunk c
        if (a < b) {
            const int r = window_scan<false>(qual, a, b, w, T);
            if (r < b) return r;
        }
        from = max(from, b);
        if (from >= send) break;
    }
    return send;
}

// Filter::trimAndCut, reference src/filter.cpp:69-189. Returns false for NULL.
// low_chunks: bit c set when chunk c (positions [16c, 16c+16)) may hold a quality below cut_right's
// threshold (~0u: unknown, every window is scanned).
template <class SQ, class QQ>
__device__ inline bool trim_and_cut_t(const fq_params& p, SQ seq, QQ qual, int l, int front, int tail,
                                      int& out_start, int& out_len, uint32_t low_chunks = ~0u) {
    const bool enF = p.cut_front, enR = p.cut_right, enT = p.cut_tail;
    if (front == 0 && tail == 0 && !enF && !enR && !enT) {
        out_start = 0;
        out_len = l;
        return true;
    }
    int rlen = l - front - tail;
    if (rlen < 0) return false;
    if (!enF && !enR && !enT) {
        out_start = front;  // resize(rlen) when front == 0, else substr(front, rlen)
        out_len = rlen;
        return true;
    }
    if (enF) {
        const int w = p.cut_front_window, thr = 33 + p.cut_front_quality;
        if (l - front - tail - w <= 0) return false;
        int s = window_scan<true>(qual, front, l - tail - w, w, thr);
        if (s > 0) s = s + w - 1;
        while (s < l && seq(s) == 'N') ++s;
        front = s;
        rlen = l - front - tail;
    }
    if (enR) {
        const int w = p.cut_right_window, thr = 33 + p.cut_right_quality;
        if (l - front - tail - w <= 0) return false;
        int s = low_chunks == ~0u ? window_scan<false>(qual, front, l - tail - w, w, thr)
                                  : low_window_scan(qual, front, l - tail - w, w, thr, low_chunks);
        if (s < l - tail - w) {
            while (s < l - 1 && qual(s) >= thr) ++s;
            rlen = s - front;
        }
    }
    if (!enR && enT) {
        const int w = p.cut_tail_window, thr = 33 + p.cut_tail_quality;
        if (l - front - tail - w <= 0) return false;
        int tot = 0;
        int t = l - tail - 1;
        for (int i = 0; i < w - 1; ++i) tot += qual(t - i);
        for (t = l - tail - 1; t - w >= front; --t) {
            tot += qual(t - w + 1);
            if (t < l - tail - 1) tot -= qual(t + 1);
            if (win_ge(tot, w, thr)) break;
        }
        if (t < l - 1) t = t - w + 1;
        while (t >= 0 && seq(t) == 'N') --t;
        rlen = t - front + 1;
    }
    if (rlen <= 0 || front >= l - 1) return false;
    out_start = front;
    out_len = min(rlen, l - front);
    return true;
}

// PolyX::trimPolyG, reference src/polyx.cpp:14-38. Returns new length; bases < 0: not recorded.
template <class SQ>
__device__ inline int trim_polyg_t(SQ d, int rlen, int compareReq, int maxMM, int per, int& bases) {
    int mismatch = 0, i = 0, firstG = rlen - 1;
    for (i = 0; i < rlen; ++i) {
        if (d(rlen - i - 1) != 'G') ++mismatch;
        else firstG = rlen - i - 1;
        int allowed = min(maxMM, max(1, (i + 1) / per));
        if (mismatch > allowed) break;
    }
    bases = -1;
    if (i + 1 >= compareReq) {
        bases = rlen - firstG;
        return (firstG > rlen || firstG < 0) ? rlen : firstG;  // Read::resize, src/read.h:181-187
    }
    return rlen;
}

// PolyX::trimPolyX, reference src/polyx.cpp:45-101
template <class SQ>
__device__ inline int trim_polyx_t(SQ d, int rlen, int mask, int compareReq, int maxMM, int per, int& poly_out,
                                   int& bases) {
    int cnt[5] = {0, 0, 0, 0, 0};
    int pos = 0;
    for (pos = 0; pos < rlen; ++pos) {
        uint8_t c = d(rlen - 1 - pos);
        int k = c == 'A' ? 0 : c == 'T' ? 1 : c == 'C' ? 2 : c == 'G' ? 3 : 4;
#pragma unroll
        for (int b = 0; b < 5; ++b) cnt[b] += (k == b);
        int cmp = pos + 1;
        int allowed = min(maxMM, max(1, cmp / per));
        bool brk = true;
#pragma unroll
        for (int b = 0; b < 5; ++b)
            if (((mask >> b) & 1) && cmp - cnt[b] <= allowed) brk = false;
        if (brk) break;
    }
    poly_out = -1;
    bases = 0;
    if (pos + 1 >= compareReq) {
        int poly = 0, maxCount = -1;
#pragma unroll
        for (int b = 0; b < 5; ++b)
            if (((mask >> b) & 1) && cnt[b] > maxCount) {
                maxCount = cnt[b];
                poly = b;
            }
        const uint8_t polyBase = poly == 0 ? 'A' : poly == 1 ? 'T' : poly == 2 ? 'C' : poly == 3 ? 'G' : 'N';
        pos = min(rlen - 1, pos);
        while (pos > 0 && d(rlen - pos - 1) != polyBase) --pos;
        int target = rlen - pos - 1;
        poly_out = poly;
        bases = pos + 1;
        return (target > rlen || target < 0) ? rlen : target;
    }
    return rlen;
}

// Pointer-like wrappers (general kernel): P is a Row (or a plain byte pointer).
template <class P>
__device__ inline int pass_filter(const fq_params& p, P seq, P qual, int rlen, bool is_null) {
    return pass_filter_t(p, Bytes<P>{seq}, PtrQual<P>{qual}, rlen, is_null);
}
template <class P>
__device__ inline bool trim_and_cut(const fq_params& p, P seq, P qual, int l, int front, int tail, int& st, int& n) {
    return trim_and_cut_t(p, Bytes<P>{seq}, PtrQual<P>{qual}, l, front, tail, st, n);
}
template <class P>
__device__ inline int trim_polyg(P d, int rlen, int compareReq, int maxMM, int per, int& bases) {
    return trim_polyg_t(Bytes<P>{d}, rlen, compareReq, maxMM, per, bases);
}
template <class P>
__device__ inline int trim_polyx(P d, int rlen, int mask, int compareReq, int maxMM, int per, int& poly, int& bases) {
    return trim_polyx_t(Bytes<P>{d}, rlen, mask, compareReq, maxMM, per, poly, bases);
}

struct Overlap {
    int overlapped, offset, len, diff;
};

// OverlapAnalysis::analyze, reference src/overlapanalysis.cpp:7-72, on views.
// revcomp(s2)[i] = comp(s2[len2-1-i]) is formed on the fly.
template <class P>
__device__ inline Overlap analyze(P s1, int len1, P s2, int len2, int limit, int require) {
    const int ccr = 50;
    Overlap r;
    for (int offset = 0; offset < len1 - require; ++offset) {
        int ol = min(len1 - offset, len2);
        int diff = 0, i = 0;
        for (i = 0; i < ol; ++i) {
            if (s1[offset + i] != comp(s2[len2 - 1 - i])) {
                ++diff;
                if (diff >= limit && i < ccr) break;
            }
        }
        if (diff < limit || (diff >= limit && i > ccr)) {
            r.overlapped = 1;
            r.offset = offset;
            r.len = ol;
            r.diff = diff;
            return r;
        }
    }
    for (int offset = 0; offset > require - len2; --offset) {
        int ol = min(len1, len2 + offset);
        int diff = 0, i = 0;
        for (i = 0; i < ol; ++i) {
            if (s1[i] != comp(s2[len2 - 1 - (i - offset)])) {
                ++diff;
                if (diff >= limit && i < ccr) break;
            }
        }
        if (diff < limit || (diff >= limit && i > ccr)) {
            r.overlapped = 1;
            r.offset = offset;
            r.len = ol;
            r.diff = diff;
            return r;
        }
    }
    r.overlapped = r.offset = r.len = r.diff = 0;
    return r;
}

// AdapterTrimmer::trimBySequence search, reference src/adaptertrimmer.cpp:29-90
template <class SQ>
__device__ inline bool trim_by_sequence_t(SQ r, int rlen, const uint8_t* ad, int alen, int& pos_out) {
    if (alen < 4) return false;
    int start = 0;
    if (alen >= 16) start = -4;
    else if (alen >= 12) start = -3;
    else if (alen >= 8) start = -2;
    for (int pos = start; pos < rlen - 4; ++pos) {
        int cmplen = min(rlen - pos, alen);
        int allowed = cmplen / 8;
        int mm = 0;
        bool matched = true;
        for (int i = max(0, -pos); i < cmplen; ++i) {
            if (ad[i] != r(i + pos)) {
                if (++mm > allowed) {
                    matched = false;
                    break;
                }
            }
        }
        if (matched) {
            pos_out = pos;
            return true;
        }
    }
    return false;
}
template <class P>
__device__ inline bool trim_by_sequence(P r, int rlen, const uint8_t* ad, int alen, int& pos_out) {
    return trim_by_sequence_t(Bytes<P>{r}, rlen, ad, alen, pos_out);
}

}  // namespace fqdev
