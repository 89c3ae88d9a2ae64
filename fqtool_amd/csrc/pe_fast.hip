// pe_fast.hip -- v2 hot path for paired-end packs on gfx950 (everything except -m merge).
//
// Mapping: one workgroup = 8 waves, one wave = a tile of 32 pairs, one LANE = one READ
// (lanes 0-31 read 1, lanes 32-63 read 2 of the same pairs), so every per-read operation of
// PairEndProcessor::processPairEnd (reference src/peprocessor.cpp:261-508) keeps all 64 lanes
// busy and the two mates of a pair are lanes l and l^32 of the same wave.
//
// Staging: each lane streams its seq row from HBM with 16-byte loads into its own LDS column
// (word (field*64 + lane): conflict-free for any per-lane position) and derives, in registers,
//   * a 2-bit base code per position (A=0 C=1 T=2 G=3, N=3, i.e. (byte>>1)&3) and
//   * an N mask (one bit per position, spaced to line up with the 2-bit codes),
// read 1 forward, read 2 already reverse-complemented (the orientation OverlapAnalysis::analyze
// compares, src/overlapanalysis.cpp:7-72).  Qualities stay in HBM/L2 and are re-read per pass.
// A tile whose bases are not all in {A,C,G,T,N}, whose quality bytes are >= 128, or whose
// reads are longer than 160 is handed to the general kernel (pe_kernel.hip) through a
// device-side tile list, so the fast path may assume that alphabet.
//
// Overlap analysis: for every candidate offset a lane compares 16 positions at once on the
// 2-bit codes (equal bytes => equal codes, so the code mismatch count is a lower bound of the
// byte mismatch count and rejecting at >= max(limit,1) is exact); the first surviving offset
// is verified exactly with codes + N masks (equal bases <=> equal code and equal N bit on this
// alphabet) applying the reference's break/accept rule.  Read 1's lane scans phase 1
// (offset >= 0), read 2's lane phase 2 (offset <= 0); the pair's answer is phase 1's if any.
//
// Statistics: Stats::statRead (src/stats.cpp:237-295) per cycle and base class into
// workgroup-private LDS histograms of u64 cells (count << 40 | sum(q+128)); each lane walks its
// read's dwords from a lane-dependent rotation so the wave's 64 atomics spread over cycles.
// Post-filter stats are accumulated as "removed" (pre minus what survives) when the surviving
// window always starts at 0, which touches only trimmed tails and failed reads.
#include <hip/hip_runtime.h>

#include "device_ops.h"
#include "engine_internal.h"

using namespace fqdev;

namespace {

constexpr int kWaves = 8;
constexpr int kBlock = 64 * kWaves;
constexpr int kMaxLen = 160;
constexpr int kRawW = kMaxLen / 4;          // raw seq dwords per lane column
constexpr int kCodeW = kMaxLen / 16;        // 2-bit code dwords (16 positions each)
constexpr int kColW = kRawW + 2 * kCodeW;   // words per lane column: raw | codes | N mask
constexpr int kCellW = 12;                  // u32 words per cycle: 6 slots x u64
constexpr int kGroupW = 4 * kCellW + 2;     // words per 4 cycles (+2 pad spreads LDS banks)
constexpr int kHistW = (kMaxLen / 4) * kGroupW;
constexpr int kSmallU64 = FQ_ACC_INSERT + 512 + 1;
constexpr int kSmallW = 2 * ((kSmallU64 + 1) & ~1);
constexpr int kScalW = 2 * 16;  // [4 stats][reads, length_sum, q20, q30] u64
constexpr int kAdW = 2 * FQ_MAX_ADAPTER / 4;
constexpr int kColsW = kWaves * kColW * 64;
constexpr int kLdsWords = kColsW + 4 * kHistW + kSmallW + kScalW + kAdW;
static_assert(kLdsWords * 4 <= 160 * 1024, "LDS budget");

constexpr unsigned long long kCount1 = 1ull << 40;
constexpr unsigned long long kQMask = kCount1 - 1;

__device__ __forceinline__ uint32_t pack4(uint32_t x) { return (x | (x >> 6) | (x >> 12) | (x >> 18)) & 0xFFu; }

// reverse the order of the 16 two-bit fields of a word
__device__ __forceinline__ uint32_t pairrev(uint32_t x) {
    uint32_t y = __builtin_bitreverse32(x);
    return ((y >> 1) & 0x55555555u) | ((y & 0x55555555u) << 1);
}

__device__ __forceinline__ uint32_t fold2(uint32_t x) { return (x | (x >> 1)) & 0x55555555u; }

// low `n` two-bit positions (spaced mask), n may be <= 0 or >= 16
__device__ __forceinline__ uint32_t posmask(int n) {
    return n >= 16 ? 0x55555555u : n <= 0 ? 0u : (((1u << (2 * n)) - 1u) & 0x55555555u);
}

// byte mask of the first `n` bytes of a dword
__device__ __forceinline__ uint32_t bytemask(int n) {
    return n >= 4 ? 0xFFFFFFFFu : n <= 0 ? 0u : ((1u << (8 * n)) - 1u);
}

struct LdsSeq {  // raw byte i of a lane column
    const uint32_t* col;
    int c;
    __device__ __forceinline__ uint8_t operator()(int i) const {
        return (uint8_t)(col[(i >> 2) * 64 + c] >> ((i & 3) * 8));
    }
};

// 16 two-bit code positions [pos, pos+16) of field `f` (codes or N mask) of column c
__device__ __forceinline__ uint32_t code_window(const uint32_t* col, int f, int c, int pos) {
    const int w = pos >> 4, sh = 2 * (pos & 15);
    const uint32_t lo = w < kCodeW ? col[(f + w) * 64 + c] : 0u;
    const uint32_t hi = w + 1 < kCodeW ? col[(f + w + 1) * 64 + c] : 0u;
    return __builtin_amdgcn_alignbit(hi, lo, sh);
}

struct OvOut {
    bool found;
    int off, ol, diff;
};

// Exact OverlapAnalysis acceptance test at one offset (src/overlapanalysis.cpp:24-40 / :49-65):
// positions compare r1 codes from p1 with rc2 codes from p2 over `ol` positions.
__device__ inline bool ov_exact(const uint32_t* col, int c1, int p1, int c2, int p2, int ol, int limit, int K,
                                int& diff_out) {
    int d50 = 0, D = 0;
    const int nw = (ol + 15) >> 4;
    for (int j = 0; j < nw; ++j) {
        const uint32_t a = code_window(col, kRawW, c1, p1 + 16 * j);
        const uint32_t b = code_window(col, kRawW, c2, p2 + 16 * j);
        const uint32_t wa = code_window(col, kRawW + kCodeW, c1, p1 + 16 * j);
        const uint32_t wb = code_window(col, kRawW + kCodeW, c2, p2 + 16 * j);
        const uint32_t mism = (fold2(a ^ b) & ~(wa | wb)) | (wa ^ wb);
        D += __popc(mism & posmask(ol - 16 * j));
        d50 += __popc(mism & posmask(min(ol, 50) - 16 * j));
    }
    diff_out = D;
    // break (rejection) happens iff the K-th mismatch lies within the first min(ol,50) positions
    if (d50 >= K) return false;
    return D < limit || ol > 50;
}

// Scan one phase: offsets k = k0 .. cnt-1 move a 16-position window of column `cm` starting at
// code position mpos0 + k against the fixed 16-position word `fixed`; returns the first offset
// whose code-level lower bound is < K (or -1).  ol(k) = min(olA - k, olB).
__device__ inline int ov_scan(const uint32_t* col, int cm, int mpos0, int k0, int cnt, uint32_t fixed, int olA,
                              int olB, int K) {
    for (int k = k0; k < cnt;) {
        const int P = mpos0 + k;
        const int w = P >> 4;
        const uint32_t lo = w < kCodeW ? col[(kRawW + w) * 64 + cm] : 0u;
        const uint32_t hi = w + 1 < kCodeW ? col[(kRawW + w + 1) * 64 + cm] : 0u;
        uint32_t bits = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            // window starting at absolute position 16w + r
            const uint32_t win = r == 0 ? lo : __builtin_amdgcn_alignbit(hi, lo, 2 * r);
            const int kk = 16 * w + r - mpos0;
            const int ol = min(olA - kk, olB);
            const int lb = __popc(fold2(win ^ fixed) & posmask(ol));
            bits |= (uint32_t)(lb < K) << r;
        }
        // keep offsets within [k, cnt)
        const int first_r = P & 15;
        bits &= ~((1u << first_r) - 1u);
        const int last = cnt - 1 - (16 * w - mpos0);  // last valid r
        if (last < 15) bits &= (last < 0) ? 0u : ((2u << last) - 1u);
        if (bits) return 16 * w + (__ffs(bits) - 1) - mpos0;
        k = 16 * (w + 1) - mpos0;
    }
    return -1;
}

__device__ __forceinline__ void sadd(unsigned long long* p, unsigned long long v) { atomicAdd(p, v); }

__global__ void __launch_bounds__(kBlock) pe_fast_kernel(fq_params p, fq_batch b, fq_read_result* __restrict__ res,
                                                         unsigned long long* __restrict__ acc, int* __restrict__ slow_tiles,
                                                         int* __restrict__ slow_count) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* col = lds + wave * kColW * 64;
    uint32_t* hist = lds + kColsW;  // [pre1, pre2, aux1, aux2] x kHistW
    unsigned long long* small = reinterpret_cast<unsigned long long*>(hist + 4 * kHistW);
    unsigned long long* scal = small + kSmallW / 2;
    uint8_t* adp = reinterpret_cast<uint8_t*>(scal + 16);
    for (int i = threadIdx.x; i < 4 * kHistW + kSmallW + kScalW; i += kBlock) hist[i] = 0;
    for (int i = threadIdx.x; i < 2 * FQ_MAX_ADAPTER; i += kBlock)
        adp[i] = i < FQ_MAX_ADAPTER ? p.adapter1[i] : p.adapter2[i - FQ_MAX_ADAPTER];
    __syncthreads();

    const int mate = lane >> 5, pl = lane & 31;
    const int mlane = lane ^ 32;
    // Profiling-only ablation bits (fq_params.reserved[0]; results are wrong when set):
    // 1 skip overlap, 2 skip passFilter scan, 4 skip stats pass, 8 skip polyG, 16 skip LDS atomics
    const int abl = p.reserved[0];
    const bool removed_mode = p.trim_front1 == 0 && p.trim_front2 == 0 && !p.cut_front;
    const int ntiles = (b.n + 31) >> 5;
    const int nchunks = min(kCodeW, b.stride >> 4);
    const int limit = p.overlap_diff_limit;
    const int K = max(limit, 1);
    const int front = mate ? p.trim_front2 : p.trim_front1;
    const int tail = mate ? p.trim_tail2 : p.trim_tail1;
    const uint8_t* my_ad = adp + (mate ? FQ_MAX_ADAPTER : 0);
    const int my_alen = mate ? p.adapter2_len : p.adapter1_len;
    const int my_maxlen = mate ? p.max_len2 : p.max_len1;
    uint32_t* my_pre = hist + mate * kHistW;
    uint32_t* my_aux = hist + (2 + mate) * kHistW;
    unsigned long long s_pre[4] = {0, 0, 0, 0}, s_aux[4] = {0, 0, 0, 0};

    for (int t = blockIdx.x * kWaves + wave; t < ntiles; t += gridDim.x * kWaves) {
        const int idx = t * 32 + pl;
        const bool valid = idx < b.n;
        const size_t roff = (size_t)(valid ? idx : 0) * b.stride;
        const uint8_t* S = (mate ? b.seq2 : b.seq1) + roff;
        const uint8_t* Q = (mate ? b.qual2 : b.qual1) + roff;
        const int L = valid ? (int)(mate ? b.len2[idx] : b.len1[idx]) : 0;

        // ---------------- staging ----------------
        bool odd = L > kMaxLen || L > p.max_cycles || L > (nchunks << 4);
        uint32_t exo = 0, qhi = 0;
        uint32_t fc[kCodeW], fw[kCodeW];
#pragma unroll
        for (int k = 0; k < kCodeW; ++k) {
            fc[k] = 0;
            fw[k] = 0;
            if (k < nchunks && valid && !odd) {
                const uint4 s4 = *reinterpret_cast<const uint4*>(S + 16 * k);
                const uint4 q4 = *reinterpret_cast<const uint4*>(Q + 16 * k);
                const uint32_t sw[4] = {s4.x, s4.y, s4.z, s4.w};
                const uint32_t qw[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    col[(4 * k + j) * 64 + lane] = sw[j];
                    const uint32_t bm = bytemask(L - (16 * k + 4 * j));
                    const uint32_t kk = (sw[j] >> 1) & 0x07070707u;
                    // canonical byte for the 3-bit key: A C T G (0-3), N (7)
                    const uint32_t canon = __builtin_amdgcn_perm(0x4E000000u, 0x47544341u, kk);
                    exo |= (canon ^ sw[j]) & bm;
                    qhi |= qw[j] & bm;
                    fc[k] |= pack4(kk & 0x03030303u) << (8 * j);
                    fw[k] |= pack4((kk >> 2) & 0x01010101u) << (8 * j);
                }
            }
        }
        const bool bad = odd || exo != 0 || (qhi & 0x80808080u) != 0;
        if (__any(bad)) {
            if (lane == 0) slow_tiles[atomicAdd(slow_count, 1)] = t;
            continue;
        }
        if (mate == 0) {
#pragma unroll
            for (int k = 0; k < kCodeW; ++k) {
                col[(kRawW + k) * 64 + lane] = fc[k];
                col[(kRawW + kCodeW + k) * 64 + lane] = fw[k];
            }
        } else {
            // reverse-complement read 2's codes: rc[j] = comp(code[L-1-j]); N stays N (3)
#pragma unroll
            for (int m = 0; m < kCodeW; ++m) {
                col[(kRawW + m) * 64 + lane] = pairrev(fc[kCodeW - 1 - m]);
                col[(kRawW + kCodeW + m) * 64 + lane] = pairrev(fw[kCodeW - 1 - m]);
            }
            const int sh = kMaxLen - L, q = sh >> 4, r2 = 2 * (sh & 15);
            for (int m = 0; m < kCodeW; ++m) {
                const int a = m + q;
                const uint32_t clo = a < kCodeW ? col[(kRawW + a) * 64 + lane] : 0u;
                const uint32_t chi = a + 1 < kCodeW ? col[(kRawW + a + 1) * 64 + lane] : 0u;
                const uint32_t wlo = a < kCodeW ? col[(kRawW + kCodeW + a) * 64 + lane] : 0u;
                const uint32_t whi = a + 1 < kCodeW ? col[(kRawW + kCodeW + a + 1) * 64 + lane] : 0u;
                const uint32_t w = __builtin_amdgcn_alignbit(whi, wlo, r2);
                const uint32_t c = __builtin_amdgcn_alignbit(chi, clo, r2) ^ (0xAAAAAAAAu & ~(w << 1));
                col[(kRawW + m) * 64 + lane] = c;
                col[(kRawW + kCodeW + m) * 64 + lane] = w;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

        const LdsSeq seq{col, lane};
        const PtrQual qual{Q};

        // ---------------- trimAndCut (src/peprocessor.cpp:292-293) ----------------
        int st = 0, n = 0;
        bool nn = valid && trim_and_cut_t(p, seq, qual, L, front, tail, st, n);
        // the shuffle must run in every lane: ds_bpermute from a lane that is switched off returns
        // whatever its register held before (e.g. the previous tile's value)
        const int nn_o = __shfl_xor(nn ? 1 : 0, 32);
        const bool both = nn && nn_o != 0;
        fq_read_result rr;
        rr.flags = nn ? 0 : FQ_RF_NULL;
        rr.code = 0;
        rr.ad_pos = rr.ad_len = rr.m_len1 = rr.m_len2 = rr.reserved = 0;

        // ---------------- polyG (src/peprocessor.cpp:295-299) ----------------
        if (both && p.polyg_enabled && !(abl & 8)) {
            int bases;
            n = trim_polyg_t(at(seq, st), n, p.polyg_compare_req, p.polyg_max_mismatch, p.polyg_one_mismatch_per, bases);
            if (bases >= 0) {
                sadd(&small[FQ_ACC_POLYX_READS + 3], 1ull);
                sadd(&small[FQ_ACC_POLYX_BASES + 3], (unsigned long long)(long long)bases);
            }
        }

        // ---------------- overlap + adapters (src/peprocessor.cpp:302-333) ----------------
        if (both && !(abl & 1)) {
            const int st_o = __shfl_xor(st, 32), n_o = __shfl_xor(n, 32), L_o = __shfl_xor(L, 32);
            const int st1 = mate ? st_o : st, n1 = mate ? n_o : n;
            const int st2 = mate ? st : st_o, n2 = mate ? n : n_o, L2 = mate ? L : L_o;
            const int c1 = mate ? mlane : lane, c2 = mate ? lane : mlane;
            const int off2 = L2 - st2 - n2;  // rc2 of the trimmed read starts here in rc coordinates
            const int req = p.overlap_require;
            OvOut mine{false, 0, 0, 0};
            if (mate == 0) {  // phase 1: offset o >= 0, r1 window moves, rc2 fixed
                const int cnt = max(0, n1 - req);
                const uint32_t fixed = code_window(col, kRawW, c2, off2);
                for (int k0 = 0;;) {
                    const int o = ov_scan(col, c1, st1, k0, cnt, fixed, n1, n2, K);
                    if (o < 0) break;
                    const int ol = min(n1 - o, n2);
                    int diff;
                    if (ov_exact(col, c1, st1 + o, c2, off2, ol, limit, K, diff)) {
                        mine = OvOut{true, o, ol, diff};
                        break;
                    }
                    k0 = o + 1;
                }
            } else {  // phase 2: offset -m <= 0, rc2 window moves, r1 fixed
                const int cnt = max(0, n2 - req);
                const uint32_t fixed = code_window(col, kRawW, c1, st1);
                for (int k0 = 0;;) {
                    const int m = ov_scan(col, c2, off2, k0, cnt, fixed, n2, n1, K);
                    if (m < 0) break;
                    const int ol = min(n1, n2 - m);
                    int diff;
                    if (ov_exact(col, c1, st1, c2, off2 + m, ol, limit, K, diff)) {
                        mine = OvOut{true, -m, ol, diff};
                        break;
                    }
                    k0 = m + 1;
                }
            }
            const int f_o = __shfl_xor(mine.found ? 1 : 0, 32);
            const int off_o = __shfl_xor(mine.off, 32), ol_o = __shfl_xor(mine.ol, 32), d_o = __shfl_xor(mine.diff, 32);
            const bool f1 = mate ? f_o != 0 : mine.found;
            const bool f2 = mate ? mine.found : f_o != 0;
            Overlap ov{0, 0, 0, 0};
            if (f1) ov = mate ? Overlap{1, off_o, ol_o, d_o} : Overlap{1, mine.off, mine.ol, mine.diff};
            else if (f2) ov = mate ? Overlap{1, mine.off, mine.ol, mine.diff} : Overlap{1, off_o, ol_o, d_o};
            if (mate == 0) {  // PairEndProcessor::statInsertSize, src/peprocessor.cpp:510-523
                int isize = p.insert_size_max;
                if (ov.overlapped) isize = ov.offset > 0 ? n1 + n2 - ov.len : ov.len;
                if (isize > p.insert_size_max) isize = p.insert_size_max;
                sadd(&small[FQ_ACC_INSERT + isize], 1ull);
            }
            if (p.adapter_trimming) {
                const int ol = ov.len;  // AdapterTrimmer::trimByOverlapAnalysis, src/adaptertrimmer.cpp:14-27
                if (ov.diff <= 5 && ov.overlapped && ov.offset < 0 && ol > n1 / 3) {
                    rr.flags |= FQ_RF_AD_OVERLAP;
                    rr.ad_pos = (uint16_t)(st + ol);
                    rr.ad_len = (uint16_t)(n - ol);
                    if (mate == 0) {
                        sadd(&small[FQ_ACC_ADAPTER_READS], 2ull);
                        sadd(&small[FQ_ACC_ADAPTER_BASES], (unsigned long long)((n1 - ol) + (n2 - ol)));
                    }
                    n = ol;
                } else if (my_alen > 0) {  // AdapterTrimmer::trimBySequence, src/adaptertrimmer.cpp:29-90
                    int pos;
                    if (trim_by_sequence_t(at(seq, st), n, my_ad, my_alen, pos)) {
                        int ad_len;
                        if (pos < 0) {
                            ad_len = my_alen + pos;
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
                        if (ad_len > 0) {
                            sadd(&small[FQ_ACC_ADAPTER_READS], 1ull);
                            sadd(&small[FQ_ACC_ADAPTER_BASES], (unsigned long long)ad_len);
                        }
                    }
                }
            }
        }

        // ---------------- polyX, maxLen (src/peprocessor.cpp:335-349) ----------------
        if (both && p.polyx_enabled) {
            int poly, bases;
            n = trim_polyx_t(at(seq, st), n, p.polyx_mask, p.polyx_compare_req, p.polyx_max_mismatch,
                             p.polyx_one_mismatch_per, poly, bases);
            if (poly >= 0) {
                sadd(&small[FQ_ACC_POLYX_READS + poly], 1ull);
                sadd(&small[FQ_ACC_POLYX_BASES + poly], (unsigned long long)(long long)bases);
            }
        }
        if (both && my_maxlen > 0 && my_maxlen < n) n = my_maxlen;

        // ---------------- passFilter (pass A, src/filter.cpp:3-52) ----------------
        int code = FQ_FAIL_LENGTH;
        if (nn && n > 0) {
            int low = 0, tq = 0, nb = 0;
            if ((p.qual_filter_enabled || p.length_filter_enabled) && !(abl & 2)) {
                const uint32_t limq = (uint32_t)(0x80 - p.low_qual_limit) * 0x01010101u;
                const int end = st + n;
                for (int c = st >> 4; c < ((end + 15) >> 4); ++c) {
                    const uint4 q4 = *reinterpret_cast<const uint4*>(Q + 16 * c);
                    const uint32_t qw[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int b0 = 16 * c + 4 * j;
                        const uint32_t bm = bytemask(end - b0) & ~bytemask(st - b0);
                        const uint32_t w = qw[j] & bm;
                        low += __popc(~((w & 0x7F7F7F7Fu) + limq) & 0x80808080u & bm);
                        tq = (int)__builtin_amdgcn_sad_u8(w, 0u, (uint32_t)tq);
                    }
                }
                tq -= 33 * n;
                // N count from the N mask (read 2's column is reverse-complemented)
                const int lo = mate ? L - st - n : st;
                for (int c = lo >> 4; c < ((lo + n + 15) >> 4); ++c) {
                    const uint32_t w = col[(kRawW + kCodeW + c) * 64 + lane];
                    nb += __popc(w & posmask(lo + n - 16 * c) & ~posmask(lo - 16 * c));
                }
            }
            code = filter_verdict(p, n, low, nb, tq, [&]() {
                int diff = 0;
                for (int i = 0; i < n - 1; ++i) diff += seq(st + i) != seq(st + i + 1);
                return diff;
            });
        }
        const int code_o = __shfl_xor(code, 32);
        const bool pair_pass = both && code == FQ_PASS_FILTER && code_o == FQ_PASS_FILTER;
        if (mate == 0 && valid) sadd(&small[FQ_ACC_FILTER + max(code, code_o)], 2ull);  // addFilterResult: +2

        // ---------------- Stats (pass B): pre, and removed/post ----------------
        if (valid && !(abl & 4)) {
            const int nd = (L + 3) >> 2;
            const int rot = nd ? lane % nd : 0;
            uint32_t q20 = 0, q30 = 0, a20 = 0, a30 = 0;
            for (int it = 0; it < nd; ++it) {
                int d = it + rot;
                if (d >= nd) d -= nd;
                const uint32_t sw = col[d * 64 + lane];
                const uint32_t qw = *reinterpret_cast<const uint32_t*>(Q + 4 * d);
                const uint32_t vm = bytemask(L - 4 * d);
                const uint32_t t20 = ((qw & 0x7F7F7F7Fu) + 0x4A4A4A4Au) & 0x80808080u;  // byte > '5'
                const uint32_t t30 = ((qw & 0x7F7F7F7Fu) + 0x40404040u) & 0x80808080u;  // byte > '?'
                q20 += __popc(t20 & vm);
                q30 += __popc(t30 & vm);
                uint32_t am;  // bytes that go to the aux histogram
                if (removed_mode) am = pair_pass ? (vm & ~bytemask(n - 4 * d)) : vm;
                else am = pair_pass ? (bytemask(st + n - 4 * d) & ~bytemask(st - 4 * d)) : 0u;
                a20 += __popc(t20 & am);
                a30 += __popc(t30 & am);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (((vm >> (8 * j)) & 1u) && !(abl & 16)) {
                        const uint32_t cls = (sw >> (8 * j)) & 7u;
                        const uint32_t slot = (cls * 3u) & 7u;
                        const unsigned long long v = kCount1 | (unsigned long long)(((qw >> (8 * j)) & 0xFFu) ^ 0x80u);
                        const int cell = d * kGroupW + j * kCellW + 2 * (int)slot;
                        atomicAdd(reinterpret_cast<unsigned long long*>(my_pre + cell), v);
                        if ((am >> (8 * j)) & 1u) {
                            const int c = removed_mode ? 4 * d + j : 4 * d + j - st;
                            const int acell = (c >> 2) * kGroupW + (c & 3) * kCellW + 2 * (int)slot;
                            atomicAdd(reinterpret_cast<unsigned long long*>(my_aux + acell), v);
                        }
                    }
                }
            }
            s_pre[0] += 1;
            s_pre[1] += (unsigned long long)L;
            s_pre[2] += q20;
            s_pre[3] += q30;
            if (removed_mode) {
                s_aux[0] += pair_pass ? 0 : 1;
                s_aux[1] += (unsigned long long)(pair_pass ? L - n : L);
            } else {
                s_aux[0] += pair_pass ? 1 : 0;
                s_aux[1] += (unsigned long long)(pair_pass ? n : 0);
            }
            s_aux[2] += a20;
            s_aux[3] += a30;
        }
        if (valid) {

            rr.start = nn ? (uint16_t)st : 0;
            rr.len = nn ? (uint16_t)n : 0;
            rr.code = (uint8_t)code;
            if (res) *reinterpret_cast<uint4*>(&res[2 * (size_t)idx + mate]) = *reinterpret_cast<const uint4*>(&rr);
        }
    }

    // per-lane stats scalars -> LDS
#pragma unroll
    for (int f = 0; f < 4; ++f) {
        if (s_pre[f]) sadd(&scal[4 * mate + f], s_pre[f]);
        if (s_aux[f]) sadd(&scal[4 * (2 + mate) + f], s_aux[f]);
    }
    __syncthreads();

    // ---------------- flush to the global accumulator ----------------
    const int nsmall = FQ_ACC_INSERT + p.insert_size_max + 1;
    for (int i = threadIdx.x; i < nsmall; i += kBlock)
        if (small[i]) atomicAdd(&acc[i], small[i]);
    const size_t st_base = acc_stats_offset(p.insert_size_max, p.max_cycles, 0);
    const size_t st_words = acc_stats_words(p.max_cycles);
    if (threadIdx.x < 16) {
        const int k = threadIdx.x >> 2, f = threadIdx.x & 3;
        unsigned long long v = scal[threadIdx.x];
        if (k >= 2 && removed_mode) v = scal[threadIdx.x - 8] - v;  // post = pre - removed
        if (v) atomicAdd(&acc[st_base + k * st_words + f], v);
    }
    const int ncyc = min(kMaxLen, p.max_cycles);
    for (int i = threadIdx.x; i < 4 * ncyc * 6; i += kBlock) {
        const int k = i / (ncyc * 6);
        const int rem = i - k * ncyc * 6;
        const int c = rem / 6, slot = rem - c * 6;
        if (slot == 0) continue;
        const int cell = (c >> 2) * kGroupW + (c & 3) * kCellW + 2 * slot;
        const unsigned long long v = *reinterpret_cast<const unsigned long long*>(hist + k * kHistW + cell);
        long long cnt = (long long)(v >> 40);
        long long qs = (long long)(v & kQMask) - 161ll * cnt;
        if (k >= 2 && removed_mode) {
            const unsigned long long pv = *reinterpret_cast<const unsigned long long*>(hist + (k - 2) * kHistW + cell);
            const long long pc = (long long)(pv >> 40);
            const long long pq = (long long)(pv & kQMask) - 161ll * pc;
            cnt = pc - cnt;
            qs = pq - qs;
        }
        if (cnt == 0 && qs == 0) continue;
        const int cls = (3 * slot) & 7;
        unsigned long long* dst = acc + st_base + k * st_words + FQ_ST_CYCLES + (size_t)c * FQ_ST_PER_CYCLE;
        atomicAdd(&dst[cls], (unsigned long long)cnt);
        atomicAdd(&dst[8 + cls], (unsigned long long)qs);
    }
}

}  // namespace

bool fq_pe_fast_supported(const fq_params& p) {
    return p.paired && !p.merge_enabled && p.insert_size_max <= 512 && p.insert_size_max >= 0;
}

hipError_t fq_pe_fast_prepare() {
    return hipFuncSetAttribute((const void*)pe_fast_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               kLdsWords * 4);
}

hipError_t fq_launch_pe_fast(const fq_params& p, const fq_batch& b, fq_read_result* res, unsigned long long* acc,
                             int* slow_tiles, int* slow_count, int grid, hipStream_t stream) {
    hipLaunchKernelGGL(pe_fast_kernel, dim3(grid), dim3(kBlock), kLdsWords * 4, stream, p, b, res, acc, slow_tiles,
                       slow_count);
    return hipGetLastError();
}
