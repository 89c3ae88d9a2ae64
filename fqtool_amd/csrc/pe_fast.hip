// pe_fast.hip -- hot path for paired-end and single-end packs on gfx950 (incl. -m merge).
//
// Mapping: one workgroup = 8 waves, one wave = a tile of 32 pairs, one LANE = one READ
// (lanes 0-31 read 1, lanes 32-63 read 2 of the same pairs), so every per-read operation of
// PairEndProcessor::processPairEnd (reference src/peprocessor.cpp:261-508) keeps all 64 lanes
// busy and the two mates of a pair are lanes l and l^32 of the same wave.
//
// Occupancy: 16 waves per CU (2 workgroups of 8, the merge variant 1 of 16); the only per-wave
// LDS is the 2-bit code / N-mask column block (5 KB), and a workgroup's Stats histograms are
// shared by its waves.
//
// Staging: each lane streams its seq and qual rows from HBM with 16-byte loads (the batch's
// chunk-interleaved tiles make each wave-wide chunk load contiguous).  Sequence bytes
// are reduced in registers to 2-bit base codes (A=0 C=1 T=2 G=3, N=3, i.e. (byte>>1)&3) plus a
// spaced N mask and go to the lane's own LDS column (word field*64 + lane: conflict-free for any
// per-lane position).  Read 1 codes are stored forward; read 2's column is the reverse complement
// of its whole 160-position row (the orientation OverlapAnalysis::analyze compares,
// src/overlapanalysis.cpp:7-72), so rc position j of a read of length L sits at index
// j + 160 - L.  Whole-read quality sums (Q20/Q30, below-limit count, total) are taken from the
// quality registers, and their running values at chunk ends are staged in LDS (prefix counts for
// passFilter's windows); qualities are not kept: later passes re-read the row (an L2 hit).
// Lowercase a c g t stay here (a flag beside the N mask); a PAIR (single-end: a read) with any other
// byte outside {A,C,G,T,N}, a quality >= 128, a read longer than the columns or an index-filter flag
// is handed to the general kernel (pe_kernel.hip) through a device-side item list, its lanes running
// on as empty lanes, so everything here may assume that alphabet and rebuild bases from codes.
//
// Per read, in the reference's order: trimAndCut (integer windows), polyG (bit-parallel: the
// 3'-end scan only changes state at non-G bases, visited with find-last-set), overlap analysis
// (read 1 lanes scan phase 1, read 2 lanes phase 2 through one code path: a 16-position
// code-mismatch lower bound rejects offsets, survivors are verified exactly with codes + N masks
// under the reference's break/accept rule), adapter trimming, polyX, maxLen, passFilter (whole-
// read sums minus the trimmed ends), then Stats::statRead for the pre and post blocks into
// workgroup-private LDS histograms of u64 cells (count << 40 | sum(q+128)); lanes walk each
// 16-position chunk from a lane-dependent rotation so the lanes of an atomic hit distinct banks.
// The LEAN instantiation drops the options the headline workloads do not use.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "device_ops.h"
#include "engine_internal.h"

using namespace fqdev;

#if FQ_MAXLEN_BUILD_LONG
namespace long320 {  // (kernel names tell the two builds apart in profiles)
#else
namespace {
#endif

#ifndef FQ_MERGE_ROTATE  // merged-part Stats walk rotated per lane (conflict-free LDS banks; slower)
#define FQ_MERGE_ROTATE 0
#endif
#ifndef FQ_ABLATE_STAGE
#define FQ_ABLATE_STAGE 0
#endif
#ifndef FQ_OPAQUE_NCH
#define FQ_OPAQUE_NCH 1
#endif
#ifndef FQ_OPAQUE_LK
#define FQ_OPAQUE_LK 1
#endif
#ifndef FQ_SCHED_PIN
#define FQ_SCHED_PIN 1
#endif
#ifndef FQ_MERGE_WAVES
#define FQ_MERGE_WAVES 16  // merge variant: one workgroup of 16 waves per CU (8: 10.8, 12: 9.4, 16: 9.0 ms per 20 M pairs)
#endif
#ifndef FQ_MERGE_BLOCKS
#define FQ_MERGE_BLOCKS 1
#endif
#ifndef FQ_LEAN_DIRECT
#define FQ_LEAN_DIRECT 1  // LEAN passFilter: a window shorter than half the read is summed directly
#endif
#ifndef FQ_LEAN_WAVES
#define FQ_LEAN_WAVES 8  // profiling: waves per workgroup of the LEAN variant
#endif
#ifndef FQ_LEAN_BLOCKS
#define FQ_LEAN_BLOCKS 2  // profiling: workgroups per CU of the LEAN variant
#endif
#ifndef FQ_MERGE_QLDS
#define FQ_MERGE_QLDS 0
#endif
#ifndef FQ_AHEAD
#define FQ_AHEAD 4  // (A/B at 20 M pairs: 3 -> 4 is -1 to -2 % on C3-C5; 5 and 6 are slower)
#endif
#ifndef FQ_NFOLD
#define FQ_NFOLD 1  // removed-mode Stats: N bases by a nibble add (0: the per-N fix-up loop, profiling)
#endif
#ifndef FQ_SCAL_PAD
#define FQ_SCAL_PAD 1  // per-read scalar copies 17 u64 apart: one LDS bank pair per copy (0: 16, profiling)
#endif
#ifndef FQ_STATS_PRIO
#define FQ_STATS_PRIO 3  // s_setprio during the Stats passes (see FQ_PRIO_TRIM)
#endif
#ifndef FQ_STATS_PRIO_ALL
#define FQ_STATS_PRIO_ALL 2  // (with FQ_STATS_PRIO) 1: up to the end of the merged part's Stats; 2: on to the end of the tile (C3 -1 %)
#endif
#ifndef FQ_PRIO_TRIM
#define FQ_PRIO_TRIM 1  // s_setprio after staging (trimAndCut)
// Issue priority rising with a wave's progress through its tile: staging 0, trimAndCut and polyG 1,
// overlap to passFilter 2, Stats 3 -- the waves nearest the end of their tile issue first, so the
// 16 waves of a CU spread over the phases and the memory / LDS work of the late phases (the Stats
// pass's quality re-reads and atomics) overlaps the VALU of the early ones.  C3 -10 %, C4 -13 %,
// C5 -10 %, C2 -3 % against staging-only priority (profiles/r05_ab_prio_*.txt).
#endif
#ifndef FQ_PRIO_POLYG
#define FQ_PRIO_POLYG 1  // s_setprio from polyG on
#endif
#ifndef FQ_PRIO_OV
#define FQ_PRIO_OV 2  // from the overlap analysis on
#endif
#ifndef FQ_PRIO_FILTER
#define FQ_PRIO_FILTER 2  // from passFilter on
#endif
#ifndef FQ_STAGE_PRIO
#define FQ_STAGE_PRIO 0  // s_setprio during staging (round 4: 1, -2 % against none; with the later phases above it, 0)
#endif
#ifndef FQ_DESYNC
#define FQ_DESYNC 0  // profiling: initial s_sleep stagger of co-resident waves
#endif
#ifndef FQ_CUT_W4
#define FQ_CUT_W4 1  // cut_right windows <= 4 decided per low chunk (0: the word-stream scan, profiling)
#endif
#ifndef FQ_FILTER_BATCH
#define FQ_FILTER_BATCH 1  // passFilter's trimmed / direct ranges: row chunks loaded four at a time
#endif
#ifndef FQ_STATS_AHEAD
#define FQ_STATS_AHEAD 2  // removed-mode Stats: quality chunks requested this many chunks ahead
#endif
#ifndef FQ_VK
#define FQ_VK 1  // staging: the SWAR masks and limits as VGPR values (a VALU op with an SGPR operand issues at half rate)
#endif
#ifndef FQ_EXO3
#define FQ_EXO3 1  // staging: exotic bytes OR-accumulated with one v_bitop3 (full rate) instead of v_sad_u8
#endif
#ifndef FQ_STG2
#define FQ_STG2 1  // staging: the chunk's code and N-flag words from two nibble-packed key words
#endif
#ifndef FQ_PG4
#define FQ_PG4 1  // polyG: the all-G groups at the scan's start (a G tail) passed over by a light loop
#endif
#ifndef FQ_PG3
#define FQ_PG3 1  // polyG: the scan loop loads group g+1's column words before deciding group g
#endif
#ifndef FQ_PG2
#define FQ_PG2 1  // polyG: group 0 decided without the loop when the break is the second non-G base
#endif
#ifndef FQ_PREFIX
#define FQ_PREFIX 1  // LEAN: per-chunk prefix counts staged in LDS, passFilter reads them (0: the trimmed-tail loop)
#endif
#ifndef FQ_PLAUNDER
#define FQ_PLAUNDER 1  // re-read fq_params / fq_batch from the kernarg segment every tile (SGPR pressure)
#endif
#ifndef FQ_ST_SH64
#define FQ_ST_SH64 1  // removed-mode Stats: slot nibbles positioned two at a time by 64-bit shifts
#endif
#ifndef FQ_ST_KM2
#define FQ_ST_KM2 1  // removed-mode Stats: kept mask by one med3 + one bitop3 per word, 64-bit spread
#endif
#ifndef FQ_ST_PF2
#define FQ_ST_PF2 1  // removed-mode Stats: column words requested two chunks ahead (no wait on the atomics)
#endif
#ifndef FQ_OVX2
#define FQ_OVX2 1  // overlap exact check: word pairs by ds_read2st64 + 64-bit shifts, the 50-position test peeled
#endif
#ifndef FQ_MRG2
#define FQ_MRG2 1  // merged-part Stats: groups unrolled (immediate row offsets), qualities through a tile buffer
#endif
#ifndef FQ_ADSEQ_LDSBITS
#define FQ_ADSEQ_LDSBITS 0  // adseq_search's candidate scan: the adapter's bit words from LDS (FixedLds) instead of v_bfe
#endif
#ifndef FQ_OV_SH64
#define FQ_OV_SH64 1  // overlap candidates: planes realigned by 64-bit shifts (one block per pass)
#endif
#ifndef FQ_OV12
#define FQ_OV12 0  // overlap candidates at the default limit 5 from the first 12 positions (not 16): slower (a false candidate in any lane costs the wave an exact check; profiles/r05_ab_ov12_stvcc.txt)
#endif
#ifndef FQ_OV_CSHIFT
#define FQ_OV_CSHIFT 1  // overlap candidates: the block words through a shift register (not a select per word on the runtime block index)
#endif
#ifndef FQ_FASTMASK
#define FQ_FASTMASK 1  // posmask at the hot sites and staging's partial-chunk byte masks by v_med3 + 64-bit shifts (neutral to -0.5 %, profiles/r05_ab_fastmask_runshift.txt)
#endif
#ifndef FQ_ST_VCC
#define FQ_ST_VCC 0  // removed-mode Stats: the rotation selects as VCC-masked v_cndmask_e32 (no gain measured, profiles/r05_ab_ov12_stvcc.txt)
#endif
#ifndef FQ_PREFETCH
#define FQ_PREFETCH 0  // profiling: after staging, pull the first FQ_PREFETCH chunks of the wave's next tile
                       // toward L2 with LDS-DMA loads (0: off; measured slower at 10)
#endif
constexpr int kAhead = FQ_AHEAD;  // staging: row chunks requested this many chunks ahead of their use
constexpr int kBlock = 1024;  // largest workgroup (the launch bound of each variant is its own size)
#ifndef FQ_MAXLEN
#define FQ_MAXLEN 160  // pe_fast_long.hip builds this file again for reads up to 320 bp
#endif
constexpr int kMaxLen = FQ_MAXLEN;
static_assert(kMaxLen % 32 == 0 && kMaxLen <= 320, "reads per column: a multiple of 32, at most 320");
constexpr int kOvBlocks = kMaxLen / 32;           // 32-offset blocks of the overlap candidate scan
constexpr int kChunks = kMaxLen / 16;             // 16-position chunks per read
constexpr int kFC = 0;                            // column fields (words): 2-bit codes,
constexpr int kFN = kChunks;                      //   spaced N mask (+ lowercase flags at the odd bits),
constexpr int kCodeW = 2 * kChunks * 64;          // code + N columns of a wave
constexpr int kQS = kMaxLen / 4 + 1;              // quality row stride (odd: conflict-free per lane)
// Stats histograms: u64 cells [cycle / 16][slot][cycle % 16], slots A C T G N + one dummy slot
// that absorbs masked-off positions.  A cell's LDS bank pair depends only on cycle % 16, so the
// 16 lanes of an atomic's lane group (distinct cycle % 16 by the per-lane rotation) never
// collide, whatever their base classes.
constexpr int kSlots = 6;
constexpr int kDummySlot = 5;
constexpr int kHistW = kChunks * kSlots * 32;
__host__ __device__ constexpr int cell(int c, int slot) { return ((c >> 4) * kSlots + slot) * 32 + 2 * (c & 15); }
// Removed-mode Stats rows: [cycle / 16][13 slots][mate][cycle % 16] u64 cells, slot = 4 * kept +
// code for A C T G (codes 0-3), 8 + 4 * kept for N (the G slot + 5, so an N is one nibble add away
// from the G that its code 3 reads as), 10 for positions beyond the read.  The mates' rows
// interleave, so a cell's byte address is base | slot << 8 | mate << 7 | (cycle % 16) << 3 plus the
// chunk's (wave-uniform) offset: the slot nibble goes in with one bit operation (statRead below).
constexpr int kRSlots = 13;
constexpr int kRNSlot = 8;   // removed N; kept N = kRNSlot + 4
__host__ __device__ constexpr int rcell(int c, int slot) { return ((c >> 4) * kRSlots + slot) * 64 + 2 * (c & 15); }
// read 2's merged parts (Layout::kMrgW): [cycle / 16][8 slot rows, A C T G N dummy + 2 unused][cycle % 16]
__host__ __device__ constexpr int mcell(int c, int slot) { return ((c >> 4) * 8 + slot) * 32 + 2 * (c & 15); }
constexpr int kRemW = 2 * kRSlots * 32 * kChunks;  // both mates' removed-mode rows
constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int kSmallU64 = FQ_ACC_INSERT;                 // FilterResult / adapter / polyX / merged counters
constexpr int kSmallW = 2 * ((kSmallU64 + 1) & ~1);
constexpr int kInsW = (512 + 1 + 1) & ~1;                 // insert-size histogram, u32 per workgroup
// per-read scalars are spread over kScalCopies LDS copies (lane % copies), each
// [4 stats][reads, length_sum, q20, q30] u64; the merge variant keeps 8 (LDS budget)
// adseq_search's adapter columns (per mate: 2-bit codes; read 2's reversed and complemented)
constexpr int kAdCW = 10;    // words of an adapter column (positions < FQ_MAX_ADAPTER, + one look-ahead)
constexpr int kAdRc = 144;   // read 2's adapter column: index y holds position kAdRc - 1 - y
static_assert(kAdRc >= FQ_MAX_ADAPTER + 15 && kAdRc + 16 <= 16 * kAdCW && FQ_MAX_ADAPTER + 16 <= 16 * kAdCW, "adapter column");
// adapter bytes of both mates, adseq_search's window words [2][8], adapter columns [2][kAdCW] and the
// (fh, fl) words of each mate's first window [2][16][2]
constexpr int kAdWinOff = 2 * FQ_MAX_ADAPTER / 4, kAdColOff = kAdWinOff + 16, kAdBitOff = kAdColOff + 2 * kAdCW;
constexpr int kAdW = kAdBitOff + 2 * 16 * 2;
static_assert(kAdBitOff % 2 == 0, "(fh, fl) pairs 8-byte aligned");
constexpr int kScalStride = FQ_SCAL_PAD ? 17 : 16;  // u64 per scalar copy (17: copies on distinct LDS bank pairs)
constexpr int kPfW = FQ_PREFETCH ? 64 : 0;             // LDS-DMA prefetch sink (never read)
// Every variant re-reads qualities from the rows in L2 (no LDS quality rows) and runs 16 waves
// per CU: LEAN and FULL as 2 workgroups of 8 waves (128 VGPRs), the merge variant, whose Stats
// blocks are larger (read 2's merged parts land at read 1's post cycles up to 319), as one
// workgroup of 16 waves.  The long-read build (320-position columns) fits one 8-wave workgroup.
template <bool LEAN, bool MERGE = false, bool PAIRED = true>
struct Layout {
    // quality rows staged in LDS (off: rows are re-read from L2); profiling switch for the merge variant
    static constexpr bool kQLds = MERGE && FQ_MERGE_QLDS;
    // Each lane's running quality / N counts (q20 | q30 << 8 | low << 16 | N << 24) at the end of every
    // kPfxStep-th row chunk, staged in LDS (word kCodeW + (chunk / kPfxStep) * 64 + lane of the wave's
    // block), so passFilter gets a window's counts from prefix words and at most kPfxStep chunks of
    // bytes.  One word per chunk takes one Stats histogram's worth of LDS, so those variants run as one
    // workgroup of 16 waves (whose waves share one histogram) instead of two of 8; the merge variant
    // (already one workgroup, with larger histograms) has room for one word per two chunks.
    // (LEAN single-end, C2, trims nothing; the long build has no room.)
    static constexpr bool kPfx = FQ_PREFIX && kMaxLen <= 160 && !kQLds && (!LEAN || PAIRED);
    static constexpr int kPfxStep = MERGE ? 2 : 1;
    static constexpr int kBlocksPerCU = (kQLds || kMaxLen > 160 || kPfx) ? 1 : MERGE ? FQ_MERGE_BLOCKS : LEAN ? FQ_LEAN_BLOCKS : 2;
    // (the long build's merge variant: its 320-position columns and 640-cycle merged Stats fit 4 waves)
    static constexpr int kWaves = MERGE ? (kQLds ? 7 : kMaxLen > 160 ? 4 : FQ_MERGE_WAVES)
                                        : kPfx ? 16 : (LEAN && kMaxLen <= 160) ? FQ_LEAN_WAVES : 8;
    static constexpr int kWavesPerEU = (kWaves * kBlocksPerCU + 3) / 4;
    static constexpr int kThreads = 64 * kWaves;
    static constexpr int kPfxW = kPfx ? kChunks / kPfxStep * 64 : 0;
    static constexpr int kWaveW = kCodeW + kPfxW + (kQLds ? 64 * kQS : 0);
    // [pre1, pre2, post1 (x2 with MERGE), post2] (+ MERGE: read 2's merged parts, cycles 0..319,
    // in removed mode, which uses blocks 0-3 as the kept/removed rows of the two mates)
    static constexpr int kHists = MERGE ? 6 : 4;
    // read 2's merged parts (removed mode): cycle rows of 8 slot rows (mcell), cycles < 2 kMaxLen + 16
    // (the last row: dummy positions past the part); 1 KiB-aligned, so a cell's byte address is
    // row base | slot << 7 | (cycle % 16) << 3
    static constexpr int kMrgW = MERGE ? (2 * kChunks + 1) * 8 * 32 : 0;
    // removed mode: both mates' kept/removed rows first, then (MERGE) read 2's merged parts
    static constexpr int kMrgOff = (cmax(4 * kHistW, kRemW) + 255) & ~255;
    static constexpr int kHistRegW = cmax(kHists * kHistW, MERGE ? kMrgOff + kMrgW : kRemW);
    static constexpr int kColsW = kWaves * kWaveW;
    static constexpr int kScalCopies = MERGE ? 8 : 16;
    static constexpr int kScalW = 2 * kScalStride * kScalCopies;
    static constexpr int kHrW = 2 * kWaves;  // per wave: hand-off list reservation (next slot, slots left)
    static constexpr int kLdsW = kColsW + kHistRegW + kSmallW + kInsW + kScalW + kAdW + kHrW + kPfW;
    static_assert(kLdsW * 4 * kBlocksPerCU <= 160 * 1024, "LDS budget");
    static_assert((kColsW & 1) == 0 && (kHistW & 1) == 0, "u64 cells must stay 8-byte aligned");
    static_assert(kThreads <= kBlock, "launch bound");
};

constexpr unsigned long long kCount1 = 1ull << 40;
constexpr int kXfixCopies = 64;  // copies of the Stats blocks for the exotic-byte moves (see the Stats fix-up)
constexpr unsigned long long kQMask = kCount1 - 1;

// x of lane l ^ 32 (the other mate of the pair): one v_permlane32_swap, no LDS round trip
// (a ds_bpermute would queue behind the workgroup's LDS atomics).  With old = src = x the swap
// leaves lanes 0-31 of x in both halves of the first result and lanes 32-63 in both halves of
// the second.
__device__ __forceinline__ int xor32(int x) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return (threadIdx.x & 32) ? r[0] : r[1];
}
__device__ __forceinline__ uint32_t xor32(uint32_t x) { return (uint32_t)xor32((int)x); }

// A uniform value kept in a VGPR (opaque to the compiler, which would otherwise keep it in an SGPR or
// rematerialise it there): on gfx950 a full-rate VALU op (and, xor, add, bitop3, ...) with an SGPR
// operand issues at the half rate of the VOP3 ops (profiles/r04_micro_opcost2.txt).
__device__ __forceinline__ uint32_t vk(uint32_t x) {
#if FQ_VK
    asm volatile("" : "+v"(x));
#endif
    return x;
}

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
// the same at the hot sites of every variant: 2n clamped to [0, 32] by one v_med3, then the low
// word of ~(~0 << 2n) by one full-rate 64-bit shift (the compare / select form costs two
// half-rate shifts and two v_cndmask with their wait states)
__device__ __forceinline__ uint32_t posmask_v(int n) {
#if FQ_FASTMASK
    int c;
    asm("v_med3_i32 %0, %1, 0, 32" : "=v"(c) : "v"(n + n));
    unsigned long long x;
    asm("v_lshlrev_b64 %0, %1, -1" : "=v"(x) : "v"(c));
    return ~(uint32_t)x & 0x55555555u;
#else
    return posmask(n);
#endif
}

// byte masks of the first n4 / 4 bytes of a 16-byte chunk, dwords 0-3 (n4 = 4 x bytes, any value):
// per 8-byte half ~((~0 << c) << c) with c = 4 x its bytes clamped to [0, 32]
[[maybe_unused]] __device__ __forceinline__ void chunk_bytemask(int n4, uint32_t m[4]) {
    int c0, c1;
    asm("v_med3_i32 %0, %1, 0, 32" : "=v"(c0) : "v"(n4));
    asm("v_med3_i32 %0, %1, 0, 32" : "=v"(c1) : "v"(n4 - 32));
    unsigned long long a, b;
    asm("v_lshlrev_b64 %0, %1, -1" : "=v"(a) : "v"(c0));
    asm("v_lshlrev_b64 %0, %1, %2" : "=v"(a) : "v"(c0), "v"(a));
    asm("v_lshlrev_b64 %0, %1, -1" : "=v"(b) : "v"(c1));
    asm("v_lshlrev_b64 %0, %1, %2" : "=v"(b) : "v"(c1), "v"(b));
    m[0] = ~(uint32_t)a;
    m[1] = ~(uint32_t)(a >> 32);
    m[2] = ~(uint32_t)b;
    m[3] = ~(uint32_t)(b >> 32);
}

// byte mask of the first `n` bytes of a dword
__device__ __forceinline__ uint32_t bytemask(int n) {
    return n >= 4 ? 0xFFFFFFFFu : n <= 0 ? 0u : ((1u << (8 * n)) - 1u);
}

// 4x4 transpose of two-bit elements, row = byte: element (r, c) at bit 8r+2c moves to 8c+2r
__device__ __forceinline__ uint32_t tr4x4(uint32_t y) {
    uint32_t t = (y ^ (y >> 6)) & 0x00CC00CCu;
    y ^= t ^ (t << 6);
    t = (y ^ (y >> 12)) & 0x0000F0F0u;
    return y ^ t ^ (t << 12);
}

// 16 consecutive two-bit positions [pos, pos+16) of field f (codes or N mask) of column c;
// positions outside the column read as 0
__device__ __forceinline__ uint32_t field_window(const uint32_t* col, int f, int c, int pos) {
    const int w = pos >> 4, sh = 2 * (pos & 15);
    const int wl = min(max(w, 0), kChunks - 1), wh = min(max(w + 1, 0), kChunks - 1);
    const uint32_t lo = col[(f + wl) * 64 + c] & ((unsigned)w < (unsigned)kChunks ? ~0u : 0u);
    const uint32_t hi = col[(f + wh) * 64 + c] & ((unsigned)(w + 1) < (unsigned)kChunks ? ~0u : 0u);
    return __builtin_amdgcn_alignbit(hi, lo, sh);
}

struct Fwd {
    uint32_t c, n;
};

// field_window for callers whose positions below 0 (or past the column) are masked off anyway: the
// words are read without the range checks (a word index below 0 reads word 0; past the column the
// next field or the next wave's column, valid LDS), so only in-column positions are exact
__device__ __forceinline__ uint32_t field_window_masked(const uint32_t* col, int f, int c, int pos) {
    const int w = pos >> 4, sh = 2 * (pos & 15);
    const uint32_t* p = col + (f + max(w, 0)) * 64 + c;
    const uint32_t lo = p[0], hi = p[w >= 0 ? 64 : 0];
    return __builtin_amdgcn_alignbit(hi, lo, sh);
}

// forward codes / N mask of positions [16F, 16F+16) of lane c's read.  Read 2 columns hold the
// reverse complement of the whole 160-position row, so forward chunk F is stored word 9-F with
// its fields reversed and complemented; positions >= L are garbage for the caller to mask.
__device__ __forceinline__ Fwd fwd_chunk(const uint32_t* col, int c, int F, bool rc) {
    const int w = rc ? kChunks - 1 - F : F;
    const bool in = (unsigned)w < (unsigned)kChunks;
    const int wc = in ? w : 0;
    uint32_t cw = in ? col[(kFC + wc) * 64 + c] : 0u;
    uint32_t nw = in ? col[(kFN + wc) * 64 + c] : 0u;
    if (rc) {
        cw = pairrev(cw);
        nw = pairrev(nw);
        cw ^= 0xAAAAAAAAu & ~(nw << 1);  // complement back, N stays code 3
    }
    return Fwd{cw, nw};
}

struct CodeSeq {  // forward base byte i rebuilt from the codes (alphabet A C G T N a c g t)
    const uint32_t* col;
    int c;
    bool rc;
    __device__ __forceinline__ uint8_t operator()(int i) const {
        const int q = rc ? kMaxLen - 1 - i : i;
        const int w = q >> 4, sh = 2 * (q & 15);
        uint32_t code = (col[(kFC + w) * 64 + c] >> sh) & 3u;
        const uint32_t nx = col[(kFN + w) * 64 + c] >> sh;  // bit 0: N, bit 1: lowercase
        code ^= rc ? 2u : 0u;
        // "ACTG", lowercase with the flag (its code is its uppercase letter's, never N); an exotic
        // byte (N bit and flag) as 0x01, which equals no letter and no 'N' (lower_flags)
        if (nx & 1u) return (nx & 2u) ? (uint8_t)1 : (uint8_t)'N';
        return (uint8_t)(((0x47544341u >> (8 * code)) & 0xFFu) | ((nx & 2u) << 4));
    }
};

struct OvOut {
    bool found;
    int off, ol, diff;
};

// Exact OverlapAnalysis acceptance test at one offset (src/overlapanalysis.cpp:24-40 / :49-65):
// positions compare r1 codes from p1 with rc2 codes from p2 over `ol` positions.  The four
// streams (codes and N masks of both sides) slide one LDS word per 16 positions; a candidate whose
// K-th mismatch lies in the first 50 positions is rejected after the first four words.
// The words are read unclamped: p1, p2 >= 0 and p + ol <= the column length, so a look-ahead word
// past the column (the next field, or the next wave's column: valid LDS) only feeds positions at
// or beyond ol, which the last word's mask drops.
template <bool X2>
__device__ inline bool ov_exact(const uint32_t* col, int c1, int p1, int c2, int p2, int ol, int limit, int K,
                                int& diff_out) {
    int d50 = 0, D = 0;
    const int nw = (ol + 15) >> 4;
    const int s1 = 2 * (p1 & 15), s2 = 2 * (p2 & 15);
    const uint32_t* A = col + (p1 >> 4) * 64 + c1;  // code word w of read 1's window: A[64 w]
    const uint32_t* B = col + (p2 >> 4) * 64 + c2;
    constexpr int kN = kFN * 64;                       // the N-mask field, kChunks words further
    const uint32_t last = posmask_v(ol - 16 * (nw - 1));  // valid positions of the last word
    if constexpr (X2) {
    // Each stream's words j and j + 1 come as one register pair (one ds_read2st64 each), realigned
    // by a full-rate 64-bit shift -- instead of a v_alignbit (half rate) on words carried over from
    // the previous step, whose rotation also cost four moves a word.  The first four words, which
    // decide the rejection within 50 positions, are peeled off the loop that counts the rest.
    auto mism_at = [&](int j) -> uint32_t {
        auto pr = [&](const uint32_t* W, int f, uint32_t s) -> uint32_t {
            const unsigned long long v = (unsigned long long)W[64 * (j + 1) + f] << 32 | W[64 * j + f];
            unsigned long long r;
            asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "v"(s), "v"(v));
            return (uint32_t)r;
        };
        const uint32_t a = pr(A, 0, (uint32_t)s1), wa = pr(A, kN, (uint32_t)s1);
        const uint32_t b = pr(B, 0, (uint32_t)s2), wb = pr(B, kN, (uint32_t)s2);
        uint32_t mism = ((fold2(a ^ b) & ~(wa | wb)) | (wa ^ wb) | (wa >> 1)) & 0x55555555u;
        if (j == nw - 1) mism &= last;
        return mism;
    };
    int j = 0;
    for (; j < 4 && j < nw; ++j) {
        const uint32_t mism = mism_at(j);
        if (j == 3) d50 = D + __popc(mism & 5u);
        D += __popc(mism);
    }
    if (nw > 3 && d50 >= K) {  // (the break happens within 50: rejected whatever follows)
        diff_out = D;
        return false;
    }
    for (; j < nw; ++j) D += __popc(mism_at(j));
    } else {
    uint32_t a0 = A[0], an0 = A[kN], b0 = B[0], bn0 = B[kN];
    for (int j = 0; j < nw; ++j) {
        const uint32_t a1 = A[64 * (j + 1)], an1 = A[64 * (j + 1) + kN];
        const uint32_t b1 = B[64 * (j + 1)], bn1 = B[64 * (j + 1) + kN];
        const uint32_t a = __builtin_amdgcn_alignbit(a1, a0, s1), wa = __builtin_amdgcn_alignbit(an1, an0, s1);
        const uint32_t b = __builtin_amdgcn_alignbit(b1, b0, s2), wb = __builtin_amdgcn_alignbit(bn1, bn0, s2);
        // (a lowercase base of read 1 -- odd flag bit of wa -- differs from every base of the
        // reverse complement, which is upper case; read 2's lowercase flags do not count)
        uint32_t mism = ((fold2(a ^ b) & ~(wa | wb)) | (wa ^ wb) | (wa >> 1)) & 0x55555555u;
        if (j == nw - 1) mism &= last;
        // mismatches within the first 50 positions: words 0-2 whole, word 3's positions 48, 49
        if (j == 3) d50 = D + __popc(mism & 5u);
        D += __popc(mism);
        if (j == 3 && d50 >= K) break;  // rejected whatever follows (the break happens within 50)
        a0 = a1; an0 = an1; b0 = b1; bn0 = bn1;
    }
    }
    if (nw <= 3) d50 = D;  // (ol <= 48: every position is within 50)
    diff_out = D;
    // break (rejection) happens iff the K-th mismatch lies within the first min(ol,50) positions
    if (d50 >= K) return false;
    return D < limit || ol > 50;
}

// (acc << 1) | (t >> 31): a flag bit shifted in from the sign of t, one v_alignbit.  Bit-flag words
// built this way need no per-bit constant (a cmp / cndmask / or chain keeps every 1 << r in a VGPR).
__device__ __forceinline__ uint32_t shift_in_sign(uint32_t acc, uint32_t t) {
    uint32_t r;
    asm("v_alignbit_b32 %0, %1, %2, 31" : "=v"(r) : "v"(acc), "v"(t));
    return r;
}

// Scan one phase: offsets k = k0 .. cnt-1 move a 16-position window of column `cm` starting at
// code position mpos0 + k against the fixed 16-position word `fixed`; returns the first offset
// whose code-level lower bound is < K (or -1).  ol(k) = min(olA - k, olB).  With FIXED_MASK the
// caller guarantees ol(k) >= min(olB, 16) for every scanned k (overlap_require >= 16), so the
// mask of compared positions is the constant `pm`.
template <bool FIXED_MASK>
__device__ inline int ov_scan(const uint32_t* col, int cm, int mpos0, int k0, int cnt, uint32_t fixed, int olA,
                              int olB, int K, uint32_t pm) {
    int w = (mpos0 + k0) >> 4;
    uint32_t lo = w < kChunks ? col[(kFC + min(w, kChunks - 1)) * 64 + cm] : 0u;
    uint32_t hi = w + 1 < kChunks ? col[(kFC + min(w + 1, kChunks - 1)) * 64 + cm] : 0u;
    // the next two window words are requested a step ahead (clamped reads, zeroed past the column)
    uint32_t nx = col[(kFC + min(w + 2, kChunks - 1)) * 64 + cm];
    for (int k = k0; k < cnt;) {
        const int P = mpos0 + k;
        const uint32_t nx_use = w + 2 < kChunks ? nx : 0u;
        nx = col[(kFC + min(w + 3, kChunks - 1)) * 64 + cm];
        // lower bounds of the 16 windows starting at absolute positions 16w + r
        int lb[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t win = r == 0 ? lo : __builtin_amdgcn_alignbit(hi, lo, 2 * r);
            uint32_t m = pm;
            if (!FIXED_MASK) {
                const int kk = 16 * w + r - mpos0;
                m = posmask(min(olA - kk, olB));
            }
            lb[r] = __popc(fold2(win ^ fixed) & m);
        }
        // common case: no window of this step comes under the bound (one min per two windows)
        int mn = lb[0];
#pragma unroll
        for (int r = 1; r < 16; r += 2) mn = min(mn, min(lb[r], r + 1 < 16 ? lb[r + 1] : lb[r]));
        if (mn < K) {
            uint32_t bits = (uint32_t)(lb[15] - K) >> 31;  // bit r: lb[r] < K
#pragma unroll
            for (int r = 14; r >= 0; --r) bits = shift_in_sign(bits, (uint32_t)(lb[r] - K));
            // keep offsets within [k, cnt)
            const int first_r = P & 15;
            bits &= ~((1u << first_r) - 1u);
            const int last = cnt - 1 - (16 * w - mpos0);  // last valid r
            if (last < 15) bits &= (last < 0) ? 0u : ((2u << last) - 1u);
            if (bits) return 16 * w + (__ffs(bits) - 1) - mpos0;
        }
        k = 16 * (w + 1) - mpos0;
        ++w;
        lo = hi;
        hi = nx_use;
    }
    return -1;
}

// the 8 two-bit fields of x's low half, each widened to a nibble
__device__ __forceinline__ uint32_t spread2to4(uint32_t x) {
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    return (x | (x << 2)) & 0x33333333u;
}


// Unshuffle: the low bits of the 16 two-bit fields of x to bits 0-15, the high bits to 16-31.
__device__ __forceinline__ uint32_t unzip2(uint32_t x) {
    uint32_t t;
    t = (x ^ (x >> 1)) & 0x22222222u;
    x ^= t ^ (t << 1);
    t = (x ^ (x >> 2)) & 0x0C0C0C0Cu;
    x ^= t ^ (t << 2);
    t = (x ^ (x >> 4)) & 0x00F000F0u;
    x ^= t ^ (t << 4);
    return __builtin_amdgcn_perm(x, x, 0x03010200u);  // swap bytes 1 and 2
}

// Full-adder step of the carry-save counters: (hi, lo) = a + b + c, bitwise
__device__ __forceinline__ void csa(uint32_t& hi, uint32_t& lo, uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t h = (a & b) | (a & c) | (b & c), l = a ^ b ^ c;
    hi = h;
    lo = l;
}

// Candidate offsets of one overlap phase, all at once (overlap_require >= 16, both windows of >= 16
// positions): bit k of cand[k >> 5] is set iff the 16 positions of the window at mpos + k of
// column cm hold fewer than K code mismatches against `fixed` (the filter ov_scan applies one
// offset at a time).  Branch-free: the moving column is realigned to mpos (LDS) and unzipped into
// bit planes H and L over positions; for compared position j the mismatch vector over the 32
// offsets of a block is ((H >> j) ^ FH_j) | ((L >> j) ^ FL_j) (FH_j, FL_j = the bits of fixed[j]
// spread over a word), and the 16 vectors are summed per offset with carry-save adders.
// Compared position j's fixed code bits, each as a word of 0s or 1s (fh: high bit, fl: low bit):
//  * FixedOwn: from the lane's own fixed word (the overlap: a window of the other mate), two v_bfe;
//  * FixedLds: precomputed in LDS (trimBySequence: the adapter's first 16 codes, the same for every
//    lane of a mate), one broadcast ds_read_b64 and no VALU.
struct FixedOwn {
    uint32_t fu;  // unzip2(fixed)
    __device__ __forceinline__ void next_block() {}
    __device__ __forceinline__ void bits(int j, uint32_t& fh, uint32_t& fl) const {
        fh = (uint32_t)__builtin_amdgcn_sbfe((int)fu, 16 + j, 1);
        fl = (uint32_t)__builtin_amdgcn_sbfe((int)fu, j, 1);
    }
};
struct FixedLds {
    uint32_t f;  // LDS byte address of [j] = (fh, fl)
    // (opaque per block: hoisted out of the block loop, the 32 words would stay live and spill)
    __device__ __forceinline__ void next_block() { asm volatile("" : "+v"(f)); }
    __device__ __forceinline__ void bits(int j, uint32_t& fh, uint32_t& fl) const {
        typedef __attribute__((address_space(3))) const uint32_t LdsW;
        const LdsW* w = reinterpret_cast<const LdsW*>((size_t)f);
        fh = w[2 * j];
        fl = w[2 * j + 1];
    }
};
template <class FX>
__device__ inline void ov_candidates(const uint32_t* col, int cm, int mpos, FX fx, int K, int cnt,
                                     uint32_t cand[kOvBlocks]) {
    // planes of the 32 positions from mpos + 32 * i (i = block): low-bit plane, high-bit plane,
    // from a stream of the column's code words (two new LDS words per block).  Unclamped: mpos >= 0,
    // and words past the column (the N field, or the next wave's column: valid LDS) only feed
    // offsets >= cnt, which the block masks drop.
    const int sh = 2 * (mpos & 15);
    const uint32_t* W = col + (kFC + (mpos >> 4)) * 64 + cm;
    uint32_t wlo = W[0];
    auto planes = [&](uint32_t& lp, uint32_t& hp) {
        const uint32_t wm = W[64], whi = W[128];
        W += 128;
        const uint32_t u0 = unzip2(__builtin_amdgcn_alignbit(wm, wlo, sh));
        const uint32_t u1 = unzip2(__builtin_amdgcn_alignbit(whi, wm, sh));
        wlo = whi;
        lp = __builtin_amdgcn_perm(u1, u0, 0x05040100u);  // u0 bits 0-15 | u1 bits 0-15 << 16
        hp = __builtin_amdgcn_perm(u1, u0, 0x07060302u);  // u0 bits 16-31 | u1 bits 16-31 << 16
    };
    uint32_t L0, H0, L1, H1;
    planes(L0, H0);
    int nblk = 2;  // blocks holding some lane's offsets (wave-uniform)
#pragma unroll
    for (int k = 2; k < kOvBlocks; ++k)
        if (__any(cnt > 32 * k)) nblk = k + 1;
#if FQ_OV_CSHIFT
    // the blocks' words enter a shift register at the top, the others moving down one (kOvBlocks - 1
    // moves per block instead of a select per word on the runtime index bk); after the loop they sit
    // kOvBlocks - nblk places too high and move down with zeros
    uint32_t creg[kOvBlocks];
#pragma unroll
    for (int i = 0; i < kOvBlocks; ++i) creg[i] = 0u;
#else
#pragma unroll
    for (int bk = 0; bk < kOvBlocks; ++bk)
        if (bk >= nblk) cand[bk] = 0u;
#endif
#pragma unroll 1
    for (int bk = 0; bk < nblk; ++bk) {
        fx.next_block();
        if (bk < kOvBlocks - 1) planes(L1, H1);
        else L1 = H1 = 0u;
        // mismatch vector of compared position j over the block's 32 offsets
#if FQ_OV_SH64
        const unsigned long long HA = (unsigned long long)H1 << 32 | H0, LA = (unsigned long long)L1 << 32 | L0;
        auto shr64 = [](unsigned long long v, int j) -> uint32_t {
            unsigned long long r;
            asm("v_lshrrev_b64 %0, %2, %1" : "=v"(r) : "v"(v), "i"(j));
            return (uint32_t)r;
        };
#endif
        auto m = [&](int j) -> uint32_t {
#if FQ_OV_SH64
            const uint32_t hs = j ? shr64(HA, j) : H0;
            const uint32_t ls = j ? shr64(LA, j) : L0;
#else
            const uint32_t hs = j ? __builtin_amdgcn_alignbit(H1, H0, j) : H0;
            const uint32_t ls = j ? __builtin_amdgcn_alignbit(L1, L0, j) : L0;
#endif
            uint32_t fh, fl;
            fx.bits(j, fh, fl);
            return (hs ^ fh) | (ls ^ fl);
        };
        uint32_t lt;
#if FQ_OV12
        if (K == 5) {
            // the default limit: an accepted offset has < 5 mismatches in its first min(ol, 50)
            // positions, so in its first 12 (ol >= 16 here) -- a weaker filter than 16 positions
            // (~0.3 random candidates per 120 offsets instead of ~0.004, each one exact check) at
            // three quarters of the cost
            uint32_t ones = 0u, twos = 0u, fours = 0u, twosA, twosB, foursA, foursB, eightsA;
            csa(twosA, ones, ones, m(0), m(1));
            csa(twosB, ones, ones, m(2), m(3));
            csa(foursA, twos, twos, twosA, twosB);
            csa(twosA, ones, ones, m(4), m(5));
            csa(twosB, ones, ones, m(6), m(7));
            csa(foursB, twos, twos, twosA, twosB);
            csa(eightsA, fours, fours, foursA, foursB);
            csa(twosA, ones, ones, m(8), m(9));
            csa(twosB, ones, ones, m(10), m(11));
            csa(foursA, twos, twos, twosA, twosB);
            // count = ones + 2 twos + 4 (fours + foursA) + 8 eightsA < 5
            lt = ~(eightsA | (fours & foursA) | ((fours | foursA) & (twos | ones)));
        } else
#endif
        {
        // 16 vectors -> bit-sliced 5-bit counts, Harley-Seal carry-save order (few live values)
        uint32_t ones = 0u, twos = 0u, fours = 0u, eights = 0u, sixteen, twosA, twosB, foursA, foursB, eightsA, eightsB;
        csa(twosA, ones, ones, m(0), m(1));
        csa(twosB, ones, ones, m(2), m(3));
        csa(foursA, twos, twos, twosA, twosB);
        csa(twosA, ones, ones, m(4), m(5));
        csa(twosB, ones, ones, m(6), m(7));
        csa(foursB, twos, twos, twosA, twosB);
        csa(eightsA, fours, fours, foursA, foursB);
        csa(twosA, ones, ones, m(8), m(9));
        csa(twosB, ones, ones, m(10), m(11));
        csa(foursA, twos, twos, twosA, twosB);
        csa(twosA, ones, ones, m(12), m(13));
        csa(twosB, ones, ones, m(14), m(15));
        csa(foursB, twos, twos, twosA, twosB);
        csa(eightsB, fours, fours, foursA, foursB);
        if (K == 5) {  // the default overlap_diff_limit: count < 5 <=> no 8s or 16s, not (4 and (2 or 1))
            lt = ~(eights | eightsA | eightsB | (fours & (twos | ones)));
        } else {  // count < K, bit-sliced against the wave-uniform K
            csa(sixteen, eights, eights, eightsA, eightsB);
            uint32_t eq = ~0u;
            lt = 0u;
            const uint32_t cb[5] = {ones, twos, fours, eights, sixteen};
#pragma unroll
            for (int i = 4; i >= 0; --i) {
                if ((K >> i) & 1) {
                    lt |= eq & ~cb[i];
                    eq &= cb[i];
                } else {
                    eq &= ~cb[i];
                }
            }
            if (K > 31) lt = ~0u;
        }
        }
        const int nb = cnt - 32 * bk;  // valid offsets of this block
#if FQ_OV_CSHIFT
        // bits [0, nb), nb clamped to [0, 32]: the low word of ~(~0 << nb) by one 64-bit shift
        int nbc;
        asm("v_med3_i32 %0, %1, 0, 32" : "=v"(nbc) : "v"(nb));
        unsigned long long nbx;
        asm("v_lshlrev_b64 %0, %1, -1" : "=v"(nbx) : "v"(nbc));
#pragma unroll
        for (int i = 0; i + 1 < kOvBlocks; ++i) creg[i] = creg[i + 1];
        creg[kOvBlocks - 1] = lt & ~(uint32_t)nbx;
#else
        cand[bk] = lt & (nb >= 32 ? ~0u : nb <= 0 ? 0u : ((1u << nb) - 1u));
#endif
        L0 = L1;
        H0 = H1;
    }
#if FQ_OV_CSHIFT
#pragma unroll 1
    for (int s = nblk; s < kOvBlocks; ++s) {
#pragma unroll
        for (int i = 0; i + 1 < kOvBlocks; ++i) creg[i] = creg[i + 1];
        creg[kOvBlocks - 1] = 0u;
    }
#pragma unroll
    for (int i = 0; i < kOvBlocks; ++i) cand[i] = creg[i];
#endif
}

// AdapterTrimmer::trimBySequence (src/adaptertrimmer.cpp:29-90): the first pos in [start, n - 4)
// whose window holds at most min(n - pos, alen) / 8 byte mismatches against the adapter.  The
// reference tests every pos byte by byte; here a code-level lower bound over the first (up to) 16
// compared positions rejects almost every pos without touching bytes, and only survivors get the
// reference's test, in pos order.  The bound counts code mismatches only (an N or a lowercase base
// shares its code with some upper-case letter), so it never exceeds the byte count: a pos it
// rejects has more mismatches than allowed.  Valid for adapters of >= 20 upper-case ACGT bytes
// (start = -4, and the windows of every negative pos lie inside the adapter's first 20 positions);
// the kernel start sets adw[5], the window words, the adapter column and its bit words (see
// pe_fast_kernel).
//  * pos in [0, n - 16]: full 16-position windows, all at once (ov_candidates; bound < alen/8 + 1,
//    a superset of every pos's own allowance).  The adapter's bits per compared position are the
//    same for every lane of a mate, so they come from LDS (FixedLds) instead of two v_bfe a position;
//  * pos in -4..-1 and [n - 15, n - 5]: one masked window each against that pos's allowance.
// The survivors' test is the reference's byte comparison restated on the columns, 16 positions a
// step: with an upper-case ACGT adapter a read byte differs from the adapter byte iff its code
// differs or it is not an upper-case A C G T (an N, a lowercase or an exotic byte: the N word's
// flags), so the mismatch count is one popcount per 16 positions (no per-byte loop whose length
// one lane's candidate imposes on its wave).
// Read 2's column is the reverse complement (forward position j of the read window at column
// kMaxLen - 1 - st - j), so its windows run down the column and its adapter words are stored
// reversed and complemented; `fixed` word k = codes of adapter positions k .. k + 15.
__device__ inline bool adseq_search(const uint32_t* col, int c, bool rc, int st, int n, const uint32_t* adw,
                                    const uint32_t* adc, uint32_t adf, int alen, int& pos_out) {
    // The reference's inner loop at pos (src/adaptertrimmer.cpp:59-71) on the columns, 16 positions a
    // step: with an upper-case ACGT adapter a read byte differs from the adapter's iff its code
    // differs or it is not an upper-case A C G T (an N, a lowercase or an exotic byte: the N word's
    // flags).  (Read windows by field_window_masked: only in-read positions are compared; adapter
    // windows from the mate's adapter column.)
    auto exact = [&](int pos) -> bool {
        const int cmplen = min(n - pos, alen), allowed = cmplen / 8;
        int mm = 0;
#pragma unroll 1
        for (int i = max(0, -pos); i < cmplen; i += 16) {
            const int m = min(16, cmplen - i), q = pos + i;
            const int sc = rc ? kMaxLen - 16 - st - q : st + q;
            const uint32_t rw = field_window_masked(col, kFC, c, sc), rn = field_window_masked(col, kFN, c, sc);
            const int x = rc ? kAdRc - 16 - i : i;
            const uint32_t* aq = adc + (x >> 4);
            const uint32_t aw = __builtin_amdgcn_alignbit(aq[1], aq[0], 2 * (x & 15));
            const uint32_t mask = rc ? 0x55555555u & ~posmask(16 - m) : posmask(m);
            mm += __popc((fold2(rw ^ aw) | rn | (rn >> 1)) & mask);
        }
        return mm <= allowed;
    };
    // pos -4 .. -1: the read's first 16 positions (one window) against adapter words 4 .. 1, the
    // first min(n, 16) read positions compared
    {
        const uint32_t r0 = field_window(col, kFC, c, rc ? kMaxLen - 16 - st : st);
        const int m0 = min(n, 16);
        const uint32_t mask = rc ? 0x55555555u & ~posmask(16 - m0) : posmask(m0);
        for (int pos = -4; pos < 0; ++pos) {
            if (pos >= n - 4) return false;
            if (__popc(fold2(r0 ^ adw[-pos]) & mask) <= min(n - pos, alen) / 8 && exact(pos)) {
                pos_out = pos;
                return true;
            }
        }
    }
    if (n >= 16) {
        uint32_t cand[kOvBlocks];
#if FQ_ADSEQ_LDSBITS
        ov_candidates(col, c, rc ? kMaxLen - st - n : st, FixedLds{adf}, alen / 8 + 1, n - 15, cand);
#else
        ov_candidates(col, c, rc ? kMaxLen - st - n : st, FixedOwn{unzip2(adw[0])}, alen / 8 + 1, n - 15, cand);
#endif
        for (;;) {  // candidates in pos order: read 1 from the lowest offset, read 2 from the highest
            int k = -1;
            if (!rc) {
#pragma unroll
                for (int bk = kOvBlocks - 1; bk >= 0; --bk)
                    if (cand[bk]) k = 32 * bk + __ffs(cand[bk]) - 1;
            } else {
#pragma unroll
                for (int bk = 0; bk < kOvBlocks; ++bk)
                    if (cand[bk]) k = 32 * bk + 31 - __clz(cand[bk]);
            }
            if (k < 0) break;
            cand[k >> 5] &= ~(1u << (k & 31));
            const int pos = rc ? n - 16 - k : k;
            if (exact(pos)) {
                pos_out = pos;
                return true;
            }
        }
    }
    // pos n - 15 .. n - 5: m = n - pos < 16 <= alen positions, all inside the read's last 16, against
    // the adapter's first m -- decided exactly from one window of the read's codes and flags (read 1:
    // its last m fields shifted down to the adapter's first m; read 2, whose window runs backwards:
    // the adapter word, reversed, shifted down instead)
    {
        const int se = rc ? kMaxLen - st - n : st + n - 16;
        const uint32_t rw = field_window(col, kFC, c, se), rn = field_window(col, kFN, c, se);
        const uint32_t aw = adw[0];
        for (int pos = max(0, n - 15); pos < n - 4; ++pos) {
            const int m = n - pos, sh = 2 * (16 - m);
            const uint32_t a = rc ? rw : rw >> sh, f = rc ? rn : rn >> sh, b = rc ? aw >> sh : aw;
            if (__popc((fold2(a ^ b) | f | (f >> 1)) & posmask(m)) <= m / 8) {
                pos_out = pos;
                return true;
            }
        }
    }
    return false;
}


// PolyX::trimPolyG (src/polyx.cpp:14-38) on the code columns, one pass over 16-position groups
// of scan indices (scan index i = forward position e - i, e = the window's last base).  A group
// is one field_window of the column: read 2's column is the reverse complement, so its scan order
// is the column order and a forward G is a stored C; read 1's group is the forward window
// reversed.  The scan changes state only at non-G bases (with maxMM >= 0 the allowance never
// shrinks, so a G never breaks it); a group whose non-G count cannot exceed the allowance at its
// first index is passed over with one popcount, otherwise its non-G bases are visited in order
// with find-first-set.  allowed(i) = min(maxMM, max(1, (i+1)/per)); (i+1)/per = ((i+1)*inv) >> 16
// with inv = ceil(65536/per) is exact for i+1 <= 161 and per <= 256 (inv = 0 for per > 256, where
// the quotient is 0 anyway).  firstGpos, the lowest G position the scan saw, is the highest G scan
// index below the break, tracked per group.  Returns the new window length; bases < 0: not recorded.
__device__ inline int polyg_bits(const uint32_t* col, int c, bool rc, int st, int n, int maxMM, int inv, int per,
                                 int compareReq, int& bases) {
    auto allowed = [&](int x) { return min(maxMM, max(1, inv ? (x * inv) >> 16 : x / per)); };  // x = i + 1
    const int e = st + n - 1;  // last forward position of the window
    int iend = n;              // scan index of the break, or rlen when the scan ran through
    int lastG = -1;            // highest scan index holding a G before the break
    if (maxMM < 0) {
        iend = 0;  // mismatch 0 > allowed at the very first base
    } else {
        int cum = 0;  // non-G bases before the current group
        const uint32_t gx = rc ? 0x55555555u : 0xFFFFFFFFu;  // (G is code 3; read 2's column holds C)
        // spaced non-G mask (N and lowercase included) of scan indices [16g, 16g + 16), in scan order
        auto nong = [&](int g) -> uint32_t {
            const int pos0 = rc ? kMaxLen - 1 - e + 16 * g : e - 16 * g - 15;
            // (positions outside [st, e] are scan indices >= n, dropped by `valid`)
            const uint32_t cw = field_window_masked(col, kFC, c, pos0), nw = field_window_masked(col, kFN, c, pos0);
            const uint32_t t = (cw ^ gx) | nw;
            uint32_t x = (t | (t >> 1)) & 0x55555555u;
            if (!rc) x = __builtin_bitreverse32(x) >> 1;  // forward window -> scan order
            return x;
        };
        uint32_t xg = nong(0);  // group g's non-G mask (group 0 first; later groups loaded one ahead)
#if FQ_PG2
        // Group 0 decides almost every read: while the allowance is 1 (scan indices < 2 per - 1) the
        // scan breaks at the second non-G base; the loop below runs only for the reads it leaves open
        // (a polyG tail, or per < 8).
        if (maxMM >= 1) {
            const uint32_t valid = posmask_v(n), x = xg & valid, x2 = x & (x - 1u);
            const int s2 = (__ffs(x2) - 1) >> 1;
            if (x2 && (maxMM == 1 || s2 + 1 < 2 * per)) {
                iend = s2;
                const uint32_t gm = ~x & valid & posmask_v(s2);  // G bases before the break
                if (gm) lastG = (31 - __clz(gm)) >> 1;
            }
        }
#endif
        int g = 0;
#if FQ_PG4
        // A polyG tail (the reads the shortcut above leaves open): its all-G groups change nothing
        // but firstGpos, so they are passed over at ~16 VALU a group (the loop below spends ~45)
        if (iend == n) {
            while (16 * (g + 1) < n && (xg & posmask_v(n - 16 * g)) == 0u) xg = nong(++g);
            if (g > 0) lastG = 16 * g - 1;  // (scan indices below 16 g are all G)
        }
#endif
        for (; 16 * g < n && iend == n; ++g) {
            const uint32_t valid = posmask_v(n - 16 * g);
#if FQ_PG3
            uint32_t x = xg & valid;
            // the next group's column words are requested before this group is decided (a G tail
            // spans several groups, and each LDS round trip otherwise stalls the few lanes that
            // scan -- and with them their wave); past the window they are masked off by `valid`
            xg = nong(g + 1);
#else
            uint32_t x = (g ? nong(g) : xg) & valid;
#endif
            uint32_t gm = ~x & valid;  // G bases of the group
            const int a0 = allowed(16 * g + 1);  // allowance at the group start
            if (cum + __popc(x) > a0) {
                uint32_t m = x;
                while (m) {
                    const int t = (__ffs(m) - 1) >> 1;
                    const int i = 16 * g + t;
                    ++cum;
                    if (cum > allowed(i + 1)) {
                        iend = i;
                        gm &= posmask(t);  // G bases before the break
                        break;
                    }
                    m &= m - 1;
                }
            } else {
                cum += __popc(x);
            }
            if (gm) lastG = 16 * g + ((31 - __clz(gm)) >> 1);
        }
    }
    bases = -1;
    if (iend + 1 < compareReq) return n;
    const int firstG = lastG >= 0 ? e - lastG - st : n - 1;  // (the reference's default is rlen-1)
    bases = n - firstG;
    return firstG < 0 ? n : firstG;  // (empty window: firstGpos -1, Read::resize(-1) is a no-op)
}

// PolyX::trimPolyX's scan (src/polyx.cpp:51-77) decided on the code column while the allowance
// keeps its first value, min(maxMM, max(1, cmp/per)) = 1 for scan indices i < 2*per - 1: with a
// constant allowance of 1 a base b is out for good from its second non-b base on, so the loop
// breaks at the largest such index over the masked bases (or at 0).  Returns true when that break
// lies in the decided range and before compareReq, i.e. the read is left as it is (the common
// case); false when the scalar restatement (trim_polyx_t) has to run.  Scan index i is forward
// position e - i (e = the window's last base), as in polyg_bits.
__device__ inline bool polyx_no_trim(const uint32_t* col, int c, bool rc, int st, int n, int mask, int maxMM, int per,
                                     int compareReq) {
    if (maxMM < 1 || per < 1 || n <= 0) return false;
    const int e = st + n - 1;
    const int pos0 = rc ? kMaxLen - 1 - e : e - 15;
    // (positions outside the window are scan indices >= lim, dropped by `valid`)
    const uint32_t cw = field_window_masked(col, kFC, c, pos0), nw = field_window_masked(col, kFN, c, pos0);
    const int lim = min(min(2 * per - 1, 16), n);  // scan indices [0, lim) are decided here
    const uint32_t valid = posmask(lim);
    int brk = 0;
    // "ATCGN"[b]: forward codes A 0, T 2, C 1, G 3 (read 2's column holds the complements)
#pragma unroll
    for (int b = 0; b < 5; ++b) {
        if (!((mask >> b) & 1)) continue;
        uint32_t nonb;  // forward-order spaced mask of the positions that are not b
        if (b < 4) {
            const uint32_t code = (uint32_t)((0x3120 >> (4 * b)) & 3) ^ (rc ? 2u : 0u);
            nonb = (fold2(cw ^ (code * 0x55555555u)) | nw | (nw >> 1)) & 0x55555555u;
        } else {  // class 4: N and every other byte (lowercase included), src/polyx.cpp:56-70
            nonb = ~(nw | (nw >> 1)) & 0x55555555u;
        }
        if (!rc) nonb = __builtin_bitreverse32(nonb) >> 1;  // forward window -> scan order
        nonb &= valid;
        const uint32_t second = nonb & (nonb - 1u);
        brk = max(brk, second ? (__ffs(second) - 1) >> 1 : 99);
    }
    return brk < lim && brk + 1 < compareReq;
}

// The four bit-7 flags of a dword's bytes as a nibble (byte k -> bit k)
__device__ __forceinline__ uint32_t flags4(uint32_t t) {
    return ((t >> 7) | (t >> 14) | (t >> 21) | (t >> 28)) & 0xFu;
}

// Filter::trimAndCut (src/filter.cpp:69-189) when cut_right is its only window option and the
// window is at most 4 bases (the default is 4): low_window_scan's result, but each chunk that holds a
// quality below the threshold (bit c of low_chunks, from staging) is decided at once from three
// 16-byte row chunks c-1, c, c+1 (one L2 round trip instead of one per 4 positions): the windows
// starting at 16c-3 .. 16c+15 are summed with v_sad_u8 on realigned dwords (exact integer
// test sum < T*w, win_ge), and the first base below the threshold at or after the first low
// window (the reference's `while (qual(s) >= thr) ++s`, which stops inside that window) comes from
// the bytes' below-threshold flags.  limr = (128 - T) per byte (qualities < 128 in these tiles).
__device__ inline bool cut_right_w4(const fq_params& p, const uint8_t* Q, int nchunks, int l, int front, int tail,
                                    uint32_t low_chunks, uint32_t limr, int& out_start, int& out_len) {
    int rlen = l - front - tail;
    if (rlen < 0) return false;
    const int w = p.cut_right_window, thr = 33 + p.cut_right_quality;
    if (l - front - tail - w <= 0) return false;
    const int send = l - tail - w;  // window starts [front, send) are scanned
    const uint32_t TW = (uint32_t)(thr * w), wm = bytemask(w);
    constexpr int cst = FQ_TILE_READS * FQ_CHUNK;
    int from = front, cut = -1;  // cut: the first base below the threshold from the first low window on
    uint32_t lc = low_chunks;
    while (lc) {
        const int c = __ffs(lc) - 1;
        lc &= lc - 1u;
        const int a = max(from, 16 * c - w + 1), bnd = min(send, 16 * c + 16);
        if (a < bnd) {
            const uint4 z = make_uint4(0u, 0u, 0u, 0u);
            const uint4 q0 = c > 0 ? *reinterpret_cast<const uint4*>(Q + cst * (c - 1)) : z;
            const uint4 q1 = *reinterpret_cast<const uint4*>(Q + cst * c);
            const uint4 q2 = c + 1 < nchunks ? *reinterpret_cast<const uint4*>(Q + cst * (c + 1)) : z;
            const uint32_t d[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
            uint32_t win = 0;  // bit j: the window starting at 16c - 3 + j is low (sum < TW)
#pragma unroll
            for (int j = 18; j >= 0; --j) {
                const int o = 13 + j;  // its byte offset in d
                const uint32_t W = (o & 3) ? __builtin_amdgcn_alignbyte(d[(o >> 2) + 1], d[o >> 2], o & 3) : d[o >> 2];
                win = shift_in_sign(win, __builtin_amdgcn_sad_u8(W & wm, 0u, 0u) - TW);
            }
            const int lo = a - (16 * c - 3), hi = bnd - (16 * c - 3);  // 0 <= lo < hi <= 19
            win &= ((1u << hi) - 1u) & ~((1u << lo) - 1u);
            if (win) {
                const int j = __ffs(win) - 1;
                // below-threshold flags of bytes 12..35 of d (bit i: byte 12 + i)
                uint32_t lowb = 0;
#pragma unroll
                for (int k = 3; k < 9; ++k) lowb |= flags4(~(d[k] + limr) & 0x80808080u) << (4 * (k - 3));
                cut = 16 * c - 3 + j + __ffs(lowb >> (j + 1)) - 1;  // (the window holds such a base)
                break;
            }
        }
        from = max(from, bnd);
        if (from >= send) break;
    }
    if (cut >= 0) rlen = cut - front;
    if (rlen <= 0 || front >= l - 1) return false;
    out_start = front;
    out_len = min(rlen, l - front);
    return true;
}

// (rare) the flags of one lane's read that holds a byte outside ACGTN: re-reads its row chunks and
// marks, in the column,
//   * a lowercase a c g t (the uppercase letter | 0x20, whose 3-bit key and code are the uppercase
//     letter's): a flag at the odd bit of the N word;
//   * any other byte ("exotic": IUPAC codes, 'n', ...): code 3 with the N bit and the odd bit, so
//     the comparing passes see a byte that equals nothing in read 1 and reads as 'N' in read 2's
//     reverse complement (src/seq.h:24-48), and Stats counts it as N until its fix-up moves it to
//     its class byte & 7 (src/stats.cpp:249).  passFilter counts only 'N' (src/filter.cpp:18):
//     staging counted an exotic byte with key bit 2 as one, so it is taken off the prefix words (pfx:
//     the lane's first prefix word, or null; step: chunks per word) and, by the caller, off nbf.
// Returns bit 0 (hand the pair over: exotic bytes where they are not taken, allow_exotic false),
// bit 1 (the read holds exotic bytes) and, from bit 2 on, the count staging took for 'N's.  xp: the lane's column word of row chunk 0 (read 2: its
// reverse complement, stepped by wstep).
typedef __attribute__((address_space(3))) uint32_t LdsU32;  // (LDS pointers: a generic one costs the caller
                                                            // a 64-bit flat address held across the tile)
template <bool PAIRED>
__device__ __attribute__((noinline)) int lower_flags(const uint8_t* S, LdsU32* xp, int wstep, int nch, int L, bool rc,
                                                    uint32_t rsel, LdsU32* pfx, int step, bool allow_exotic) {
    constexpr int cst = FQ_TILE_READS * FQ_CHUNK;
    bool exotic = false;
    int ntot = 0;
    for (int k = 0; k < nch; ++k, xp += wstep) {
        const uint4 s4 = *reinterpret_cast<const uint4*>(S + cst * k);
        const uint32_t sw[4] = {s4.x, s4.y, s4.z, s4.w};
        const int Lk = L - 16 * k;
        uint32_t x4 = 0, e4 = 0, ncnt = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t sr = PAIRED ? __builtin_amdgcn_perm(sw[3 - j], sw[j], rsel) : sw[j];
            const uint32_t bms = rc ? ~bytemask(16 - Lk - 4 * j) : bytemask(Lk - 4 * j);
            const uint32_t kk = (sr >> 1) & 0x07070707u;
            const uint32_t canon = __builtin_amdgcn_perm(0x4E000000u, 0x47544341u, kk);
            const uint32_t d = (sr ^ canon) & bms;  // per byte: 0 canonical, 0x20 lowercase
            const uint32_t t = d ^ 0x20202020u;
            const uint32_t low = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & ~((kk & 0x04040404u) << 5) &
                                 0x80808080u;  // d == 0x20 and not 'n' (whose key is N's)
            const uint32_t nz = (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;
            const uint32_t ex = nz & ~low;
            ncnt += __popc(ex & ((kk & 0x04040404u) << 5));  // (staging's N flag: key bit 2)
            x4 |= (low >> 7) << (2 * j);
            e4 |= (ex >> 7) << (2 * j);
        }
        const uint32_t vm = rc ? 0x55555555u & ~posmask(16 - Lk) : posmask(Lk);
        const uint32_t ef = tr4x4(e4) & vm;
        xp[kFN * 64] |= ((tr4x4(x4) & vm) << 1) | ef | (ef << 1);
        if (ef) {
            exotic = true;
            xp[kFC * 64] |= ef | (ef << 1);  // code 3
            ntot += (int)ncnt;
            if (pfx)
                for (int j = k / step; (j + 1) * step <= nch; ++j) pfx[j * 64] -= ncnt << 24;
        }
    }
    return (exotic && !allow_exotic ? 1 : 0) | (exotic ? 2 : 0) | ntot << 2;
}

__device__ __forceinline__ void sadd(unsigned long long* p, unsigned long long v) { atomicAdd(p, v); }

typedef __attribute__((address_space(3))) unsigned long long LdsU64;  // a u64 at an LDS byte address

// base[v] += w for every lane with `on`: one LDS atomic per distinct v in the wave instead of one
// per lane (lanes of a tile mostly share a value, e.g. the filter code 0).  Wave-uniform call.
__device__ __forceinline__ void count_by_value(unsigned long long* base, bool on, int v, unsigned long long w) {
    unsigned long long m = __ballot(on);
    while (m) {
        const int first = __ffsll((long long)m) - 1;
        const int c = __builtin_amdgcn_readlane(v, first);
        const unsigned long long mc = __ballot(on && v == c);
        m &= ~mc;
        if ((int)(threadIdx.x & 63) == first) atomicAdd(&base[c], w * (unsigned long long)__popcll(mc));
    }
}



// Profiling aid: per-phase wave cycles (s_memtime deltas summed over waves), compiled in with
// -DFQ_PHASE_STAMPS (make STAMPS=1), collected when fq_params.reserved[1] != 0 and read back with
// fq_debug_phase_cycles().
constexpr int kPhases = 8;  // staging, trim, polyG, overlap, polyX/maxlen, filter, stats, store
__device__ unsigned long long g_phase_cycles[kPhases];

__device__ __forceinline__ void hadd(uint32_t* base, int word, unsigned long long v) {
    atomicAdd(reinterpret_cast<unsigned long long*>(base + word), v);
}

// histogram slot (A C T G N) -> Stats base class (byte & 7), src/stats.cpp:249
__device__ __forceinline__ int slot_class(int s) { return (0x67431 >> (4 * s)) & 0xF; }

// LEAN: the option set of the headline workloads (no trimming/cutting windows, -e, polyX, adapter
// sequences, maxLen or low-complexity filter), instantiated separately so the hot loop carries
// neither their code nor their parameters.
// PAIRED: a tile is 32 pairs, lanes l and l+32 holding the two mates of a pair (read 2's column
// reverse-complemented for the overlap scan); single-end: a tile is 64 reads, one per lane, with
// SingleEndProcessor::processSingleEnd's order (src/seprocessor.cpp:290-360).
// BaseCorrector::correctByOverlapAnalysis (src/basecorrector.cpp:14-70) for one pair with
// 0 < diff <= 5, run by both lanes of the pair (the decisions are pair-uniform; each lane applies
// its own read's corrections).  A mismatch of the overlap (as OverlapAnalysis counts it: N == N,
// N != base) where one side is >= Q30 and the other <= Q14 takes the good side's base
// (complemented) and quality.  Each correction is applied where the later steps read the read: the
// lane's code column (read 2's column holds the reverse complement, so the new code is the other
// column's code as stored), its quality row in HBM (rewritten in place, as the general kernel
// does), and the whole-read sums that passFilter and the post statistics derive their window sums
// from.  The pre-trimming statistics must see the original read (src/peprocessor.cpp:276-277):
// the removed-mode Stats pass counts the corrected base, so the removed block gets
// (original - corrected) at the base's cycle (pre = kept + removed), and the per-read pre Q20/Q30
// scalar gets the negated deltas.  Host side: the FASTQ text is corrected from the read-2 record's
// (offset, overlap length, window length), flags FQ_RF_CORRECTED.
__device__ inline bool correct_pair_fast(const fq_params& p, uint32_t* col, uint32_t* lds, const fq_batch& b, size_t roff,
                                         int mate, int lane_x, int mlane, int st1, int st2, int n2, const Overlap& ov,
                                         const uint8_t* Q, fq_read_result& rr, uint32_t& q20, uint32_t& q30,
                                         uint32_t& lowf, uint32_t& tqf, uint32_t& nbf, uint32_t limq,
                                         unsigned long long* pre_q, int rem_block, bool removed, unsigned long long* acc) {
    const int ol = ov.len;
    const int start1 = max(0, ov.offset), start2 = n2 - max(0, -ov.offset) - 1;
    const int a0 = st1 + start1;                  // read 1's forward position at overlap index 0
    const int b0 = kMaxLen - 1 - (st2 + start2);  // read 2's column (reverse complement) index at 0
    const int c1 = mate ? mlane : lane_x, c2 = mate ? lane_x : mlane;
    const RowQual Q1{b.qual1 + roff, b.stride >> 2}, Q2{b.qual2 + roff, b.stride >> 2};
    uint8_t* myq = const_cast<uint8_t*>(Q);
    const int good = 33 + 30, bad = 33 + 14;  // util::num2qual(30), util::num2qual(14)
    int corrected = 0;
    bool cr1 = false, cr2 = false;
    int d20 = 0, d30 = 0;
    // the whole-read sums' per-byte terms (staging's SWAR tests on one byte)
    auto f20 = [](uint32_t q) { return (int)(((q + 0x4Au) >> 7) & 1u); };
    auto f30 = [](uint32_t q) { return (int)(((q + 0x40u) >> 7) & 1u); };
    auto flow = [&](uint32_t q) { return (int)((~(q + (limq & 0xFFu)) >> 7) & 1u); };
    for (int j = 0; 16 * j < ol; ++j) {
        const uint32_t a = field_window(col, kFC, c1, a0 + 16 * j), wa = field_window(col, kFN, c1, a0 + 16 * j);
        const uint32_t bb = field_window(col, kFC, c2, b0 + 16 * j), wb = field_window(col, kFN, c2, b0 + 16 * j);
        uint32_t mism = ((fold2(a ^ bb) & ~(wa | wb)) | (wa ^ wb)) & posmask(ol - 16 * j);
        while (mism) {
            const int t = (__ffs(mism) - 1) >> 1;
            mism &= mism - 1u;
            const int i = 16 * j + t;
            const int p1 = a0 + i, p2 = st2 + start2 - i;
            const uint32_t x1 = (uint32_t)Q1(p1), x2 = (uint32_t)Q2(p2);
            // read 1's forward code / N flag; read 2's column code (its complement) / N flag
            const uint32_t k1 = (a >> (2 * t)) & 3u, n1 = (wa >> (2 * t)) & 1u;
            const uint32_t k2 = (bb >> (2 * t)) & 3u, nb2 = (wb >> (2 * t)) & 1u;
            int side;  // the read that takes the other's base: 1, 2, or 0 (none)
            if ((int)x1 >= good && (int)x2 <= bad) side = 2;
            else if ((int)x2 >= good && (int)x1 <= bad) side = 1;
            else continue;
            ++corrected;
            if (side == 1) cr1 = true;
            else cr2 = true;
            if (side != mate + 1) continue;
            // this lane's read: forward position P, column index ci, new column code / N flag
            const int P = mate ? p2 : p1, ci = mate ? b0 + i : p1;
            const uint32_t ncode = mate ? k1 : k2, nN = mate ? n1 : nb2;
            const uint32_t ocode = mate ? k2 : k1, oN = mate ? nb2 : n1;
            const uint32_t xo = mate ? x2 : x1, xn = mate ? x1 : x2;
            const int w = ci >> 4, sh = 2 * (ci & 15);
            uint32_t& cw = col[(kFC + w) * 64 + lane_x];
            uint32_t& nw = col[(kFN + w) * 64 + lane_x];
            cw = (cw & ~(3u << sh)) | (ncode << sh);
            nw = (nw & ~(1u << sh)) | (nN << sh);
            myq[(P >> 4) * (FQ_TILE_READS * FQ_CHUNK) + (P & 15)] = (uint8_t)xn;
            const int e20 = f20(xn) - f20(xo), e30 = f30(xn) - f30(xo);
            d20 += e20;
            d30 += e30;
            q20 += (uint32_t)e20;
            q30 += (uint32_t)e30;
            lowf += (uint32_t)(flow(xn) - flow(xo));
            tqf += xn - xo;
            nbf += nN - oN;
            // forward codes (read 2's column holds complements; N stays code 3) -> removed slots
            // (removed mode), or the pre block's slots A C T G N with the +128 quality bias
            // (pre/post mode: front trimming, UMI)
            const uint32_t fo = mate && !oN ? ocode ^ 2u : ocode, fn = mate && !nN ? ncode ^ 2u : ncode;
            if (removed) {
                const int so = oN ? kRNSlot : (int)fo, sn = nN ? kRNSlot : (int)fn;
                atomicAdd(reinterpret_cast<unsigned long long*>(lds + rem_block + rcell(P, so)), kCount1 | (unsigned long long)xo);
                atomicAdd(reinterpret_cast<unsigned long long*>(lds + rem_block + rcell(P, sn)), 0ull - (kCount1 | (unsigned long long)xn));
            } else {
                const int so = oN ? 4 : (int)fo, sn = nN ? 4 : (int)fn;
                atomicAdd(reinterpret_cast<unsigned long long*>(lds + rem_block + cell(P, so)), kCount1 | (unsigned long long)(xo | 0x80u));
                atomicAdd(reinterpret_cast<unsigned long long*>(lds + rem_block + cell(P, sn)), 0ull - (kCount1 | (unsigned long long)(xn | 0x80u)));
            }
        }
    }
    if (!corrected) return false;
    if (d20 | d30) atomicAdd(pre_q, 0ull - (unsigned long long)((long long)d20 * 4294967296LL + (long long)d30));
    if (mate ? cr2 : cr1) rr.flags |= FQ_RF_CORRECTED;
    if (mate) {  // what the host needs to correct the text (as fq_pack_kernel's correct_pair)
        rr.m_len1 = (uint16_t)(int16_t)ov.offset;
        rr.m_len2 = (uint16_t)ol;
        rr.reserved = (uint16_t)n2;
    } else {
        unsigned long long* tail = acc + acc_stats_offset(p.insert_size_max, p.max_cycles, 4);
        atomicAdd(&tail[FQ_ACC_TAIL_CORRECTED_READS], (cr1 && cr2) ? 2ull : 1ull);
        atomicAdd(&tail[FQ_ACC_TAIL_CORRECTED_BASES], (unsigned long long)corrected);
    }
    return true;  // (pair-uniform: both lanes walk the same mismatches)
}

// Per-launch constants derived from fq_params.  With FQ_PLAUNDER the kernel derives them again at the
// top of every tile from a re-read of the kernarg segment (see the tile loop).
#define FQ_DERIVE_PARAMS() \
    [[maybe_unused]] const int abl = p.reserved[0]; \
    [[maybe_unused]] const int nchunks = FIX ? kChunks : min(kChunks, b.stride >> 4); \
    [[maybe_unused]] const int limit = p.overlap_diff_limit; \
    [[maybe_unused]] const int K = max(limit, 1); \
    [[maybe_unused]] const int req = p.overlap_require; \
    [[maybe_unused]] const uint32_t limq = (uint32_t)(0x80 - p.low_qual_limit) * 0x01010101u; \
    /* cut_right threshold 33 + q, in 0..93 (CLI range): the same SWAR below-threshold test */ \
    [[maybe_unused]] const bool lowr_ok = p.cut_right && 33 + p.cut_right_quality >= 1 && 33 + p.cut_right_quality <= 127; \
    [[maybe_unused]] const uint32_t limr = lowr_ok ? (uint32_t)(0x80 - (33 + p.cut_right_quality)) * 0x01010101u : 0u; \
    /* cut_right as the only window option, window <= 4: cut_right_w4 */ \
    /* UMI in the reads (src/umiprocessor.cpp:10-89, trimFront before trimAndCut): trimAndCut runs on */ \
    /* the read from umi_cut(umi_front, len) on (the general path of trim_and_cut_t) */ \
    [[maybe_unused]] const bool umi = XTRA && (p.umi_front1 > 0 || p.umi_front2 > 0); \
    [[maybe_unused]] const bool cut_w4 = FQ_CUT_W4 && lowr_ok && !umi && !p.cut_front && !p.cut_tail && p.cut_right_window >= 1 && \
                        p.cut_right_window <= 4; \
    /* Without front trimming every kept window starts at 0, so each base lands in exactly one of */ \
    /* two disjoint blocks: "kept" (inside a passing read's window; the post block) or "removed" */ \
    /* (trimmed tails, failed pairs; the pre block), one LDS atomic per base.  At the flush */ \
    /* pre = kept + removed and post = kept. */ \
    [[maybe_unused]] const bool removed_mode = LEAN || (p.trim_front1 == 0 && p.trim_front2 == 0 && !p.cut_front && !umi); \
    [[maybe_unused]] const int g_per = max(p.polyg_one_mismatch_per, 1); \
    /* (i+1)/per as ((i+1)*inv) >> 16, exact while per * (kMaxLen + 1) < 65536; else inv = 0: division */ \
    [[maybe_unused]] const int g_inv = g_per * (kMaxLen + 1) < 65536 ? (65536 + g_per - 1) / g_per : 0;

// XTRA: the -c / UMI / -e instantiation of the full variants (kept apart so the other variants'
// register allocation does not carry that code)
// FIX: rows of exactly kChunks chunks (the batch stride is the column length: 160, or 320 in the long
// build), so every per-chunk offset and bound is a compile-time constant
template <bool LEAN, bool PAIRED, bool MERGE, bool XTRA = false, bool FIX = false>
__global__ void __launch_bounds__((Layout<LEAN, MERGE, PAIRED>::kThreads)) __attribute__((amdgpu_waves_per_eu(Layout<LEAN, MERGE, PAIRED>::kWavesPerEU))) pe_fast_kernel(fq_params p, fq_batch b, fq_read_result* __restrict__ res,
                                                         unsigned long long* __restrict__ acc, int* __restrict__ slow_tiles,
                                                         int* __restrict__ slow_count, unsigned long long* __restrict__ xfix) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int lane = threadIdx.x & 63;
    const int wave = MERGE ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : threadIdx.x >> 6;  // an SGPR frees merge !FIX from its one spill
    using LY = Layout<LEAN, MERGE, PAIRED>;
    constexpr int kWaves = LY::kWaves, kThreads = LY::kThreads;
    // the paired exact check where it fits the registers (FULL without -m spills with it)
    constexpr bool kOvx2 = FQ_OVX2 && (LEAN || MERGE);
    uint32_t* col = lds + wave * LY::kWaveW;  // code / N columns: word field*64 + lane
    uint32_t* qrows = col + kCodeW;           // full variant: quality rows, row = lane
    uint32_t* hist = lds + LY::kColsW;        // [pre1, pre2, post1, post2] x kHistW (post1 x2 with MERGE)
    unsigned long long* small = reinterpret_cast<unsigned long long*>(hist + LY::kHistRegW);
    unsigned int* ins = reinterpret_cast<unsigned int*>(small + kSmallW / 2);
    unsigned long long* scal = reinterpret_cast<unsigned long long*>(ins + kInsW);
    uint8_t* adp = reinterpret_cast<uint8_t*>(scal + kScalStride * LY::kScalCopies);
    int* hres = reinterpret_cast<int*>(adp) + kAdW;  // [wave][next slot, slots left]
    for (int i = threadIdx.x; i < LY::kHrW; i += kThreads) hres[i] = 0;
    for (int i = threadIdx.x; i < LY::kHistRegW + kSmallW + kInsW + LY::kScalW; i += kThreads) hist[i] = 0;
    for (int i = threadIdx.x; i < 2 * FQ_MAX_ADAPTER; i += kThreads)
        adp[i] = i < FQ_MAX_ADAPTER ? p.adapter1[i] : p.adapter2[i - FQ_MAX_ADAPTER];
    // adseq_search's words: [mate * 8 + k] = 2-bit codes of adapter positions k .. k + 15 (k < 5;
    // read 2: reversed and complemented, column order), [mate * 8 + 5] = 1 when the filter applies
    // (>= 20 upper-case ACGT bytes)
    uint32_t* adw = reinterpret_cast<uint32_t*>(adp) + 2 * FQ_MAX_ADAPTER / 4;
    if (threadIdx.x < 12) {
        const int m = threadIdx.x / 6, k = threadIdx.x % 6;
        const uint8_t* a = m ? p.adapter2 : p.adapter1;
        const int alen = m ? p.adapter2_len : p.adapter1_len;
        uint32_t w = 0;
        if (k < 5) {
            for (int j = 0; j < 16; ++j) w |= (uint32_t)((a[k + j] >> 1) & 3) << (2 * j);  // A C T G -> 0 1 2 3
            if (m) w = pairrev(w) ^ 0xAAAAAAAAu;
        } else {
            w = alen >= 20 && alen <= FQ_MAX_ADAPTER;
            for (int j = 0; j < alen && j < FQ_MAX_ADAPTER; ++j) {
                const uint8_t ch = a[j];
                if (ch != 'A' && ch != 'C' && ch != 'G' && ch != 'T') w = 0;
            }
        }
        adw[8 * m + k] = w;
    } else if (threadIdx.x < 12 + 2 * kAdCW) {
        // adapter columns: mate 0 word w = codes of positions 16 w .. 16 w + 15; mate 1 index y = the
        // complemented code of position kAdRc - 1 - y (positions past the buffer: code 0, never compared)
        const int m = (threadIdx.x - 12) / kAdCW, w = (threadIdx.x - 12) % kAdCW;
        const uint8_t* a = m ? p.adapter2 : p.adapter1;
        uint32_t v = 0;
        for (int f = 0; f < 16; ++f) {
            const int y = 16 * w + f, q = m ? kAdRc - 1 - y : y;
            if (q >= 0 && q < FQ_MAX_ADAPTER) v |= (uint32_t)(((a[q] >> 1) & 3) ^ (m ? 2 : 0)) << (2 * f);
        }
        adw[kAdColOff - kAdWinOff + m * kAdCW + w] = v;
    } else if (threadIdx.x >= 64 && threadIdx.x < 64 + 2 * 16) {
        // (fh, fl) of compared position j of each mate's first window (adw[8 m], as ov_candidates'
        // FixedOwn would derive them)
        const int m = (threadIdx.x - 64) >> 4, j = (threadIdx.x - 64) & 15;
        const uint8_t* a = m ? p.adapter2 : p.adapter1;
        uint32_t w = 0;
        for (int f = 0; f < 16; ++f) w |= (uint32_t)((a[f] >> 1) & 3) << (2 * f);
        if (m) w = pairrev(w) ^ 0xAAAAAAAAu;
        const uint32_t fu = unzip2(w);
        adw[kAdBitOff - kAdWinOff + 2 * (16 * m + j)] = 0u - ((fu >> (16 + j)) & 1u);
        adw[kAdBitOff - kAdWinOff + 2 * (16 * m + j) + 1] = 0u - ((fu >> j) & 1u);
    }
    __syncthreads();

    const int ntiles = PAIRED ? (b.n + 31) >> 5 : (b.n + 63) >> 6;
    // Profiling-only ablation bits (fq_params.reserved[0]; results are wrong when set):
    // 1 skip overlap, 2 skip passFilter scan, 4 skip stats pass, 8 skip polyG, 16 skip LDS atomics,
    // 32 skip the polyG counters, 64 accept the first scan candidate unchecked, 128 skip the scan,
    // 1024 skip trimAndCut (FULL), 2048 skip polyX
    FQ_DERIVE_PARAMS()
#ifdef FQ_PHASE_STAMPS
    const bool stamps = p.reserved[1] != 0;
    unsigned long long ph[kPhases] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long t_last = stamps ? clock64() : 0;
#define FQ_STAMP(i)                                \
    if (stamps) {                                  \
        const unsigned long long now_ = clock64(); \
        ph[i] += now_ - t_last;                    \
        t_last = now_;                             \
    }
#else
#define FQ_STAMP(i)
#endif

#if FQ_DESYNC
    {   // profiling: stagger the waves that share a SIMD (wave w, w + 4 of both workgroups of a CU)
        const int slot = (wave >> 2) + 2 * (blockIdx.x & 1);
        for (int i = 0; i < slot * FQ_DESYNC; ++i) __builtin_amdgcn_s_sleep(127);
    }
#endif
    // hand-off list: a wave reserves kItems slots at a time (its reservation lives in LDS, hres,
    // read only on the rare hand-off path)
    constexpr int kItems = PAIRED ? 32 : 64;
    constexpr int kHole = 0x7FFFFFFF;
    for (int t = blockIdx.x * kWaves + wave; t < ntiles; t += gridDim.x * kWaves) {
#if FQ_PLAUNDER
        // The parameters and the batch descriptor are re-read from the kernarg segment every tile
        // (scalar loads, cached): kept live across the tile loop they overflow the SGPR file, and the
        // spills cost VALU (v_writelane / v_readlane) and scratch traffic inside the loop.
        typedef const __attribute__((address_space(4))) fq_params KParams;
        typedef const __attribute__((address_space(4))) fq_batch KBatch;
        // (the kernel's first two arguments, at their ABI offsets in the kernarg segment: p at 0, b at
        // the next multiple of its alignment; taking &p instead would copy p to scratch)
        const __attribute__((address_space(4))) char* ka_ =
            (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
        KParams* kp_ = (KParams*)ka_;
        KBatch* kb_ = (KBatch*)(ka_ + ((sizeof(fq_params) + alignof(fq_batch) - 1) & ~(alignof(fq_batch) - 1)));
        asm volatile("" : "+s"(kp_), "+s"(kb_));
        const fq_params& p = *(const fq_params*)kp_;
        const fq_batch& b = *(const fq_batch*)kb_;
        FQ_DERIVE_PARAMS()
#endif
        // Per-lane values are derived from an opaque copy of the lane id inside the loop: left to
        // itself the compiler hoists dozens of them out of the tile loop and spills them.
        int lane_x = lane;
        asm volatile("" : "+v"(lane_x));
        const int mate = PAIRED ? lane_x >> 5 : 0, pl = lane_x & 31;
        const int mlane = lane_x ^ 32;
        const bool rc = PAIRED && mate == 1;
        const int front = mate ? p.trim_front2 : p.trim_front1;
        const int tail = mate ? p.trim_tail2 : p.trim_tail1;
        const uint8_t* my_ad = adp + (mate ? FQ_MAX_ADAPTER : 0);
        const int my_alen = mate ? p.adapter2_len : p.adapter1_len;
        const int my_maxlen = mate ? p.max_len2 : p.max_len1;
        uint32_t* my_pre = hist + mate * kHistW;
        uint32_t* my_post = hist + (2 + (MERGE ? 2 : 1) * mate) * kHistW;  // post block, or the "removed" block
        const int r = lane_x & 15;  // stats rotation within a chunk
        uint32_t* qrow = qrows + lane_x * kQS;
#ifdef FQ_SAME_TILE  // profiling only: every wave re-reads a few L2-resident tiles (results invalid)
        const int tt = t & (FQ_SAME_TILE - 1);
        const int idx = PAIRED ? tt * 32 + pl : tt * 64 + lane_x;
#else
        const int idx = PAIRED ? t * 32 + pl : t * 64 + lane_x;
#endif
        bool valid = idx < b.n;  // (both cleared below for a pair handed to the general kernel)
        int L = valid ? (int)(mate ? b.len2[idx] : b.len1[idx]) : 0;

        // ---------------- staging ----------------
#if FQ_STAGE_PRIO || FQ_STATS_PRIO_ALL == 2
        __builtin_amdgcn_s_setprio(FQ_STAGE_PRIO);
#endif
        // chunk-interleaved batch tiles (include/fqengine.h): chunk k of this lane's row is 512 B
        // after chunk k-1, so each chunk load of the wave is one (PE: two planes x 32 rows) or
        // two (SE: 64 rows) 512-byte contiguous runs
        constexpr int cst = FQ_TILE_READS * FQ_CHUNK;
        const int ridx = valid ? idx : 0;
        const size_t roff = (size_t)(ridx / FQ_TILE_READS) * FQ_TILE_READS * b.stride + (ridx % FQ_TILE_READS) * FQ_CHUNK;
        const uint8_t* S = (mate ? b.seq2 : b.seq1) + roff;
        const uint8_t* Q = (mate ? b.qual2 : b.qual1) + roff;
        // quality chunk F of this lane's row: from the LDS row (full) or the row in L2 (LEAN)
        auto qchunk = [&](int F) -> uint4 {
            if (!LY::kQLds) return *reinterpret_cast<const uint4*>(Q + cst * F);
            return make_uint4(qrow[4 * F], qrow[4 * F + 1], qrow[4 * F + 2], qrow[4 * F + 3]);
        };
        // (merge: a merged read, at most len1 + len2 long, must fit max_cycles as well)
        const bool odd = L > kMaxLen || L > p.max_cycles || L > (nchunks << 4) ||
                         (MERGE && L + xor32(L) > p.max_cycles);
        uint32_t exo = 0, qhi = 0, q20 = 0, q30 = 0, lowf = 0, tqf = 0, nbf = 0;  // whole-read sums
        const uint32_t k80 = vk(0x80808080u), limq_v = vk(limq);  // (VGPR operands: full-rate VALU)
        // FULL with cut_right: bit k = chunk k holds a quality below its threshold (shifted in from
        // the top chunk by chunk, reversed after staging)
        uint32_t lowr = 0;
        // column word of chunk k: k for read 1, 9-k for read 2 (stepped, not precomputed, so the
        // ten addresses are not kept live across tiles)
        uint32_t* wp = col + lane_x + (rc ? (kChunks - 1) * 64 : 0);
        const int wstep = rc ? -64 : 64;
        // read 2: v_perm selector reversing a dword pair's bytes (0x04050607: src0 reversed), and the
        // complement mask of its codes
        const uint32_t rsel = rc ? 0x04050607u : 0x03020100u;
        const uint32_t rcx = rc ? 0xAAAAAAAAu : 0u;
        // Row chunks are requested kAhead ahead of their use (software pipelining: one HBM round
        // trip per tile instead of one per chunk); every row is readable up to its stride, so
        // the look-ahead loads are clamped, never guarded.  Only the chunks that some lane's read
        // does not fill (wave-uniform test) pay for byte masks.
        // opaque per tile: the per-chunk offsets and in-row flags derived from it would otherwise
        // be hoisted out of the tile loop and spilled
        int nch = nchunks;
#if FQ_OPAQUE_NCH
        if constexpr (!FIX) asm volatile("" : "+s"(nch));
#endif
        const int lastc = nch - 1;
        uint4 sb[kChunks], qb[kChunks];
#pragma unroll
        for (int k = 0; k < kAhead && k < kChunks; ++k) {
            sb[k] = *reinterpret_cast<const uint4*>(S + cst * min(k, lastc));
            qb[k] = *reinterpret_cast<const uint4*>(Q + cst * min(k, lastc));
        }
#pragma unroll
        for (int k = 0; k < kChunks; ++k) {
            const uint4 s4 = sb[k], q4 = qb[k];
            if (k + kAhead < kChunks) {
                sb[k + kAhead] = *reinterpret_cast<const uint4*>(S + cst * min(k + kAhead, lastc));
                qb[k + kAhead] = *reinterpret_cast<const uint4*>(Q + cst * min(k + kAhead, lastc));
            }
#if FQ_SCHED_PIN
            // keep the loads where they are: left alone, the scheduler hoists them all to the top
            // of the tile and then waits for every one of them before chunk 0
            __builtin_amdgcn_sched_barrier(0);
#endif
#if FQ_ABLATE_STAGE == 1  // profiling only: loads consumed, nothing computed (results invalid)
            if (k < nch) tqf ^= s4.x ^ s4.y ^ s4.z ^ s4.w ^ q4.x ^ q4.y ^ q4.z ^ q4.w;
            if (false) {
#else
            if (k < nch) {
#endif
                const uint32_t sw[4] = {s4.x, s4.y, s4.z, s4.w};
                const uint32_t qw[4] = {q4.x, q4.y, q4.z, q4.w};
                uint32_t cc = 0, nn4 = 0, lr = 0;
                uint32_t kkj[4];  // (FQ_STG2) the four dwords' 3-bit keys
                // bases of this chunk still in the read; opaque, or the masks of all ten chunks
                // (functions of L alone) are computed up front and kept live across the loop
                int Lk = L - 16 * k;
#if FQ_OPAQUE_LK
                asm volatile("" : "+v"(Lk));
#endif
                const bool full = __all(Lk >= 16);
                // per dword: codes, N flags, exotic-byte check and the quality sums; bytes >= 128
                // send the tile to the general kernel, so q + c (c < 128) never carries into the
                // next byte for the bytes that count.  FULL: every byte is inside the read (the
                // common case, no byte masks).
                uint32_t pbm[4], pbms[4];  // (FQ_FASTMASK: a partial chunk's byte masks, made once)
                // (not in the full non-merge variants: the eight live masks spill there)
                constexpr bool kChunkMask = FQ_FASTMASK && (LEAN || MERGE);
                auto dword = [&](int j, auto full_c) {
                    constexpr bool FULL = decltype(full_c)::value;
                    if (LY::kQLds) qrow[4 * k + j] = qw[j];
                    const uint32_t bm = FULL ? 0xFFFFFFFFu : kChunkMask ? pbm[j] : bytemask(Lk - 4 * j);
                    // read 2 (the column holds its reverse complement): the chunk's bytes reversed
                    // (dword 3 - j byte-swapped, one v_perm), so its codes come out in column order
                    const uint32_t sr = PAIRED ? __builtin_amdgcn_perm(sw[3 - j], sw[j], rsel) : sw[j];
                    const uint32_t bms = FULL ? 0xFFFFFFFFu : kChunkMask ? pbms[j] : rc ? ~bytemask(16 - Lk - 4 * j) : bm;
                    const uint32_t kk = (sr >> 1) & 0x07070707u;
                    // canonical byte for the 3-bit key: A C T G (0-3), N (7)
                    const uint32_t canon = __builtin_amdgcn_perm(0x4E000000u, 0x47544341u, kk);
                    // sum of |canon - byte| (one v_sad_u8): zero iff every byte is canonical, and
                    // at most 40 dwords x 4 x 255 per tile, so it never wraps
#if FQ_EXO3
                    // (or the OR of byte ^ canon: nonzero iff some byte is not canonical)
                    exo |= FULL ? (canon ^ sr) : ((canon ^ sr) & bms);
#else
                    exo = FULL ? __builtin_amdgcn_sad_u8(canon, sr, exo)
                               : __builtin_amdgcn_sad_u8(canon & bms, sr & bms, exo);
#endif
                    const uint32_t qm = FULL ? qw[j] : (qw[j] & bm);
                    qhi |= qm;
                    const uint32_t m80 = FULL ? k80 : (k80 & bm);
                    q20 += __popc((qm + 0x4A4A4A4Au) & m80);  // q > '5'
                    q30 += __popc(qm & 0x40404040u);  // q > '?' (= bit 6: q < 128 here; qm already masked)
                    lowf += __popc(~(qm + limq_v) & m80);        // q < limit
                    // whole-read quality total: only -e reads it (passFilter's mean quality),
                    // which runs on the XTRA instantiations (with -m the merge variant's)
                    if (!LEAN && XTRA) tqf = __builtin_amdgcn_sad_u8(qm, 0u, tqf);
                    if (!LEAN) lr |= ~(qm + limr) & (0x80808080u & bm);         // q < cut_right threshold
#if FQ_STG2
                    kkj[j] = kk;
#else
                    cc |= (kk & 0x03030303u) << (2 * j);
                    nn4 |= ((kk >> 2) & 0x01010101u) << (2 * j);
#endif
                };
                if (full) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) dword(j, std::true_type{});
                } else {
                    if constexpr (kChunkMask) {
                    // the first Lk bytes; read 2's staged bytes are the last Lk (its chunk reversed)
                    const int n4 = 4 * Lk;
                    chunk_bytemask(n4, pbm);
                    if (PAIRED) {
                        uint32_t rm[4];
                        chunk_bytemask(64 - n4, rm);
#pragma unroll
                        for (int j = 0; j < 4; ++j) pbms[j] = rc ? ~rm[j] : pbm[j];
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j) pbms[j] = pbm[j];
                    }
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) dword(j, std::false_type{});
                }
#if FQ_STG2
                {
                    // the keys of dwords 0 and 2 (1 and 3) share each byte in nibbles: code field j at
                    // bits 2j of the byte and N flag j at bit 2j come out of two masked merges
                    // (7 VALU for the chunk instead of ~18 in per-dword shifts)
                    const uint32_t p02 = kkj[0] | (kkj[2] << 4), p13 = kkj[1] | (kkj[3] << 4);
                    uint32_t c13;
                    asm("v_lshlrev_b32 %0, 2, %1" : "=v"(c13) : "v"(p13));
                    const uint32_t m33 = vk(0x33333333u);
                    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xAC" : "=v"(cc) : "v"(m33), "v"(c13), "v"(p02));  // m33 ? p02 : c13
                    nn4 = ((p02 >> 2) & 0x11111111u) | (p13 & 0x44444444u);
                }
#endif
                if (!LEAN) lowr = shift_in_sign(lowr, lr | (0u - lr));  // (sign set iff lr != 0)
                // N flags are kept only for positions inside the read (later passes rely on it);
                // read 2's chunk is reversed: its positions inside the read are the high ones
                const uint32_t vmask = full ? 0x55555555u : rc ? 0x55555555u & ~posmask_v(16 - Lk) : posmask_v(Lk);
                uint32_t fck = tr4x4(cc);
                const uint32_t fwk = tr4x4(nn4) & vmask;
                nbf += __popc(fwk);
                // read 2: the column is the reverse complement of the 160-position row, so the
                // read's rc position j sits at index j + (160 - L); garbage beyond L lands below.
                // Complement: code ^ 2 for A C G T, N stays code 3.
                fck ^= rcx & ~(fwk << 1);
#if FQ_ABLATE_STAGE == 2  // profiling only: no LDS column writes (results invalid)
                tqf ^= fck ^ fwk;
#else
                wp[kFC * 64] = fck;
                wp[kFN * 64] = fwk;
#endif
                wp += wstep;
                if constexpr (LY::kPfx)  // counts through chunk k (each <= 160): q20 | q30 << 8 | low << 16 | N << 24
                    if ((k + 1) % LY::kPfxStep == 0)
                        col[kCodeW + k / LY::kPfxStep * 64 + lane_x] =
                            __builtin_amdgcn_perm(__builtin_amdgcn_perm(nbf, lowf, 0x0c0c0400u),
                                                  __builtin_amdgcn_perm(q30, q20, 0x0c0c0400u), 0x05040100u);
            }
        }
        // Lowercase a c g t (the uppercase letter | 0x20: the same 3-bit key, so the same code) stay
        // on this kernel with a flag at the odd bit of the N word, for the steps that compare bytes:
        // read 1 against the reverse complement (which upper-cases them, src/seq.h:24-48), polyG,
        // polyX, adapter sequences, the complexity filter.  The Stats bucket byte & 7 is the
        // uppercase letter's (src/stats.cpp:249) and passFilter counts only 'N' (src/filter.cpp:18),
        // so those passes need nothing.  Any other byte outside ACGTN hands the pair over.  Rare: only
        // lanes holding such a byte re-read their row (from L2) here.
        if (!LEAN) lowr = nch > 0 ? __builtin_bitreverse32(lowr) >> (32 - nch) : 0u;  // chunk k to bit k
        bool hard = false, xl = false, xe = false;
        if (__any(exo != 0)) {
            if (exo != 0) {
                // exotic bytes stay here unless the passes that compare them as bytes need more
                // than "equals nothing": the low-complexity filter (two exotic bytes may be equal),
                // the merged read (read 2's exotic bytes become N inside it), -c, or an adapter
                // sequence holding such a byte
                bool ad_ok = true;
                for (int i = 0; i < my_alen; ++i) {
                    const uint32_t a = my_ad[i] & 0xDFu;
                    ad_ok = ad_ok && (a == 'A' || a == 'C' || a == 'G' || a == 'T' || my_ad[i] == 'N');
                }
                const bool allow = !MERGE && !p.complexity_enabled && ad_ok;
                // (LDS pointers from word offsets: no generic pointer to hold across the tile)
                auto lds_at = [&](const uint32_t* q) { return (LdsU32*)(size_t)(4u * (uint32_t)(q - lds)); };
                const int lf = lower_flags<PAIRED>(S, lds_at(col + lane_x + (rc ? (kChunks - 1) * 64 : 0)), wstep, nch, L, rc,
                                                   rsel, LY::kPfx ? lds_at(col + kCodeW + lane_x) : nullptr, LY::kPfxStep, allow);
                hard = (lf & 1) != 0;
                xe = (lf & 2) != 0;
                nbf -= (uint32_t)(lf >> 2);
                // (-c rewrites bases across the pair: its pairs with lowercase go over)
                if (XTRA && p.correction_enabled) hard = true;
                xl = !hard;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        const bool tile_x = __any(xl);  // some kept lane carries lowercase flags
        // (index filter: a pair the host dropped counts only in the pre-filter Stats,
        // src/peprocessor.cpp:283-286 -- rare, so it goes over too)
        const bool bad = odd || hard || (qhi & 0x80808080u) != 0 ||
                         (b.flags && valid && (b.flags[idx] & FQ_BF_INDEX_FILTERED));
        for (int k = nch; k < kChunks; ++k) {  // unused tail of the row
            wp[kFC * 64] = 0u;
            wp[kFN * 64] = 0u;
            wp += wstep;
        }
        // Pairs (single-end: reads) this kernel cannot take -- a read longer than the columns or
        // max_cycles, a byte outside ACGTN and acgt, a quality >= 128, an index-filtered pair -- are
        // handed to the general kernel one by one (item list: pair / read indices); the rest of
        // the tile stays here, the handed-over lanes continuing as empty lanes (valid false,
        // length 0).
        if (__any(bad)) {
            // bit i of hm: pair (single-end: read) i of the tile goes over
            const unsigned long long bm = __ballot(bad);
            const unsigned long long hm = PAIRED ? ((bm | (bm >> 32)) & 0xFFFFFFFFull) : bm;
            const int me = PAIRED ? pl : lane_x;
            const bool pbad = (hm >> me) & 1ull;
            // slots come from the wave's reservation of one tile's worth (kItems), so one
            // same-address atomic serves many tiles; an outgrown reservation's rest becomes holes
            // (kHole >= n: the general kernel skips them), as does the last one's at the end
            const int k = (int)__popcll(hm);
            int hb = hres[2 * wave], hl = hres[2 * wave + 1];
            if (k > hl) {
                if (lane_x < hl) slow_tiles[hb + lane_x] = kHole;
                int base = 0;
                if (lane == 0) base = atomicAdd(slow_count, kItems);
                hb = __shfl(base, 0);
                hl = kItems;
            }
            if (pbad && mate == 0) slow_tiles[hb + (int)__popcll(hm & ((1ull << me) - 1ull))] = idx;
            if (lane == 0) {
                hres[2 * wave] = hb + k;
                hres[2 * wave + 1] = hl - k;
            }
            if (pbad) {
                valid = false;
                L = 0;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#if FQ_STAGE_PRIO || FQ_PRIO_TRIM
        __builtin_amdgcn_s_setprio(FQ_PRIO_TRIM);  // (the phases after staging, up to polyG)
#endif
#if FQ_PREFETCH
        // The wave's next tile is one contiguous run of R * stride bytes per plane (R = 32 pairs or
        // 64 reads; planes span whole 32-read tiles, so the run is clamped to the rows that exist):
        // one dword per 128-byte line, loaded into a never-read LDS sink, so the next staging finds
        // its rows in L2 / the Infinity Cache while this tile computes.  The asm loads are outside
        // hipcc's waitcnt bookkeeping; any later counted vmcnt wait covers them (older loads retire
        // first), so nothing waits on them before the quality re-reads of the filter / stats.
        {
            const int tn = t + gridDim.x * kWaves;
            if (tn < ntiles) {
                constexpr int R = PAIRED ? 32 : 64;
                const int rows = min(R, ((b.n + 31) & ~31) - tn * R);
                // (PAIRED: the first FQ_PREFETCH chunks of the 32 rows, 512 B each)
                const int run = PAIRED ? min(rows * b.stride, FQ_PREFETCH * 512) : rows * b.stride;
                const uint32_t sink = (uint32_t)(LY::kLdsW - kPfW) * 4u;
                const uint8_t* planes[4] = {b.seq1, b.qual1, b.seq2, b.qual2};
#pragma unroll
                for (int pi = 0; pi < (PAIRED ? 4 : 2); ++pi) {
                    const uint8_t* base = planes[pi] + (size_t)tn * R * b.stride;
                    for (int off = lane_x * 128; off < run; off += 64 * 128) {
                        const uint8_t* g = base + off;
                        unsigned keep;
                        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                                     : "=&s"(keep) : "v"(g), "s"(sink));
                    }
                }
            }
        }
#endif
#if FQ_ABLATE_STAGE >= 3  // profiling only: staging, then straight to the result store
        if (valid && res)
            *reinterpret_cast<uint4*>(&res[PAIRED ? 2 * (size_t)idx + mate : (size_t)idx]) =
                make_uint4(tqf, q20 + q30 + lowf + nbf, exo, FQ_ABLATE_STAGE == 4 ? L : 0);
        continue;
#endif

        FQ_STAMP(0)
        const CodeSeq seq{col, lane, rc};
        const LdsQual qual{qrow};  // trimAndCut windows (full variant only)

        // ---------------- trimAndCut (src/peprocessor.cpp:292-293) ----------------
        int st = 0, n = 0;
        bool nn;
        if (LEAN) {  // Filter::trimAndCut with nothing to trim returns the read as is (src/filter.cpp:71-75)
            nn = valid;
            n = L;
        } else {
            if constexpr (LY::kQLds)
                nn = valid && trim_and_cut_t(p, seq, qual, L, front, tail, st, n, lowr_ok ? lowr : ~0u);
            else if (XTRA && umi) {
                // UmiProcessor::process cuts min(umi_front, len - 1) bases (a read of length 0 keeps
                // them), src/peprocessor.cpp:288-290 / src/seprocessor.cpp:309-311
                const int uf = mate ? p.umi_front2 : p.umi_front1;
                const int u = (uf > 0 && L > 0) ? min(uf, L - 1) : 0;
                // (cut_right's low-chunk hint in the cut read's chunks: chunk c spans row chunks
                // c + u/16 and c + (u+15)/16, so the union of their bits is a safe superset)
                const uint32_t lowu = lowr_ok ? ((lowr >> (u >> 4)) | (lowr >> ((u + 15) >> 4))) : ~0u;
                nn = valid && trim_and_cut_t(p, at(seq, u), at(RowQual{Q, b.stride >> 2}, u), L - u, front, tail, st, n, lowu);
                st += u;
            } else
                nn = valid && ((abl & 1024) ? (n = L, true)
                               : cut_w4 ? cut_right_w4(p, Q, nchunks, L, front, tail, lowr, limr, st, n)
                                        : trim_and_cut_t(p, seq, RowQual{Q, b.stride >> 2}, L, front, tail, st, n, lowr_ok ? lowr : ~0u));
        }
        // the shuffle must run in every lane: ds_bpermute from a lane that is switched off returns
        // whatever its register held before (e.g. the previous tile's value)
        const int nn_o = PAIRED ? xor32(nn ? 1 : 0) : 1;
        const bool both = nn && nn_o != 0;
        fq_read_result rr;
        rr.flags = nn ? 0 : FQ_RF_NULL;
        rr.code = 0;
        rr.ad_pos = rr.ad_len = rr.m_len1 = rr.m_len2 = rr.reserved = 0;

        FQ_STAMP(1)
        // ---------------- polyG (src/peprocessor.cpp:295-299) ----------------
#if FQ_PRIO_POLYG || FQ_PRIO_OV || FQ_PRIO_FILTER
        __builtin_amdgcn_s_setprio(FQ_PRIO_POLYG);  // (issue priority by phase: FQ_PRIO_TRIM)
#endif
        if (both && p.polyg_enabled && !(abl & 8)) {
            int bases;
            n = polyg_bits(col, lane, rc, st, n, p.polyg_max_mismatch, g_inv, g_per, p.polyg_compare_req, bases);
            if (bases >= 0 && !(abl & 32))  // (reads << 32 | bases) into the lane's scalar copy
                sadd(&scal[kScalStride * (lane_x & (LY::kScalCopies - 1)) + 4 * mate + 2], (1ull << 32) | (unsigned long long)bases);
        }

        FQ_STAMP(2)
        // AdapterTrimmer::trimBySequence, src/adaptertrimmer.cpp:29-90
        auto by_sequence = [&]() {
            int pos;
            const uint32_t* my_adw = adw + 8 * mate;
            if (my_adw[5] ? adseq_search(col, lane, rc, st, n, my_adw, adw + (kAdColOff - kAdWinOff) + kAdCW * mate,
                                         (uint32_t)(size_t)(const __attribute__((address_space(3))) uint32_t*)(adw + (kAdBitOff - kAdWinOff) + 32 * mate),
                                         my_alen, pos)
                          : trim_by_sequence_t(at(seq, st), n, my_ad, my_alen, pos)) {
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
                if (ad_len > 0) sadd(&scal[kScalStride * (lane_x & (LY::kScalCopies - 1)) + 4 * mate + 3], (1ull << 32) | (unsigned long long)ad_len);
            }
        };
        // OverlapAnalysis::analyze (src/overlapanalysis.cpp:7-72) of the pair's current windows;
        // both lanes of the pair call it together and get the same result
        auto pair_overlap = [&]() -> Overlap {
            const int st_o = xor32(st), n_o = xor32(n);
            const int st1 = mate ? st_o : st, n1 = mate ? n_o : n;
            const int st2 = mate ? st : st_o, n2 = mate ? n : n_o;
            const int c1 = mate ? mlane : lane, c2 = mate ? lane : mlane;
            const int off2 = kMaxLen - st2 - n2;  // column index where rc2 of the trimmed read starts
            // read 1 lanes: phase 1 (offset o >= 0: r1 window moves, rc2 fixed);
            // read 2 lanes: phase 2 (offset -m <= 0: rc2 window moves, r1 fixed)
            const int cm = mate ? c2 : c1, mpos = mate ? off2 : st1;
            const int olA = mate ? n2 : n1, olB = mate ? n1 : n2;
            const uint32_t fixed = field_window(col, kFC, mate ? c1 : c2, mate ? st1 : off2);
            const int cnt = max(0, olA - req);
            const uint32_t pm = posmask_v(olB);
            OvOut mine{false, 0, 0, 0};
            if (abl & 512) atomicAdd(&g_phase_cycles[1], 1ull);  // profiling: scanning lanes
            // bit-plane candidates when every lane compares full 16-position windows
            const bool planes = req >= 16 && !__any(olB < 16) && !(abl & 128);
            if (planes) {
                uint32_t cand[kOvBlocks];
                ov_candidates(col, cm, mpos, FixedOwn{unzip2(fixed)}, K, cnt, cand);
                for (;;) {  // candidates in offset order until one passes the exact test
                    int o = -1;
#pragma unroll
                    for (int bk = kOvBlocks - 1; bk >= 0; --bk)
                        if (cand[bk]) o = 32 * bk + __ffs(cand[bk]) - 1;
                    if (o < 0) break;
                    cand[o >> 5] &= cand[o >> 5] - 1u;
                    const int ol = min(olA - o, olB);
                    int diff = 0;
                    if (abl & 512) atomicAdd(&g_phase_cycles[0], 1ull);  // profiling: exact checks
                    if ((abl & 64) || ov_exact<kOvx2>(col, c1, mate ? st1 : st1 + o, c2, mate ? off2 + o : off2, ol, limit, K, diff)) {
                        mine = OvOut{true, mate ? -o : o, ol, diff};
                        break;
                    }
                }
            }
            for (int k0 = 0; !planes && !(abl & 128);) {
                const int o = req >= 16 ? ov_scan<true>(col, cm, mpos, k0, cnt, fixed, olA, olB, K, pm)
                                        : ov_scan<false>(col, cm, mpos, k0, cnt, fixed, olA, olB, K, pm);
                if (o < 0) break;
                const int ol = min(olA - o, olB);
                int diff = 0;
                if (abl & 512) atomicAdd(&g_phase_cycles[0], 1ull);  // profiling: exact checks
                if ((abl & 64) || ov_exact<kOvx2>(col, c1, mate ? st1 : st1 + o, c2, mate ? off2 + o : off2, ol, limit, K, diff)) {
                    mine = OvOut{true, mate ? -o : o, ol, diff};
                    break;
                }
                k0 = o + 1;
            }
            const int f_o = xor32(mine.found ? 1 : 0);
            const int off_o = xor32(mine.off), ol_o = xor32(mine.ol), d_o = xor32(mine.diff);
            const bool f1 = mate ? f_o != 0 : mine.found;
            const bool f2 = mate ? mine.found : f_o != 0;
            Overlap ov{0, 0, 0, 0};
            if (f1) ov = mate ? Overlap{1, off_o, ol_o, d_o} : Overlap{1, mine.off, mine.ol, mine.diff};
            else if (f2) ov = mate ? Overlap{1, mine.off, mine.ol, mine.diff} : Overlap{1, off_o, ol_o, d_o};
            return ov;
        };
        // ---------------- overlap + adapters (src/peprocessor.cpp:302-333) ----------------
#if FQ_PRIO_POLYG || FQ_PRIO_OV || FQ_PRIO_FILTER
        __builtin_amdgcn_s_setprio(FQ_PRIO_OV);
#endif
        Overlap ov1{0, 0, 0, 0};  // (merge) the first analysis and the windows it saw
        int n1a = -1, n2a = -1;
        bool ad_ov = false, corr = false;  // (corr: -c changed a base of the pair)
        if (PAIRED && both && !(abl & 1)) {
            const Overlap ov = pair_overlap();
            const int n_o = xor32(n);
            const int n1 = mate ? n_o : n, n2 = mate ? n : n_o;
            if (MERGE) {
                ov1 = ov;
                n1a = n1;
                n2a = n2;
            }
            if (mate == 0) {  // PairEndProcessor::statInsertSize, src/peprocessor.cpp:510-523
                int isize = p.insert_size_max;
                if (ov.overlapped) isize = ov.offset > 0 ? n1 + n2 - ov.len : ov.len;
                if (isize > p.insert_size_max) isize = p.insert_size_max;
                atomicAdd(&ins[isize], 1u);
            }
            if constexpr (XTRA) {
                // BaseCorrector::correctByOverlapAnalysis (src/basecorrector.cpp:14-70), pair-uniform
                if (p.correction_enabled && ov.diff > 0 && ov.diff <= 5) {
                    const int st_o = xor32(st);
                    corr = correct_pair_fast(p, col, lds, b, roff, mate, lane_x, mlane, mate ? st_o : st, mate ? st : st_o, n2,
                                      ov, Q, rr, q20, q30, lowf, tqf, nbf, limq,
                                      scal + kScalStride * (lane_x & (LY::kScalCopies - 1)) + 4 * mate + 1,
                                      removed_mode ? LY::kColsW + mate * 32 : LY::kColsW + mate * kHistW,
                                      removed_mode, acc);
                }
            }
            if (p.adapter_trimming) {
                const int ol = ov.len;  // AdapterTrimmer::trimByOverlapAnalysis, src/adaptertrimmer.cpp:14-27
                if (ov.diff <= 5 && ov.overlapped && ov.offset < 0 && ol > n1 / 3) {
                    ad_ov = true;
                    rr.flags |= FQ_RF_AD_OVERLAP;
                    rr.ad_pos = (uint16_t)(st + ol);
                    rr.ad_len = (uint16_t)(n - ol);
                    if (mate == 0)
                        sadd(&scal[kScalStride * (lane_x & (LY::kScalCopies - 1)) + 3], (2ull << 32) | (unsigned long long)((n1 - ol) + (n2 - ol)));
                    n = ol;
                } else if (!LEAN && my_alen > 0) {
                    by_sequence();
                }
            }
        }
        if (!PAIRED && !LEAN && nn && p.adapter_trimming && my_alen > 0) by_sequence();  // src/seprocessor.cpp:320-323

        FQ_STAMP(3)
        // ---------------- polyX, maxLen (src/peprocessor.cpp:335-349) ----------------
        if (!LEAN && both && p.polyx_enabled && !(abl & 2048) &&
            !polyx_no_trim(col, lane, rc, st, n, p.polyx_mask, p.polyx_max_mismatch, p.polyx_one_mismatch_per,
                           p.polyx_compare_req)) {
            int poly, bases;
            n = trim_polyx_t(at(seq, st), n, p.polyx_mask, p.polyx_compare_req, p.polyx_max_mismatch,
                             p.polyx_one_mismatch_per, poly, bases);
            if (poly >= 0) {
                sadd(&small[FQ_ACC_POLYX_READS + poly], 1ull);
                sadd(&small[FQ_ACC_POLYX_BASES + poly], (unsigned long long)(long long)bases);
            }
        }
        if (!LEAN && both && my_maxlen > 0 && my_maxlen < n) n = my_maxlen;

        // ---------------- merge (src/peprocessor.cpp:351-385, OverlapAnalysis::merge
        // src/overlapanalysis.cpp:74-104): the merged read is r1[0, m1) + revcomp(r2)[ol, ol+m2) ----
        bool merged = false;
        int m1 = 0, m2 = 0, mol = 0;
        if (MERGE && both) {
            // OverlapAnalysis::analyze of the current windows (src/peprocessor.cpp:354).  Known
            // without a scan (pair-uniform test): when neither window changed since the first
            // analysis, the same result; when only trimByOverlapAnalysis cut both reads to the
            // phase-2 overlap ol = len2 - k (offset -k), the trimmed pair compares exactly the same
            // bases at offset 0, the first offset phase 1 tries, so {1, 0, ol, diff}.
            const int n_o = xor32(n);
            const int n1c = mate ? n_o : n, n2c = mate ? n : n_o;
            // (-c: a corrected pair compares other bases than the first analysis did, so the same
            // windows are analysed again; the derived case still holds: its offset 0 compares the
            // overlap the first analysis accepted, with mismatches only removed by the correction)
            const bool same = !corr && n1a >= 0 && n1c == n1a && n2c == n2a;
            const bool derived = n1a >= 0 && ad_ov && n1c == ov1.len && n2c == ov1.len && ov1.len == n2a + ov1.offset;
            Overlap ov2 = same ? ov1 : Overlap{1, 0, ov1.len, ov1.diff};
            if (!same && !derived) ov2 = pair_overlap();  // pair-uniform branch (the mate lanes swap values)
            if (ov2.overlapped) {
                merged = true;
                mol = ov2.len;
                const int n_o = xor32(n);
                const int n1 = mate ? n_o : n, n2 = mate ? n : n_o;
                if (mol) {
                    m1 = min(mol + max(0, ov2.offset), n1);
                    m2 = ov2.offset > 0 ? max(0, n2 - mol) : 0;
                }
            }
        }
        // the window that the filter and the post stats see: the read's own [st, st+n), or its
        // part of the merged read (read 2: forward positions [st+n-ol-m2, st+n-ol), reversed)
        const int ws = (MERGE && merged && mate) ? st + n - mol - m2 : st;
        const int wn = (MERGE && merged) ? (mate ? m2 : m1) : n;

        FQ_STAMP(4)
        // ---------------- passFilter (src/filter.cpp:3-52) ----------------
#if FQ_PRIO_POLYG || FQ_PRIO_OV || FQ_PRIO_FILTER
        __builtin_amdgcn_s_setprio(FQ_PRIO_FILTER);
#endif
        int code = FQ_FAIL_LENGTH;
        uint32_t w20 = 0, w30 = 0;  // Q20/Q30 of the window, for the post stats
        int low = 0, tq = 0, nb = 0;
        // Prefix counts (LY::kPfx) unless -c rewrote qualities after staging or -e needs the total
        const bool use_pfx = LY::kPfx && !(XTRA && p.correction_enabled) && !(p.avg_qual_limit > 0) && !(abl & 2);
        if (use_pfx && nn && wn > 0) {
            // packed counts (q20 | q30 << 8 | low << 16 | N << 24) of chunk F's first nb bytes (1..16)
            auto chunk_counts = [&](int F, int nbytes) -> uint32_t {
                const uint4 q4 = qchunk(F);
                const uint32_t qw[4] = {q4.x, q4.y, q4.z, q4.w};
                uint32_t c20 = 0, c30 = 0, cl = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t bm = bytemask(nbytes - 4 * j), qm = qw[j] & bm, m80 = k80 & bm;
                    c20 += __popc((qm + 0x4A4A4A4Au) & m80);
                    c30 += __popc(qm & 0x40404040u);
                    cl += __popc(~(qm + limq_v) & m80);
                }
                // N bits of the chunk's first nbytes positions (read 2's column is reversed)
                // (an exotic byte's N bit comes with its flag: not an 'N')
                const uint32_t nw = col[(kFN + (rc ? kChunks - 1 - F : F)) * 64 + lane_x];
                const uint32_t cn = __popc(nw & ~(nw >> 1) & (rc ? 0x55555555u & ~posmask(16 - nbytes) : posmask(nbytes)));
                return c20 | c30 << 8 | cl << 16 | cn << 24;
            };
            // counts of forward positions [0, x): the prefix word through chunk (c / step) * step - 1,
            // then the chunks up to c - 1 and chunk c's bytes below x (wave-uniform branches)
            auto p_at = [&](int x) -> uint32_t {
                const int c = x >> 4, rb = x & 15, j = c / LY::kPfxStep;
                uint32_t v = col[kCodeW + max(j - 1, 0) * 64 + lane_x] & (j > 0 ? ~0u : 0u);
                if (LY::kPfxStep == 2 && __any(c & 1) && (c & 1)) v += chunk_counts(c - 1, 16);
                if (__any(rb != 0) && rb != 0) v += chunk_counts(c, rb);
                return v;
            };
            // window [ws, ws + wn) (ws = 0 unless front trimming, UMI or read 2's part of a merged read)
            uint32_t v = p_at(ws + wn);
            if (__any(ws > 0) && ws > 0) v -= p_at(ws);
            w20 = v & 0xFFu;
            w30 = (v >> 8) & 0xFFu;
            low = (int)((v >> 16) & 0xFFu);
            nb = (int)(v >> 24);
            if (!(MERGE && merged))
                code = filter_verdict(p, n, low, nb, -33 * n, [&]() {
                    if (LEAN) return 0;  // not reached: LEAN excludes the complexity filter
                    int diff = 0;
                    for (int i = 0; i < n - 1; ++i) diff += seq(st + i) != seq(st + i + 1);
                    return diff;
                });
        } else if (nn && wn > 0) {
            // window sums = whole-read sums (from staging) minus the trimmed head [0, ws) and
            // tail [ws+wn, L): the trimmed parts are usually a few bases.  (FULL: a window
            // shorter than half the read, e.g. read 2's part of a merged read, is summed directly:
            // "subtracted" from 0 and negated.)
            const bool direct = (!LEAN || FQ_LEAN_DIRECT) && 2 * wn < L;
            low = direct ? 0 : (int)lowf;
            tq = direct ? 0 : (int)tqf;
            nb = direct ? 0 : (int)nbf;
            w20 = direct ? 0u : q20;
            w30 = direct ? 0u : q30;
            if (!(abl & 2)) {
                const int end = ws + wn;
                const bool need_tq = p.avg_qual_limit > 0;  // the total quality only feeds -e
#pragma unroll
                for (int part = 0; part < 2; ++part) {
                    // forward range [a0, a1)
                    const int a0 = direct ? (part ? L : ws) : (part ? end : 0);
                    const int a1 = direct ? (part ? L : end) : (part ? L : ws);
                    const int F0 = a0 >> 4, F1 = (a1 + 15) >> 4;
                    // subtract the bytes of row chunk F inside [a0, a1)
                    auto sub = [&](const uint4 cur, int F) {
                        const uint32_t wq[4] = {cur.x, cur.y, cur.z, cur.w};
                        // in-range flags at bit 7 of each byte, SWAR: byte k of dword j holds
                        // 128 + (4j + k) - lo (resp. - hi), >= 128 iff the position is >= lo (>= hi)
                        const uint32_t lo = (uint32_t)min(max(a0 - 16 * F, 0), 16), hi = (uint32_t)min(max(a1 - 16 * F, 0), 16);
                        const uint32_t b1 = 0x83828180u - lo * 0x01010101u, b2 = 0x83828180u - hi * 0x01010101u;
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const uint32_t rf = (b1 + 0x04040404u * j) & ~(b2 + 0x04040404u * j) & 0x80808080u;
                            // (no carry reaches an in-range byte: the bytes below a1 <= L are qualities < 128,
                            // the only bytes >= 128 are row padding past L, whose carries run upward)
                            const uint32_t w7 = wq[j];
                            low -= __popc(~(w7 + limq) & rf);
                            w20 -= __popc((w7 + 0x4A4A4A4Au) & rf);
                            w30 -= __popc((w7 + 0x40404040u) & rf);
                            if (need_tq) tq -= (int)__builtin_amdgcn_sad_u8(wq[j] & ((rf >> 7) * 0xFFu), 0u, 0u);
                        }
                    };
#if FQ_FILTER_BATCH
                    if ((!LEAN || FQ_LEAN_DIRECT) && a0 < a1) {
                        // (FULL) the range's row chunks from L2, four requested together per round
                        // trip (LEAN, whose ranges are the trimmed tails only, is faster as below)
                        for (int Fb = F0; Fb < F1; Fb += 4) {
                            uint4 qa[4];
#pragma unroll
                            for (int i = 0; i < 4; ++i) qa[i] = qchunk(min(Fb + i, nchunks - 1));
#pragma unroll
                            for (int i = 0; i < 4; ++i)
                                if (Fb + i < F1) sub(qa[i], Fb + i);
                        }
                    } else if (LEAN && part == 1 && a0 < a1) {
                        uint4 qa[2];
#pragma unroll
                        for (int i = 0; i < 2; ++i) qa[i] = qchunk(max(F1 - 1 - i, 0));
#pragma unroll
                        for (int i = 0; i < 2; ++i)
                            if (F1 - 1 - i >= F0) sub(qa[i], F1 - 1 - i);
                        for (int F = F1 - 3; F >= F0; --F) sub(qchunk(F), F);
                    }
#else
                    if (part == 1 && a0 < a1) {
                        // the tail, from the 3' end: its last two chunks are requested together
                        // (one L2 round trip for most reads), longer adapter tails loop
                        uint4 qa[2];
#pragma unroll
                        for (int i = 0; i < 2; ++i) qa[i] = qchunk(max(F1 - 1 - i, 0));
#pragma unroll
                        for (int i = 0; i < 2; ++i)
                            if (F1 - 1 - i >= F0) sub(qa[i], F1 - 1 - i);
                        for (int F = F1 - 3; F >= F0; --F) sub(qchunk(F), F);
                    } else if (!LEAN) {
                        // row chunks come from L2; the next one is requested before this one is used
                        uint4 cur = qchunk(min(F0, nchunks - 1));
                        for (int F = F0; F < F1; ++F) {
                            const uint4 nxt = qchunk(min(F + 1, nchunks - 1));
                            sub(cur, F);
                            cur = nxt;
                        }
                    }
#endif
                    // N bits of the same range (read 2's column is reverse-complemented)
                    const int s0 = rc ? kMaxLen - a1 : a0, s1 = rc ? kMaxLen - a0 : a1;
                    for (int c = s0 >> 4; c < ((s1 + 15) >> 4); ++c) {
                        const uint32_t w = col[(kFN + c) * 64 + lane_x];
                        nb -= __popc(w & ~(w >> 1) & posmask(s1 - 16 * c) & ~posmask(s0 - 16 * c));
                    }
                }
                if (direct) {
                    low = -low;
                    tq = -tq;
                    nb = -nb;
                    w20 = 0u - w20;
                    w30 = 0u - w30;
                }
            }
            if (!(MERGE && merged))
                code = filter_verdict(p, n, low, nb, tq - 33 * n, [&]() {
                    if (LEAN) return 0;  // not reached: LEAN excludes the complexity filter
                    int diff = 0;
                    for (int i = 0; i < n - 1; ++i) diff += seq(st + i) != seq(st + i + 1);
                    return diff;
                });
        }
        int mlen = 0;
        if (MERGE && merged) {  // passFilter of the merged read: the sums of its two parts
            mlen = m1 + m2;
            low += xor32(low);
            nb += xor32(nb);
            tq += xor32(tq);
            w20 += xor32(w20);
            w30 += xor32(w30);
            // Filter::passLowComplexityFliter of the merged read (src/filter.cpp:54-67): adjacent
            // differences within read 1's part (bytes as they are), within read 2's part (its
            // bytes complemented, util::complement: upper-cased, so compared upper-cased), and
            // across the junction (read 1's last byte against the complement of read 2's byte at
            // the part's high end, which comes first in the merged read)
            int cdiff = 0;
            if (p.complexity_enabled) {
                int d = 0;
                for (int i = 0; i + 1 < wn; ++i) {
                    const int x = seq(ws + i), y = seq(ws + i + 1);
                    d += mate ? (x & 0xDF) != (y & 0xDF) : x != y;
                }
                int edge = 0;
                if (wn > 0) {
                    const int x = seq(ws + wn - 1);
                    if (!mate) edge = x;
                    else switch (x & 0xDF) {
                        case 'A': edge = 'T'; break;
                        case 'C': edge = 'G'; break;
                        case 'G': edge = 'C'; break;
                        case 'T': edge = 'A'; break;
                        default: edge = 'N';
                    }
                }
                const int d_o = xor32(d), e_o = xor32(edge);
                cdiff = d + d_o + ((m1 > 0 && m2 > 0 && edge != e_o) ? 1 : 0);
            }
            // (OverlapAnalysis::merge returns NULL for ol 0)
            code = (mol == 0 || mlen == 0) ? FQ_FAIL_LENGTH
                                           : filter_verdict(p, mlen, low, nb, tq - 33 * mlen, [&]() { return cdiff; });
        }
        const int code_o = PAIRED ? xor32(code) : code;
        const bool pair_pass = both && code == FQ_PASS_FILTER && code_o == FQ_PASS_FILTER;
        bool post_on;  // this lane's window goes to a post block
        if (MERGE && merged) {
            if (mate == 0) {
                sadd(&small[FQ_ACC_FILTER + code], 2ull);  // addFilterResult(result, 2)
                if (code == FQ_PASS_FILTER) sadd(&small[FQ_ACC_MERGED_PAIRS], 1ull);
                rr.flags |= FQ_RF_OVERLAP | FQ_RF_MERGED;
                rr.m_len1 = (uint16_t)m1;
                rr.m_len2 = (uint16_t)m2;
            }
            post_on = code == FQ_PASS_FILTER;
        } else if (MERGE && both && !p.discard_unmerged) {  // unmerged reads are filtered one by one
            sadd(&small[FQ_ACC_FILTER + code], 1ull);
            post_on = code == FQ_PASS_FILTER;
        } else if (PAIRED) {
            // addFilterResult(max(r1, r2), 2)
            if (MERGE) {
                if (mate == 0 && valid) sadd(&small[FQ_ACC_FILTER + max(code, code_o)], 2ull);
            } else {
                count_by_value(small + FQ_ACC_FILTER, mate == 0 && valid, max(code, code_o), 2ull);
            }
            post_on = !MERGE && pair_pass;
        } else {
            count_by_value(small + FQ_ACC_FILTER, valid, code, 1ull);  // src/seprocessor.cpp:339
            post_on = pair_pass;
        }

        FQ_STAMP(5)
        if (tile_x) {  // (rare) the lowercase flags have served: the Stats passes read spaced N masks
            if (!MERGE && xe && valid && !(abl & 4)) {
                // exotic bytes: the passes below count them as N (class 6, code 3 + N bit); move each
                // to its class byte & 7 (src/stats.cpp:249) in the pre block and, inside the post
                // window, the post block (rare).  The moves go to one of kXfixCopies copies of the
                // four Stats blocks in global memory (by workgroup, so a column of IUPAC codes does
                // not funnel every workgroup's atomics into one address), summed into the
                // accumulator after the launch (fq_launch_xfix_fold).  The row's address is
                // re-derived here (S itself is not kept live this far).
                const size_t sw = acc_stats_words(p.max_cycles);
                unsigned long long* xf = xfix + (size_t)(blockIdx.x & (kXfixCopies - 1)) * 4 * sw;
                xfix[kXfixCopies * 4 * sw] = 1ull;  // (the fold's flag)
                constexpr int cst = FQ_TILE_READS * FQ_CHUNK;
                int ix = idx;
                asm volatile("" : "+v"(ix));
                const uint8_t* Sx = (mate ? b.seq2 : b.seq1) + (size_t)(ix / FQ_TILE_READS) * FQ_TILE_READS * b.stride +
                                    (ix % FQ_TILE_READS) * FQ_CHUNK;
                for (int c = 0; c < kChunks; ++c) {
                    const uint32_t w = col[(kFN + c) * 64 + lane_x];
                    uint32_t ex = w & (w >> 1) & 0x55555555u;
                    while (ex) {
                        const int t = (__ffs(ex) - 1) >> 1;
                        ex &= ex - 1u;
                        const int q = 16 * c + t, P = rc ? kMaxLen - 1 - q : q;
                        const int off = cst * (P >> 4) + (P & 15);
                        const int cls = Sx[off] & 7;
                        if (cls == 6) continue;
                        const unsigned long long qv = (unsigned long long)(Q[off] - 33);
                        auto move = [&](int k, int cyc) {
                            unsigned long long* dst = xf + (size_t)k * sw + FQ_ST_CYCLES + (size_t)cyc * FQ_ST_PER_CYCLE;
                            atomicAdd(&dst[6], ~0ull);
                            atomicAdd(&dst[8 + 6], 0ull - qv);
                            atomicAdd(&dst[cls], 1ull);
                            atomicAdd(&dst[8 + cls], qv);
                        };
                        move(mate, P);
                        if (post_on && P >= ws && P < ws + wn) move(2 + mate, P - ws);
                    }
                }
            }
            if (xl)
                for (int c = 0; c < kChunks; ++c) col[(kFN + c) * 64 + lane_x] &= 0x55555555u;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        // ---------------- Stats::statRead, pre and post (src/peprocessor.cpp:276-277,400-401) ----
        if (valid && !(abl & 4)) {
            // per-read Stats scalars: (reads, length_sum) packed as count << 32 | sum, plus
            // q20 << 32 | q30, into one of 16 LDS copies (lanes l, l + 16 share one); first, so
            // that none of these values stays live through the passes below
            unsigned long long* sc = scal + kScalStride * (lane_x & (LY::kScalCopies - 1)) + 4 * mate;
            sadd(&sc[0], (1ull << 32) | (unsigned long long)L);
            sadd(&sc[1], ((unsigned long long)q20 << 32) | q30);
            const bool post_here = (MERGE && merged) ? (post_on && mate == 0) : post_on;
            if (post_here) {
                sadd(&sc[8], (1ull << 32) | (unsigned long long)((MERGE && merged) ? mlen : n));
                sadd(&sc[9], ((unsigned long long)w20 << 32) | w30);
            }
        }
#if FQ_STATS_PRIO
        __builtin_amdgcn_s_setprio(FQ_STATS_PRIO);  // (the Stats pass: highest, FQ_PRIO_TRIM)
#endif
        if (valid && !(abl & 4) && removed_mode) {
            // Every kept window is a prefix [0, wlen): each base goes to exactly one cell, kept or
            // removed (pre = kept + removed at the flush), one LDS atomic per base.  Per chunk the
            // 16 slot numbers are built as nibbles (SWAR), rotated by r positions like the
            // qualities, so a base costs a nibble extract, an address and a byte extract.
            // (merge: read 2's part of a merged read is not a prefix of read 2; it goes to read 1's
            // post block at other cycles, below, and read 2's own bases only to its pre block)
            const int wlen = post_on && !(MERGE && merged && mate) ? wn : 0;
            const int dsel = r >> 2, rr4 = 4 * (r & 7);
            [[maybe_unused]] const bool rswap = r >= 8;
#if FQ_ST_VCC
            // the lanes whose rotation takes the next dword / the other half (dsel & 2 == rswap)
            const unsigned long long msel1 = __builtin_amdgcn_ballot_w64((dsel & 1) != 0);
            const unsigned long long msel2 = __builtin_amdgcn_ballot_w64((dsel & 2) != 0);
#endif
            // LDS byte address of rotated position t's cell in slot 0 of chunk 0 (this mate's rows):
            // bits 8-11 are clear, the slot nibble is or-ed in (rcell)
            static_assert((LY::kColsW * 4) % 4096 == 0, "removed-mode rows: 4 KiB aligned");
            uint32_t rwb[16];
            const uint32_t blk0 = (uint32_t)(LY::kColsW + mate * 32) * 4u;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                rwb[t] = blk0 + 8u * (uint32_t)((t + r) & 15);
                asm volatile("" : "+v"(rwb[t]));  // kept whole (not re-split into base + offset per use)
            }
            const uint32_t slot_m = vk(0xF00u);
            // quality chunks rotate through kSA + 1 registers (requested kSA chunks ahead)
            constexpr int kSA = FQ_STATS_AHEAD;
            uint4 qb[kSA + 1];
#pragma unroll
            for (int i = 0; i < kSA; ++i) qb[i] = qchunk(min(i, nchunks - 1));
            // this lane's column word of forward chunk F: cw0 + F * cstep (read 2's column is reversed)
            const uint32_t* cwp = col + lane_x + (rc ? (kChunks - 1) * 64 : 0);
            const int cstep = rc ? -64 : 64;
            [[maybe_unused]] auto fwd_at = [&](const uint32_t* wp_) {
                uint32_t cw = wp_[kFC * 64], nw = wp_[kFN * 64];
                if (rc) {
                    cw = pairrev(cw);
                    nw = pairrev(nw);
                    cw ^= 0xAAAAAAAAu & ~(nw << 1);  // complement back, N stays code 3
                }
                return Fwd{cw, nw};
            };
            // PF2: raw column words of chunks F and F + 1 (requested two chunks ahead: the wait for
            // chunk F's words then does not cover the atomics issued since).  Two more live VGPRs:
            // the FULL non-merge variants would spill, so they read one chunk ahead.
            constexpr bool kPf2 = FQ_ST_PF2 && (LEAN || (MERGE && !XTRA));
            uint32_t rw0c = 0, rw0n = 0, rw1c = 0, rw1n = 0;
            Fwd fn{0u, 0u};
            if constexpr (kPf2) {
                rw0c = cwp[kFC * 64], rw0n = cwp[kFN * 64];
                rw1c = cwp[cstep + kFC * 64], rw1n = cwp[cstep + kFN * 64];
                cwp += cstep;
            } else {
                fn = fwd_at(cwp);
            }
#if FQ_ST_KM2
            const uint32_t m0f = vk(0x0F0F0F0Fu), m33 = vk(0x33333333u), m44 = vk(0x44444444u);
#endif
            // nibble prefix masks from one 64-bit shift: ~(~0 << 4 * clamp(len, 0, 16)), the
            // 64th bit never needed (nibble 15's top bit is 0 in 0x4444... and 0xAAAA... masks)
            const int w4 = 4 * wlen, l4 = 4 * L;
#pragma unroll
            for (int F = 0; F < kChunks; ++F) {
                if (F < nch) {  // wave-uniform; positions >= L are dummies
                    Fwd f = fn;
                    if constexpr (kPf2) {
                        uint32_t fc = rw0c, fnw = rw0n;
                        if (rc) {
                            fc = pairrev(fc);
                            fnw = pairrev(fnw);
                            fc ^= 0xAAAAAAAAu & ~(fnw << 1);  // complement back, N stays code 3
                        }
                        f = Fwd{fc, fnw};
                        rw0c = rw1c;
                        rw0n = rw1n;
                        if (F + 2 < kChunks) {
                            cwp += cstep;
                            rw1c = cwp[kFC * 64];
                            rw1n = cwp[kFN * 64];
                        }
                    }
                    const uint32_t q0 = qb[F % (kSA + 1)].x, q1 = qb[F % (kSA + 1)].y, q2 = qb[F % (kSA + 1)].z,
                                   q3 = qb[F % (kSA + 1)].w;
                    if (F + kSA < kChunks) qb[(F + kSA) % (kSA + 1)] = qchunk(min(F + kSA, nchunks - 1));
                    // (chunks from nch on are zero-filled by staging: no clamp)
                    if (!kPf2 && F + 1 < kChunks) {
                        cwp += cstep;
                        fn = fwd_at(cwp);
                    }
                    const int vl = L - 16 * F;
                    // slot 4 * kept + code; an N (code 3) reads as a G here
#if FQ_ST_KM2
                    // kept nibbles: ~(~0 << s), s = clamp(4 wlen - 64 F, 0, 63) (one v_med3); the
                    // codes spread to nibbles for both halves at once by 64-bit shifts, masked by
                    // one v_bitop3 per word, the kept bit or-ed in by another
                    int sk;
                    asm("v_med3_i32 %0, %1, 0, 63" : "=v"(sk) : "v"(w4 - 64 * F));
                    const unsigned long long km = ~0ull << sk;
                    uint32_t lo, hi;
                    {
                        const uint32_t x0 = __builtin_amdgcn_perm(f.c, f.c, 0x0c010c00u);  // code bytes 0, 1 to bytes 0, 2
                        const uint32_t x1 = __builtin_amdgcn_perm(f.c, f.c, 0x0c030c02u);  // code bytes 2, 3
                        unsigned long long X = (unsigned long long)x1 << 32 | x0, X4, X2;
                        asm("v_lshlrev_b64 %0, 4, %1" : "=v"(X4) : "v"(X));
                        const uint32_t y0 = (x0 | (uint32_t)X4) & m0f, y1 = (x1 | (uint32_t)(X4 >> 32)) & m0f;
                        X = (unsigned long long)y1 << 32 | y0;
                        asm("v_lshlrev_b64 %0, 2, %1" : "=v"(X2) : "v"(X));
                        const uint32_t z0 = (y0 | (uint32_t)X2) & m33, z1 = (y1 | (uint32_t)(X2 >> 32)) & m33;
                        lo = (~(uint32_t)km & m44) | z0;
                        hi = (~(uint32_t)(km >> 32) & m44) | z1;
                    }
#else
                    const unsigned long long km = ~(~0ull << min(max(w4 - 64 * F, 0), 63));
                    uint32_t lo = spread2to4(f.c) + ((uint32_t)km & 0x44444444u);
                    uint32_t hi = spread2to4(f.c >> 16) + ((uint32_t)(km >> 32) & 0x44444444u);
#endif
#if FQ_NFOLD
                    // N bases: their slot kRNSlot + 4 * kept is the G slot + 5, one nibble add (staging
                    // kept N flags only inside the read)
                    if (__any(f.n != 0)) {
                        // (n0 nibbles are 0 or 1: n0 | n0 << 2 is 5 n0, one v_lshl_or)
                        const uint32_t n0 = spread2to4(f.n), n1 = spread2to4(f.n >> 16);
                        uint32_t n05, n15;
                        asm("v_lshl_or_b32 %0, %1, 2, %1" : "=v"(n05) : "v"(n0));
                        asm("v_lshl_or_b32 %0, %1, 2, %1" : "=v"(n15) : "v"(n1));
                        lo += n05;
                        hi += n15;
                    }
#endif
                    if (__any(vl < 16)) {  // positions beyond the read (kept is 0 there) -> dummy slot 10
                        const unsigned long long vm = ~0ull << min(max(l4 - 64 * F, 0), 63);
                        const uint32_t dlo = (uint32_t)vm, dhi = vl >= 16 ? 0u : (uint32_t)(vm >> 32);
                        lo = (lo & ~dlo) | (dlo & 0xAAAAAAAAu);
                        hi = (hi & ~dhi) | (dhi & 0xAAAAAAAAu);
                    }
#if !FQ_NFOLD
                    // N bases (profiling baseline): move each from its G cell (slot 4 * kept + 3) to
                    // slot kRNSlot + 4 * kept
                    uint32_t nv = f.n;
                    if (__any(nv != 0)) {
                        const uint32_t qs[4] = {q0, q1, q2, q3};
                        while (nv) {
                            const int t = (__ffs(nv) - 1) >> 1;
                            nv &= nv - 1;
                            const int kept = 16 * F + t < wlen ? 1 : 0;
                            const unsigned long long v = kCount1 | (unsigned long long)__builtin_amdgcn_ubfe(qs[t >> 2], 8 * (t & 3), 8);
                            const uint32_t a = (uint32_t)(LY::kColsW + mate * 32) * 4u +
                                               (uint32_t)(F * kRSlots * 64 * 4) + 8u * (uint32_t)t;
                            __hip_atomic_fetch_add(reinterpret_cast<LdsU64*>((size_t)(a + (uint32_t)(kRNSlot + 4 * kept) * 256u)), v,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            __hip_atomic_fetch_add(reinterpret_cast<LdsU64*>((size_t)(a + (uint32_t)(4 * kept + 3) * 256u)), 0ull - v,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                    }
#endif
                    // rotate by r positions: rotated position t is 16F + (t + r) % 16
#if FQ_ST_VCC
                    // (the ten selects against two per-lane masks: left to itself the compiler keeps
                    // both masks in SGPR pairs and issues v_cndmask_b32_e64 at half rate; with the
                    // mask in VCC the e32 form issues at full rate)
                    uint32_t xa, xb, a0, a1, a2, a3;
                    {
                        uint32_t t0, t1, t2, t3;
                        asm("s_mov_b64 vcc, %[m1]\n\t"
                            "v_cndmask_b32_e32 %[t0], %[q0], %[q1], vcc\n\t"
                            "v_cndmask_b32_e32 %[t1], %[q1], %[q2], vcc\n\t"
                            "v_cndmask_b32_e32 %[t2], %[q2], %[q3], vcc\n\t"
                            "v_cndmask_b32_e32 %[t3], %[q3], %[q0], vcc\n\t"
                            "s_mov_b64 vcc, %[m2]\n\t"
                            "v_cndmask_b32_e32 %[a0], %[t0], %[t2], vcc\n\t"
                            "v_cndmask_b32_e32 %[a1], %[t1], %[t3], vcc\n\t"
                            "v_cndmask_b32_e32 %[a2], %[t2], %[t0], vcc\n\t"
                            "v_cndmask_b32_e32 %[a3], %[t3], %[t1], vcc\n\t"
                            "v_cndmask_b32_e32 %[xa], %[lo], %[hi], vcc\n\t"
                            "v_cndmask_b32_e32 %[xb], %[hi], %[lo], vcc"
                            : [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [a0] "=&v"(a0),
                              [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), [xa] "=&v"(xa), [xb] "=&v"(xb)
                            : [m1] "s"(msel1), [m2] "s"(msel2), [q0] "v"(q0), [q1] "v"(q1), [q2] "v"(q2), [q3] "v"(q3),
                              [lo] "v"(lo), [hi] "v"(hi)
                            : "vcc");
                    }
                    const uint32_t klo = __builtin_amdgcn_alignbit(xb, xa, rr4), khi = __builtin_amdgcn_alignbit(xa, xb, rr4);
#else
                    const uint32_t xa = rswap ? hi : lo, xb = rswap ? lo : hi;
                    const uint32_t klo = __builtin_amdgcn_alignbit(xb, xa, rr4), khi = __builtin_amdgcn_alignbit(xa, xb, rr4);
                    const uint32_t t0 = (dsel & 1) ? q1 : q0, t1 = (dsel & 1) ? q2 : q1;
                    const uint32_t t2 = (dsel & 1) ? q3 : q2, t3 = (dsel & 1) ? q0 : q3;
                    const uint32_t a0 = (dsel & 2) ? t2 : t0, a1 = (dsel & 2) ? t3 : t1;
                    const uint32_t a2 = (dsel & 2) ? t0 : t2, a3 = (dsel & 2) ? t1 : t3;
#endif
                    // quality bytes (< 128 here): the low word of a cell increment
                    const uint32_t qr[4] = {__builtin_amdgcn_alignbyte(a1, a0, r & 3), __builtin_amdgcn_alignbyte(a2, a1, r & 3),
                                            __builtin_amdgcn_alignbyte(a3, a2, r & 3), __builtin_amdgcn_alignbyte(a0, a3, r & 3)};
                    // slot nibble t % 8 at bits 8-11: a right shift of the word (nibbles 2-7) or of the
                    // word shifted left by 8 (nibbles 0-1; one 64-bit shift gives both words' copies,
                    // the high one with klo's top byte in its low bits, masked off)
#if FQ_ST_SH64
                    // nibble u of both words to bits 8-11 by one 64-bit shift of {khi, klo} (its low
                    // word: klo's nibble u, its high word: khi's): steps t and t + 8 share it
                    const unsigned long long K = (unsigned long long)khi << 32 | klo;
                    // (one v_lshlrev_b64 / v_lshrrev_b64 each, full rate; left to itself the compiler
                    // splits them into a v_alignbit and a shift)
                    unsigned long long Ks[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        if (u == 2) Ks[u] = K;
                        else if (u < 2) asm("v_lshlrev_b64 %0, %2, %1" : "=v"(Ks[u]) : "v"(K), "i"(8 - 4 * u));
                        else asm("v_lshrrev_b64 %0, %2, %1" : "=v"(Ks[u]) : "v"(K), "i"(4 * (u - 2)));
                    }
#else
                    const unsigned long long k8 = ((unsigned long long)khi << 32 | klo) << 8;
                    const uint32_t klo8 = (uint32_t)k8, khi8 = (uint32_t)(k8 >> 32);
#endif
#pragma unroll
                    for (int t = 0; t < 16; ++t) {
                        const int u = t & 7;
#if FQ_ST_SH64
                        const uint32_t ksh = t < 8 ? (uint32_t)Ks[u] : (uint32_t)(Ks[u] >> 32);
#else
                        const uint32_t kw = u < 2 ? (t < 8 ? klo8 : khi8) : (t < 8 ? klo : khi);
                        const uint32_t ksh = u < 2 ? kw >> (4 * u) : kw >> (4 * (u - 2));
#endif
                        // (byte 0 and 3 by one full-rate op, 1 and 2 by a bit-field extract)
                        const uint32_t qw = qr[t >> 2];
                        const uint32_t qv = (t & 3) == 0 ? qw & 0xFFu : (t & 3) == 3 ? qw >> 24 : __builtin_amdgcn_ubfe(qw, 8 * (t & 3), 8);
                        uint32_t a;  // rwb[t] | (ksh & 0xF00): one v_bitop3
                        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xEA" : "=v"(a) : "v"(ksh), "v"(slot_m), "v"(rwb[t]));
                        a += (uint32_t)(F * kRSlots * 64 * 4);  // (folds into the ds offset)
                        __hip_atomic_fetch_add(reinterpret_cast<LdsU64*>((size_t)a), kCount1 | (unsigned long long)qv,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
            }
        }
#if FQ_STATS_PRIO && !FQ_STATS_PRIO_ALL
        __builtin_amdgcn_s_setprio(0);
#endif
        // read 2's merged-part start, known to both lanes of the pair (all lanes swap)
        const int ws2 = MERGE ? (mate ? ws : xor32(ws)) : 0;
        if (MERGE && removed_mode && valid && !(abl & 4) && merged && post_on) {
            // Read 2's part of the merged read, rc(r2)[ol, ol + m2) at merged cycles m1 .. m1+m2-1
            // (OverlapAnalysis::merge src/overlapanalysis.cpp:74-104, then Stats::statRead of the
            // merged read, src/peprocessor.cpp:361): read 2's column holds the reverse complement,
            // so merged position j is column index 159 - pos_hi + j (codes already complemented);
            // its quality is read 2's byte at forward position pos_hi - j.  Cells: cycle rows of
            // the extra block, count << 40 | sum(q); N bases are counted as G and moved.  Both
            // lanes of the pair share the part (m1, m2 are pair-uniform): 16-position group J goes
            // to the lane of mate J % 2, so no lane of a merged pair idles here.
            const uint32_t xb = (uint32_t)(LY::kColsW + LY::kMrgOff) * 4u;
            const int c2 = lane_x | 32;  // read 2's column
            const int pos_hi = ws2 + m2 - 1;
            const int ci0 = kMaxLen - 1 - pos_hi;
            // FQ_MERGE_ROTATE=1: each lane walks its groups rotated by rl = (lane - m1) % 16
            // positions: at step t it takes part position 16 J + (t + rl) % 16, merged cycle c with
            // c % 16 = (t + lane) % 16, so the 16 lanes of an LDS group hit 16 bank pairs whatever
            // their m1.  Unrotated (the default), the cycles of a step depend on m1 and collide: 39 %
            // of the C4 kernel's LDS cycles are bank conflicts, 4.6 % rotated -- but the rotation's
            // VALU (+104 per tile) costs more than the conflicts (C4 +1-2 % per launch,
            // profiles/r04_ab_merge_rotate.txt): the LDS waits overlap other waves' VALU.
            // rb[t]: byte address of step t's slot-0 cell (mcell) for the lane's next J.
            static_assert((LY::kColsW + LY::kMrgOff) % 256 == 0, "merged-part rows: 1 KiB aligned");
            constexpr bool kRot = FQ_MERGE_ROTATE != 0;
            const int rl = kRot ? (lane_x - m1) & 15 : 0;
            uint32_t rb[16];
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int c = m1 + ((t + rl) & 15) + 16 * mate;
                rb[t] = xb + (uint32_t)((c >> 4) << 10 | (c & 15) << 3);
                asm volatile("" : "+v"(rb[t]));
            }
            const uint32_t mslot_m = vk(0x380u);
            const bool mswap = rl >= 8;
            const int rr4m = 4 * (rl & 7);
            // qualities: qa is in reversed position order v = 15 - u (byte v % 4 of qa[v / 4]);
            // rotated by rv = -rl bytes, step t's byte is at reversed index 15 - t
            const int rv = (16 - rl) & 15, vsel = rv >> 2;
            // quality dwords of forward positions [hi - 15, hi], hi = pos_hi - 16J: words
            // wl0 - 4J .. wl0 - 4J + 4; the lane's next group (J + 2) is requested one group ahead
            const int wl0 = (pos_hi - 15) >> 2, sh = (pos_hi - 15) & 3;  // (negative only for dummies)
            const uint8_t* Q2 = b.qual2 + roff;
            const uint32_t* qrow2 = qrows + c2 * kQS;
            auto qword = [&](int wi) -> uint32_t {
                if constexpr (LY::kQLds) return qrow2[min(max(wi, 0), kQS - 1)];
                else return RowQual{Q2, b.stride >> 2}.word(max(wi, 0));
            };
            uint32_t qw5[5];
#if FQ_MRG2
            if constexpr (!kRot && !LY::kQLds) {
                // The lane's groups J = mate + 2k unrolled (k < kMrgIter): the cell rows of group k are
                // 2048 k bytes on (an immediate of the atomics), and its quality dwords 1024 k bytes
                // back in the row.  The dwords come through a buffer over the wave's tile of read 2's
                // quality plane: an offset outside the tile (a dummy position before the row) reads 0
                // instead of faulting, so no clamping; the 5 offsets are computed once.
                constexpr int kMrgIter = (kMaxLen + 31) / 32;
                const size_t tile_off = (size_t)__builtin_amdgcn_readfirstlane(t) * FQ_TILE_READS * (size_t)b.stride;
                const __amdgpu_buffer_rsrc_t qr2 = __builtin_amdgcn_make_buffer_rsrc(
                    (void*)(b.qual2 + tile_off), (short)0, FQ_TILE_READS * b.stride, 0x00020000);
                int vo[5];
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    const int w = wl0 - 4 * mate + i;
                    vo[i] = (w >> 2) * (FQ_TILE_READS * FQ_CHUNK) + ((w & 3) << 2) + pl * FQ_CHUNK;
                }
#pragma unroll
                for (int i = 0; i < 5; ++i) qw5[i] = __builtin_amdgcn_raw_buffer_load_b32(qr2, vo[i], 0, 0);
                // slot nibble to bits 7-9: nibble u of both words by one 64-bit shift (as FQ_ST_SH64)
#pragma unroll
                for (int k = 0; k < kMrgIter; ++k) {
                    const int J = mate + 2 * k;
                    if (!__any(16 * J < m2)) break;  // (wave-uniform)
                    if (16 * J < m2) {
                        const uint32_t cw = field_window_masked(col, kFC, c2, ci0 + 16 * J);
                        const uint32_t nw = field_window_masked(col, kFN, c2, ci0 + 16 * J);
                        uint32_t qn[5] = {0u, 0u, 0u, 0u, 0u};
                        if (k + 1 < kMrgIter)
#pragma unroll
                            for (int i = 0; i < 5; ++i) qn[i] = __builtin_amdgcn_raw_buffer_load_b32(qr2, vo[i] - 1024 * (k + 1), 0, 0);
                        uint32_t qa[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) qa[i] = __builtin_amdgcn_alignbyte(qw5[i + 1], qw5[i], sh);
                        auto qbyte = [&](int tt) -> uint32_t {  // step tt: part position tt, byte 3 - tt % 4 of qa[3 - tt / 4]
                            const uint32_t qw = qa[(15 - tt) >> 2];
                            const int bs = (15 - tt) & 3;
                            return bs == 0 ? qw & 0xFFu : bs == 3 ? qw >> 24 : __builtin_amdgcn_ubfe(qw, 8 * bs, 8);
                        };
                        const int rem = m2 - 16 * J;
                        const unsigned long long dm = ~0ull << min(4 * max(rem, 0), 63);
                        uint32_t nlo = spread2to4(cw), nhi = spread2to4(cw >> 16);
                        const uint32_t dlo = (uint32_t)dm, dhi = rem >= 16 ? 0u : (uint32_t)(dm >> 32);
                        nlo = (nlo & ~dlo) | (dlo & 0x55555555u);  // 5 = kDummySlot
                        nhi = (nhi & ~dhi) | (dhi & 0x55555555u);
                        // nibble u of {nhi, nlo} to bits 7-9: K << 7 (u 0), K << 3 (u 1), K >> (4u - 7)
                        const unsigned long long K = (unsigned long long)nhi << 32 | nlo;
                        unsigned long long Ks[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            if (u < 2) asm("v_lshlrev_b64 %0, %2, %1" : "=v"(Ks[u]) : "v"(K), "i"(7 - 4 * u));
                            else asm("v_lshrrev_b64 %0, %2, %1" : "=v"(Ks[u]) : "v"(K), "i"(4 * u - 7));
                        }
#pragma unroll
                        for (int tt = 0; tt < 16; ++tt) {
                            const uint32_t ksh = tt < 8 ? (uint32_t)Ks[tt & 7] : (uint32_t)(Ks[tt & 7] >> 32);
                            uint32_t a;
                            asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xEA" : "=v"(a) : "v"(ksh), "v"(mslot_m), "v"(rb[tt]));
                            a += 2048u * (uint32_t)k;  // (folds into the ds offset)
                            __hip_atomic_fetch_add(reinterpret_cast<LdsU64*>((size_t)a), kCount1 | (unsigned long long)qbyte(tt),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                        uint32_t nv = nw & posmask(rem);
                        while (nv) {  // N (code 3): from the G slot (3) to the N slot (4)
                            const int tt = (__ffs(nv) - 1) >> 1;
                            nv &= nv - 1;
                            const unsigned long long v =
                                kCount1 | (unsigned long long)__builtin_amdgcn_ubfe(qa[3 - (tt >> 2)], 8 * (3 - (tt & 3)), 8);
                            const int c = m1 + 16 * J + tt;
                            const uint32_t a = xb + (uint32_t)((c >> 4) << 10 | (c & 15) << 3);
                            __hip_atomic_fetch_add(reinterpret_cast<LdsU64*>((size_t)(a + 4u * 128u)), v, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                            __hip_atomic_fetch_add(reinterpret_cast<LdsU64*>((size_t)(a + 3u * 128u)), 0ull - v,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
#pragma unroll
                        for (int i = 0; i < 5; ++i) qw5[i] = qn[i];
                    }
                }
            } else
#endif
            {
#pragma unroll
            for (int i = 0; i < 5; ++i) qw5[i] = qword(wl0 - 4 * mate + i);
            for (int J = mate; 16 * J < m2; J += 2) {
                // (ci0 >= 0; positions past the part are the dummy slot / masked by rem)
                const uint32_t cw = field_window_masked(col, kFC, c2, ci0 + 16 * J);
                const uint32_t nw = field_window_masked(col, kFN, c2, ci0 + 16 * J);
                uint32_t qn[5];
#pragma unroll
                for (int i = 0; i < 5; ++i) qn[i] = qword(wl0 - 4 * (J + 2) + i);
                // qualities ascending in qa[0..3]: part position u is byte 3 - u % 4 of qa[3 - u / 4]
                uint32_t qa[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) qa[i] = __builtin_amdgcn_alignbyte(qw5[i + 1], qw5[i], sh);
                // rotated: reversed index x = 4k + b is byte b of qv4[k], position u = (15 - x + rl) % 16
                uint32_t qv4[4] = {qa[0], qa[1], qa[2], qa[3]};
                if constexpr (kRot) {
                const uint32_t t0 = (vsel & 1) ? qa[1] : qa[0], t1 = (vsel & 1) ? qa[2] : qa[1];
                const uint32_t t2 = (vsel & 1) ? qa[3] : qa[2], t3 = (vsel & 1) ? qa[0] : qa[3];
                const uint32_t a0 = (vsel & 2) ? t2 : t0, a1 = (vsel & 2) ? t3 : t1;
                const uint32_t a2 = (vsel & 2) ? t0 : t2, a3 = (vsel & 2) ? t1 : t3;
                qv4[0] = __builtin_amdgcn_alignbyte(a1, a0, rv & 3), qv4[1] = __builtin_amdgcn_alignbyte(a2, a1, rv & 3);
                qv4[2] = __builtin_amdgcn_alignbyte(a3, a2, rv & 3), qv4[3] = __builtin_amdgcn_alignbyte(a0, a3, rv & 3);
                }
                auto qbyte = [&](int t) -> uint32_t {  // step t (bytes 0 and 3 by one full-rate op)
                    const uint32_t qw = qv4[(15 - t) >> 2];
                    const int bs = (15 - t) & 3;
                    return bs == 0 ? qw & 0xFFu : bs == 3 ? qw >> 24 : __builtin_amdgcn_ubfe(qw, 8 * bs, 8);
                };
                // slot nibbles: code, or the dummy slot beyond the part
                const int rem = m2 - 16 * J;
                const unsigned long long dm = ~0ull << min(4 * max(rem, 0), 63);
                uint32_t nlo = spread2to4(cw), nhi = spread2to4(cw >> 16);
                const uint32_t dlo = (uint32_t)dm, dhi = rem >= 16 ? 0u : (uint32_t)(dm >> 32);
                nlo = (nlo & ~dlo) | (dlo & 0x55555555u);  // 5 = kDummySlot
                nhi = (nhi & ~dhi) | (dhi & 0x55555555u);
                // rotated by rl nibbles: nibble t of {khi:klo} is part position (t + rl) % 16
                uint32_t klo = nlo, khi = nhi;
                if constexpr (kRot) {
                    const uint32_t xa = mswap ? nhi : nlo, xb2 = mswap ? nlo : nhi;
                    klo = __builtin_amdgcn_alignbit(xb2, xa, rr4m), khi = __builtin_amdgcn_alignbit(xa, xb2, rr4m);
                }
                // slot nibble t % 8 to bits 7-9 by one right shift (of the words shifted left by 8
                // for nibbles 0-1, as in the removed-mode pass above), or-ed into the cell address
                const unsigned long long k8 = ((unsigned long long)khi << 32 | klo) << 8;
                const uint32_t nlo8 = (uint32_t)k8, nhi8 = (uint32_t)(k8 >> 32);
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    const int u = t & 7;
                    const uint32_t ksh = u < 2 ? (t < 8 ? nlo8 : nhi8) >> (4 * u + 1) : (t < 8 ? klo : khi) >> (4 * u - 7);
                    uint32_t a;
                    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xEA" : "=v"(a) : "v"(ksh), "v"(mslot_m), "v"(rb[t]));
                    __hip_atomic_fetch_add(reinterpret_cast<LdsU64*>((size_t)a), kCount1 | (unsigned long long)qbyte(t),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                uint32_t nv = nw & posmask(rem);
                while (nv) {  // N (code 3): from the G slot (3) to the N slot (4)
                    const int t = (__ffs(nv) - 1) >> 1;
                    nv &= nv - 1;
                    const unsigned long long v =
                        kCount1 | (unsigned long long)__builtin_amdgcn_ubfe(qa[3 - (t >> 2)], 8 * (3 - (t & 3)), 8);
                    const int c = m1 + 16 * J + t;  // (rb[t] recomputed: t is not a constant)
                    const uint32_t a = xb + (uint32_t)((c >> 4) << 10 | (c & 15) << 3);
                    __hip_atomic_fetch_add(reinterpret_cast<LdsU64*>((size_t)(a + 4u * 128u)), v, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(reinterpret_cast<LdsU64*>((size_t)(a + 3u * 128u)), 0ull - v,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
#pragma unroll
                for (int i = 0; i < 5; ++i) qw5[i] = qn[i];
#pragma unroll
                for (int t = 0; t < 16; ++t) rb[t] += 2048u;  // (J + 2: two cycle rows on)
            }
            }
        }
#if FQ_STATS_PRIO && FQ_STATS_PRIO_ALL == 1
        __builtin_amdgcn_s_setprio(0);
#endif
        if (valid && !(abl & 4) && !removed_mode) {
            const int wlen = post_on ? wn : 0;  // post window [ws, ws + wlen)
            // merged pairs: both parts go to read 1's post block, read 2's part reversed and
            // complemented (merged cycle c0 - pos)
            uint32_t* post_h = (MERGE && merged) ? hist + 2 * kHistW : my_post;
            const bool rev = MERGE && merged && mate;
            const int c0 = st + n - 1 - mol + m1;
            const int nchl = (L + 15) >> 4;
            const int dsel = r >> 2;
            // chunk F+1's codes (LDS) and the qualities of chunks F+1, F+2 (the row again, now from
            // L2) are in flight while chunk F's atomics issue
            Fwd fn = fwd_chunk(col, lane_x, 0, rc);
            uint4 qn = qchunk(0);
            uint4 qnn = qchunk(min(1, nchunks - 1));
            for (int F = 0; F < nchl; ++F) {
                const Fwd f = fn;
                const uint32_t q0 = qn.x, q1 = qn.y, q2 = qn.z, q3 = qn.w;
                qn = qnn;
                qnn = qchunk(min(F + 2, nchunks - 1));
                fn = fwd_chunk(col, lane_x, min(F + 1, nchunks - 1), rc);
                // rotate the chunk by r positions: position t of the rotated view is 16F + (t+r)%16
                const uint32_t cr = __builtin_amdgcn_alignbit(f.c, f.c, 2 * r);
                const uint32_t nr = __builtin_amdgcn_alignbit(f.n, f.n, 2 * r);
                const uint32_t t0 = (dsel & 1) ? q1 : q0, t1 = (dsel & 1) ? q2 : q1;
                const uint32_t t2 = (dsel & 1) ? q3 : q2, t3 = (dsel & 1) ? q0 : q3;
                const uint32_t a0 = (dsel & 2) ? t2 : t0, a1 = (dsel & 2) ? t3 : t1;
                const uint32_t a2 = (dsel & 2) ? t0 : t2, a3 = (dsel & 2) ? t1 : t3;
                const uint32_t qr[4] = {__builtin_amdgcn_alignbyte(a1, a0, r & 3), __builtin_amdgcn_alignbyte(a2, a1, r & 3),
                                        __builtin_amdgcn_alignbyte(a3, a2, r & 3), __builtin_amdgcn_alignbyte(a0, a3, r & 3)};
#pragma unroll
                for (int wi = 0; wi < 4; ++wi) {
                    const uint32_t qw = qr[wi];
#pragma unroll
                    for (int bi = 0; bi < 4; ++bi) {
                        const int tt = 4 * wi + bi;
                        const int pos = 16 * F + ((tt + r) & 15);
                        const uint32_t qv = (qw >> (8 * bi)) & 0xFFu;
                        const int slot = (int)(((cr >> (2 * tt)) & 3u) + ((nr >> (2 * tt)) & 1u));
                        const unsigned long long v = kCount1 | (unsigned long long)(qv | 0x80u);
                        if (!(abl & 16)) {
                            hadd(my_pre, cell(pos, pos < L ? slot : kDummySlot), v);
                            const bool inw = (unsigned)(pos - ws) < (unsigned)wlen;
                            int cyc = pos - ws, sl = slot;
                            if (MERGE && rev) {
                                cyc = c0 - pos;
                                sl = slot < 4 ? slot ^ 2 : 4;  // A<->T, C<->G
                            }
                            hadd(post_h, inw ? cell(cyc, sl) : cell(pos, kDummySlot), v);
                        }
                    }
                }
            }
        }
        FQ_STAMP(6)
        if (abl & 256) {  // profiling only: 512 extra independent VALU ops per tile (issue-rate probe)
            uint32_t d0 = lane_x, d1 = lane_x + 1, d2 = lane_x + 2, d3 = lane_x + 3;
#pragma unroll
            for (int i = 0; i < 128; ++i)
                asm volatile("v_xor_b32 %0, %0, %4\n\tv_xor_b32 %1, %1, %4\n\tv_xor_b32 %2, %2, %4\n\tv_xor_b32 %3, %3, %4"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(L));
            if ((d0 ^ d1 ^ d2 ^ d3) == 0x9E3779B9u) rr.reserved = 1;
        }
        if (valid) {
            rr.start = nn ? (uint16_t)st : 0;
            rr.len = nn ? (uint16_t)n : 0;
            rr.code = (uint8_t)code;
            // one 16-byte store (a struct copy compiles to four partial stores)
            const uint4 w = make_uint4((uint32_t)rr.start | (uint32_t)rr.len << 16,
                                       (uint32_t)rr.code | (uint32_t)rr.flags << 8 | (uint32_t)rr.ad_pos << 16,
                                       (uint32_t)rr.ad_len | (uint32_t)rr.m_len1 << 16,
                                       (uint32_t)rr.m_len2 | (uint32_t)rr.reserved << 16);
            if (res) *reinterpret_cast<uint4*>(&res[PAIRED ? 2 * (size_t)idx + mate : (size_t)idx]) = w;
        }
    }
    if (lane < hres[2 * wave + 1]) slow_tiles[hres[2 * wave] + lane] = kHole;  // the rest of the last reservation

    FQ_STAMP(7)
#ifdef FQ_PHASE_STAMPS
    if (stamps && lane == 0)
        for (int i = 0; i < kPhases; ++i) atomicAdd(&g_phase_cycles[i], ph[i]);
#endif
#undef FQ_STAMP
    __syncthreads();

    // ---------------- flush to the global accumulator ----------------
    for (int i = threadIdx.x; i < FQ_ACC_INSERT; i += kThreads)
        if (small[i]) atomicAdd(&acc[i], small[i]);
    for (int i = threadIdx.x; i <= p.insert_size_max; i += kThreads)
        if (ins[i]) atomicAdd(&acc[FQ_ACC_INSERT + i], (unsigned long long)ins[i]);
    const size_t st_base = acc_stats_offset(p.insert_size_max, p.max_cycles, 0);
    const size_t st_words = acc_stats_words(p.max_cycles);
    if (threadIdx.x < 16) {  // stats k: [reads << 32 | length_sum, q20 << 32 | q30] -> the four words
        const int k = threadIdx.x >> 2, f = threadIdx.x & 3;
        unsigned long long v = 0;
        for (int c = 0; c < LY::kScalCopies; ++c) {
            const unsigned long long w = scal[kScalStride * c + 4 * k + (f >> 1)];
            v += (f & 1) ? (w & 0xFFFFFFFFull) : (w >> 32);
        }
        if (v) atomicAdd(&acc[st_base + k * st_words + f], v);  // FQ_ST_READS, _LENGTH_SUM, _Q20, _Q30
    } else if (threadIdx.x < 18) {  // polyG (slot 2) and adapter (slot 3) counters: reads << 32 | bases
        const int slot = threadIdx.x - 14;
        unsigned long long rd = 0, bs = 0;
        for (int c = 0; c < LY::kScalCopies; ++c)
            for (int m = 0; m < 2; ++m) {
                const unsigned long long w = scal[kScalStride * c + 4 * m + slot];
                rd += w >> 32;
                bs += w & 0xFFFFFFFFull;
            }
        if (rd) atomicAdd(&acc[slot == 2 ? FQ_ACC_POLYX_READS + 3 : FQ_ACC_ADAPTER_READS], rd);
        if (bs) atomicAdd(&acc[slot == 2 ? FQ_ACC_POLYX_BASES + 3 : FQ_ACC_ADAPTER_BASES], bs);
    }
    if (removed_mode) {  // pre = kept + removed, post = kept
        const int ncyc = min(kMaxLen, p.max_cycles);
        for (int i = threadIdx.x; i < 2 * ncyc * 5; i += kThreads) {
            const int k = i / (ncyc * 5), j = i - k * ncyc * 5;
            const int c = j / 5, slot = j - c * 5;  // slots A C T G N
            const uint32_t* hk = hist + k * 32;
            const unsigned long long kept = *reinterpret_cast<const unsigned long long*>(hk + rcell(c, slot < 4 ? 4 + slot : kRNSlot + 4));
            const unsigned long long rem = *reinterpret_cast<const unsigned long long*>(hk + rcell(c, slot < 4 ? slot : kRNSlot));
            const int cls = slot_class(slot);
            const unsigned long long vals[2] = {kept + rem, kept};
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
                const long long cnt = (long long)(vals[pp] >> 40);
                const long long qs = (long long)(vals[pp] & kQMask) - 33ll * cnt;  // cells hold sum(q), q = byte
                if (cnt == 0 && qs == 0) continue;
                unsigned long long* dst = acc + st_base + (k + 2 * pp) * st_words + FQ_ST_CYCLES + (size_t)c * FQ_ST_PER_CYCLE;
                atomicAdd(&dst[cls], (unsigned long long)cnt);
                atomicAdd(&dst[8 + cls], (unsigned long long)qs);
            }
        }
    }
    if (MERGE && removed_mode) {  // read 2's merged parts: post1 (acc block 2) at cycles < 320
        const int ncyc = min(2 * kMaxLen, p.max_cycles);
        const uint32_t* hx = hist + LY::kMrgOff;
        for (int i = threadIdx.x; i < ncyc * 5; i += kThreads) {
            const int c = i / 5, slot = i - c * 5;
            const unsigned long long v = *reinterpret_cast<const unsigned long long*>(hx + mcell(c, slot));
            const long long cnt = (long long)(v >> 40);
            const long long qs = (long long)(v & kQMask) - 33ll * cnt;
            if (cnt == 0 && qs == 0) continue;
            const int cls = slot_class(slot);
            unsigned long long* dst = acc + st_base + 2 * st_words + FQ_ST_CYCLES + (size_t)c * FQ_ST_PER_CYCLE;
            atomicAdd(&dst[cls], (unsigned long long)cnt);
            atomicAdd(&dst[8 + cls], (unsigned long long)qs);
        }
    }
    for (int k = 0; k < 4 && !removed_mode; ++k) {
      const int ncyc = min((MERGE && k == 2) ? 2 * kMaxLen : kMaxLen, p.max_cycles);
      const uint32_t* hk = hist + (k == 3 && MERGE ? 4 : k) * kHistW;
      for (int i = threadIdx.x; i < ncyc * 5; i += kThreads) {
        const int c = i / 5, slot = i - c * 5;
        const unsigned long long v = *reinterpret_cast<const unsigned long long*>(hk + cell(c, slot));
        const unsigned long long w = v;
        const long long cnt = (long long)(w >> 40);
        const long long qs = (long long)(w & kQMask) - 161ll * cnt;  // undo the +128 bias, -33
        if (cnt == 0 && qs == 0) continue;
        const int cls = slot_class(slot);
        unsigned long long* dst = acc + st_base + k * st_words + FQ_ST_CYCLES + (size_t)c * FQ_ST_PER_CYCLE;
        atomicAdd(&dst[cls], (unsigned long long)cnt);
        atomicAdd(&dst[8 + cls], (unsigned long long)qs);
      }
    }
}

}  // namespace
#if FQ_MAXLEN_BUILD_LONG
using namespace long320;
#endif

#if FQ_MAXLEN == 160
bool fq_pe_fast_supported(const fq_params& p) {
    // -c runs on the XTRA instantiations (with -m the merge variant's); its Stats fix-up goes to the
    // removed-mode block, or with front trimming / UMI to the pre block.  Single-end -c is a no-op
    // (SingleEndProcessor never corrects, src/seprocessor.cpp).  UMI with -m: the merge variant's
    // -c / UMI instantiation, whose Stats run in pre/post mode.
    return p.insert_size_max <= 512 && p.insert_size_max >= 0 &&
           (!p.merge_enabled || p.paired);
}

// profiling aid (tools/ablate.py --phases): read and clear the per-phase cycle totals
extern "C" __attribute__((visibility("default"))) int fq_debug_phase_cycles(unsigned long long* out, int n) {
    unsigned long long h[kPhases];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_phase_cycles), sizeof h) != hipSuccess) return -3;
    const unsigned long long z[kPhases] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), z, sizeof z) != hipSuccess) return -3;
    for (int i = 0; i < n && i < kPhases; ++i) out[i] = h[i];
    return 0;
}
#define FQ_PREPARE fq_pe_fast_prepare
#define FQ_LAUNCH fq_launch_pe_fast
#else  // the long-read build (pe_fast_long.hip): no merge variant
#define FQ_PREPARE fq_pe_fast_long_prepare
#define FQ_LAUNCH fq_launch_pe_fast_long
#endif

// every instantiation (and its FIX twin) may use the LDS its layout declares
template <bool LEAN, bool PAIRED, bool MERGE, bool XTRA>
static hipError_t set_lds() {
    const int bytes = Layout<LEAN, MERGE, PAIRED>::kLdsW * 4 + (LEAN ? 4096 : 0);  // (LEAN: + profiling pad, reserved[2])
    hipError_t e = hipFuncSetAttribute((const void*)pe_fast_kernel<LEAN, PAIRED, MERGE, XTRA, false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, bytes > 160 * 1024 ? 160 * 1024 : bytes);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute((const void*)pe_fast_kernel<LEAN, PAIRED, MERGE, XTRA, true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, bytes > 160 * 1024 ? 160 * 1024 : bytes);
}

hipError_t FQ_PREPARE() {
    hipError_t e;
    if ((e = set_lds<true, true, false, false>()) != hipSuccess) return e;
    if ((e = set_lds<false, true, false, false>()) != hipSuccess) return e;
    if ((e = set_lds<true, false, false, false>()) != hipSuccess) return e;
    if ((e = set_lds<false, false, false, false>()) != hipSuccess) return e;
    // the -c / UMI instantiations of the full variants
    if ((e = set_lds<false, true, false, true>()) != hipSuccess) return e;
    if ((e = set_lds<false, false, false, true>()) != hipSuccess) return e;
#if FQ_MAXLEN == 160
    if ((e = set_lds<false, true, true, false>()) != hipSuccess) return e;
    if ((e = set_lds<false, true, true, true>()) != hipSuccess) return e;
    return fq_pe_fast_long_prepare();
#else
    if ((e = set_lds<false, true, true, false>()) != hipSuccess) return e;
    return set_lds<false, true, true, true>();
#endif
}

template <bool LEAN, bool PAIRED, bool MERGE, bool XTRA>
static void launch_variant(const fq_params& p, const fq_batch& b, fq_read_result* res, unsigned long long* acc,
                           int* slow_tiles, int* slow_count, unsigned long long* xfix, int grid, int extra_lds,
                           hipStream_t stream) {
    using LY = Layout<LEAN, MERGE, PAIRED>;
    const dim3 g(grid * LY::kBlocksPerCU), t(LY::kThreads);
    const size_t lds = LY::kLdsW * 4 + extra_lds;
    if (b.stride == 16 * kChunks)
        hipLaunchKernelGGL((pe_fast_kernel<LEAN, PAIRED, MERGE, XTRA, true>), g, t, lds, stream, p, b, res, acc, slow_tiles,
                           slow_count, xfix);
    else
        hipLaunchKernelGGL((pe_fast_kernel<LEAN, PAIRED, MERGE, XTRA, false>), g, t, lds, stream, p, b, res, acc, slow_tiles,
                           slow_count, xfix);
}

hipError_t FQ_LAUNCH(const fq_params& p, const fq_batch& b, fq_read_result* res, unsigned long long* acc,
                     int* slow_tiles, int* slow_count, unsigned long long* xfix, int grid, hipStream_t stream) {
#if FQ_MAXLEN == 160
    // rows longer than 160 bytes: the 320-position build (reads beyond 320 bp are handed off per tile)
    if (b.stride > kMaxLen)
        return fq_launch_pe_fast_long(p, b, res, acc, slow_tiles, slow_count, xfix, grid, stream);
#endif
    const bool lean = p.trim_front1 == 0 && p.trim_tail1 == 0 && p.trim_front2 == 0 && p.trim_tail2 == 0 &&
                      !(p.avg_qual_limit > 0) &&
                      !p.cut_front && !p.cut_right && !p.cut_tail && !p.polyx_enabled && p.adapter1_len == 0 &&
                      p.adapter2_len == 0 && p.max_len1 <= 0 && p.max_len2 <= 0 && !p.complexity_enabled &&
                      !p.correction_enabled && p.umi_front1 <= 0 && p.umi_front2 <= 0;
    // -c, UMI and -e (the whole-read quality total) run on the XTRA instantiations (lean is false then)
    const bool xtra = p.correction_enabled || p.umi_front1 > 0 || p.umi_front2 > 0 || p.avg_qual_limit > 0;
    const int pad = p.reserved[2] > 0 && p.reserved[2] <= 4096 ? p.reserved[2] : 0;  // profiling: extra LDS (LEAN)
    if (p.merge_enabled && xtra)  // -c / UMI / -e with -m
        launch_variant<false, true, true, true>(p, b, res, acc, slow_tiles, slow_count, xfix, grid, 0, stream);
    else if (p.merge_enabled)
        launch_variant<false, true, true, false>(p, b, res, acc, slow_tiles, slow_count, xfix, grid, 0, stream);
    else
    if (p.paired && lean)
        launch_variant<true, true, false, false>(p, b, res, acc, slow_tiles, slow_count, xfix, grid, pad, stream);
    else if (p.paired && xtra)
        launch_variant<false, true, false, true>(p, b, res, acc, slow_tiles, slow_count, xfix, grid, 0, stream);
    else if (p.paired)
        launch_variant<false, true, false, false>(p, b, res, acc, slow_tiles, slow_count, xfix, grid, 0, stream);
    else if (lean)
        launch_variant<true, false, false, false>(p, b, res, acc, slow_tiles, slow_count, xfix, grid, pad, stream);
    else if (xtra)
        launch_variant<false, false, false, true>(p, b, res, acc, slow_tiles, slow_count, xfix, grid, 0, stream);
    else
        launch_variant<false, false, false, false>(p, b, res, acc, slow_tiles, slow_count, xfix, grid, 0, stream);
    return hipGetLastError();
}
#undef FQ_PREPARE
#undef FQ_LAUNCH

#if FQ_MAXLEN == 160
// The exotic-byte Stats moves (kXfixCopies copies of the four Stats blocks, see the fix-up in the
// kernel) summed into the accumulator and cleared, when the flag after the copies is set.
namespace {
__global__ void xfix_fold_kernel(unsigned long long* __restrict__ acc, unsigned long long* __restrict__ xfix, size_t words) {
    if (!xfix[kXfixCopies * words]) return;
    for (size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += (size_t)gridDim.x * blockDim.x) {
        unsigned long long v = 0;
        for (int c = 0; c < kXfixCopies; ++c) {
            v += xfix[(size_t)c * words + w];
            xfix[(size_t)c * words + w] = 0ull;
        }
        if (v) atomicAdd(&acc[w], v);
    }
}
__global__ void xfix_flag_clear_kernel(unsigned long long* __restrict__ xfix, size_t words) {
    xfix[kXfixCopies * words] = 0ull;
}
}  // namespace

size_t fq_xfix_words(int32_t max_cycles) { return (size_t)kXfixCopies * 4 * fq_acc_stats_words(max_cycles) + 1; }

hipError_t fq_launch_xfix_fold(unsigned long long* acc_stats, unsigned long long* xfix, int32_t max_cycles, hipStream_t s) {
    const size_t words = 4 * fq_acc_stats_words(max_cycles);
    hipLaunchKernelGGL(xfix_fold_kernel, dim3(64), dim3(256), 0, s, acc_stats, xfix, words);
    hipLaunchKernelGGL(xfix_flag_clear_kernel, dim3(1), dim3(1), 0, s, xfix, words);
    return hipGetLastError();
}
#endif
