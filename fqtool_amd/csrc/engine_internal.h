// engine_internal.h -- launch entry points shared between the engine's translation units.
#pragma once

// largest fq_params.max_cycles an engine accepts (reads beyond it fail the pack with FQ_E_TOO_LONG)
#define FQ_MAX_CYCLES_LIMIT 4096

#include <hip/hip_runtime.h>

#include "../../include/fqengine.h"

// General kernel workgroup: 8 waves (one LDS histogram copy per workgroup, 2 workgroups per CU
// at <= 160 cycles: 16 waves per CU; it uses ~70 VGPRs, so registers allow more)
constexpr int kPackThreads = 512;
size_t fq_pack_kernel_lds_bytes(const fq_params& p);
hipError_t fq_pack_kernel_set_lds(const fq_params& p);
// General kernel (any bytes, any length <= max_cycles, merge): all pairs, or only the pairs
// (single-end: reads) whose indices are listed in tiles[0 .. *ntiles) when tiles != nullptr.
hipError_t fq_launch_pack_kernel(const fq_params& p, const fq_batch& b, fq_read_result* res, unsigned long long* acc,
                                 int* err, int grid, hipStream_t stream, const int* tiles = nullptr,
                                 const int* ntiles = nullptr);
// Fast kernels (pe_fast.hip); the indices of pairs / reads they cannot take are appended to
// slow_tiles (room for one per pair / read).
bool fq_pe_fast_supported(const fq_params& p);
hipError_t fq_pe_fast_prepare();
hipError_t fq_launch_pe_fast(const fq_params& p, const fq_batch& b, fq_read_result* res, unsigned long long* acc,
                             int* slow_tiles, int* slow_count, unsigned long long* xfix, int grid, hipStream_t stream);
// the fast kernels' exotic-byte Stats moves: a zeroed buffer of fq_xfix_words(max_cycles) words per
// engine, folded into the accumulator's Stats blocks (acc_stats: their first word) after each launch
size_t fq_xfix_words(int32_t max_cycles);
hipError_t fq_launch_xfix_fold(unsigned long long* acc_stats, unsigned long long* xfix, int32_t max_cycles, hipStream_t s);
// the same kernels built for rows of up to 320 bytes (pe_fast_long.hip; fq_launch_pe_fast
// forwards batches with stride > 160 to it, except -m)
hipError_t fq_pe_fast_long_prepare();
hipError_t fq_launch_pe_fast_long(const fq_params& p, const fq_batch& b, fq_read_result* res, unsigned long long* acc,
                                  int* slow_tiles, int* slow_count, unsigned long long* xfix, int grid, hipStream_t stream);
hipError_t fq_launch_synth(const fq_batch& b, uint64_t seed, uint64_t first_index, int read_len, hipStream_t stream);
// Duplication analysis of one pack into a table (dup.hip); order_base orders the pack's reads
// against other packs (the pack's sequence number).
int fq_dup_pack(fq_dup* d, const fq_batch& b, int paired, unsigned long long order_base, hipStream_t s);
const char* fq_dup_error(const fq_dup* d);
int fq_dup_device(const fq_dup* d, int* device);
// FASTQ-text packs (text.hip): tile planes built from the text; output text of the passing records
hipError_t fq_launch_text_tiles(const char* d_text, const fq_text_rec* d_rec, int n, int stride, uint8_t* seq,
                                uint8_t* qual, uint16_t* lens, hipStream_t s);
size_t fq_text_scan_temp_bytes(int n);
hipError_t fq_launch_text_out(const char* d_text, const fq_text_rec* d_rec, const fq_read_result* d_res, int n, int paired,
                              int m, uint32_t* d_size, uint32_t* d_off, void* d_temp, size_t temp_bytes, char* d_out,
                              unsigned long long* d_total, hipStream_t s);
// -m: the merged output stream of a PE text pack (text.hip), into d_out (mate 0's output)
hipError_t fq_launch_merge_out(const char* d_text1, const char* d_text2, const fq_text_rec* d_rec1,
                               const fq_text_rec* d_rec2, const fq_read_result* d_res, int n, int discard,
                               uint32_t* d_size, uint32_t* d_off, void* d_temp, size_t temp_bytes, char* d_out,
                               unsigned long long* d_total, hipStream_t s);
// Raw FASTQ streams (raw.hip): per (window, mate) device state of the record indexing
struct fq_raw_state {
    uint32_t text_start;  // buffer offset of the window's text (the carried bytes first)
    uint32_t carry_in;    // bytes carried over from the previous window
    uint32_t avail;       // carry_in + the window's raw bytes
    uint32_t overflow;    // the carry did not fit (nothing is indexed)
    int32_t first_bad;    // lowest index of a complete record that is not plain (INT_MAX: none)
    int32_t complete;     // records whose four lines are in the text (capped by the record capacity)
    int32_t max_len;      // longest sequence of the plain records
    uint32_t total_lines;
    uint32_t consumed;    // text bytes taken by the pack's records
    int32_t n;            // records (pairs) of the pack
    uint32_t pad[2];
};
struct fq_raw_text_args {
    char* text[2];
    const char* prev_text[2];
    const fq_raw_state* prev_state;  // previous window's states, nullptr at the start of the stream
    fq_raw_state* state;             // [2]
    uint32_t raw_bytes[2];
    uint32_t carry_cap;              // the raw bytes land at this buffer offset
    uint32_t nblocks;                // 4 KiB blocks of the buffer
    uint32_t* bcnt[2];
    uint32_t* bbase[2];
    uint32_t* lines[2];
    uint32_t cap_lines;
    int cap_records;
    fq_text_rec* rec[2];
    int max_len;                     // longest sequence the engine takes (longer: not plain)
};
size_t fq_raw_scan_temp_bytes(int nblocks, int n);
hipError_t fq_launch_raw_index(const fq_raw_text_args& a, int mates, int cap_batch, void* d_temp, size_t temp_bytes,
                               hipStream_t s);
// trimmed-adapter entries of mate m appended to its output text (at *d_text_total, within cap bytes
// of d_out; *d_total = the entries' bytes, ~0 if they would not fit)
hipError_t fq_launch_raw_adapters(const char* d_text, const fq_text_rec* d_rec, const fq_read_result* d_res, int n,
                                  int paired, int m, uint32_t* d_size, uint32_t* d_off, void* d_temp, size_t temp_bytes,
                                  char* d_out, const unsigned long long* d_text_total, unsigned long long cap,
                                  unsigned long long* d_total, hipStream_t s);
