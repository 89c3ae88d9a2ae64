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
                             int* slow_tiles, int* slow_count, int grid, hipStream_t stream);
// the same kernels built for rows of up to 320 bytes (pe_fast_long.hip; fq_launch_pe_fast
// forwards batches with stride > 160 to it, except -m)
hipError_t fq_pe_fast_long_prepare();
hipError_t fq_launch_pe_fast_long(const fq_params& p, const fq_batch& b, fq_read_result* res, unsigned long long* acc,
                                  int* slow_tiles, int* slow_count, int grid, hipStream_t stream);
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
