// text.hip -- GPU-side ingest and egress of FASTQ-text packs (fq_engine_submit_text):
//   * text_tile_kernel builds the chunk-interleaved batch planes (include/fqengine.h) straight
//     from the input FASTQ bytes, replacing the host's tile packing (FqReader's Read objects and
//     the pack planes: src/fqreader.cpp:90-195, src/read.h);
//   * text_size_kernel / hipcub exclusive scans / text_write_kernel assemble the output FASTQ of
//     the records that pass, in input order, as Read::toString writes them (src/read.h:166-168:
//     name, sequence, strand and quality lines, the trimmed window [start, start + len)), routed as
//     PairEndProcessor / SingleEndProcessor route passing reads to out1 / out2
//     (src/peprocessor.cpp:402-403, :457-491; src/seprocessor.cpp:337-350).
// Byte copies are lane per record (records are a few hundred bytes; PCIe, not these kernels,
// bounds the path).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "engine_internal.h"

namespace {

// one thread per (read, 16-byte chunk): 32 consecutive threads write one 512-byte tile chunk run
__global__ void text_tile_kernel(const char* __restrict__ text, const fq_text_rec* __restrict__ rec, int n, int stride,
                                 uint8_t* __restrict__ seq, uint8_t* __restrict__ qual, uint16_t* __restrict__ lens) {
    const int nch = stride >> 4;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long per_tile = (long long)FQ_TILE_READS * nch;
    const long long tile = t / per_tile;
    const int within = (int)(t - tile * per_tile);
    const int k = within / FQ_TILE_READS, i32 = within % FQ_TILE_READS;
    const long long r = tile * FQ_TILE_READS + i32;
    if (r >= n) return;
    const fq_text_rec R = rec[r];
    const int len = R.len;
    if (k == 0) lens[r] = (uint16_t)len;
    const int j0 = 16 * k;
    uint32_t s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
    const uint8_t* ps = reinterpret_cast<const uint8_t*>(text) + R.seq_off + j0;
    const uint8_t* pq = reinterpret_cast<const uint8_t*>(text) + R.qual_off + j0;
    const int m = min(16, len - j0);
#pragma unroll
    for (int b = 0; b < 16; ++b) {
        if (b < m) {
            s[b >> 2] |= (uint32_t)ps[b] << (8 * (b & 3));
            q[b >> 2] |= (uint32_t)pq[b] << (8 * (b & 3));
        }
    }
    const size_t o = (size_t)tile * FQ_TILE_READS * stride + (size_t)k * (FQ_TILE_READS * FQ_CHUNK) + (size_t)i32 * FQ_CHUNK;
    *reinterpret_cast<uint4*>(seq + o) = make_uint4(s[0], s[1], s[2], s[3]);
    *reinterpret_cast<uint4*>(qual + o) = make_uint4(q[0], q[1], q[2], q[3]);
}

__device__ __forceinline__ bool passes(const fq_read_result& r) {
    return !(r.flags & (FQ_RF_NULL | FQ_RF_INDEX_FILTERED)) && r.code == FQ_PASS_FILTER;
}

// output bytes of record i of mate m (0 when not written): PE writes a pair only when both pass
__global__ void text_size_kernel(const fq_read_result* __restrict__ res, const fq_text_rec* __restrict__ rec, int n,
                                 int paired, int m, uint32_t* __restrict__ size) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    bool ok;
    if (paired) ok = passes(res[2 * (size_t)i]) && passes(res[2 * (size_t)i + 1]);
    else ok = passes(res[i]);
    const fq_read_result& r = res[paired ? 2 * (size_t)i + m : (size_t)i];
    size[i] = ok ? (uint32_t)rec[i].name_len + rec[i].strand_len + 2u * r.len + 4u : 0u;
}

__global__ void text_total_kernel(const uint32_t* __restrict__ size, const uint32_t* __restrict__ off, int n,
                                  unsigned long long* __restrict__ total) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *total = n ? (unsigned long long)off[n - 1] + size[n - 1] : 0ull;
}

__device__ __forceinline__ void copy_bytes(char* __restrict__ d, const char* __restrict__ s, int n) {
    for (int b = 0; b < n; ++b) d[b] = s[b];
}

__global__ void text_write_kernel(const char* __restrict__ text, const fq_text_rec* __restrict__ rec,
                                  const fq_read_result* __restrict__ res, int n, int paired, int m,
                                  const uint32_t* __restrict__ size, const uint32_t* __restrict__ off,
                                  char* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || size[i] == 0) return;
    const fq_text_rec R = rec[i];
    const fq_read_result& r = res[paired ? 2 * (size_t)i + m : (size_t)i];
    char* d = out + off[i];
    copy_bytes(d, text + R.name_off, R.name_len);
    d += R.name_len;
    *d++ = '\n';
    copy_bytes(d, text + R.seq_off + r.start, r.len);
    d += r.len;
    *d++ = '\n';
    copy_bytes(d, text + R.strand_off, R.strand_len);
    d += R.strand_len;
    *d++ = '\n';
    copy_bytes(d, text + R.qual_off + r.start, r.len);
    d += r.len;
    *d = '\n';
}

}  // namespace

hipError_t fq_launch_text_tiles(const char* d_text, const fq_text_rec* d_rec, int n, int stride, uint8_t* seq,
                                uint8_t* qual, uint16_t* lens, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const long long threads = (long long)((n + FQ_TILE_READS - 1) / FQ_TILE_READS) * FQ_TILE_READS * (stride >> 4);
    hipLaunchKernelGGL(text_tile_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, d_text, d_rec, n,
                       stride, seq, qual, lens);
    return hipGetLastError();
}

size_t fq_text_scan_temp_bytes(int n) {
    size_t bytes = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, n);
    return bytes;
}

hipError_t fq_launch_text_out(const char* d_text, const fq_text_rec* d_rec, const fq_read_result* d_res, int n, int paired,
                              int m, uint32_t* d_size, uint32_t* d_off, void* d_temp, size_t temp_bytes, char* d_out,
                              unsigned long long* d_total, hipStream_t s) {
    if (n <= 0) return hipMemsetAsync(d_total, 0, sizeof(unsigned long long), s);
    const dim3 g((n + 255) / 256), b(256);
    hipLaunchKernelGGL(text_size_kernel, g, b, 0, s, d_res, d_rec, n, paired, m, d_size);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t tb = temp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(d_temp, tb, d_size, d_off, n, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(text_total_kernel, dim3(1), dim3(64), 0, s, d_size, d_off, n, d_total);
    hipLaunchKernelGGL(text_write_kernel, g, b, 0, s, d_text, d_rec, d_res, n, paired, m, d_size, d_off, d_out);
    return hipGetLastError();
}
