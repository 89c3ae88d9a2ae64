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

// ---- -m (merge_enabled): the merged output stream ----
// PairEndProcessor's merge branch (src/peprocessor.cpp:351-385) as the host formats it
// (fqtool_amd/host/processor.cpp format_range): per pair with both reads kept, the merged read when
// the pair merged and it passes (OverlapAnalysis::merge, src/overlapanalysis.cpp:74-104: name
// "_merged_<m1>_<m2>" spliced in before the name's first space, r1[0, m1) + revcomp(r2[0, m2)),
// qualities r1's then r2's reversed, read 1's strand line), else (unless --discard_unmerged) each
// read that passes; nothing reaches out1 / out2.  One thread per pair.
__device__ __forceinline__ int dec_digits(int v) {
    int d = 1;
    while (v >= 10) {
        v /= 10;
        ++d;
    }
    return d;
}

__device__ __forceinline__ char* put_dec(char* d, int v) {
    const int nd = dec_digits(v);
    for (int k = nd - 1; k >= 0; --k) {
        d[k] = (char)('0' + v % 10);
        v /= 10;
    }
    return d + nd;
}

// the name's first space (or -1)
__device__ __forceinline__ int first_space(const char* s, int n) {
    for (int k = 0; k < n; ++k)
        if (s[k] == ' ') return k;
    return -1;
}

__device__ __forceinline__ char comp_base(char c) {
    switch (c) {
        case 'A': case 'a': return 'T';
        case 'T': case 't': return 'A';
        case 'C': case 'c': return 'G';
        case 'G': case 'g': return 'C';
        default: return 'N';
    }
}

__device__ __forceinline__ uint32_t read_bytes(const fq_text_rec& R, const fq_read_result& r) {
    return (uint32_t)R.name_len + R.strand_len + 2u * r.len + 4u;
}

__device__ __forceinline__ bool merged_kind(const fq_read_result& a, const fq_read_result& b, int discard, bool& mrg) {
    const bool nn = !(a.flags & (FQ_RF_NULL | FQ_RF_INDEX_FILTERED)) && !(b.flags & FQ_RF_NULL);
    mrg = nn && (a.flags & FQ_RF_MERGED);
    return nn && (mrg || !discard);
}

__global__ void merge_size_kernel(const char* __restrict__ text1, const fq_text_rec* __restrict__ rec1,
                                  const fq_text_rec* __restrict__ rec2, const fq_read_result* __restrict__ res, int n,
                                  int discard, uint32_t* __restrict__ size) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const fq_read_result &a = res[2 * (size_t)i], &b = res[2 * (size_t)i + 1];
    bool mrg;
    uint32_t z = 0;
    if (merged_kind(a, b, discard, mrg)) {
        if (mrg) {
            if (a.code == FQ_PASS_FILTER) {
                const fq_text_rec R = rec1[i];
                const int m1 = a.m_len1, m2 = a.m_len2;
                const uint32_t tag = 9u + dec_digits(m1) + dec_digits(m2);
                const int sp = first_space(text1 + R.name_off, R.name_len);
                const uint32_t name = sp < 0 ? tag : (uint32_t)R.name_len - 1u + tag;
                z = name + R.strand_len + 2u * (uint32_t)(m1 + m2) + 4u;
            }
        } else {
            if (a.code == FQ_PASS_FILTER) z += read_bytes(rec1[i], a);
            if (b.code == FQ_PASS_FILTER) z += read_bytes(rec2[i], b);
        }
    }
    size[i] = z;
}

__device__ __forceinline__ char* put_read(char* d, const char* text, const fq_text_rec& R, const fq_read_result& r) {
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
    *d++ = '\n';
    return d;
}

__global__ void merge_write_kernel(const char* __restrict__ text1, const char* __restrict__ text2,
                                   const fq_text_rec* __restrict__ rec1, const fq_text_rec* __restrict__ rec2,
                                   const fq_read_result* __restrict__ res, int n, int discard,
                                   const uint32_t* __restrict__ size, const uint32_t* __restrict__ off,
                                   char* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || size[i] == 0) return;
    const fq_read_result &a = res[2 * (size_t)i], &b = res[2 * (size_t)i + 1];
    bool mrg;
    merged_kind(a, b, discard, mrg);
    char* d = out + off[i];
    const fq_text_rec R1 = rec1[i], R2 = rec2[i];
    if (!mrg) {
        if (a.code == FQ_PASS_FILTER) d = put_read(d, text1, R1, a);
        if (b.code == FQ_PASS_FILTER) put_read(d, text2, R2, b);
        return;
    }
    const int m1 = a.m_len1, m2 = a.m_len2;
    const char* nm = text1 + R1.name_off;
    const int sp = first_space(nm, R1.name_len);
    if (sp >= 0) {
        copy_bytes(d, nm, sp - 1);  // (the reference drops the byte before the space)
        d += sp - 1;
    }
    const char tag[8] = {'_', 'm', 'e', 'r', 'g', 'e', 'd', '_'};
    copy_bytes(d, tag, 8);
    d = put_dec(d + 8, m1);
    *d++ = '_';
    d = put_dec(d, m2);
    if (sp >= 0) {
        copy_bytes(d, nm + sp, R1.name_len - sp);
        d += R1.name_len - sp;
    }
    *d++ = '\n';
    // sequence: r1's window [0, m1), then r2's window [0, m2) reverse-complemented
    const char* s1 = text1 + R1.seq_off + a.start;
    const char* s2 = text2 + R2.seq_off + b.start;
    copy_bytes(d, s1, m1);
    d += m1;
    for (int j = 0; j < m2; ++j) d[j] = comp_base(s2[m2 - 1 - j]);
    d += m2;
    *d++ = '\n';
    copy_bytes(d, text1 + R1.strand_off, R1.strand_len);
    d += R1.strand_len;
    *d++ = '\n';
    const char* q1 = text1 + R1.qual_off + a.start;
    const char* q2 = text2 + R2.qual_off + b.start;
    copy_bytes(d, q1, m1);
    d += m1;
    for (int j = 0; j < m2; ++j) d[j] = q2[m2 - 1 - j];
    d += m2;
    *d = '\n';
}

}  // namespace

hipError_t fq_launch_merge_out(const char* d_text1, const char* d_text2, const fq_text_rec* d_rec1,
                               const fq_text_rec* d_rec2, const fq_read_result* d_res, int n, int discard,
                               uint32_t* d_size, uint32_t* d_off, void* d_temp, size_t temp_bytes, char* d_out,
                               unsigned long long* d_total, hipStream_t s) {
    if (n <= 0) return hipMemsetAsync(d_total, 0, sizeof(unsigned long long), s);
    const dim3 g((n + 255) / 256), b(256);
    hipLaunchKernelGGL(merge_size_kernel, g, b, 0, s, d_text1, d_rec1, d_rec2, d_res, n, discard, d_size);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t tb = temp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(d_temp, tb, d_size, d_off, n, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(text_total_kernel, dim3(1), dim3(64), 0, s, d_size, d_off, n, d_total);
    hipLaunchKernelGGL(merge_write_kernel, g, b, 0, s, d_text1, d_text2, d_rec1, d_rec2, d_res, n, discard, d_size, d_off,
                       d_out);
    return hipGetLastError();
}

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
