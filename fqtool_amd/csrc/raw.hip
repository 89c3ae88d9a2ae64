// raw.hip -- record indexing of raw FASTQ bytes on the GPU (fq_engine_raw_*, include/fqengine.h).
//
// Replaces FqReader::read / FqReaderPair::read (src/fqreader.cpp:90-195, :254-267) for the plain
// part of an input.  Per mate and window, in a device buffer laid out as
//     [ ... | carry (bytes after the previous pack's last record) | raw window bytes | slack ]
//                ^ text_start          carry_cap ^
// the kernels
//   raw_carry_kernel    copy the previous window's unconsumed bytes in front of the new ones;
//   raw_count_kernel    count the line terminators ('\n' and '\r', as the host reader's bitmap)
//                       of every 4 KiB block;
//   (hipcub scan)       block bases of the line index;
//   raw_lines_kernel    write every terminator's buffer offset into the line index;
//   raw_records_kernel  cut record i from lines 4i .. 4i+3 (the window starts at a record) and
//                       test it "plain" (every line ends in '\n' and is non-empty, the first
//                       starts with '@', quality and sequence lengths agree, fields fit the
//                       engine): on plain records FqReader::read is four lines per record;
//   raw_pair_kernel     pairs = min over the mates of the leading plain records, bytes consumed.
// The pack's records then go through the text-pack path (text.hip) unchanged.  Byte-parallel
// work in 16-byte aligned loads; the record cut is lane per record.
#include <hip/hip_runtime.h>

#include <climits>

#include <hipcub/hipcub.hpp>

#include "engine_internal.h"

namespace {

constexpr int kBlk = 4096;  // bytes per count / lines block (256 threads x 16 bytes)

__device__ __forceinline__ uint32_t term_mask16(uint4 v) {
    uint32_t m = 0;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t c = (w[k] >> (8 * b)) & 0xFF;
            m |= (uint32_t)(c == '\n' || c == '\r') << (4 * k + b);
        }
    return m;
}

// terminators of the 16 bytes at buffer offset o that lie in [lo, hi)
__device__ __forceinline__ uint32_t block_mask(const char* buf, uint32_t o, uint32_t lo, uint32_t hi) {
    if (o + 16 <= lo || o >= hi) return 0;
    uint32_t m = term_mask16(*reinterpret_cast<const uint4*>(buf + o));
    if (o < lo) m &= ~0u << (lo - o);
    if (o + 16 > hi) m &= (1u << (hi - o)) - 1u;
    return m;
}

__global__ void raw_carry_kernel(fq_raw_text_args a) {
    const int m = blockIdx.y;
    const fq_raw_state* ps = a.prev_state ? a.prev_state + m : nullptr;
    uint32_t carry = ps ? ps->avail - ps->consumed : 0u;
    const bool over = carry > a.carry_cap || (ps && ps->overflow);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // (an overflow indexes nothing: the host resumes before the carried bytes)
        fq_raw_state& s = a.state[m];
        s.text_start = a.carry_cap - (over ? 0u : carry);
        s.carry_in = carry;
        s.avail = over ? 0u : carry + a.raw_bytes[m];
        s.overflow = over ? 1u : 0u;
        s.first_bad = INT_MAX;
        s.complete = 0;
        s.max_len = 0;
        s.total_lines = 0;
        s.consumed = 0;
        s.n = 0;
    }
    if (!ps || !carry || over) return;
    const char* src = a.prev_text[m] + ps->text_start + ps->consumed;
    char* dst = a.text[m] + (a.carry_cap - carry);
    for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) * 16u; i < carry; i += gridDim.x * blockDim.x * 16u) {
        const uint32_t k = min(16u, carry - i);
        for (uint32_t b = 0; b < k; ++b) dst[i + b] = src[i + b];
    }
}

__device__ __forceinline__ uint32_t block_sum_u32(uint32_t v, uint32_t* sh) {
    // 256 threads = 4 waves of 64
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    return sh[0] + sh[1] + sh[2] + sh[3];
}

__global__ __launch_bounds__(256) void raw_count_kernel(fq_raw_text_args a) {
    const int m = blockIdx.y;
    __shared__ uint32_t sh[4];
    const fq_raw_state& s = a.state[m];
    const uint32_t lo = s.text_start, hi = s.text_start + s.avail;
    const uint32_t o = blockIdx.x * kBlk + threadIdx.x * 16u;
    const uint32_t c = (uint32_t)__popc(block_mask(a.text[m], o, lo, hi));
    const uint32_t t = block_sum_u32(c, sh);
    if (threadIdx.x == 0) a.bcnt[m][blockIdx.x] = t;
}

__global__ __launch_bounds__(256) void raw_lines_kernel(fq_raw_text_args a) {
    const int m = blockIdx.y;
    __shared__ uint32_t sh[4];
    const fq_raw_state& s = a.state[m];
    const uint32_t lo = s.text_start, hi = s.text_start + s.avail;
    const uint32_t o = blockIdx.x * kBlk + threadIdx.x * 16u;
    uint32_t mk = block_mask(a.text[m], o, lo, hi);
    // exclusive prefix of the terminator counts over the block's 256 threads
    const uint32_t c = (uint32_t)__popc(mk);
    uint32_t incl = c;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) sh[w] = incl;
    __syncthreads();
    uint32_t base = a.bbase[m][blockIdx.x];
    for (int k = 0; k < w; ++k) base += sh[k];
    uint32_t idx = base + incl - c;
    uint32_t* lines = a.lines[m];
    while (mk) {
        const int b = __ffs(mk) - 1;
        mk &= mk - 1;
        if (idx < a.cap_lines) lines[idx] = o + (uint32_t)b;
        ++idx;
    }
}

__global__ __launch_bounds__(256) void raw_records_kernel(fq_raw_text_args a) {
    const int m = blockIdx.y;
    fq_raw_state& s = a.state[m];
    const uint32_t nb = a.nblocks;
    uint32_t total = a.bbase[m][nb - 1] + a.bcnt[m][nb - 1];
    if (total > a.cap_lines) total = a.cap_lines;
    int complete = (int)(total / 4u);
    if (complete > a.cap_records) complete = a.cap_records;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        s.total_lines = total;
        s.complete = complete;
    }
    if (i >= complete) return;
    const uint32_t* L = a.lines[m];
    const char* t = a.text[m];
    const uint32_t x = i ? L[4 * i - 1] + 1u : s.text_start;
    const uint32_t t0 = L[4 * i], t1 = L[4 * i + 1], t2 = L[4 * i + 2], t3 = L[4 * i + 3];
    const uint32_t name_len = t0 - x, len = t1 - t0 - 1u, strand_len = t2 - t1 - 1u;
    const bool plain = t0 > x && t1 > t0 + 1u && t2 > t1 + 1u && t3 > t2 + 1u && t[x] == '@' && t[t0] == '\n' &&
                       t[t1] == '\n' && t[t2] == '\n' && t[t3] == '\n' && t3 - t2 == t1 - t0 && name_len <= 65535u &&
                       strand_len <= 65535u && len <= (uint32_t)a.max_len;
    if (!plain) {
        atomicMin(&s.first_bad, i);
        return;
    }
    fq_text_rec r;
    r.name_off = x;
    r.seq_off = t0 + 1u;
    r.strand_off = t1 + 1u;
    r.qual_off = t2 + 1u;
    r.name_len = (uint16_t)name_len;
    r.strand_len = (uint16_t)strand_len;
    r.len = (uint16_t)len;
    r.pad = 0;
    a.rec[m][i] = r;
    atomicMax(&s.max_len, (int)len);
}

__global__ void raw_pair_kernel(fq_raw_text_args a, int mates, int cap_batch) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int n = cap_batch;
    for (int m = 0; m < mates; ++m) {
        const fq_raw_state& s = a.state[m];
        const int c = s.overflow ? 0 : min(s.first_bad, s.complete);
        n = min(n, c);
    }
    for (int m = 0; m < mates; ++m) {
        fq_raw_state& s = a.state[m];
        s.n = n;
        s.consumed = n ? a.lines[m][4 * n - 1] + 1u - s.text_start : 0u;
    }
}

// trimmed-adapter entries of mate m (FilterResult::addAdapterTrimmed's strings): per read with an
// adapter, "u16 ad_len, u8 neg, then ad_len bytes of the read (neg = 0) or u16 ad_pos (neg = 1:
// the string is the adapter parameter's [ad_pos, ad_pos + ad_len))"
__device__ __forceinline__ uint32_t ad_entry_bytes(const fq_read_result& r) {
    if (!(r.flags & (FQ_RF_AD_OVERLAP | FQ_RF_AD_SEQ)) || r.ad_len == 0) return 0u;
    return (r.flags & FQ_RF_AD_NEG) ? 5u : 3u + r.ad_len;
}

__global__ void raw_ad_size_kernel(const fq_read_result* __restrict__ res, int n, int paired, int m, uint32_t* __restrict__ size) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    size[i] = ad_entry_bytes(res[paired ? 2 * (size_t)i + m : (size_t)i]);
}

__global__ void raw_ad_write_kernel(const char* __restrict__ text, const fq_text_rec* __restrict__ rec,
                                    const fq_read_result* __restrict__ res, int n, int paired, int m,
                                    const uint32_t* __restrict__ size, const uint32_t* __restrict__ off,
                                    char* __restrict__ out, const unsigned long long* __restrict__ text_total,
                                    unsigned long long cap, unsigned long long* __restrict__ total) {
    // the entries follow the pack's output text in the same buffer (copied back with it); they
    // fit: per record, output + entry <= input + 3 bytes, and the copy spans input + 3n + 16
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long base = *text_total;
    const unsigned long long end = base + (unsigned long long)off[n - 1] + size[n - 1];
    if (i == n - 1) *total = end <= cap ? end - base : ~0ull;
    if (i >= n || size[i] == 0 || end > cap) return;
    const fq_read_result& r = res[paired ? 2 * (size_t)i + m : (size_t)i];
    char* d = out + base + off[i];
    d[0] = (char)(r.ad_len & 0xFF);
    d[1] = (char)(r.ad_len >> 8);
    if (r.flags & FQ_RF_AD_NEG) {
        d[2] = 1;
        d[3] = (char)(r.ad_pos & 0xFF);
        d[4] = (char)(r.ad_pos >> 8);
        return;
    }
    d[2] = 0;
    const char* s = text + rec[i].seq_off + r.ad_pos;
    for (int b = 0; b < r.ad_len; ++b) d[3 + b] = s[b];
}

}  // namespace

size_t fq_raw_scan_temp_bytes(int nblocks, int n) {
    size_t a = 0, b = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, a, (const uint32_t*)nullptr, (uint32_t*)nullptr, nblocks);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr, n);
    return a > b ? a : b;
}

hipError_t fq_launch_raw_index(const fq_raw_text_args& a, int mates, int cap_batch, void* d_temp, size_t temp_bytes,
                               hipStream_t s) {
    const dim3 b(256);
    hipLaunchKernelGGL(raw_carry_kernel, dim3(64, mates), b, 0, s, a);
    hipLaunchKernelGGL(raw_count_kernel, dim3(a.nblocks, mates), b, 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    for (int m = 0; m < mates; ++m) {
        size_t tb = temp_bytes;
        e = hipcub::DeviceScan::ExclusiveSum(d_temp, tb, a.bcnt[m], a.bbase[m], (int)a.nblocks, s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(raw_lines_kernel, dim3(a.nblocks, mates), b, 0, s, a);
    hipLaunchKernelGGL(raw_records_kernel, dim3((a.cap_records + 255) / 256, mates), b, 0, s, a);
    hipLaunchKernelGGL(raw_pair_kernel, dim3(1), dim3(64), 0, s, a, mates, cap_batch);
    return hipGetLastError();
}

hipError_t fq_launch_raw_adapters(const char* d_text, const fq_text_rec* d_rec, const fq_read_result* d_res, int n,
                                  int paired, int m, uint32_t* d_size, uint32_t* d_off, void* d_temp, size_t temp_bytes,
                                  char* d_out, const unsigned long long* d_text_total, unsigned long long cap,
                                  unsigned long long* d_total, hipStream_t s) {
    if (n <= 0) return hipMemsetAsync(d_total, 0, sizeof(unsigned long long), s);
    const dim3 g((n + 255) / 256), b(256);
    hipLaunchKernelGGL(raw_ad_size_kernel, g, b, 0, s, d_res, n, paired, m, d_size);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t tb = temp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(d_temp, tb, d_size, d_off, n, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(raw_ad_write_kernel, g, b, 0, s, d_text, d_rec, d_res, n, paired, m, d_size, d_off, d_out,
                       d_text_total, cap, d_total);
    return hipGetLastError();
}
