// kmer.hip -- the k-mer work of the adapter-detection pre-pass on gfx950:
// Evaluator::evaluateAdapterSeq's 10-mer histogram and getAdapterWithSeed's seed search
// (reference src/evaluator.cpp:265-279 and :392-405).
//
// The reads (<= 256 Ki per mate) are uploaded once as one byte array + offsets.  Lane per read,
// a rolling 2-bit key and a run length of valid (uppercase ACGT) bases give every window's key
// without recomputing it (Evaluator::seq2int's incremental form yields exactly the key of every
// all-valid window); windows start at `first` and end keylen + shift_tail bases before the read's
// end.  Counting is a global-atomic histogram over 4^keylen bins; the seed search appends
// (read << 32 | pos) to a list whose order the host's prefix trees do not depend on.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/fqengine.h"

// All the set's work runs on its own non-blocking stream, with buffers allocated once and kept
// (hipFree synchronises the device, and the legacy default stream serialises with the engines'
// streams: either would tie the pre-pass to the pipeline's kernels running beside it).
struct fq_kmer_set {
    int device = 0;
    int32_t n = 0;
    uint8_t* seq = nullptr;
    uint32_t* off = nullptr;
    hipStream_t stream = nullptr;
    uint32_t* counts = nullptr;  // 4^keylen bins (grown on demand)
    size_t counts_bins = 0;
    unsigned long long* occ = nullptr;  // [count, occurrences...] (grown on demand)
    size_t occ_cap = 0;
};

namespace {

__device__ __forceinline__ int code2(uint8_t c) {
    return c == 'A' ? 0 : c == 'T' ? 1 : c == 'C' ? 2 : c == 'G' ? 3 : -1;
}

// calls visit(pos, key) for every all-valid window [pos, pos + k) with first <= pos <= len - k - tail
template <class F>
__device__ inline void windows(const uint8_t* s, int len, int k, int first, int tail, F visit) {
    const int last = len - k - tail;
    if (last < first) return;
    const uint32_t mask = (k >= 16) ? 0xFFFFFFFFu : ((1u << (2 * k)) - 1u);
    uint32_t key = 0;
    int run = 0;
    for (int i = first; i < last + k; ++i) {
        const int b = code2(s[i]);
        run = b < 0 ? 0 : run + 1;
        key = ((key << 2) | (uint32_t)(b & 3)) & mask;
        if (run >= k) visit(i - k + 1, key);
    }
}

__global__ void kmer_count_kernel(const uint8_t* seq, const uint32_t* off, int n, int k, int first, int tail,
                                  uint32_t* counts) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint8_t* s = seq + off[r];
    windows(s, (int)(off[r + 1] - off[r]), k, first, tail, [&](int, uint32_t key) { atomicAdd(&counts[key], 1u); });
}

__global__ void kmer_find_kernel(const uint8_t* seq, const uint32_t* off, int n, int k, int first, int tail,
                                 uint32_t seed, unsigned long long* occ, unsigned long long cap,
                                 unsigned long long* nocc) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint8_t* s = seq + off[r];
    windows(s, (int)(off[r + 1] - off[r]), k, first, tail, [&](int pos, uint32_t key) {
        if (key != seed) return;
        const unsigned long long slot = atomicAdd(nocc, 1ull);
        if (slot < cap) occ[slot] = ((unsigned long long)r << 32) | (unsigned)pos;
    });
}

}  // namespace

extern "C" {

int fq_kmer_open(int device, const uint8_t* seq, const uint32_t* off, int32_t n, fq_kmer_set** out) {
    if (!out || n < 0 || (n > 0 && (!seq || !off))) return FQ_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return FQ_E_NO_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return FQ_E_HIP;
    fq_kmer_set* s = new fq_kmer_set();
    s->device = device;
    s->n = n;
    const size_t bytes = n ? off[n] : 0;
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
        fq_kmer_close(s);
        return FQ_E_HIP;
    }
    if (hipMalloc(&s->seq, bytes ? bytes : 1) != hipSuccess ||
        hipMalloc(&s->off, ((size_t)n + 1) * sizeof(uint32_t)) != hipSuccess) {
        fq_kmer_close(s);
        return FQ_E_NOMEM;
    }
    if ((bytes && hipMemcpyAsync(s->seq, seq, bytes, hipMemcpyHostToDevice, s->stream) != hipSuccess) ||
        (n && hipMemcpyAsync(s->off, off, ((size_t)n + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, s->stream) != hipSuccess) ||
        hipStreamSynchronize(s->stream) != hipSuccess) {
        fq_kmer_close(s);
        return FQ_E_HIP;
    }
    *out = s;
    return FQ_OK;
}

int fq_kmer_close(fq_kmer_set* s) {
    if (!s) return FQ_OK;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->seq) (void)hipFree(s->seq);
    if (s->off) (void)hipFree(s->off);
    if (s->counts) (void)hipFree(s->counts);
    if (s->occ) (void)hipFree(s->occ);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return FQ_OK;
}

int fq_kmer_count(fq_kmer_set* s, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t* counts) {
    if (!s || keylen < 1 || keylen > 12 || first < 0 || !counts) return FQ_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return FQ_E_HIP;
    const size_t bins = (size_t)1 << (2 * keylen);
    if (bins > s->counts_bins) {
        if (s->counts) (void)hipFree(s->counts);
        s->counts = nullptr;
        s->counts_bins = 0;
        if (hipMalloc(&s->counts, bins * 4) != hipSuccess) return FQ_E_NOMEM;
        s->counts_bins = bins;
    }
    hipError_t e = hipMemsetAsync(s->counts, 0, bins * 4, s->stream);
    if (e == hipSuccess && s->n > 0) {
        hipLaunchKernelGGL(kmer_count_kernel, dim3((s->n + 255) / 256), dim3(256), 0, s->stream, s->seq, s->off, s->n,
                           keylen, first, shift_tail, s->counts);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(counts, s->counts, bins * 4, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    return e == hipSuccess ? FQ_OK : FQ_E_HIP;
}

int fq_kmer_find(fq_kmer_set* s, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t seed, uint64_t* occ,
                 size_t cap, size_t* n_out) {
    if (!s || keylen < 1 || keylen > 12 || first < 0 || !n_out || (cap && !occ)) return FQ_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return FQ_E_HIP;
    if (cap + 1 > s->occ_cap) {
        if (s->occ) (void)hipFree(s->occ);
        s->occ = nullptr;
        s->occ_cap = 0;
        if (hipMalloc(&s->occ, (cap + 1) * 8) != hipSuccess) return FQ_E_NOMEM;
        s->occ_cap = cap + 1;
    }
    unsigned long long* d = s->occ;
    hipError_t e = hipMemsetAsync(d, 0, 8, s->stream);
    if (e == hipSuccess && s->n > 0) {
        hipLaunchKernelGGL(kmer_find_kernel, dim3((s->n + 255) / 256), dim3(256), 0, s->stream, s->seq, s->off, s->n,
                           keylen, first, shift_tail, seed, d + 1, (unsigned long long)cap, d);
        e = hipGetLastError();
    }
    unsigned long long n = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&n, d, 8, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (e == hipSuccess && n && cap) {
        e = hipMemcpyAsync(occ, d + 1, (size_t)std::min<unsigned long long>(n, cap) * 8, hipMemcpyDeviceToHost, s->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    }
    *n_out = (size_t)n;
    return e == hipSuccess ? FQ_OK : FQ_E_HIP;
}

}  // extern "C"
