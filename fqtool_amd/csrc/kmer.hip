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

struct fq_kmer_set {
    int device = 0;
    int32_t n = 0;
    uint8_t* seq = nullptr;
    uint32_t* off = nullptr;
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
    if (hipMalloc(&s->seq, bytes ? bytes : 1) != hipSuccess ||
        hipMalloc(&s->off, ((size_t)n + 1) * sizeof(uint32_t)) != hipSuccess) {
        fq_kmer_close(s);
        return FQ_E_NOMEM;
    }
    if ((bytes && hipMemcpy(s->seq, seq, bytes, hipMemcpyHostToDevice) != hipSuccess) ||
        (n && hipMemcpy(s->off, off, ((size_t)n + 1) * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess)) {
        fq_kmer_close(s);
        return FQ_E_HIP;
    }
    *out = s;
    return FQ_OK;
}

int fq_kmer_close(fq_kmer_set* s) {
    if (!s) return FQ_OK;
    (void)hipSetDevice(s->device);
    if (s->seq) (void)hipFree(s->seq);
    if (s->off) (void)hipFree(s->off);
    delete s;
    return FQ_OK;
}

int fq_kmer_count(fq_kmer_set* s, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t* counts) {
    if (!s || keylen < 1 || keylen > 12 || first < 0 || !counts) return FQ_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return FQ_E_HIP;
    const size_t bins = (size_t)1 << (2 * keylen);
    uint32_t* d = nullptr;
    if (hipMalloc(&d, bins * 4) != hipSuccess) return FQ_E_NOMEM;
    hipError_t e = hipMemset(d, 0, bins * 4);
    if (e == hipSuccess && s->n > 0) {
        hipLaunchKernelGGL(kmer_count_kernel, dim3((s->n + 255) / 256), dim3(256), 0, 0, s->seq, s->off, s->n, keylen,
                           first, shift_tail, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(counts, d, bins * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? FQ_OK : FQ_E_HIP;
}

int fq_kmer_find(fq_kmer_set* s, int32_t keylen, int32_t first, int32_t shift_tail, uint32_t seed, uint64_t* occ,
                 size_t cap, size_t* n_out) {
    if (!s || keylen < 1 || keylen > 12 || first < 0 || !n_out || (cap && !occ)) return FQ_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return FQ_E_HIP;
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, (cap + 1) * 8) != hipSuccess) return FQ_E_NOMEM;
    hipError_t e = hipMemset(d, 0, 8);
    if (e == hipSuccess && s->n > 0) {
        hipLaunchKernelGGL(kmer_find_kernel, dim3((s->n + 255) / 256), dim3(256), 0, 0, s->seq, s->off, s->n, keylen,
                           first, shift_tail, seed, d + 1, (unsigned long long)cap, d);
        e = hipGetLastError();
    }
    unsigned long long n = 0;
    if (e == hipSuccess) e = hipMemcpy(&n, d, 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess && n && cap) e = hipMemcpy(occ, d + 1, (size_t)std::min<unsigned long long>(n, cap) * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    *n_out = (size_t)n;
    return e == hipSuccess ? FQ_OK : FQ_E_HIP;
}

}  // extern "C"
