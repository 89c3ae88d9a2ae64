// dup.hip -- duplication analysis (-d) on gfx950: Duplicate::statRead / statPair / addRecord /
// statAll, reference src/duplicate.cpp:46-166.
//
// The reference keeps, per key (the first keylen bases of read 1 as 2-bit codes, truncated to
// 32 bits), the smallest 32-mer seen (read 2's first 32 bases in PE; bases len-37 .. len-6 in
// SE), how many reads carried that smallest 32-mer, and a GC value that is the first read's
// GC ratio (x255, rounded) while that first read's 32-mer is still the minimum, else 0.  It
// updates the table read by read in input order under a mutex.  Here one pack is processed as:
//   1. dup_reads_kernel: lane per read -> (key | invalid, 32-mer, rounded GC) from the batch rows
//      (16-byte chunk loads of the tiled planes);
//   2. a stable radix sort of the reads by key (hipCUB), so each key's reads are contiguous and
//      still in input order;
//   3. dup_walk_kernel: one lane per distinct key applies the reference's addRecord sequence to
//      that key's table entry -- no two lanes touch the same entry, so the result is exactly the
//      sequential one.  The entry also remembers the global order of its first read
//      (seq_no << 32 | index) so tables of engines that saw interleaved packs merge exactly.
// statAll is a grid-stride reduction of the table into the histogram / GC sums.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <string>
#include <vector>

#include "../../include/fqengine.h"
#include "device_ops.h"
#include "engine_internal.h"

using namespace fqdev;

struct fq_dup {
    int device = 0;
    int keylen = 12;
    uint64_t keys = 0;  // table entries: min(4^keylen, 2^32)
    // table (SoA)
    unsigned long long* kmer = nullptr;  // smallest 32-mer
    uint32_t* count = nullptr;           // reads carrying it (0 = key never seen)
    uint8_t* gc = nullptr;               // the reference's mGC
    unsigned long long* first = nullptr;  // order key of the key's first read
    // per-pack scratch
    size_t cap = 0;
    unsigned long long *skey = nullptr, *skey2 = nullptr, *rkmer = nullptr;
    uint32_t *sidx = nullptr, *sidx2 = nullptr;
    uint8_t* rgc = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    std::string err;
};

namespace {

constexpr unsigned long long kInvalid = 1ull << 32;

// Duplicate::seq2int, src/duplicate.cpp:20-44: A0 T1 C2 G3, anything else invalidates
__device__ __forceinline__ int code2(uint8_t c) {
    switch (c) {
        case 'A': return 0;
        case 'T': return 1;
        case 'C': return 2;
        case 'G': return 3;
        default: return -1;
    }
}

template <class R>
__device__ inline bool seq2int(R r, int start, int k, unsigned long long& out) {
    unsigned long long v = 0;
    for (int i = 0; i < k; ++i) {
        const int c = code2(r[start + i]);
        if (c < 0) return false;
        v = (v << 2) | (unsigned long long)c;
    }
    out = v;
    return true;
}

// C/G bases of a row (uint8 counter as in the reference), 16-byte chunk loads
__device__ inline uint32_t count_gc(Row r, int len) {
    uint32_t n = 0;
    for (int c = 0; c * 16 < len; ++c) {
        const uint4 w = *reinterpret_cast<const uint4*>(r.base + c * (FQ_TILE_READS * FQ_CHUNK));
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
        const int m = min(16, len - c * 16);
#pragma unroll
        for (int b = 0; b < 16; ++b) {
            const uint8_t ch = (uint8_t)(ws[b >> 2] >> ((b & 3) * 8));
            n += (b < m) && (ch == 'C' || ch == 'G');
        }
    }
    return n;
}

__global__ void dup_reads_kernel(fq_batch b, int paired, int keylen, unsigned long long* skey, uint32_t* sidx,
                                 unsigned long long* rkmer, uint8_t* rgc) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    sidx[i] = (uint32_t)i;
    skey[i] = kInvalid;
    const Row s1 = batch_row(b.seq1, b.stride, i);
    const int l1 = b.len1[i];
    unsigned long long key = 0, kmer = 0;
    uint32_t gcn = 0;
    int total = 0;
    if (paired) {  // Duplicate::statPair, src/duplicate.cpp:101-130
        const Row s2 = batch_row(b.seq2, b.stride, i);
        const int l2 = b.len2[i];
        if (l1 < 32 || l2 < 32) return;
        if (!seq2int(s1, 0, keylen, key) || !seq2int(s2, 0, 32, kmer)) return;
        gcn = (count_gc(s1, l1) + count_gc(s2, l2)) & 0xFF;
        total = l1 + l2;
    } else {  // Duplicate::statRead, src/duplicate.cpp:71-99
        if (l1 < 32) return;
        const int start2 = max(0, l1 - 32 - 5);
        if (!seq2int(s1, 0, keylen, key) || !seq2int(s1, start2, 32, kmer)) return;
        gcn = count_gc(s1, l1) & 0xFF;
        total = l1;
    }
    skey[i] = (unsigned long long)(uint32_t)key;  // (uint32_t)ret
    rkmer[i] = kmer;
    rgc[i] = (uint8_t)round(255.0 * (double)gcn / (double)total);
}

// Duplicate::addRecord over each key's reads in input order, src/duplicate.cpp:46-69
__global__ void dup_walk_kernel(int n, const unsigned long long* skey, const uint32_t* sidx,
                                const unsigned long long* rkmer, const uint8_t* rgc, unsigned long long order_base,
                                unsigned long long* kmer_t, uint32_t* count_t, uint8_t* gc_t,
                                unsigned long long* first_t) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const unsigned long long key = skey[j];
    if (key >= kInvalid || (j > 0 && skey[j - 1] == key)) return;
    unsigned long long mk = kmer_t[key];
    uint32_t cnt = count_t[key];
    uint8_t g = gc_t[key];
    unsigned long long fst = first_t[key];
    for (int k = j; k < n && skey[k] == key; ++k) {
        const uint32_t i = sidx[k];
        const unsigned long long km = rkmer[i];
        // the read's GC is computed only while the key is unseen (src/duplicate.cpp:88-96)
        const uint8_t gi = cnt == 0 ? rgc[i] : 0;
        if (cnt == 0) {
            cnt = 1;
            mk = km;
            g = gi;
            fst = order_base | i;
        } else if (mk == km) {
            ++cnt;
        } else if (mk > km) {
            mk = km;
            cnt = 1;
            g = gi;
        }
    }
    kmer_t[key] = mk;
    count_t[key] = cnt;
    gc_t[key] = g;
    first_t[key] = fst;
}

// dst := dst (+) src, as if src's reads had been interleaved with dst's by their order keys
__global__ void dup_merge_kernel(unsigned long long nkeys, unsigned long long* dk, uint32_t* dc, uint8_t* dg,
                                 unsigned long long* df, const unsigned long long* sk, const uint32_t* sc,
                                 const uint8_t* sg, const unsigned long long* sf) {
    for (unsigned long long key = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; key < nkeys;
         key += (unsigned long long)gridDim.x * blockDim.x) {
        const uint32_t cs = sc[key];
        if (cs == 0) continue;
        const uint32_t cd = dc[key];
        if (cd == 0) {
            dk[key] = sk[key];
            dc[key] = cs;
            dg[key] = sg[key];
            df[key] = sf[key];
            continue;
        }
        const unsigned long long m = min(dk[key], sk[key]);
        const uint32_t c = (dk[key] == m ? cd : 0) + (sk[key] == m ? cs : 0);
        // the GC is the first read's while its 32-mer is the minimum
        const bool src_first = sf[key] < df[key];
        const uint8_t g = src_first ? (sk[key] == m ? sg[key] : 0) : (dk[key] == m ? dg[key] : 0);
        dk[key] = m;
        dc[key] = c;
        dg[key] = g;
        df[key] = src_first ? sf[key] : df[key];
    }
}

// Duplicate::statAll, src/duplicate.cpp:132-166: hist[count] (count > hist_size -> the last bin;
// count == hist_size lands past the reference's array and is not reported), GC sums per bin
__global__ void dup_stat_kernel(unsigned long long nkeys, const uint32_t* count_t, const uint8_t* gc_t, int hist_size,
                                unsigned long long* hist, unsigned long long* gcsum, unsigned long long* totals) {
    extern __shared__ uint32_t sh[];  // [hist_size] counts, [hist_size] gc sums
    for (int i = threadIdx.x; i < 2 * hist_size; i += blockDim.x) sh[i] = 0;
    __syncthreads();
    unsigned long long tot = 0, dup = 0;
    for (unsigned long long key = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; key < nkeys;
         key += (unsigned long long)gridDim.x * blockDim.x) {
        const uint32_t c = count_t[key];
        if (c == 0) continue;
        tot += c;
        dup += c - 1;
        const int bin = c > (uint32_t)hist_size ? hist_size - 1 : (int)c;
        if (bin < hist_size) {
            atomicAdd(&sh[bin], 1u);
            atomicAdd(&sh[hist_size + bin], (uint32_t)gc_t[key]);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        tot += __shfl_down(tot, off);
        dup += __shfl_down(dup, off);
    }
    if ((threadIdx.x & 63) == 0) {
        if (tot) atomicAdd(&totals[0], tot);
        if (dup) atomicAdd(&totals[1], dup);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < hist_size; i += blockDim.x) {
        if (sh[i]) atomicAdd(&hist[i], (unsigned long long)sh[i]);
        if (sh[hist_size + i]) atomicAdd(&gcsum[i], (unsigned long long)sh[hist_size + i]);
    }
}

int dup_fail(fq_dup* d, hipError_t e, const char* what) {
    d->err = std::string(what) + ": " + hipGetErrorString(e);
    return FQ_E_HIP;
}

#define DUP_TRY(d, call)                                        \
    do {                                                        \
        hipError_t _e = (call);                                 \
        if (_e != hipSuccess) return dup_fail(d, _e, #call);    \
    } while (0)

int ensure_cap(fq_dup* d, size_t n, hipStream_t s) {
    if (n <= d->cap) return FQ_OK;
    DUP_TRY(d, hipStreamSynchronize(s));
    for (void* p : {(void*)d->skey, (void*)d->skey2, (void*)d->rkmer, (void*)d->sidx, (void*)d->sidx2, (void*)d->rgc,
                    d->tmp})
        if (p) (void)hipFree(p);
    d->skey = d->skey2 = d->rkmer = nullptr;
    d->sidx = d->sidx2 = nullptr;
    d->rgc = nullptr;
    d->tmp = nullptr;
    d->cap = 0;
    const size_t cap = n < 4096 ? 4096 : n;
    DUP_TRY(d, hipMalloc(&d->skey, cap * 8));
    DUP_TRY(d, hipMalloc(&d->skey2, cap * 8));
    DUP_TRY(d, hipMalloc(&d->rkmer, cap * 8));
    DUP_TRY(d, hipMalloc(&d->sidx, cap * 4));
    DUP_TRY(d, hipMalloc(&d->sidx2, cap * 4));
    DUP_TRY(d, hipMalloc(&d->rgc, cap));
    d->tmp_bytes = 0;
    DUP_TRY(d, hipcub::DeviceRadixSort::SortPairs(nullptr, d->tmp_bytes, d->skey, d->skey2, d->sidx, d->sidx2, (int)cap,
                                                  0, 33, s));
    DUP_TRY(d, hipMalloc(&d->tmp, d->tmp_bytes ? d->tmp_bytes : 1));
    d->cap = cap;
    return FQ_OK;
}

}  // namespace

int fq_dup_pack(fq_dup* d, const fq_batch& b, int paired, unsigned long long order_base, hipStream_t s) {
    if (b.n <= 0) return FQ_OK;
    int rc = ensure_cap(d, (size_t)b.n, s);
    if (rc != FQ_OK) return rc;
    const int grid = (b.n + 255) / 256;
    hipLaunchKernelGGL(dup_reads_kernel, dim3(grid), dim3(256), 0, s, b, paired, d->keylen, d->skey, d->sidx, d->rkmer,
                       d->rgc);
    DUP_TRY(d, hipGetLastError());
    size_t tb = d->tmp_bytes;
    DUP_TRY(d, hipcub::DeviceRadixSort::SortPairs(d->tmp, tb, d->skey, d->skey2, d->sidx, d->sidx2, b.n, 0, 33, s));
    hipLaunchKernelGGL(dup_walk_kernel, dim3(grid), dim3(256), 0, s, b.n, d->skey2, d->sidx2, d->rkmer, d->rgc,
                       order_base << 32, d->kmer, d->count, d->gc, d->first);
    DUP_TRY(d, hipGetLastError());
    return FQ_OK;
}

const char* fq_dup_error(const fq_dup* d) { return d ? d->err.c_str() : ""; }

int fq_dup_device(const fq_dup* d, int* device) {
    if (!d || !device) return FQ_E_INVALID;
    *device = d->device;
    return FQ_OK;
}

extern "C" {

int fq_dup_create(int device, int32_t keylen, fq_dup** out) {
    if (!out || keylen < 1 || keylen > 31) return FQ_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return FQ_E_NO_DEVICE;
    fq_dup* d = new fq_dup();
    d->device = device;
    d->keylen = keylen;
    // keys are truncated to 32 bits (src/duplicate.cpp:79), so 2^32 entries cover keylen > 16
    d->keys = keylen >= 16 ? (1ull << 32) : (1ull << (2 * keylen));
    auto bail = [&](int rc) {
        fq_dup_destroy(d);
        return rc;
    };
    if (hipSetDevice(device) != hipSuccess) return bail(FQ_E_HIP);
    if (hipMalloc(&d->kmer, d->keys * 8) != hipSuccess || hipMalloc(&d->count, d->keys * 4) != hipSuccess ||
        hipMalloc(&d->gc, d->keys) != hipSuccess || hipMalloc(&d->first, d->keys * 8) != hipSuccess)
        return bail(FQ_E_NOMEM);
    if (fq_dup_reset(d) != FQ_OK) return bail(FQ_E_HIP);
    *out = d;
    return FQ_OK;
}

int fq_dup_destroy(fq_dup* d) {
    if (!d) return FQ_OK;
    (void)hipSetDevice(d->device);
    (void)hipDeviceSynchronize();
    for (void* p : {(void*)d->kmer, (void*)d->count, (void*)d->gc, (void*)d->first, (void*)d->skey, (void*)d->skey2,
                    (void*)d->rkmer, (void*)d->sidx, (void*)d->sidx2, (void*)d->rgc, d->tmp})
        if (p) (void)hipFree(p);
    delete d;
    return FQ_OK;
}

int fq_dup_reset(fq_dup* d) {
    if (!d) return FQ_E_INVALID;
    DUP_TRY(d, hipSetDevice(d->device));
    DUP_TRY(d, hipMemset(d->count, 0, d->keys * 4));
    DUP_TRY(d, hipMemset(d->kmer, 0, d->keys * 8));
    DUP_TRY(d, hipMemset(d->gc, 0, d->keys));
    DUP_TRY(d, hipMemset(d->first, 0, d->keys * 8));
    DUP_TRY(d, hipDeviceSynchronize());
    return FQ_OK;
}

int fq_dup_merge(fq_dup* dst, const fq_dup* src) {
    if (!dst || !src || dst->keys != src->keys) return FQ_E_INVALID;
    DUP_TRY(dst, hipSetDevice(src->device));
    DUP_TRY(dst, hipDeviceSynchronize());
    DUP_TRY(dst, hipSetDevice(dst->device));
    DUP_TRY(dst, hipDeviceSynchronize());
    const unsigned long long* sk = src->kmer;
    const uint32_t* sc = src->count;
    const uint8_t* sg = src->gc;
    const unsigned long long* sf = src->first;
    void* stage[4] = {nullptr, nullptr, nullptr, nullptr};
    if (src->device != dst->device) {  // bring the source table over (peer copy, or staged by the runtime)
        const size_t bytes[4] = {src->keys * 8, src->keys * 4, src->keys, src->keys * 8};
        const void* from[4] = {src->kmer, src->count, src->gc, src->first};
        for (int k = 0; k < 4; ++k) {
            if (hipMalloc(&stage[k], bytes[k]) != hipSuccess) {
                for (void* p : stage)
                    if (p) (void)hipFree(p);
                return FQ_E_NOMEM;
            }
            DUP_TRY(dst, hipMemcpyPeer(stage[k], dst->device, from[k], src->device, bytes[k]));
        }
        sk = (const unsigned long long*)stage[0];
        sc = (const uint32_t*)stage[1];
        sg = (const uint8_t*)stage[2];
        sf = (const unsigned long long*)stage[3];
    }
    hipLaunchKernelGGL(dup_merge_kernel, dim3(4096), dim3(256), 0, 0, dst->keys, dst->kmer, dst->count, dst->gc,
                       dst->first, sk, sc, sg, sf);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    for (void* p : stage)
        if (p) (void)hipFree(p);
    if (e != hipSuccess) return dup_fail(dst, e, "dup_merge_kernel");
    return FQ_OK;
}

int fq_dup_stat(fq_dup* d, int32_t hist_size, uint64_t* hist, uint64_t* gc_sum, uint64_t* totals) {
    if (!d || hist_size < 1 || hist_size > 16384 || !hist || !gc_sum || !totals) return FQ_E_INVALID;
    DUP_TRY(d, hipSetDevice(d->device));
    unsigned long long* buf = nullptr;
    const size_t words = 2 * (size_t)hist_size + 2;
    DUP_TRY(d, hipMalloc(&buf, words * 8));
    hipError_t e = hipMemset(buf, 0, words * 8);
    const size_t lds = 2 * (size_t)hist_size * 4;
    if (e == hipSuccess && lds > 64 * 1024)
        e = hipFuncSetAttribute((const void*)dup_stat_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(dup_stat_kernel, dim3(2048), dim3(256), lds, 0, d->keys, d->count, d->gc, hist_size, buf,
                           buf + hist_size, buf + 2 * hist_size);
        e = hipGetLastError();
    }
    std::vector<unsigned long long> h(words);
    if (e == hipSuccess) e = hipMemcpy(h.data(), buf, words * 8, hipMemcpyDeviceToHost);
    (void)hipFree(buf);
    if (e != hipSuccess) return dup_fail(d, e, "dup_stat_kernel");
    for (int i = 0; i < hist_size; ++i) {
        hist[i] = h[(size_t)i];
        gc_sum[i] = h[(size_t)hist_size + i];
    }
    totals[0] = h[2 * (size_t)hist_size];
    totals[1] = h[2 * (size_t)hist_size + 1];
    return FQ_OK;
}

}  // extern "C"
