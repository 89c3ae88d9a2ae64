// synth.hip -- seeded synthetic 150 bp workload generated directly in HBM.
//
// Counter-based: every pair derives its draws from splitmix64(seed ^ index * K), so any shard of
// the 100 M / 1 B pair configs is generated independently on its own GPU.  Integer-only, so the
// host twin used by the tests produces the same bytes.  One thread per (pair, mate) row; each
// thread packs its bases into dwords and stores whole dwords.
#include <hip/hip_runtime.h>

#include "engine_internal.h"

namespace {

__device__ __forceinline__ uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ uint8_t acgt(uint64_t v) {
    const uint32_t packed = 'A' | ('C' << 8) | ('G' << 16) | ('T' << 24);
    return (uint8_t)(packed >> (8 * (v & 3)));
}

__device__ __forceinline__ uint8_t syn_comp(uint8_t c) {
    return c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : c == 'T' ? 'A' : 'N';
}

__constant__ char kAd[2][34] = {"AGATCGGAAGAGCACACGTCTGAACTCCAGTCA", "AGATCGGAAGAGCGTCGTGTAGGGAAAGAGTGT"};

__global__ void synth_kernel(fq_batch b, uint64_t seed, uint64_t first, int L) {
    const int mates = b.seq2 ? 2 : 1;
    const long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= (long long)b.n * mates) return;
    const int pair = (int)(row / mates);
    const int mate = (int)(row - (long long)pair * mates);
    const uint64_t key = sm64(seed ^ ((first + (uint64_t)pair) * 0xD1B54A32D192ED03ull));
    const uint64_t r0 = sm64(key + 1);
    long long S = (long long)(r0 & 0xFFFF) + (long long)((r0 >> 16) & 0xFFFF) + (long long)((r0 >> 32) & 0xFFFF) +
                  (long long)((r0 >> 48) & 0xFFFF);
    long long ins = 220 + (S - 131070) * 60 / 37837;
    ins = ins < 60 ? 60 : ins > 600 ? 600 : ins;
    const uint64_t rm = sm64(key + 2 + (uint64_t)mate);
    const int polyg = ((rm & 0xFFFF) % 100 < 5) ? 10 + (int)(((rm >> 16) & 0xFFFF) % 51) : 0;
    const int lowq = (((rm >> 32) & 0xFFFF) % 100 < 2) ? 100 + (int)((rm >> 48) % 51) : L;
    // the read's chunk 0 in the chunk-interleaved batch tiles; byte i at (i / 16) * 512 + i % 16
    const size_t roff = (size_t)(pair / FQ_TILE_READS) * FQ_TILE_READS * b.stride + (pair % FQ_TILE_READS) * FQ_CHUNK;
    uint8_t* seq = (uint8_t*)(mate ? b.seq2 : b.seq1) + roff;
    uint8_t* qual = (uint8_t*)(mate ? b.qual2 : b.qual1) + roff;
    uint32_t sw = 0, qw = 0;
    for (int i = 0; i < L; ++i) {
        uint8_t base;
        if (i < ins) {
            const int k = mate ? (int)ins - 1 - i : i;
            const uint8_t f = acgt(sm64((key ^ 0x5BD1E9955BD1E995ull) + (uint64_t)k));
            base = mate ? syn_comp(f) : f;
        } else {
            const int j = i - (int)ins;
            base = j < 33 ? (uint8_t)kAd[mate][j] : (uint8_t)'G';
        }
        if (i >= L - polyg) base = 'G';
        const uint64_t hm = sm64((key ^ (0xA5A5A5A5A5A5A5A5ull * (uint64_t)(2 + mate))) + (uint64_t)i);
        if ((hm & 0x3FF) < 1) {
            base = 'N';
        } else if (((hm >> 10) & 0x3FF) < 3) {
            const int idx = base == 'A' ? 0 : base == 'C' ? 1 : base == 'G' ? 2 : 3;
            base = acgt((uint64_t)(idx + 1 + (int)((hm >> 20) % 3)));
        }
        const int n = (int)((hm >> 24) & 0xFF) + (int)((hm >> 32) & 0xFF) + (int)((hm >> 40) & 0xFF) - 382;
        int q = (3600 - 6 * i + n * 300 / 128) / 100;
        q = q < 2 ? 2 : q > 41 ? 41 : q;
        if (i >= lowq) q = 2 + (int)((hm >> 48) % 11);
        if (base == 'N') q = 2;
        sw |= (uint32_t)base << (8 * (i & 3));
        qw |= (uint32_t)(q + 33) << (8 * (i & 3));
        if ((i & 3) == 3 || i == L - 1) {
            const size_t o = (size_t)(i >> 4) * (FQ_TILE_READS * FQ_CHUNK) + (i & 12);
            *reinterpret_cast<uint32_t*>(seq + o) = sw;
            *reinterpret_cast<uint32_t*>(qual + o) = qw;
            sw = qw = 0;
        }
    }
    uint16_t* len = (uint16_t*)(mate ? b.len2 : b.len1);
    len[pair] = (uint16_t)L;
}

}  // namespace

hipError_t fq_launch_synth(const fq_batch& b, uint64_t seed, uint64_t first_index, int read_len, hipStream_t stream) {
    const long long rows = (long long)b.n * (b.seq2 ? 2 : 1);
    const int block = 256;
    const long long grid = (rows + block - 1) / block;
    if (grid <= 0) return hipSuccess;
    hipLaunchKernelGGL(synth_kernel, dim3((unsigned)grid), dim3(block), 0, stream, b, seed, first_index, read_len);
    return hipGetLastError();
}
