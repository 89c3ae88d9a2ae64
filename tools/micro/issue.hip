// Micro-benchmark (profiling aid): issue cost of the instruction patterns the fast kernels are made
// of, at 1, 2, 3 and 4 waves per SIMD (one workgroup per CU, LDS-pinned).  Each mode runs a loop of
// inline-asm blocks; the result is SIMD cycles per listed instruction:
//   kernel_s x 2.4e9 x 1024 SIMDs / (waves x iterations x instructions per iteration)
// (at the nominal clock; compare modes with each other, not with the clock).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define R8(x) x x x x x x x x

template <int MODE>
__global__ void k_issue(uint32_t* out, int iters) {
    extern __shared__ uint32_t lds[];
    const int lane = threadIdx.x & 63;
    uint32_t a = lane, b = lane + 1, c = lane + 2, d = lane + 3, e = lane + 4, f = lane + 5, g = lane + 6,
             h = lane + 7;
    uint32_t s0 = 1, s1 = 2;
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    uint32_t addr = (threadIdx.x * 8) & 1023;
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == 0) {  // 64 independent v_xor (8 chains)
            asm volatile(R8("v_xor_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n v_xor_b32 %2, %2, %8\n v_xor_b32 %3, %3, %8\n"
                            "v_xor_b32 %4, %4, %8\n v_xor_b32 %5, %5, %8\n v_xor_b32 %6, %6, %8\n v_xor_b32 %7, %7, %8\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
                         : "v"(lane));
        } else if constexpr (MODE == 1) {  // 64 dependent v_xor (one chain)
            asm volatile(R8(R8("v_xor_b32 %0, %0, %1\n")) : "+v"(a) : "v"(lane));
        } else if constexpr (MODE == 2) {  // 64 v_xor in 2 interleaved chains
            asm volatile(R8(R8("v_xor_b32 %0, %0, %2\n v_xor_b32 %1, %1, %2\n")) : "+v"(a), "+v"(b) : "v"(lane));
        } else if constexpr (MODE == 3) {  // 16 x (v_cmp -> s_cbranch_vccz) uniform branch: 32 instructions
            asm volatile(R8("v_cmp_eq_u32 vcc, %0, %1\n s_cbranch_vccz 0\n v_cmp_eq_u32 vcc, %0, %1\n s_cbranch_vccz 0\n")
                         : "+v"(a) : "v"(b) : "vcc");
        } else if constexpr (MODE == 4) {  // 16 x (v_readlane -> s_add): 32 instructions (+ hazard nops)
            asm volatile(R8("v_readlane_b32 %0, %2, 0\n s_nop 3\n s_add_u32 %1, %1, %0\n v_readlane_b32 %0, %2, 1\n s_nop 3\n s_add_u32 %1, %1, %0\n")
                         : "=&s"(s0), "+s"(s1) : "v"(a) : "scc");
        } else if constexpr (MODE == 5) {  // 8 divergent ifs: v_cmp, s_and_saveexec, 2 VALU, s_or exec = 5 each
            asm volatile(R8("v_cmp_gt_u32 vcc, 32, %2\n s_and_saveexec_b64 s[40:41], vcc\n v_xor_b32 %0, %0, %2\n v_xor_b32 %1, %1, %2\n s_or_b64 exec, exec, s[40:41]\n")
                         : "+v"(a), "+v"(b) : "v"(c) : "vcc", "s40", "s41");
        } else if constexpr (MODE == 6) {  // 16 x (ds_read_b32 -> wait -> dependent v_add): 48 instructions
            asm volatile(R8("ds_read_b32 %1, %0\n s_waitcnt lgkmcnt(0)\n v_add_u32 %0, %1, %0\n ds_read_b32 %1, %0\n s_waitcnt lgkmcnt(0)\n v_and_b32 %0, 1020, %1\n")
                         : "+v"(addr), "=&v"(b));
        } else if constexpr (MODE == 7) {  // 32 v_permlane32_swap (4 independent pairs)
            asm volatile(R8("v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %2, %3\n v_permlane32_swap_b32 %4, %5\n v_permlane32_swap_b32 %6, %7\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
        } else if constexpr (MODE == 8) {  // 48 VALU + 16 SALU, independent
            asm volatile(R8("v_xor_b32 %0, %0, %6\n v_xor_b32 %1, %1, %6\n s_add_u32 %4, %4, 3\n v_xor_b32 %2, %2, %6\n"
                            "v_xor_b32 %3, %3, %6\n s_add_u32 %5, %5, 5\n v_xor_b32 %0, %0, %6\n v_xor_b32 %1, %1, %6\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "+s"(s1)
                         : "v"(lane)
                         : "scc");
        } else if constexpr (MODE == 9) {  // 32 v_lshlrev_b64 (4 independent)
            asm volatile(R8("v_lshlrev_b64 %0, 1, %0\n v_lshlrev_b64 %1, 1, %1\n v_lshlrev_b64 %2, 1, %2\n v_lshlrev_b64 %3, 1, %3\n")
                         : "+v"(*(uint64_t*)&a), "+v"(*(uint64_t*)&c), "+v"(*(uint64_t*)&e), "+v"(*(uint64_t*)&g));
        } else if constexpr (MODE == 10) {  // 32 v_mad_u64_u32 (4 independent)
            asm volatile(R8("v_mad_u64_u32 %0, s[42:43], %4, 5, %0\n v_mad_u64_u32 %1, s[42:43], %4, 5, %1\n"
                            "v_mad_u64_u32 %2, s[42:43], %4, 5, %2\n v_mad_u64_u32 %3, s[42:43], %4, 5, %3\n")
                         : "+v"(*(uint64_t*)&a), "+v"(*(uint64_t*)&c), "+v"(*(uint64_t*)&e), "+v"(*(uint64_t*)&g)
                         : "v"(lane)
                         : "s42", "s43");
        } else if constexpr (MODE == 11) {  // 64 independent v_bcnt (accumulating, 8 chains)
            asm volatile(R8("v_bcnt_u32_b32 %0, %8, %0\n v_bcnt_u32_b32 %1, %8, %1\n v_bcnt_u32_b32 %2, %8, %2\n v_bcnt_u32_b32 %3, %8, %3\n"
                            "v_bcnt_u32_b32 %4, %8, %4\n v_bcnt_u32_b32 %5, %8, %5\n v_bcnt_u32_b32 %6, %8, %6\n v_bcnt_u32_b32 %7, %8, %7\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
                         : "v"(lane));
        } else if constexpr (MODE == 12) {  // 32 independent v_bitop3 / v_perm / v_alignbit / v_bfe (VOP3, 8 chains)
            asm volatile(R8("v_bitop3_b32 %0, %0, %8, %1 bitop3:0x96\n v_perm_b32 %1, %1, %8, %2\n v_alignbit_b32 %2, %2, %8, 3\n v_bfe_u32 %3, %3, 2, 4\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
                         : "v"(lane));
        } else if constexpr (MODE == 13) {  // 16 ds_add_u64 (distinct bank pairs) + 16 v_xor
            asm volatile(R8("ds_add_u64 %0, %2\n v_xor_b32 %1, %1, %3\n ds_add_u64 %0, %2 offset:256\n v_xor_b32 %1, %1, %3\n")
                         : "+v"(addr), "+v"(b) : "v"(*(uint64_t*)&c), "v"(lane) : "memory");
        } else if constexpr (MODE == 14) {  // 64 dependent v_xor in 2 waves' worth of... : v_sad_u8 chain (dependent)
            asm volatile(R8(R8("v_sad_u8 %0, %1, 0, %0\n")) : "+v"(a) : "v"(lane));
        } else if constexpr (MODE == 15) {  // dependent VOP3 chain (v_bitop3 64)
            asm volatile(R8(R8("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96\n")) : "+v"(a) : "v"(lane));
        }
    }
    if ((a ^ b ^ c ^ d ^ e ^ f ^ g ^ h ^ s1 ^ addr) == 0x9E3779B9u) out[blockIdx.x] = a;
}

static const int kInstr[] = {64, 64, 64, 32, 32, 40, 48, 32, 64, 32, 32, 64, 32, 32, 64, 64};
static const char* kName[] = {"v_xor independent (8 chains)",  "v_xor dependent chain",
                              "v_xor 2 chains",                "v_cmp->s_cbranch_vccz",
                              "v_readlane->s_nop3->s_add",     "divergent if (cmp,saveexec,2valu,or)",
                              "ds_read_b32->wait->v_add",      "v_permlane32_swap x4 indep",
                              "3 VALU : 1 SALU independent",   "v_lshlrev_b64 x4 indep",
                              "v_mad_u64_u32 x4 indep",        "v_bcnt indep (8 chains)",
                              "VOP3 mix bitop3/perm/align/bfe","ds_add_u64 + v_xor",
                              "v_sad_u8 dependent chain",      "v_bitop3 dependent chain"};

template <int M>
static float run(int cus, int wps, int iters, uint32_t* out) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const size_t lds = 96 * 1024;  // one workgroup per CU
    (void)hipFuncSetAttribute((const void*)k_issue<M>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_issue<M>, dim3(cus), dim3(256 * wps), lds, 0, out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    return best;
}

template <int M>
static void mode(int cus, uint32_t* out) {
    const int iters = 20000;
    printf("%-40s", kName[M]);
    for (int wps = 1; wps <= 4; ++wps) {
        const float ms = run<M>(cus, wps, iters, out);
        const double cyc = ms * 1e-3 * 2.4e9 / ((double)wps * iters * kInstr[M]);  // per SIMD
        printf("  w%d %6.2f", wps, cyc);
    }
    printf("   (SIMD cycles per instruction)\n");
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t* out;
    (void)hipMalloc(&out, 4 * 4096);
    mode<0>(cus, out);
    mode<1>(cus, out);
    mode<2>(cus, out);
    mode<3>(cus, out);
    mode<4>(cus, out);
    mode<5>(cus, out);
    mode<6>(cus, out);
    mode<7>(cus, out);
    mode<8>(cus, out);
    mode<9>(cus, out);
    mode<10>(cus, out);
    mode<11>(cus, out);
    mode<12>(cus, out);
    mode<13>(cus, out);
    mode<14>(cus, out);
    mode<15>(cus, out);
    return 0;
}
