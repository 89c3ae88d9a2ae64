// profiling aid (round 4): issue cost of the select / compare / shift idioms the compiler emits on
// gfx950 -- v_cndmask reading VCC vs an SGPR pair vs a bitop3 select on a VGPR mask, VOP3 operands
// from SGPRs vs VGPRs, 32-bit left shifts as v_lshlrev_b64.  8 independent chains, 16 waves per CU.
// hipcc -O3 --offload-arch=gfx950 tools/micro/sel.hip -o build/micro/sel
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#define R4(x) x x x x
#define C8(f) f("%0") f("%1") f("%2") f("%3") f("%4") f("%5") f("%6") f("%7")
#define OUTS "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
// pattern bodies (one chain step each; %8, %9 = VGPR inputs, %10 = VGPR constant)
#define P_CMP_VCC(r) "v_cmp_gt_u32_e32 vcc, %8, " r "\n s_nop 1\n v_cndmask_b32_e32 " r ", %9, " r ", vcc\n "
#define P_CMP_SGPR(r) "v_cmp_gt_u32_e64 s[44:45], %8, " r "\n s_nop 1\n v_cndmask_b32_e64 " r ", %9, " r ", s[44:45]\n "
#define P_SUB_ASHR_BITOP3(r) "v_sub_u32_e32 %14, %8, " r "\n v_ashrrev_i32_e32 %14, 31, %14\n v_bitop3_b32 " r ", %9, " r ", %14 bitop3:0xd8\n "
#define P_CND_VCC_ONLY(r) "v_cndmask_b32_e32 " r ", %9, " r ", vcc\n "
#define P_CND_VCC_7XOR(r) "v_cndmask_b32_e32 " r ", %9, " r ", vcc\n v_xor_b32_e32 " r ", %8, " r "\n v_xor_b32_e32 " r ", %9, " r "\n v_xor_b32_e32 " r ", %8, " r "\n v_xor_b32_e32 " r ", %9, " r "\n v_xor_b32_e32 " r ", %8, " r "\n v_xor_b32_e32 " r ", %9, " r "\n v_xor_b32_e32 " r ", %8, " r "\n "
#define P_CND_SGPR_7XOR(r) "v_cndmask_b32_e64 " r ", %9, " r ", s[44:45]\n v_xor_b32_e32 " r ", %8, " r "\n v_xor_b32_e32 " r ", %9, " r "\n v_xor_b32_e32 " r ", %8, " r "\n v_xor_b32_e32 " r ", %9, " r "\n v_xor_b32_e32 " r ", %8, " r "\n v_xor_b32_e32 " r ", %9, " r "\n v_xor_b32_e32 " r ", %8, " r "\n "
#define P_BITOP3_SGPRK(r) "v_bitop3_b32 " r ", " r ", %8, s46 bitop3:0x80\n "
#define P_BITOP3_VGPRK(r) "v_bitop3_b32 " r ", " r ", %8, %10 bitop3:0x80\n "
#define P_ADD_SGPR(r) "v_add_u32_e32 " r ", s46, " r "\n "
#define P_ADD_VGPRK(r) "v_add_u32_e32 " r ", %10, " r "\n "
#define P_SHL32(r) "v_lshlrev_b32_e32 " r ", 3, " r "\n "
#define P_SHL64(r) "v_lshlrev_b64 %13, 3, %12\n v_xor_b32_e32 " r ", %14, " r "\n "
#define P_CMP_BRANCH(r) "v_cmp_gt_u32_e32 vcc, %8, " r "\n s_cbranch_vccz 1f\n v_xor_b32_e32 " r ", %9, " r "\n 1:\n "
#define P_MIN(r) "v_min_u32_e32 " r ", %8, " r "\n "
#define P_MED3(r) "v_med3_u32 " r ", %8, " r ", %9\n "
#define P_DSADD_4XOR(r) "ds_add_u64 %11, %12\n v_xor_b32_e32 " r ", %8, " r "\n v_xor_b32_e32 " r ", %9, " r "\n v_xor_b32_e32 " r ", %8, " r "\n v_xor_b32_e32 " r ", %9, " r "\n "
#define P64_LSHR_INL "v_lshrrev_b64 %0, 3, %0\n v_lshrrev_b64 %1, 3, %1\n v_lshrrev_b64 %2, 3, %2\n v_lshrrev_b64 %3, 3, %3\n "
#define P64_LSHL_INL "v_lshlrev_b64 %0, 3, %0\n v_lshlrev_b64 %1, 3, %1\n v_lshlrev_b64 %2, 3, %2\n v_lshlrev_b64 %3, 3, %3\n "
#define P64_LSHR_V "v_lshrrev_b64 %0, %4, %0\n v_lshrrev_b64 %1, %4, %1\n v_lshrrev_b64 %2, %4, %2\n v_lshrrev_b64 %3, %4, %3\n "
#define P64_ASHR_INL "v_ashrrev_i64 %0, 3, %0\n v_ashrrev_i64 %1, 3, %1\n v_ashrrev_i64 %2, 3, %2\n v_ashrrev_i64 %3, 3, %3\n "
#define P64_ADD "v_lshl_add_u64 %0, %0, 0, %1\n v_lshl_add_u64 %1, %1, 0, %2\n v_lshl_add_u64 %2, %2, 0, %3\n v_lshl_add_u64 %3, %3, 0, %0\n "
#define P_ASHR16(r) "v_ashrrev_i16_e32 " r ", 15, " r "\n "
#define P_ALIGNBIT_V(r) "v_alignbit_b32 " r ", " r ", %8, %9\n "
#define MIX_BFE_XOR "v_bfe_u32 %0, %0, 2, 4\n v_xor_b32_e32 %4, %8, %4\n v_bfe_u32 %1, %1, 2, 4\n v_xor_b32_e32 %5, %8, %5\n v_bfe_u32 %2, %2, 2, 4\n v_xor_b32_e32 %6, %8, %6\n v_bfe_u32 %3, %3, 2, 4\n v_xor_b32_e32 %7, %8, %7\n "
#define MIX_BFE_3XOR "v_bfe_u32 %0, %0, 2, 4\n v_xor_b32_e32 %2, %8, %2\n v_xor_b32_e32 %3, %8, %3\n v_xor_b32_e32 %4, %8, %4\n v_bfe_u32 %1, %1, 2, 4\n v_xor_b32_e32 %5, %8, %5\n v_xor_b32_e32 %6, %8, %6\n v_xor_b32_e32 %7, %8, %7\n "
#define MIX_PERM_XOR "v_perm_b32 %0, %0, %8, %9\n v_xor_b32_e32 %4, %8, %4\n v_perm_b32 %1, %1, %8, %9\n v_xor_b32_e32 %5, %8, %5\n v_perm_b32 %2, %2, %8, %9\n v_xor_b32_e32 %6, %8, %6\n v_perm_b32 %3, %3, %8, %9\n v_xor_b32_e32 %7, %8, %7\n "
#define MIX_BCNT_ADD "v_bcnt_u32_b32 %0, %0, %8\n v_add_u32_e32 %4, %8, %4\n v_bcnt_u32_b32 %1, %1, %8\n v_add_u32_e32 %5, %8, %5\n v_bcnt_u32_b32 %2, %2, %8\n v_add_u32_e32 %6, %8, %6\n v_bcnt_u32_b32 %3, %3, %8\n v_add_u32_e32 %7, %8, %7\n "
#define MIX_CND_XOR "v_cndmask_b32_e64 %0, %9, %0, s[44:45]\n v_xor_b32_e32 %4, %8, %4\n v_cndmask_b32_e64 %1, %9, %1, s[44:45]\n v_xor_b32_e32 %5, %8, %5\n v_cndmask_b32_e64 %2, %9, %2, s[44:45]\n v_xor_b32_e32 %6, %8, %6\n v_cndmask_b32_e64 %3, %9, %3, s[44:45]\n v_xor_b32_e32 %7, %8, %7\n "
#define MIX_SGPRXOR_XOR "v_xor_b32_e64 %0, s46, %0\n v_xor_b32_e32 %4, %8, %4\n v_xor_b32_e64 %1, s46, %1\n v_xor_b32_e32 %5, %8, %5\n v_xor_b32_e64 %2, s46, %2\n v_xor_b32_e32 %6, %8, %6\n v_xor_b32_e64 %3, s46, %3\n v_xor_b32_e32 %7, %8, %7\n "
#define DEP_BFE_XOR "v_bfe_u32 %0, %0, 2, 4\n v_xor_b32_e32 %0, %8, %0\n v_bfe_u32 %1, %1, 2, 4\n v_xor_b32_e32 %1, %8, %1\n v_bfe_u32 %2, %2, 2, 4\n v_xor_b32_e32 %2, %8, %2\n v_bfe_u32 %3, %3, 2, 4\n v_xor_b32_e32 %3, %8, %3\n "
#define DEP_XOR2 "v_xor_b32_e32 %0, %8, %0\n v_xor_b32_e32 %1, %8, %1\n v_xor_b32_e32 %0, %9, %0\n v_xor_b32_e32 %1, %9, %1\n v_xor_b32_e32 %0, %8, %0\n v_xor_b32_e32 %1, %8, %1\n v_xor_b32_e32 %0, %9, %0\n v_xor_b32_e32 %1, %9, %1\n "
#define RUNM(P) for (int it = 0; it < iters; ++it) asm volatile(R4(R4(P)) : OUTS : "v"(x), "v"(y) : "vcc", "s44", "s45", "s46", "memory")
#define P_BFE3(r) "v_bfe_u32 %14, " r ", 4, 4\n v_lshl_add_u32 %15, %14, 7, %8\n v_bfe_u32 " r ", " r ", 8, 8\n "

template <int MODE>
__global__ void k_sel(uint32_t* out, int iters) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[8192];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 8192; i += blockDim.x) lds[i] = i;
    __syncthreads();
    uint32_t a = lane, b = lane + 1, c = lane + 2, d = lane + 3, e = lane + 4, f = lane + 5, g = lane + 6, h = lane + 7;
    uint32_t x = lane * 3 + 1, y = lane * 5 + 2, k = 0x80808080u;
    const uint32_t addr = (uint32_t)(lane & 15) * 8u + (uint32_t)(lane >> 4) * 128u;
    unsigned long long q = lane, t64 = lane, p0 = lane, p1 = lane + 1, p2 = lane + 2, p3 = lane + 3;
    uint32_t t0 = lane ^ 5, t1 = lane ^ 9;
    asm volatile("s_mov_b32 s44, 0x05040100\n s_mov_b32 s45, 0\n s_mov_b32 s46, 0x80808080\n s_mov_b64 vcc, s[44:45]" ::: "s44", "s45", "s46", "vcc");
#define RUN(P) for (int it = 0; it < iters; ++it) asm volatile(R4(C8(P)) : OUTS : "v"(x), "v"(y), "v"(k), "v"(addr), "v"(q), "v"(t64), "v"(t0), "v"(t1) : "vcc", "s44", "s45", "s46", "memory")
    if constexpr (MODE == 0) RUN(P_CMP_VCC);
    if constexpr (MODE == 1) RUN(P_CMP_SGPR);
    if constexpr (MODE == 2) RUN(P_SUB_ASHR_BITOP3);
    if constexpr (MODE == 3) RUN(P_CND_VCC_ONLY);
    if constexpr (MODE == 4) RUN(P_CND_VCC_7XOR);
    if constexpr (MODE == 5) RUN(P_CND_SGPR_7XOR);
    if constexpr (MODE == 6) RUN(P_BITOP3_SGPRK);
    if constexpr (MODE == 7) RUN(P_BITOP3_VGPRK);
    if constexpr (MODE == 8) RUN(P_ADD_SGPR);
    if constexpr (MODE == 9) RUN(P_ADD_VGPRK);
    if constexpr (MODE == 10) RUN(P_SHL32);
    if constexpr (MODE == 11) RUN(P_SHL64);
    if constexpr (MODE == 12) RUN(P_CMP_BRANCH);
    if constexpr (MODE == 13) RUN(P_MIN);
    if constexpr (MODE == 14) RUN(P_MED3);
    if constexpr (MODE == 15) RUN(P_DSADD_4XOR);
    if constexpr (MODE == 16) RUN(P_BFE3);
#define RUN64(P) for (int it = 0; it < iters; ++it) asm volatile(R4(R4(P)) : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(x) : "memory")
    if constexpr (MODE == 17) RUN64(P64_LSHR_INL);
    if constexpr (MODE == 18) RUN64(P64_LSHL_INL);
    if constexpr (MODE == 19) RUN64(P64_LSHR_V);
    if constexpr (MODE == 20) RUN64(P64_ASHR_INL);
    if constexpr (MODE == 21) RUN64(P64_ADD);
    if constexpr (MODE == 22) RUN(P_ASHR16);
    if constexpr (MODE == 23) RUN(P_ALIGNBIT_V);
    if constexpr (MODE == 24) RUNM(MIX_BFE_XOR);
    if constexpr (MODE == 25) RUNM(MIX_BFE_3XOR);
    if constexpr (MODE == 26) RUNM(MIX_PERM_XOR);
    if constexpr (MODE == 27) RUNM(MIX_BCNT_ADD);
    if constexpr (MODE == 28) RUNM(MIX_CND_XOR);
    if constexpr (MODE == 29) RUNM(MIX_SGPRXOR_XOR);
    if constexpr (MODE == 30) RUNM(DEP_BFE_XOR);
    if constexpr (MODE == 31) RUNM(DEP_XOR2);
    if ((a ^ b ^ c ^ d ^ e ^ f ^ g ^ h ^ (uint32_t)(p0 ^ p1 ^ p2 ^ p3)) == 0x9E3779B9u) out[blockIdx.x] = a;
}
static const char* kName[] = {
    "cmp_e32 vcc + s_nop1 + cndmask_e32 vcc", "cmp_e64 s[] + s_nop1 + cndmask_e64 s[]", "sub + ashr31 + bitop3 select",
    "cndmask_e32 vcc (vcc from s_mov)", "cndmask_e32 vcc + 7 xor", "cndmask_e64 s[] + 7 xor", "bitop3 with sgpr const",
    "bitop3 with vgpr const", "add_e32 sgpr", "add_e32 vgpr const", "lshlrev_b32 (32-bit shl)", "lshlrev_b64 + mov (32-bit shl)",
    "cmp_e32 vcc + s_cbranch_vccz + xor", "min_u32", "med3_u32", "ds_add_u64 + 4 xor", "bfe + lshl_add + bfe (stats base)",
    "lshrrev_b64 inline", "lshlrev_b64 inline", "lshrrev_b64 vgpr shift", "ashrrev_i64 inline", "lshl_add_u64 (64-bit add)", "ashrrev_i16", "alignbit vgpr shift",
    "mix 4 bfe : 4 xor", "mix 2 bfe : 6 xor", "mix 4 perm : 4 xor", "mix 4 bcnt : 4 add", "mix 4 cndmask_e64 sgpr : 4 xor",
    "mix 4 xor_e64 sgpr : 4 xor", "4 dependent bfe->xor chains", "2 dependent xor chains"};
static const int kInst[] = {3, 3, 3, 1, 8, 8, 1, 1, 1, 1, 1, 2, 3, 1, 1, 5, 3, 2, 2, 2, 2, 2, 1, 1, 4, 4, 4, 4, 4, 4, 4, 4};  // instructions per chain step (s_nop counted)
static int g_block = 1024;
template <int M>
static void run(int cus, uint32_t* out) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 1000;
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_sel<M>, dim3(cus), dim3(g_block), 0, 0, out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double steps = (g_block / 256.0) * iters * 32;  // per wave: iters x 4 x 8 chain steps; g_block/256 waves per SIMD
    const double cyc = best * 1e-3 * 2.4e9 / steps;
    printf("%-42s %7.2f SIMD cycles per chain step  (%5.2f per instruction, %d instr)\n", kName[M], cyc, cyc / kInst[M], kInst[M]);
}
template <int M>
static void all(int cus, uint32_t* out) {
    if constexpr (M < 32) {
        run<M>(cus, out);
        all<M + 1>(cus, out);
    }
}
int main(int argc, char** argv) {
    if (argc > 1) g_block = 256 * atoi(argv[1]);  // waves per SIMD (default 4)
    printf("waves per SIMD: %d\n", g_block / 256);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t* out;
    (void)hipMalloc(&out, 4 * 4096);
    all<0>(cus, out);
    return 0;
}
