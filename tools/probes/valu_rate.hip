// Probe: issue rate of integer VALU instructions on gfx950 (MI355X).
// 2 x 1024-thread workgroups per CU (8 waves/SIMD), each lane runs 8
// independent chains of one instruction; prints cycles per wave-instruction
// per SIMD (2 = full rate wave64 on a 32-lane SIMD, 4 = half rate).
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 4096

#define BODY8(INS)                                                                                 \
    asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" \
                 INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8" \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)  \
                 : "v"(k))
#define BODY8_3(INS, TAIL)                                                                           \
    asm volatile(INS " %0, %0, %8, %9" TAIL "\n\t" INS " %1, %1, %8, %9" TAIL "\n\t" INS " %2, %2, %8, %9" TAIL \
                 "\n\t" INS " %3, %3, %8, %9" TAIL "\n\t" INS " %4, %4, %8, %9" TAIL "\n\t" INS            \
                 " %5, %5, %8, %9" TAIL "\n\t" INS " %6, %6, %8, %9" TAIL "\n\t" INS " %7, %7, %8, %9" TAIL \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)      \
                 : "v"(k), "v"(k2))

#define BODY8_SDWA()                                                                                 \
    asm volatile("v_xor_b32_sdwa %0, %0, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t" \
                 "v_xor_b32_sdwa %1, %1, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t" \
                 "v_xor_b32_sdwa %2, %2, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t" \
                 "v_xor_b32_sdwa %3, %3, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t" \
                 "v_xor_b32_sdwa %4, %4, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t" \
                 "v_xor_b32_sdwa %5, %5, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t" \
                 "v_xor_b32_sdwa %6, %6, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t" \
                 "v_xor_b32_sdwa %7, %7, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0" \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)  \
                 : "v"(k))
#define BODY8_CND()                                                                                 \
    asm volatile("v_cndmask_b32 %0, %0, %8, vcc\n\tv_cndmask_b32 %1, %1, %8, vcc\n\tv_cndmask_b32 %2, %2, %8, vcc\n\t" \
                 "v_cndmask_b32 %3, %3, %8, vcc\n\tv_cndmask_b32 %4, %4, %8, vcc\n\tv_cndmask_b32 %5, %5, %8, vcc\n\t" \
                 "v_cndmask_b32 %6, %6, %8, vcc\n\tv_cndmask_b32 %7, %7, %8, vcc" \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)  \
                 : "v"(k))

#define BODY8_RAW(STR, C1, C2)                                                                          \
    asm volatile(STR : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)     \
                 : "v"(k), "v"(k2) : C1, C2)
#define R8(F) F(0) "\n\t" F(1) "\n\t" F(2) "\n\t" F(3) "\n\t" F(4) "\n\t" F(5) "\n\t" F(6) "\n\t" F(7)
#define CNDS(i) "v_cndmask_b32_e64 %" #i ", %" #i ", %8, s[40:41]"
#define CMPS(i) "v_cmp_gt_u32_e64 s[40:41], %" #i ", %8"
#define LSLI(i) "v_lshlrev_b32 %" #i ", 3, %" #i
#define LSRI(i) "v_lshrrev_b32 %" #i ", 3, %" #i
#define XORC(i) "v_xor_b32 %" #i ", 0x7070707, %" #i
#define ANDC(i) "v_and_b32 %" #i ", 0x7070707, %" #i
#define DSR8(i) "ds_read_u8 %" #i ", %" #i " offset:64"
#define DSRB(i) "ds_read_b32 %" #i ", %" #i " offset:64"
#define MOVD(i) "v_mov_b32_dpp %" #i ", %" #i " row_shr:1 row_mask:0xf bank_mask:0xf"

template <int OP>
__global__ __launch_bounds__(1024, 8) void rate_k(uint32_t *out, uint32_t seed)
{
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7;
    const uint32_t k = seed * 3u + threadIdx.x, k2 = seed ^ 0x07070707u;
    asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(k), "v"(k2) : "vcc");
    __shared__ uint32_t lds[16384];
    if (OP == 42 || OP == 43) {
        lds[threadIdx.x] = threadIdx.x;
        __syncthreads();
        a0 = (threadIdx.x & 31) * 4; a1 = a0; a2 = a0; a3 = a0; a4 = a0; a5 = a0; a6 = a0; a7 = a0;
        asm volatile("" :: "v"(lds[0]));
    }
    for (int i = 0; i < ITERS; ++i) {
        if (OP == 0)
            BODY8("v_xor_b32");
        if (OP == 1)
            BODY8("v_and_b32");
        if (OP == 2)
            BODY8("v_or_b32");
        if (OP == 3)
            BODY8("v_add_u32");
        if (OP == 4)
            BODY8("v_sub_u32");
        if (OP == 5)
            BODY8("v_lshlrev_b32");
        if (OP == 6)
            BODY8("v_lshrrev_b32");
        if (OP == 7)
            BODY8("v_min_u32");
        if (OP == 8)
            BODY8("v_max_u32");
        if (OP == 9)
            BODY8("v_min_i32");
        if (OP == 10)
            BODY8("v_mul_u32_u24");
        if (OP == 11)
            BODY8("v_mul_lo_u32");
        if (OP == 12)
            BODY8("v_add_f32");
        if (OP == 13)
            BODY8("v_pk_add_u16");
        if (OP == 14)
            BODY8("v_pk_min_u16");
        if (OP == 15)
            BODY8("v_add_u16");
        if (OP == 16)
            BODY8("v_min_u16");
        if (OP == 17)
            BODY8("v_lshlrev_b16");
        if (OP == 18)
            BODY8_SDWA();
        if (OP == 19)
            BODY8_3("v_bitop3_b32", " bitop3:0x96");
        if (OP == 20)
            BODY8_3("v_perm_b32", "");
        if (OP == 21)
            BODY8_3("v_lshl_add_u32", "");
        if (OP == 22)
            BODY8_3("v_add_lshl_u32", "");
        if (OP == 23)
            BODY8_3("v_lshl_or_b32", "");
        if (OP == 24)
            BODY8_3("v_and_or_b32", "");
        if (OP == 25)
            BODY8_3("v_or3_b32", "");
        if (OP == 26)
            BODY8_3("v_add3_u32", "");
        if (OP == 27)
            BODY8_3("v_alignbyte_b32", "");
        if (OP == 28)
            BODY8_3("v_alignbit_b32", "");
        if (OP == 29)
            BODY8_3("v_bfe_u32", "");
        if (OP == 30)
            BODY8_3("v_bfi_b32", "");
        if (OP == 31)
            BODY8_3("v_xad_u32", "");
        if (OP == 32)
            BODY8_3("v_med3_u32", "");
        if (OP == 33)
            BODY8_3("v_min3_u32", "");
        if (OP == 34)
            BODY8_3("v_mad_u32_u24", "");
        if (OP == 35)
            BODY8_CND();
        if (OP == 36)
            BODY8_RAW(R8(CNDS), "s40", "s41");
        if (OP == 37)
            BODY8_RAW(R8(CMPS), "s40", "s41");
        if (OP == 38)
            BODY8_RAW(R8(LSLI), "memory", "memory");
        if (OP == 39)
            BODY8_RAW(R8(LSRI), "memory", "memory");
        if (OP == 40)
            BODY8_RAW(R8(XORC), "memory", "memory");
        if (OP == 41)
            BODY8_RAW(R8(ANDC), "memory", "memory");
        if (OP == 42) {
            BODY8_RAW(R8(DSR8), "memory", "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        if (OP == 43) {
            BODY8_RAW(R8(DSRB), "memory", "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        if (OP == 44)
            BODY8_RAW(R8(MOVD), "memory", "memory");
    }
    out[blockIdx.x * 1024 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int OP>
static void run(const char *name, uint32_t *d, int cus)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 2 * cus;
    hipLaunchKernelGGL(rate_k<OP>, dim3(blocks), dim3(1024), 0, 0, d, 1u);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL(rate_k<OP>, dim3(blocks), dim3(1024), 0, 0, d, (uint32_t)r);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    // wave-instructions per SIMD: 8 waves x ITERS x 8
    const double insts = 8.0 * ITERS * 8.0;
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0); // kHz
    const double cycles = ms * 1e-3 * clk * 1e3;
    printf("%-16s %8.3f ms  %5.2f cycles/wave-instr/SIMD (clock %d MHz)\n", name, ms, cycles / insts, clk / 1000);
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *d;
    hipMalloc(&d, (size_t)2 * cus * 1024 * 4);
    run<0>("v_xor_b32", d, cus);
    run<1>("v_and_b32", d, cus);
    run<2>("v_or_b32", d, cus);
    run<3>("v_add_u32", d, cus);
    run<4>("v_sub_u32", d, cus);
    run<5>("v_lshlrev_b32", d, cus);
    run<6>("v_lshrrev_b32", d, cus);
    run<7>("v_min_u32", d, cus);
    run<8>("v_max_u32", d, cus);
    run<9>("v_min_i32", d, cus);
    run<10>("v_mul_u32_u24", d, cus);
    run<11>("v_mul_lo_u32", d, cus);
    run<12>("v_add_f32", d, cus);
    run<13>("v_pk_add_u16", d, cus);
    run<14>("v_pk_min_u16", d, cus);
    run<15>("v_add_u16", d, cus);
    run<16>("v_min_u16", d, cus);
    run<17>("v_lshlrev_b16", d, cus);
    run<18>("v_xor_b32_sdwa_pad", d, cus);
    run<19>("v_bitop3_b32", d, cus);
    run<20>("v_perm_b32", d, cus);
    run<21>("v_lshl_add_u32", d, cus);
    run<22>("v_add_lshl_u32", d, cus);
    run<23>("v_lshl_or_b32", d, cus);
    run<24>("v_and_or_b32", d, cus);
    run<25>("v_or3_b32", d, cus);
    run<26>("v_add3_u32", d, cus);
    run<27>("v_alignbyte_b32", d, cus);
    run<28>("v_alignbit_b32", d, cus);
    run<29>("v_bfe_u32", d, cus);
    run<30>("v_bfi_b32", d, cus);
    run<31>("v_xad_u32", d, cus);
    run<32>("v_med3_u32", d, cus);
    run<33>("v_min3_u32", d, cus);
    run<34>("v_mad_u32_u24", d, cus);
    run<35>("v_cndmask_b32_vcc", d, cus);
    run<36>("v_cndmask_e64_s", d, cus);
    run<37>("v_cmp_e64_s", d, cus);
    run<38>("v_lshlrev_imm", d, cus);
    run<39>("v_lshrrev_imm", d, cus);
    run<40>("v_xor_lit", d, cus);
    run<41>("v_and_lit", d, cus);
    run<42>("ds_read_u8(8,wait)", d, cus);
    run<43>("ds_read_b32(8,wait)", d, cus);
    run<44>("v_mov_dpp", d, cus);
    hipFree(d);
    return 0;
}
