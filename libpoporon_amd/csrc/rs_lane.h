/*
 * rs_lane.h -- device helpers shared by the lane-per-codeword RS kernels
 * (rs_correct.hip, rs_fast.hip): wave reductions over ballots / DPP, byte
 * tests, the root-map iterator and the reference's gf_mod.
 */
#ifndef POPORON_AMD_RS_LANE_H
#define POPORON_AMD_RS_LANE_H

#include <hip/hip_runtime.h>

#include "rs_device.h"

/* LDS reads from a byte address (address space 3, made from an integer;
 * going through an integer keeps the compiler from reasoning about the
 * bounds of a C++ object).  What a read past the workgroup's allocation
 * returns depends on the allocation: past the end of the whole 160 KiB LDS
 * it reads 0 (tools/probes/lds_oob.hip), which rs_correct_k's zero sentinel
 * relies on (its table ends exactly there: static_assert LDS_END == 163840 in
 * rs_correct.hip); past a smaller allocation it may read another
 * workgroup's LDS (tools/probes/lds_oob64.hip), so the split kernels keep
 * every read inside their own tables (rs_fast.hip header). */
typedef __attribute__((address_space(3))) const uint8_t lds_u8;
typedef __attribute__((address_space(3))) const uint16_t lds_u16;
typedef unsigned lds_u32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const lds_u32x4_t lds_u32x4;

__device__ __forceinline__ uint32_t lds8(uint32_t a) { return *(lds_u8 *)(size_t)a; }
__device__ __forceinline__ uint32_t lds16(uint32_t a) { return *(lds_u16 *)(size_t)a; }
__device__ __forceinline__ lds_u32x4_t lds128(uint32_t a) { return *(lds_u32x4 *)(size_t)a; }
__device__ __forceinline__ void lds_st8(uint32_t a, uint32_t v)
{
    *(__attribute__((address_space(3))) uint8_t *)(size_t)a = (uint8_t)v;
}
/* LDS byte address of a __shared__ object (also makes the object escape,
 * so its stores are never dropped as unread) */
template <typename T> __device__ __forceinline__ uint32_t lds_addr(const T *p)
{
    return (uint32_t)(size_t)(__attribute__((address_space(3))) const T *)p;
}

/* gf_mod of src/internal/common.h:102-110 on the uint16 truncation of v */
__device__ __forceinline__ uint32_t mod255(uint32_t v) { return (v & 0xffffu) % 255u; }
/* x < 510 -> x mod 255; sentinel x >= 767 -> x - 255 (still >= 512) */
__device__ __forceinline__ uint32_t red(uint32_t x) { return min(x, x - 255u); }
/* stored byte log (255 = zero) -> register log: max(s, (s - 254) * 1024) as
 * signed ints is s for s <= 254 and 1024 for 255 (mad + max, no compare) */
__device__ __forceinline__ uint32_t conv(uint32_t s8)
{
    return (uint32_t)max((int32_t)s8, ((int32_t)s8 - 254) * 1024);
}

/* u16 halves of packed log pairs: entry 2k low, 2k+1 high */
__device__ __forceinline__ uint32_t half(const uint32_t *a, int i)
{
    return (i & 1) ? (a[i >> 1] >> 16) : (a[i >> 1] & 0xffffu);
}

/* (x + y) mod 255 * 128 for scaled logs x, y < 255 * 128: three full-rate
 * 16-bit ops instead of add, add, half-rate v_min_u32 (gfx950's VOP2 16-bit
 * ops zero bits 31:16 of the result: tools/probes/u16_hi.hip) */
__device__ __forceinline__ uint32_t addmod7(uint32_t x, uint32_t y)
{
    uint32_t t, u, r;
    asm("v_add_u16 %0, %1, %2" : "=v"(t) : "v"(x), "v"(y));
    asm("v_subrev_u16 %0, 0x7f80, %1" : "=v"(u) : "v"(t)); /* t - 255 * 128, wraps above t when t < 255 * 128 */
    asm("v_min_u16 %0, %1, %2" : "=v"(r) : "v"(t), "v"(u));
    return r;
}

/* Persistent loops: issue priority falling with the wave's progress (it =
 * batches done), so the waves that are behind win the issue arbitration
 * (priority, then age) and a workgroup's waves finish together instead of
 * the oldest first, which left the last batches running at low occupancy:
 * LFSR encode / remainder 5 % faster (profiles/r03_grid_rounds.log). */
__device__ __forceinline__ void prio_by_progress(uint32_t it)
{
    switch (it) {
    case 0: __builtin_amdgcn_s_setprio(3); break;
    case 1: __builtin_amdgcn_s_setprio(2); break;
    case 2: __builtin_amdgcn_s_setprio(1); break;
    default: __builtin_amdgcn_s_setprio(0); break;
    }
}

/* (a + inc) reduced below WRAP = 255 * row bytes (a < WRAP, or the all-zero
 * rows' WRAP + j stepping by WRAP; inc <= WRAP): the Chien row addresses.
 * Three VOP2 ops (add, subtract with the borrow into VCC, select on VCC)
 * instead of two adds and a half-rate v_min_u32: rs_chien_k 0.068 -> 0.062 ms
 * (profiles/r03_chien_vcc.log) */
template <uint32_t WRAP>
__device__ __forceinline__ uint32_t chien_step(uint32_t a, uint32_t inc)
{
    uint32_t t1, t2, r;
    asm("v_add_u32_e32 %0, %3, %4\n\t"
        "v_subrev_co_u32_e32 %1, vcc, %5, %0\n\t"
        "v_cndmask_b32_e32 %2, %1, %0, vcc"
        : "=&v"(t1), "=&v"(t2), "=v"(r)
        : "v"(a), "v"(inc), "i"(WRAP)
        : "vcc");
    return r;
}

/* a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96) */
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

/* Maximum of v (< 64) over the ACTIVE lanes of the wave, bit by bit from
 * ballots.  (A shuffle butterfly is wrong here: lanes that have left the
 * codeword's control flow do not forward partial maxima.) */
__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
    uint32_t m = 0;
#pragma unroll
    for (int b = 5; b >= 0; --b) {
        const uint32_t c = m | (1u << b);
        if (__ballot(v >= c) != 0ull)
            m = c;
    }
    return m;
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) { return 63u - wave_max(63u - v); }

/* Maximum of v over all 64 lanes -- only where every lane of the wave is
 * active.  DPP row shifts give each row's inclusive maximum in its lane 15,
 * two row broadcasts fold the rows into lane 63. */
__device__ __forceinline__ uint32_t wave_max_full(uint32_t v)
{
    uint32_t x = v;
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true)); /* row_shr:1 */
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true)); /* row_shr:2 */
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true)); /* row_shr:4 */
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true)); /* row_shr:8 */
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false)); /* row_bcast:15 */
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false)); /* row_bcast:31 */
    return __builtin_amdgcn_readlane(x, 63);
}

/* byte-wise zero test: bit 8b + 7 set iff byte b of v is zero, every other bit clear */
__device__ __forceinline__ uint32_t zero80(uint32_t v)
{
    const uint32_t t = (v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    return __builtin_amdgcn_bitop3_b32(t, v, 0x7F7F7F7Fu, 0x01); /* ~(t | v | 0x7F7F7F7F) */
}

/* byte-wise zero test of 16 bytes -> 16-bit mask (bit b: byte b is zero) */
__device__ __forceinline__ uint32_t zero_bytes16(const uint32_t (&v)[4])
{
    uint32_t m = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t z = ~(((v[d] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v[d] | 0x7F7F7F7Fu); /* bit 8b+7 */
        const uint32_t t = (z >> 7) & 0x01010101u;
        m |= ((t * 0x10204080u) >> 28) << (4 * d);
    }
    return m;
}

/* Walks a 256-bit root map over i' = i mod 255 in the reference's order
 * (src/decode.c:117-141): i = 1..254 ascending, then i = 255 (bit 0).  No
 * per-lane loops. */
struct RootIter {
    uint32_t w[9]; /* w[0..7]: bits of i' (bit 0 of w[0] removed), w[8]: the i = 255 bit */
    __device__ __forceinline__ void init(const uint32_t (&rb)[8])
    {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            w[k] = rb[k];
        w[8] = rb[0] & 1u;
        w[0] &= ~1u;
    }
    __device__ __forceinline__ uint32_t next()
    {
        uint32_t sel = 8, bits = w[8];
#pragma unroll
        for (int k = 7; k >= 0; --k) {
            const bool nz = w[k] != 0u;
            sel = nz ? (uint32_t)k : sel;
            bits = nz ? w[k] : bits;
        }
        const uint32_t b = __builtin_ctz(bits | 0x80000000u);
        const uint32_t clr = bits & (bits - 1u);
#pragma unroll
        for (int k = 0; k < 9; ++k)
            w[k] = (sel == (uint32_t)k) ? clr : w[k];
        return sel < 8u ? 32u * sel + b : 255u;
    }
};

#endif
