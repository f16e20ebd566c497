/*
 * bitslice_enc.hip -- prototype of a bit-sliced RS(255,223) encoder
 * (VERDICT r04 "next round" #1; cost model and result: DESIGN.md section 7).
 * Not part of the product library: built by tools/probes/bitslice_run.py into
 * tools/probes/_build/, timed against rs_lfsr_k<ENCODE> on the same box, its
 * parity compared byte for byte with the product encoder's.
 *
 * One lane = 32 consecutive codewords (wire layout, 255-byte rows); bit c of
 * every register is codeword c.  Per group of 4 message bytes the lane gathers
 * one (unaligned) dword of each of its 32 rows and transposes the 32 x 32 bit
 * block in registers (two v_perm byte stages, three shift/bitop3 stages): the
 * 32 message planes of 4 steps.  The LFSR's 256 state planes live in a ring
 * of registers and one revolution of 32 steps is generated code
 * (tools/probes/gen_bitslice.py -> bs_net.h, generated on demand and not committed: 8 + 22 + 256 VALU ops a step).
 * A zero byte is prepended to the message (224 steps = 7 revolutions; a
 * leading zero leaves the parity unchanged), so the ring ends unrotated.
 * At the end the 256 planes are transposed back and stored as 8 dwords per
 * row.
 *
 *   BS_MODE 0  the encoder (gather, transpose, LFSR, transpose, store)
 *   BS_MODE 1  the LFSR steps alone: message planes from a register hash
 *   BS_MODE 2  the gathers and transposes alone (planes XORed into a sink)
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef BS_MODE
#define BS_MODE 0
#endif

#include "bs_net.h"

/* 32 x 32 bit transpose: bit k of a[c] <-> bit c of a[k] */
__device__ __forceinline__ void transpose32(uint32_t (&a)[32])
{
#pragma unroll
    for (int c = 0; c < 16; ++c) { /* j = 16: half-words */
        const uint32_t x = a[c], y = a[c + 16];
        a[c] = __builtin_amdgcn_perm(y, x, 0x05040100u);
        a[c + 16] = __builtin_amdgcn_perm(y, x, 0x07060302u);
    }
#pragma unroll
    for (int c = 0; c < 32; ++c) { /* j = 8: bytes */
        if (c & 8)
            continue;
        const uint32_t x = a[c], y = a[c + 8];
        a[c] = __builtin_amdgcn_perm(y, x, 0x06020400u);
        a[c + 8] = __builtin_amdgcn_perm(y, x, 0x07030501u);
    }
#pragma unroll
    for (int js = 2; js >= 0; --js) { /* j = 4, 2, 1 */
        const int j = 1 << js;
        const uint32_t m = js == 2 ? 0x0F0F0F0Fu : js == 1 ? 0x33333333u : 0x55555555u;
#pragma unroll
        for (int c = 0; c < 32; ++c) {
            if (c & j)
                continue;
            const uint32_t t = __builtin_amdgcn_bitop3_b32(a[c] >> j, a[c + j], m, 0x28); /* (A ^ B) & C */
            a[c + j] ^= t;
            a[c] ^= t << j;
        }
    }
}

__device__ __forceinline__ uint32_t ldu32(const uint8_t *p)
{
    return *reinterpret_cast<const uint32_t *>(p); /* unaligned dword: global_load_dword */
}

__global__ __launch_bounds__(64, 1) void bs_encode_k(const uint8_t *__restrict__ data, uint8_t *__restrict__ out,
                                                     size_t count, uint32_t *__restrict__ sink)
{
    const size_t L = (size_t)blockIdx.x * 64u + threadIdx.x;
    if (32u * L >= count)
        return;
    const uint8_t *row = data + 32u * L * 255u;
    uint32_t R_[32][8];
#pragma unroll
    for (int k = 0; k < 32; ++k)
#pragma unroll
        for (int b = 0; b < 8; ++b)
            R_[k][b] = 0u;
    uint32_t A0[32], A1[32];
    uint32_t acc = 0;
#if BS_MODE != 1
#pragma unroll
    for (int c = 0; c < 32; ++c)
        A0[c] = ldu32(row + 255u * c);
#endif
#define R(k, b) R_[k][b]
#define D(s, b) (((s) >> 2) & 1 ? A1 : A0)[8 * ((s) & 3) + (b)]
#if BS_MODE == 1
#define BS_GROUP(q)                                                                                   \
    do {                                                                                              \
        uint32_t *cur = ((q) & 1) ? A1 : A0;                                                          \
        const uint32_t g = 8u * rev + (q), hsh = (uint32_t)L * 0x9E3779B9u ^ g * 0x85EBCA6Bu;         \
        _Pragma("unroll") for (int k = 0; k < 32; ++k) cur[k] = g ? hsh ^ (uint32_t)k * 0xC2B2AE35u : 0u; \
    } while (0)
#else
#define BS_GROUP(q)                                                                                   \
    do {                                                                                              \
        uint32_t *cur = ((q) & 1) ? A1 : A0, *nxt = ((q) & 1) ? A0 : A1;                              \
        const uint32_t g = 8u * rev + (q);                                                            \
        if (g == 0u) {                                                                                \
            _Pragma("unroll") for (int c = 0; c < 32; ++c) cur[c] <<= 8; /* the prepended zero byte */ \
        }                                                                                             \
        transpose32(*reinterpret_cast<uint32_t(*)[32]>(cur));                                         \
        if (g + 1u < 56u) {                                                                           \
            _Pragma("unroll") for (int c = 0; c < 32; ++c) nxt[c] = ldu32(row + 255u * c + 4u * (g + 1u) - 1u); \
        }                                                                                             \
        if (BS_MODE == 2) {                                                                           \
            _Pragma("unroll") for (int k = 0; k < 32; ++k) acc ^= cur[k];                             \
        }                                                                                             \
    } while (0)
#endif
#pragma unroll 1
    for (uint32_t rev = 0; rev < 7u; ++rev) {
#if BS_MODE == 2
#pragma unroll
        for (int q = 0; q < 8; ++q)
            BS_GROUP(q);
#else
        BS_REVOLUTION();
#endif
    }
#if BS_MODE == 0
    uint8_t *orow = out + 32u * L * 255u + 223u;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        uint32_t a[32];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int b = 0; b < 8; ++b)
                a[8 * q + b] = R_[4 * g + q][b];
        transpose32(a);
#pragma unroll
        for (int c = 0; c < 32; ++c)
            *reinterpret_cast<uint32_t *>(orow + 255u * c + 4u * g) = a[c];
    }
#elif BS_MODE == 1
#pragma unroll
    for (int k = 0; k < 32; ++k)
#pragma unroll
        for (int b = 0; b < 8; ++b)
            acc ^= R_[k][b] * (uint32_t)(8 * k + b + 1);
    sink[L] = acc;
#else
    sink[L] = acc;
#endif
#undef R
#undef D
}

extern "C" int bs_encode(const void *data, void *out, size_t count, void *sink, void *stream)
{
    const size_t lanes = (count + 31) / 32;
    hipLaunchKernelGGL(bs_encode_k, dim3((uint32_t)((lanes + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                       (const uint8_t *)data, (uint8_t *)out, count, (uint32_t *)sink);
    return (int)hipGetLastError();
}
