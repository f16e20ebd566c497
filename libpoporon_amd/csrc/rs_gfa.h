/*
 * rs_gfa.h -- the address-form GF(2^8) table of the lane-per-codeword split
 * kernels (rs_fast.hip, rs_errata.hip): its LDS fill and accessors, and a
 * compile-time loop.  Table layout and zero sentinels: rs_fast.hip header.
 */
#ifndef POPORON_AMD_RS_GFA_H
#define POPORON_AMD_RS_GFA_H

#include <hip/hip_runtime.h>

#include <type_traits>

#include "rs_device.h"
#include "rs_lane.h"

#define Z0 RS_Z0       /* zero sentinels: AZ = 128 Z0 + 4r, SZ = 128 Z0 - 1 (rs_fast.hip header) */
#define SZ (128u * Z0 - 1u)

/* ------------------------------------------------------------------------ */
/* GF table (rs_bm_k, rs_forney_k)                                          */
/* ------------------------------------------------------------------------ */

/* the table image (RsDevTables::gfa) into LDS: every load first, then the
 * stores (a rolled copy waits for each load: one L2 round trip apiece) */
template <int WG>
__device__ __forceinline__ void fill_gfa(uint32_t *lgf, const RsDevTables *__restrict__ T)
{
    if constexpr ((512 * 32 / 4) % WG != 0) {
        for (uint32_t t = threadIdx.x; t < 512u * 32u / 4u; t += WG)
            reinterpret_cast<uint4 *>(lgf)[t] = T->gfa[t];
        return;
    }
    constexpr int K = 512 * 32 / 4 / WG;
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
        v[k] = T->gfa[threadIdx.x + k * WG];
#pragma unroll
    for (int k = 0; k < K; ++k)
        reinterpret_cast<uint4 *>(lgf)[threadIdx.x + k * WG] = v[k];
}

struct GfA {
    uint32_t pofs; /* 4 (lane & 31) + 1: this replica's exp byte of log 0 */
    /* this replica's address-form zero */
    __device__ __forceinline__ uint32_t az() const { return pofs + SZ; }
    /* exp of an address-form log plus a plain scaled log */
    __device__ __forceinline__ uint32_t expa(uint32_t a) const { return lds8(a); }
    /* address-form log of v < 256 (AZ for 0) */
    __device__ __forceinline__ uint32_t loga(uint32_t v) const { return lds16(pofs + 1u + (v << 7)); }
    /* plain scaled log 128 log v (SZ for 0) */
    __device__ __forceinline__ uint32_t logs(uint32_t v) const { return loga(v) - pofs; }
    /* log (0..254) of an address-form log, 255 for zero */
    __device__ __forceinline__ uint32_t plog(uint32_t a) const { return (a & 1u) ? (a - pofs) >> 7 : 255u; }
    /* address-form log of a stored byte log (255 = zero) */
    __device__ __forceinline__ uint32_t afrom(uint32_t b) const { return b < 255u ? (b << 7) + pofs : az(); }
    /* alpha^l of a plain log l < 255 */
    __device__ __forceinline__ uint32_t exp(uint32_t l) const { return lds8(pofs + (l << 7)); }
    /* "log-entry address" form of a value v: pofs + 1 + 128 v, the address
     * loga reads (bits 7..14 = v, the replica offset below: XOR of v << 7
     * adds to v); its log is one ds_read_u16 */
    __device__ __forceinline__ uint32_t hz() const { return pofs + 1u; }
    __device__ __forceinline__ uint32_t logh(uint32_t h) const { return lds16(h); }
};

/* v << 7 for a byte v in one full-rate 16-bit op (VOP2 16-bit results zero
 * bits 31:16 on gfx950) */
__device__ __forceinline__ uint32_t shl7(uint32_t v)
{
    uint32_t r;
    asm("v_lshlrev_b16 %0, 7, %1" : "=v"(r) : "v"(v));
    return r;
}

/* compile-time loop: f(std::integral_constant<int, i>) for i = I, I+S, ... < E */
template <int I, int E, int S, class F>
__device__ __forceinline__ void static_for(F &&f)
{
    if constexpr (I < E) {
        f(std::integral_constant<int, I>{});
        static_for<I + S, E, S>(f);
    }
}

#endif
