// keccak.cuh — Keccak-f[1600] / Keccak-256 for one lane per thread on CDNA4.
//
// The reference hashes concrete SHA3 inputs with eth-hash's Keccak-256 (0x01
// domain pad, NOT NIST SHA3-256) — keccak_function_manager.py:57-68 ->
// support_utils.py:93-101.  The 25-word state lives in 50 VGPRs; every index
// is a compile-time constant after unrolling, rotations by constants lower to
// v_alignbit_b32 pairs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

__constant__ uint64_t kKeccakRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull,
    0x8000000080008000ull, 0x000000000000808bull, 0x0000000080000001ull,
    0x8000000080008081ull, 0x8000000000008009ull, 0x000000000000008aull,
    0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull,
    0x8000000000008003ull, 0x8000000000008002ull, 0x8000000000000080ull,
    0x000000000000800aull, 0x800000008000000aull, 0x8000000080008081ull,
    0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

// 64-bit rotate by a compile-time constant as two v_alignbit_b32 funnel shifts
// on the 32-bit halves (alignbit(a, b, s) = low word of (a:b) >> s).  Written
// out: the (v << r) | (v >> 64 - r) form lowers to 64-bit shift pairs plus ors,
// two to three times the instructions, and at one wave per SIMD (kernel 1's C2
// grid) Keccak-f's instruction count is its latency.
__device__ __forceinline__ uint64_t krotl(uint64_t v, int r) {
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    uint32_t nh, nl;
    if (r == 0) return v;
    if (r < 32) {
        nh = __builtin_amdgcn_alignbit(hi, lo, 32 - r);
        nl = __builtin_amdgcn_alignbit(lo, hi, 32 - r);
    } else if (r == 32) {
        nh = lo; nl = hi;
    } else {
        nh = __builtin_amdgcn_alignbit(lo, hi, 64 - r);
        nl = __builtin_amdgcn_alignbit(hi, lo, 64 - r);
    }
    return ((uint64_t)nh << 32) | nl;
}

// gfx950 v_bitop3_b32: any 3-input bitwise function in one VALU instruction
// (truth-table index = S0*4 + S1*2 + S2).  Keccak's theta parities and theta
// update are 3-way XORs (0x96) and chi's a ^ (~b & c) is table 0xD2: on 32-bit
// halves that is one instruction where the xor / bfi+xor forms take two — at one
// wave per SIMD (kernel 1's C2 grid) the VALU instruction count is the latency.
__device__ __forceinline__ uint64_t k_xor3(uint64_t a, uint64_t b, uint64_t c) {
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0x96);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0x96);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t k_chi(uint64_t a, uint64_t b, uint64_t c) {   // a ^ (~b & c)
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0xD2);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0xD2);
    return ((uint64_t)hi << 32) | lo;
}

// In-place rounds: theta with 5 column parities, rho+pi as the single 24-cycle
// of the lane permutation (one temporary), chi row by row (5 temporaries) — about
// 70 live VGPRs instead of the 120 of a two-array formulation.
__device__ __forceinline__ void keccak_f1600(uint64_t st[25]) {
    constexpr int PILN[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4,
                              15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};
    constexpr int ROTC[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14,
                              27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
    for (int round = 0; round < 24; ++round) {
        uint64_t bc[5];
#pragma unroll
        for (int x = 0; x < 5; ++x) bc[x] = k_xor3(k_xor3(st[x], st[x + 5], st[x + 10]), st[x + 15], st[x + 20]);
#pragma unroll
        for (int x = 0; x < 5; ++x) {
            const uint64_t r = krotl(bc[(x + 1) % 5], 1);
#pragma unroll
            for (int y = 0; y < 25; y += 5) st[y + x] = k_xor3(st[y + x], bc[(x + 4) % 5], r);
        }
        uint64_t t = st[1];
#pragma unroll
        for (int i = 0; i < 24; ++i) {
            const int j = PILN[i];
            const uint64_t tmp = st[j];
            st[j] = krotl(t, ROTC[i]);
            t = tmp;
        }
#pragma unroll
        for (int y = 0; y < 25; y += 5) {
#pragma unroll
            for (int x = 0; x < 5; ++x) bc[x] = st[y + x];
#pragma unroll
            for (int x = 0; x < 5; ++x) st[y + x] = k_chi(bc[x], bc[(x + 1) % 5], bc[(x + 2) % 5]);
        }
        st[0] ^= kKeccakRC[round];
    }
}
