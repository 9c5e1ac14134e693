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

__device__ __forceinline__ uint64_t krotl(uint64_t v, int r) {
    return r == 0 ? v : ((v << r) | (v >> (64 - r)));
}

__device__ __forceinline__ void keccak_f1600(uint64_t st[25]) {
    constexpr int RHO[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                             25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
    for (int round = 0; round < 24; ++round) {
        uint64_t C[5], D[5], B[25];
#pragma unroll
        for (int x = 0; x < 5; ++x) C[x] = st[x] ^ st[x + 5] ^ st[x + 10] ^ st[x + 15] ^ st[x + 20];
#pragma unroll
        for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ krotl(C[(x + 1) % 5], 1);
#pragma unroll
        for (int i = 0; i < 25; ++i) st[i] ^= D[i % 5];
#pragma unroll
        for (int x = 0; x < 5; ++x)
#pragma unroll
            for (int y = 0; y < 5; ++y) B[y + 5 * ((2 * x + 3 * y) % 5)] = krotl(st[x + 5 * y], RHO[x + 5 * y]);
#pragma unroll
        for (int y = 0; y < 5; ++y)
#pragma unroll
            for (int x = 0; x < 5; ++x)
                st[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
        st[0] ^= kKeccakRC[round];
    }
}
