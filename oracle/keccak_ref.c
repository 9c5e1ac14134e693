/*
 * keccak_ref.c — Keccak-256 for the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * The reference hashes concrete SHA3 inputs with eth-hash (>=0.3.1,<0.4.0,
 * requirements.txt:13; call site support_utils.py:93-101 via
 * keccak_function_manager.py:57-68), i.e. original Keccak-256 with the 0x01
 * domain pad — NOT NIST SHA3-256 (pad 0x06).  The pad byte is a parameter so
 * the permutation can be cross-checked against hashlib.sha3_256 in tests.
 */
#include <stdint.h>
#include <string.h>
#include <stddef.h>

static const uint64_t RC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull,
    0x8000000080008000ull, 0x000000000000808bull, 0x0000000080000001ull,
    0x8000000080008081ull, 0x8000000000008009ull, 0x000000000000008aull,
    0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull,
    0x8000000000008003ull, 0x8000000000008002ull, 0x8000000000000080ull,
    0x000000000000800aull, 0x800000008000000aull, 0x8000000080008081ull,
    0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

/* rotation offsets r[x][y] and the pi step computed on the fly */
static const int ROT[5][5] = {
    {0, 36, 3, 41, 18}, {1, 44, 10, 45, 2}, {62, 6, 43, 15, 61},
    {28, 55, 25, 21, 56}, {27, 20, 39, 8, 14}};

static inline uint64_t rol(uint64_t v, int r) { return r ? (v << r) | (v >> (64 - r)) : v; }

static void keccak_f(uint64_t A[25]) {  /* A[x + 5y] */
    for (int round = 0; round < 24; ++round) {
        uint64_t C[5], D[5], B[25];
        for (int x = 0; x < 5; ++x)
            C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
        for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rol(C[(x + 1) % 5], 1);
        for (int i = 0; i < 25; ++i) A[i] ^= D[i % 5];
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y)
                B[y + 5 * ((2 * x + 3 * y) % 5)] = rol(A[x + 5 * y], ROT[x][y]);
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y)
                A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
        A[0] ^= RC[round];
    }
}

void orc_keccak256_pad(const uint8_t *in, size_t len, uint8_t pad, uint8_t out[32]) {
    uint64_t A[25];
    memset(A, 0, sizeof A);
    const size_t rate = 136;
    while (len >= rate) {
        for (size_t i = 0; i < rate / 8; ++i) {
            uint64_t v = 0;
            for (int b = 0; b < 8; ++b) v |= (uint64_t)in[8 * i + b] << (8 * b);
            A[i] ^= v;
        }
        keccak_f(A);
        in += rate; len -= rate;
    }
    uint8_t block[136];
    memset(block, 0, sizeof block);
    memcpy(block, in, len);
    block[len] ^= pad;
    block[rate - 1] ^= 0x80;
    for (size_t i = 0; i < rate / 8; ++i) {
        uint64_t v = 0;
        for (int b = 0; b < 8; ++b) v |= (uint64_t)block[8 * i + b] << (8 * b);
        A[i] ^= v;
    }
    keccak_f(A);
    for (int i = 0; i < 4; ++i)
        for (int b = 0; b < 8; ++b) out[8 * i + b] = (uint8_t)(A[i] >> (8 * b));
}

void orc_keccak256(const uint8_t *in, size_t len, uint8_t out[32]) {
    orc_keccak256_pad(in, len, 0x01, out);
}
