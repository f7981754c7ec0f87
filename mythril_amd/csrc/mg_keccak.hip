// Per-lane Keccak-256 (Keccak-f[1600], rate 136, 0x01 padding) — the hash
// the reference computes on the host for concrete SHA3 inputs
// (mythril/laser/ethereum/keccak_function_manager.py:43-57, via
// ethereum.utils.sha3) and, per witness, in _replace_with_actual_sha
// (mythril/analysis/solver.py:119-152).  One lane hashes one message; the
// 25 64-bit lanes of the state stay in VGPRs (50 registers) and the rotates
// lower to v_alignbit pairs.

#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV static __device__ __forceinline__

__constant__ uint64_t kRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

DEV uint64_t rotl64(uint64_t v, int n) { return n ? (v << n) | (v >> (64 - n)) : v; }

DEV void keccak_f(uint64_t* A) {
    // rho rotation offsets indexed by lane x + 5*y
    constexpr int rho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                             25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
#pragma unroll 1
    for (int rnd = 0; rnd < 24; ++rnd) {
        uint64_t C[5], Dd[5], B[25];
#pragma unroll
        for (int x = 0; x < 5; ++x) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
#pragma unroll
        for (int x = 0; x < 5; ++x) Dd[x] = C[(x + 4) % 5] ^ rotl64(C[(x + 1) % 5], 1);
#pragma unroll
        for (int x = 0; x < 5; ++x)
#pragma unroll
            for (int y = 0; y < 5; ++y) {
                const int i = x + 5 * y;
                // B[y, 2x+3y] = rot(A[x,y] ^ D[x], r[x,y])
                B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(A[i] ^ Dd[x], rho[i]);
            }
#pragma unroll
        for (int y = 0; y < 5; ++y)
#pragma unroll
            for (int x = 0; x < 5; ++x)
                A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
        A[0] ^= kRC[rnd];
    }
}

__global__ __launch_bounds__(256) void mg_keccak256_kernel(const uint8_t* __restrict__ data,
                                                           const uint64_t* __restrict__ offsets,
                                                           const uint32_t* __restrict__ lens,
                                                           uint32_t n, uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* msg = data + offsets[i];
    const uint32_t len = lens[i];
    uint64_t A[25];
#pragma unroll
    for (int k = 0; k < 25; ++k) A[k] = 0;
    const uint32_t rate = 136;
    const uint32_t nblocks = len / rate + 1;   // padding always adds a block tail
    for (uint32_t blk = 0; blk < nblocks; ++blk) {
        const uint32_t base = blk * rate;
#pragma unroll
        for (int k = 0; k < 17; ++k) {
            uint64_t lane = 0;
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const uint32_t pos = base + 8 * k + b;
                uint64_t byte = pos < len ? msg[pos] : 0u;
                if (pos == len) byte |= 0x01u;
                if (pos == base + rate - 1 && blk == nblocks - 1) byte |= 0x80u;
                lane |= byte << (8 * b);
            }
            A[k] ^= lane;
        }
        keccak_f(A);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int b = 0; b < 8; ++b) out[(size_t)i * 32 + 8 * k + b] = (uint8_t)(A[k] >> (8 * b));
}

hipError_t mg_launch_keccak(const uint8_t* d_data, const uint64_t* d_off, const uint32_t* d_len,
                            uint32_t n, uint8_t* d_out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(mg_keccak256_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, d_data,
                       d_off, d_len, n, d_out);
    return hipGetLastError();
}
