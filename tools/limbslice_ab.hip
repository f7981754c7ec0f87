// A/B of the two data layouts for 256-bit lane arithmetic (SURVEY §7.1.4(ii),
// DESIGN.md §7 "limb-sliced layout"): the engine's lane-per-candidate layout
// (one candidate per lane, its 8 limbs in 8 VGPRs) against the limb-sliced
// layout north_star names ("wavefront-level carry propagation": 8 lanes per
// candidate, one limb per lane, carries and comparisons resolved across the
// 8 lanes with DPP row shifts).  Both kernels run the same per-candidate
// chain — x = x + y; y = y ^ x; acc += (x <u y) — over the same inputs, and
// both results are checked against a host model, so the A/B compares
// correct code.  Reported: candidate-iterations per second and VALU
// instructions per candidate-iteration (from the kernels' code, counted by
// the host from the disassembly is not needed: the rate is what matters).
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/limbslice_ab.hip -o tools/limbslice_ab
// Run:   tools/limbslice_ab            (prints one JSON line)

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

static const int ITERS = 256;

// ---- lane per candidate ---------------------------------------------------
__global__ __launch_bounds__(256) void lane_kernel(const uint32_t* __restrict__ xin,
                                                   const uint32_t* __restrict__ yin,
                                                   uint32_t* __restrict__ out, int n) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    uint32_t x[8], y[8];
#pragma unroll
    for (int k = 0; k < 8; k++) { x[k] = xin[8 * c + k]; y[k] = yin[8 * c + k]; }
    uint32_t acc = 0;
    for (int it = 0; it < ITERS; it++) {
        // x = x + y (carry chain)
        uint32_t carry = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            uint64_t s = (uint64_t)x[k] + y[k] + carry;
            x[k] = (uint32_t)s;
            carry = (uint32_t)(s >> 32);
        }
        // y ^= x
#pragma unroll
        for (int k = 0; k < 8; k++) y[k] ^= x[k];
        // acc += x <u y (borrow chain)
        uint32_t borrow = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            uint64_t d = (uint64_t)x[k] - y[k] - borrow;
            borrow = (uint32_t)(d >> 63);
        }
        acc += borrow;
    }
#pragma unroll
    for (int k = 0; k < 8; k++) out[8 * c + k] = x[k];
    out[8 * n + c] = acc;
}

// ---- limb-sliced: 8 lanes per candidate --------------------------------------
// DPP row_shr:d within each 16-lane row; lanes whose source would cross their
// 8-lane group take `fill` (k < d).
template <int D>
__device__ __forceinline__ uint32_t shr_grp(uint32_t v, int k, uint32_t fill) {
    uint32_t s = (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x110 + D, 0xf, 0xf, false);
    return k >= D ? s : fill;
}
template <int D>
__device__ __forceinline__ uint32_t shl_grp(uint32_t v, int k, uint32_t fill) {
    uint32_t s = (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x100 + D, 0xf, 0xf, false);
    return k + D < 8 ? s : fill;
}

__global__ __launch_bounds__(256) void slice_kernel(const uint32_t* __restrict__ xin,
                                                    const uint32_t* __restrict__ yin,
                                                    uint32_t* __restrict__ out, int n) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    int c = t >> 3, k = t & 7;                 // candidate, limb
    if (c >= n) return;
    uint32_t x = xin[8 * c + k], y = yin[8 * c + k];
    uint32_t acc = 0;
    for (int it = 0; it < ITERS; it++) {
        // x = x + y: per-limb sum, then carries by a Kogge-Stone prefix over
        // the group's (generate, propagate) pairs
        uint32_t s = x + y;
        uint32_t g = s < x, p = s == 0xFFFFFFFFu;
        uint32_t g1 = shr_grp<1>(g, k, 0), p1 = shr_grp<1>(p, k, 1);
        g = g | (p & g1); p = p & p1;
        uint32_t g2 = shr_grp<2>(g, k, 0), p2 = shr_grp<2>(p, k, 1);
        g = g | (p & g2); p = p & p2;
        uint32_t g4 = shr_grp<4>(g, k, 0);
        g = g | (p & g4);
        uint32_t cin = shr_grp<1>(g, k, 0);     // carry into limb k = carry out of 0..k-1
        x = s + cin;
        y ^= x;
        // x <u y: the highest limb where they differ decides (suffix scan of
        // (lt, eq) from limb 7 down), the group's answer read at limb 0
        uint32_t lt = x < y, eq = x == y;
        uint32_t l1 = shl_grp<1>(lt, k, 0), e1 = shl_grp<1>(eq, k, 1);
        lt = l1 | (e1 & lt); eq = eq & e1;
        uint32_t l2 = shl_grp<2>(lt, k, 0), e2 = shl_grp<2>(eq, k, 1);
        lt = l2 | (e2 & lt); eq = eq & e2;
        uint32_t l4 = shl_grp<4>(lt, k, 0), e4 = shl_grp<4>(eq, k, 1);
        lt = l4 | (e4 & lt);
        acc += lt;                              // meaningful at k == 0
    }
    out[8 * c + k] = x;
    if (k == 0) out[8 * n + c] = acc;
}

// ---- host model ---------------------------------------------------------------
static void model(const uint32_t* xin, const uint32_t* yin, uint32_t* out, int n) {
    for (int c = 0; c < n; c++) {
        uint32_t x[8], y[8];
        memcpy(x, xin + 8 * c, 32);
        memcpy(y, yin + 8 * c, 32);
        uint32_t acc = 0;
        for (int it = 0; it < ITERS; it++) {
            uint64_t carry = 0;
            for (int k = 0; k < 8; k++) { uint64_t s = (uint64_t)x[k] + y[k] + carry; x[k] = (uint32_t)s; carry = s >> 32; }
            for (int k = 0; k < 8; k++) y[k] ^= x[k];
            int lt = 0;
            for (int k = 7; k >= 0; k--) if (x[k] != y[k]) { lt = x[k] < y[k]; break; }
            acc += lt;
        }
        memcpy(out + 8 * c, x, 32);
        out[8 * n + c] = acc;
    }
}

int main() {
    const int n = 1 << 20;                      // candidates
    std::vector<uint32_t> xin(8 * (size_t)n), yin(8 * (size_t)n);
    uint64_t s = 0x6d797468;
    auto next = [&]() { s += 0x9E3779B97F4A7C15ull; uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return z ^ (z >> 31); };
    for (size_t i = 0; i < xin.size(); i++) {
        uint64_t r = next();
        xin[i] = (uint32_t)r;
        // some all-ones limbs so carries ripple across lanes
        yin[i] = (r >> 60) == 0 ? 0xFFFFFFFFu : (uint32_t)(r >> 32);
    }
    uint32_t *dx, *dy, *da, *db;
    size_t bytes = 8 * (size_t)n * 4, obytes = 9 * (size_t)n * 4;
    CHK(hipMalloc(&dx, bytes)); CHK(hipMalloc(&dy, bytes));
    CHK(hipMalloc(&da, obytes)); CHK(hipMalloc(&db, obytes));
    CHK(hipMemcpy(dx, xin.data(), bytes, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dy, yin.data(), bytes, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    auto run = [&](bool sliced, int reps) {
        dim3 block(256), grid(sliced ? (8 * n + 255) / 256 : (n + 255) / 256);
        for (int w = 0; w < 2; w++) {
            if (sliced) hipLaunchKernelGGL(slice_kernel, grid, block, 0, 0, dx, dy, db, n);
            else hipLaunchKernelGGL(lane_kernel, grid, block, 0, 0, dx, dy, da, n);
        }
        CHK(hipEventRecord(e0));
        for (int r = 0; r < reps; r++) {
            if (sliced) hipLaunchKernelGGL(slice_kernel, grid, block, 0, 0, dx, dy, db, n);
            else hipLaunchKernelGGL(lane_kernel, grid, block, 0, 0, dx, dy, da, n);
        }
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        return ms / reps;
    };
    float ms_lane = run(false, 10), ms_slice = run(true, 10);
    std::vector<uint32_t> a(9 * (size_t)n), b(9 * (size_t)n), want(9 * (size_t)n);
    CHK(hipMemcpy(a.data(), da, obytes, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(b.data(), db, obytes, hipMemcpyDeviceToHost));
    const int nchk = 1 << 14;                   // host model on a prefix
    model(xin.data(), yin.data(), want.data(), nchk);
    bool ok_lane = true, ok_slice = true;
    for (int c = 0; c < nchk; c++) {
        for (int k = 0; k < 8; k++) {
            ok_lane &= a[8 * c + k] == want[8 * c + k];
            ok_slice &= b[8 * c + k] == want[8 * c + k];
        }
        ok_lane &= a[8 * (size_t)n + c] == want[8 * (size_t)nchk + c];
        ok_slice &= b[8 * (size_t)n + c] == want[8 * (size_t)nchk + c];
    }
    double work = (double)n * ITERS;            // candidate-iterations (add + xor + ult)
    printf("{\"candidates\": %d, \"iterations\": %d, \"lane_ms\": %.3f, \"slice_ms\": %.3f, "
           "\"lane_cand_iters_per_s\": %.4g, \"slice_cand_iters_per_s\": %.4g, "
           "\"lane_over_slice\": %.2f, \"lane_correct\": %s, \"slice_correct\": %s}\n",
           n, ITERS, ms_lane, ms_slice, work / (ms_lane * 1e-3), work / (ms_slice * 1e-3),
           ms_slice / ms_lane, ok_lane ? "true" : "false", ok_slice ? "true" : "false");
    return (ok_lane && ok_slice) ? 0 : 1;
}
