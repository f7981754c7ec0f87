// Empirical probe of gfx950 VALU/SALU hazards relevant to the assembly
// interpreter, at 1 and 8 waves/SIMD.  Each test computes a value through a
// sequence that may be hazardous and writes it; the host compares with the
// value the ISA semantics give and counts mismatching lanes.
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/hazard_probe.hip -o tools/hazard_probe

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

#define REP 64

// T0: 256-bit add as a back-to-back v_add_co/v_addc carry chain, repeated
__global__ __launch_bounds__(64) void t_carry(uint32_t* out, uint32_t seed) {
    uint32_t x = threadIdx.x * 0x9E3779B9u + seed;
    uint32_t a0 = x, a1 = ~x, a2 = x ^ 0x55555555u, a3 = 0xFFFFFFFFu, a4 = x * 3, a5 = 0xFFFFFFFFu,
             a6 = x >> 3, a7 = 0;
    const uint32_t b = 0xFFFFFFFFu - (threadIdx.x & 3);
    for (int r = 0; r < REP; ++r) {
        asm volatile("v_add_co_u32 %0, vcc, %0, %8\n v_addc_co_u32 %1, vcc, %1, %8, vcc\n"
                     "v_addc_co_u32 %2, vcc, %2, %8, vcc\n v_addc_co_u32 %3, vcc, %3, %8, vcc\n"
                     "v_addc_co_u32 %4, vcc, %4, %8, vcc\n v_addc_co_u32 %5, vcc, %5, %8, vcc\n"
                     "v_addc_co_u32 %6, vcc, %6, %8, vcc\n v_addc_co_u32 %7, vcc, %7, %8, vcc\n"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b) : "vcc");
    }
    uint32_t* o = out + (blockIdx.x * 64 + threadIdx.x) * 8;
    o[0] = a0; o[1] = a1; o[2] = a2; o[3] = a3; o[4] = a4; o[5] = a5; o[6] = a6; o[7] = a7;
}

// T1: v_cmp vcc -> v_cndmask (0 wait states), repeated with changing data
__global__ __launch_bounds__(64) void t_cmpmask(uint32_t* out, uint32_t seed) {
    uint32_t x = threadIdx.x * 0x9E3779B9u + seed, acc = 0;
    for (int r = 0; r < REP; ++r) {
        uint32_t t;
        asm volatile("v_cmp_gt_u32 vcc, %1, %2\n v_cndmask_b32 %0, 0, 1, vcc\n"
                     : "=v"(t) : "v"(x), "v"(x * 7 + (uint32_t)r) : "vcc");
        acc = acc * 2 + t;
        x = x * 1664525u + 1013904223u;
    }
    out[blockIdx.x * 64 + threadIdx.x] = acc;
}

// T2: v_cmp_e64 -> SGPR pair -> v_cndmask_e64 (0 wait states)
__global__ __launch_bounds__(64) void t_cmpsgpr(uint32_t* out, uint32_t seed) {
    uint32_t x = threadIdx.x * 0x9E3779B9u + seed, acc = 0;
    for (int r = 0; r < REP; ++r) {
        uint32_t t;
        asm volatile("v_cmp_gt_u32_e64 s[40:41], %1, %2\n v_cndmask_b32_e64 %0, 0, 1, s[40:41]\n"
                     : "=v"(t) : "v"(x), "v"(x * 7 + (uint32_t)r) : "s40", "s41");
        acc = acc * 2 + t;
        x = x * 1664525u + 1013904223u;
    }
    out[blockIdx.x * 64 + threadIdx.x] = acc;
}

// T3: class selection as in the generator: save exec, block 1 under a mask,
// restore exec, v_cmp_e64 (0 wait) -> s_and exec -> block 2
__global__ __launch_bounds__(64) void t_execcmp(uint32_t* out, uint32_t seed) {
    const uint32_t cls = (threadIdx.x * 37u + seed) % 100u;
    uint32_t v1 = 0, v2 = 0;
    asm volatile(
        "s_mov_b64 s[44:45], exec\n"
        "v_cmp_le_u32_e64 s[40:41], 50, %2\n"
        "v_cmp_gt_u32_e64 s[42:43], %3, %2\n"
        "s_and_b64 s[40:41], s[40:41], s[42:43]\n"
        "s_and_b64 exec, s[40:41], s[44:45]\n"
        "s_cbranch_execz 1f\n"
        "v_mov_b32 %0, 1\n"
        "1:\n"
        "s_mov_b64 exec, s[44:45]\n"
        "v_cmp_le_u32_e64 s[40:41], %3, %2\n"
        "v_cmp_gt_u32_e64 s[42:43], %4, %2\n"
        "s_and_b64 s[40:41], s[40:41], s[42:43]\n"
        "s_and_b64 exec, s[40:41], s[44:45]\n"
        "s_cbranch_execz 2f\n"
        "v_mov_b32 %1, 1\n"
        "2:\n"
        "s_mov_b64 exec, s[44:45]\n"
        : "+v"(v1), "+v"(v2) : "v"(cls), "s"(70u), "s"(85u) : "s40", "s41", "s42", "s43", "s44", "s45", "exec");
    out[blockIdx.x * 64 + threadIdx.x] = v1 | (v2 << 1) | (cls << 8);
}

// T4: SMEM base overwritten right after issue
// (the overwriting value is another valid pointer: a late read gives 10)
__global__ __launch_bounds__(64) void t_smembase(uint32_t* out, const uint32_t* tab) {
    uint32_t r;
    asm volatile(
        "s_mov_b64 s[40:41], %1\n"
        "s_load_dword s42, s[40:41], 0x4\n"
        "s_mov_b64 s[40:41], %2\n"
        "s_waitcnt lgkmcnt(0)\n"
        "v_mov_b32 %0, s42\n"
        : "=v"(r) : "s"(tab), "s"(tab + 2) : "s40", "s41", "s42");
    out[blockIdx.x * 64 + threadIdx.x] = r;
}

static void ref_carry(uint32_t tid, uint32_t seed, uint32_t* o) {
    uint32_t x = tid * 0x9E3779B9u + seed;
    uint32_t a[8] = {x, ~x, x ^ 0x55555555u, 0xFFFFFFFFu, x * 3, 0xFFFFFFFFu, x >> 3, 0};
    const uint32_t b = 0xFFFFFFFFu - (tid & 3);
    for (int r = 0; r < REP; ++r) {
        uint64_t c = 0;
        for (int j = 0; j < 8; ++j) { uint64_t s = (uint64_t)a[j] + b + c; a[j] = (uint32_t)s; c = s >> 32; }
    }
    for (int j = 0; j < 8; ++j) o[j] = a[j];
}

static uint32_t ref_cmp(uint32_t tid, uint32_t seed) {
    uint32_t x = tid * 0x9E3779B9u + seed, acc = 0;
    for (int r = 0; r < REP; ++r) {
        uint32_t t = x > x * 7 + (uint32_t)r;
        acc = acc * 2 + t;
        x = x * 1664525u + 1013904223u;
    }
    return acc;
}

int main() {
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const int waves[] = {1, 8};
    const uint32_t seed = 12345;
    uint32_t *d_out, *d_tab;
    const size_t maxb = (size_t)cus * 4 * 8;
    CHK(hipMalloc(&d_out, maxb * 64 * 8 * 4));
    std::vector<uint32_t> tab = {7, 0xABCD1234u, 9, 10};
    CHK(hipMalloc(&d_tab, 16));
    CHK(hipMemcpy(d_tab, tab.data(), 16, hipMemcpyHostToDevice));
    std::vector<uint32_t> h(maxb * 64 * 8);
    for (int w : waves) {
        const int blocks = cus * 4 * w;
        const size_t n = (size_t)blocks * 64;
        // T0
        hipLaunchKernelGGL(t_carry, dim3(blocks), dim3(64), 0, 0, d_out, seed);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(h.data(), d_out, n * 32, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < n; ++i) {
            uint32_t o[8];
            ref_carry(i % 64, seed, o);
            for (int j = 0; j < 8; ++j) bad += h[i * 8 + j] != o[j];
        }
        printf("{\"test\": \"carry_chain_back_to_back\", \"waves\": %d, \"bad_limbs\": %zu, \"limbs\": %zu}\n", w, bad, n * 8);
        // T1, T2
        for (int k = 0; k < 2; ++k) {
            hipLaunchKernelGGL(k ? t_cmpsgpr : t_cmpmask, dim3(blocks), dim3(64), 0, 0, d_out, seed);
            CHK(hipDeviceSynchronize());
            CHK(hipMemcpy(h.data(), d_out, n * 4, hipMemcpyDeviceToHost));
            bad = 0;
            for (size_t i = 0; i < n; ++i) bad += h[i] != ref_cmp(i % 64, seed);
            printf("{\"test\": \"%s\", \"waves\": %d, \"bad_lanes\": %zu, \"lanes\": %zu}\n",
                   k ? "vcmp_e64_sgpr_then_cndmask" : "vcmp_vcc_then_cndmask", w, bad, n);
        }
        // T3
        hipLaunchKernelGGL(t_execcmp, dim3(blocks), dim3(64), 0, 0, d_out, seed);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(h.data(), d_out, n * 4, hipMemcpyDeviceToHost));
        bad = 0;
        for (size_t i = 0; i < n; ++i) {
            const uint32_t cls = ((uint32_t)(i % 64) * 37u + seed) % 100u;
            const uint32_t want = (cls >= 50 && cls < 70 ? 1u : 0u) | (cls >= 70 && cls < 85 ? 2u : 0u) | (cls << 8);
            bad += h[i] != want;
        }
        printf("{\"test\": \"exec_restore_then_vcmp\", \"waves\": %d, \"bad_lanes\": %zu, \"lanes\": %zu}\n", w, bad, n);
        // T4
        hipLaunchKernelGGL(t_smembase, dim3(blocks), dim3(64), 0, 0, d_out, (const uint32_t*)d_tab);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(h.data(), d_out, n * 4, hipMemcpyDeviceToHost));
        bad = 0;
        for (size_t i = 0; i < n; ++i) bad += h[i] != 0xABCD1234u;
        printf("{\"test\": \"smem_base_overwritten_after_issue\", \"waves\": %d, \"bad_lanes\": %zu}\n", w, bad);
    }
    return 0;
}
