// Second instruction microbenchmark (gfx950): 64-bit moves (plain and
// GPR-indexed), 64-bit compares, packed 2 x 32-bit moves (v_pk_mov_b32), 32-bit integer multiplies, and whether a
// SALU stream of one wave co-issues with a VALU stream of another wave on
// the same SIMD.  Reports SIMD cycles per instruction (2.4 GHz clock).
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/ubench2.hip -o tools/ubench2

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2000
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)
#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

__global__ __launch_bounds__(64) void k_mov64(uint32_t* out, uint32_t s) {   // 128 instrs
    for (int i = 0; i < ITERS; ++i)
        asm volatile(R16("v_mov_b64 v[40:41], v[100:101]\n v_mov_b64 v[42:43], v[102:103]\n"
                         "v_mov_b64 v[44:45], v[104:105]\n v_mov_b64 v[46:47], v[106:107]\n"
                         "v_mov_b64 v[48:49], v[108:109]\n v_mov_b64 v[50:51], v[110:111]\n"
                         "v_mov_b64 v[52:53], v[112:113]\n v_mov_b64 v[54:55], v[114:115]\n")
                     ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49",
                       "v50", "v51", "v52", "v53", "v54", "v55");
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

__global__ __launch_bounds__(64) void k_mov64idx(uint32_t* out, uint32_t s) {  // 16 x (on + 4 + off) = 96
    for (int i = 0; i < ITERS; ++i)
        asm volatile(R16("s_set_gpr_idx_on %0, gpr_idx(SRC0)\n"
                         "v_mov_b64 v[40:41], v[100:101]\n v_mov_b64 v[42:43], v[102:103]\n"
                         "v_mov_b64 v[44:45], v[104:105]\n v_mov_b64 v[46:47], v[106:107]\n"
                         "s_set_gpr_idx_off\n")
                     :: "s"(s) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

__global__ __launch_bounds__(64) void k_cmp64(uint32_t* out, uint32_t s) {    // 128 instrs
    for (int i = 0; i < ITERS; ++i)
        asm volatile(R16("v_cmp_eq_u64_e64 s[40:41], v[100:101], v[102:103]\n"
                         "v_cmp_eq_u64_e64 s[42:43], v[104:105], v[106:107]\n"
                         "v_cmp_eq_u64_e64 s[44:45], v[108:109], v[110:111]\n"
                         "v_cmp_eq_u64_e64 s[46:47], v[112:113], v[114:115]\n"
                         "v_cmp_eq_u64_e64 s[48:49], v[100:101], v[106:107]\n"
                         "v_cmp_eq_u64_e64 s[50:51], v[104:105], v[110:111]\n"
                         "v_cmp_eq_u64_e64 s[52:53], v[108:109], v[114:115]\n"
                         "v_cmp_eq_u64_e64 s[54:55], v[112:113], v[102:103]\n")
                     ::: "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49",
                       "s50", "s51", "s52", "s53", "s54", "s55");
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

__global__ __launch_bounds__(64) void k_pkmov(uint32_t* out, uint32_t s) {    // 128 instrs
    for (int i = 0; i < ITERS; ++i)
        asm volatile(R16("v_pk_mov_b32 v[40:41], v[100:101], v[102:103] op_sel:[1,0]\n"
                         "v_pk_mov_b32 v[42:43], v[104:105], v[106:107] op_sel:[1,0]\n"
                         "v_pk_mov_b32 v[44:45], v[108:109], v[110:111] op_sel:[1,0]\n"
                         "v_pk_mov_b32 v[46:47], v[112:113], v[114:115] op_sel:[1,0]\n"
                         "v_pk_mov_b32 v[48:49], v[100:101], v[106:107] op_sel:[1,0]\n"
                         "v_pk_mov_b32 v[50:51], v[104:105], v[110:111] op_sel:[1,0]\n"
                         "v_pk_mov_b32 v[52:53], v[108:109], v[114:115] op_sel:[1,0]\n"
                         "v_pk_mov_b32 v[54:55], v[112:113], v[102:103] op_sel:[1,0]\n")
                     ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49",
                       "v50", "v51", "v52", "v53", "v54", "v55");
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

__global__ __launch_bounds__(64) void k_mullo(uint32_t* out, uint32_t s) {    // 128
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < ITERS; ++i)
        asm volatile(R16("v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n"
                         "v_mul_lo_u32 %3, %3, %8\n v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n"
                         "v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n")
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "s"(s));
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ __launch_bounds__(64) void k_mulhi(uint32_t* out, uint32_t s) {    // 128
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < ITERS; ++i)
        asm volatile(R16("v_mul_hi_u32 %0, %0, %8\n v_mul_hi_u32 %1, %1, %8\n v_mul_hi_u32 %2, %2, %8\n"
                         "v_mul_hi_u32 %3, %3, %8\n v_mul_hi_u32 %4, %4, %8\n v_mul_hi_u32 %5, %5, %8\n"
                         "v_mul_hi_u32 %6, %6, %8\n v_mul_hi_u32 %7, %7, %8\n")
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "s"(s));
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// mixed: in a 512-thread block (2 waves per SIMD), waves 0-3 run a VALU
// stream and waves 4-7 run an equally long SALU stream (or VALU when
// mode == 0).  Time vs VALU-only tells whether SALU co-issues.
__global__ __launch_bounds__(512) void k_mixed(uint32_t* out, uint32_t s, uint32_t mode) {
    const uint32_t w = threadIdx.x >> 6;
    uint32_t acc = threadIdx.x;
    if (w < 4 || mode == 0) {
        for (int i = 0; i < ITERS; ++i)
            asm volatile(R16("v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
                             "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
                             "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n")
                         : "+v"(acc) : "s"(s));
    } else {
        for (int i = 0; i < ITERS; ++i)
            asm volatile(R16("s_add_u32 s90, s90, %0\n s_add_u32 s91, s91, %0\n s_add_u32 s92, s92, %0\n"
                             "s_add_u32 s93, s93, %0\n s_add_u32 s94, s94, %0\n s_add_u32 s95, s95, %0\n"
                             "s_add_u32 s96, s96, %0\n s_add_u32 s97, s97, %0\n")
                         :: "s"(s) : "s90", "s91", "s92", "s93", "s94", "s95", "s96", "s97", "scc");
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint32_t* d_out;
    CHK(hipMalloc(&d_out, (size_t)cus * 4 * 8 * 64 * 4 + (size_t)cus * 8 * 512 * 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    struct { const char* name; kfn fn; int instrs; } bs[] = {
        {"v_mov_b64", k_mov64, 128}, {"v_mov_b64 gpr_idx (+2 SALU/4)", k_mov64idx, 96},
        {"v_cmp_eq_u64_e64", k_cmp64, 128}, {"v_pk_mov_b32", k_pkmov, 128},
        {"v_mul_lo_u32", k_mullo, 128},
        {"v_mul_hi_u32", k_mulhi, 128}};
    for (auto& b : bs) {
        for (int w : {1, 3, 8}) {
            const int blocks = cus * 4 * w;
            float ms = 0;
            for (int rep = 0; rep < 2; ++rep) {
                CHK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(b.fn, dim3(blocks), dim3(64), 0, 0, d_out, 1u);
                CHK(hipEventRecord(e1, 0));
                CHK(hipEventSynchronize(e1));
                CHK(hipEventElapsedTime(&ms, e0, e1));
            }
            const double cyc = ms * 1e-3 * 2.4e9 / ((double)w * ITERS * b.instrs);
            printf("{\"bench\": \"%s\", \"waves_per_simd\": %d, \"simd_cycles_per_instr\": %.3f}\n",
                   b.name, w, cyc);
        }
    }
    for (int mode = 0; mode < 2; ++mode) {
        float ms = 0;
        for (int rep = 0; rep < 2; ++rep) {
            CHK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k_mixed, dim3(cus), dim3(512), 0, 0, d_out, 1u, (uint32_t)mode);
            CHK(hipEventRecord(e1, 0));
            CHK(hipEventSynchronize(e1));
            CHK(hipEventElapsedTime(&ms, e0, e1));
        }
        printf("{\"bench\": \"%s\", \"ms\": %.4f, \"simd_cycles_per_valu_instr_of_wave0\": %.3f}\n",
               mode ? "VALU wave + SALU wave per SIMD" : "two VALU waves per SIMD", ms,
               ms * 1e-3 * 2.4e9 / ((double)ITERS * 128));
    }
    return 0;
}
