// Instruction-level microbenchmarks for the interpreter design (gfx950).
// Each kernel runs ITERS iterations of a 16x-unrolled inline-asm body; the
// host reports SIMD cycles per body instruction at several waves/SIMD
// (1 wave = 1 block of 64 threads; grid = CUs * 4 * waves blocks).
//
//   int32 VALU peak (independent v_add_u32), carry chains, v_mad_u64_u32,
//   GPR-index moves (gfx950 has no v_movrels), SALU, taken s_cbranch, s_setpc dispatch.
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/ubench.hip -o tools/ubench

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>

#define ITERS 2000
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

// 8 independent v_add_u32 per group, 16 groups per iteration -> 128 instrs
__global__ __launch_bounds__(64) void k_add(uint32_t* out, uint32_t s) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(R16("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n"
                         "v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n"
                         "v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n")
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "s"(s));
    }
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// 256-bit add as a dependent carry chain: 8 instrs per add, 16 adds
__global__ __launch_bounds__(64) void k_addc(uint32_t* out, uint32_t s) {
    uint32_t a0 = threadIdx.x, a1 = 1, a2 = 2, a3 = 3, a4 = 4, a5 = 5, a6 = 6, a7 = 7;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(R16("v_add_co_u32 %0, vcc, %0, %8\n v_addc_co_u32 %1, vcc, %1, %8, vcc\n"
                         "v_addc_co_u32 %2, vcc, %2, %8, vcc\n v_addc_co_u32 %3, vcc, %3, %8, vcc\n"
                         "v_addc_co_u32 %4, vcc, %4, %8, vcc\n v_addc_co_u32 %5, vcc, %5, %8, vcc\n"
                         "v_addc_co_u32 %6, vcc, %6, %8, vcc\n v_addc_co_u32 %7, vcc, %7, %8, vcc\n")
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(s) : "vcc");
    }
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// 4 independent v_mad_u64_u32 per group (8 instrs... 4), 16 groups -> 64 instrs
__global__ __launch_bounds__(64) void k_mad(uint32_t* out, uint32_t s) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint32_t m = threadIdx.x | 1;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(R16("v_mad_u64_u32 %0, s[80:81], %4, %5, %0\n"
                         "v_mad_u64_u32 %1, s[80:81], %4, %5, %1\n"
                         "v_mad_u64_u32 %2, s[80:81], %4, %5, %2\n"
                         "v_mad_u64_u32 %3, s[80:81], %4, %5, %3\n")
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
                     : "v"(m), "s"(s) : "s80", "s81");
    }
    out[blockIdx.x * 64 + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3);
}

// GPR-index read: s_set_gpr_idx_on + 8 v_mov + off, 16 groups -> 160 instrs (128 VALU)
__global__ __launch_bounds__(64) void k_gpridx(uint32_t* out, uint32_t s) {
    uint32_t acc = 0;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(R16("s_set_gpr_idx_on %1, gpr_idx(SRC0)\n"
                         "v_mov_b32 v40, v100\n v_mov_b32 v41, v116\n v_mov_b32 v42, v132\n"
                         "v_mov_b32 v43, v148\n v_mov_b32 v44, v164\n v_mov_b32 v45, v180\n"
                         "v_mov_b32 v46, v196\n v_mov_b32 v47, v212\n"
                         "s_set_gpr_idx_off\n")
                     "v_add_u32 %0, %0, v47\n"
                     : "+v"(acc) : "s"(s)
                     : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v100", "v116",
                       "v132", "v148", "v164", "v180", "v196", "v212");
    }
    out[blockIdx.x * 64 + threadIdx.x] = acc;
}

// one dependent v_add_u32 chain (latency), 128 instrs
__global__ __launch_bounds__(64) void k_dep(uint32_t* out, uint32_t s) {
    uint32_t a0 = threadIdx.x;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(R16("v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
                         "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
                         "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n")
                     : "+v"(a0) : "s"(s));
    }
    out[blockIdx.x * 64 + threadIdx.x] = a0;
}

// GPR-indexed ALU op in place: s_set_gpr_idx_on (SRC0,DST) + 8 v_add + off -> 160 instrs
__global__ __launch_bounds__(64) void k_gpridx_alu(uint32_t* out, uint32_t s) {
    uint32_t acc = 0;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(R16("s_set_gpr_idx_on %1, gpr_idx(SRC0,DST)\n"
                         "v_add_u32 v100, v100, v40\n v_add_u32 v116, v116, v41\n v_add_u32 v132, v132, v42\n"
                         "v_add_u32 v148, v148, v43\n v_add_u32 v164, v164, v44\n v_add_u32 v180, v180, v45\n"
                         "v_add_u32 v196, v196, v46\n v_add_u32 v212, v212, v47\n"
                         "s_set_gpr_idx_off\n")
                     "v_add_u32 %0, %0, v212\n"
                     : "+v"(acc) : "s"(s)
                     : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v100", "v116",
                       "v132", "v148", "v164", "v180", "v196", "v212");
    }
    out[blockIdx.x * 64 + threadIdx.x] = acc;
}

// independent SALU adds, 8 per group, 16 groups -> 128 instrs
__global__ __launch_bounds__(64) void k_salu(uint32_t* out, uint32_t s) {
    uint32_t acc = 0;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(R16("s_add_u32 s90, s90, %1\n s_add_u32 s91, s91, %1\n s_add_u32 s92, s92, %1\n"
                         "s_add_u32 s93, s93, %1\n s_add_u32 s94, s94, %1\n s_add_u32 s95, s95, %1\n"
                         "s_add_u32 s96, s96, %1\n s_add_u32 s97, s97, %1\n")
                     "v_add_u32 %0, %0, s97\n"
                     : "+v"(acc) : "s"(s)
                     : "s90", "s91", "s92", "s93", "s94", "s95", "s96", "s97", "scc");
    }
    out[blockIdx.x * 64 + threadIdx.x] = acc;
}

// taken conditional branch: s_cmp + s_cbranch_scc1 to the next line -> 32 instrs
__global__ __launch_bounds__(64) void k_branch(uint32_t* out, uint32_t s) {
    uint32_t acc = 0;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(R16("s_cmp_eq_u32 %1, %1\n s_cbranch_scc1 1f\n s_nop 0\n 1:\n")
                     "v_add_u32 %0, %0, %1\n"
                     : "+v"(acc) : "s"(s) : "scc");
    }
    out[blockIdx.x * 64 + threadIdx.x] = acc;
}

// computed jump: s_getpc_b64 + s_add_u32 + s_addc_u32 + s_setpc_b64 -> 64 instrs
__global__ __launch_bounds__(64) void k_setpc(uint32_t* out, uint32_t s) {
    uint32_t acc = 0;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(R16("s_getpc_b64 s[90:91]\n s_add_u32 s90, s90, 12\n s_addc_u32 s91, s91, 0\n"
                         "s_setpc_b64 s[90:91]\n")
                     "v_add_u32 %0, %0, %1\n"
                     : "+v"(acc) : "s"(s) : "s90", "s91", "scc");
    }
    out[blockIdx.x * 64 + threadIdx.x] = acc;
}

// scalar load (cached, same address) + wait: 16 x (s_load_dwordx4 + waitcnt) -> 32
__global__ __launch_bounds__(64) void k_sload(uint32_t* out, const uint32_t* p) {
    uint32_t acc = 0;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(R16("s_load_dwordx4 s[92:95], %1, 0x0\n s_waitcnt lgkmcnt(0)\n")
                     "v_add_u32 %0, %0, s93\n"
                     : "+v"(acc) : "s"(p) : "s92", "s93", "s94", "s95");
    }
    out[blockIdx.x * 64 + threadIdx.x] = acc;
}

typedef void (*kfn)(uint32_t*, uint32_t);

struct Bench { const char* name; const void* fn; int instrs; int ptr_arg; };

int main(int argc, char** argv) {
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    double clk_ghz = 2.4;
    Bench bs[] = {
        {"v_add_u32 indep", (const void*)k_add, 128, 0},
        {"v_addc carry chain", (const void*)k_addc, 128, 0},
        {"v_mad_u64_u32 indep4", (const void*)k_mad, 64, 0},
        {"gpr_idx 8-mov read", (const void*)k_gpridx, 160, 0},
        {"v_add_u32 dependent", (const void*)k_dep, 128, 0},
        {"gpr_idx in-place 8 add", (const void*)k_gpridx_alu, 160, 0},
        {"s_add indep", (const void*)k_salu, 128, 0},
        {"s_cbranch taken", (const void*)k_branch, 32, 0},
        {"s_setpc jump", (const void*)k_setpc, 64, 0},
        {"s_load+wait", (const void*)k_sload, 32, 1},
    };
    const int waves[] = {1, 2, 3, 4, 8};
    uint32_t* d_out;
    const size_t max_blocks = (size_t)cus * 4 * 8;
    CHK(hipMalloc(&d_out, max_blocks * 64 * sizeof(uint32_t)));
    CHK(hipMemset(d_out, 0, max_blocks * 64 * sizeof(uint32_t)));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    printf("{\"device\": \"%s\", \"cus\": %d}\n", prop.name, cus);
    for (auto& b : bs) {
        for (int w : waves) {
            const int blocks = cus * 4 * w;
            for (int rep = 0; rep < 2; ++rep) {
                CHK(hipEventRecord(e0, 0));
                if (b.ptr_arg)
                    hipLaunchKernelGGL((void (*)(uint32_t*, const uint32_t*))b.fn, dim3(blocks),
                                       dim3(64), 0, 0, d_out, (const uint32_t*)d_out);
                else
                    hipLaunchKernelGGL((kfn)b.fn, dim3(blocks), dim3(64), 0, 0, d_out, 3u);
                CHK(hipGetLastError());
                CHK(hipEventRecord(e1, 0));
                CHK(hipEventSynchronize(e1));
                float ms;
                CHK(hipEventElapsedTime(&ms, e0, e1));
                if (rep == 1) {
                    // cycles per instruction per SIMD (all waves of that SIMD)
                    const double instrs_per_simd = (double)w * ITERS * b.instrs;
                    const double cyc = ms * 1e-3 * clk_ghz * 1e9 / instrs_per_simd;
                    printf("{\"bench\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, "
                           "\"simd_cycles_per_instr\": %.3f, \"wave_cycles_per_instr\": %.3f}\n",
                           b.name, w, ms, cyc, cyc * w);
                }
            }
        }
    }
    CHK(hipFree(d_out));
    return 0;
}
