// VALU issue rates on gfx950 in one harness, clock-independent: every wave
// stamps s_memtime (shader clock) around its loop, so the result is SIMD
// cycles per wave64 instruction = elapsed cycles / (waves on the SIMD x
// instructions per wave), with no assumed clock; s_memrealtime (100 MHz)
// gives the clock the chip actually ran at.  Reconciles the int32 ceiling
// used by mythril_amd/roofline.py with MI355X_MICROARCH.md's "a wave64 VALU
// instruction issues over 2 cycles" (v_fma_f32) — measured, per instruction.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/valu_rate

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <map>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

#define ITERS 4000
#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

struct Stamp { uint64_t t0, t1, r0, r1; uint32_t hw, xcc, pad0, pad1; };

#define BODY8(ins) R16(ins "0\n" ins "1\n" ins "2\n" ins "3\n" ins "4\n" ins "5\n" ins "6\n" ins "7\n")

// 8 independent accumulators v[40..47] (+ v[48..55] for 64-bit ops), 128
// instructions per iteration; the operand is a second register.
#define KERNEL(NAME, TEXT)                                                        \
    __global__ __launch_bounds__(64) void NAME(Stamp* st, uint32_t s) {           \
        asm volatile("v_mov_b32 v60, %0\n v_mov_b32 v61, %0" ::"v"(threadIdx.x)   \
                     : "v60", "v61");                                             \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                         \
        const uint64_t r0 = __builtin_amdgcn_s_memrealtime();                     \
        for (int i = 0; i < ITERS; ++i)                                           \
            asm volatile(R16(TEXT) ::: "v40", "v41", "v42", "v43", "v44", "v45",   \
                         "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53",  \
                         "v54", "v55", "v60", "v61", "vcc");                      \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                         \
        const uint64_t r1 = __builtin_amdgcn_s_memrealtime();                     \
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);            \
        const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);           \
        if (threadIdx.x == 0) st[blockIdx.x] = Stamp{t0, t1, r0, r1, hw, xcc, 0, 0}; \
    }

KERNEL(k_fma_f32, "v_fma_f32 v40, v40, v60, v61\n v_fma_f32 v41, v41, v60, v61\n"
                  "v_fma_f32 v42, v42, v60, v61\n v_fma_f32 v43, v43, v60, v61\n"
                  "v_fma_f32 v44, v44, v60, v61\n v_fma_f32 v45, v45, v60, v61\n"
                  "v_fma_f32 v46, v46, v60, v61\n v_fma_f32 v47, v47, v60, v61\n")
KERNEL(k_pk_fma_f32, "v_pk_fma_f32 v[40:41], v[40:41], v[60:61], v[60:61]\n"
                     "v_pk_fma_f32 v[42:43], v[42:43], v[60:61], v[60:61]\n"
                     "v_pk_fma_f32 v[44:45], v[44:45], v[60:61], v[60:61]\n"
                     "v_pk_fma_f32 v[46:47], v[46:47], v[60:61], v[60:61]\n"
                     "v_pk_fma_f32 v[48:49], v[48:49], v[60:61], v[60:61]\n"
                     "v_pk_fma_f32 v[50:51], v[50:51], v[60:61], v[60:61]\n"
                     "v_pk_fma_f32 v[52:53], v[52:53], v[60:61], v[60:61]\n"
                     "v_pk_fma_f32 v[54:55], v[54:55], v[60:61], v[60:61]\n")
KERNEL(k_add_u32, "v_add_u32 v40, v40, v60\n v_add_u32 v41, v41, v60\n v_add_u32 v42, v42, v60\n"
                  "v_add_u32 v43, v43, v60\n v_add_u32 v44, v44, v60\n v_add_u32 v45, v45, v60\n"
                  "v_add_u32 v46, v46, v60\n v_add_u32 v47, v47, v60\n")
KERNEL(k_add_f32, "v_add_f32 v40, v40, v60\n v_add_f32 v41, v41, v60\n v_add_f32 v42, v42, v60\n"
                  "v_add_f32 v43, v43, v60\n v_add_f32 v44, v44, v60\n v_add_f32 v45, v45, v60\n"
                  "v_add_f32 v46, v46, v60\n v_add_f32 v47, v47, v60\n")
KERNEL(k_xor_b32, "v_xor_b32 v40, v40, v60\n v_xor_b32 v41, v41, v60\n v_xor_b32 v42, v42, v60\n"
                  "v_xor_b32 v43, v43, v60\n v_xor_b32 v44, v44, v60\n v_xor_b32 v45, v45, v60\n"
                  "v_xor_b32 v46, v46, v60\n v_xor_b32 v47, v47, v60\n")
KERNEL(k_pk_mov_b32, "v_pk_mov_b32 v[40:41], v[60:61], v[40:41] op_sel:[0,1]\n"
                     "v_pk_mov_b32 v[42:43], v[60:61], v[42:43] op_sel:[0,1]\n"
                     "v_pk_mov_b32 v[44:45], v[60:61], v[44:45] op_sel:[0,1]\n"
                     "v_pk_mov_b32 v[46:47], v[60:61], v[46:47] op_sel:[0,1]\n"
                     "v_pk_mov_b32 v[48:49], v[60:61], v[48:49] op_sel:[0,1]\n"
                     "v_pk_mov_b32 v[50:51], v[60:61], v[50:51] op_sel:[0,1]\n"
                     "v_pk_mov_b32 v[52:53], v[60:61], v[52:53] op_sel:[0,1]\n"
                     "v_pk_mov_b32 v[54:55], v[60:61], v[54:55] op_sel:[0,1]\n")
KERNEL(k_addc_chain, "v_add_co_u32 v40, vcc, v40, v60\n v_addc_co_u32 v41, vcc, v41, v60, vcc\n"
                     "v_addc_co_u32 v42, vcc, v42, v60, vcc\n v_addc_co_u32 v43, vcc, v43, v60, vcc\n"
                     "v_addc_co_u32 v44, vcc, v44, v60, vcc\n v_addc_co_u32 v45, vcc, v45, v60, vcc\n"
                     "v_addc_co_u32 v46, vcc, v46, v60, vcc\n v_addc_co_u32 v47, vcc, v47, v60, vcc\n")
KERNEL(k_mad_u64, "v_mad_u64_u32 v[40:41], vcc, v60, v61, v[40:41]\n"
                  "v_mad_u64_u32 v[42:43], vcc, v60, v61, v[42:43]\n"
                  "v_mad_u64_u32 v[44:45], vcc, v60, v61, v[44:45]\n"
                  "v_mad_u64_u32 v[46:47], vcc, v60, v61, v[46:47]\n"
                  "v_mad_u64_u32 v[48:49], vcc, v60, v61, v[48:49]\n"
                  "v_mad_u64_u32 v[50:51], vcc, v60, v61, v[50:51]\n"
                  "v_mad_u64_u32 v[52:53], vcc, v60, v61, v[52:53]\n"
                  "v_mad_u64_u32 v[54:55], vcc, v60, v61, v[54:55]\n")


#define IND8(op, tail) op " v40, v40" tail "\n" op " v41, v41" tail "\n" op " v42, v42" tail "\n" \
    op " v43, v43" tail "\n" op " v44, v44" tail "\n" op " v45, v45" tail "\n" op " v46, v46" tail "\n" \
    op " v47, v47" tail "\n"
KERNEL(k_mov_b32, IND8("v_mov_b32", "") )
KERNEL(k_mul_lo_u32, IND8("v_mul_lo_u32", ", v60"))
KERNEL(k_mul_hi_u32, IND8("v_mul_hi_u32", ", v60"))
KERNEL(k_alignbit, IND8("v_alignbit_b32", ", v60, v61"))
KERNEL(k_bfe_u32, IND8("v_bfe_u32", ", 3, 5"))
KERNEL(k_or3_b32, IND8("v_or3_b32", ", v60, v61"))
KERNEL(k_lshl_add, IND8("v_lshl_add_u32", ", 5, v61"))
KERNEL(k_cndmask, IND8("v_cndmask_b32", ", v60, vcc"))
KERNEL(k_sub_co_ind, "v_sub_co_u32 v40, vcc, v40, v60\n v_sub_co_u32 v41, vcc, v41, v60\n"
                     "v_sub_co_u32 v42, vcc, v42, v60\n v_sub_co_u32 v43, vcc, v43, v60\n"
                     "v_sub_co_u32 v44, vcc, v44, v60\n v_sub_co_u32 v45, vcc, v45, v60\n"
                     "v_sub_co_u32 v46, vcc, v46, v60\n v_sub_co_u32 v47, vcc, v47, v60\n")
KERNEL(k_mov_b64, "v_mov_b64 v[40:41], v[60:61]\n v_mov_b64 v[42:43], v[60:61]\n"
                  "v_mov_b64 v[44:45], v[60:61]\n v_mov_b64 v[46:47], v[60:61]\n"
                  "v_mov_b64 v[48:49], v[60:61]\n v_mov_b64 v[50:51], v[60:61]\n"
                  "v_mov_b64 v[52:53], v[60:61]\n v_mov_b64 v[54:55], v[60:61]\n")
KERNEL(k_lshr_b64, "v_lshrrev_b64 v[40:41], 3, v[40:41]\n v_lshrrev_b64 v[42:43], 3, v[42:43]\n"
                   "v_lshrrev_b64 v[44:45], 3, v[44:45]\n v_lshrrev_b64 v[46:47], 3, v[46:47]\n"
                   "v_lshrrev_b64 v[48:49], 3, v[48:49]\n v_lshrrev_b64 v[50:51], 3, v[50:51]\n"
                   "v_lshrrev_b64 v[52:53], 3, v[52:53]\n v_lshrrev_b64 v[54:55], 3, v[54:55]\n")
KERNEL(k_cmp_vcc, "v_cmp_lt_u32 vcc, v40, v60\n v_cmp_lt_u32 vcc, v41, v60\n"
                  "v_cmp_lt_u32 vcc, v42, v60\n v_cmp_lt_u32 vcc, v43, v60\n"
                  "v_cmp_lt_u32 vcc, v44, v60\n v_cmp_lt_u32 vcc, v45, v60\n"
                  "v_cmp_lt_u32 vcc, v46, v60\n v_cmp_lt_u32 vcc, v47, v60\n")

#define KERNEL_S(NAME, TEXT)                                                      \
    __global__ __launch_bounds__(64) void NAME(Stamp* st, uint32_t s) {           \
        asm volatile("v_mov_b32 v60, %0\n v_mov_b32 v61, %0\n s_mov_b64 s[40:41], -1\n" \
                     "v_cmp_lt_u32 vcc, v60, 3" ::"v"(threadIdx.x)                \
                     : "v60", "v61", "s40", "s41", "vcc");                        \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                         \
        const uint64_t r0 = __builtin_amdgcn_s_memrealtime();                     \
        for (int i = 0; i < ITERS; ++i)                                           \
            asm volatile(R16(TEXT) ::: "v40", "v41", "v42", "v43", "v44", "v45",   \
                         "v46", "v47", "v60", "v61", "vcc", "s40", "s41");        \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                         \
        const uint64_t r1 = __builtin_amdgcn_s_memrealtime();                     \
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);            \
        const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);           \
        if (threadIdx.x == 0) st[blockIdx.x] = Stamp{t0, t1, r0, r1, hw, xcc, 0, 0}; \
    }
KERNEL_S(k_cnd_vcc_init, IND8("v_cndmask_b32", ", v60, vcc"))
KERNEL_S(k_cnd_e64_sgpr, IND8("v_cndmask_b32_e64", ", v60, s[40:41]"))
KERNEL_S(k_cnd_e64_vcc, IND8("v_cndmask_b32_e64", ", v60, vcc"))
KERNEL_S(k_cmp_then_cnd, "v_cmp_lt_u32 vcc, v40, v60\n v_cndmask_b32 v40, v40, v61, vcc\n"
                         "v_cmp_lt_u32 vcc, v41, v60\n v_cndmask_b32 v41, v41, v61, vcc\n"
                         "v_cmp_lt_u32 vcc, v42, v60\n v_cndmask_b32 v42, v42, v61, vcc\n"
                         "v_cmp_lt_u32 vcc, v43, v60\n v_cndmask_b32 v43, v43, v61, vcc\n")
KERNEL_S(k_cmp_e64_then_cnd, "v_cmp_lt_u32_e64 s[40:41], v40, v60\n v_cndmask_b32_e64 v40, v40, v61, s[40:41]\n"
                         "v_cmp_lt_u32_e64 s[40:41], v41, v60\n v_cndmask_b32_e64 v41, v41, v61, s[40:41]\n"
                         "v_cmp_lt_u32_e64 s[40:41], v42, v60\n v_cndmask_b32_e64 v42, v42, v61, s[40:41]\n"
                         "v_cmp_lt_u32_e64 s[40:41], v43, v60\n v_cndmask_b32_e64 v43, v43, v61, s[40:41]\n")
KERNEL_S(k_cmp_vcc_only, "v_cmp_lt_u32 vcc, v40, v60\n v_add_u32 v40, v40, v61\n"
                         "v_cmp_lt_u32 vcc, v41, v60\n v_add_u32 v41, v41, v61\n"
                         "v_cmp_lt_u32 vcc, v42, v60\n v_add_u32 v42, v42, v61\n"
                         "v_cmp_lt_u32 vcc, v43, v60\n v_add_u32 v43, v43, v61\n")
KERNEL_S(k_sub_u32, IND8("v_sub_u32", ", v60"))
KERNEL_S(k_and_or, "v_and_b32 v40, v40, v60\n v_or_b32 v41, v41, v60\n v_and_b32 v42, v42, v60\n"
                   "v_or_b32 v43, v43, v60\n v_and_b32 v44, v44, v60\n v_or_b32 v45, v45, v60\n"
                   "v_and_b32 v46, v46, v60\n v_or_b32 v47, v47, v60\n")
KERNEL_S(k_lshl_b32, IND8("v_lshlrev_b32", ", v60"))
KERNEL_S(k_mul_u24, IND8("v_mul_u32_u24", ", v60"))
KERNEL_S(k_add3, IND8("v_add3_u32", ", v60, v61"))
KERNEL_S(k_xor_e64, IND8("v_xor_b32_e64", ", v60"))

struct B { const char* name; void (*fn)(Stamp*, uint32_t); double lane_ops_per_ins; };

int main() {
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    B bs[] = {{"v_fma_f32", k_fma_f32, 1}, {"v_pk_fma_f32", k_pk_fma_f32, 2},
              {"v_add_f32", k_add_f32, 1}, {"v_add_u32", k_add_u32, 1},
              {"v_xor_b32", k_xor_b32, 1}, {"v_pk_mov_b32", k_pk_mov_b32, 2},
              {"v_add/addc_co chain", k_addc_chain, 1}, {"v_mad_u64_u32", k_mad_u64, 1},
              {"v_mov_b32", k_mov_b32, 1}, {"v_mul_lo_u32", k_mul_lo_u32, 1},
              {"v_mul_hi_u32", k_mul_hi_u32, 1}, {"v_alignbit_b32", k_alignbit, 1},
              {"v_bfe_u32", k_bfe_u32, 1}, {"v_or3_b32", k_or3_b32, 1},
              {"v_lshl_add_u32", k_lshl_add, 1}, {"v_cndmask_b32 (vcc)", k_cndmask, 1},
              {"v_sub_co_u32 (independent)", k_sub_co_ind, 1}, {"v_mov_b64", k_mov_b64, 2},
              {"v_lshrrev_b64", k_lshr_b64, 2}, {"v_cmp_lt_u32 (vcc)", k_cmp_vcc, 1},
              {"v_cndmask_b32 vcc (vcc set)", k_cnd_vcc_init, 1},
              {"v_cndmask_b32_e64 s[40:41]", k_cnd_e64_sgpr, 1},
              {"v_cndmask_b32_e64 vcc", k_cnd_e64_vcc, 1},
              {"v_cmp vcc + v_cndmask pair", k_cmp_then_cnd, 1},
              {"v_cmp_e64 sgpr + cndmask pair", k_cmp_e64_then_cnd, 1},
              {"v_cmp vcc + v_add pair", k_cmp_vcc_only, 1},
              {"v_sub_u32", k_sub_u32, 1}, {"v_and/or_b32", k_and_or, 1},
              {"v_lshlrev_b32", k_lshl_b32, 1}, {"v_mul_u32_u24", k_mul_u24, 1},
              {"v_add3_u32", k_add3, 1}, {"v_xor_b32_e64 (VOP3 form)", k_xor_e64, 1}};
    const char* sel = getenv("VALU_RATE_INS");        // substring filter on names
    const char* only = getenv("VALU_RATE_ONLY");       // comma list of wave counts
    std::vector<int> waves = {1, 2, 3, 4, 5, 6, 8};
    if (only) {
        waves.clear();
        for (const char* p = only; *p;) {
            waves.push_back(atoi(p));
            while (*p && *p != ',') ++p;
            if (*p) ++p;
        }
    }
    Stamp* d_st;
    CHK(hipMalloc(&d_st, sizeof(Stamp) * cus * 4 * 8));
    printf("{\"device\": \"%s\", \"cus\": %d, \"instructions_per_wave\": %d}\n", prop.name, cus,
           ITERS * 128);
    for (auto& b : bs) {
        if (sel && !strstr(b.name, sel) && strcmp(sel, "new") != 0) continue;
        if (sel && strcmp(sel, "new") == 0 && b.fn != k_cnd_vcc_init && b.fn != k_cnd_e64_sgpr &&
            b.fn != k_cnd_e64_vcc && b.fn != k_cmp_then_cnd && b.fn != k_cmp_e64_then_cnd &&
            b.fn != k_cmp_vcc_only && b.fn != k_sub_u32 && b.fn != k_and_or && b.fn != k_lshl_b32 &&
            b.fn != k_mul_u24 && b.fn != k_add3 && b.fn != k_xor_e64 && b.fn != k_cndmask)
            continue;
        for (int w : waves) {
            const int blocks = cus * 4 * w;
            double cyc = 0, ghz = 0;
            for (int rep = 0; rep < 3; ++rep) {
                hipLaunchKernelGGL(b.fn, dim3(blocks), dim3(64), 0, 0, d_st, 3u);
                CHK(hipGetLastError());
                CHK(hipDeviceSynchronize());
            }
            std::vector<Stamp> st(blocks);
            CHK(hipMemcpy(st.data(), d_st, sizeof(Stamp) * blocks, hipMemcpyDeviceToHost));
            std::vector<double> c(blocks), g(blocks);
            for (int i = 0; i < blocks; ++i) {
                c[i] = (double)(st[i].t1 - st[i].t0);
                g[i] = c[i] / (double)(st[i].r1 - st[i].r0) * 0.1;   // GHz
            }
            std::sort(c.begin(), c.end());
            std::sort(g.begin(), g.end());
            cyc = c[blocks / 2];
            ghz = g[blocks / 2];
            // per SIMD (XCC, SE, SH, CU, SIMD from HW_ID): instructions of all
            // its waves over the span from the first start to the last end;
            // independent of how many waves were co-resident
            std::map<uint64_t, std::pair<std::pair<uint64_t, uint64_t>, int>> simd;
            for (int i = 0; i < blocks; ++i) {
                const uint32_t hw = st[i].hw;
                const uint64_t key = ((uint64_t)(st[i].xcc & 15) << 16) | (((hw >> 13) & 7) << 12) |
                                     (((hw >> 12) & 1) << 11) | (((hw >> 8) & 15) << 4) |
                                     ((hw >> 4) & 3);
                auto it = simd.find(key);
                if (it == simd.end())
                    simd[key] = {{st[i].t0, st[i].t1}, 1};
                else {
                    it->second.first.first = std::min(it->second.first.first, st[i].t0);
                    it->second.first.second = std::max(it->second.first.second, st[i].t1);
                    it->second.second += 1;
                }
            }
            std::vector<double> tput;
            int maxw = 0;
            for (auto& kv : simd) {
                const double span = (double)(kv.second.first.second - kv.second.first.first);
                tput.push_back(kv.second.second * (double)ITERS * 128 / span);
                maxw = std::max(maxw, kv.second.second);
            }
            std::sort(tput.begin(), tput.end());
            const double ipc = tput[tput.size() / 2];
            // a wave's loop spans all w co-resident waves of its SIMD
            const double per_ins = cyc / ((double)w * ITERS * 128);
            printf("{\"ins\": \"%s\", \"waves_per_simd\": %d, \"simds_seen\": %zu, "
                   "\"max_waves_on_a_simd\": %d, \"simd_ins_per_cycle\": %.3f, "
                   "\"simd_cycles_per_ins\": %.3f, \"wave_cycles_per_ins\": %.3f, "
                   "\"clock_ghz\": %.3f, \"chip_lane_ops_per_s_T_at_2_4GHz\": %.2f}\n",
                   b.name, w, simd.size(), maxw, ipc, 1.0 / ipc, cyc / ((double)ITERS * 128), ghz,
                   256.0 * 4 * 64 * b.lane_ops_per_ins * ipc * 2.4e9 / 1e12);
            (void)per_ins;
        }
    }
    return 0;
}
