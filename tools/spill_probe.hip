// Spill-placement probe (gfx950): where should the interpreter's spill
// slots live so that their traffic stays in the XCD's L2?
//
// Every kernel runs at the interpreter's occupancy (256-lane blocks, 168
// VGPRs -> 3 waves/SIMD) and has each lane write S 32-byte slots and read
// them back, R rounds (the spill / reload pattern of a program whose values
// do not fit the register file).  Three placements:
//   scratch : per-lane private memory (scratch_store/load, hardware scratch
//             wave slots), what mg_interp_asm uses beyond the LDS tier;
//   hwid    : a global buffer indexed by the wave's hardware slot
//             (XCC, SE, SH, CU, SIMD, wave id from s_getreg), wave-contiguous
//             [slot][half][lane] x 16 B;
//   block   : a global buffer indexed by blockIdx (every block its own area:
//             the footprint of a launch, no reuse across blocks).
// The host prints wall time per dispatch; HBM bytes per dispatch come from
// separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/profile_spill.sh).
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/spill_probe.hip -o tools/spill_probe

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

#define MAXS 32
#define CLOBBER_TO_168 "v100", "v120", "v140", "v160", "v167"

// wave's hardware slot: XCC_ID (reg 20) and HW_ID (reg 4) fields
__device__ __forceinline__ uint32_t hw_slot() {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7;
    const uint32_t wave = hw & 15, simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1,
                   se = (hw >> 13) & 7;
    return (((((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd) * 16) + wave;
}

__global__ __launch_bounds__(256, 3) void k_scratch(uint32_t* out, int S, int R) {
    uint4 buf[2 * MAXS];
    uint4 acc = make_uint4(threadIdx.x, blockIdx.x, 1, 2);
    for (int r = 0; r < R; ++r) {
        for (int s = 0; s < 2 * S; ++s) {
            uint4 v = acc;
            v.x += s;
            buf[s] = v;
        }
        asm volatile("" ::: "memory");
        for (int s = 0; s < 2 * S; ++s) {
            const uint4 v = buf[s];
            acc.x ^= v.x; acc.y += v.y; acc.z ^= v.z; acc.w += v.w;
        }
    }
    asm volatile("" ::: CLOBBER_TO_168);
    out[blockIdx.x * 256 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

__global__ __launch_bounds__(256, 3) void k_global(uint32_t* out, uint4* area, int S, int R,
                                                   int by_block, uint32_t* max_slot) {
    const uint32_t wave_in_block = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t slot = by_block ? blockIdx.x * 4 + wave_in_block : hw_slot();
    if (lane == 0 && !by_block) atomicMax(max_slot, slot);
    uint4* w = area + (size_t)slot * (2 * MAXS) * 64;      // [slot][half][lane]
    uint4 acc = make_uint4(threadIdx.x, blockIdx.x, 1, 2);
    for (int r = 0; r < R; ++r) {
        for (int s = 0; s < 2 * S; ++s) {
            uint4 v = acc;
            v.x += s;
            w[s * 64 + lane] = v;
        }
        asm volatile("" ::: "memory");
        for (int s = 0; s < 2 * S; ++s) {
            const uint4 v = w[s * 64 + lane];
            acc.x ^= v.x; acc.y += v.y; acc.z ^= v.z; acc.w += v.w;
        }
    }
    asm volatile("" ::: CLOBBER_TO_168);
    out[blockIdx.x * 256 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

int main(int argc, char** argv) {
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const int R = argc > 1 ? atoi(argv[1]) : 8;
    const int blocks = cus * 3 * 16;                 // 16 block generations per CU
    uint32_t *d_out, *d_max;
    uint4* d_area;
    const size_t slots_hw = 8ull * 8 * 2 * 16 * 4 * 16;
    const size_t slots_blk = (size_t)blocks * 4;
    const size_t n_slots = slots_hw > slots_blk ? slots_hw : slots_blk;
    CHK(hipMalloc(&d_out, (size_t)blocks * 256 * 4));
    CHK(hipMalloc(&d_max, 4));
    CHK(hipMemset(d_max, 0, 4));
    CHK(hipMalloc(&d_area, n_slots * 2 * MAXS * 64 * sizeof(uint4)));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    printf("{\"device\": \"%s\", \"cus\": %d, \"blocks\": %d, \"rounds\": %d}\n", prop.name, cus,
           blocks, R);
    const int sizes[] = {2, 4, 6, 8, 12, 16, 24, 32};
    for (int kind = 0; kind < 3; ++kind) {
        for (int S : sizes) {
            for (int rep = 0; rep < 2; ++rep) {
                CHK(hipEventRecord(e0, 0));
                if (kind == 0)
                    hipLaunchKernelGGL(k_scratch, dim3(blocks), dim3(256), 0, 0, d_out, S, R);
                else
                    hipLaunchKernelGGL(k_global, dim3(blocks), dim3(256), 0, 0, d_out, d_area, S, R,
                                       kind == 2, d_max);
                CHK(hipGetLastError());
                CHK(hipEventRecord(e1, 0));
                CHK(hipEventSynchronize(e1));
                float ms;
                CHK(hipEventElapsedTime(&ms, e0, e1));
                if (rep == 1) {
                    const double bytes = 2.0 * blocks * 256.0 * S * 32.0 * R;   // written + read
                    printf("{\"kind\": \"%s\", \"S\": %d, \"ms\": %.4f, \"spill_bytes\": %.4g, "
                           "\"GB_s\": %.1f}\n", kind == 0 ? "scratch" : (kind == 1 ? "hwid" : "block"),
                           S, ms, bytes, bytes / (ms * 1e-3) / 1e9);
                }
            }
        }
    }
    uint32_t mx = 0;
    CHK(hipMemcpy(&mx, d_max, 4, hipMemcpyDeviceToHost));
    printf("{\"max_hw_slot\": %u, \"slots_allocated\": %zu}\n", mx, n_slots);
    return 0;
}
