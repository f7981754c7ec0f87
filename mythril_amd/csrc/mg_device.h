/* Structures shared by the HIP kernels (mg_interp_asm.hip) and the C-ABI host
 * layer (mg_api.cpp).  Device-resident; never crosses the C ABI. */
#ifndef MG_DEVICE_H
#define MG_DEVICE_H

#include <stdint.h>
#include "mythgpu.h"

/* LDS spill area of one 256-lane block: n_lds REGIONS of 8 KiB, each two
 * 4 KiB HALVES laid out [lane] x 16 B (conflict-free ds_*_b128).  The
 * translator places a 256-bit value in any two free halves and a one-limb
 * value in one dword of a half (mg_host.cpp place_spills).  With six regions
 * (the default tier: 3 blocks x 48 KiB of the CU's 160 KiB) a 13th half
 * fills the CU to 3 x 52 KiB. */
#define MG_BLOCK_LANES 256u
static inline uint32_t mg_lds_halves(uint32_t n_lds) {
    return 2u * n_lds + (n_lds == 6u ? 1u : 0u);
}
static inline uint32_t mg_lds_half_offset(uint32_t h) {   /* byte offset of lane 0 */
    return h * MG_BLOCK_LANES * 16u;
}
/* the last dword of the last half a context can use fits a DS offset */
static_assert((2u * MG_MAX_LDS_DS - 1u) * MG_BLOCK_LANES * 16u + 12u <= 0xFFFFu,
              "LDS halves beyond a DS instruction's 16-bit offset");
static inline uint32_t mg_lds_bytes(uint32_t n_lds) {
    return mg_lds_halves(n_lds) * MG_BLOCK_LANES * 16u;
}

/* Device form of a leaf generator descriptor (mg_leafgen + host-computed
 * fields): 8 words, read by the kernels with one scalar load. */
struct mg_leafgen_dev {
    uint32_t width;
    uint32_t pool_off_b;       /* byte offset (from the const table) of the
                                  leaf's pool expanded to v-1, v, v+1 triples */
    uint32_t pool_n;
    uint32_t pct_uniform, pct_small, pct_boundary;
    uint32_t salt_lo, salt_hi; /* prog_seed*C1 ^ (leaf+1)*C2 (oracle/gen_ref) */
};

/* One loaded program as the kernel sees it (read with scalar loads). */
struct mg_pdesc {
    const uint32_t* code;      /* n_ins x 4 words (IR)                      */
    const uint32_t* consts;    /* n_consts x 8 words (+ translator masks)  */
    const mg_leafgen_dev* gen; /* n_leaves generator descriptors           */
    uint32_t n_ins;
    uint32_t n_leaves;
    uint32_t n_lds;            /* LDS spill slots                          */
    uint32_t n_probes;
    uint64_t prog_seed;        /* per-program stream salt (generator mode) */
    const uint32_t* xcode;     /* translated 8-word records (mg_interp_asm) */
    const uint32_t* btab;      /* generator boundary table (context-wide):
                                  [kind 0..5][p 0..255] x 8 words, see
                                  mg_boundary_table in mg_api.cpp         */
    uint64_t jit_entry;        /* compiled program (mythril_amd/jit.py,
                                  mg_jit_attach): code address the kernel
                                  calls instead of interpreting the records;
                                  0 = interpret                            */
};
static_assert(__builtin_offsetof(mg_pdesc, consts) == 0x8 &&
              __builtin_offsetof(mg_pdesc, xcode) == 0x30 &&
              __builtin_offsetof(mg_pdesc, btab) == 0x38 &&
              __builtin_offsetof(mg_pdesc, jit_entry) == 0x40,
              "mg_pdesc layout is read by the assembly (asmgen.PDESC_*)");

/* Per-launch arguments (passed by value). */
struct mg_run {
    const uint32_t* leaves;    /* SoA [leaf][limb][stride]  (eval mode)    */
    uint64_t stride;           /* assignments per limb row (eval/probes)   */
    uint64_t n_assign;         /* lanes to evaluate per program            */
    uint64_t* root_bits;       /* [prog][words_per_prog]                   */
    uint64_t words_per_prog;
    uint32_t* probes;          /* [probe][limb][stride] (single program)   */
    unsigned long long* first_sat; /* [prog], atomicMin of candidate index */
    uint32_t* leaves_out;      /* generator mode: dump generated leaves    */
    uint64_t seed;             /* generator seed                           */
    uint64_t first_index;      /* candidate index of lane 0                */
    uint32_t skip_solved;      /* search: a wave whose first candidate index
                                  is at or beyond its program's first_sat
                                  (read with a memory-side atomic, so hits
                                  of other XCDs in the same launch count)
                                  returns at once                          */
    const uint64_t* first_per_prog; /* witness regeneration: program p's
                                  candidate index (first_index ignored);
                                  ~0 = unsolved, the program returns      */
    uint64_t lout_prog_words;  /* leaves_out stride between programs       */
    uint64_t probe_prog_words; /* witness regeneration: probes stride
                                  between programs (0: one program)        */
};

#endif
