/* Structures shared by the HIP kernels (mg_kernels.hip) and the C-ABI host
 * layer (mg_api.cpp).  Device-resident; never crosses the C ABI. */
#ifndef MG_DEVICE_H
#define MG_DEVICE_H

#include <stdint.h>
#include "mythgpu.h"

/* One loaded program as the kernel sees it (read with scalar loads). */
struct mg_pdesc {
    const uint32_t* code;      /* n_ins x 4 words                          */
    const uint32_t* consts;    /* n_consts x 8 words                       */
    const mg_leafgen* gen;     /* n_leaves generator descriptors           */
    uint32_t n_ins;
    uint32_t n_leaves;
    uint32_t n_lds;            /* LDS spill slots                          */
    uint32_t n_probes;
    uint64_t prog_seed;        /* per-program stream salt (generator mode) */
};

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
};

#endif
