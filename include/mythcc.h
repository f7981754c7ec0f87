/*
 * mythcc — the native host compiler: get_model constraint DAG -> mythgpu IR
 * program (include/mythgpu_ir.h).  Host-only C++ (no GPU), one call per
 * independent constraint group.
 *
 * It computes exactly what mythril_amd/ir.py `compile_constraints` (with
 * mythril_amd/solve.py for search mode) computes — the same lowering,
 * model construction, schedule, register allocation, constant table and
 * leaf pools, instruction for instruction (tests/test_native_compiler.py
 * compares the two on every DAG the test corpora hold) — in a fraction of
 * the time: the reference's get_model (mythril/support/model.py:15-49) is
 * called once per JUMPI and transaction end (mythril/laser/ethereum/svm.py:
 * 201-203, 257-262, mythril/analysis/solver.py:6, mythril/laser/ethereum/
 * state/constraints.py:5/:32), and on a GPU miss the compile is pure
 * latency in front of z3.
 *
 * Input: the source DAG (hash-consed SMT terms, mythril_amd/smt/node.py) as
 * flat arrays in topological order (operands before users), node indices
 * 0..n_nodes-1.  Operator names are the SMT-LIB names listed by
 * mgc_source_ops() (index = op code); an operator outside that list is
 * passed as MGC_SOP_OTHER with its name in `str` (lowering it raises
 * "unsupported").
 */
#ifndef MYTHCC_H
#define MYTHCC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGC_OK 0
#define MGC_UNSUPPORTED 1      /* the group needs z3 (ir.Unsupported)          */
#define MGC_ERROR 2            /* malformed input / internal error            */

#define MGC_MAX_SOURCE_WIDTH 65536   /* widths outside [1, this] are rejected */

#define MGC_SORT_BV 0
#define MGC_SORT_BOOL 1
#define MGC_SORT_ARRAY 2

/* leaf eviction policy (ir.LEAF_REMAT) */
#define MGC_REMAT_SPILL 0
#define MGC_REMAT_SCRATCH 1    /* "scratch" / "scratchK" (remat_k = K)         */
#define MGC_REMAT_ALWAYS 2

typedef struct mgc_input {
    int32_t n_nodes;
    const int32_t* op;         /* source op code (mgc_source_ops index)       */
    const int32_t* sort;       /* MGC_SORT_*                                  */
    const int32_t* width;      /* BV width, 1 for Bool, range width for arrays */
    const int32_t* dom;        /* array domain width, else 0                  */
    const int64_t* id;         /* hash-consing id (creation order)            */
    const int32_t* arg_off;    /* n_nodes + 1 offsets into args               */
    const int32_t* args;       /* operand node indices                        */
    const int64_t* p0;         /* extract hi / zero_extend k / sign_extend k / apply domain */
    const int64_t* p1;         /* extract lo                                  */
    const int32_t* str;        /* var / array / function / unknown-op name index, or -1 */
    const int32_t* cval_off;   /* bvnum: offset of its value limbs in cval, else -1 */
    const uint32_t* cval;      /* little-endian 32-bit limbs, ceil(width/32) per numeral */
    const char* strings;       /* n_strings NUL-terminated names, back to back */
    int32_t n_strings;
    int32_t n_cons;
    const int32_t* cons;       /* constraint node indices (Bool)              */
    int32_t n_probes;
    const int32_t* probes;     /* probe node indices                          */
    int32_t n_tables;          /* initial table sizes (ir table_sizes)        */
    const int32_t* table_name; /* string index per table                      */
    const int32_t* table_size;
    int32_t default_entries;
    int32_t nreg;
    int32_t n_extra;           /* extra constants, 8 limbs each (mod 2^256)   */
    const uint32_t* extra;
    int32_t leaf_pools;
    int32_t const_keys;
    int32_t solve;
    int32_t remat_mode;        /* MGC_REMAT_*                                 */
    int32_t remat_k;
    int32_t keep_clean;
    /* search mode (mythril_amd/model.py _compile_search_uncached):
     * search_hints: add every numeral of the constraints (rounded up to a
     *   multiple of 64, and small ones as 4-byte selectors) to the constant
     *   pool (model.harvest_hints);
     * abi_presets: pin the ABI offset words of calldata arrays read at
     *   symbolic offsets and compile the query under those presets
     *   (mythril_amd/abi.py plan / view); the presets come back in the
     *   metadata ("presets"). */
    int32_t search_hints;
    int32_t abi_presets;
    int32_t n_cval;            /* length of cval (limbs)                       */
    int32_t n_string_bytes;    /* length of strings (bytes)                    */
} mgc_input;

typedef struct mgc_result mgc_result;

/* Operator names, '\n'-separated, in op-code order. */
const char* mgc_source_ops(void);

/* Compile.  Returns MGC_OK / MGC_UNSUPPORTED / MGC_ERROR; *out is set in
 * every case (mgc_error() holds the message) and must be freed. */
int mgc_compile(const mgc_input* in, mgc_result** out);

const char* mgc_error(const mgc_result* r);
/* n_ins x 4 instruction words (mythgpu_ir.h layout) */
const uint32_t* mgc_code(const mgc_result* r, int32_t* n_ins);
/* constant table: n_rows x 8 limbs; the first n_const_values rows are the
 * CONST values (ascending), the rest the leaf pools */
const uint32_t* mgc_table(const mgc_result* r, int32_t* n_rows, int32_t* n_const_values);
/* everything else as one JSON object:
 *   leaves        [[name, width, kind, source, chunk, entry], ...] in leaf
 *                 index order (kind: var | key | val | else | cval | aux)
 *   n_lds, n_probes, n_roots, n_user_probes
 *   table_sizes   [[name, entries], ...]; table_kinds [[name, array|func]]
 *   table_ckeys   [[name, [hex key, ...]], ...] (constant-keyed entries)
 *   pool_ranges   [[offset, count], ...] per leaf, rows of the table
 *   derived       [[leaf index, probe index], ...] (search mode)
 *   entry_keys    [[table, [[probe index per 256-bit key chunk], ...]], ...]
 *   lnodes, spills, reloads, hist [[op, count]], hist_order [op, ...]
 *   presets       {"vars": [[name, hex]], "arrays": [[name, [[offset, byte]]]]}
 *                 (abi_presets, when offsets were pinned) */
const char* mgc_meta(const mgc_result* r);
void mgc_free(mgc_result* r);

#ifdef __cplusplus
}
#endif

#endif
