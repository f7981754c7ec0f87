/*
 * libmythgpu — C ABI of the MI355X batched constraint-evaluation engine.
 *
 * Drop-in boundary: the reference's only solver entry point is
 *   mythril/support/model.py:15-49   get_model(constraints, minimize, maximize,
 *                                              enforce_execution_time)
 * which builds a z3.Optimize and calls check()/model() through
 *   mythril/laser/smt/solver/solver.py:47-64  BaseSolver.check / .model.
 * The Python shim (mythril_amd/model.py) keeps get_model's signature and
 * contract and calls this library through ctypes for the witness search; the
 * entries below replace, respectively:
 *   mg_load_program   — Optimize.add(constraints)       solver.py:28-37
 *   mg_search         — Optimize.check() (SAT side)     solver.py:47-57
 *   mg_eval*          — Model.eval over many models     laser/smt/model.py:44-59
 *   mg_keccak256      — find_concrete_keccak            keccak_function_manager.py:43-57
 *
 * All pointers are caller-owned.  Functions return 0 on success and a
 * negative MG_E* code on failure (message: mg_last_error).  No exceptions
 * cross the ABI.  Calls on one mg_ctx are synchronous unless they take a
 * stream argument; use one mg_ctx per host thread.
 */
#ifndef MYTHGPU_H
#define MYTHGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MG_OK 0
#define MG_E_ARG (-1)      /* invalid argument / malformed program          */
#define MG_E_HIP (-2)      /* HIP runtime error                              */
#define MG_E_NODEV (-3)    /* no usable GPU                                  */
#define MG_E_NOMEM (-4)

typedef struct mg_ctx mg_ctx;
typedef struct mg_prog mg_prog;
typedef struct mg_batch mg_batch;
typedef struct mg_jit mg_jit;

/* Device candidate generator for one leaf (free variable / table cell),
 * generator v9 (restated bit-exactly by oracle/gen_ref.py):
 *   salt = prog_seed * 0xD1B54A32D192ED03 ^ (leaf + 1) * 0x8CB92BA72F3D8DD7
 *   ss   = seed ^ salt
 *   s    = (ss ^ index) + 0x9E3779B97F4A7C15        (mod 2^64)
 *   z    = (s ^ (s >> 32)) * 0xBF58476D1CE4E5B9     (mod 2^64)
 *   r0   = z ^ (z >> 32)                            (v5-v8: SplitMix64(ss ^ index))
 *   x    = lo(r0) ^ hi(r0)                          (32 bits)
 *   cls  = mulhi(((lo32(index >> 6) ^ lo32(ss)) * 0x2545F491 mod 2^32)
 *                ^ hi32(ss), 100)                   (one class per leaf per
 *                                                    group of 64 indices: a
 *                                                    wave from a multiple of
 *                                                    64 runs one class's code)
 * and by class (thresholds are cumulative percentages):
 *   pct_uniform <= cls < pct_small   r0 (< 2^64)
 *   pct_small <= cls < pct_boundary  {0, 1, 2^(w-1), 2^256-1, 2^k+1, 2^k-1},
 *                                    kind = mulhi(lo, 6), k = mulhi(lo * 0x9E3779B1, w)
 *   cls >= pct_boundary, pool_n > 0  consts[pool_off + e] + delta - 1,
 *                                    e = mulhi(lo, pool_n), delta = mulhi(lo * 0x85EBCA6B, 3)
 *   otherwise (uniform)              r0 in limbs 0-1; limb pair k = 1..3 is
 *                                    x * C_k + r0 (mod 2^64), C = 0x85EBCA6B,
 *                                    0xC2B2AE35, 0x27D4EB2F
 * every value masked to the leaf's width. */
typedef struct mg_leafgen {
    uint32_t width;
    uint32_t pool_off;
    uint32_t pool_n;
    uint32_t pct_uniform;
    uint32_t pct_small;
    uint32_t pct_boundary;
} mg_leafgen;

typedef struct mg_gen {
    uint64_t seed;          /* stream seed                                  */
    uint64_t first_index;   /* candidate index of the first lane (sharding) */
} mg_gen;

/* One context per (device, host thread).  SURVEY §8b proposed
 * mg_init(uint32_t device_mask, ...) with one context owning several devices;
 * this ABI deliberately takes ONE device index instead:
 *   - the multi-GPU design is one process per GPU (bench.py under
 *     torch.distributed.run) or, inside one process, one context per device
 *     driven from its own host thread (mythril_amd/model.py
 *     batch_search_devices: the C calls release the GIL), so a context never
 *     has to fan a call out over devices itself;
 *   - a context owns one stream, one workspace and one program cache, all
 *     per device; a mask would need per-device copies of each behind one
 *     handle and serialise the devices inside a call.
 * A mask maps onto this by calling mg_init once per set bit.  Every entry
 * point makes the context's device current (hipSetDevice) before it touches
 * device memory, so one thread may drive contexts on different devices.
 * MYTHGPU_LDS_SLOTS (LDS spill regions per lane; default: the layout's,
 * mg_layouts) must be an integer 0..MG_MAX_LDS_DS, else MG_E_ARG.
 *
 * Register layouts: the library holds one assembly
 * interpreter per layout — 16 slots at three waves per SIMD and 11 slots
 * (MG_NREG_W4) in 128 VGPRs at four — and a context runs ONE of them:
 * mg_init_layout(device, nreg) picks it (mg_init = the 16-slot layout).
 * Programs loaded into a context must be compiled for its slot count
 * (mg_load_program refuses a slot index >= nreg), so a caller chooses the
 * layout per batch by choosing the context it loads the batch into. */
int mg_init(int device, mg_ctx** out);
int mg_init_layout(int device, uint32_t nreg, mg_ctx** out);
/* The layouts this library holds (no GPU needed): out[3i..3i+2] = (slots,
 * waves per SIMD, default LDS spill regions) of layout i, for as many as n
 * words hold; returns the number of layouts. */
int mg_layouts(uint32_t* out, uint32_t n);
void mg_free(mg_ctx* ctx);
const char* mg_last_error(const mg_ctx* ctx);
/* Device time (ms, HIP events on the context stream) of the last synchronous
 * mg_eval / mg_eval_gen / mg_search / mg_batch_search: the evaluation or
 * search launches only (no copies, no witness regeneration).  Feeds
 * SolverStatistics' kernel time (reference solver_statistics.py:29-43). */
float mg_last_kernel_ms(const mg_ctx* ctx);
/* CU count, device name; available after mg_init. */
int mg_device_info(mg_ctx* ctx, char* name, size_t name_len, int* n_cus);

/* Upload one compiled program (IR of include/mythgpu_ir.h).  n_spill_slots
 * spill slots are used by SPILL/RELOAD; the first MG_MAX_LDS of them live in
 * LDS, the rest (<= MG_MAX_PSLOTS) in per-lane scratch. */
int mg_load_program(mg_ctx* ctx, const uint32_t* code, uint32_t n_ins,
                    const uint32_t* consts, uint32_t n_consts,
                    const mg_leafgen* leaves, uint32_t n_leaves,
                    uint32_t n_spill_slots, uint32_t n_probes, uint64_t prog_seed,
                    mg_prog** out);
void mg_free_program(mg_prog* prog);

/* Evaluate under caller assignments (host buffers).
 *   leaves_soa : [n_leaves][8][n_assign] u32 limbs, little-endian
 *   root_bits  : [ceil(n_assign/64)] u64, bit i = conjunction of ROOTs
 *   probes     : [n_probes][8][n_assign] u32, or NULL */
int mg_eval(mg_ctx* ctx, const mg_prog* prog, const uint32_t* leaves_soa, uint64_t n_assign,
            uint64_t* root_bits, uint32_t* probes);

/* Evaluate under device-generated assignments (candidate indices
 * gen->first_index ...).  leaves_out: [n_leaves][8][n_assign] or NULL. */
int mg_eval_gen(mg_ctx* ctx, const mg_prog* prog, const mg_gen* gen, uint64_t n_assign,
                uint64_t* root_bits, uint32_t* probes, uint32_t* leaves_out);

/* Witness search: smallest candidate index in [gen->first_index,
 * gen->first_index + n_cand) whose assignment satisfies every ROOT, or -1.
 * witness_leaves ([n_leaves][8], may be NULL) receives its leaf values.  The
 * whole range is queued on the device at once (no host round trip per
 * chunk); waves beyond the first witness found so far exit immediately. */
int mg_search(mg_ctx* ctx, const mg_prog* prog, const mg_gen* gen, uint64_t n_cand,
              int64_t* first_sat, uint32_t* witness_leaves);

/* Corpus batches: many programs, one launch.  Device-pointer API for
 * resident benchmarking; stream is a hipStream_t (NULL = the context's own
 * stream, which the synchronous calls also use).
 *   d_root_bits : device [n_progs][ceil(n_assign/64)] u64 (may be NULL)
 *   d_first_sat : device [n_progs] u64, atomicMin'ed (preset to ~0)
 * Launches may be queued on several caller streams: freeing a program or a
 * batch waits for the last launch on every stream the context has seen
 * before its device block is reused.                                       */
int mg_batch_create(mg_ctx* ctx, const mg_prog* const* progs, uint32_t n_progs, mg_batch** out);
void mg_batch_free(mg_batch* batch);
int mg_batch_eval_gen(mg_ctx* ctx, mg_batch* batch, uint64_t seed, uint64_t first_index,
                      uint64_t n_assign, uint64_t* d_root_bits, uint64_t* d_first_sat,
                      void* stream);

/* Batched witness search (replaces the per-state Constraints.is_possible ->
 * get_model loop at mythril/laser/ethereum/svm.py:201-203 and :257-262):
 * for every program of the batch, the smallest candidate index in
 * [gen->first_index, gen->first_index + n_cand) that satisfies it, or -1, in
 * first_sat[n_progs].  All programs share each launch; waves of programs
 * already solved stop consuming lanes, with no host round trip.
 * witness_leaves (may be NULL): [n_progs][max_leaves][8] u32, the leaf values
 * of each solved program's witness (one regeneration launch for all);
 * max_leaves must be >= the batch's largest leaf count. */
int mg_batch_search(mg_ctx* ctx, mg_batch* batch, const mg_gen* gen, uint64_t n_cand,
                    int64_t* first_sat, uint32_t* witness_leaves, uint32_t max_leaves);
/* mg_batch_search plus, in the same regeneration launch, each solved
 * program's probe values at its witness (witness_probes: [n_progs]
 * [max_probes][8] u32, max_probes >= the batch's largest probe count;
 * witness_leaves must be given too): a solve-mode program's derived leaves
 * and argument-keyed table keys, so a batch of hits needs no per-hit
 * mg_eval_gen (round 5). */
int mg_batch_search_probes(mg_ctx* ctx, mg_batch* batch, const mg_gen* gen, uint64_t n_cand,
                           int64_t* first_sat, uint32_t* witness_leaves, uint32_t max_leaves,
                           uint32_t* witness_probes, uint32_t max_probes);

/* Compiled programs (batch path without interpretive dispatch; built on the
 * host by mythril_amd/jit.py): ``image`` is a gfx950 code object holding the
 * straight-line code of programs[0..n_progs) and their entry table
 * ``mg_jit_table``: row 0 = (MG_JIT_MAGIC, the first 16 hex digits of
 * mg_asm_digest() of the interpreter the code was generated for — pinned
 * registers, descriptor layout), row i + 1 = (entry offset of program i from
 * the table, fingerprint of the records program i was compiled from: every
 * word of its records with handler ids in word 0).  Attaching points each
 * program's descriptor at its code; evaluations of those programs — and
 * batches created afterwards — then run the code instead of dispatching
 * records (same results, same kernel).  MG_E_ARG when the header names
 * another interpreter, an entry lies outside the image's executable sections
 * or a row's fingerprint is not the loaded program's (code compiled for other
 * records — another opcode, variant, operand or constant — is never entered).
 * Same role as mg_load_program for Optimize.add (solver.py:28-37),
 * specialised for the batched evaluation (laser/smt/model.py:44-59). */
#define MG_JIT_MAGIC 0x4D474A4954763033ull   /* "MGJITv03" */
int mg_jit_attach(mg_ctx* ctx, mg_prog* const* progs, uint32_t n_progs, const void* image,
                  size_t image_size, mg_jit** out);
/* Back to the interpreter for those programs; unloads the code object.
 * Free batches created while attached first. */
void mg_jit_detach(mg_jit* jit);

/* Keccak-256 (0x01 padding) of n messages, one GPU lane per message.
 *   data/offsets/lens describe the messages in one host byte buffer;
 *   out: n x 32 bytes. */
int mg_keccak256(mg_ctx* ctx, const uint8_t* data, const uint64_t* offsets,
                 const uint32_t* lens, uint32_t n, uint8_t* out);

/* The HIP runtime this library runs on in this process: hipRuntimeGetVersion
 * and the file of the libamdhip64 it resolved to (a process that loaded
 * PyTorch first binds torch's bundled runtime; bench.py reports both). */
int mg_runtime_info(int* hip_version, char* path, size_t path_len);
/* Library/ABI version (no GPU needed). */
int mg_version(void);
/* Digest of the generated gfx950 assembly the library was built from (no
 * GPU needed; mythril_amd/asmgen.py digest()): of the 16-slot interpreter,
 * and of the interpreter of any layout (NULL for a slot count it lacks). */
const char* mg_asm_digest(void);
const char* mg_asm_digest_layout(uint32_t nreg);
/* Host-only (no GPU): translate a validated IR program compiled for the
 * nreg-slot layout into the 8-word records of that layout's assembly
 * interpreter, given its handler offset table (mg_load_program does this
 * with the table queried from the device).
 *   records: up to (2 * n_ins + 3) x 8 words (a WAITVM record may precede
 *   an instruction); masks: mask entries appended after the
 *   program's n_consts constants (8 words each).  Sizes are returned in
 *   *n_record_words / *n_mask_words; MG_E_ARG when a buffer is too small. */
int mg_translate(const uint32_t* code, uint32_t n_ins, uint32_t n_consts, uint32_t n_lds,
                 uint32_t nreg, const uint32_t* handler_off, uint32_t n_handlers,
                 uint32_t* records, uint32_t max_record_words, uint32_t* n_record_words,
                 uint32_t* masks, uint32_t max_mask_words, uint32_t* n_mask_words);
/* Build configuration (no GPU needed): out[0..3] = version, MG_NREG (the
 * most slots any layout has; mg_layouts lists them), MG_MAX_LDS,
 * MG_MAX_PSLOTS. */
int mg_config(uint32_t* out, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif
