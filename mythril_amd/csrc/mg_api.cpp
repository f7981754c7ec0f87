// C ABI of libmythgpu (include/mythgpu.h).  Host-side validation, device
// memory management and kernel launches.  Every program is validated before
// upload so that no instruction can index outside the register file, the LDS
// spill area, the constant pool, the leaf table or the probe buffer.

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <algorithm>
#include <vector>

#include <cstddef>
#include <cstdlib>
#include <map>
#include <elf.h>
#include <dlfcn.h>

#include "mythgpu.h"
#include "mythgpu_ir.h"
#include "mg_device.h"
#include "mg_asm_handlers.h"
#include "mg_host.h"

// the interpreter of each register layout (mg_interp_asm.hip, one
// translation unit per layout; mg_find_layout lists them)
typedef hipError_t (*mg_launch_fn)(const mg_pdesc* d_descs, uint32_t n_progs, const mg_run& run,
                                   uint32_t mode, uint32_t lds_slots, uint32_t* table,
                                   hipStream_t stream);
hipError_t mg_launch_asm_r16(const mg_pdesc*, uint32_t, const mg_run&, uint32_t, uint32_t, uint32_t*,
                             hipStream_t);
hipError_t mg_launch_asm_r11(const mg_pdesc*, uint32_t, const mg_run&, uint32_t, uint32_t, uint32_t*,
                             hipStream_t);
const char* mg_asm_digest_r16(void);
const char* mg_asm_digest_r11(void);
static_assert(MG_NREG == 16 && MG_NREG_W4 == 11, "one interpreter per layout: _r16, _r11");

static mg_launch_fn layout_launch(uint32_t nreg) {
    return nreg == MG_NREG_W4 ? mg_launch_asm_r11 : mg_launch_asm_r16;
}

hipError_t mg_launch_keccak(const uint8_t* d_data, const uint64_t* d_off, const uint32_t* d_len,
                            uint32_t n, uint8_t* d_out, hipStream_t stream);


struct mg_ctx {
    int device = 0;
    // register layout of this context's interpreter (mg_init_layout): its
    // slot count, kernel and LDS spill regions per lane (the layout's default
    // — 6 fill the CU at three 256-lane blocks, 13 halves; 5 at four blocks —
    // unless MYTHGPU_LDS_SLOTS sets it)
    uint32_t nreg = MG_NREG;
    mg_launch_fn launch_asm = mg_launch_asm_r16;
    hipStream_t stream = nullptr;
    std::string err;
    char name[256] = {0};
    int cus = 0;
    // assembly interpreter: handler byte offsets (query launch at init) and
    // LDS spill slots per 256-lane block
    uint32_t hoff[MGA_NUM_HANDLERS] = {0};
    uint32_t lds_slots = 6;
    // generator boundary-value table (device, 48 KiB; MG_BTAB_WORDS)
    uint32_t* d_btab = nullptr;
    // grow-only device workspace for synchronous calls
    void* ws = nullptr;
    size_t ws_size = 0;
    // device time of the last synchronous eval / search (HIP events around
    // its launches on the context stream; mg_last_kernel_ms)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float last_ms = 0.f;
    // device blocks of programs and batches (dev_alloc): power-of-two size
    // classes; classes below MG_SLAB_CLASS_MAX are carved from slabs, larger
    // ones are whole allocations; freed blocks wait on a per-class list, so
    // a get_model query's loads and frees make no hipMalloc / hipFree (each
    // costs tens of microseconds, and hipFree synchronises the device)
    std::map<size_t, std::vector<void*>> free_blocks;
    std::vector<void*> slabs, large;
    uint8_t* slab_cur = nullptr;
    size_t slab_left = 0;
    // the last launch on each caller stream (mg_batch_eval_gen), one event
    // per stream: a freed block is reused only after every launch that
    // might read it completed, on whichever streams they were queued
    struct ext_stream { hipStream_t stream; hipEvent_t ev; bool pending; };
    std::vector<ext_stream> ext;
    // pinned host staging for program uploads (grow-only): the blob is
    // assembled in place and copied at pinned-DMA rate; a leaf-pool-heavy
    // search program is ~1 MB (the pools' (v-1, v, v+1) triples)
    uint8_t* h_stage = nullptr;
    size_t h_stage_size = 0;
};

static void timing_begin(mg_ctx* ctx) {
    ctx->last_ms = 0.f;
    if (ctx->ev0) (void)hipEventRecord(ctx->ev0, ctx->stream);
}

static void timing_end(mg_ctx* ctx) {
    if (ctx->ev1) (void)hipEventRecord(ctx->ev1, ctx->stream);
}

// after the stream was synchronised
static void timing_read(mg_ctx* ctx) {
    float ms = 0.f;
    if (ctx->ev0 && ctx->ev1 && hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1) == hipSuccess)
        ctx->last_ms = ms;
}

struct mg_jit;

struct mg_prog {
    mg_ctx* ctx = nullptr;
    mg_jit* jit = nullptr;          // the compiled-program image it is attached to
    void* d_blob = nullptr;         // code | consts | gen | desc | xcode
    size_t blob_cls = 0;            // its dev_alloc size class
    mg_pdesc* d_desc = nullptr;
    mg_pdesc h_desc;                // host copy (batches copy it from here)
    uint32_t n_ins = 0, n_consts = 0, n_leaves = 0, n_lds = 0, n_probes = 0;
    uint64_t rec_fp = 0;            // records' fingerprint (rec_fingerprint)
};

// Fingerprint of a program's records with HANDLER IDS in word 0 (the
// translator run with the identity table, before word 0 becomes this
// library's handler offset): every word times successive powers of
// 0x100000001B3 mod 2^64, plus the record count (mythril_amd/jit.py
// records_fingerprint).  The handler id names the operation and its variant,
// so two programs whose records differ only in an opcode (ADD / SUB, ULT /
// SLT) differ here.  A compiled-program image carries it per entry, so
// mg_jit_attach refuses code built for other records.
static uint64_t rec_fingerprint(const std::vector<uint32_t>& rec) {
    uint64_t h = 0, p = 1;
    for (size_t r = 0; r + 8 <= rec.size(); r += 8)
        for (int k = 0; k < 8; ++k) {
            p *= 0x100000001B3ull;
            h += (uint64_t)rec[r + k] * p;
        }
    return h + rec.size() / 8;
}

// The identity handler table: the translator then writes handler ids into
// word 0 (fingerprinted, then mapped through the context's offsets).
// Built once by a function-local static (thread-safe initialisation: two
// contexts may load programs from two host threads at once).
static const uint32_t* identity_handlers() {
    struct table {
        uint32_t t[MGA_NUM_HANDLERS];
        table() {
            for (uint32_t h = 0; h < MGA_NUM_HANDLERS; ++h) t[h] = h;
        }
    };
    static const table tab;
    return tab.t;
}

static uint32_t kernel_lds_slots(const mg_ctx* ctx, uint32_t n_lds) {
    return n_lds < ctx->lds_slots ? n_lds : ctx->lds_slots;
}

static hipError_t launch(const mg_ctx* ctx, int gen, const mg_pdesc* d_descs, uint32_t n_progs,
                         const mg_run& run, uint32_t n_lds, hipStream_t stream) {
    return ctx->launch_asm(d_descs, n_progs, run, gen ? 1u : 0u, kernel_lds_slots(ctx, n_lds),
                           nullptr, stream);
}

// A loaded compiled-program code object (mythril_amd/jit.py) and the
// programs whose descriptors point into it.
struct mg_jit {
    mg_ctx* ctx = nullptr;
    hipModule_t module = nullptr;
    std::vector<mg_prog*> progs;
};

struct mg_batch {
    mg_ctx* ctx = nullptr;
    mg_pdesc* d_descs = nullptr;
    size_t descs_cls = 0;
    uint32_t n = 0;
    uint32_t max_lds = 0;
    uint32_t max_leaves = 0;
    uint32_t max_probes = 0;
};

static int fail(mg_ctx* ctx, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    return code;
}

#define HIPCHECK(ctx, expr)                                                              \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return fail(ctx, MG_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),  \
                        __FILE__, __LINE__);                                            \
    } while (0)

#define MG_SLAB_BYTES ((size_t)4 << 20)
#define MG_SLAB_CLASS_MAX ((size_t)256 << 10)
#define MG_BLOCK_MIN ((size_t)4 << 10)

static size_t block_class(size_t bytes) {
    size_t c = MG_BLOCK_MIN;
    while (c < bytes) c <<= 1;
    return c;
}

// A device block of at least `bytes` (256-byte aligned); *cls receives its
// size class for dev_release.
static hipError_t dev_alloc(mg_ctx* ctx, size_t bytes, void** out, size_t* cls) {
    const size_t c = block_class(bytes);
    *cls = c;
    auto it = ctx->free_blocks.find(c);
    if (it != ctx->free_blocks.end() && !it->second.empty()) {
        *out = it->second.back();
        it->second.pop_back();
        return hipSuccess;
    }
    if (c > MG_SLAB_CLASS_MAX) {
        hipError_t e = hipMalloc(out, c);
        if (e == hipSuccess) ctx->large.push_back(*out);
        return e;
    }
    if (ctx->slab_left < c) {
        void* slab = nullptr;
        hipError_t e = hipMalloc(&slab, MG_SLAB_BYTES);
        if (e != hipSuccess) return e;
        ctx->slabs.push_back(slab);
        ctx->slab_cur = (uint8_t*)slab;
        ctx->slab_left = MG_SLAB_BYTES;
    }
    *out = ctx->slab_cur;                   // classes are powers of two <= the slab
    ctx->slab_cur += c;
    ctx->slab_left -= c;
    return hipSuccess;
}

// Back to its class list once no queued launch can still read it: the
// context stream and the last launch on every caller stream are waited for
// (what the hipFree this replaces did by synchronising the device).
static void dev_release(mg_ctx* ctx, void* p, size_t cls) {
    if (!p) return;
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& x : ctx->ext)
        if (x.pending) {
            (void)hipEventSynchronize(x.ev);
            x.pending = false;
        }
    ctx->free_blocks[cls].push_back(p);
}

// Note a launch on a caller stream (its event is recorded after it).
static hipError_t ext_launched(mg_ctx* ctx, hipStream_t s) {
    for (auto& x : ctx->ext)
        if (x.stream == s) {
            x.pending = true;
            return hipEventRecord(x.ev, s);
        }
    hipEvent_t ev = nullptr;
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess)                   // no event: wait now; nothing stays pending
        return hipStreamSynchronize(s);
    ctx->ext.push_back({s, ev, true});
    return hipEventRecord(ev, s);
}

static int workspace(mg_ctx* ctx, size_t bytes, void** out) {
    if (bytes > ctx->ws_size) {
        if (ctx->ws) (void)hipFree(ctx->ws);
        ctx->ws = nullptr;
        ctx->ws_size = 0;
        size_t sz = bytes < (1u << 20) ? (1u << 20) : bytes;
        HIPCHECK(ctx, hipMalloc(&ctx->ws, sz));
        ctx->ws_size = sz;
    }
    *out = ctx->ws;
    return MG_OK;
}


// One launch in query mode: the assembly interpreter writes the byte offset
// of every handler (relative to its dispatch base) into a table.
static int query_handlers(mg_ctx* ctx) {
    void* d = nullptr;
    const size_t tab_b = sizeof(uint32_t) * MGA_NUM_HANDLERS;
    HIPCHECK(ctx, hipMalloc(&d, tab_b + 256));
    mg_pdesc* d_desc = (mg_pdesc*)((uint8_t*)d + tab_b);
    mg_pdesc zero;
    memset(&zero, 0, sizeof zero);
    zero.consts = (const uint32_t*)d;
    zero.xcode = (const uint32_t*)d;
    hipError_t e = hipMemcpy(d_desc, &zero, sizeof zero, hipMemcpyHostToDevice);
    mg_run run;
    memset(&run, 0, sizeof run);
    run.n_assign = 1;
    run.stride = 1;
    if (e == hipSuccess) e = ctx->launch_asm(d_desc, 1, run, 2u, 0, (uint32_t*)d, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(ctx->hoff, d, tab_b, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(ctx, MG_E_HIP, "handler query: %s", hipGetErrorString(e));
    for (int h = 0; h < MGA_NUM_HANDLERS; ++h)
        if (ctx->hoff[h] == 0 || ctx->hoff[h] > (1u << 24))
            return fail(ctx, MG_E_HIP, "handler query: bad offset %u for %d", ctx->hoff[h], h);
    return MG_OK;
}

extern "C" {


// Boundary values of the candidate generator as a table the LEAF handler
// indexes by kind * 256 + p (oracle/gen_ref.py gen_leaf, boundary class):
// kind 0: 0, 1: 1, 2: 1 << p (p = width - 1), 3: 2^256 - 1, 4: (1 << p) + 1,
// 5: (1 << p) - 1 (p = k); the handler masks to the width afterwards.
#define MG_BTAB_WORDS (6 * 256 * 8)
static void mg_boundary_table(uint32_t* t) {
    memset(t, 0, MG_BTAB_WORDS * 4);
    for (uint32_t p = 0; p < 256; ++p) {
        uint32_t* e1 = t + (1 * 256 + p) * 8;
        uint32_t* e2 = t + (2 * 256 + p) * 8;
        uint32_t* e3 = t + (3 * 256 + p) * 8;
        uint32_t* e4 = t + (4 * 256 + p) * 8;
        uint32_t* e5 = t + (5 * 256 + p) * 8;
        e1[0] = 1;
        e2[p >> 5] = 1u << (p & 31);
        for (int j = 0; j < 8; ++j) e3[j] = ~0u;
        e4[p >> 5] = 1u << (p & 31);
        e4[0] += 1;                              // p = 0: 1 + 1 = 2
        for (uint32_t j = 0; j < (p >> 5); ++j) e5[j] = ~0u;
        e5[p >> 5] = (1u << (p & 31)) - 1;
    }
}

int mg_init(int device, mg_ctx** out) { return mg_init_layout(device, MG_NREG, out); }

const char* mg_asm_digest(void) { return mg_asm_digest_r16(); }

const char* mg_asm_digest_layout(uint32_t nreg) {
    if (nreg == MG_NREG) return mg_asm_digest_r16();
    if (nreg == MG_NREG_W4) return mg_asm_digest_r11();
    return nullptr;
}

int mg_init_layout(int device, uint32_t nreg, mg_ctx** out) {
    if (!out) return MG_E_ARG;
    *out = nullptr;
    const mg_layout_info* lay = mg_find_layout(nreg);
    if (!lay) return MG_E_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return MG_E_NODEV;
    if (device < 0 || device >= n) return MG_E_NODEV;
    mg_ctx* ctx = new mg_ctx();
    ctx->device = device;
    ctx->nreg = nreg;
    ctx->launch_asm = layout_launch(nreg);
    ctx->lds_slots = lay->lds_slots;
    if (hipSetDevice(device) != hipSuccess) {
        delete ctx;
        return MG_E_NODEV;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
        snprintf(ctx->name, sizeof ctx->name, "%s (%s)", prop.name, prop.gcnArchName);
        ctx->cus = prop.multiProcessorCount;
    }
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return MG_E_HIP;
    }
    if (hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) {
        mg_free(ctx);
        return MG_E_HIP;
    }
    if (const char* l = getenv("MYTHGPU_LDS_SLOTS")) {
        // a region count whose halves a DS offset cannot reach is refused
        // here, not found later by the assembler
        char* end = nullptr;
        const long v = strtol(l, &end, 10);
        if (end == l || *end || v < 0 || v > MG_MAX_LDS_DS) {
            mg_free(ctx);
            return MG_E_ARG;
        }
        ctx->lds_slots = (uint32_t)v;
    }
    if (query_handlers(ctx) != MG_OK) {
        mg_free(ctx);
        return MG_E_HIP;
    }
    {
        std::vector<uint32_t> bt(MG_BTAB_WORDS);
        mg_boundary_table(bt.data());
        if (hipMalloc(&ctx->d_btab, MG_BTAB_WORDS * 4) != hipSuccess ||
            hipMemcpy(ctx->d_btab, bt.data(), MG_BTAB_WORDS * 4, hipMemcpyHostToDevice) !=
                hipSuccess) {
            mg_free(ctx);
            return MG_E_HIP;
        }
    }
    *out = ctx;
    return MG_OK;
}

void mg_free(mg_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->ws) (void)hipFree(ctx->ws);
    if (ctx->d_btab) (void)hipFree(ctx->d_btab);
    for (void* q : ctx->slabs) (void)hipFree(q);
    for (void* q : ctx->large) (void)hipFree(q);
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    for (auto& x : ctx->ext) {
        (void)hipEventSynchronize(x.ev);
        (void)hipEventDestroy(x.ev);
    }
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int mg_runtime_info(int* hip_version, char* path, size_t path_len) {
    if (hip_version) {
        *hip_version = 0;
        if (hipRuntimeGetVersion(hip_version) != hipSuccess) *hip_version = 0;
    }
    if (path && path_len) {
        path[0] = 0;
        Dl_info info;
        if (dladdr((void*)&hipRuntimeGetVersion, &info) && info.dli_fname)
            snprintf(path, path_len, "%s", info.dli_fname);
    }
    return MG_OK;
}

const char* mg_last_error(const mg_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }

float mg_last_kernel_ms(const mg_ctx* ctx) { return ctx ? ctx->last_ms : 0.f; }

int mg_device_info(mg_ctx* ctx, char* name, size_t name_len, int* n_cus) {
    if (!ctx) return MG_E_ARG;
    if (name && name_len) snprintf(name, name_len, "%s", ctx->name);
    if (n_cus) *n_cus = ctx->cus;
    return MG_OK;
}

int mg_load_program(mg_ctx* ctx, const uint32_t* code, uint32_t n_ins, const uint32_t* consts,
                    uint32_t n_consts, const mg_leafgen* leaves, uint32_t n_leaves,
                    uint32_t n_spill_slots, uint32_t n_probes, uint64_t prog_seed,
                    mg_prog** out) {
    if (!ctx || !out || (n_ins && !code) || (n_consts && !consts) || (n_leaves && !leaves))
        return fail(ctx, MG_E_ARG, "null argument");
    *out = nullptr;
    const uint32_t n_lds_slots = n_spill_slots < MG_MAX_LDS ? n_spill_slots : MG_MAX_LDS;
    int rc = mg_validate(ctx ? &ctx->err : nullptr, code, n_ins, n_consts, leaves, n_leaves, n_lds_slots, n_spill_slots,
                         n_probes, ctx->nreg);
    if (rc) return rc;
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    // assembly records + translator masks (appended to the constant table);
    // word 0 holds handler ids until the fingerprint is taken
    std::vector<uint32_t> rec;
    MaskPool pool;
    mg_translate_records(identity_handlers(), code, n_ins, n_consts,
                         kernel_lds_slots(ctx, n_spill_slots), ctx->nreg, rec, pool);
    const uint32_t n_masks = (uint32_t)(pool.words.size() / 8);
    const uint32_t n_const_all = n_consts + n_masks + n_consts * 3;
    // device leaf descriptors: byte pool offsets and the per-leaf stream salt
    std::vector<mg_leafgen_dev> gdev(n_leaves);
    for (uint32_t i = 0; i < n_leaves; ++i) {
        const uint64_t salt = (prog_seed * 0xD1B54A32D192ED03ull) ^
                              ((uint64_t)(i + 1) * 0x8CB92BA72F3D8DD7ull);
        gdev[i] = {leaves[i].width, (n_consts + n_masks + 3 * leaves[i].pool_off) * 32u,
                   leaves[i].pool_n,
                   leaves[i].pct_uniform, leaves[i].pct_small, leaves[i].pct_boundary,
                   (uint32_t)salt, (uint32_t)(salt >> 32)};
    }
    // LEAFD records carry their leaf's generator parameters (asmgen.py
    // LEAFD_*: no descriptor load in the handler): pool offset, salt, pool
    // size and the class thresholds packed one per byte
    for (size_t r = 0; r + 8 <= rec.size(); r += 8) {
        if (rec[r] >= MGA_NUM_HANDLERS || rec[r] / (2 * MGA_NVAR) != MGA_LEAFD) continue;
        const uint32_t li = rec[r + 4];
        if (li >= n_leaves) continue;            // eval mode only (no generator)
        const mg_leafgen_dev& g = gdev[li];
        rec[r + 1] = g.pool_off_b;
        rec[r + 2] = g.salt_lo;
        rec[r + 3] = g.salt_hi;
        rec[r + 5] = g.pool_n;
        rec[r + 7] = g.pct_uniform | g.pct_small << 8 | g.pct_boundary << 16;
    }
    const uint64_t rec_fp = rec_fingerprint(rec);
    // handler ids -> this library's handler offsets (the zeroed pad record
    // stays zero)
    for (size_t r = 0; r + 8 <= rec.size(); r += 8)
        if (r + 8 < rec.size() || rec[r] != 0) rec[r] = ctx->hoff[rec[r] % MGA_NUM_HANDLERS];
    // 8 zeroed NOPs after the IR code: the C++ interpreter prefetches ahead
    const size_t code_b = (size_t)(n_ins + 8) * 16, const_b = (size_t)n_const_all * 32,
                 gen_b = gdev.size() * sizeof(mg_leafgen_dev), rec_b = rec.size() * 4;
    auto align = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t off_const = align(code_b), off_gen = off_const + align(const_b),
                 off_desc = off_gen + align(gen_b), off_rec = off_desc + align(sizeof(mg_pdesc)),
                 total = off_rec + align(rec_b);
    if (total > ctx->h_stage_size) {
        if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
        ctx->h_stage = nullptr;
        ctx->h_stage_size = 0;
        size_t sz = (size_t)4 << 20;
        while (sz < total) sz <<= 1;
        HIPCHECK(ctx, hipHostMalloc((void**)&ctx->h_stage, sz, hipHostMallocDefault));
        ctx->h_stage_size = sz;
    }
    uint8_t* blob = ctx->h_stage;   // free: every upload below is synchronous
    memset(blob, 0, total);
    if (n_ins) memcpy(blob, code, (size_t)n_ins * 16);   // + zeroed NOP padding
    if (n_consts) memcpy(blob + off_const, consts, (size_t)n_consts * 32);
    if (!pool.words.empty())
        memcpy(blob + off_const + (size_t)n_consts * 32, pool.words.data(), pool.words.size() * 4);
    // generator pools expanded to (v - 1, v, v + 1) triples (mod 2^256), so
    // the pool class is one indexed load (pool[e] + delta - 1, gen_ref.py)
    {
        uint32_t* pm = (uint32_t*)(blob + off_const + (size_t)(n_consts + n_masks) * 32);
        for (uint32_t c = 0; c < n_consts; ++c) {
            const uint32_t* v = consts + (size_t)c * 8;
            uint32_t* o = pm + (size_t)c * 24;
            uint64_t bm = 1, bp = 1;             // borrow of v - 1, carry of v + 1
            for (int j = 0; j < 8; ++j) {
                o[j] = v[j] - (uint32_t)bm;
                bm = bm && v[j] == 0;
                o[8 + j] = v[j];
                o[16 + j] = v[j] + (uint32_t)bp;
                bp = bp && v[j] == 0xFFFFFFFFu;
            }
        }
    }
    if (gen_b) memcpy(blob + off_gen, gdev.data(), gen_b);
    memcpy(blob + off_rec, rec.data(), rec_b);
    void* d = nullptr;
    size_t cls = 0;
    HIPCHECK(ctx, dev_alloc(ctx, total, &d, &cls));
    uint8_t* db = (uint8_t*)d;
    mg_pdesc desc;
    memset(&desc, 0, sizeof desc);
    desc.code = (const uint32_t*)db;
    desc.consts = (const uint32_t*)(db + off_const);
    desc.gen = (const mg_leafgen_dev*)(db + off_gen);
    desc.n_ins = n_ins;
    desc.n_leaves = n_leaves;
    desc.n_lds = n_lds_slots;
    desc.n_probes = n_probes;
    desc.prog_seed = prog_seed;
    desc.xcode = (const uint32_t*)(db + off_rec);
    desc.btab = ctx->d_btab;
    memcpy(blob + off_desc, &desc, sizeof desc);
    hipError_t e = hipMemcpyAsync(d, blob, total, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
        dev_release(ctx, d, cls);
        return fail(ctx, MG_E_HIP, "upload: %s", hipGetErrorString(e));
    }
    mg_prog* p = new mg_prog();
    p->ctx = ctx;
    p->rec_fp = rec_fp;
    p->d_blob = d;
    p->blob_cls = cls;
    p->d_desc = (mg_pdesc*)(db + off_desc);
    p->h_desc = desc;
    p->n_ins = n_ins;
    p->n_consts = n_consts;
    p->n_leaves = n_leaves;
    p->n_lds = n_lds_slots;
    p->n_probes = n_probes;
    *out = p;
    return MG_OK;
}

void mg_free_program(mg_prog* p) {
    if (!p) return;
    (void)hipSetDevice(p->ctx->device);
    if (p->jit) {                   // a later detach must not write into a reused block
        auto& v = p->jit->progs;
        v.erase(std::remove(v.begin(), v.end(), p), v.end());
    }
    dev_release(p->ctx, p->d_blob, p->blob_cls);
    delete p;
}

static mg_run empty_run() {
    mg_run r;
    memset(&r, 0, sizeof r);
    return r;
}

int mg_eval(mg_ctx* ctx, const mg_prog* prog, const uint32_t* leaves_soa, uint64_t n_assign,
            uint64_t* root_bits, uint32_t* probes) {
    if (!ctx || !prog || !root_bits || (prog->n_leaves && !leaves_soa))
        return fail(ctx, MG_E_ARG, "null argument");
    if (n_assign == 0) return MG_OK;
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    const uint64_t words = (n_assign + 63) / 64;
    const size_t leaf_b = (size_t)prog->n_leaves * 8 * n_assign * 4;
    const size_t probe_b = probes ? (size_t)prog->n_probes * 8 * n_assign * 4 : 0;
    const size_t root_b = words * 8;
    void* ws;
    int rc = workspace(ctx, leaf_b + probe_b + root_b + 256, &ws);
    if (rc) return rc;
    uint8_t* base = (uint8_t*)ws;
    mg_run run = empty_run();
    run.leaves = (const uint32_t*)base;
    run.root_bits = (uint64_t*)(base + leaf_b);
    run.probes = probes ? (uint32_t*)(base + leaf_b + root_b) : nullptr;
    run.stride = n_assign;
    run.n_assign = n_assign;
    run.words_per_prog = words;
    if (leaf_b)
        HIPCHECK(ctx, hipMemcpyAsync(base, leaves_soa, leaf_b, hipMemcpyHostToDevice, ctx->stream));
    timing_begin(ctx);
    HIPCHECK(ctx, launch(ctx, 0, prog->d_desc, 1, run, prog->n_lds, ctx->stream));
    timing_end(ctx);
    HIPCHECK(ctx, hipMemcpyAsync(root_bits, run.root_bits, root_b, hipMemcpyDeviceToHost,
                                 ctx->stream));
    if (probes && probe_b)
        HIPCHECK(ctx, hipMemcpyAsync(probes, run.probes, probe_b, hipMemcpyDeviceToHost,
                                     ctx->stream));
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    timing_read(ctx);
    return MG_OK;
}

int mg_eval_gen(mg_ctx* ctx, const mg_prog* prog, const mg_gen* gen, uint64_t n_assign,
                uint64_t* root_bits, uint32_t* probes, uint32_t* leaves_out) {
    if (!ctx || !prog || !gen || !root_bits) return fail(ctx, MG_E_ARG, "null argument");
    if (n_assign == 0) return MG_OK;
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    const uint64_t words = (n_assign + 63) / 64;
    const size_t leaf_b = leaves_out ? (size_t)prog->n_leaves * 8 * n_assign * 4 : 0;
    const size_t probe_b = probes ? (size_t)prog->n_probes * 8 * n_assign * 4 : 0;
    const size_t root_b = words * 8;
    void* ws;
    int rc = workspace(ctx, leaf_b + probe_b + root_b + 256, &ws);
    if (rc) return rc;
    uint8_t* base = (uint8_t*)ws;
    mg_run run = empty_run();
    run.root_bits = (uint64_t*)base;
    run.probes = probes ? (uint32_t*)(base + root_b) : nullptr;
    run.leaves_out = leaves_out ? (uint32_t*)(base + root_b + probe_b) : nullptr;
    run.stride = n_assign;
    run.n_assign = n_assign;
    run.words_per_prog = words;
    run.seed = gen->seed;
    run.first_index = gen->first_index;
    if (leaf_b) HIPCHECK(ctx, hipMemsetAsync(run.leaves_out, 0, leaf_b, ctx->stream));
    timing_begin(ctx);
    HIPCHECK(ctx, launch(ctx, 1, prog->d_desc, 1, run, prog->n_lds, ctx->stream));
    timing_end(ctx);
    HIPCHECK(ctx, hipMemcpyAsync(root_bits, run.root_bits, root_b, hipMemcpyDeviceToHost,
                                 ctx->stream));
    if (probe_b)
        HIPCHECK(ctx, hipMemcpyAsync(probes, run.probes, probe_b, hipMemcpyDeviceToHost,
                                     ctx->stream));
    if (leaf_b)
        HIPCHECK(ctx, hipMemcpyAsync(leaves_out, run.leaves_out, leaf_b, hipMemcpyDeviceToHost,
                                     ctx->stream));
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    timing_read(ctx);
    return MG_OK;
}

// Candidates per launch of a search: launches are queued back to back with
// no host round trip; a wave whose candidates all lie beyond the program's
// current first witness exits at once (mg_run.skip_solved), so the search
// stops consuming lanes as soon as a witness is known.
#define MG_SEARCH_LAUNCH (1ull << 26)

int mg_search(mg_ctx* ctx, const mg_prog* prog, const mg_gen* gen, uint64_t n_cand,
              int64_t* first_sat, uint32_t* witness_leaves) {
    if (!ctx || !prog || !gen || !first_sat) return fail(ctx, MG_E_ARG, "null argument");
    *first_sat = -1;
    if (n_cand == 0) return MG_OK;
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    const size_t leaf_b = (size_t)prog->n_leaves * 8 * 4;
    void* ws;
    int rc = workspace(ctx, 256 + leaf_b, &ws);
    if (rc) return rc;
    unsigned long long* d_first = (unsigned long long*)ws;
    HIPCHECK(ctx, hipMemsetAsync(d_first, 0xFF, 8, ctx->stream));
    timing_begin(ctx);
    for (uint64_t done = 0; done < n_cand; done += MG_SEARCH_LAUNCH) {
        mg_run run = empty_run();
        run.n_assign = n_cand - done < MG_SEARCH_LAUNCH ? n_cand - done : MG_SEARCH_LAUNCH;
        run.stride = run.n_assign;
        run.first_sat = d_first;
        run.seed = gen->seed;
        run.first_index = gen->first_index + done;
        run.skip_solved = 1;
        HIPCHECK(ctx, launch(ctx, 1, prog->d_desc, 1, run, prog->n_lds, ctx->stream));
    }
    timing_end(ctx);
    unsigned long long h = ~0ull;
    HIPCHECK(ctx, hipMemcpyAsync(&h, d_first, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    timing_read(ctx);
    if (h != ~0ull) *first_sat = (int64_t)h;
    if (*first_sat >= 0 && witness_leaves && prog->n_leaves) {
        // regenerate the winning candidate (counter-based streams: no gather)
        mg_run run = empty_run();
        run.n_assign = 1;
        run.stride = 1;
        run.seed = gen->seed;
        run.first_index = (uint64_t)*first_sat;
        run.leaves_out = (uint32_t*)((uint8_t*)ws + 256);
        HIPCHECK(ctx, hipMemsetAsync(run.leaves_out, 0, leaf_b, ctx->stream));
        HIPCHECK(ctx, launch(ctx, 1, prog->d_desc, 1, run, prog->n_lds, ctx->stream));
        HIPCHECK(ctx, hipMemcpyAsync(witness_leaves, run.leaves_out, leaf_b,
                                     hipMemcpyDeviceToHost, ctx->stream));
        HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    }
    return MG_OK;
}

int mg_batch_create(mg_ctx* ctx, const mg_prog* const* progs, uint32_t n_progs, mg_batch** out) {
    if (!ctx || !out || (n_progs && !progs)) return fail(ctx, MG_E_ARG, "null argument");
    *out = nullptr;
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    std::vector<mg_pdesc> descs(n_progs);
    uint32_t max_lds = 0, max_leaves = 0, max_probes = 0;
    for (uint32_t i = 0; i < n_progs; ++i) {
        if (!progs[i] || progs[i]->ctx != ctx) return fail(ctx, MG_E_ARG, "program %u", i);
        descs[i] = progs[i]->h_desc;
        if (progs[i]->n_lds > max_lds) max_lds = progs[i]->n_lds;
        if (progs[i]->n_leaves > max_leaves) max_leaves = progs[i]->n_leaves;
        if (progs[i]->n_probes > max_probes) max_probes = progs[i]->n_probes;
    }
    mg_batch* b = new mg_batch();
    b->ctx = ctx;
    b->n = n_progs;
    b->max_lds = max_lds;
    b->max_leaves = max_leaves;
    b->max_probes = max_probes;
    if (n_progs) {
        void* d = nullptr;
        hipError_t e = dev_alloc(ctx, sizeof(mg_pdesc) * n_progs, &d, &b->descs_cls);
        b->d_descs = (mg_pdesc*)d;
        if (e == hipSuccess)
            e = hipMemcpy(b->d_descs, descs.data(), sizeof(mg_pdesc) * n_progs,
                          hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            if (b->d_descs) dev_release(ctx, b->d_descs, b->descs_cls);
            delete b;
            return fail(ctx, MG_E_HIP, "batch upload: %s", hipGetErrorString(e));
        }
    }
    *out = b;
    return MG_OK;
}

void mg_batch_free(mg_batch* b) {
    if (!b) return;
    (void)hipSetDevice(b->ctx->device);
    if (b->d_descs) dev_release(b->ctx, b->d_descs, b->descs_cls);
    delete b;
}

int mg_batch_eval_gen(mg_ctx* ctx, mg_batch* b, uint64_t seed, uint64_t first_index,
                      uint64_t n_assign, uint64_t* d_root_bits, uint64_t* d_first_sat,
                      void* stream) {
    if (!ctx || !b) return fail(ctx, MG_E_ARG, "null argument");
    if (b->ctx != ctx) return fail(ctx, MG_E_ARG, "batch belongs to another context");
    // like every other entry point: the caller's thread may have another
    // device current (two contexts on two devices driven from one thread)
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    const uint64_t words = (n_assign + 63) / 64;
    for (uint32_t p0 = 0; p0 < b->n; p0 += 65535) {
        const uint32_t np = b->n - p0 < 65535 ? b->n - p0 : 65535;
        mg_run run = empty_run();
        run.n_assign = n_assign;
        run.stride = n_assign;
        run.words_per_prog = words;
        run.root_bits = d_root_bits ? d_root_bits + (size_t)p0 * words : nullptr;
        run.first_sat = d_first_sat ? (unsigned long long*)d_first_sat + p0 : nullptr;
        run.seed = seed;
        run.first_index = first_index;
        HIPCHECK(ctx, launch(ctx, 1, b->d_descs + p0, np, run, b->max_lds, s));
    }
    if (s != ctx->stream) HIPCHECK(ctx, ext_launched(ctx, s));
    return MG_OK;
}

int mg_batch_search(mg_ctx* ctx, mg_batch* b, const mg_gen* gen, uint64_t n_cand,
                    int64_t* first_sat, uint32_t* witness_leaves, uint32_t max_leaves) {
    return mg_batch_search_probes(ctx, b, gen, n_cand, first_sat, witness_leaves, max_leaves,
                                  nullptr, 0);
}

int mg_batch_search_probes(mg_ctx* ctx, mg_batch* b, const mg_gen* gen, uint64_t n_cand,
                           int64_t* first_sat, uint32_t* witness_leaves, uint32_t max_leaves,
                           uint32_t* witness_probes, uint32_t max_probes) {
    if (!ctx || !b || !gen || (b->n && !first_sat)) return fail(ctx, MG_E_ARG, "null argument");
    if (b->ctx != ctx) return fail(ctx, MG_E_ARG, "batch belongs to another context");
    if (witness_leaves && max_leaves < b->max_leaves)
        return fail(ctx, MG_E_ARG, "witness rows hold %u leaves, a program has %u", max_leaves,
                    b->max_leaves);
    if (witness_probes && (!witness_leaves || max_probes < b->max_probes))
        return fail(ctx, MG_E_ARG, "probe rows hold %u probes, a program has %u", max_probes,
                    b->max_probes);
    for (uint32_t i = 0; i < b->n; ++i) first_sat[i] = -1;
    if (n_cand == 0 || b->n == 0) return MG_OK;
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    const size_t first_b = ((size_t)b->n * 8 + 255) & ~(size_t)255;
    const size_t wit_b = witness_leaves ? (size_t)b->n * max_leaves * 8 * 4 : 0;
    const size_t wit_b_al = (wit_b + 255) & ~(size_t)255;
    const size_t prb_b = witness_probes ? (size_t)b->n * max_probes * 8 * 4 : 0;
    void* ws;
    int rc = workspace(ctx, first_b + wit_b_al + prb_b, &ws);
    if (rc) return rc;
    unsigned long long* d_first = (unsigned long long*)ws;
    HIPCHECK(ctx, hipMemsetAsync(d_first, 0xFF, (size_t)b->n * 8, ctx->stream));
    timing_begin(ctx);
    // every program's whole candidate range, queued with no host round trip;
    // waves of solved programs exit at once (skip_solved)
    for (uint64_t done = 0; done < n_cand; done += MG_SEARCH_LAUNCH) {
        for (uint32_t p0 = 0; p0 < b->n; p0 += 65535) {
            const uint32_t np = b->n - p0 < 65535 ? b->n - p0 : 65535;
            mg_run run = empty_run();
            run.n_assign = n_cand - done < MG_SEARCH_LAUNCH ? n_cand - done : MG_SEARCH_LAUNCH;
            run.stride = run.n_assign;
            run.first_sat = d_first + p0;
            run.seed = gen->seed;
            run.first_index = gen->first_index + done;
            run.skip_solved = 1;
            HIPCHECK(ctx, launch(ctx, 1, b->d_descs + p0, np, run, b->max_lds, ctx->stream));
        }
    }
    timing_end(ctx);
    if (witness_leaves) {
        // one launch regenerates every program's winning candidate: lane 0
        // of program p evaluates candidate first_sat[p] (solved programs only)
        // (and, when asked, its probe values: what a solve-mode witness
        // computes besides the generated leaves)
        uint32_t* d_wit = (uint32_t*)((uint8_t*)ws + first_b);
        uint32_t* d_prb = prb_b ? (uint32_t*)((uint8_t*)ws + first_b + wit_b_al) : nullptr;
        HIPCHECK(ctx, hipMemsetAsync(d_wit, 0, wit_b, ctx->stream));
        if (prb_b) HIPCHECK(ctx, hipMemsetAsync(d_prb, 0, prb_b, ctx->stream));
        for (uint32_t p0 = 0; p0 < b->n; p0 += 65535) {
            const uint32_t np = b->n - p0 < 65535 ? b->n - p0 : 65535;
            mg_run run = empty_run();
            run.n_assign = 1;
            run.stride = 1;
            run.seed = gen->seed;
            run.first_per_prog = (const uint64_t*)(d_first + p0);
            run.leaves_out = d_wit + (size_t)p0 * max_leaves * 8;
            run.lout_prog_words = (uint64_t)max_leaves * 8;
            if (d_prb) {
                run.probes = d_prb + (size_t)p0 * max_probes * 8;
                run.probe_prog_words = (uint64_t)max_probes * 8;
            }
            HIPCHECK(ctx, launch(ctx, 1, b->d_descs + p0, np, run, b->max_lds, ctx->stream));
        }
        HIPCHECK(ctx, hipMemcpyAsync(witness_leaves, d_wit, wit_b, hipMemcpyDeviceToHost,
                                     ctx->stream));
        if (prb_b)
            HIPCHECK(ctx, hipMemcpyAsync(witness_probes, d_prb, prb_b, hipMemcpyDeviceToHost,
                                         ctx->stream));
    }
    std::vector<unsigned long long> h(b->n, ~0ull);
    HIPCHECK(ctx, hipMemcpyAsync(h.data(), d_first, (size_t)b->n * 8, hipMemcpyDeviceToHost,
                                 ctx->stream));
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    timing_read(ctx);
    for (uint32_t i = 0; i < b->n; ++i) first_sat[i] = h[i] == ~0ull ? -1 : (int64_t)h[i];
    return MG_OK;
}

// The byte range of the executable sections of a code object and the
// address of its mg_jit_table symbol (both as link-time virtual addresses),
// read from the ELF itself with every offset bounds-checked: the entries an
// image names must lie in its code.
struct jit_layout {
    std::vector<std::pair<uint64_t, uint64_t>> text;   // [begin, end) of SHF_EXECINSTR sections
    uint64_t table = 0;
    bool found = false;
};

static bool elf_layout(const uint8_t* img, size_t n, jit_layout* out) {
    if (n < sizeof(Elf64_Ehdr) || memcmp(img, ELFMAG, SELFMAG) != 0 || img[EI_CLASS] != ELFCLASS64)
        return false;
    Elf64_Ehdr eh;
    memcpy(&eh, img, sizeof eh);
    if (eh.e_shentsize != sizeof(Elf64_Shdr) || eh.e_shoff > n ||
        (uint64_t)eh.e_shnum * sizeof(Elf64_Shdr) > n - eh.e_shoff)
        return false;
    std::vector<Elf64_Shdr> sh(eh.e_shnum);
    if (eh.e_shnum) memcpy(sh.data(), img + eh.e_shoff, eh.e_shnum * sizeof(Elf64_Shdr));
    for (const Elf64_Shdr& s : sh)
        if ((s.sh_flags & SHF_EXECINSTR) && s.sh_size)
            out->text.push_back({s.sh_addr, s.sh_addr + s.sh_size});
    for (const Elf64_Shdr& s : sh) {
        if ((s.sh_type != SHT_SYMTAB && s.sh_type != SHT_DYNSYM) || s.sh_link >= sh.size() ||
            s.sh_entsize != sizeof(Elf64_Sym) || s.sh_offset > n || s.sh_size > n - s.sh_offset)
            continue;
        const Elf64_Shdr& st = sh[s.sh_link];
        if (st.sh_offset > n || st.sh_size > n - st.sh_offset) continue;
        const char* names = (const char*)img + st.sh_offset;
        for (uint64_t k = 0; k < s.sh_size / sizeof(Elf64_Sym); ++k) {
            Elf64_Sym sym;
            memcpy(&sym, img + s.sh_offset + k * sizeof(Elf64_Sym), sizeof sym);
            static const char want[] = "mg_jit_table";
            if (sym.st_name + sizeof want > st.sh_size) continue;
            if (memcmp(names + sym.st_name, want, sizeof want) == 0) {
                out->table = sym.st_value;
                out->found = true;
                return true;
            }
        }
    }
    return true;
}

// Compiled programs: load the code object, read its entry table
// (mg_jit_table: a header row (MG_JIT_MAGIC, the asm digest of the
// interpreter the code was generated with: pinned registers, descriptor
// layout), then per program its entry relative to the table and its records'
// fingerprint) and point the programs' descriptors at their code.  Batches
// created afterwards copy the entries; the interpreter kernel then calls the
// code instead of dispatching records.  Every entry must lie inside an
// executable section of the image (read from its ELF headers) so a malformed
// image cannot send the kernel to an arbitrary address.
int mg_jit_attach(mg_ctx* ctx, mg_prog* const* progs, uint32_t n_progs, const void* image,
                  size_t image_size, mg_jit** out) {
    if (!ctx || !out || !image || !image_size || (n_progs && !progs))
        return fail(ctx, MG_E_ARG, "null argument");
    *out = nullptr;
    for (uint32_t i = 0; i < n_progs; ++i)
        if (!progs[i] || progs[i]->ctx != ctx) return fail(ctx, MG_E_ARG, "program %u", i);
    jit_layout lay;
    if (!elf_layout((const uint8_t*)image, image_size, &lay) || !lay.found || lay.text.empty())
        return fail(ctx, MG_E_ARG, "JIT image: not a code object with mg_jit_table and code");
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    hipModule_t mod = nullptr;
    HIPCHECK(ctx, hipModuleLoadData(&mod, image));
    hipDeviceptr_t d_table = nullptr;
    size_t table_b = 0;
    hipError_t e = hipModuleGetGlobal(&d_table, &table_b, mod, "mg_jit_table");
    // row 0: header; rows 1..n: (entry - table, records' fingerprint)
    std::vector<int64_t> row(2 * ((size_t)n_progs + 1));
    if (e == hipSuccess && table_b != ((size_t)n_progs + 1) * 16) e = hipErrorInvalidValue;
    if (e == hipSuccess) e = hipMemcpy(row.data(), d_table, table_b, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        (void)hipModuleUnload(mod);
        return fail(ctx, MG_E_HIP, "JIT image: %s (table %zu bytes for %u programs)",
                    hipGetErrorString(e), table_b, n_progs);
    }
    const uint64_t want_digest = strtoull(mg_asm_digest_layout(ctx->nreg), nullptr, 16);
    if ((uint64_t)row[0] != MG_JIT_MAGIC || (uint64_t)row[1] != want_digest) {
        (void)hipModuleUnload(mod);
        return fail(ctx, MG_E_ARG, "JIT image: built for another interpreter (header %016llx, "
                    "asm digest %016llx; this library %016llx)", (unsigned long long)row[0],
                    (unsigned long long)row[1], (unsigned long long)want_digest);
    }
    for (uint32_t i = 0; i < n_progs; ++i) {
        const int64_t rel = row[2 * (i + 1)];
        const uint64_t fp = (uint64_t)row[2 * (i + 1) + 1];
        if (rel == 0 && fp == 0) continue;                  // not compiled: interpreter
        const uint64_t at = lay.table + (uint64_t)rel;
        bool inside = false;
        for (const auto& t : lay.text) inside |= at >= t.first && at + 4 <= t.second;
        if (!inside || (rel & 3)) {
            (void)hipModuleUnload(mod);
            return fail(ctx, MG_E_ARG, "JIT image: entry %u at %lld outside the code", i,
                        (long long)rel);
        }
        if (fp != progs[i]->rec_fp) {
            (void)hipModuleUnload(mod);
            return fail(ctx, MG_E_ARG, "JIT image: entry %u was compiled for other records "
                        "(fingerprint %016llx, loaded program %016llx)", i,
                        (unsigned long long)fp, (unsigned long long)progs[i]->rec_fp);
        }
    }
    mg_jit* j = new mg_jit();
    j->ctx = ctx;
    j->module = mod;
    for (uint32_t i = 0; i < n_progs; ++i) {
        if (row[2 * (i + 1)] == 0) continue;                // stays on the interpreter
        const uint64_t entry = (uint64_t)(uintptr_t)d_table + (uint64_t)row[2 * (i + 1)];
        e = hipMemcpy((uint8_t*)progs[i]->d_desc + offsetof(mg_pdesc, jit_entry), &entry,
                      sizeof entry, hipMemcpyHostToDevice);
        if (e == hipSuccess) memcpy(&progs[i]->h_desc.jit_entry, &entry, sizeof entry);
        if (e != hipSuccess) {
            mg_jit_detach(j);
            return fail(ctx, MG_E_HIP, "JIT attach: %s", hipGetErrorString(e));
        }
        if (progs[i]->jit && progs[i]->jit != j) {    // re-attached: the old image lets go
            auto& v = progs[i]->jit->progs;
            v.erase(std::remove(v.begin(), v.end(), progs[i]), v.end());
        }
        progs[i]->jit = j;
        j->progs.push_back(progs[i]);
    }
    *out = j;
    return MG_OK;
}

// Back to the interpreter for every attached program (their descriptors'
// entries cleared), then the code object is unloaded.  Batches created while
// attached keep stale entries: free them first.
void mg_jit_detach(mg_jit* j) {
    if (!j) return;
    (void)hipSetDevice(j->ctx->device);
    const uint64_t zero = 0;
    for (mg_prog* p : j->progs) {
        (void)hipMemcpy((uint8_t*)p->d_desc + offsetof(mg_pdesc, jit_entry), &zero, sizeof zero,
                        hipMemcpyHostToDevice);
        memcpy(&p->h_desc.jit_entry, &zero, sizeof zero);
        p->jit = nullptr;
    }
    (void)hipDeviceSynchronize();
    if (j->module) (void)hipModuleUnload(j->module);
    delete j;
}

int mg_keccak256(mg_ctx* ctx, const uint8_t* data, const uint64_t* offsets, const uint32_t* lens,
                 uint32_t n, uint8_t* out) {
    if (!ctx || (n && (!offsets || !lens || !out))) return fail(ctx, MG_E_ARG, "null argument");
    if (n == 0) return MG_OK;
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t end = offsets[i] + lens[i];
        if (end > total) total = end;
    }
    if (total && !data) return fail(ctx, MG_E_ARG, "null data");
    const size_t off_b = (size_t)n * 8, len_b = (size_t)n * 4, out_b = (size_t)n * 32;
    void* ws;
    int rc = workspace(ctx, total + off_b + len_b + out_b + 1024, &ws);
    if (rc) return rc;
    uint8_t* base = (uint8_t*)ws;
    uint64_t* d_off = (uint64_t*)base;
    uint32_t* d_len = (uint32_t*)(base + off_b);
    uint8_t* d_out = base + ((off_b + len_b + 255) & ~(size_t)255);
    uint8_t* d_data = d_out + ((out_b + 255) & ~(size_t)255);
    HIPCHECK(ctx, hipMemcpyAsync(d_off, offsets, off_b, hipMemcpyHostToDevice, ctx->stream));
    HIPCHECK(ctx, hipMemcpyAsync(d_len, lens, len_b, hipMemcpyHostToDevice, ctx->stream));
    if (total)
        HIPCHECK(ctx, hipMemcpyAsync(d_data, data, total, hipMemcpyHostToDevice, ctx->stream));
    HIPCHECK(ctx, mg_launch_keccak(d_data, d_off, d_len, n, d_out, ctx->stream));
    HIPCHECK(ctx, hipMemcpyAsync(out, d_out, out_b, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    return MG_OK;
}

}  // extern "C"
