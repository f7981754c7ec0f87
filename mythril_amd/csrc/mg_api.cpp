// C ABI of libmythgpu (include/mythgpu.h).  Host-side validation, device
// memory management and kernel launches.  Every program is validated before
// upload so that no instruction can index outside the register file, the LDS
// spill area, the constant pool, the leaf table or the probe buffer.

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mythgpu.h"
#include "mythgpu_ir.h"
#include "mg_device.h"

hipError_t mg_launch_interp(int gen, const mg_pdesc* d_descs, uint32_t n_progs, const mg_run& run,
                            uint32_t lds_slots, hipStream_t stream);
hipError_t mg_launch_keccak(const uint8_t* d_data, const uint64_t* d_off, const uint32_t* d_len,
                            uint32_t n, uint8_t* d_out, hipStream_t stream);

#define MG_VERSION 1

struct mg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    char name[256] = {0};
    int cus = 0;
    // grow-only device workspace for synchronous calls
    void* ws = nullptr;
    size_t ws_size = 0;
};

struct mg_prog {
    mg_ctx* ctx = nullptr;
    void* d_blob = nullptr;         // code | consts | gen | desc
    mg_pdesc* d_desc = nullptr;
    uint32_t n_ins = 0, n_consts = 0, n_leaves = 0, n_lds = 0, n_probes = 0;
};

struct mg_batch {
    mg_ctx* ctx = nullptr;
    mg_pdesc* d_descs = nullptr;
    uint32_t n = 0;
    uint32_t max_lds = 0;
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

extern "C" {

int mg_version(void) { return MG_VERSION; }

int mg_config(uint32_t* out, uint32_t n) {
    const uint32_t cfg[4] = {MG_VERSION, MG_NREG, MG_MAX_LDS, MG_MAX_PSLOTS};
    if (!out) return MG_E_ARG;
    for (uint32_t i = 0; i < n && i < 4; ++i) out[i] = cfg[i];
    return MG_OK;
}

int mg_init(int device, mg_ctx** out) {
    if (!out) return MG_E_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return MG_E_NODEV;
    if (device < 0 || device >= n) return MG_E_NODEV;
    mg_ctx* ctx = new mg_ctx();
    ctx->device = device;
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
    *out = ctx;
    return MG_OK;
}

void mg_free(mg_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->ws) (void)hipFree(ctx->ws);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* mg_last_error(const mg_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }

int mg_device_info(mg_ctx* ctx, char* name, size_t name_len, int* n_cus) {
    if (!ctx) return MG_E_ARG;
    if (name && name_len) snprintf(name, name_len, "%s", ctx->name);
    if (n_cus) *n_cus = ctx->cus;
    return MG_OK;
}

static int validate(mg_ctx* ctx, const uint32_t* code, uint32_t n_ins, uint32_t n_consts,
                    const mg_leafgen* leaves, uint32_t n_leaves, uint32_t n_lds,
                    uint32_t n_spill, uint32_t n_probes) {
    if (n_lds > MG_MAX_LDS) return fail(ctx, MG_E_ARG, "too many LDS slots (%u)", n_lds);
    if (n_spill < n_lds || n_spill - n_lds > MG_MAX_PSLOTS)
        return fail(ctx, MG_E_ARG, "spill slots %u (LDS %u)", n_spill, n_lds);
    for (uint32_t i = 0; i < n_leaves; ++i) {
        const mg_leafgen& g = leaves[i];
        if (g.width < 1 || g.width > MG_MAX_WIDTH)
            return fail(ctx, MG_E_ARG, "leaf %u: width %u", i, g.width);
        if ((uint64_t)g.pool_off + g.pool_n > n_consts)
            return fail(ctx, MG_E_ARG, "leaf %u: pool outside const table", i);
        if (!(g.pct_uniform <= g.pct_small && g.pct_small <= g.pct_boundary &&
              g.pct_boundary <= 100))
            return fail(ctx, MG_E_ARG, "leaf %u: class thresholds", i);
    }
    for (uint32_t pc = 0; pc < n_ins; ++pc) {
        const uint32_t* in = code + 4 * pc;
        const uint32_t op = in[0] & 0xFF, w = (in[0] >> 8) & 0x3FF, imm0 = in[2];
        if (op >= MG_NUM_OPS) return fail(ctx, MG_E_ARG, "ins %u: bad opcode %u", pc, op);
        if ((in[0] & ~(0x3FFFFu | MG_ROOT_FLAG)) != 0)
            return fail(ctx, MG_E_ARG, "ins %u: reserved bits set", pc);
        for (int k = 0; k < 4; ++k)
            if (((in[1] >> (8 * k)) & 0xFF) >= MG_NREG)
                return fail(ctx, MG_E_ARG, "ins %u: slot out of range", pc);
        const bool needs_w = op != MG_NOP && op != MG_SPILL && op != MG_OUT && op != MG_ROOT;
        if (needs_w && (w < 1 || w > MG_MAX_WIDTH))
            return fail(ctx, MG_E_ARG, "ins %u: width %u", pc, w);
        switch (op) {
        case MG_CONST:
            if (imm0 >= n_consts) return fail(ctx, MG_E_ARG, "ins %u: const %u", pc, imm0);
            break;
        case MG_LEAF:
            if (imm0 >= n_leaves) return fail(ctx, MG_E_ARG, "ins %u: leaf %u", pc, imm0);
            break;
        case MG_SPILL:
        case MG_RELOAD:
            if (imm0 >= n_spill) return fail(ctx, MG_E_ARG, "ins %u: spill slot %u", pc, imm0);
            break;
        case MG_OUT:
            if (imm0 >= n_probes) return fail(ctx, MG_E_ARG, "ins %u: probe %u", pc, imm0);
            break;
        case MG_CONCAT:
            if (imm0 < 1 || imm0 >= w) return fail(ctx, MG_E_ARG, "ins %u: concat split", pc);
            break;
        case MG_EXTRACT:
            if (imm0 + w > MG_MAX_WIDTH) return fail(ctx, MG_E_ARG, "ins %u: extract range", pc);
            break;
        case MG_SEXT:
            if (imm0 < 1 || imm0 > w) return fail(ctx, MG_E_ARG, "ins %u: sext width", pc);
            break;
        default:
            break;
        }
    }
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
    int rc = validate(ctx, code, n_ins, n_consts, leaves, n_leaves, n_lds_slots, n_spill_slots,
                      n_probes);
    if (rc) return rc;
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    // 8 zeroed NOPs after the code: the interpreter prefetches up to 8 ahead
    const size_t code_b = (size_t)(n_ins + 8) * 16, const_b = (size_t)n_consts * 32,
                 gen_b = (size_t)n_leaves * sizeof(mg_leafgen);
    auto align = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t off_const = align(code_b), off_gen = off_const + align(const_b),
                 off_desc = off_gen + align(gen_b), total = off_desc + align(sizeof(mg_pdesc));
    std::vector<uint8_t> blob(total, 0);
    if (n_ins) memcpy(blob.data(), code, (size_t)n_ins * 16);   // + zeroed NOP padding
    if (const_b) memcpy(blob.data() + off_const, consts, const_b);
    if (gen_b) memcpy(blob.data() + off_gen, leaves, gen_b);
    void* d = nullptr;
    HIPCHECK(ctx, hipMalloc(&d, total));
    uint8_t* db = (uint8_t*)d;
    mg_pdesc desc;
    desc.code = (const uint32_t*)db;
    desc.consts = (const uint32_t*)(db + off_const);
    desc.gen = (const mg_leafgen*)(db + off_gen);
    desc.n_ins = n_ins;
    desc.n_leaves = n_leaves;
    desc.n_lds = n_lds_slots;
    desc.n_probes = n_probes;
    desc.prog_seed = prog_seed;
    memcpy(blob.data() + off_desc, &desc, sizeof desc);
    hipError_t e = hipMemcpy(d, blob.data(), total, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(d);
        return fail(ctx, MG_E_HIP, "upload: %s", hipGetErrorString(e));
    }
    mg_prog* p = new mg_prog();
    p->ctx = ctx;
    p->d_blob = d;
    p->d_desc = (mg_pdesc*)(db + off_desc);
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
    (void)hipFree(p->d_blob);
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
    HIPCHECK(ctx, mg_launch_interp(0, prog->d_desc, 1, run, prog->n_lds, ctx->stream));
    HIPCHECK(ctx, hipMemcpyAsync(root_bits, run.root_bits, root_b, hipMemcpyDeviceToHost,
                                 ctx->stream));
    if (probes && probe_b)
        HIPCHECK(ctx, hipMemcpyAsync(probes, run.probes, probe_b, hipMemcpyDeviceToHost,
                                     ctx->stream));
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
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
    HIPCHECK(ctx, mg_launch_interp(1, prog->d_desc, 1, run, prog->n_lds, ctx->stream));
    HIPCHECK(ctx, hipMemcpyAsync(root_bits, run.root_bits, root_b, hipMemcpyDeviceToHost,
                                 ctx->stream));
    if (probe_b)
        HIPCHECK(ctx, hipMemcpyAsync(probes, run.probes, probe_b, hipMemcpyDeviceToHost,
                                     ctx->stream));
    if (leaf_b)
        HIPCHECK(ctx, hipMemcpyAsync(leaves_out, run.leaves_out, leaf_b, hipMemcpyDeviceToHost,
                                     ctx->stream));
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    return MG_OK;
}

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
    // chunk so that a single launch stays well under a second
    const uint64_t chunk = 1ull << 24;
    for (uint64_t done = 0; done < n_cand; done += chunk) {
        mg_run run = empty_run();
        run.n_assign = n_cand - done < chunk ? n_cand - done : chunk;
        run.stride = run.n_assign;
        run.first_sat = d_first;
        run.seed = gen->seed;
        run.first_index = gen->first_index + done;
        HIPCHECK(ctx, mg_launch_interp(1, prog->d_desc, 1, run, prog->n_lds, ctx->stream));
        unsigned long long h = ~0ull;
        HIPCHECK(ctx, hipMemcpyAsync(&h, d_first, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
        if (h != ~0ull) {
            *first_sat = (int64_t)h;
            break;
        }
    }
    if (*first_sat >= 0 && witness_leaves && prog->n_leaves) {
        // regenerate the winning candidate (counter-based streams: no gather)
        mg_run run = empty_run();
        run.n_assign = 1;
        run.stride = 1;
        run.seed = gen->seed;
        run.first_index = (uint64_t)*first_sat;
        run.leaves_out = (uint32_t*)((uint8_t*)ws + 256);
        HIPCHECK(ctx, hipMemsetAsync(run.leaves_out, 0, leaf_b, ctx->stream));
        HIPCHECK(ctx, mg_launch_interp(1, prog->d_desc, 1, run, prog->n_lds, ctx->stream));
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
    uint32_t max_lds = 0;
    for (uint32_t i = 0; i < n_progs; ++i) {
        if (!progs[i] || progs[i]->ctx != ctx) return fail(ctx, MG_E_ARG, "program %u", i);
        HIPCHECK(ctx, hipMemcpy(&descs[i], progs[i]->d_desc, sizeof(mg_pdesc),
                                hipMemcpyDeviceToHost));
        if (progs[i]->n_lds > max_lds) max_lds = progs[i]->n_lds;
    }
    mg_batch* b = new mg_batch();
    b->ctx = ctx;
    b->n = n_progs;
    b->max_lds = max_lds;
    if (n_progs) {
        hipError_t e = hipMalloc(&b->d_descs, sizeof(mg_pdesc) * n_progs);
        if (e == hipSuccess)
            e = hipMemcpy(b->d_descs, descs.data(), sizeof(mg_pdesc) * n_progs,
                          hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            if (b->d_descs) (void)hipFree(b->d_descs);
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
    if (b->d_descs) (void)hipFree(b->d_descs);
    delete b;
}

int mg_batch_eval_gen(mg_ctx* ctx, mg_batch* b, uint64_t seed, uint64_t first_index,
                      uint64_t n_assign, uint64_t* d_root_bits, uint64_t* d_first_sat,
                      void* stream) {
    if (!ctx || !b) return fail(ctx, MG_E_ARG, "null argument");
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
        HIPCHECK(ctx, mg_launch_interp(1, b->d_descs + p0, np, run, b->max_lds, s));
    }
    return MG_OK;
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
