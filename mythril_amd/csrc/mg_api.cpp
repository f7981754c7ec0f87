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

#include <cstdlib>
#include <map>

#include "mythgpu.h"
#include "mythgpu_ir.h"
#include "mg_device.h"
#include "mg_asm_handlers.h"

hipError_t mg_launch_asm(const mg_pdesc* d_descs, uint32_t n_progs, const mg_run& run,
                         uint32_t mode, uint32_t lds_slots, uint32_t* table, hipStream_t stream);
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
    // assembly interpreter: handler byte offsets (query launch at init),
    // LDS spill slots per 256-lane block, and the kernel choice
    uint32_t hoff[MGA_NUM_HANDLERS] = {0};
    uint32_t lds_slots = 6;
    bool use_asm = true;
    // generator boundary-value table (device, 48 KiB; MG_BTAB_WORDS)
    uint32_t* d_btab = nullptr;
    // grow-only device workspace for synchronous calls
    void* ws = nullptr;
    size_t ws_size = 0;
};

struct mg_prog {
    mg_ctx* ctx = nullptr;
    void* d_blob = nullptr;         // code | consts | gen | desc | xcode
    mg_pdesc* d_desc = nullptr;
    uint32_t n_ins = 0, n_consts = 0, n_leaves = 0, n_lds = 0, n_probes = 0;
};

static uint32_t kernel_lds_slots(const mg_ctx* ctx, uint32_t n_lds) {
    return ctx->use_asm ? (n_lds < ctx->lds_slots ? n_lds : ctx->lds_slots) : n_lds;
}

// one place that picks the kernel: the assembly interpreter (default) or the
// compiled C++ interpreter kept for A/B (MYTHGPU_KERNEL=cxx)
static hipError_t launch(const mg_ctx* ctx, int gen, const mg_pdesc* d_descs, uint32_t n_progs,
                         const mg_run& run, uint32_t n_lds, hipStream_t stream) {
    if (ctx->use_asm)
        return mg_launch_asm(d_descs, n_progs, run, gen ? 1u : 0u, kernel_lds_slots(ctx, n_lds),
                             nullptr, stream);
    return mg_launch_interp(gen, d_descs, n_progs, run, n_lds, stream);
}

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

static int validate(mg_ctx* ctx, const uint32_t* code, uint32_t n_ins, uint32_t n_consts,
                    const mg_leafgen* leaves, uint32_t n_leaves, uint32_t n_lds,
                    uint32_t n_spill, uint32_t n_probes);

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
    if (e == hipSuccess) e = mg_launch_asm(d_desc, 1, run, 2u, 0, (uint32_t*)d, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(ctx->hoff, d, tab_b, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(ctx, MG_E_HIP, "handler query: %s", hipGetErrorString(e));
    for (int h = 0; h < MGA_NUM_HANDLERS; ++h)
        if (ctx->hoff[h] == 0 || ctx->hoff[h] > (1u << 24))
            return fail(ctx, MG_E_HIP, "handler query: bad offset %u for %d", ctx->hoff[h], h);
    return MG_OK;
}

// ---- IR -> assembly-interpreter records (8 words each) ----------------------
//
// w0 handler byte offset | w1 8*dst | w2 8*a | w3 8*b | w4 8*c / funnel index /
// leaf or probe index | w5 immediate (const / spill byte offset, funnel shift,
// source width) | w6 width | w7 byte offset of an 8- (SEXT: 16-) word mask
// entry appended to the constant table.  The record after a heavy op lives in
// bank A, otherwise banks alternate (asmgen.py: prefetch into the other bank).

struct MaskPool {
    uint32_t base;                                  // first entry index
    std::vector<uint32_t> words;
    std::map<std::vector<uint32_t>, uint32_t> where;
    uint32_t add(const std::vector<uint32_t>& w) {  // returns a byte offset
        auto it = where.find(w);
        if (it != where.end()) return it->second;
        const uint32_t off = (base + (uint32_t)(words.size() / 8)) * 32u;
        words.insert(words.end(), w.begin(), w.end());
        where[w] = off;
        return off;
    }
};

static std::vector<uint32_t> mask_lt(uint32_t w) {     // bits < w
    std::vector<uint32_t> m(8);
    for (uint32_t j = 0; j < 8; ++j)
        m[j] = j < w / 32 ? 0xFFFFFFFFu : (j == w / 32 ? ((1u << (w % 32)) - 1u) : 0u);
    return m;
}

static std::vector<uint32_t> mask_ge(uint32_t w) {     // bits >= w
    std::vector<uint32_t> m = mask_lt(w);
    for (auto& x : m) x = ~x;
    return m;
}

static bool is_compare(uint32_t op) {
    return op == MG_EQ || op == MG_ULT || op == MG_ULE || op == MG_SLT || op == MG_SLE ||
           op == MG_UMULNO;
}

// ops with a one-limb (W32) handler when operands and result fit 32 bits
static bool has_w32(uint32_t op) {
    switch (op) {
    case MG_ADD: case MG_SUB: case MG_AND: case MG_OR: case MG_XOR: case MG_NOT: case MG_NEG:
    case MG_ITE: case MG_EQ: case MG_ULT: case MG_ULE: case MG_EXTRACT: case MG_MOV:
    case MG_CONST:
        return true;
    default:
        return false;
    }
}

// register slots an IR instruction reads or writes (bit mask)
static uint32_t slots_touched(uint32_t op, uint32_t d, uint32_t a, uint32_t b, uint32_t c) {
    switch (op) {
    case MG_NOP: return 0;
    case MG_CONST: case MG_LEAF: case MG_RELOAD: return 1u << d;
    case MG_SPILL: case MG_OUT: case MG_ROOT: return 1u << a;
    case MG_NOT: case MG_NEG: case MG_MOV: case MG_SEXT:
        return (1u << d) | (1u << a);
    // the funnel shifts read one slot beyond their operand (masked off, but
    // the registers are read): the next slot for EXTRACT, the previous one
    // for CONCAT's high part
    case MG_EXTRACT: return ((1u << d) | (3u << a)) & ((1u << MG_NREG) - 1);
    case MG_CONCAT: return (1u << d) | (1u << a) | (a ? 1u << (a - 1) : 0u) | (1u << b);
    case MG_ITE: return (1u << d) | (1u << a) | (1u << b) | (1u << c);
    default: return (1u << d) | (1u << a) | (1u << b);
    }
}

// slots an instruction reads (its destination only when it is also an operand)
static uint32_t slots_read(uint32_t op, uint32_t d, uint32_t a, uint32_t b, uint32_t c) {
    uint32_t m = slots_touched(op, d, a, b, c);
    switch (op) {
    case MG_NOP: case MG_CONST: case MG_LEAF: case MG_RELOAD: return 0;
    case MG_SPILL: case MG_OUT: case MG_ROOT: return m;
    default: break;
    }
    const bool d_operand = d == a || (op != MG_NOT && op != MG_NEG && op != MG_MOV &&
                                      op != MG_EXTRACT && op != MG_SEXT && d == b) ||
                           (op == MG_ITE && d == c) || (op == MG_EXTRACT && d == a + 1) ||
                           (op == MG_CONCAT && a && d == a - 1);
    return d_operand ? m : m & ~(1u << d);
}

static void translate(const uint32_t* hoff, const uint32_t* code, uint32_t n_ins, uint32_t n_consts,
                      uint32_t n_lds, std::vector<uint32_t>& rec, MaskPool& pool) {
    pool.base = n_consts;
    const uint32_t ones = pool.add(mask_lt(256));
    rec.clear();
    rec.reserve((size_t)(n_ins + 4) * 8);
    // clean[s]: limbs 1..7 of slot s are known to be zero (its last value had
    // at most 32 bits); registers start uninitialised
    bool clean[MG_NREG];
    for (int k = 0; k < MG_NREG; ++k) clean[k] = false;
    // slots whose LEAFD loads may still be in flight: a WAITVM record goes
    // before the first instruction that reads or writes one of them
    uint32_t pending = 0;
    int bank = 0;
    auto emit = [&rec]() {
        rec.resize(rec.size() + 8, 0);
        return rec.data() + rec.size() - 8;
    };
    // the last record emitted, when it is a LEAFD / RELOADD: a wait right
    // after it folds into that record (word W = 1, the handler waits)
    size_t last_ld = SIZE_MAX;
    auto wait_vm = [&]() {
        if (last_ld != SIZE_MAX && last_ld + 8 == rec.size()) {
            rec[last_ld + 6] = 1;           // the LEAFD / RELOADD waits itself
        } else {
            emit()[0] = hoff[MGA_HID(MGA_WAITVM, 0, bank)];
            bank = 1 - bank;
        }
        pending = 0;
    };
    // Issue order: every scratch RELOAD and 256-bit LEAF moves up (at most 24
    // places) past the instructions that leave its destination slot (and spill
    // slot) alone, so its loads are in flight early (RELOADD / LEAFD) and
    // waited for only at the first instruction that touches the slot.
    std::vector<uint32_t> order(n_ins);
    for (uint32_t i = 0; i < n_ins; ++i) order[i] = i;
    for (uint32_t q = 0; q < n_ins; ++q) {
        const uint32_t* in = code + 4 * order[q];
        const bool leafd = (in[0] & 0xFF) == MG_LEAF && ((in[0] >> 8) & 0x3FF) == 256;
        if (!leafd && ((in[0] & 0xFF) != MG_RELOAD || in[2] < n_lds)) continue;
        const uint32_t rd = in[1] & 0xFF, slot = leafd ? 0xFFFFFFFFu : in[2];
        uint32_t t = q;
        while (t > 0 && q - t < 24) {
            const uint32_t* p = code + 4 * order[t - 1];
            const uint32_t pop = p[0] & 0xFF;
            if (slots_touched(pop, p[1] & 0xFF, (p[1] >> 8) & 0xFF, (p[1] >> 16) & 0xFF,
                              (p[1] >> 24) & 0xFF) & (1u << rd))
                break;
            if (pop == MG_SPILL && p[2] == slot) break;
            --t;
        }
        if (t < q) {
            const uint32_t moved = order[q];
            for (uint32_t k = q; k > t; --k) order[k] = order[k - 1];
            order[t] = moved;
        }
    }
    for (uint32_t pc = 0; pc <= n_ins; ++pc) {
        if (pc == n_ins) {          // HALT, then one zeroed record (prefetch pad)
            if (pending) wait_vm();
            emit()[0] = hoff[MGA_HID(MGA_HALT, 0, bank)];
            emit();
            break;
        }
        const uint32_t* in = code + 4 * order[pc];
        const uint32_t op = in[0] & 0xFF, w = (in[0] >> 8) & 0x3FF, imm = in[2];
        const uint32_t d = in[1] & 0xFF, a = (in[1] >> 8) & 0xFF, b = (in[1] >> 16) & 0xFF,
                       c = (in[1] >> 24) & 0xFF;
        // a store-chain link: t = (a == b) of wide values, consumed only by
        // the next instruction, an ITE on t -> one EQSEL record
        if (op == MG_EQ && w > 32 && !(in[0] & MG_ROOT_FLAG) && pc + 1 < n_ins) {
            const uint32_t* nx = code + 4 * order[pc + 1];
            const uint32_t nd = nx[1] & 0xFF, na = (nx[1] >> 8) & 0xFF, nb = (nx[1] >> 16) & 0xFF,
                           nc = (nx[1] >> 24) & 0xFF;
            bool fuse = (nx[0] & 0xFF) == MG_ITE && !(nx[0] & MG_ROOT_FLAG) && nc == d &&
                        na != d && nb != d;
            for (uint32_t q = pc + 2; fuse && q < n_ins; ++q) {     // is t dead after the ITE?
                const uint32_t* f = code + 4 * order[q];
                const uint32_t fop = f[0] & 0xFF, fd = f[1] & 0xFF, fa = (f[1] >> 8) & 0xFF,
                               fb = (f[1] >> 16) & 0xFF, fc = (f[1] >> 24) & 0xFF;
                if (slots_read(fop, fd, fa, fb, fc) & (1u << d)) fuse = false;
                else if (slots_touched(fop, fd, fa, fb, fc) & (1u << d)) break;   // rewritten
            }
            if (fuse) {
                const uint32_t touch = slots_touched(op, d, a, b, c) | slots_touched(MG_ITE, nd, na, nb, nc);
                if (pending & touch) wait_vm();
                uint32_t* r = emit();
                uint32_t var;
                r[1] = 8 * nd; r[2] = 8 * a; r[3] = 8 * b;
                if (nd == na) { var = MGA_V_NEG; r[4] = 8 * nb; }          // keep F[d] where equal
                else if (nd == nb) { var = 0; r[4] = 8 * na; }             // take F[a] where equal
                else { var = MGA_V_GEN; r[4] = 8 * na; r[5] = 8 * nb; }
                r[0] = hoff[MGA_HID(MGA_EQSEL, var, bank)];
                bank = 1 - bank;
                clean[nd] = ((nx[0] >> 8) & 0x3FF) <= 32;     // canonical values
                ++pc;
                continue;
            }
        }
        const bool leafd = op == MG_LEAF && w == 256;
        const bool reloadd = op == MG_RELOAD && imm >= n_lds;
        if (pending && (slots_touched(op, d, a, b, c) & pending)) wait_vm();
        if (leafd || reloadd) pending |= 1u << d;
        uint32_t* r = emit();
        uint32_t var = (in[0] & MG_ROOT_FLAG) ? MGA_V_ROOT : 0;
        const bool writes = op != MG_NOP && op != MG_SPILL && op != MG_OUT && op != MG_ROOT;
        // result fits one limb: Bool results, or values of at most 32 bits
        const bool narrow = is_compare(op) || (writes && w <= 32);
        const bool w32 = has_w32(op) && w <= 32;       // compares: w = operand width
        if (w32) var |= MGA_V_W32;
        if (writes && narrow && clean[d]) var |= MGA_V_DC;
        const uint32_t maskv = w32 ? (w < 32 ? MGA_V_MASK : 0) : ((w >= 1 && w < 256) ? MGA_V_MASK : 0);
        r[1] = 8 * d; r[2] = 8 * a; r[3] = 8 * b; r[4] = 8 * c; r[5] = 0; r[6] = w; r[7] = ones;
        int aop = MGA_NOP;
        switch (op) {
        case MG_NOP: aop = MGA_NOP; break;
        case MG_CONST: aop = MGA_CONST; r[5] = imm * 32u; break;
        case MG_LEAF:
            aop = MGA_LEAF; r[4] = imm;
            if (leafd) { aop = MGA_LEAFD; var = d; }
            else if (maskv) { var |= MGA_V_MASK; r[7] = pool.add(mask_lt(w)); }
            break;
        case MG_SPILL:              // spills and reloads: the variant is the slot
            if (imm < n_lds) { aop = MGA_SPILL_LDS; var = a; r[5] = imm * 2u * 256u * 16u; }
            else { aop = MGA_SPILL_SCR; var = a; r[5] = (imm - n_lds) * 32u; }
            break;
        case MG_RELOAD:
            if (imm < n_lds) { aop = MGA_RELOAD_LDS; var = d; r[5] = imm * 2u * 256u * 16u; }
            else { aop = MGA_RELOADD; var = d; r[5] = (imm - n_lds) * 32u; }
            break;
        case MG_ADD: aop = MGA_ADD; goto masked;
        case MG_SUB: aop = MGA_SUB; goto masked;
        case MG_MUL: aop = MGA_MUL; goto masked;
        case MG_NEG: aop = MGA_NEG; goto masked;
        case MG_NOT: aop = MGA_NOT; goto masked;
        case MG_UDIV: aop = MGA_UDIV; goto masked;
        case MG_UREM: aop = MGA_UREM; goto masked;
        case MG_SDIV: aop = MGA_SDIV; goto masked;
        case MG_SREM: aop = MGA_SREM; goto masked;
        case MG_SMOD: aop = MGA_SMOD; goto masked;
        case MG_SHL: aop = MGA_SHL; goto masked;
        case MG_LSHR: aop = MGA_LSHR; goto masked;
        case MG_ASHR: aop = MGA_ASHR; goto masked;
        case MG_SLT: aop = MGA_SLT; goto masked;
        case MG_SLE: aop = MGA_SLE; goto masked;
        case MG_UMULNO: aop = MGA_UMULNO;
        masked:
            if (maskv) { var |= MGA_V_MASK; r[7] = pool.add(mask_lt(w)); }
            break;
        case MG_AND: aop = MGA_AND; break;
        case MG_OR: aop = MGA_OR; break;
        case MG_XOR: aop = MGA_XOR; break;
        case MG_EQ: aop = MGA_EQ; break;
        case MG_ULT: aop = MGA_ULT; break;
        case MG_ULE: aop = MGA_ULE; break;
        case MG_ITE: aop = MGA_ITE; break;
        case MG_CONCAT: {           // R = a << imm | b: static limb shift in the variant
            aop = MGA_CONCATQ;
            const uint32_t q = imm >> 5, bs = imm & 31;
            var = q | (bs ? 8u : 0u);
            r[4] = 8 * a + 8 - q - (bs ? 1 : 0);
            r[5] = bs ? 32 - bs : 0;
            r[7] = ~((1u << bs) - 1u);              // limb q: bits >= bs from a
            break;
        }
        case MG_EXTRACT:            // R = (a >> imm) & mask(w)
            r[4] = 8 * a + (imm >> 5) + 8;
            r[5] = imm & 31;
            if (w > 32) {           // static result limbs; top-limb mask inline
                aop = MGA_EXTRACTN;
                var = (w + 31) / 32 - 1;
                r[7] = (w & 31) ? (1u << (w & 31)) - 1u : 0xFFFFFFFFu;
            } else {
                aop = MGA_EXTRACT;
                r[7] = pool.add(mask_lt(w));
            }
            break;
        case MG_SEXT: {             // from imm bits to w bits: 16-word mask entry
            aop = MGA_SEXT;
            r[5] = imm;
            std::vector<uint32_t> m = mask_lt(imm), m2 = mask_lt(w);
            m.insert(m.end(), m2.begin(), m2.end());
            r[7] = pool.add(m);
            break;
        }
        case MG_OUT: aop = MGA_OUT; r[4] = imm; break;
        case MG_ROOT: aop = MGA_ROOT; break;
        case MG_MOV: aop = MGA_MOV; break;
        default: aop = MGA_NOP; break;
        }
        // in place: the destination is operand a's slot (swap operands of
        // commutative ops, use the reversed forms SUBR / ITEN otherwise)
        if (!(var & MGA_V_W32)) {
            const bool comm = op == MG_ADD || op == MG_AND || op == MG_OR || op == MG_XOR;
            if ((comm || op == MG_SUB || op == MG_ITE) && d == b && d != a) {
                const uint32_t t = r[2]; r[2] = r[3]; r[3] = t;
                if (op == MG_SUB) aop = MGA_SUBR;
                if (op == MG_ITE) aop = MGA_ITEN;
                var |= MGA_V_IP;
            } else if ((comm || op == MG_SUB || op == MG_ITE || op == MG_NOT || op == MG_NEG) &&
                       d == a) {
                var |= MGA_V_IP;
            }
        }
        r[0] = hoff[MGA_HID(aop, var, bank)];
        if (aop == MGA_LEAFD || aop == MGA_RELOADD) {
            r[6] = 0;
            last_ld = (size_t)(r - rec.data());
        }
        if (writes) clean[d] = narrow;
        bank = mga_is_heavy(aop) ? 0 : 1 - bank;
    }
}

extern "C" {

int mg_version(void) { return MG_VERSION; }

int mg_translate(const uint32_t* code, uint32_t n_ins, uint32_t n_consts, uint32_t n_lds,
                 const uint32_t* handler_off, uint32_t n_handlers, uint32_t* records,
                 uint32_t max_record_words, uint32_t* n_record_words, uint32_t* masks,
                 uint32_t max_mask_words, uint32_t* n_mask_words) {
    if ((n_ins && !code) || !handler_off || n_handlers != MGA_NUM_HANDLERS || !n_record_words ||
        !n_mask_words)
        return MG_E_ARG;
    // leaf and probe tables are not known here: only their indices' shape
    int rc = validate(nullptr, code, n_ins, n_consts, nullptr, 0xFFFFFFFFu, MG_MAX_LDS,
                      MG_MAX_LDS + MG_MAX_PSLOTS, 0xFFFFFFFFu);
    if (rc) return rc;
    if (n_lds > MG_MAX_LDS) return MG_E_ARG;
    std::vector<uint32_t> rec;
    MaskPool pool;
    translate(handler_off, code, n_ins, n_consts, n_lds, rec, pool);
    *n_record_words = (uint32_t)rec.size();
    *n_mask_words = (uint32_t)pool.words.size();
    if (rec.size() > max_record_words || pool.words.size() > max_mask_words) return MG_E_ARG;
    if (records) memcpy(records, rec.data(), rec.size() * 4);
    if (masks && !pool.words.empty()) memcpy(masks, pool.words.data(), pool.words.size() * 4);
    return MG_OK;
}

int mg_config(uint32_t* out, uint32_t n) {
    const uint32_t cfg[4] = {MG_VERSION, MG_NREG, MG_MAX_LDS, MG_MAX_PSLOTS};
    if (!out) return MG_E_ARG;
    for (uint32_t i = 0; i < n && i < 4; ++i) out[i] = cfg[i];
    return MG_OK;
}

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
    if (const char* k = getenv("MYTHGPU_KERNEL")) ctx->use_asm = strcmp(k, "cxx") != 0;
    if (const char* l = getenv("MYTHGPU_LDS_SLOTS")) {
        const long v = strtol(l, nullptr, 10);
        if (v >= 0 && v <= MG_MAX_LDS) ctx->lds_slots = (uint32_t)v;
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
    if (ctx->ws) (void)hipFree(ctx->ws);
    if (ctx->d_btab) (void)hipFree(ctx->d_btab);
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
    for (uint32_t i = 0; leaves && i < n_leaves; ++i) {
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
    // assembly records + translator masks (appended to the constant table)
    std::vector<uint32_t> rec;
    MaskPool pool;
    translate(ctx->hoff, code, n_ins, n_consts, kernel_lds_slots(ctx, n_spill_slots), rec, pool);
    // generator pools expanded to (v - 1, v, v + 1) triples (mod 2^256), so
    // the pool class is one indexed load (pool[e] + delta - 1, gen_ref.py)
    const uint32_t n_masks = (uint32_t)(pool.words.size() / 8);
    std::vector<uint32_t> pm(consts ? (size_t)n_consts * 24 : 0);
    for (uint32_t c = 0; c < n_consts; ++c) {
        const uint32_t* v = consts + (size_t)c * 8;
        uint32_t* o = pm.data() + (size_t)c * 24;
        uint64_t bm = 1, bp = 1;                 // borrow of v - 1, carry of v + 1
        for (int j = 0; j < 8; ++j) {
            o[j] = v[j] - (uint32_t)bm;
            bm = bm && v[j] == 0;
            o[8 + j] = v[j];
            o[16 + j] = v[j] + (uint32_t)bp;
            bp = bp && v[j] == 0xFFFFFFFFu;
        }
    }
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
    // 8 zeroed NOPs after the IR code: the C++ interpreter prefetches ahead
    const size_t code_b = (size_t)(n_ins + 8) * 16, const_b = (size_t)n_const_all * 32,
                 gen_b = gdev.size() * sizeof(mg_leafgen_dev), rec_b = rec.size() * 4;
    auto align = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t off_const = align(code_b), off_gen = off_const + align(const_b),
                 off_desc = off_gen + align(gen_b), off_rec = off_desc + align(sizeof(mg_pdesc)),
                 total = off_rec + align(rec_b);
    std::vector<uint8_t> blob(total, 0);
    if (n_ins) memcpy(blob.data(), code, (size_t)n_ins * 16);   // + zeroed NOP padding
    if (n_consts) memcpy(blob.data() + off_const, consts, (size_t)n_consts * 32);
    if (!pool.words.empty())
        memcpy(blob.data() + off_const + (size_t)n_consts * 32, pool.words.data(),
               pool.words.size() * 4);
    if (!pm.empty())
        memcpy(blob.data() + off_const + (size_t)(n_consts + n_masks) * 32, pm.data(),
               pm.size() * 4);
    if (gen_b) memcpy(blob.data() + off_gen, gdev.data(), gen_b);
    memcpy(blob.data() + off_rec, rec.data(), rec_b);
    void* d = nullptr;
    HIPCHECK(ctx, hipMalloc(&d, total));
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
    HIPCHECK(ctx, launch(ctx, 0, prog->d_desc, 1, run, prog->n_lds, ctx->stream));
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
    HIPCHECK(ctx, launch(ctx, 1, prog->d_desc, 1, run, prog->n_lds, ctx->stream));
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
        HIPCHECK(ctx, launch(ctx, 1, prog->d_desc, 1, run, prog->n_lds, ctx->stream));
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
        HIPCHECK(ctx, launch(ctx, 1, b->d_descs + p0, np, run, b->max_lds, s));
    }
    return MG_OK;
}

int mg_batch_search(mg_ctx* ctx, mg_batch* b, const mg_gen* gen, uint64_t n_cand,
                    int64_t* first_sat) {
    if (!ctx || !b || !gen || (b->n && !first_sat)) return fail(ctx, MG_E_ARG, "null argument");
    for (uint32_t i = 0; i < b->n; ++i) first_sat[i] = -1;
    if (n_cand == 0 || b->n == 0) return MG_OK;
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    void* ws;
    int rc = workspace(ctx, (size_t)b->n * 8, &ws);
    if (rc) return rc;
    unsigned long long* d_first = (unsigned long long*)ws;
    HIPCHECK(ctx, hipMemsetAsync(d_first, 0xFF, (size_t)b->n * 8, ctx->stream));
    std::vector<unsigned long long> h(b->n, ~0ull);
    // ~2^24 lanes per launch over all programs (a launch stays well under a
    // second); solved programs' blocks exit at once in later chunks
    uint64_t chunk = (1ull << 24) / b->n;
    chunk = chunk < 4096 ? 4096 : (chunk + 255) & ~255ull;
    for (uint64_t done = 0; done < n_cand; done += chunk) {
        for (uint32_t p0 = 0; p0 < b->n; p0 += 65535) {
            const uint32_t np = b->n - p0 < 65535 ? b->n - p0 : 65535;
            mg_run run = empty_run();
            run.n_assign = n_cand - done < chunk ? n_cand - done : chunk;
            run.stride = run.n_assign;
            run.first_sat = d_first + p0;
            run.seed = gen->seed;
            run.first_index = gen->first_index + done;
            run.skip_solved = 1;
            HIPCHECK(ctx, launch(ctx, 1, b->d_descs + p0, np, run, b->max_lds, ctx->stream));
        }
        HIPCHECK(ctx, hipMemcpyAsync(h.data(), d_first, (size_t)b->n * 8, hipMemcpyDeviceToHost,
                                     ctx->stream));
        HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
        bool all = true;
        for (uint32_t i = 0; i < b->n; ++i) all = all && h[i] != ~0ull;
        if (all) break;
    }
    for (uint32_t i = 0; i < b->n; ++i) first_sat[i] = h[i] == ~0ull ? -1 : (int64_t)h[i];
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
