// MI355X (gfx950) interpreter for mythgpu IR — one lane = one candidate
// assignment, 256-bit values as 8 x 32-bit limbs, SMT-LIB 2.6 bit-vector
// semantics (the theory z3 evaluates for mythril/support/model.py:15-49).
//
// Design:
//  * The instruction stream is wave-uniform: 16-byte instructions read with
//    scalar loads, decoded in SALU, dispatched by a uniform switch — no
//    opcode divergence.
//  * The register file lives in VGPRs as 8 per-limb v16 vectors
//    (F0..F7[slot]).  Operands are read with GPR-index mode
//    (s_set_gpr_idx_on ... gpr_idx(SRC0)), and every instruction writes its
//    result once, at a single point of the loop body, with gpr_idx(DST) — so
//    the compiler never copies the file (a conditional write would).
//  * Values that do not fit the 15 VGPR slots are spilled to LDS in a
//    [slot][half][lane][4] layout (conflict-free ds_{read,write}_b128).
//  * Carry chains use v_add_co/v_addc_co (__builtin_addc), products
//    v_mad_u64_u32; division is Knuth D with a Moller-Granlund 2-by-1
//    reciprocal, branch-free so lanes never diverge.
//  * No MFMA: the work is integer VALU.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mythgpu_ir.h"
#include "mg_device.h"

// one GPR-indexed vector per limb; MG_NREG must be a register-tuple size
// (8, 12 or 16) for index-mode moves
typedef uint32_t vfile __attribute__((ext_vector_type(MG_NREG)));
// constant address space: uniform loads through it become s_load (scalar
// cache), which keeps opcodes and slot indices in SGPRs
typedef __attribute__((address_space(4))) const uint32_t cu32;
typedef __attribute__((address_space(4))) const mg_leafgen_dev cgen;

#define DEV static __device__ __forceinline__

// ---------------------------------------------------------------------------
// 256-bit helpers (arrays of 8 limbs, index 0 = least significant)
// ---------------------------------------------------------------------------

DEV void add256(const uint32_t* a, const uint32_t* b, uint32_t* r) {
    unsigned c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = __builtin_addc(a[j], b[j], c, &c);
}

// r = a - b; returns the final borrow (1 if a < b unsigned)
DEV unsigned sub256(const uint32_t* a, const uint32_t* b, uint32_t* r) {
    unsigned bo = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = __builtin_subc(a[j], b[j], bo, &bo);
    return bo;
}

DEV unsigned ult256(const uint32_t* a, const uint32_t* b) {
    unsigned bo = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) (void)__builtin_subc(a[j], b[j], bo, &bo);
    return bo;
}

DEV void neg256(const uint32_t* a, uint32_t* r) {
    unsigned bo = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = __builtin_subc(0u, a[j], bo, &bo);
}

DEV unsigned is_zero256(const uint32_t* a) {
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) o |= a[j];
    return o == 0;
}

// low 256 bits of a*b (schoolbook, row-wise with 64-bit mad accumulation)
DEV void mul256(const uint32_t* a, const uint32_t* b, uint32_t* r) {
    uint32_t t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t carry = 0;
#pragma unroll
        for (int j = 0; j < 7 - i; ++j) {
            uint64_t p = (uint64_t)a[i] * b[j] + t[i + j] + carry;
            t[i + j] = (uint32_t)p;
            carry = (uint32_t)(p >> 32);
        }
        t[7] = t[7] + a[i] * b[7 - i] + carry;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = t[j];
}

// full 512-bit product
DEV void mul512(const uint32_t* a, const uint32_t* b, uint32_t* r) {
#pragma unroll
    for (int j = 0; j < 16; ++j) r[j] = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t carry = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint64_t p = (uint64_t)a[i] * b[j] + r[i + j] + carry;
            r[i + j] = (uint32_t)p;
            carry = (uint32_t)(p >> 32);
        }
        r[i + 8] = carry;
    }
}

// per-lane variable left shift of an N-limb value by s (0 <= s < 32*N).
template <int N>
DEV void shl_n(const uint32_t* x, uint32_t s, uint32_t* r) {
    uint32_t t[N];
#pragma unroll
    for (int j = 0; j < N; ++j) t[j] = x[j];
    const uint32_t q = s >> 5, b = s & 31;
#pragma unroll
    for (int st = 1; st < N; st <<= 1) {
        const bool on = (q & st) != 0;
#pragma unroll
        for (int j = N - 1; j >= 0; --j) t[j] = on ? (j >= st ? t[j - st] : 0u) : t[j];
    }
    // bit shift; (lo >> 1) >> (31 - b) avoids the b == 0 shift-by-32 case
#pragma unroll
    for (int j = N - 1; j >= 1; --j) t[j] = (t[j] << b) | ((t[j - 1] >> 1) >> (31 - b));
    t[0] <<= b;
#pragma unroll
    for (int j = 0; j < N; ++j) r[j] = t[j];
}

// per-lane variable logical right shift of an N-limb value by s (< 32*N),
// producing the low M limbs.  v_alignbit does the funnel (b == 0 exact).
template <int N, int M>
DEV void shr_n(const uint32_t* x, uint32_t s, uint32_t* r) {
    uint32_t t[N + 1];
#pragma unroll
    for (int j = 0; j < N; ++j) t[j] = x[j];
    t[N] = 0;
    const uint32_t q = s >> 5, b = s & 31;
#pragma unroll
    for (int st = 1; st < N; st <<= 1) {
        const bool on = (q & st) != 0;
#pragma unroll
        for (int j = 0; j < N; ++j) t[j] = on ? (j + st < N ? t[j + st] : 0u) : t[j];
    }
#pragma unroll
    for (int j = 0; j < M; ++j) r[j] = __builtin_amdgcn_alignbit(t[j + 1], t[j], b);
}

// number of leading zeros of a nonzero 256-bit value (0..255); 256 if zero
DEV uint32_t clz256(const uint32_t* v) {
    uint32_t lz = 256;
#pragma unroll
    for (int j = 0; j < 8; ++j) lz = v[j] ? (uint32_t)((7 - j) * 32) + __builtin_clz(v[j]) : lz;
    return lz;
}

// Unsigned 256/256 division, Knuth algorithm D on 32-bit digits, fully
// unrolled and branch-free.  Requires v != 0 (callers substitute 1).
DEV void udivrem256(const uint32_t* u, const uint32_t* v, uint32_t* q, uint32_t* rem) {
    const uint32_t sh = clz256(v);           // normalise: top bit of vn set
    uint32_t vn[8];
    shl_n<8>(v, sh, vn);
    uint32_t un[17];
    {
        uint32_t u16[16];
#pragma unroll
        for (int j = 0; j < 8; ++j) { u16[j] = u[j]; u16[j + 8] = 0; }
        shl_n<16>(u16, sh, un);
        un[16] = 0;
    }
    const uint32_t d = vn[7];
    const uint32_t d6 = vn[6];
    // Moller-Granlund reciprocal v = floor((2^64-1)/d) - 2^32 (d >= 2^31)
    const uint32_t dinv = (uint32_t)(0xFFFFFFFFFFFFFFFFull / d);

#pragma unroll
    for (int j = 7; j >= 0; --j) {
        const uint32_t u2 = un[j + 8], u1 = un[j + 7], u0 = un[j + 6];
        // 2-by-1 division of (u2:u1) by d via the reciprocal (valid if u2 < d)
        const uint32_t a2 = u2 < d ? u2 : 0u;
        uint64_t qq = (uint64_t)dinv * a2 + (((uint64_t)a2 << 32) | u1);
        uint32_t q1 = (uint32_t)(qq >> 32) + 1u;
        const uint32_t q0 = (uint32_t)qq;
        uint32_t r = u1 - q1 * d;
        const bool c1 = r > q0;
        q1 = c1 ? q1 - 1u : q1;
        r = c1 ? r + d : r;
        const bool c2 = r >= d;
        q1 = c2 ? q1 + 1u : q1;
        r = c2 ? r - d : r;
        // u2 == d (the only u2 >= d case): qhat = b-1, rhat = u1 + d (may be >= b)
        const bool big = u2 >= d;
        uint32_t qh = big ? 0xFFFFFFFFu : q1;
        uint64_t rh = big ? (uint64_t)u1 + d : (uint64_t)r;
        // Knuth's two-digit test, at most two corrections
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            const bool fix = (rh >> 32) == 0 &&
                             (uint64_t)qh * d6 > ((rh << 32) | u0);
            qh = fix ? qh - 1u : qh;
            rh = fix ? rh + d : rh;
        }
        // multiply-subtract qh * vn from un[j .. j+8]
        unsigned bo = 0;
        uint32_t carry = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint64_t p = (uint64_t)qh * vn[i] + carry;
            carry = (uint32_t)(p >> 32);
            un[j + i] = __builtin_subc(un[j + i], (uint32_t)p, bo, &bo);
        }
        un[j + 8] = __builtin_subc(un[j + 8], carry, bo, &bo);
        // add back when the partial remainder went negative (probability
        // ~2/2^32 per lane: skipped unless some lane of the wave needs it)
        if (__any(bo)) {
            const uint32_t m = 0u - bo;
            unsigned c = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) un[j + i] = __builtin_addc(un[j + i], vn[i] & m, c, &c);
            un[j + 8] += c & bo;
        }
        // the window's top digit is now 0 and never read again: keep the
        // quotient digit there (no separate live quotient registers)
        un[j + 8] = qh - bo;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j] = un[j + 8];
    un[8] = 0;
    shr_n<9, 8>(un, sh, rem);
}

// ---------------------------------------------------------------------------
// width helpers (w is wave-uniform)
// ---------------------------------------------------------------------------

// mask of the bits of limb j that lie below width w (w uniform -> SALU)
DEV uint32_t limb_mask(uint32_t w, int j) {
    const uint32_t top = w >> 5, rem = w & 31;
    return (uint32_t)j < top ? 0xFFFFFFFFu : ((uint32_t)j == top ? (1u << rem) - 1u : 0u);
}

DEV void mask_to(uint32_t* x, uint32_t w) {
    if (w < 256) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] &= limb_mask(w, j);
    }
}

// sign-extend from w bits to 256 (in place)
DEV void sext_from(uint32_t* x, uint32_t w) {
    if (w < 256) {
        const uint32_t sb = w - 1;
        uint32_t sl = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) sl = (uint32_t)j == (sb >> 5) ? x[j] : sl;
        const uint32_t neg = 0u - ((sl >> (sb & 31)) & 1u);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] |= neg & ~limb_mask(w, j);
    }
}

DEV uint32_t sign256(const uint32_t* x) { return x[7] >> 31; }

// ---------------------------------------------------------------------------
// device candidate generator (SplitMix64 streams; mirrored by oracle/gen_ref.py)
// ---------------------------------------------------------------------------

DEV uint64_t sm64(uint64_t& s) {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

DEV uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

// candidate generator, v2 range reduction (multiply-high); mirrored by
// oracle/gen_ref.py and the assembly interpreter (asmgen._gen_leaf)
DEV void gen_leaf(uint64_t seed, uint32_t leaf, uint64_t idx, cgen* g, cu32* consts,
                  uint32_t* out) {
    const uint32_t w = g->width;
    uint64_t s = seed ^ (((uint64_t)g->salt_hi << 32) | g->salt_lo) ^ (idx * 0x9E3779B97F4A7C15ull);
    const uint64_t r0 = sm64(s);
    const uint32_t cls = mulhi32((uint32_t)(r0 >> 32), 100u);
    const uint32_t lo = (uint32_t)r0;
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = 0;
    const uint32_t pool_n = g->pool_n;
    if (cls < g->pct_small && cls >= g->pct_uniform) {
        const uint64_t r = sm64(s);
        out[0] = (uint32_t)r;
        out[1] = (uint32_t)(r >> 32);
    } else if (cls < g->pct_boundary && cls >= g->pct_small) {
        const uint32_t kind = mulhi32(lo, 6u);
        const uint32_t k = mulhi32(lo * 0x9E3779B1u, w);
        const uint32_t bit = (kind == 2) ? w - 1 : (kind == 1 ? 0u : k);
        if (kind != 0 && kind != 3) {
#pragma unroll
            for (int j = 0; j < 8; ++j) out[j] = (bit >> 5) == (uint32_t)j ? (1u << (bit & 31)) : 0u;
        }
        uint32_t add[8];
        const uint32_t up = (kind == 3 || kind == 5) ? 0xFFFFFFFFu : 0u;
        add[0] = kind == 4 ? 1u : up;
#pragma unroll
        for (int j = 1; j < 8; ++j) add[j] = up;
        add256(out, add, out);
    } else if (cls >= g->pct_boundary && pool_n > 0) {
        const uint32_t e = mulhi32(lo, pool_n);
        const uint32_t delta = mulhi32(lo * 0x85EBCA6Bu, 3u);
        // pool expanded to (v - 1, v, v + 1) triples at load (mg_api.cpp)
        cu32* p = consts + (size_t)g->pool_off_b / 4 + (size_t)(e * 3 + delta) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) out[j] = p[j];
    } else {                    // uniform (also the pool class without a pool)
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
            const uint64_t r = sm64(s);
            out[j] = (uint32_t)r;
            out[j + 1] = (uint32_t)(r >> 32);
        }
    }
    mask_to(out, w);
}

// ---------------------------------------------------------------------------
// the interpreter
// ---------------------------------------------------------------------------

#define BLOCK 256

#define READ_SLOT(dst, idx)                                                    \
    do {                                                                       \
        dst[0] = F0[idx]; dst[1] = F1[idx]; dst[2] = F2[idx]; dst[3] = F3[idx];  \
        dst[4] = F4[idx]; dst[5] = F5[idx]; dst[6] = F6[idx]; dst[7] = F7[idx];  \
    } while (0)

#ifndef MG_WAVES_PER_SIMD
#define MG_WAVES_PER_SIMD 2
#endif

template <int GEN>
__global__ __launch_bounds__(BLOCK, MG_WAVES_PER_SIMD) void mg_interp(const mg_pdesc* __restrict__ descs,
                                                      mg_run run) {
    extern __shared__ uint4 lds[];
    const uint32_t prog = blockIdx.y;
    if (run.skip_solved && run.first_sat[prog] < run.first_index) return;
    const __attribute__((address_space(4))) mg_pdesc* D =
        (const __attribute__((address_space(4))) mg_pdesc*)(descs + prog);
    cu32* code = (cu32*)D->code;
    cu32* consts = (cu32*)D->consts;
    const uint32_t n_ins = D->n_ins;
    const uint32_t tid = threadIdx.x;
    const uint64_t gid = (uint64_t)blockIdx.x * BLOCK + tid;
    const bool active = gid < run.n_assign;
    const uint64_t lane_idx = active ? gid : 0;   // inactive lanes replay lane 0

    vfile F0, F1, F2, F3, F4, F5, F6, F7;
#pragma unroll
    for (int i = 0; i < MG_NREG; ++i) {
        F0[i] = 0; F1[i] = 0; F2[i] = 0; F3[i] = 0;
        F4[i] = 0; F5[i] = 0; F6[i] = 0; F7[i] = 0;
    }
    uint32_t root = 1;
    const uint32_t n_lds = D->n_lds;
    uint4 pspill[2 * MG_MAX_PSLOTS];   // per-lane scratch tier (uniform index)

    // software-pipelined fetch: the next instruction's scalar loads are in
    // flight while the current one executes (the host pads code with a NOP)
    // Instruction fetch: the next instruction's s_load is issued before the
    // current one executes and waited for only at the end of the iteration
    // (left to itself the compiler sinks the load to the back-edge and
    // exposes the scalar-cache latency on every instruction).
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t* ip = (const uint32_t*)code;
    u32x4 cur;
    asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)"
                 : "=s"(cur) : "s"(ip) : "memory");
    for (uint32_t pc = 0; pc < n_ins; ++pc) {
        u32x4 nxt;
        asm volatile("s_load_dwordx4 %0, %1, 0x10" : "=s"(nxt) : "s"(ip) : "memory");
        const uint32_t w0 = cur.x, w1 = cur.y, imm0 = cur.z;
        const uint32_t op = w0 & 0xFF;
        const uint32_t w = (w0 >> 8) & 0x3FF;
        // slot fields are < MG_NREG (validated on upload)
        const uint32_t sd = w1 & 31, sa = (w1 >> 8) & 31, sb = (w1 >> 16) & 31, sc = (w1 >> 24) & 31;

        // operands are read inside the cases that need them (GPR-index moves)
        uint32_t x[8], y[8], r[8];
#define RX READ_SLOT(x, sa)
#define RY READ_SLOT(y, sb)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = 0;

        switch (op) {
        case MG_CONST: {
            cu32* p = consts + (size_t)imm0 * 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = p[j];
            __builtin_amdgcn_s_waitcnt(0xC07F);       // lgkmcnt(0)
            break;
        }
        case MG_LEAF: {
            if (GEN) {
                gen_leaf(run.seed, imm0, run.first_index + lane_idx, (cgen*)D->gen + imm0,
                         consts, r);
                if (run.leaves_out && active) {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        run.leaves_out[((size_t)imm0 * 8 + j) * run.stride + gid] = r[j];
                }
            } else {
                const uint32_t* p = run.leaves + (size_t)imm0 * 8 * run.stride + lane_idx;
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = p[(size_t)j * run.stride];
                __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
                mask_to(r, w);
            }
            break;
        }
        case MG_SPILL: {
            RX;
            const uint4 a = make_uint4(x[0], x[1], x[2], x[3]);
            const uint4 b = make_uint4(x[4], x[5], x[6], x[7]);
            if (imm0 < n_lds) {
                uint4* s = lds + ((size_t)imm0 * 2) * BLOCK + tid;
                s[0] = a;
                s[BLOCK] = b;
            } else {
                const uint32_t k = 2 * (imm0 - n_lds);
                pspill[k] = a;
                pspill[k + 1] = b;
            }
            break;
        }
        case MG_RELOAD: {
            uint4 a, b;
            if (imm0 < n_lds) {
                const uint4* s = lds + ((size_t)imm0 * 2) * BLOCK + tid;
                a = s[0];
                b = s[BLOCK];
            } else {
                const uint32_t k = 2 * (imm0 - n_lds);
                a = pspill[k];
                b = pspill[k + 1];
            }
            r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
            r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
            __builtin_amdgcn_s_waitcnt(0);            // LDS / scratch results in
            break;
        }
        case MG_ADD: RX; RY; add256(x, y, r); mask_to(r, w); break;
        case MG_SUB: RX; RY; (void)sub256(x, y, r); mask_to(r, w); break;
        case MG_NEG: RX; neg256(x, r); mask_to(r, w); break;
        case MG_MUL: RX; RY; mul256(x, y, r); mask_to(r, w); break;
        case MG_AND:
            RX; RY;
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = x[j] & y[j];
            break;
        case MG_OR:
            RX; RY;
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = x[j] | y[j];
            break;
        case MG_XOR:
            RX; RY;
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = x[j] ^ y[j];
            break;
        case MG_NOT:
            RX;
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = ~x[j];
            mask_to(r, w);
            break;
        case MG_UDIV:
        case MG_UREM: {
            RX; RY;
            const uint32_t z = is_zero256(y);
            y[0] |= z;                               // divisor 0 -> 1 (fixed below)
            uint32_t q[8], m[8];
            udivrem256(x, y, q, m);
            // with the divisor forced to 1, q == x: x need not stay live
            if (op == MG_UDIV) {
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = z ? 0xFFFFFFFFu : q[j];
                mask_to(r, w);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = z ? q[j] : m[j];
            }
            break;
        }
        case MG_SDIV:
        case MG_SREM:
        case MG_SMOD: {
            RX; RY;
            sext_from(x, w);
            sext_from(y, w);
            const uint32_t ns = sign256(x), nt = sign256(y);
            uint32_t as[8], at[8], tmp[8];
            neg256(x, tmp);
#pragma unroll
            for (int j = 0; j < 8; ++j) as[j] = ns ? tmp[j] : x[j];
            neg256(y, tmp);
#pragma unroll
            for (int j = 0; j < 8; ++j) at[j] = nt ? tmp[j] : y[j];
            const uint32_t z = is_zero256(at);
            at[0] |= z;
            uint32_t q[8], m[8];
            udivrem256(as, at, q, m);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                m[j] = z ? q[j] : m[j];         // |t| forced to 1: q == |s|
                q[j] = z ? 0xFFFFFFFFu : q[j];
            }
            if (op == MG_SDIV) {
                neg256(q, tmp);
                const bool flip = ns != nt;
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = flip ? tmp[j] : q[j];
            } else if (op == MG_SREM) {
                neg256(m, tmp);
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = ns ? tmp[j] : m[j];
            } else {
                // bvsmod: u == 0 -> 0; (+,+) u; (-,+) t-u; (+,-) u+t; (-,-) -u
                RY;                     // t again (not kept live across the division)
                sext_from(y, w);
                const uint32_t uz = is_zero256(m);
                uint32_t nu[8], s1[8], s2[8];
                neg256(m, nu);
                add256(nu, y, s1);      // -u + t
                add256(m, y, s2);       //  u + t
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    uint32_t v = (!ns && !nt) ? m[j] : (ns && !nt) ? s1[j] : (!ns && nt) ? s2[j] : nu[j];
                    r[j] = uz ? 0u : v;
                }
            }
            mask_to(r, w);
            break;
        }
        case MG_SHL:
        case MG_LSHR:
        case MG_ASHR: {
            RX; RY;
            uint32_t hi = y[1] | y[2] | y[3] | y[4] | y[5] | y[6] | y[7];
            const bool over = hi != 0 || y[0] >= w;
            const uint32_t s = y[0] & 255u;
            if (op == MG_SHL) {
                shl_n<8>(x, s, r);
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = over ? 0u : r[j];
                mask_to(r, w);
            } else if (op == MG_LSHR) {
                shr_n<8, 8>(x, s, r);
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = over ? 0u : r[j];
            } else {
                sext_from(x, w);
                const uint32_t sm = 0u - sign256(x);
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] ^= sm;
                shr_n<8, 8>(x, s, r);
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = over ? sm : (r[j] ^ sm);
                mask_to(r, w);
            }
            break;
        }
        case MG_EQ: {
            RX; RY;
            uint32_t o = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) o |= x[j] ^ y[j];
            r[0] = o == 0;
            break;
        }
        case MG_ULT: RX; RY; r[0] = ult256(x, y); break;
        case MG_ULE: RX; RY; r[0] = 1u - ult256(y, x); break;
        case MG_SLT:
        case MG_SLE: {
            RX; RY;
            sext_from(x, w);
            sext_from(y, w);
            x[7] ^= 0x80000000u;
            y[7] ^= 0x80000000u;
            r[0] = op == MG_SLT ? ult256(x, y) : 1u - ult256(y, x);
            break;
        }
        case MG_UMULNO: {
            RX; RY;
            uint32_t p[16];
            mul512(x, y, p);
            uint32_t o = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) o |= p[j] & ~limb_mask(w, j);
            r[0] = o == 0;
            break;
        }
        case MG_ITE: {
            RX; RY;
            const uint32_t cflag = F0[sc] & 1u;
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = cflag ? x[j] : y[j];
            break;
        }
        case MG_CONCAT: {
            RX; RY;
            uint32_t t[8];
            shl_n<8>(x, imm0, t);
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = t[j] | y[j];
            mask_to(r, w);
            break;
        }
        case MG_EXTRACT:
            RX;
            shr_n<8, 8>(x, imm0, r);
            mask_to(r, w);
            break;
        case MG_SEXT:
            RX;
            sext_from(x, imm0);
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = x[j];
            mask_to(r, w);
            break;
        case MG_OUT:
            RX;
            if (run.probes && active) {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    run.probes[((size_t)imm0 * 8 + j) * run.stride + gid] = x[j];
            }
            break;
        case MG_ROOT: root &= F0[sa] & 1u; break;
        case MG_MOV:
            RX;
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = x[j];
            break;
        default: break;
        }
#undef RX
#undef RY
        // fused ROOT: the result of this instruction is a conjunct of the root
        root &= r[0] | ((w0 & MG_ROOT_FLAG) ? 0u : 1u);   // Bool results are 0/1

        // single write point: F[sd] = r  (gpr_idx(DST) moves, no file copies)
        F0[sd] = r[0]; F1[sd] = r[1]; F2[sd] = r[2]; F3[sd] = r[3];
        F4[sd] = r[4]; F5[sd] = r[5]; F6[sd] = r[6]; F7[sd] = r[7];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        cur = nxt;
        ip += 4;
    }

    const unsigned long long bits = __ballot(active && root);
    const uint32_t lane = tid & 63;
    const uint64_t wave_base = gid - lane;
    if (lane == 0 && wave_base < run.n_assign) {
        if (run.root_bits) run.root_bits[prog * run.words_per_prog + (wave_base >> 6)] = bits;
        if (run.first_sat && bits) {
            const unsigned long long first = run.first_index + wave_base + __builtin_ctzll(bits);
            atomicMin(run.first_sat + prog, first);
        }
    }
}

// ---------------------------------------------------------------------------
// launch wrappers (C++ linkage, used by mg_api.cpp)
// ---------------------------------------------------------------------------

hipError_t mg_launch_interp(int gen, const mg_pdesc* d_descs, uint32_t n_progs, const mg_run& run,
                            uint32_t lds_slots, hipStream_t stream) {
    const uint64_t blocks = (run.n_assign + BLOCK - 1) / BLOCK;
    if (blocks == 0 || n_progs == 0) return hipSuccess;
    if (blocks > 0x7FFFFFFFull || n_progs > 65535) return hipErrorInvalidValue;
    dim3 grid((uint32_t)blocks, n_progs);
    const size_t lds_bytes = (size_t)lds_slots * 2 * BLOCK * sizeof(uint4);
    if (gen)
        hipLaunchKernelGGL(mg_interp<1>, grid, dim3(BLOCK), lds_bytes, stream, d_descs, run);
    else
        hipLaunchKernelGGL(mg_interp<0>, grid, dim3(BLOCK), lds_bytes, stream, d_descs, run);
    return hipGetLastError();
}
