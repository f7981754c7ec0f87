/*
 * ORACLE — test infrastructure and CPU baseline only (never linked into the
 * product library).
 *
 * C restatement of z3's evaluation of a get_model constraint DAG under a
 * candidate model (the reference's path: mythril/support/model.py:15-49 →
 * z3.Optimize.check / Model.eval; SMT-LIB 2.6 FixedSizeBitVectors with
 * hi_div0, as restated in oracle/smtlib_ref.py, which pins this file in
 * tests/test_evalref.py).  It evaluates the SOURCE DAG (not the GPU IR):
 * values are 512-bit (8 x u64 limbs; the _wide build, -DL=16, 1024-bit for
 * DAGs with wider nodes: keccak inputs of three words), division is Knuth D on 64-bit digits
 * with __int128 estimates, arrays are resolved by walking store chains,
 * free arrays / UFs by first-match table lookup.  Assignments are either
 * given (SoA leaf values) or rebuilt with the same SplitMix64 candidate
 * generator the device uses (oracle/gen_ref.py).
 *
 * Parallelism: OpenMP over assignments.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef L
#define L 8                      /* 8 x 64 = 512 bits (-DL=16: the wide build) */
#endif
typedef struct { uint64_t w[L]; } V;

enum {
    E_NUM = 1, E_VAR, E_TRUE, E_FALSE, E_ADD, E_SUB, E_MUL, E_UDIV, E_UREM, E_SDIV, E_SREM,
    E_SMOD, E_AND, E_OR, E_XOR, E_NOT, E_NEG, E_SHL, E_LSHR, E_ASHR, E_CONCAT, E_EXTRACT,
    E_ZEXT, E_SEXT, E_EQ, E_ULT, E_ULE, E_SLT, E_SLE, E_UMULNO, E_ITE, E_BAND, E_BOR,
    E_BXOR, E_BNOT, E_SELECT, E_STORE, E_KARR, E_ARRVAR, E_APPLY
};

/* node record: op, width, a0, a1, a2, p0, p1, unused */
#define NW 8

typedef struct {
    uint32_t key_w, val_w, entries;
    const uint32_t* key_leaf;   /* [entries] leaf index of chunk 0 of key  */
    const uint32_t* val_leaf;   /* [entries]                               */
    uint32_t else_leaf;
    /* constant-keyed entries, matched first (ir.scan_const_keys) */
    uint32_t n_ckeys;
    const uint32_t* ckey;       /* [n_ckeys] const index of the key        */
    const uint32_t* cval_leaf;  /* [n_ckeys] leaf index of chunk 0 of value */
} table_t;

static void vzero(V* a) { memset(a, 0, sizeof *a); }

static void vmask(V* a, uint32_t w) {
    for (int i = 0; i < L; ++i) {
        int lo = 64 * i;
        if ((int)w >= lo + 64) continue;
        if ((int)w <= lo) a->w[i] = 0;
        else a->w[i] &= (~0ull) >> (64 - (w - lo));
    }
}

static int vbit(const V* a, uint32_t b) { return (int)((a->w[b / 64] >> (b % 64)) & 1); }

static int vcmp(const V* a, const V* b) {
    for (int i = L - 1; i >= 0; --i) {
        if (a->w[i] != b->w[i]) return a->w[i] < b->w[i] ? -1 : 1;
    }
    return 0;
}

static int viszero(const V* a) {
    uint64_t o = 0;
    for (int i = 0; i < L; ++i) o |= a->w[i];
    return o == 0;
}

static void vadd(const V* a, const V* b, V* r) {
    unsigned __int128 c = 0;
    for (int i = 0; i < L; ++i) {
        c += (unsigned __int128)a->w[i] + b->w[i];
        r->w[i] = (uint64_t)c;
        c >>= 64;
    }
}

static void vsub(const V* a, const V* b, V* r) {
    uint64_t br = 0;
    for (int i = 0; i < L; ++i) {
        unsigned __int128 t = (unsigned __int128)a->w[i] - b->w[i] - br;
        r->w[i] = (uint64_t)t;
        br = (uint64_t)(t >> 64) & 1;
    }
}

static void vneg(const V* a, V* r) {
    V z;
    vzero(&z);
    vsub(&z, a, r);
}

static void vmul(const V* a, const V* b, V* r) {   /* low L * 64 bits */
    uint64_t t[L] = {0};
    for (int i = 0; i < L; ++i) {
        unsigned __int128 c = 0;
        for (int j = 0; i + j < L; ++j) {
            c += (unsigned __int128)a->w[i] * b->w[j] + t[i + j];
            t[i + j] = (uint64_t)c;
            c >>= 64;
        }
    }
    memcpy(r->w, t, sizeof t);
}

static void vshl(const V* a, uint32_t s, V* r) {
    V t;
    vzero(&t);
    uint32_t q = s / 64, b = s % 64;
    for (int i = L - 1; i >= (int)q; --i) {
        uint64_t v = a->w[i - q] << b;
        if (b && i - (int)q - 1 >= 0) v |= a->w[i - q - 1] >> (64 - b);
        t.w[i] = v;
    }
    *r = t;
}

static void vlshr(const V* a, uint32_t s, V* r) {
    V t;
    vzero(&t);
    uint32_t q = s / 64, b = s % 64;
    for (int i = 0; i + (int)q < L; ++i) {
        uint64_t v = a->w[i + q] >> b;
        if (b && i + q + 1 < L) v |= a->w[i + q + 1] << (64 - b);
        t.w[i] = v;
    }
    *r = t;
}

/* Knuth algorithm D on 64-bit digits (Hacker's Delight divmnu), with
 * __int128 for the 128/64 digit estimate; data-dependent loop bounds. */
static void vdivmod(const V* u, const V* v, V* q, V* rem) {
    int n = L, m = L;
    while (n > 0 && v->w[n - 1] == 0) --n;
    while (m > 0 && u->w[m - 1] == 0) --m;
    vzero(q);
    if (m < n || vcmp(u, v) < 0) {
        *rem = *u;
        return;
    }
    if (n == 1) {
        unsigned __int128 r = 0;
        for (int j = m - 1; j >= 0; --j) {
            unsigned __int128 num = (r << 64) | u->w[j];
            q->w[j] = (uint64_t)(num / v->w[0]);
            r = num % v->w[0];
        }
        vzero(rem);
        rem->w[0] = (uint64_t)r;
        return;
    }
    const int s = __builtin_clzll(v->w[n - 1]);
    uint64_t vn[L], un[L + 1];
    for (int i = n - 1; i > 0; --i)
        vn[i] = (v->w[i] << s) | (s ? v->w[i - 1] >> (64 - s) : 0);
    vn[0] = v->w[0] << s;
    un[m] = s ? u->w[m - 1] >> (64 - s) : 0;
    for (int i = m - 1; i > 0; --i)
        un[i] = (u->w[i] << s) | (s ? u->w[i - 1] >> (64 - s) : 0);
    un[0] = u->w[0] << s;
    const unsigned __int128 B = (unsigned __int128)1 << 64;
    for (int j = m - n; j >= 0; --j) {
        unsigned __int128 num = ((unsigned __int128)un[j + n] << 64) | un[j + n - 1];
        unsigned __int128 qhat = num / vn[n - 1];
        unsigned __int128 rhat = num % vn[n - 1];
        while (qhat >= B ||
               qhat * vn[n - 2] > ((rhat << 64) | un[j + n - 2])) {
            qhat -= 1;
            rhat += vn[n - 1];
            if (rhat >= B) break;
        }
        __int128 t, k = 0;
        for (int i = 0; i < n; ++i) {
            unsigned __int128 p = qhat * vn[i];
            t = (__int128)un[i + j] - k - (__int128)(uint64_t)p;
            un[i + j] = (uint64_t)t;
            k = (__int128)(p >> 64) - (t >> 64);
        }
        t = (__int128)un[j + n] - k;
        un[j + n] = (uint64_t)t;
        q->w[j] = (uint64_t)qhat;
        if (t < 0) {
            q->w[j] -= 1;
            unsigned __int128 c = 0;
            for (int i = 0; i < n; ++i) {
                c += (unsigned __int128)un[i + j] + vn[i];
                un[i + j] = (uint64_t)c;
                c >>= 64;
            }
            un[j + n] += (uint64_t)c;
        }
    }
    vzero(rem);
    for (int i = 0; i < n; ++i)
        rem->w[i] = (un[i] >> s) | (s ? un[i + 1] << (64 - s) : 0);
}

static void vudiv(const V* a, const V* b, uint32_t w, V* r) {
    if (viszero(b)) {
        for (int i = 0; i < L; ++i) r->w[i] = ~0ull;
        vmask(r, w);
        return;
    }
    V m;
    vdivmod(a, b, r, &m);
}

static void vurem(const V* a, const V* b, V* r) {
    if (viszero(b)) {
        *r = *a;
        return;
    }
    V q;
    vdivmod(a, b, &q, r);
}

static void vnegw(const V* a, uint32_t w, V* r) {
    vneg(a, r);
    vmask(r, w);
}

static void vsdiv(const V* s, const V* t, uint32_t w, V* r) {
    int ms = vbit(s, w - 1), mt = vbit(t, w - 1);
    V as = *s, at = *t, x;
    if (ms) vnegw(s, w, &as);
    if (mt) vnegw(t, w, &at);
    vudiv(&as, &at, w, &x);
    if (ms != mt) vnegw(&x, w, r);
    else *r = x;
}

static void vsrem(const V* s, const V* t, uint32_t w, V* r) {
    int ms = vbit(s, w - 1), mt = vbit(t, w - 1);
    V as = *s, at = *t, x;
    if (ms) vnegw(s, w, &as);
    if (mt) vnegw(t, w, &at);
    vurem(&as, &at, &x);
    if (ms) vnegw(&x, w, r);
    else *r = x;
}

static void vsmod(const V* s, const V* t, uint32_t w, V* r) {
    int ms = vbit(s, w - 1), mt = vbit(t, w - 1);
    V as = *s, at = *t, u, x;
    if (ms) vnegw(s, w, &as);
    if (mt) vnegw(t, w, &at);
    vurem(&as, &at, &u);
    if (viszero(&u) || (!ms && !mt)) {
        *r = u;
        return;
    }
    if (ms && !mt) {
        vnegw(&u, w, &x);
        vadd(&x, t, r);
    } else if (!ms && mt) {
        vadd(&u, t, r);
    } else {
        vneg(&u, r);
    }
    vmask(r, w);
}

static int vslt(const V* a, const V* b, uint32_t w) {
    int sa = vbit(a, w - 1), sb = vbit(b, w - 1);
    if (sa != sb) return sa > sb;
    return vcmp(a, b) < 0;
}

static void vsext(const V* a, uint32_t from, uint32_t to, V* r) {
    *r = *a;
    if (vbit(a, from - 1)) {
        for (uint32_t b = from; b < to; ++b) r->w[b / 64] |= 1ull << (b % 64);
    }
}

static uint32_t shift_amount(const V* b, uint32_t w, int* over) {
    int hi = 0;
    for (int i = 1; i < L; ++i) hi |= b->w[i] != 0;
    *over = hi || b->w[0] >= w;
    return *over ? 0 : (uint32_t)b->w[0];
}

typedef struct {
    const uint32_t* nodes;
    uint32_t n_nodes;
    const uint64_t* consts;   /* [n][8] */
    const table_t* tables;
    uint32_t n_tables;
} dag_t;

static void leaf_value(const V* leaves, uint32_t idx, uint32_t width, V* out) {
    /* a leaf value wider than 256 bits is split in 256-bit chunk leaves */
    vzero(out);
    uint32_t chunks = (width + 255) / 256;
    for (uint32_t k = 0; k < chunks; ++k)
        for (int i = 0; i < 4; ++i) out->w[4 * k + i] = leaves[idx + k].w[i];
    vmask(out, width);
}

static void table_lookup(const dag_t* g, const V* leaves, uint32_t t, const V* key, V* out) {
    const table_t* T = &g->tables[t];
    for (uint32_t e = 0; e < T->n_ckeys; ++e) {
        V k;
        memcpy(k.w, g->consts + (size_t)T->ckey[e] * L, sizeof k.w);
        if (vcmp(&k, key) == 0) {
            leaf_value(leaves, T->cval_leaf[e], T->val_w, out);
            return;
        }
    }
    for (uint32_t e = 0; e < T->entries; ++e) {
        V k;
        leaf_value(leaves, T->key_leaf[e], T->key_w, &k);
        if (vcmp(&k, key) == 0) {
            leaf_value(leaves, T->val_leaf[e], T->val_w, out);
            return;
        }
    }
    leaf_value(leaves, T->else_leaf, T->val_w, out);
}

static void select_arr(const dag_t* g, const V* vals, const V* leaves, uint32_t arr,
                       const V* idx, V* out) {
    for (;;) {
        const uint32_t* n = g->nodes + (size_t)arr * NW;
        switch (n[0]) {
        case E_STORE:
            if (vcmp(&vals[n[3]], idx) == 0) {
                *out = vals[n[4]];
                return;
            }
            arr = n[2];
            break;
        case E_KARR:
            *out = vals[n[2]];
            return;
        case E_ARRVAR:
            table_lookup(g, leaves, n[5], idx, out);
            return;
        case E_ITE:
            arr = vals[n[2]].w[0] ? n[3] : n[4];
            break;
        default:
            vzero(out);
            return;
        }
    }
}

static void eval_dag(const dag_t* g, const V* leaves, V* vals) {
    for (uint32_t i = 0; i < g->n_nodes; ++i) {
        const uint32_t* n = g->nodes + (size_t)i * NW;
        const uint32_t op = n[0], w = n[1];
        const V* a = &vals[n[2]];
        const V* b = &vals[n[3]];
        const V* c = &vals[n[4]];
        V r;
        vzero(&r);
        int over;
        switch (op) {
        case E_NUM: memcpy(r.w, g->consts + (size_t)n[5] * L, sizeof r.w); break;
        case E_VAR: leaf_value(leaves, n[5], w, &r); break;
        case E_TRUE: r.w[0] = 1; break;
        case E_FALSE: break;
        case E_ADD: vadd(a, b, &r); vmask(&r, w); break;
        case E_SUB: vsub(a, b, &r); vmask(&r, w); break;
        case E_MUL: vmul(a, b, &r); vmask(&r, w); break;
        case E_UDIV: vudiv(a, b, w, &r); break;
        case E_UREM: vurem(a, b, &r); break;
        case E_SDIV: vsdiv(a, b, w, &r); break;
        case E_SREM: vsrem(a, b, w, &r); break;
        case E_SMOD: vsmod(a, b, w, &r); break;
        case E_AND: case E_BAND: for (int k = 0; k < L; ++k) r.w[k] = a->w[k] & b->w[k]; break;
        case E_OR: case E_BOR: for (int k = 0; k < L; ++k) r.w[k] = a->w[k] | b->w[k]; break;
        case E_XOR: case E_BXOR: for (int k = 0; k < L; ++k) r.w[k] = a->w[k] ^ b->w[k]; break;
        case E_NOT: case E_BNOT: for (int k = 0; k < L; ++k) r.w[k] = ~a->w[k]; vmask(&r, w); break;
        case E_NEG: vneg(a, &r); vmask(&r, w); break;
        case E_SHL: {
            uint32_t s = shift_amount(b, w, &over);
            if (!over) { vshl(a, s, &r); vmask(&r, w); }
            break;
        }
        case E_LSHR: {
            uint32_t s = shift_amount(b, w, &over);
            if (!over) vlshr(a, s, &r);
            break;
        }
        case E_ASHR: {
            uint32_t s = shift_amount(b, w, &over);
            V t;
            vsext(a, w, L * 64, &t);
            if (over) {
                if (vbit(a, w - 1)) for (int k = 0; k < L; ++k) r.w[k] = ~0ull;
            } else {
                int neg = vbit(a, w - 1);
                vlshr(&t, s, &r);
                if (neg) for (uint32_t q = L * 64 - s; q < L * 64; ++q) r.w[q / 64] |= 1ull << (q % 64);
            }
            vmask(&r, w);
            break;
        }
        case E_CONCAT: vshl(a, n[5], &r); for (int k = 0; k < L; ++k) r.w[k] |= b->w[k]; break;
        case E_EXTRACT: vlshr(a, n[6], &r); vmask(&r, w); break;
        case E_ZEXT: r = *a; break;
        case E_SEXT: vsext(a, w - n[5], w, &r); break;
        case E_EQ: r.w[0] = vcmp(a, b) == 0; break;
        case E_ULT: r.w[0] = vcmp(a, b) < 0; break;
        case E_ULE: r.w[0] = vcmp(a, b) <= 0; break;
        case E_SLT: r.w[0] = vslt(a, b, n[5]); break;
        case E_SLE: r.w[0] = !vslt(b, a, n[5]); break;
        case E_UMULNO: {
            /* a, b < 2^w with w <= 256, so the full product fits L * 64 bits */
            V p;
            vmul(a, b, &p);
            V m = p;
            vlshr(&p, n[5], &m);
            r.w[0] = viszero(&m);
            break;
        }
        case E_ITE: r = a->w[0] ? *b : *c; break;
        case E_SELECT: select_arr(g, vals, leaves, n[2], b, &r); break;
        case E_APPLY: table_lookup(g, leaves, n[5], a, &r); break;
        case E_STORE: case E_KARR: case E_ARRVAR: break;   /* resolved by select */
        default: break;
        }
        vals[i] = r;
    }
}

/* ---- device candidate generator (port of gen_leaf / oracle/gen_ref.py) ---- */

static uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

/* v9 mixer: s += GOLD; z = (s ^ (s >> 32)) * MIX1; r0 = z ^ (z >> 32) */
static uint64_t sm64(uint64_t* s) {
    *s += 0x9E3779B97F4A7C15ull;
    uint64_t z = (*s ^ (*s >> 32)) * 0xBF58476D1CE4E5B9ull;
    return z ^ (z >> 32);
}

static void gen_leaf(uint64_t seed, uint64_t prog_seed, uint32_t leaf, uint64_t idx, uint32_t w,
                     const uint64_t* pool, uint32_t pool_n, const uint32_t pct[3], V* out) {
    const uint64_t ss = seed ^ (prog_seed * 0xD1B54A32D192ED03ull) ^
                        ((uint64_t)(leaf + 1) * 0x8CB92BA72F3D8DD7ull);
    uint64_t s = ss ^ idx;                                                /* v5 */
    uint64_t r0 = sm64(&s);
    /* v2 range reduction: multiply-high (Lemire) instead of modulo; v8: the
     * class once per group of 64 candidate indices (idx >> 6) */
    const uint32_t y = (((uint32_t)(idx >> 6) ^ (uint32_t)ss) * 0x2545F491u) ^ (uint32_t)(ss >> 32);
    uint32_t cls = mulhi32(y, 100u), lo = (uint32_t)r0;
    vzero(out);
    if (cls >= pct[0] && cls < pct[1]) {
        out->w[0] = r0;                       /* v3: the class word itself */
    } else if (cls >= pct[1] && cls < pct[2]) {
        uint32_t kind = mulhi32(lo, 6u), k = mulhi32(lo * 0x9E3779B1u, w);
        if (kind == 1) out->w[0] = 1;
        if (kind == 2) out->w[(w - 1) / 64] = 1ull << ((w - 1) % 64);
        if (kind == 3) for (int i = 0; i < 4; ++i) out->w[i] = ~0ull;
        if (kind == 4 || kind == 5) {
            V one, p;
            vzero(&one);
            one.w[0] = 1;
            vzero(&p);
            p.w[k / 64] = 1ull << (k % 64);
            if (kind == 4) vadd(&p, &one, out);
            else vsub(&p, &one, out);
        }
    } else if (cls >= pct[2] && pool_n > 0) {
        uint32_t e = mulhi32(lo, pool_n), delta = mulhi32(lo * 0x85EBCA6Bu, 3u);
        V one, p;
        vzero(&one);
        one.w[0] = 1;
        vzero(&p);
        memcpy(p.w, pool + (size_t)e * L, 4 * sizeof(uint64_t));   /* entries are L words */
        if (delta == 0) vsub(&p, &one, out);
        else if (delta == 2) vadd(&p, &one, out);
        else *out = p;
        for (int i = 4; i < L; ++i) out->w[i] = 0;
    } else {
        /* v6: r0, limb pair k = x * C_k + r0 with x = lo ^ hi of r0 */
        static const uint64_t pair_mul[3] = {0x85EBCA6Bull, 0xC2B2AE35ull, 0x27D4EB2Full};
        uint64_t x = (uint32_t)r0 ^ (uint32_t)(r0 >> 32);
        out->w[0] = r0;
        for (int k = 0; k < 3; ++k) out->w[k + 1] = x * pair_mul[k] + r0;
    }
    vmask(out, w);
}

/* ---- entry points (ctypes) ---- */

typedef struct {
    uint32_t key_w, val_w, entries, else_leaf;
    uint32_t key_leaf_off, val_leaf_off;   /* offsets into a shared u32 array */
    uint32_t n_ckeys, ckey_off, cval_leaf_off;
} table_desc;

static void make_tables(const table_desc* td, uint32_t n, const uint32_t* leafidx, table_t* out) {
    for (uint32_t t = 0; t < n; ++t) {
        out[t].key_w = td[t].key_w;
        out[t].val_w = td[t].val_w;
        out[t].entries = td[t].entries;
        out[t].key_leaf = leafidx + td[t].key_leaf_off;
        out[t].val_leaf = leafidx + td[t].val_leaf_off;
        out[t].else_leaf = td[t].else_leaf;
        out[t].n_ckeys = td[t].n_ckeys;
        out[t].ckey = leafidx + td[t].ckey_off;
        out[t].cval_leaf = leafidx + td[t].cval_leaf_off;
    }
}

/* Limbs per value of this build (consts, pool and vals_out use this stride). */
int ev_limbs(void) { return L; }

/* -2 when a node or table is wider than this build's values (the caller
 * picks the wide build; nothing is evaluated). */
static int too_wide(const uint32_t* nodes, uint32_t n_nodes, const table_desc* td, uint32_t n_tables) {
    for (uint32_t i = 0; i < n_nodes; ++i)
        if (nodes[(size_t)i * NW + 1] > L * 64) return 1;
    for (uint32_t t = 0; t < n_tables; ++t)
        if (td[t].key_w > L * 64 || td[t].val_w > L * 64) return 1;
    return 0;
}

/* Evaluate under generated candidates [first, first + n): root bits. */
int ev_run_gen(const uint32_t* nodes, uint32_t n_nodes, const uint64_t* consts,
               const table_desc* td, uint32_t n_tables, const uint32_t* leafidx,
               const uint32_t* roots, uint32_t n_roots, const uint32_t* leaf_widths,
               uint32_t n_leaves, const uint64_t* pool, uint32_t pool_n, const uint32_t* pct,
               uint64_t seed, uint64_t prog_seed, uint64_t first, uint64_t n,
               uint8_t* root_out, int threads) {
    table_t tabs[64];
    if (n_tables > 64) return -1;
    if (too_wide(nodes, n_nodes, td, n_tables)) return -2;
    make_tables(td, n_tables, leafidx, tabs);
    dag_t g = {nodes, n_nodes, consts, tabs, n_tables};
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
    {
        V* vals = (V*)malloc(sizeof(V) * (n_nodes ? n_nodes : 1));
        V* leaves = (V*)malloc(sizeof(V) * (n_leaves ? n_leaves : 1));
#pragma omp for schedule(dynamic, 64)
        for (int64_t a = 0; a < (int64_t)n; ++a) {
            for (uint32_t l = 0; l < n_leaves; ++l)
                gen_leaf(seed, prog_seed, l, first + (uint64_t)a, leaf_widths[l], pool, pool_n, pct,
                         &leaves[l]);
            eval_dag(&g, leaves, vals);
            uint8_t ok = 1;
            for (uint32_t r = 0; r < n_roots; ++r) ok &= (uint8_t)(vals[roots[r]].w[0] & 1);
            root_out[a] = ok;
        }
        free(vals);
        free(leaves);
    }
    return 0;
}

/* Per-root bits under explicit leaf values: root_out[a * n_roots + r]. */
int ev_run_leaves_roots(const uint32_t* nodes, uint32_t n_nodes, const uint64_t* consts,
                        const table_desc* td, uint32_t n_tables, const uint32_t* leafidx,
                        const uint32_t* roots, uint32_t n_roots, uint32_t n_leaves,
                        const uint64_t* leaves_in, uint64_t n, uint8_t* root_out, int threads) {
    table_t tabs[64];
    if (n_tables > 64) return -1;
    if (too_wide(nodes, n_nodes, td, n_tables)) return -2;
    make_tables(td, n_tables, leafidx, tabs);
    dag_t g = {nodes, n_nodes, consts, tabs, n_tables};
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel
    {
        V* vals = (V*)malloc(sizeof(V) * (n_nodes ? n_nodes : 1));
        V* leaves = (V*)malloc(sizeof(V) * (n_leaves ? n_leaves : 1));
#pragma omp for schedule(dynamic, 64)
        for (int64_t a = 0; a < (int64_t)n; ++a) {
            for (uint32_t l = 0; l < n_leaves; ++l) {
                vzero(&leaves[l]);
                for (int i = 0; i < 4; ++i) leaves[l].w[i] = leaves_in[((uint64_t)a * n_leaves + l) * 4 + i];
            }
            eval_dag(&g, leaves, vals);
            for (uint32_t r = 0; r < n_roots; ++r)
                root_out[(uint64_t)a * n_roots + r] = (uint8_t)(vals[roots[r]].w[0] & 1);
        }
        free(vals);
        free(leaves);
    }
    return 0;
}

/* Evaluate under explicit leaf values: leaves [n_leaves][4 x u64] per
 * assignment (AoS, n of them); writes every node value for assignment 0..n-1
 * into vals_out ([n][n_nodes][8 x u64]) when non-NULL, and root bits. */
int ev_run_leaves(const uint32_t* nodes, uint32_t n_nodes, const uint64_t* consts,
                  const table_desc* td, uint32_t n_tables, const uint32_t* leafidx,
                  const uint32_t* roots, uint32_t n_roots, uint32_t n_leaves,
                  const uint64_t* leaves_in, uint64_t n, uint64_t* vals_out, uint8_t* root_out) {
    table_t tabs[64];
    if (n_tables > 64) return -1;
    if (too_wide(nodes, n_nodes, td, n_tables)) return -2;
    make_tables(td, n_tables, leafidx, tabs);
    dag_t g = {nodes, n_nodes, consts, tabs, n_tables};
    V* vals = (V*)malloc(sizeof(V) * (n_nodes ? n_nodes : 1));
    V* leaves = (V*)malloc(sizeof(V) * (n_leaves ? n_leaves : 1));
    for (uint64_t a = 0; a < n; ++a) {
        for (uint32_t l = 0; l < n_leaves; ++l) {
            vzero(&leaves[l]);
            for (int i = 0; i < 4; ++i) leaves[l].w[i] = leaves_in[(a * n_leaves + l) * 4 + i];
        }
        eval_dag(&g, leaves, vals);
        uint8_t ok = 1;
        for (uint32_t r = 0; r < n_roots; ++r) ok &= (uint8_t)(vals[roots[r]].w[0] & 1);
        root_out[a] = ok;
        if (vals_out) memcpy(vals_out + a * n_nodes * L, vals, sizeof(V) * n_nodes);
    }
    free(vals);
    free(leaves);
    return 0;
}
