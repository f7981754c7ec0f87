// mythcc — native host compiler (include/mythcc.h).
//
// Constraint DAG -> mythgpu IR, the same pipeline as mythril_amd/ir.py
// compile_constraints and mythril_amd/solve.py Solver, pass for pass and in
// the same creation order (node ids order the schedule, so the emitted
// program is identical — tests/test_native_compiler.py holds the two
// together on every test corpus).  Each section names the Python function
// it mirrors; the design notes live there and in DESIGN.md §3.1/§3.4.
//
// The path it serves is the reference's get_model (mythril/support/
// model.py:15-49): one compile per independent constraint group the GPU
// pre-filter searches.  Python is ~30 ms per cold C3/C4 query; this is
// well under a millisecond, so the drop-in's miss latency is the search.

#include "mythcc.h"
#include "mythgpu_ir.h"

#include <algorithm>
#include <memory>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <chrono>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <tuple>
#include <utility>
#include <vector>

namespace {

// ---------------------------------------------------------------------------
// fixed-width integers: 384-bit two's complement (every LNode value is <= 256
// bits; intervals and bounds need 257, the ABI offset arithmetic a sign)
// ---------------------------------------------------------------------------
struct U {
    static const int N = 6;
    uint64_t w[N];
    U() { std::memset(w, 0, sizeof w); }
    static U of(uint64_t x) { U r; r.w[0] = x; return r; }
    bool zero() const {
        for (int i = 0; i < N; i++) if (w[i]) return false;
        return true;
    }
    bool neg() const { return w[N - 1] >> 63; }
    int bitlen() const {           // of a non-negative value
        for (int i = N - 1; i >= 0; i--)
            if (w[i]) return 64 * i + 64 - __builtin_clzll(w[i]);
        return 0;
    }
    int popcount() const {
        int c = 0;
        for (int i = 0; i < N; i++) c += __builtin_popcountll(w[i]);
        return c;
    }
    bool bit(int k) const { return k < 64 * N && ((w[k >> 6] >> (k & 63)) & 1); }
};

static U operator+(const U& a, const U& b) {
    U r; unsigned __int128 c = 0;
    for (int i = 0; i < U::N; i++) { c += (unsigned __int128)a.w[i] + b.w[i]; r.w[i] = (uint64_t)c; c >>= 64; }
    return r;
}
static U operator~(const U& a) { U r; for (int i = 0; i < U::N; i++) r.w[i] = ~a.w[i]; return r; }
static U operator-(const U& a, const U& b) { return a + ~b + U::of(1); }
static U operator&(const U& a, const U& b) { U r; for (int i = 0; i < U::N; i++) r.w[i] = a.w[i] & b.w[i]; return r; }
static U operator|(const U& a, const U& b) { U r; for (int i = 0; i < U::N; i++) r.w[i] = a.w[i] | b.w[i]; return r; }
static U operator^(const U& a, const U& b) { U r; for (int i = 0; i < U::N; i++) r.w[i] = a.w[i] ^ b.w[i]; return r; }
static U operator*(const U& a, const U& b) {
    U r;
    for (int i = 0; i < U::N; i++) {
        unsigned __int128 c = 0;
        for (int j = 0; i + j < U::N; j++) {
            c += (unsigned __int128)a.w[i] * b.w[j] + r.w[i + j];
            r.w[i + j] = (uint64_t)c; c >>= 64;
        }
    }
    return r;
}
struct BadShift : std::runtime_error { BadShift() : std::runtime_error("negative shift") {} };
static U shl(const U& a, int k) {
    if (k < 0) throw BadShift();
    U r; if (k >= 64 * U::N) return r;
    int q = k >> 6, s = k & 63;
    for (int i = U::N - 1; i >= q; i--) {
        uint64_t v = a.w[i - q] << s;
        if (s && i - q - 1 >= 0) v |= a.w[i - q - 1] >> (64 - s);
        r.w[i] = v;
    }
    return r;
}
static U shr(const U& a, int k) {      // logical
    if (k < 0) throw BadShift();
    U r; if (k >= 64 * U::N) return r;
    int q = k >> 6, s = k & 63;
    for (int i = 0; i + q < U::N; i++) {
        uint64_t v = a.w[i + q] >> s;
        if (s && i + q + 1 < U::N) v |= a.w[i + q + 1] << (64 - s);
        r.w[i] = v;
    }
    return r;
}
static U sar(const U& a, int k) {      // arithmetic
    if (!a.neg()) return shr(a, k);
    return ~shr(~a, k);
}
static bool operator==(const U& a, const U& b) { return std::memcmp(a.w, b.w, sizeof a.w) == 0; }
static bool operator!=(const U& a, const U& b) { return !(a == b); }
static bool operator<(const U& a, const U& b) {   // unsigned
    for (int i = U::N - 1; i >= 0; i--) if (a.w[i] != b.w[i]) return a.w[i] < b.w[i];
    return false;
}
static bool operator>(const U& a, const U& b) { return b < a; }
static bool operator<=(const U& a, const U& b) { return !(b < a); }
static bool operator>=(const U& a, const U& b) { return !(a < b); }
static U umin(const U& a, const U& b) { return b < a ? b : a; }
static U umax(const U& a, const U& b) { return a < b ? b : a; }
static U mask_slow(int w) { return shl(U::of(1), w) - U::of(1); }
static const U* mask_table() {          // (function-local static: thread-safe)
    static const std::vector<U> t = [] {
        std::vector<U> v(64 * U::N + 1);
        for (int w = 0; w <= 64 * U::N; w++) v[w] = mask_slow(w);
        return v;
    }();
    return t.data();
}
static const U* const MASKS = mask_table();
static inline const U& mask(int w) { return MASKS[w < 0 ? 0 : (w > 64 * U::N ? 64 * U::N : w)]; }
static U U1(int k) { return shl(U::of(1), k); }
static bool nz(const U& a) { return !a.zero(); }

static std::string hex(const U& a) {
    char buf[8];
    std::string s;
    bool started = false;
    for (int i = U::N - 1; i >= 0; i--) {
        for (int nib = 15; nib >= 0; nib--) {
            int d = (a.w[i] >> (4 * nib)) & 15;
            if (!started && !d) continue;
            started = true;
            std::snprintf(buf, sizeof buf, "%x", d);
            s += buf;
        }
    }
    return started ? s : "0";
}

// arbitrary-length non-negative integers for source numerals (a table key
// may be a 512-bit Keccak input): little-endian 32-bit limbs, normalised
struct Big {
    std::vector<uint32_t> l;
    void norm() { while (!l.empty() && !l.back()) l.pop_back(); }
    bool operator==(const Big& o) const { return l == o.l; }
    bool operator<(const Big& o) const {
        if (l.size() != o.l.size()) return l.size() < o.l.size();
        for (size_t i = l.size(); i-- > 0;) if (l[i] != o.l[i]) return l[i] < o.l[i];
        return false;
    }
    // bits [256 k, 256 k + 256) as U
    U chunk(int k) const {
        U r;
        for (int j = 0; j < 8; j++) {
            size_t idx = (size_t)8 * k + j;
            if (idx < l.size()) r.w[j / 2] |= (uint64_t)l[idx] << (32 * (j & 1));
        }
        return r;
    }
    U low384() const {
        U r;
        for (size_t j = 0; j < l.size() && j < 12; j++) r.w[j / 2] |= (uint64_t)l[j] << (32 * (j & 1));
        return r;
    }
    std::string hexs() const {
        if (l.empty()) return "0";
        char buf[16];
        std::string s;
        std::snprintf(buf, sizeof buf, "%x", l.back());
        s += buf;
        for (size_t i = l.size() - 1; i-- > 0;) { std::snprintf(buf, sizeof buf, "%08x", l[i]); s += buf; }
        return s;
    }
};

static Big big_of(const U& u) {
    Big b;
    for (int j = 0; j < 2 * U::N; j++) b.l.push_back((uint32_t)(u.w[j / 2] >> (32 * (j & 1))));
    b.norm();
    return b;
}

// dynamic bit sets (Python int bit sets in ir.py / solve.py)
struct Bits {
    std::vector<uint64_t> w;
    void set(int k) { if ((size_t)(k >> 6) >= w.size()) w.resize((k >> 6) + 1, 0); w[k >> 6] |= 1ull << (k & 63); }
    void orw(const Bits& o) { if (o.w.size() > w.size()) w.resize(o.w.size(), 0); for (size_t i = 0; i < o.w.size(); i++) w[i] |= o.w[i]; }
    bool meets(const Bits& o) const {
        size_t n = std::min(w.size(), o.w.size());
        for (size_t i = 0; i < n; i++) if (w[i] & o.w[i]) return true;
        return false;
    }
    bool any() const { for (auto x : w) if (x) return true; return false; }
    int count() const { int c = 0; for (auto x : w) c += __builtin_popcountll(x); return c; }
    template <class F> void each(F f) const {        // ascending
        for (size_t i = 0; i < w.size(); i++) {
            uint64_t x = w[i];
            while (x) { int b = __builtin_ctzll(x); f((int)(64 * i + b)); x &= x - 1; }
        }
    }
    // (self & ~o) != 0
    bool any_minus(const Bits& o) const {
        for (size_t i = 0; i < w.size(); i++) if (w[i] & ~(i < o.w.size() ? o.w[i] : 0)) return true;
        return false;
    }
    // self & ~o
    Bits minus(const Bits& o) const {
        Bits r; r.w = w;
        for (size_t i = 0; i < r.w.size() && i < o.w.size(); i++) r.w[i] &= ~o.w[i];
        return r;
    }
};

struct Unsupported : std::runtime_error { using std::runtime_error::runtime_error; };
struct MemoMiss {};               // a Python KeyError on the lowering memo

// insertion-ordered map (Python dict semantics where iteration order counts)
template <class K, class V, class H = std::hash<K>>
struct OMap {
    std::vector<std::pair<K, V>> items;
    std::unordered_map<K, size_t, H> idx;
    V* find(const K& k) { auto it = idx.find(k); return it == idx.end() ? nullptr : &items[it->second].second; }
    const V* find(const K& k) const { auto it = idx.find(k); return it == idx.end() ? nullptr : &items[it->second].second; }
    bool has(const K& k) const { return idx.count(k) != 0; }
    V& setdefault(const K& k, const V& d) {
        auto it = idx.find(k);
        if (it != idx.end()) return items[it->second].second;
        idx.emplace(k, items.size());
        items.emplace_back(k, d);
        return items.back().second;
    }
    void put(const K& k, const V& v) { setdefault(k, v) = v; }
    size_t size() const { return items.size(); }
    void truncate(size_t n) {                // drop the entries inserted after the first n
        while (items.size() > n) { idx.erase(items.back().first); items.pop_back(); }
    }
};

// ---------------------------------------------------------------------------
// source DAG
// ---------------------------------------------------------------------------
enum SOp {
    S_BVNUM, S_TRUE, S_FALSE, S_VAR, S_BVSUB, S_BVUDIV, S_BVUREM, S_BVSDIV, S_BVSREM, S_BVSMOD,
    S_BVSHL, S_BVLSHR, S_BVASHR, S_BVADD, S_BVMUL, S_BVAND, S_BVOR, S_BVXOR, S_AND, S_OR,
    S_BVNEG, S_BVNOT, S_NOT, S_XOR, S_IMPLIES, S_BVULT, S_BVULE, S_BVUGT, S_BVUGE, S_BVSLT,
    S_BVSLE, S_BVSGT, S_BVSGE, S_UMULNO, S_EQ, S_DISTINCT, S_ITE, S_CONCAT, S_EXTRACT, S_ZEXT,
    S_SEXT, S_SELECT, S_APPLY, S_STORE, S_K, S_ARRAY, S_OTHER
};
static const char* const SOP_NAMES =
    "bvnum\ntrue\nfalse\nvar\nbvsub\nbvudiv\nbvurem\nbvsdiv\nbvsrem\nbvsmod\n"
    "bvshl\nbvlshr\nbvashr\nbvadd\nbvmul\nbvand\nbvor\nbvxor\nand\nor\n"
    "bvneg\nbvnot\nnot\nxor\n=>\nbvult\nbvule\nbvugt\nbvuge\nbvslt\n"
    "bvsle\nbvsgt\nbvsge\nbvumul_noovfl\n=\ndistinct\nite\nconcat\nextract\nzero_extend\n"
    "sign_extend\nselect\napply\nstore\nK\narray\n?";

struct Src {
    int op, sort, width, dom;
    int64_t id;
    std::vector<int> args;
    int64_t p0, p1;
    std::string str;
    Big val;
    bool is_array() const { return sort == MGC_SORT_ARRAY; }
    bool is_bool() const { return sort == MGC_SORT_BOOL; }
};

static const int CHUNK = 256;
static const int MAX_SPILL = MG_MAX_LDS + MG_MAX_PSLOTS;
static const int LDS_TIER = 6;
static const int POOL_CAP = 128;
static const int ARG_ENTRIES_CAP = 64;

// post-order of everything under roots (smt/node.py topo_order)
static std::vector<int> topo(const std::vector<Src>& S, const std::vector<int>& roots) {
    std::vector<char> seen(S.size(), 0);
    std::vector<int> out;
    std::vector<std::pair<int, bool>> stack;
    for (int r : roots) {
        if (seen[r]) continue;
        stack.assign(1, {r, false});
        while (!stack.empty()) {
            auto [n, done] = stack.back();
            stack.pop_back();
            if (done) { out.push_back(n); continue; }
            if (seen[n]) continue;
            seen[n] = 1;
            stack.push_back({n, true});
            const auto& a = S[n].args;
            for (size_t i = a.size(); i-- > 0;)
                if (!seen[a[i]]) stack.push_back({a[i], false});
        }
    }
    return out;
}

// ---------------------------------------------------------------------------
// lowered DAG (ir.LNode)
// ---------------------------------------------------------------------------
// operand list of an LNode: up to three inline (every op but an n-ary AND),
// so building and hashing nodes allocates nothing
struct Args {
    int n = 0;
    int a[3] = {0, 0, 0};
    std::vector<int> more;
    Args() {}
    Args(std::initializer_list<int> il) { assign(il.begin(), il.end()); }
    Args(const std::vector<int>& v) { assign(v.data(), v.data() + v.size()); }
    template <class It> void assign(It b, It e) {
        n = (int)(e - b);
        if (n <= 3) { std::copy(b, e, a); more.clear(); }
        else more.assign(b, e);
    }
    const int* begin() const { return n <= 3 ? a : more.data(); }
    const int* end() const { return begin() + n; }
    int* begin() { return n <= 3 ? a : more.data(); }
    int* end() { return begin() + n; }
    size_t size() const { return (size_t)n; }
    bool empty() const { return n == 0; }
    int operator[](size_t i) const { return begin()[i]; }
    int& operator[](size_t i) { return begin()[i]; }
    int back() const { return begin()[n - 1]; }
    bool operator==(const Args& o) const { return n == o.n && std::equal(begin(), end(), o.begin()); }
    bool operator!=(const Args& o) const { return !(*this == o); }
};

struct LN {
    int op, width;
    Args args;
    bool has_imm;
    U imm;
    int64_t birth;
};

enum LeafKind { K_VAR, K_KEY, K_VAL, K_ELSE, K_CVAL, K_AUX };
static const char* KIND_NAMES[] = {"var", "key", "val", "else", "cval", "aux"};

struct Leaf {
    std::string name;
    int width;
    int kind;
    std::string source;
    int chunk, entry;
};

static bool is_pred(int op) {
    return op == MG_EQ || op == MG_ULT || op == MG_ULE || op == MG_SLT || op == MG_SLE || op == MG_UMULNO;
}
static bool is_cmp(int op) {      // ir._CMP_OPS
    return op == MG_EQ || op == MG_ULT || op == MG_ULE || op == MG_SLT || op == MG_SLE;
}
static bool is_order(int op) { return op == MG_ULT || op == MG_ULE || op == MG_SLT || op == MG_SLE; }

typedef std::vector<int> Chunks;


struct Lowerer {
    const std::vector<Src>& S;
    std::vector<LN> ln;
    // hash-consing table: open addressing over node ids (a node's key is
    // its own fields, so the table stores ids and hashes only)
    std::vector<int> slot_id;
    std::vector<uint64_t> slot_hash;
    size_t n_slots_used = 0;
    std::vector<Leaf> leaves;
    std::unordered_map<std::string, int> leaf_ids;
    std::vector<Chunks> memo;
    std::vector<char> has_memo;
    std::unordered_map<std::string, Chunks> sel_memo;
    OMap<std::string, int> table_sizes;
    OMap<std::string, std::string> table_kinds;
    int default_entries;
    int64_t birth = 0;
    OMap<std::string, std::vector<Big>> table_ckeys;
    bool solve = false;
    std::unordered_set<std::string> solve_tables;
    OMap<std::string, std::vector<std::pair<Chunks, Chunks>>> arg_entries;

    Lowerer(const std::vector<Src>& s, int de) : S(s), default_entries(de) {
        memo.resize(S.size());
        has_memo.assign(S.size(), 0);
    }

    // -- hash-consed constructors (ir._Lowerer.mk / const / leaf) --------------
    static uint64_t key_hash(int op, int width, const Args& args, bool has_imm, const U& imm) {
        uint64_t h = (uint64_t)op * 0x9E3779B97F4A7C15ull ^ (uint64_t)width * 0xC2B2AE3D27D4EB4Full;
        for (int a : args) h = (h ^ (uint64_t)(uint32_t)a) * 0x100000001B3ull;
        if (has_imm) for (int i = 0; i < U::N; i++) h = (h ^ imm.w[i]) * 0x100000001B3ull;
        h ^= h >> 29;
        return h | 1;                                  // 0 marks an empty slot
    }
    void rehash(size_t n) {
        std::vector<int> ids(n, -1);
        std::vector<uint64_t> hs(n, 0);
        for (size_t i = 0; i < slot_id.size(); i++) {
            if (slot_id[i] < 0) continue;
            size_t j = slot_hash[i] & (n - 1);
            while (ids[j] >= 0) j = (j + 1) & (n - 1);
            ids[j] = slot_id[i];
            hs[j] = slot_hash[i];
        }
        slot_id.swap(ids);
        slot_hash.swap(hs);
    }
    int mk(int op, int width, Args args, bool has_imm = false, const U& imm = U()) {
        if (op == MG_CONCAT && width == MG_MAX_WIDTH && ln[args[0]].op == MG_EXTRACT &&
            ln[args[0]].imm.zero() && ln[ln[args[0]].args[0]].width == MG_MAX_WIDTH)
            args[0] = ln[args[0]].args[0];
        const U key_imm = has_imm ? imm : U();
        if (2 * (n_slots_used + 1) > slot_id.size()) rehash(slot_id.empty() ? 4096 : 2 * slot_id.size());
        uint64_t h = key_hash(op, width, args, has_imm, key_imm);
        size_t j = h & (slot_id.size() - 1);
        while (slot_id[j] >= 0) {
            if (slot_hash[j] == h) {
                const LN& o = ln[slot_id[j]];
                if (o.op == op && o.width == width && o.has_imm == has_imm && o.args == args &&
                    (!has_imm || o.imm == key_imm))
                    return slot_id[j];
            }
            j = (j + 1) & (slot_id.size() - 1);
        }
        int64_t b = birth;
        for (int a : args) if (ln[a].birth > b) b = ln[a].birth;
        int id = (int)ln.size();
        ln.push_back(LN{op, width, std::move(args), has_imm, key_imm, b});
        slot_id[j] = id;
        slot_hash[j] = h;
        n_slots_used++;
        return id;
    }
    int mki(int op, int width, Args args, int64_t imm) { return mk(op, width, std::move(args), true, U::of((uint64_t)imm)); }
    int cnst(const U& value, int width) { return mk(MG_CONST, width, {}, true, value & mask(width)); }
    int cnst(uint64_t value, int width) { return cnst(U::of(value), width); }
    int leaf(const std::string& name, int width, int kind, const std::string& source, int chunk = 0, int entry = 0) {
        auto it = leaf_ids.find(name);
        int idx;
        if (it == leaf_ids.end()) {
            idx = (int)leaves.size();
            leaf_ids.emplace(name, idx);
            leaves.push_back(Leaf{name, width, kind, source, chunk, entry});
        } else {
            idx = it->second;
        }
        return mki(MG_LEAF, width, {}, idx);
    }

    // -- chunk helpers ------------------------------------------------------------
    static int nchunks(int w) { return (w + CHUNK - 1) / CHUNK; }
    static int chunk_width(int w, int i) { return std::min(CHUNK, w - CHUNK * i); }

    int bits(const Chunks& chunks, int w, int lo, int hi) {
        int ci = lo / CHUNK, cj = hi / CHUNK;
        if (ci == cj) {
            int c = chunks.at(ci);
            int cw = chunk_width(w, ci);
            int l0 = lo - CHUNK * ci, h0 = hi - CHUNK * ci;
            if (l0 == 0 && h0 == cw - 1) return c;
            return mki(MG_EXTRACT, h0 - l0 + 1, {c}, l0);
        }
        int low_w = CHUNK * (ci + 1) - lo;
        int low = bits(chunks, w, lo, CHUNK * (ci + 1) - 1);
        int high = bits(chunks, w, CHUNK * cj, hi);
        return mki(MG_CONCAT, hi - lo + 1, {high, low}, low_w);
    }

    Chunks assemble(const std::vector<std::pair<Chunks, int>>& pieces) {
        int total = 0;
        for (auto& p : pieces) total += p.second;
        struct Seg { const Chunks* ch; int w, off; };
        std::vector<Seg> segs;
        int off = 0;
        for (size_t i = pieces.size(); i-- > 0;) {
            segs.push_back({&pieces[i].first, pieces[i].second, off});
            off += pieces[i].second;
        }
        Chunks out;
        for (int k = 0; k < nchunks(total); k++) {
            int lo_k = CHUNK * k, hi_k = std::min(total, CHUNK * (k + 1)) - 1;
            int acc = -1, acc_w = 0;
            for (auto& s : segs) {
                int a = std::max(lo_k, s.off), b = std::min(hi_k, s.off + s.w - 1);
                if (a > b) continue;
                int part = bits(*s.ch, s.w, a - s.off, b - s.off);
                int pw = b - a + 1;
                if (acc < 0) { acc = part; acc_w = pw; }
                else { acc = mki(MG_CONCAT, acc_w + pw, {part, acc}, acc_w); acc_w += pw; }
            }
            out.push_back(acc);
        }
        return out;
    }

    const Chunks& M(int s) {          // self.memo[n.id] (KeyError -> MemoMiss)
        if (!has_memo[s]) throw MemoMiss();
        return memo[s];
    }

    // -- main lowering (ir._Lowerer.lower) -------------------------------------
    // post-order of the nodes under n not lowered yet (ir._Lowerer._pending:
    // a lowered node's operands are not walked again)
    std::vector<char> pend_seen_;
    std::vector<int> pending(int n) {
        if (pend_seen_.size() < S.size()) pend_seen_.assign(S.size(), 0);
        std::vector<int> out, touched;
        std::vector<std::pair<int, bool>> stack{{n, false}};
        while (!stack.empty()) {
            auto [m, done] = stack.back();
            stack.pop_back();
            if (done) { out.push_back(m); continue; }
            if (pend_seen_[m] || has_memo[m]) continue;
            pend_seen_[m] = 1;
            touched.push_back(m);
            stack.push_back({m, true});
            const auto& a = S[m].args;
            for (size_t i = a.size(); i-- > 0;)
                if (!pend_seen_[a[i]] && !has_memo[a[i]]) stack.push_back({a[i], false});
        }
        for (int m : touched) pend_seen_[m] = 0;
        return out;
    }

    const Chunks& lower(int n) {
        if (has_memo[n]) return memo[n];
        std::vector<int> nodes = pending(n);
        std::unordered_set<int> skip;
        for (int m : nodes)
            if (S[m].op == S_EXTRACT && is_carry(m)) {
                int s = S[m].args[0];
                skip.insert(s); skip.insert(S[s].args[0]); skip.insert(S[s].args[1]);
            }
        int64_t saved = birth;
        for (int m : nodes) {
            if (has_memo[m] || S[m].is_array() || (skip.count(m) && m != n)) continue;
            birth = S[m].id;
            try {
                Chunks r = lower_one(m);
                memo[m] = std::move(r);
                has_memo[m] = 1;
            } catch (MemoMiss&) {
                throw Unsupported("operand lowered only as part of a pattern");
            }
            birth = S[m].id;
        }
        birth = saved ? std::max(saved, birth) : birth;
        if (!has_memo[n]) throw Unsupported("operand lowered only as part of a pattern");
        return memo[n];
    }

    int narrow(int s) {
        const Chunks& ch = M(s);
        if (ch.size() != 1)
            throw Unsupported(opname(s) + " on a " + std::to_string(S[s].width) + "-bit value");
        return ch[0];
    }

    std::string opname(int s) {
        // built once, thread-safely (compiles may run on several threads:
        // the CPython front-end releases the GIL)
        static const std::vector<std::string> names = [] {
            std::vector<std::string> v;
            std::string all(SOP_NAMES);
            size_t p = 0;
            while (true) {
                size_t q = all.find('\n', p);
                v.push_back(all.substr(p, q == std::string::npos ? std::string::npos : q - p));
                if (q == std::string::npos) break;
                p = q + 1;
            }
            return v;
        }();
        return S[s].op == S_OTHER ? S[s].str : names[S[s].op];
    }

    int fold(int op, int width, const Chunks& args) {
        int acc = args[0];
        for (size_t i = 1; i < args.size(); i++) acc = mk(op, width, {acc, args[i]});
        return acc;
    }

    // ir._Lowerer._by_constant; returns -1 for None
    int by_constant(int op, int w, int n) {
        const Src& s = S[n];
        if (S[s.args[1]].op != S_BVNUM) return -1;
        const Big& cb = S[s.args[1]].val;
        int x = narrow(s.args[0]);
        // constants beyond 2^64 only matter as "c >= w" / "not a power of two"
        bool huge = cb.l.size() > 2;
        uint64_t c = 0;
        for (size_t j = 0; j < cb.l.size() && j < 2; j++) c |= (uint64_t)cb.l[j] << (32 * j);
        if (op == S_BVUDIV || op == S_BVUREM) {
            bool pow2;
            int k = 0;
            if (huge) {
                int ones = 0, top = 0;
                for (size_t j = 0; j < cb.l.size(); j++) {
                    ones += __builtin_popcount(cb.l[j]);
                    if (cb.l[j]) top = (int)(32 * j + 31 - __builtin_clz(cb.l[j]));
                }
                pow2 = ones == 1;
                k = top;
            } else {
                pow2 = c && !(c & (c - 1));
                if (pow2) k = 63 - __builtin_clzll(c);
            }
            if (!pow2) return -1;
            if (op == S_BVUREM) return k == 0 ? cnst(0, w) : mki(MG_EXTRACT, k, {x}, 0);
            op = S_BVLSHR; c = (uint64_t)k; huge = false;
        }
        if (op != S_BVSHL && op != S_BVLSHR && op != S_BVASHR) return -1;
        if (!huge && c == 0) return x;
        bool ge = huge || c >= (uint64_t)w;
        if (op == S_BVASHR) {
            int cc = ge ? w - 1 : (int)std::min<uint64_t>(c, (uint64_t)(w - 1));
            int e = mki(MG_EXTRACT, w - cc, {x}, cc);
            return mki(MG_SEXT, w, {e}, w - cc);
        }
        if (ge) return cnst(0, w);
        int cc = (int)c;
        if (op == S_BVLSHR) return mki(MG_EXTRACT, w - cc, {x}, cc);
        int e = mki(MG_EXTRACT, w - cc, {x}, 0);
        int z = cnst(0, cc);
        return mki(MG_CONCAT, w, {e, z}, cc);
    }

    Chunks lower_one(int n) {
        const Src& s = S[n];
        int op = s.op, w = s.width;
        if (w > CHUNK) return lower_wide(n);
        auto A = [&](int i) { return narrow(s.args[i]); };
        switch (op) {
        case S_BVNUM: return {cnst(s.val.chunk(0), w)};
        case S_TRUE: return {cnst(1, 1)};
        case S_FALSE: return {cnst(0, 1)};
        case S_VAR: return {leaf(s.str, w, K_VAR, s.str)};
        default: break;
        }
        int simple = -1;
        switch (op) {
        case S_BVSUB: simple = MG_SUB; break;
        case S_BVUDIV: simple = MG_UDIV; break;
        case S_BVUREM: simple = MG_UREM; break;
        case S_BVSDIV: simple = MG_SDIV; break;
        case S_BVSREM: simple = MG_SREM; break;
        case S_BVSMOD: simple = MG_SMOD; break;
        case S_BVSHL: simple = MG_SHL; break;
        case S_BVLSHR: simple = MG_LSHR; break;
        case S_BVASHR: simple = MG_ASHR; break;
        default: break;
        }
        if (simple >= 0) {
            int red = by_constant(op, w, n);
            if (red >= 0) return {red};
            int a = A(0), b = A(1);
            return {mk(simple, w, {a, b})};
        }
        int nary = -1;
        switch (op) {
        case S_BVADD: nary = MG_ADD; break;
        case S_BVMUL: nary = MG_MUL; break;
        case S_BVAND: case S_AND: nary = MG_AND; break;
        case S_BVOR: case S_OR: nary = MG_OR; break;
        case S_BVXOR: nary = MG_XOR; break;
        default: break;
        }
        if (nary >= 0) {
            Chunks xs;
            for (size_t i = 0; i < s.args.size(); i++) xs.push_back(A((int)i));
            return {fold(nary, w, xs)};
        }
        if (op == S_BVNEG) return {mk(MG_NEG, w, {A(0)})};
        if (op == S_BVNOT || op == S_NOT) return {mk(MG_NOT, w, {A(0)})};
        if (op == S_XOR) { int a = A(0), b = A(1); return {mk(MG_XOR, 1, {a, b})}; }
        if (op == S_IMPLIES) {
            int a = A(0);
            int na = mk(MG_NOT, 1, {a});
            int b = A(1);
            return {mk(MG_OR, 1, {na, b})};
        }
        int kop = -1; bool swap = false;
        switch (op) {
        case S_BVULT: kop = MG_ULT; break;
        case S_BVULE: kop = MG_ULE; break;
        case S_BVUGT: kop = MG_ULT; swap = true; break;
        case S_BVUGE: kop = MG_ULE; swap = true; break;
        case S_BVSLT: kop = MG_SLT; break;
        case S_BVSLE: kop = MG_SLE; break;
        case S_BVSGT: kop = MG_SLT; swap = true; break;
        case S_BVSGE: kop = MG_SLE; swap = true; break;
        case S_UMULNO: kop = MG_UMULNO; break;
        default: break;
        }
        if (kop >= 0) {
            int a = A(0), b = A(1);
            if (swap) std::swap(a, b);
            return {mk(kop, S[s.args[0]].width, {a, b})};
        }
        if (op == S_EQ || op == S_DISTINCT) {
            for (int a : s.args) if (S[a].is_array()) throw Unsupported("array equality");
            return {eq_or_distinct(op, n)};
        }
        if (op == S_ITE) {
            if (s.is_array()) throw Unsupported("array-valued ite outside select");
            int c = A(0), a = A(1), b = A(2);
            return {mk(MG_ITE, w, {c, a, b})};
        }
        if (op == S_CONCAT) {
            int word = calldata_word(n);
            if (word >= 0) return {word};
            std::vector<std::pair<Chunks, int>> pieces;
            for (int a : s.args) pieces.push_back({M(a), S[a].width});
            return assemble(pieces);
        }
        if (op == S_EXTRACT) {
            int carry = carry_pattern(n);
            if (carry >= 0) return {carry};
            int src = s.args[0];
            return {bits(M(src), S[src].width, (int)s.p1, (int)s.p0)};
        }
        if (op == S_ZEXT) return {narrow(s.args[0])};
        if (op == S_SEXT) return {mki(MG_SEXT, w, {A(0)}, S[s.args[0]].width)};
        if (op == S_SELECT) {
            Chunks idx = M(s.args[1]);
            return select(s.args[0], idx, S[s.args[1]].width, w);
        }
        if (op == S_APPLY) {
            Chunks key = M(s.args[0]);
            return table_lookup(s.str, key, (int)s.p0, w, "func");
        }
        throw Unsupported("operator " + opname(n));
    }

    int eq_parts(const Chunks& x, const Chunks& y, int w) {
        Chunks parts;
        for (size_t k = 0; k < x.size(); k++)
            parts.push_back(mk(MG_EQ, w > CHUNK ? chunk_width(w, (int)k) : w, {x[k], y.at(k)}));
        return fold(MG_AND, 1, parts);
    }

    int eq_or_distinct(int op, int n) {
        const Src& s = S[n];
        std::vector<const Chunks*> args;
        for (int a : s.args) args.push_back(&M(a));
        int w = S[s.args[0]].width;
        if (op == S_EQ) return eq_parts(*args[0], *args[1], w);
        Chunks terms;
        for (size_t i = 0; i < args.size(); i++)
            for (size_t j = i + 1; j < args.size(); j++) {
                int e = eq_parts(*args[i], *args[j], w);
                terms.push_back(mk(MG_NOT, 1, {e}));
            }
        return fold(MG_AND, 1, terms);
    }

    bool is_carry(int n) const {
        const Src& x = S[n];
        int64_t hi = x.p0, lo = x.p1;
        const Src& s = S[x.args[0]];
        if (hi != lo || s.op != S_BVADD || s.args.size() != 2 || hi != s.width - 1) return false;
        const Src& a = S[s.args[0]];
        const Src& b = S[s.args[1]];
        return a.op == S_ZEXT && b.op == S_ZEXT && a.p0 == 1 && b.p0 == 1 &&
               S[a.args[0]].width <= CHUNK;
    }

    int carry_pattern(int n) {
        if (!is_carry(n)) return -1;
        const Src& s = S[S[n].args[0]];
        int x = S[s.args[0]].args[0], y = S[s.args[1]].args[0];
        int lx = lower(x)[0];
        int ly = lower(y)[0];
        int sum = mk(MG_ADD, S[x].width, {lx, ly});
        return mk(MG_ULT, S[x].width, {sum, lx});
    }

    Chunks lower_wide(int n) {
        const Src& s = S[n];
        int op = s.op, w = s.width;
        if (op == S_BVNUM) {
            Chunks out;
            for (int k = 0; k < nchunks(w); k++) out.push_back(cnst(s.val.chunk(k), chunk_width(w, k)));
            return out;
        }
        if (op == S_VAR) {
            Chunks out;
            for (int k = 0; k < nchunks(w); k++)
                out.push_back(leaf(s.str + "#" + std::to_string(k), chunk_width(w, k), K_VAR, s.str, k));
            return out;
        }
        if (op == S_CONCAT) {
            std::vector<std::pair<Chunks, int>> pieces;
            for (int a : s.args) pieces.push_back({M(a), S[a].width});
            return assemble(pieces);
        }
        if (op == S_EXTRACT) {
            int src = s.args[0];
            int hi = (int)s.p0, lo = (int)s.p1;
            const Chunks& sc = M(src);
            std::vector<std::pair<Chunks, int>> pieces;
            for (int k = nchunks(w) - 1; k >= 0; k--) {
                int b = bits(sc, S[src].width, lo + CHUNK * k, std::min(hi, lo + CHUNK * k + CHUNK - 1));
                pieces.push_back({{b}, std::min(CHUNK, hi - lo + 1 - CHUNK * k)});
            }
            return assemble(pieces);
        }
        if (op == S_ZEXT) {
            int src = s.args[0];
            int pad = w - S[src].width;
            std::vector<std::pair<Chunks, int>> pieces;
            while (pad > 0) {
                int pw = std::min(CHUNK, pad);
                pieces.push_back({{cnst(0, pw)}, pw});
                pad -= pw;
            }
            pieces.push_back({M(src), S[src].width});
            return assemble(pieces);
        }
        if (op == S_ITE) {
            int c = narrow(s.args[0]);
            Chunks a = M(s.args[1]), b = M(s.args[2]);
            return ite_chunks(c, a, b);
        }
        if (op == S_SELECT) {
            Chunks idx = M(s.args[1]);
            return select(s.args[0], idx, S[s.args[1]].width, w);
        }
        if (op == S_APPLY) {
            Chunks key = M(s.args[0]);
            return table_lookup(s.str, key, (int)s.p0, w, "func");
        }
        throw Unsupported(opname(n) + " on a " + std::to_string(w) + "-bit value");
    }

    // -- the calldata word (ir._Lowerer._calldata_word) --------------------------
    // x = base + c (mod 2^256), nested adds of numerals folded: base -1 for
    // a numeral
    void index_parts(int x, int& base, U& c) const {
        c = U();
        while (true) {
            const Src& s = S[x];
            if (s.op == S_BVNUM) { base = -1; c = (c + s.val.chunk(0)) & mask(256); return; }
            if (s.op != S_BVADD || s.args.size() != 2) { base = x; return; }
            int a = s.args[0], b = s.args[1];
            if (S[b].op == S_BVNUM && S[a].op != S_BVNUM) { c = (c + S[b].val.chunk(0)) & mask(256); x = a; }
            else if (S[a].op == S_BVNUM && S[b].op != S_BVNUM) { c = (c + S[a].val.chunk(0)) & mask(256); x = b; }
            else { base = x; return; }
        }
    }

    int calldata_word(int n) {
        const Src& s = S[n];
        if (s.width != 256 || s.args.size() != 32) return -1;
        int size = -1, arr = -1, base = -1, off = -1;
        U c0;
        for (int i = 0; i < 32; i++) {
            const Src& x = S[s.args[i]];
            if (x.op != S_ITE || x.width != 8) return -1;
            const Src& cond = S[x.args[0]];
            const Src& sel = S[x.args[1]];
            const Src& zero = S[x.args[2]];
            if (zero.op != S_BVNUM || !zero.val.l.empty() || cond.op != S_BVSLT || sel.op != S_SELECT)
                return -1;
            int idx = sel.args[1];
            if (cond.args[0] != idx || S[idx].width != 256) return -1;
            if (i == 0) {
                size = cond.args[1];
                arr = sel.args[0];
                if (S[arr].op != S_ARRAY) return -1;
                index_parts(idx, base, c0);
                off = idx;
            } else if (cond.args[1] != size || sel.args[0] != arr) {
                return -1;
            } else {
                int b;
                U c;
                index_parts(idx, b, c);
                if (b != base || !(c == ((c0 + U::of((uint64_t)i)) & mask(256)))) return -1;
            }
        }
        const std::string& name = S[arr].str;
        const std::vector<Big>* ck = table_ckeys.find(name);
        if ((ck && !ck->empty()) || (solve && solve_tables.count(name))) return -1;
        table_kinds.put(name, "array");
        int entries = table_sizes.setdefault(name, default_entries);
        int o = narrow(off), sz = narrow(size);
        int acc = mk(MG_BCAST, 256, {cell(name, K_ELSE, 0, 8)[0]});
        for (int e = entries - 1; e >= 0; e--) {
            int key = cell(name, K_KEY, e, 256)[0];
            int delta = mk(MG_SUB, 256, {key, o});
            int val = cell(name, K_VAL, e, 8)[0];
            acc = mk(MG_CDWE, 256, {acc, delta, val});
        }
        return mk(MG_CDWX, 256, {acc, o, sz});
    }

    // -- arrays and uninterpreted functions ----------------------------------------
    int chunk_eq(const Chunks& x, const Chunks& y, int w) {
        Chunks parts;
        for (size_t k = 0; k < x.size(); k++) parts.push_back(mk(MG_EQ, chunk_width(w, (int)k), {x[k], y.at(k)}));
        return fold(MG_AND, 1, parts);
    }

    Chunks ite_chunks(int c, const Chunks& a, const Chunks& b) {
        Chunks out;
        for (size_t i = 0; i < a.size() && i < b.size(); i++)
            out.push_back(mk(MG_ITE, std::max(ln[a[i]].width, ln[b[i]].width), {c, a[i], b[i]}));
        return out;
    }

    Chunks cell(const std::string& name, int kind, int e, int width) {
        std::string tag;
        switch (kind) {
        case K_KEY: tag = "k" + std::to_string(e); break;
        case K_VAL: tag = "v" + std::to_string(e); break;
        case K_ELSE: tag = "else"; break;
        default: tag = "c" + std::to_string(e); break;
        }
        Chunks out;
        for (int k = 0; k < nchunks(width); k++)
            out.push_back(leaf(name + "#" + tag + "#" + std::to_string(k), chunk_width(width, k), kind, name, k, e));
        return out;
    }

    Chunks const_key(const Big& v, int kw) {
        Chunks c;
        for (int k = 0; k < nchunks(kw); k++) c.push_back(cnst(v.chunk(k), chunk_width(kw, k)));
        return c;
    }

    Chunks table_lookup(const std::string& name, const Chunks& key, int kw, int vw, const char* kind) {
        table_kinds.put(name, kind);
        std::string mkey = "T" + name;
        mkey.push_back('\0');
        mkey.append((const char*)key.data(), 4 * key.size());
        auto hit = sel_memo.find(mkey);
        if (hit != sel_memo.end()) return hit->second;
        int entries = table_sizes.setdefault(name, default_entries);
        static const std::vector<Big> none;
        const std::vector<Big>* ckp = table_ckeys.find(name);
        const std::vector<Big>& ckeys = ckp ? *ckp : none;
        bool has_kval = true;
        for (int k : key) if (ln[k].op != MG_CONST) { has_kval = false; break; }
        Big kval;
        if (has_kval) {
            for (size_t i = 0; i < key.size(); i++) {
                Big part = big_of(ln[key[i]].imm);
                if (kval.l.size() < 8 * i + part.l.size()) kval.l.resize(8 * i + part.l.size(), 0);
                for (size_t j = 0; j < part.l.size(); j++) kval.l[8 * i + j] |= part.l[j];
            }
            kval.norm();
        }
        int kidx = -1;
        if (has_kval)
            for (size_t i = 0; i < ckeys.size(); i++) if (ckeys[i] == kval) { kidx = (int)i; break; }
        Chunks acc;
        if (kidx >= 0) {
            acc = cell(name, K_CVAL, kidx, vw);
        } else if (solve && solve_tables.count(name)) {
            auto& ents = arg_entries.setdefault(name, {});
            Chunks val = cell(name, K_VAL, (int)ents.size(), vw);
            acc = val;
            for (size_t i = ents.size(); i-- > 0;) {
                int e = chunk_eq(key, ents[i].first, kw);
                acc = ite_chunks(e, ents[i].second, acc);
            }
            ents.push_back({key, val});
            table_sizes.put(name, (int)ents.size());
            if (!has_kval)
                for (size_t i = ckeys.size(); i-- > 0;) {
                    Chunks c = const_key(ckeys[i], kw);
                    int e = chunk_eq(key, c, kw);
                    Chunks cv = cell(name, K_CVAL, (int)i, vw);
                    acc = ite_chunks(e, cv, acc);
                }
        } else {
            acc = cell(name, K_ELSE, 0, vw);
            for (int e = entries - 1; e >= 0; e--) {
                Chunks kc = cell(name, K_KEY, e, kw);
                int q = chunk_eq(key, kc, kw);
                Chunks vc = cell(name, K_VAL, e, vw);
                acc = ite_chunks(q, vc, acc);
            }
            if (!has_kval)
                for (size_t i = ckeys.size(); i-- > 0;) {
                    Chunks c = const_key(ckeys[i], kw);
                    int q = chunk_eq(key, c, kw);
                    Chunks cv = cell(name, K_CVAL, (int)i, vw);
                    acc = ite_chunks(q, cv, acc);
                }
        }
        sel_memo[mkey] = acc;
        return acc;
    }

    Chunks select(int arr, const Chunks& idx, int iw, int vw) {
        std::string mkey = "A" + std::to_string(arr);
        mkey.push_back('\0');
        mkey.append((const char*)idx.data(), 4 * idx.size());
        auto hit = sel_memo.find(mkey);
        if (hit != sel_memo.end()) return hit->second;
        std::vector<int> chain;
        int a = arr;
        while (S[a].op == S_STORE) { chain.push_back(a); a = S[a].args[0]; }
        Chunks base;
        if (S[a].op == S_K) {
            base = lower(S[a].args[0]);
        } else if (S[a].op == S_ARRAY) {
            base = table_lookup(S[a].str, idx, iw, vw, "array");
        } else if (S[a].op == S_ITE) {
            int c = narrow_node(S[a].args[0]);
            Chunks x = select(S[a].args[1], idx, iw, vw);
            Chunks y = select(S[a].args[2], idx, iw, vw);
            base = ite_chunks(c, x, y);
        } else {
            throw Unsupported("array term " + opname(a));
        }
        Chunks acc = base;
        for (size_t i = chain.size(); i-- > 0;) {
            int st = chain[i];
            Chunks j = lower(S[st].args[1]);
            Chunks v = lower(S[st].args[2]);
            int e = chunk_eq(idx, j, iw);
            acc = ite_chunks(e, v, acc);
        }
        sel_memo[mkey] = acc;
        return acc;
    }

    int narrow_node(int n) {
        const Chunks& ch = lower(n);
        if (ch.size() != 1) throw Unsupported("wide condition");
        return ch[0];
    }
};

// ---------------------------------------------------------------------------
// search-mode model construction (mythril_amd/solve.py Solver)
// ---------------------------------------------------------------------------
static const int PASSES = 6;
static const int MAX_REFUSALS = 4;          // solve.MAX_REFUSALS
static const int SCHEDULE_MIN_SCRATCH = 10; // ir.SCHEDULE_MIN_SCRATCH
static const int MAX_DOMAIN = 16;
static const int MAX_BRANCHES = 4;
static const int MAX_OR = 64;
static const int BRANCH_DEPTH = 2;
static const int SELECTOR_WIDTH = 8;

// rewrite memo; an overlay reads through to its parent (solve._Overlay).
// Overlays live one at a time per solver over a shared dense table: a slot
// belongs to the overlay whose generation it carries (no hashing, no clear)
struct OverlayTable {
    std::vector<int> val, gen;
    int next_gen = 0;
};
struct Memo {
    std::vector<int> dense;                 // base memo: LNode id -> result
    const Memo* parent = nullptr;
    OverlayTable* ov = nullptr;             // overlay: local writes
    int gen = 0;
    int get(int k) const {
        if (!parent) return (size_t)k < dense.size() ? dense[k] : -1;
        if ((size_t)k < ov->gen.size() && ov->gen[k] == gen) return ov->val[k];
        return parent->get(k);
    }
    void put(int k, int v) {
        if (parent) {
            if ((size_t)k >= ov->gen.size()) {
                size_t sz = std::max<size_t>(k + 1, 2 * ov->gen.size());
                ov->gen.resize(sz, 0);
                ov->val.resize(sz, -1);
            }
            ov->gen[k] = gen;
            ov->val[k] = v;
            return;
        }
        if ((size_t)k >= dense.size()) dense.resize(std::max<size_t>(k + 1, 2 * dense.size()), -1);
        dense[k] = v;
    }
    void overlay_on(const Memo* p, OverlayTable* t) {
        parent = p;
        ov = t;
        gen = ++t->next_gen;
    }
};

struct Interval { U lo, hi; };
struct Bound { int e; U lo, hi; int w; };

struct Solver {
    Lowerer& lw;
    std::vector<LN>& ln;
    OMap<int, int> repl;                   // LEAF id -> definition
    // dense mirror of repl for the lookups (rewrite, depends, try_define):
    // LEAF id -> definition, -1 when undefined
    std::vector<int> repl_of_;
    const int* repl_find(int x) const {
        return (size_t)x < repl_of_.size() && repl_of_[x] >= 0 ? &repl_of_[x] : nullptr;
    }
    void repl_put(int k, int v) {
        repl.put(k, v);
        if ((size_t)k >= repl_of_.size()) repl_of_.resize(std::max<size_t>(k + 1, 2 * repl_of_.size()), -1);
        repl_of_[k] = v;
    }
    void repl_truncate(size_t n) {
        for (size_t i = n; i < repl.items.size(); i++) repl_of_[repl.items[i].first] = -1;
        repl.truncate(n);
    }
    int one, zero;
    int n_aux = 0, n_branch = 0;
    std::unordered_set<int> selectors, or_seen;
    std::vector<char> clean_;
    bool is_clean(int x) const { return (size_t)x < clean_.size() && clean_[x]; }
    void set_clean(int x) { if ((size_t)x >= clean_.size()) clean_.resize(std::max<size_t>(x + 1, 2 * clean_.size()), 0); clean_[x] = 1; }
    std::vector<int> stamp_;
    int stamp_gen_ = 0;
    int new_stamp() { return ++stamp_gen_; }
    bool stamped(int x, int g) { if ((size_t)x >= stamp_.size()) stamp_.resize(std::max<size_t>(x + 1, 2 * stamp_.size()), 0); if (stamp_[x] == g) return true; stamp_[x] = g; return false; }
    // leaf dependency sets, one row of dep_w words per LNode in one arena
    // (no allocation per node; re-laid out when a leaf index outgrows it)
    int dep_w = 0;
    std::vector<uint64_t> dep;
    std::vector<char> has_dep;
    struct DepRow {
        const uint64_t* p;
        int w;
        bool meets(const Bits& o) const {
            int n = std::min(w, (int)o.w.size());
            for (int i = 0; i < n; i++) if (p[i] & o.w[i]) return true;
            return false;
        }
        template <class F> void each(F f) const {
            for (int i = 0; i < w; i++) {
                uint64_t x = p[i];
                while (x) { int b = __builtin_ctzll(x); f(64 * i + b); x &= x - 1; }
            }
        }
    };
    std::vector<Interval> ivl_;
    std::vector<char> has_ivl_;
    std::unordered_set<std::string> joint_done;
    std::unordered_map<int, int> leaf_imm, leaf_node;
    bool dm_valid = false;
    Bits dm;
    Memo base_memo;
    Memo* run_memo = &base_memo;
    std::unordered_map<int, int> depth;
    bool unsat = false;
    bool dead = false;                      // run: a root folded to false
    // run repeats the construction after refusing the definition that made
    // a root fold to false: leaves by id, generated leaves by their ordinal
    // in the construction (key)
    std::unordered_map<int, int> aux_seq;
    std::unordered_set<int> refused;
    // leaves defined from an overflow test's atoms (the module's check)
    bool wrap_ctx = false;
    std::unordered_set<int> wrap_defs;

    std::vector<std::pair<int, bool>> rw_stack_;

    explicit Solver(Lowerer& l) : lw(l), ln(l.ln) {
        one = lw.cnst(1, 1);
        zero = lw.cnst(0, 1);
    }

    const LN& N(int i) const { return ln[i]; }

    // -- rewriting ----------------------------------------------------------------
    Interval interval(int n) {
        if ((size_t)n < has_ivl_.size() && has_ivl_[n]) return ivl_[n];
        U top = mask(ln[n].width);
        Interval r;
        int op = ln[n].op;
        if (op == MG_CONST) {
            r = {ln[n].imm, ln[n].imm};
        } else if (op == MG_ADD) {
            Interval a = interval(ln[n].args[0]), b = interval(ln[n].args[1]);
            U hs = a.hi + b.hi;
            r = hs <= top ? Interval{a.lo + b.lo, hs} : Interval{U(), top};
        } else if (op == MG_ITE) {
            Interval a = interval(ln[n].args[1]), b = interval(ln[n].args[2]);
            r = {umin(a.lo, b.lo), umax(a.hi, b.hi)};
        } else if (is_pred(op)) {
            r = {U(), U::of(1)};
        } else {
            r = {U(), top};
        }
        if ((size_t)n >= has_ivl_.size()) { size_t sz = std::max<size_t>(n + 1, 2 * has_ivl_.size()); has_ivl_.resize(sz, 0); ivl_.resize(sz); }
        ivl_[n] = r;
        has_ivl_[n] = 1;
        return r;
    }

    int cmp_fold(int op, int w, int a, int b) {
        Interval A = interval(a), B = interval(b);
        if (op == MG_SLT || op == MG_SLE) {
            U half = U1(w - 1);
            if (A.hi >= half || B.hi >= half) return -1;
        }
        if (op == MG_ULT || op == MG_SLT) {
            if (A.hi < B.lo) return one;
            if (A.lo >= B.hi) return zero;
        } else {
            if (A.hi <= B.lo) return one;
            if (A.lo > B.hi) return zero;
        }
        return -1;
    }

    bool const_fold(int x, const Args& args, U& out) {
        int w = ln[x].width, op = ln[x].op;
        U m = mask(w);
        auto v = [&](int i) { return ln[args[i]].imm; };
        switch (op) {
        case MG_CONCAT: out = (shl(v(0), (int)ln[x].imm.w[0]) | v(1)) & m; return true;
        case MG_EXTRACT: out = shr(v(0), (int)ln[x].imm.w[0]) & m; return true;
        case MG_AND: out = v(0) & v(1) & m; return true;
        case MG_OR: out = (v(0) | v(1)) & m; return true;
        case MG_XOR: out = (v(0) ^ v(1)) & m; return true;
        case MG_SUB: out = (v(0) - v(1)) & m; return true;
        case MG_MUL: out = (v(0) * v(1)) & m; return true;
        case MG_NOT: out = ~v(0) & m; return true;
        default: return false;
        }
    }

    bool all_const(const Args& args) const {
        for (int a : args) if (ln[a].op != MG_CONST) return false;
        return true;
    }

    int fold(int x, const Args& args) {
        int op = ln[x].op;
        if ((op == MG_CONCAT || op == MG_EXTRACT || op == MG_AND || op == MG_OR || op == MG_XOR ||
             op == MG_SUB || op == MG_MUL || op == MG_NOT) && all_const(args)) {
            U c;
            if (const_fold(x, args, c)) return lw.cnst(c, ln[x].width);
        }
        if (is_order(op) && !all_const(args)) {
            int r = cmp_fold(op, ln[x].width, args[0], args[1]);
            if (r >= 0) return r;
        }
        if (op == MG_EQ) {
            int a = args[0], b = args[1];
            if (a == b) return one;
            if (ln[a].op == MG_CONST && ln[b].op == MG_CONST) return ln[a].imm == ln[b].imm ? one : zero;
            int ya = a, yb = b;
            U ca, cb;
            if (ln[a].op == MG_ADD && ln[ln[a].args[1]].op == MG_CONST) { ya = ln[a].args[0]; ca = ln[ln[a].args[1]].imm; }
            if (ln[b].op == MG_ADD && ln[ln[b].args[1]].op == MG_CONST) { yb = ln[b].args[0]; cb = ln[ln[b].args[1]].imm; }
            if (ya == yb && ln[a].width == ln[b].width && ln[ya].op != MG_CONST) return ca == cb ? one : zero;
            Interval A = interval(a), B = interval(b);
            if (A.hi < B.lo || B.hi < A.lo) return zero;
        } else if (op == MG_ADD) {
            int a = args[0], b = args[1];
            if (ln[a].op == MG_CONST && ln[b].op != MG_CONST) std::swap(a, b);
            if (ln[b].op == MG_CONST) {
                int w = ln[x].width;
                if (ln[a].op == MG_CONST) return lw.cnst((ln[a].imm + ln[b].imm) & mask(w), w);
                if (ln[b].imm.zero() && ln[a].width <= w) return a;
                if (ln[a].op == MG_ADD && ln[a].width == w && ln[ln[a].args[1]].op == MG_CONST) {
                    int y = ln[a].args[0];
                    int c = lw.cnst((ln[ln[a].args[1]].imm + ln[b].imm) & mask(w), w);
                    return lw.mk(MG_ADD, w, {y, c});
                }
                if (!(a == args[0] && b == args[1])) return lw.mk(MG_ADD, w, {a, b});
            }
        } else if (is_order(op) && all_const(args)) {
            U a = ln[args[0]].imm, b = ln[args[1]].imm;
            if (op == MG_SLT || op == MG_SLE) {
                U half = U1(ln[x].width - 1);      // signed order = unsigned order of a ^ half
                a = a ^ half; b = b ^ half;
            }
            bool r = (op == MG_ULT || op == MG_SLT) ? a < b : a <= b;
            return r ? one : zero;
        } else if (op == MG_ITE) {
            int c = args[0];
            if (ln[c].op == MG_CONST) return (ln[c].imm.w[0] & 1) ? args[1] : args[2];
            if (args[1] == args[2]) return args[1];
        } else if ((op == MG_AND || op == MG_OR) && ln[x].width == 1) {
            uint64_t absorb = op == MG_AND ? 0 : 1;
            Chunks rest;
            for (int a : args) {
                if (ln[a].op == MG_CONST) {
                    if ((ln[a].imm.w[0] & 1) == absorb) return ln[a].width == 1 ? a : lw.cnst(absorb, 1);
                    continue;
                }
                rest.push_back(a);
            }
            if (rest.empty()) return lw.cnst(1 - absorb, 1);
            if (rest.size() == 1) return rest[0];
            if (rest[0] == rest[1]) return rest[0];
        } else if (op == MG_NOT && ln[x].width == 1) {
            int a = args[0];
            if (ln[a].op == MG_CONST) return lw.cnst(1 - (ln[a].imm.w[0] & 1), 1);
            if (ln[a].op == MG_NOT && ln[a].width == 1) return ln[a].args[0];
        }
        bool same = true;
        for (size_t i = 0; i < args.size(); i++) if (args[i] != ln[x].args[i]) { same = false; break; }
        if (same) return x;
        return lw.mk(op, ln[x].width, args, ln[x].has_imm, ln[x].imm);
    }

    void dep_layout(size_t rows, int w) {          // grow rows and / or width
        if (w != dep_w) {
            std::vector<uint64_t> d(rows * (size_t)w, 0);
            for (size_t r = 0; r < has_dep.size(); r++)
                if (has_dep[r]) std::copy(dep.begin() + r * dep_w, dep.begin() + r * dep_w + dep_w, d.begin() + r * w);
            dep.swap(d);
            dep_w = w;
        } else {
            dep.resize(rows * (size_t)w, 0);
        }
        has_dep.resize(rows, 0);
    }

    DepRow depof(int n) {
        if ((size_t)n < has_dep.size() && has_dep[n]) return DepRow{dep.data() + (size_t)n * dep_w, dep_w};
        int need_w = (int)(lw.leaves.size() + 63) / 64 + 1;
        if (has_dep.size() < ln.size() || need_w > dep_w)   // geometric: nodes keep being created
            dep_layout(std::max(ln.size(), 2 * has_dep.size()), std::max(dep_w, need_w));
        dep_stack_.clear();
        dep_stack_.push_back(n);
        while (!dep_stack_.empty()) {
            int x = dep_stack_.back();
            if (has_dep[x]) { dep_stack_.pop_back(); continue; }
            bool pend = false;
            for (int a : ln[x].args) if (!has_dep[a]) { dep_stack_.push_back(a); pend = true; }
            if (pend) continue;
            dep_stack_.pop_back();
            uint64_t* row = dep.data() + (size_t)x * dep_w;
            if (ln[x].op == MG_LEAF) {
                int li = (int)ln[x].imm.w[0];
                row[li >> 6] |= 1ull << (li & 63);
            } else {
                for (int a : ln[x].args) {
                    const uint64_t* src = dep.data() + (size_t)a * dep_w;
                    for (int i = 0; i < dep_w; i++) row[i] |= src[i];
                }
            }
            has_dep[x] = 1;
        }
        return DepRow{dep.data() + (size_t)n * dep_w, dep_w};
    }
    std::vector<int> dep_stack_;

    const Bits& defmask() {
        if (!dm_valid) {
            dm = Bits();
            for (auto& kv : repl.items) dm.set(leaf_imm[kv.first]);
            dm_valid = true;
        }
        return dm;
    }

    int rewrite(int n, Memo& memo) {
        const Bits& dmask = defmask();
        auto& stack = rw_stack_;
        stack.clear();
        stack.push_back({n, false});
        while (!stack.empty()) {
            auto [x, done] = stack.back();
            stack.pop_back();
            if (!done) {
                int r = memo.get(x);
                if (r >= 0 && !depof(r).meets(dmask)) continue;
            }
            if (ln[x].op == MG_LEAF) {
                const int* e = repl_find(x);
                if (!e) { memo.put(x, x); continue; }
                int ev = *e;
                int r = memo.get(ev);
                if (r >= 0 && !depof(r).meets(dmask)) memo.put(x, r);
                else { stack.push_back({x, false}); stack.push_back({ev, false}); }
                continue;
            }
            if (ln[x].args.empty()) { memo.put(x, x); continue; }
            if (!done) {
                if (is_clean(x) && !depof(x).meets(dmask)) { memo.put(x, x); continue; }
                stack.push_back({x, true});
                Args args = ln[x].args;
                for (int a : args) {
                    int r = memo.get(a);
                    if (r < 0 || depof(r).meets(dmask)) stack.push_back({a, false});
                }
                continue;
            }
            Args args = ln[x].args;
            for (int& a : args) {
                int r = memo.get(a);
                if (r < 0) throw std::runtime_error("rewrite: operand missing");
                a = r;
            }
            int r = fold(x, args);
            set_clean(r);
            memo.put(x, r);
        }
        return memo.get(n);
    }

    // -- small constructors -------------------------------------------------------
    int not_(int a) {
        if (ln[a].op == MG_CONST) return lw.cnst(1 - (ln[a].imm.w[0] & 1), 1);
        if (ln[a].op == MG_NOT && ln[a].width == 1) return ln[a].args[0];
        return lw.mk(MG_NOT, 1, {a});
    }
    int eq_(int a, const U& k) {
        if (nz(shr(k, ln[a].width))) return zero;
        if (ln[a].op == MG_CONST) return ln[a].imm == k ? one : zero;
        int c = lw.cnst(k, ln[a].width);
        return lw.mk(MG_EQ, ln[a].width, {a, c});
    }
    int ext(int a, int off, int k) {
        if (off == 0 && k == ln[a].width) return a;
        if (ln[a].op == MG_CONST) return lw.cnst(shr(ln[a].imm, off) & mask(k), k);
        if (ln[a].op == MG_EXTRACT) return ext(ln[a].args[0], (int)ln[a].imm.w[0] + off, k);
        return lw.mki(MG_EXTRACT, k, {a}, off);
    }
    int hi_part(int a) {
        int hi = ln[a].args[0];
        int lw_ = (int)ln[a].imm.w[0];
        int hw = ln[a].width - lw_;
        return ln[hi].width == hw ? hi : ext(hi, 0, hw);
    }

    // -- atoms --------------------------------------------------------------------
    bool split_eq(int x, Chunks& out) {
        int a = ln[x].args[0], b = ln[x].args[1];
        if (ln[a].op == MG_CONST && ln[b].op != MG_CONST) std::swap(a, b);
        if (ln[b].op != MG_CONST) return false;
        U k = ln[b].imm;
        int aop = ln[a].op;
        if (is_pred(aop) || ((aop == MG_AND || aop == MG_OR || aop == MG_NOT) && ln[a].width == 1)) {
            if (k > U::of(1)) { out = {zero}; return true; }
            out = {k.zero() ? not_(a) : a};
            return true;
        }
        if (aop == MG_ITE) {
            int c = ln[a].args[0], p = ln[a].args[1], q = ln[a].args[2];
            if (ln[p].op == MG_CONST && ln[q].op == MG_CONST) {
                if (ln[p].imm == k && ln[q].imm == k) { out = {}; return true; }
                if (ln[p].imm == k) { out = {c}; return true; }
                if (ln[q].imm == k) { out = {not_(c)}; return true; }
                out = {zero};
                return true;
            }
            if (ln[q].op == MG_CONST) {
                if (ln[q].imm != k) { int e = eq_(p, k); out = {c, e}; return true; }
                Interval iv = interval(p);
                out = {(iv.lo <= k && k <= iv.hi) ? eq_(p, k) : not_(c)};
                return true;
            }
            if (ln[p].op == MG_CONST) {
                if (ln[p].imm != k) { int nc = not_(c); int e = eq_(q, k); out = {nc, e}; return true; }
                Interval iv = interval(q);
                out = {(iv.lo <= k && k <= iv.hi) ? eq_(q, k) : c};
                return true;
            }
            int e1 = eq_(p, k);
            int e2 = eq_(q, k);
            out = {e1, e2};
            return true;
        }
        if (aop == MG_AND && ln[a].width > 1) {
            int m = ln[a].args[0], z = ln[a].args[1];
            if (ln[z].op == MG_CONST) std::swap(m, z);
            if (ln[m].op != MG_CONST) return false;
            U mi = ln[m].imm;
            if (nz(k & ~mi)) { out = {zero}; return true; }
            U zm = mask(ln[z].width);
            if ((mi & zm) == zm) { out = {eq_(z, k)}; return true; }
            U low = mi & zm;
            if ((low & (low + U::of(1))).zero()) {
                int e = ext(z, 0, low.bitlen());
                out = {eq_(e, k)};
                return true;
            }
            return false;
        }
        if (aop == MG_CONCAT) {
            if (nz(shr(k, ln[a].width))) { out = {zero}; return true; }
            int lw_ = (int)ln[a].imm.w[0];
            int lo = ln[a].args[1];
            int e1 = eq_(lo, k & mask(lw_));
            int h = hi_part(a);
            int e2 = eq_(h, shr(k, lw_));
            out = {e1, e2};
            return true;
        }
        if (aop == MG_EXTRACT) {
            int y = ln[a].args[0], off = (int)ln[a].imm.w[0], w = ln[a].width;
            if (ln[y].op == MG_CONCAT) {
                int lw_ = (int)ln[y].imm.w[0];
                int lo = ln[y].args[1];
                if (off + w <= lw_) { int e = ext(lo, off, w); out = {eq_(e, k)}; return true; }
                int hi = hi_part(y);
                if (off >= lw_) { int e = ext(hi, off - lw_, w); out = {eq_(e, k)}; return true; }
                int n_lo = lw_ - off;
                int e1 = ext(lo, off, n_lo);
                int q1 = eq_(e1, k & mask(n_lo));
                int e2 = ext(hi, 0, w - n_lo);
                int q2 = eq_(e2, shr(k, n_lo));
                out = {q1, q2};
                return true;
            }
            if (ln[y].op == MG_ITE) {
                int c = ln[y].args[0], p = ln[y].args[1], q = ln[y].args[2];
                int ep = ext(p, off, w);
                int eq = ext(q, off, w);
                int it = lw.mk(MG_ITE, w, {c, ep, eq});
                int kc = lw.cnst(k, w);
                out = {lw.mk(MG_EQ, w, {it, kc})};
                return true;
            }
        }
        return false;
    }

    int neg_eq(int y) {        // -1 for None
        int a = ln[y].args[0], b = ln[y].args[1];
        if (ln[a].op == MG_CONST && ln[b].op != MG_CONST) std::swap(a, b);
        if (ln[b].op != MG_CONST) return -1;
        int aop = ln[a].op;
        if (is_pred(aop) || ((aop == MG_AND || aop == MG_OR || aop == MG_NOT) && ln[a].width == 1)) {
            if (ln[b].imm > U::of(1)) return one;
            return ln[b].imm.zero() ? a : not_(a);
        }
        if (aop != MG_ITE) return -1;
        int c = ln[a].args[0], p = ln[a].args[1], q = ln[a].args[2];
        if (ln[p].op != MG_CONST || ln[q].op != MG_CONST) return -1;
        const U k = ln[b].imm;
        if (ln[p].imm == k && ln[q].imm == k) return zero;
        if (ln[p].imm == k) return not_(c);
        if (ln[q].imm == k) return c;
        return one;
    }

    template <class V> static bool contains(const V& v, int x) { return std::find(v.begin(), v.end(), x) != v.end(); }

    // atoms of a rewritten root, kept across passes and branches: a rewrite
    // result holds no defined leaf, so neither do the parts split from it,
    // and the walk below is a function of that node alone (its splits,
    // folds and intervals are structural; nodes it builds are hash-consed,
    // so a repeated walk would build nothing new)
    struct AtomsOf { Chunks out; bool unsat; };
    std::unordered_map<int, AtomsOf> atoms_of_;
    OverlayTable overlay_table_;

    Chunks atoms(int root, Memo& memo) {
        const int r0 = rewrite(root, memo);
        auto hit = atoms_of_.find(r0);
        if (hit != atoms_of_.end()) {
            unsat |= hit->second.unsat;
            return hit->second.out;
        }
        const bool unsat_in = unsat;
        unsat = false;
        Chunks out = atoms_walk(r0, memo);
        atoms_of_.emplace(r0, AtomsOf{out, unsat});
        unsat |= unsat_in;
        return out;
    }

    Chunks atoms_walk(int r0, Memo& memo) {
        Chunks out;
        Chunks stack{r0};
        const int g = new_stamp();
        while (!stack.empty()) {
            int x = stack.back();
            stack.pop_back();
            if (stamped(x, g)) continue;
            const int op = ln[x].op;
            if (op == MG_CONST) {
                if (!(ln[x].imm.w[0] & 1)) unsat = true;
                continue;
            }
            if (op == MG_AND && ln[x].width == 1) {
                for (int a : ln[x].args) stack.push_back(a);
                continue;
            }
            if (op == MG_NOT && ln[x].width == 1) {
                int y = ln[x].args[0];
                if (ln[y].op == MG_OR && ln[y].width == 1) {
                    Args ya = ln[y].args;
                    for (int a : ya) stack.push_back(not_(a));
                    continue;
                }
                if (ln[y].op == MG_EQ) {
                    int r = neg_eq(y);
                    if (r >= 0) { stack.push_back(r); continue; }
                }
                bool ord = is_order(ln[y].op);
                if (!ord) out.push_back(x);
                if (!ord && ln[y].op == MG_UMULNO && ln[ln[y].args[1]].op != MG_CONST) {
                    int b_ = ln[y].args[1];
                    int w_ = ln[y].width;
                    int e1 = eq_(b_, mask(ln[b_].width));
                    int e2 = eq_(b_, U1(w_ - 1));
                    int o = lw.mk(MG_OR, 1, {e1, e2});
                    stack.push_back(rewrite(o, memo));
                }
                if (!ord) continue;
            }
            if (op == MG_EQ) {
                Chunks parts;
                if (split_eq(x, parts)) {
                    for (int p : parts) stack.push_back(rewrite(p, memo));
                    continue;
                }
            }
            if (op == MG_ULT && ln[ln[x].args[0]].op == MG_ADD && contains(ln[ln[x].args[0]].args, ln[x].args[1])) {
                int s_ = ln[x].args[0], a_ = ln[x].args[1];
                int other = ln[s_].args[0] == a_ ? ln[s_].args[1] : ln[s_].args[0];
                out.push_back(x);
                if (ln[other].op != MG_CONST) {
                    int e = eq_(other, mask(ln[other].width));
                    stack.push_back(rewrite(e, memo));
                }
                continue;
            }
            if (op == MG_OR && ln[x].width == 1) {
                int le = as_ule(x);
                if (le >= 0) { stack.push_back(le); continue; }
            }
            Bound b;
            bool hb = bound(x, b);
            if (hb && (ln[b.e].op == MG_ITE || ln[b.e].op == MG_CONCAT || ln[b.e].op == MG_MUL)) {
                Chunks parts;
                if (split_bound(b.e, b.lo, b.hi, b.w, parts)) {
                    if (ln[b.e].op != MG_ITE) out.push_back(x);
                    for (int p : parts) stack.push_back(rewrite(p, memo));
                    continue;
                }
            }
            if (!hb) {
                Chunks parts;
                if (order_via_arm(x, parts)) {
                    out.push_back(x);
                    for (int p : parts) stack.push_back(rewrite(p, memo));
                    continue;
                }
            }
            out.push_back(x);
        }
        return out;
    }

    bool order_via_arm(int x, Chunks& out) {
        bool neg = ln[x].op == MG_NOT && ln[x].width == 1;
        int y = neg ? ln[x].args[0] : x;
        if (ln[y].op != MG_ULT && ln[y].op != MG_ULE) return false;
        int a = ln[y].args[0], s = ln[y].args[1];
        bool strict = ln[y].op == MG_ULT;
        if (neg) { std::swap(a, s); strict = !strict; }
        if (ln[s].op != MG_ITE) return false;
        U k;
        Chunks conds;
        if (!max_arm(s, k, conds)) return false;
        if (strict && k.zero()) return false;        // hi < 0
        U hi = strict ? k - U::of(1) : k;
        out = conds;
        Chunks mb = mk_bound(a, U(), hi, ln[y].width);
        out.insert(out.end(), mb.begin(), mb.end());
        return true;
    }

    bool max_arm(int s, U& best_k, Chunks& best_conds, int depth_ = 8) {
        bool have = false;
        struct It { int n; Chunks conds; int d; };
        std::vector<It> stack{{s, {}, 0}};
        while (!stack.empty()) {
            It it = std::move(stack.back());
            stack.pop_back();
            if (ln[it.n].op == MG_CONST) {
                if (!have || ln[it.n].imm > best_k) { best_k = ln[it.n].imm; best_conds = it.conds; have = true; }
            } else if (ln[it.n].op == MG_ITE && it.d < depth_) {
                int c = ln[it.n].args[0];
                Chunks c1 = it.conds; c1.push_back(c);
                int a1 = ln[it.n].args[1], a2 = ln[it.n].args[2];
                stack.push_back({a1, c1, it.d + 1});
                Chunks c2 = it.conds; c2.push_back(not_(c));
                stack.push_back({a2, c2, it.d + 1});
            }
        }
        return have;
    }

    int as_ule(int x) {
        if (ln[x].args.size() != 2) throw std::runtime_error("or with more than two operands");
        int p = ln[x].args[0], q = ln[x].args[1];
        int pairs[2][2] = {{p, q}, {q, p}};
        for (auto& pr : pairs) {
            int lt = pr[0], e = pr[1];
            if (ln[lt].op == MG_ULT && ln[e].op == MG_EQ) {
                int e0 = ln[e].args[0], e1 = ln[e].args[1];
                int l0 = ln[lt].args[0], l1 = ln[lt].args[1];
                bool same = (e0 == l0 || e0 == l1) && (e1 == l0 || e1 == l1) &&
                            (l0 == e0 || l0 == e1) && (l1 == e0 || l1 == e1);
                if (same) return lw.mk(MG_ULE, ln[lt].width, ln[lt].args);
            }
        }
        return -1;
    }

    // -- bounds ---------------------------------------------------------------------
    bool bound(int x, Bound& out) {
        bool neg = false;
        if (ln[x].op == MG_NOT && ln[x].width == 1) { x = ln[x].args[0]; neg = true; }
        int op = ln[x].op;
        if (!is_order(op)) return false;
        int a = ln[x].args[0], b = ln[x].args[1];
        int w = ln[x].width;
        U top = mask(w);
        bool strict = op == MG_ULT || op == MG_SLT;
        bool ac = ln[a].op == MG_CONST, bc = ln[b].op == MG_CONST;
        if (op == MG_SLT || op == MG_SLE) {
            if (neg) return false;
            top = mask(w - 1);
            if (!bc && !ac) return false;
            U k = bc ? ln[b].imm : ln[a].imm;
            if (k > top || ac == bc) return false;
        }
        if (bc && !ac) {
            U k = ln[b].imm;
            if (!neg) {
                if (!(nz(k) || !strict)) return false;
                out = {a, U(), strict ? k - U::of(1) : k, w};
                return true;
            }
            if (!(k < top || strict)) return false;
            out = {a, strict ? k : k + U::of(1), top, w};
            return true;
        }
        if (ac && !bc) {
            U k = ln[a].imm;
            if (!neg) {
                if (!(k < top || !strict)) return false;
                out = {b, strict ? k + U::of(1) : k, top, w};
                return true;
            }
            if (!(nz(k) || strict)) return false;
            out = {b, U(), strict ? k : k - U::of(1), w};
            return true;
        }
        return false;
    }

    Chunks mk_bound(int e, const U& lo, const U& hi, int w) {
        Chunks out;
        if (lo > hi) return {zero};
        if (nz(lo)) { int c = lw.cnst(lo, w); out.push_back(lw.mk(MG_ULE, w, {c, e})); }
        if (hi < mask(w)) { int c = lw.cnst(hi, w); out.push_back(lw.mk(MG_ULE, w, {e, c})); }
        return out;
    }

    static void append(Chunks& a, const Chunks& b) { a.insert(a.end(), b.begin(), b.end()); }

    bool split_ite_bound(int e, const U& lo, const U& hi, int w, Chunks& out) {
        int c = ln[e].args[0], p = ln[e].args[1], q = ln[e].args[2];
        bool pc = ln[p].op == MG_CONST, qc = ln[q].op == MG_CONST;
        if (pc && !qc) {
            bool inside = lo <= ln[p].imm && ln[p].imm <= hi;
            out = mk_bound(q, lo, hi, w);
            if (!inside) out.push_back(not_(c));
            return true;
        }
        if (qc && !pc) {
            bool inside = lo <= ln[q].imm && ln[q].imm <= hi;
            out = mk_bound(p, lo, hi, w);
            if (!inside) out.push_back(c);
            return true;
        }
        if (!pc && !qc) {
            out = mk_bound(p, lo, hi, w);
            append(out, mk_bound(q, lo, hi, w));
            return true;
        }
        return false;
    }

    bool split_bound(int e, const U& lo, const U& hi, int w, Chunks& out) {
        if (ln[e].op == MG_ITE) return split_ite_bound(e, lo, hi, w, out);
        if (ln[e].op == MG_CONCAT) {
            out.clear();
            while (ln[e].op == MG_CONCAT) {
                int lw_ = (int)ln[e].imm.w[0];
                if (nz(shr(hi, lw_))) break;
                int h = hi_part(e);
                out.push_back(eq_(h, U()));
                e = ln[e].args[1];
            }
            if (ln[e].op != MG_CONCAT) { append(out, mk_bound(e, lo, hi, ln[e].width)); return true; }
            if (nz(lo)) return !out.empty();
            int lw_ = (int)ln[e].imm.w[0];
            int h = hi_part(e);
            append(out, mk_bound(h, U(), shr(hi, lw_) - U::of(1), ln[h].width));
            return true;
        }
        if (nz(lo)) return false;
        if (ln[e].op == MG_MUL) {
            int k = (hi + U::of(1)).bitlen() - 1;
            int a = ln[e].args[0], b = ln[e].args[1];
            out = mk_bound(a, U(), U1(k / 2) - U::of(1), w);
            append(out, mk_bound(b, U(), U1(k - k / 2) - U::of(1), w));
            return true;
        }
        return false;
    }

    // -- definitions ------------------------------------------------------------------
    bool depends(int e, int leaf) {
        const int g = new_stamp();
        Chunks stack{e};
        while (!stack.empty()) {
            int x = stack.back();
            stack.pop_back();
            if (x == leaf) return true;
            if (stamped(x, g)) continue;
            if (ln[x].op == MG_LEAF) {
                const int* d = repl_find(x);
                if (d) stack.push_back(*d);
                continue;
            }
            for (int a : ln[x].args) stack.push_back(a);
        }
        return false;
    }

    bool try_define(int leaf, int e) {
        if (ln[leaf].op != MG_LEAF || repl_find(leaf)) return false;
        if (selectors.count(leaf) && ln[e].op != MG_CONST) return false;
        if (!refused.empty() && refused.count(key(leaf))) return false;
        if (ln[e].width > ln[leaf].width && !(ln[e].op == MG_CONST && shr(ln[e].imm, ln[leaf].width).zero()))
            return false;
        if (depends(e, leaf)) return false;
        repl_put(leaf, e);
        if (wrap_ctx) wrap_defs.insert(leaf);
        leaf_imm[leaf] = (int)ln[leaf].imm.w[0];
        leaf_node[leaf] = leaf;
        if (dm_valid) dm.set(leaf_imm[leaf]);   // the mask only grows here
        return true;
    }

    Chunks ite_leaves(int x, size_t limit = 16) {
        Chunks out, stack;
        if (ln[x].op == MG_ITE) stack.push_back(x);
        while (!stack.empty() && out.size() < limit) {
            int y = stack.back();
            stack.pop_back();
            for (int arm : {ln[y].args[1], ln[y].args[2]}) {
                if (ln[arm].op == MG_LEAF) out.push_back(arm);
                else if (ln[arm].op == MG_ITE) stack.push_back(arm);
            }
        }
        return out;
    }

    bool domain(int x) {
        Chunks disj, stack{x};
        while (!stack.empty()) {
            int y = stack.back();
            stack.pop_back();
            if (ln[y].op == MG_OR && ln[y].width == 1) for (int a : ln[y].args) stack.push_back(a);
            else disj.push_back(y);
        }
        if ((int)disj.size() > MAX_DOMAIN) return false;
        int leaf = -1;
        std::vector<U> ks;
        for (int d : disj) {
            if (ln[d].op != MG_EQ) return false;
            int a = ln[d].args[0], b = ln[d].args[1];
            if (ln[a].op == MG_CONST) std::swap(a, b);
            if (ln[a].op != MG_LEAF || ln[b].op != MG_CONST || (leaf >= 0 && a != leaf)) return false;
            leaf = a;
            bool have = false;
            for (auto& k : ks) if (k == ln[b].imm) { have = true; break; }
            if (!have) ks.push_back(ln[b].imm);
        }
        if (leaf < 0 || repl.has(leaf)) return false;
        int sel = selector();
        int span = 1 << SELECTOR_WIDTH;
        int lw_ = ln[leaf].width;
        int e = lw.cnst(ks.back(), lw_);
        for (int i = (int)ks.size() - 2; i >= 0; i--) {
            int t = lw.cnst((uint64_t)(span * (i + 1) / (int)ks.size()), SELECTOR_WIDTH);
            int u = lw.mk(MG_ULT, SELECTOR_WIDTH, {sel, t});
            int k = lw.cnst(ks[i], lw_);
            e = lw.mk(MG_ITE, lw_, {u, k, e});
        }
        return try_define(leaf, e);
    }

    int selector() {
        int sel = aux(SELECTOR_WIDTH);
        selectors.insert(sel);
        return sel;
    }
    int aux(int width) {
        n_aux++;
        int leaf = lw.leaf("aux#" + std::to_string(n_aux), width, K_AUX, "");
        aux_seq.emplace(leaf, (int)aux_seq.size());
        return leaf;
    }
    int key(int leaf) const {
        auto it = aux_seq.find(leaf);
        return it == aux_seq.end() ? leaf : -1 - it->second;
    }

    int define(const Chunks& atoms_) {
        int n = 0;
        for (int x : atoms_) {
            if (ln[x].op == MG_EQ) {
                int p = ln[x].args[0], q = ln[x].args[1];
                bool done = false;
                int pairs[2][2] = {{p, q}, {q, p}};
                for (auto& pr : pairs)
                    if (ln[pr[0]].op == MG_LEAF && try_define(pr[0], pr[1])) { done = true; break; }
                if (!done) {
                    for (auto& pr : pairs) {
                        for (int arm : ite_leaves(pr[0]))
                            if (try_define(arm, pr[1])) { done = true; break; }
                        if (done) break;
                    }
                }
                n += done;
            } else if (ln[x].op == MG_OR && ln[x].width == 1 && !or_seen.count(x)) {
                or_seen.insert(x);
                int d = domain(x) ? 1 : 0;
                n += d ? d : branches(x);
            }
        }
        return n;
    }

    int ranges(const Chunks& atoms_) {
        struct Info { int e; U lo, hi; int j; U res; };
        OMap<int, Info> info;
        for (int x : atoms_) {
            Bound b;
            if (bound(x, b) && ln[b.e].op == MG_LEAF) {
                Info& r = info.setdefault(b.e, Info{b.e, U(), mask(ln[b.e].width), 0, U()});
                r.lo = umax(r.lo, b.lo);
                r.hi = umin(r.hi, b.hi);
            } else if (ln[x].op == MG_EQ) {
                int a = ln[x].args[0], k = ln[x].args[1];
                if (ln[a].op == MG_CONST) std::swap(a, k);
                if (ln[a].op == MG_EXTRACT && ln[a].imm.zero() && ln[ln[a].args[0]].op == MG_LEAF &&
                    ln[k].op == MG_CONST) {
                    int leaf = ln[a].args[0];
                    Info& r = info.setdefault(leaf, Info{leaf, U(), mask(ln[leaf].width), 0, U()});
                    if (ln[a].width > r.j) { r.j = ln[a].width; r.res = ln[k].imm; }
                }
            }
        }
        int n = 0;
        for (auto& kv : info.items) {
            Info r = kv.second;
            int leaf = r.e;
            int lwid = ln[leaf].width;
            if (repl.has(leaf) || r.lo > r.hi || (!r.j && r.lo.zero() && r.hi == mask(lwid))) continue;
            U base = shl(shr(r.lo, r.j), r.j) | r.res;
            if (base < r.lo) base = base + U1(r.j);
            if (base > r.hi) continue;
            U room = shr(r.hi - base, r.j) + U::of(1);
            int a = selectors.count(leaf) ? 0 : room.bitlen() - 1;
            int e = lw.cnst(base, lwid);
            if (a > 0) {
                int ax = aux(a);
                int step = ax;
                if (r.j) { int z = lw.cnst(0, r.j); step = lw.mki(MG_CONCAT, a + r.j, {ax, z}, r.j); }
                e = nz(base) ? lw.mk(MG_ADD, lwid, {e, step}) : step;
            }
            n += try_define(leaf, e);
        }
        return n;
    }

    int branches(int x) {
        Chunks disj, stack{x};
        while (!stack.empty()) {
            int y = stack.back();
            stack.pop_back();
            if (ln[y].op == MG_OR && ln[y].width == 1) {
                const Args& ya = ln[y].args;
                for (size_t i = ya.size(); i-- > 0;) stack.push_back(ya[i]);
            } else {
                disj.push_back(y);
            }
        }
        if ((int)disj.size() > MAX_BRANCHES || n_branch >= MAX_OR) return 0;
        // definitions only append to repl: the state before the disjuncts
        // is its length, and rolling back truncates (solve.py copies the dict)
        const size_t saved = repl.size();
        bool unsat_saved = unsat;
        std::vector<OMap<int, int>> per;
        for (int d : disj) {
            unsat = false;
            Memo overlay;
            overlay.overlay_on(run_memo, &overlay_table_);
            Chunks at = atoms(d, overlay);
            if (unsat) { per.emplace_back(); continue; }
            define(at);
            ranges(at);
            OMap<int, int> defs;
            for (size_t i = saved; i < repl.items.size(); i++) defs.put(repl.items[i].first, repl.items[i].second);
            per.push_back(std::move(defs));
            repl_truncate(saved);
            dm_valid = false;
        }
        unsat = unsat_saved;
        OMap<int, char> leaves;
        for (auto& defs : per) for (auto& kv : defs.items) leaves.setdefault(kv.first, 0);
        if (!leaves.size()) return 0;
        n_branch++;
        int sel = selector();
        int span = 1 << SELECTOR_WIDTH;
        int n = 0;
        for (auto& lk : leaves.items) {
            int k = lk.first;
            int leaf = leaf_node[k];
            auto dit = depth.find(k);
            int d = dit == depth.end() ? 0 : dit->second;
            if (d >= BRANCH_DEPTH) continue;
            int free_ = -1;
            Chunks arms;
            for (auto& defs : per) {
                const int* e = defs.find(k);
                int ev;
                if (!e) {
                    if (free_ < 0) { free_ = aux(ln[leaf].width); depth[free_] = d + 1; }
                    ev = free_;
                } else {
                    ev = *e;
                }
                arms.push_back(ev);
            }
            int e = arms.back();
            for (int i = (int)arms.size() - 2; i >= 0; i--) {
                int t = lw.cnst((uint64_t)(span * (i + 1) / (int)arms.size()), SELECTOR_WIDTH);
                int u = lw.mk(MG_ULT, SELECTOR_WIDTH, {sel, t});
                e = lw.mk(MG_ITE, ln[leaf].width, {u, arms[i], e});
            }
            n += try_define(leaf, e);
        }
        return n;
    }

    bool reads_own(int y, const std::string& name) {
        bool own = false, bad = false;
        DepRow d = depof(y);
        d.each([&](int li) {
            if (bad) return;
            const Leaf& leaf = lw.leaves[li];
            if (leaf.source == name) own = true;
            else {
                const std::string suf = "calldatasize";
                const std::string& nm = leaf.name;
                if (!(nm.size() >= suf.size() && nm.compare(nm.size() - suf.size(), suf.size(), suf) == 0))
                    bad = true;
            }
        });
        return bad ? false : own;
    }

    Chunks abi_offsets() {
        Chunks out;
        for (auto& te : lw.arg_entries.items) {
            const std::string& name = te.first;
            auto& ents = te.second;
            const std::vector<Big>* ck = lw.table_ckeys.find(name);
            if (!ck || ck->empty() || ents[0].first.size() != 1) continue;
            struct Span { int y; U lo, hi; };
            OMap<int, Span> spans;
            Memo memo;
            for (auto& kvp : ents) {
                int k = rewrite(kvp.first[0], memo);
                int y = k;
                U c;
                if (ln[k].op == MG_ADD && ln[ln[k].args[1]].op == MG_CONST) { y = ln[k].args[0]; c = ln[ln[k].args[1]].imm; }
                if (ln[y].op == MG_CONST || nz(shr(c, 32)) || !reads_own(y, name)) continue;
                Span& r = spans.setdefault(y, Span{y, c, c});
                r.lo = umin(r.lo, c);
                r.hi = umax(r.hi, c);
            }
            Big mx = *std::max_element(ck->begin(), ck->end());
            U nxt = mx.low384() + U::of(1);
            for (auto& sp : spans.items) {
                const Span& s = sp.second;
                U diff = nxt - s.lo;
                U base = shl(sar(diff + U::of(31), 5), 5);     // ceil((nxt - lo) / 32) * 32
                int c = lw.cnst(base, ln[s.y].width);
                out.push_back(lw.mk(MG_EQ, ln[s.y].width, {s.y, c}));
                nxt = base + s.hi + U::of(1);
            }
        }
        return out;
    }

    Chunks joint_bounds(const Chunks& atoms_) {
        struct G { int e; U lo, hi; int w, k; };
        OMap<int, G> groups;
        for (int a : atoms_) {
            Bound b;
            if (!bound(a, b) || ln[b.e].op == MG_LEAF || ln[b.e].op == MG_CONST) continue;
            G& g = groups.setdefault(b.e, G{b.e, U(), mask(b.w), b.w, 0});
            g.lo = umax(g.lo, b.lo);
            g.hi = umin(g.hi, b.hi);
            g.k++;
        }
        Chunks parts;
        for (auto& kv : groups.items) {
            const G& g = kv.second;
            std::string key = std::to_string(g.e) + ":" + hex(g.lo) + ":" + hex(g.hi);
            if (g.k >= 2 && g.lo <= g.hi && !joint_done.count(key)) {
                joint_done.insert(key);
                int eop = ln[g.e].op;
                Chunks sp;
                bool ok = (eop == MG_CONCAT || eop == MG_ITE || eop == MG_MUL) && split_bound(g.e, g.lo, g.hi, g.w, sp);
                append(parts, ok ? sp : mk_bound(g.e, g.lo, g.hi, g.w));
            }
        }
        return parts;
    }

    bool is_wrap_test(int r) {
        int x = r;
        while (ln[x].op == MG_AND && ln[x].width == 1 && ln[x].args.size() == 2 && ln[ln[x].args[0]].op == MG_CONST)
            x = ln[x].args[1];
        if (ln[x].op == MG_NOT && ln[x].width == 1 && ln[ln[x].args[0]].op == MG_UMULNO) return true;
        return ln[x].op == MG_ULT && ln[ln[x].args[0]].op == MG_ADD && contains(ln[ln[x].args[0]].args, ln[x].args[1]);
    }

    // the definition (index into the insertion-ordered definitions) that
    // completes root r's folding to false: the shortest prefix under which
    // it folds to false ends with it; -1 when r is false with none
    // (solve.Solver._culprit)
    int culprit(int r) {
        const std::vector<std::pair<int, int>> items = repl.items;
        auto set_prefix = [&](size_t m) {
            repl_truncate(0);
            for (size_t i = 0; i < m; i++) repl_put(items[i].first, items[i].second);
            dm_valid = false;
        };
        auto false_under = [&](size_t m) {
            set_prefix(m);
            Memo fresh;
            int x = rewrite(r, fresh);
            return ln[x].op == MG_CONST && !(ln[x].imm.w[0] & 1);
        };
        int res;
        if (false_under(0)) {
            res = -1;
        } else {
            size_t lo = 0, hi = items.size();   // false_under(hi) holds
            while (hi - lo > 1) {
                size_t mid = (lo + hi) / 2;
                if (false_under(mid)) hi = mid;
                else lo = mid;
            }
            res = (int)hi - 1;
        }
        set_prefix(items.size());
        return res;
    }

    void run(Chunks& roots, std::vector<std::pair<int, int>>& defs_out) {
        int64_t saved_birth = lw.birth;
        lw.birth = 0;
        Chunks pins = abi_offsets();
        if (!pins.empty()) {
            int root = pins.size() > 1 ? lw.mk(MG_AND, 1, pins) : pins[0];
            Memo m;
            define(atoms(root, m));
        }
        Chunks order;
        for (int r : roots) if (is_wrap_test(r)) order.push_back(r);
        for (int r : roots) if (!is_wrap_test(r)) order.push_back(r);
        const std::vector<std::pair<int, int>> base = repl.items;
        Memo memo;
        for (int attempt = 0; attempt <= MAX_REFUSALS; attempt++) {
            int at_pass = -1;
            const int d = passes(order, memo, at_pass);
            if (d < 0) break;
            // a root folded to false under the construction: completed by
            // an overflow test's definition or in the first pass, the
            // query's own conditions meeting (the group needs no program
            // beyond that root, model._ground_value); otherwise heuristic
            // commits conflicting: refuse the definition that completed it
            // and construct again, up to MAX_REFUSALS times
            // (solve.Solver.run)
            int k = at_pass > 0 && attempt < MAX_REFUSALS ? culprit(d) : -1;
            if (k >= 0 && wrap_defs.count(repl.items[k].first)) k = -1;  // the check's own choice
            if (k < 0) {
                dead = true;
                roots = {rewrite(d, memo)};
                defs_out.clear();
                lw.birth = saved_birth;
                run_memo = &base_memo;
                return;
            }
            refused.insert(key(repl.items[k].first));
            repl_truncate(0);
            for (auto& kv : base) repl_put(kv.first, kv.second);
            dm_valid = false;
            or_seen.clear();
            joint_done.clear();
            n_branch = 0;
            aux_seq.clear();
            wrap_defs.clear();
            depth.clear();
        }
        for (auto& r : roots) r = rewrite(r, memo);
        defs_out.clear();
        for (auto& kv : repl.items) {
            int li = (int)ln[leaf_node[kv.first]].imm.w[0];
            int e = rewrite(kv.second, memo);
            defs_out.push_back({li, e});
        }
        lw.birth = saved_birth;
        run_memo = &base_memo;
    }

    // the definition passes over a fresh memo; the first root that folds to
    // false (and the pass it folded in), or -1 (solve.Solver._passes)
    int passes(const Chunks& order, Memo& memo, int& at_pass) {
        memo.dense.clear();
        run_memo = &memo;
        for (int pass = 0; pass < PASSES; pass++) {
            int found = 0;
            Chunks every;
            for (int r : order) {
                wrap_ctx = is_wrap_test(r);
                Chunks at = atoms(r, memo);
                const int rr = rewrite(r, memo);
                if (ln[rr].op == MG_CONST && !(ln[rr].imm.w[0] & 1)) {
                    wrap_ctx = false;
                    at_pass = pass;
                    return r;
                }
                append(every, at);
                found += define(at);
            }
            wrap_ctx = false;
            if (found) for (auto& a : every) a = rewrite(a, memo);
            Chunks extra;
            for (int part : joint_bounds(every)) append(extra, atoms(part, memo));
            if (!extra.empty()) {
                found += define(extra);
                append(every, extra);
            }
            found += ranges(every);
            if (!found) break;
        }
        return -1;
    }
};

// ---------------------------------------------------------------------------
// scheduling, register allocation, pools (ir._schedule / _fuse_roots /
// _allocate / _leaf_pools)
// ---------------------------------------------------------------------------
static std::vector<int> schedule(const std::vector<LN>& ln, const Chunks& sinks) {
    std::vector<char> seen(ln.size(), 0);
    std::vector<int> out;
    std::vector<int> stack(sinks.begin(), sinks.end());
    while (!stack.empty()) {
        int n = stack.back();
        stack.pop_back();
        if (seen[n]) continue;
        seen[n] = 1;
        out.push_back(n);
        for (int a : ln[n].args) if (!seen[a]) stack.push_back(a);
    }
    std::sort(out.begin(), out.end(), [&](int a, int b) {
        if (ln[a].birth != ln[b].birth) return ln[a].birth < ln[b].birth;
        return a < b;
    });
    std::vector<int> lazy;
    std::vector<char> placed(ln.size(), 0);
    for (int n : out) {
        if (ln[n].op == MG_LEAF) continue;
        for (int a : ln[n].args)
            if (ln[a].op == MG_LEAF && !placed[a]) { placed[a] = 1; lazy.push_back(a); }
        lazy.push_back(n);
    }
    for (int n : out) if (ln[n].op == MG_LEAF && !placed[n]) lazy.push_back(n);
    return lazy;
}

// ir._schedule_demand: the sinks in (birth, id) order, each sink's operands
// not yet scheduled in post-order (a value right before its first consumer)
static std::vector<int> schedule_demand(const std::vector<LN>& ln, const Chunks& sinks) {
    std::vector<int> ss(sinks.begin(), sinks.end());
    std::sort(ss.begin(), ss.end(), [&](int a, int b) {
        if (ln[a].birth != ln[b].birth) return ln[a].birth < ln[b].birth;
        return a < b;
    });
    std::vector<char> seen(ln.size(), 0);
    std::vector<int> out;
    std::vector<std::pair<int, bool>> stack;
    for (int s : ss) {
        stack.push_back({s, false});
        while (!stack.empty()) {
            auto [n, done] = stack.back();
            stack.pop_back();
            if (done) { out.push_back(n); continue; }
            if (seen[n]) continue;
            seen[n] = 1;
            stack.push_back({n, true});
            const auto& args = ln[n].args;
            for (size_t k = args.size(); k-- > 0;)
                if (!seen[args[k]]) stack.push_back({args[k], false});
        }
    }
    return out;
}

static std::vector<int> fuse_roots(const std::vector<LN>& ln, const std::vector<int>& order,
                                   std::unordered_set<int>& fused) {
    std::vector<int> out;
    for (int n : order) {
        if (ln[n].op == MG_ROOT && !out.empty() && out.back() == ln[n].args[0] && !fused.count(ln[n].args[0])) {
            fused.insert(ln[n].args[0]);
            continue;
        }
        out.push_back(n);
    }
    return out;
}

struct Ins { uint32_t op, width, d, a, b, c, imm, flags; };

struct UHash {
    size_t operator()(const U& u) const {
        uint64_t h = 1469598103934665603ull;
        for (int i = 0; i < U::N; i++) h = (h ^ u.w[i]) * 1099511628211ull;
        return (size_t)h;
    }
};

struct Alloc {
    const std::vector<LN>& ln;
    const std::vector<int>& order;
    const std::unordered_map<U, int, UHash>& const_index;
    const std::unordered_set<int>& fused;
    int nreg, trash;
    int remat_mode, remat_k;
    bool keep_clean;
    // per LNode id: its uses (positions in order, CSR), the scan pointer
    // into them, its register / spill slot (-1: none)
    std::vector<int> use_off, use_pos, ptr, reg_of, lds_of;
    bool has_reg(int v) const { return reg_of[v] >= 0; }
    bool has_lds(int v) const { return lds_of[v] >= 0; }
    std::vector<std::pair<int, int>> holder;          // (reg, value), insertion order
    std::vector<int> free_regs;
    std::unordered_map<int, bool> reg_clean;
    std::vector<int> free_lds;
    int n_lds = 0, n_spill = 0, n_reload = 0;
    std::vector<Ins> ins;
    static const int64_t FAR = 1ll << 60;

    Alloc(const std::vector<LN>& l, const std::vector<int>& o, const std::unordered_map<U, int, UHash>& ci,
          const std::unordered_set<int>& f, int nr, int rm, int rk, bool kc)
        : ln(l), order(o), const_index(ci), fused(f), nreg(nr), trash(nr - 1), remat_mode(rm), remat_k(rk),
          keep_clean(kc) {}

    int64_t next_use(int v, int64_t i) {
        int b = use_off[v], e = use_off[v + 1];
        int& p = ptr[v];
        while (b + p < e && use_pos[b + p] < i) p++;
        return b + p < e ? use_pos[b + p] : FAR;
    }
    bool free_to_drop(int v) const { return ln[v].op == MG_CONST || has_lds(v); }
    bool droppable_when_full(int v) const { return free_to_drop(v) || ln[v].op == MG_LEAF; }
    bool clean_of(int r) const { auto it = reg_clean.find(r); return it != reg_clean.end() && it->second; }
    void holder_del(int r) {
        for (size_t i = 0; i < holder.size(); i++) if (holder[i].first == r) { holder.erase(holder.begin() + i); return; }
    }
    static bool in(const std::vector<int>& v, int x) { return std::find(v.begin(), v.end(), x) != v.end(); }
    static void remove(std::vector<int>& v, int x) { v.erase(std::find(v.begin(), v.end(), x)); }

    static bool protects(const Args& p, int v) { for (int a : p) if (a == v) return true; return false; }
    int alloc_reg(int i, const Args& protect, bool oldest = false) {
        if (!free_regs.empty()) {
            int r;
            if (oldest) { r = free_regs.front(); free_regs.erase(free_regs.begin()); }
            else { r = free_regs.back(); free_regs.pop_back(); }
            return r;
        }
        int victim = -1;
        int64_t far = -1;
        for (auto& hv : holder) {
            int v = hv.second;
            if (protects(protect, v)) continue;
            int64_t nu = next_use(v, i);
            if (nu > far) { victim = v; far = nu; }
        }
        if (victim < 0) throw Unsupported("register pressure");
        if (!free_to_drop(victim) && free_lds.empty() && n_lds >= MAX_SPILL) {
            victim = -1; far = -1;
            for (auto& hv : holder) {
                int v = hv.second;
                if (protects(protect, v) || !droppable_when_full(v)) continue;
                int64_t nu = next_use(v, i);
                if (nu > far) { victim = v; far = nu; }
            }
            if (victim < 0) throw Unsupported("spill budget exceeded");
        }
        int r = reg_of[victim];
        reg_of[victim] = -1;
        holder_del(r);
        bool slots_left = !free_lds.empty() || n_lds < MAX_SPILL;
        if (ln[victim].op == MG_LEAF && !has_lds(victim) && remat_mode != MGC_REMAT_SPILL) {
            int tier = LDS_TIER + (remat_mode == MGC_REMAT_SCRATCH ? remat_k : 0);
            bool cheap_free = (!free_lds.empty() && *std::min_element(free_lds.begin(), free_lds.end()) < tier) ||
                              n_lds < tier;
            if (remat_mode == MGC_REMAT_ALWAYS || !cheap_free) slots_left = false;
        }
        if (!free_to_drop(victim) && slots_left) {
            int s;
            if (!free_lds.empty()) {
                s = *std::min_element(free_lds.begin(), free_lds.end());
                remove(free_lds, s);
            } else {
                s = n_lds++;
            }
            lds_of[victim] = s;
            ins.push_back({MG_SPILL, 1, (uint32_t)trash, (uint32_t)r, 0, 0, (uint32_t)s, 0});
            n_spill++;
        }
        return r;
    }

    void materialise(int v, int r) {
        reg_clean[r] = ln[v].width <= 32;
        if (ln[v].op == MG_CONST) {
            ins.push_back({MG_CONST, (uint32_t)ln[v].width, (uint32_t)r, 0, 0, 0, (uint32_t)const_index.at(ln[v].imm), 0});
        } else if (has_lds(v)) {
            ins.push_back({MG_RELOAD, (uint32_t)ln[v].width, (uint32_t)r, 0, 0, 0, (uint32_t)lds_of[v], 0});
            n_reload++;
        } else {
            ins.push_back({MG_LEAF, (uint32_t)ln[v].width, (uint32_t)r, 0, 0, 0, (uint32_t)ln[v].imm.w[0], 0});
        }
    }

    void release(int v, int i) {
        if (next_use(v, i + 1) >= FAR) {
            if (has_reg(v)) {
                int r = reg_of[v];
                reg_of[v] = -1;
                holder_del(r);
                free_regs.push_back(r);
            }
            if (has_lds(v)) {
                int s = lds_of[v];
                lds_of[v] = -1;
                free_lds.push_back(s);
            }
        }
    }

    void run() {
        size_t nn = ln.size();
        use_off.assign(nn + 1, 0);
        ptr.assign(nn, 0);
        reg_of.assign(nn, -1);
        lds_of.assign(nn, -1);
        for (size_t i = 0; i < order.size(); i++)
            for (int a : ln[order[i]].args) use_off[a + 1]++;
        for (size_t v = 0; v < nn; v++) use_off[v + 1] += use_off[v];
        use_pos.assign(use_off[nn], 0);
        {
            std::vector<int> fill(use_off.begin(), use_off.end() - 1);
            for (size_t i = 0; i < order.size(); i++)
                for (int a : ln[order[i]].args) use_pos[fill[a]++] = (int)i;
        }
        for (int r = nreg - 1; r >= 0; r--) free_regs.push_back(r);
        for (size_t ii = 0; ii < order.size(); ii++) {
            int i = (int)ii;
            int n = order[ii];
            const LN& N = ln[n];
            const Args& protect = N.args;
            for (int a : N.args) {
                if (!has_reg(a)) {
                    int r = alloc_reg(i, protect, ln[a].op != MG_CONST);
                    materialise(a, r);
                    reg_of[a] = r;
                    holder.push_back({r, a});
                }
            }
            Args slots = N.args;
            for (int& a : slots) a = reg_of[a];
            for (size_t k = 0; k < N.args.size(); k++) {
                int a = N.args[k];
                bool seen = false;
                for (size_t j = 0; j < k; j++) if (N.args[j] == a) { seen = true; break; }
                if (!seen) release(a, i);
            }
            if (N.op == MG_ROOT || N.op == MG_OUT) {
                ins.push_back({(uint32_t)N.op, 1, (uint32_t)trash, (uint32_t)slots[0], 0, 0,
                               N.has_imm ? (uint32_t)N.imm.w[0] : 0u, 0});
                continue;
            }
            uint32_t flags = fused.count(n) ? (uint32_t)MG_ROOT_FLAG : 0u;
            int d = -1;
            if (use_off[n] == use_off[n + 1]) {
                if (!free_regs.empty()) {
                    d = free_regs.back();
                } else {
                    d = alloc_reg(i, {});
                    free_regs.push_back(d);
                }
                bool nw = fused.count(n) && (is_cmp(N.op) ||
                          ((N.op == MG_AND || N.op == MG_OR || N.op == MG_XOR) && N.width <= 32));
                if (!nw) reg_clean[d] = N.width <= 32;
            } else {
                if ((N.op == MG_ADD || N.op == MG_SUB || N.op == MG_AND || N.op == MG_OR || N.op == MG_XOR ||
                     N.op == MG_NOT || N.op == MG_NEG || N.op == MG_ITE || N.op == MG_CDWE ||
                     N.op == MG_CDWX) && N.width > 32) {
                    std::vector<int> cand;
                    if (N.op == MG_ITE) { for (size_t k = 1; k < 3 && k < slots.size(); k++) cand.push_back(slots[k]); }
                    else if (N.op == MG_CDWE || N.op == MG_CDWX) cand.push_back(slots[0]);
                    else { for (size_t k = 0; k < 2 && k < slots.size(); k++) cand.push_back(slots[k]); }
                    for (int r : cand)
                        if (in(free_regs, r)) { remove(free_regs, r); d = r; break; }
                }
                if (d < 0 && N.width <= 32) {
                    for (size_t k = free_regs.size(); k-- > 0;)
                        if (clean_of(free_regs[k])) { d = free_regs[k]; free_regs.erase(free_regs.begin() + k); break; }
                }
                if (d < 0 && N.width > 32 && keep_clean) {
                    for (size_t k = free_regs.size(); k-- > 0;)
                        if (!clean_of(free_regs[k])) { d = free_regs[k]; free_regs.erase(free_regs.begin() + k); break; }
                }
                if (d < 0) d = alloc_reg(i, {});
                reg_clean[d] = N.width <= 32;
                reg_of[n] = d;
                holder.push_back({d, n});
            }
            uint32_t a = slots.size() > 0 ? slots[0] : 0, b = slots.size() > 1 ? slots[1] : 0, c = 0, imm = 0;
            uint32_t width = N.width;
            if (N.op == MG_CONST) imm = const_index.at(N.imm);
            else if (N.op == MG_LEAF) imm = (uint32_t)N.imm.w[0];
            else if (N.op == MG_EXTRACT || N.op == MG_CONCAT || N.op == MG_SEXT) imm = (uint32_t)N.imm.w[0];
            else if (is_pred(N.op)) width = (uint32_t)N.imm.w[0];
            else if (N.op == MG_ITE) { c = slots[0]; a = slots[1]; b = slots[2]; }
            else if (N.op == MG_CDWE || N.op == MG_CDWX) c = slots[2];
            ins.push_back({(uint32_t)N.op, width, (uint32_t)d, a, b, c, imm, flags});
        }
    }
};

static std::vector<U> pool_values(const U& c, int w) {
    U M256 = mask(256);
    std::vector<U> out{c, (c + U::of(63)) & M256 & ~U::of(63)};
    if (w < 256) {
        int top = std::max(8, c.bitlen());
        for (int k = 0; k < top; k += 8) out.push_back(shr(c, k) & mask(w));
    }
    return out;
}

static std::vector<std::vector<U>> leaf_pools(const std::vector<LN>& ln, const std::vector<int>& order,
                                              const std::vector<Leaf>& leaves) {
    std::vector<U> values;
    for (int n : order) if (ln[n].op == MG_CONST) values.push_back(ln[n].imm);
    std::sort(values.begin(), values.end());
    values.erase(std::unique(values.begin(), values.end()), values.end());
    std::unordered_map<U, int, UHash> cidx;
    for (size_t i = 0; i < values.size(); i++) cidx[values[i]] = (int)i;
    // the leaves / constants under every node: one row of bits per node of
    // the order, in two arenas (ir._leaf_pools' Python int bit sets)
    const size_t wl = (leaves.size() + 63) / 64 + 1, wc = (values.size() + 63) / 64 + 1;
    std::vector<int> row(ln.size(), -1);
    for (size_t i = 0; i < order.size(); i++) row[order[i]] = (int)i;
    std::vector<uint64_t> under_l(order.size() * wl, 0), under_c(order.size() * wc, 0);
    std::vector<uint64_t> done(leaves.size() * wc, 0);      // constants already drawn from
    std::vector<std::vector<U>> pools(leaves.size());
    // pool membership: values below 2^16 in a per-leaf bitmap (narrow leaves
    // draw mostly byte slices, nearly all duplicates), the rest hashed
    // (open addressing over indices into the pool: at most POOL_CAP entries)
    std::vector<std::vector<int16_t>> pool_set(leaves.size());
    std::vector<std::vector<uint64_t>> pool_small(leaves.size());
    std::unordered_map<int64_t, std::vector<U>> pv;
    U M256 = mask(256);
    for (size_t i = 0; i < order.size(); i++) {
        int n = order[i];
        const LN& N = ln[n];
        uint64_t* ls = &under_l[i * wl];
        uint64_t* cs = &under_c[i * wc];
        if (N.op == MG_LEAF) {
            int li = (int)N.imm.w[0];
            ls[li >> 6] |= 1ull << (li & 63);
            continue;
        }
        if (N.op == MG_CONST) {
            int ci = cidx[N.imm];
            cs[ci >> 6] |= 1ull << (ci & 63);
            continue;
        }
        for (int a : N.args) {
            const uint64_t* al = &under_l[(size_t)row[a] * wl];
            const uint64_t* ac = &under_c[(size_t)row[a] * wc];
            for (size_t k = 0; k < wl; k++) ls[k] |= al[k];
            for (size_t k = 0; k < wc; k++) cs[k] |= ac[k];
        }
        int cnt = 0;
        for (size_t k = 0; k < wc; k++) cnt += __builtin_popcountll(cs[k]);
        if (cnt > POOL_CAP) {                    // keep the POOL_CAP smallest constants
            int kept = 0;
            for (size_t k = 0; k < wc; k++) {
                uint64_t x = cs[k], keep = 0;
                while (x && kept < POOL_CAP) { uint64_t b = x & (~x + 1); keep |= b; x ^= b; kept++; }
                cs[k] = keep;
            }
        }
        bool any_c = false;
        for (size_t k = 0; k < wc; k++) any_c |= cs[k] != 0;
        if (!is_cmp(N.op) || !any_c) continue;
        for (size_t kl = 0; kl < wl; kl++) {
            uint64_t lx = ls[kl];
            while (lx) {
                int li = (int)(64 * kl + __builtin_ctzll(lx));
                lx &= lx - 1;
                auto& p = pools[li];
                if ((int)p.size() >= POOL_CAP) continue;
                uint64_t* dn = &done[(size_t)li * wc];
                bool fresh_c = false;
                for (size_t k = 0; k < wc; k++) fresh_c |= (cs[k] & ~dn[k]) != 0;
                if (!fresh_c) continue;
                auto& ps = pool_set[li];
                auto& small = pool_small[li];
                if (small.empty()) { small.assign(1024, 0); ps.assign(4 * POOL_CAP, -1); }
                int w = leaves[li].width;
                bool full = false;
                for (size_t k = 0; k < wc && !full; k++) {
                    uint64_t nw = cs[k] & ~dn[k];
                    dn[k] |= nw;
                    while (nw && !full) {
                        int ci = (int)(64 * k + __builtin_ctzll(nw));
                        nw &= nw - 1;
                        const U& c = values[ci];
                        int64_t key = (int64_t)ci * 4096 + w;
                        auto it = pv.find(key);
                        if (it == pv.end()) {
                            std::vector<U> vals = pool_values(c, w);
                            for (auto& v : vals) v = v & M256;
                            it = pv.emplace(key, std::move(vals)).first;
                        }
                        for (auto& v : it->second) {
                            bool fresh;
                            if (!(v.w[0] >> 16) && !v.w[1] && !v.w[2] && !v.w[3] && !v.w[4] && !v.w[5]) {
                                uint64_t& word = small[v.w[0] >> 6];
                                uint64_t bit = 1ull << (v.w[0] & 63);
                                fresh = !(word & bit);
                                word |= bit;
                            } else {
                                uint64_t h = v.w[0] * 0x9E3779B97F4A7C15ull ^ v.w[1] * 0xC2B2AE3D27D4EB4Full ^
                                             v.w[2] * 0x165667B19E3779F9ull ^ v.w[3] * 0x27D4EB2F165667C5ull;
                                size_t slot = (h ^ (h >> 32)) & (ps.size() - 1);
                                fresh = true;
                                while (ps[slot] >= 0) {
                                    if (p[ps[slot]] == v) { fresh = false; break; }
                                    slot = (slot + 1) & (ps.size() - 1);
                                }
                                if (fresh) ps[slot] = (int16_t)p.size();
                            }
                            if (fresh) p.push_back(v);
                            if ((int)p.size() >= POOL_CAP) break;
                        }
                        if ((int)p.size() >= POOL_CAP) full = true;
                    }
                }
            }
        }
    }
    return pools;
}

// ir.scan_const_keys
// (``order``: topo(S, roots), computed once by the caller)
static OMap<std::string, std::vector<Big>> scan_const_keys(const std::vector<Src>& S, const std::vector<int>& order,
                                                           int cap, int max_links,
                                                           std::unordered_map<std::string, int>& sym_counts) {
    OMap<std::string, std::vector<Big>> out;
    std::unordered_map<std::string, std::vector<std::string>> dummy;
    OMap<std::string, std::unordered_set<int>> sym;
    auto note = [&](const std::string& name, int key) {
        if (S[key].op == S_BVNUM) {
            auto& d = out.setdefault(name, {});
            if ((int)d.size() < cap) {
                bool have = false;
                for (auto& v : d) if (v == S[key].val) { have = true; break; }
                if (!have) d.push_back(S[key].val);
            }
        } else {
            sym.setdefault(name, {}).insert(key);
        }
    };
    for (int n : order) {
        if (S[n].op == S_SELECT) {
            std::vector<int> stack{S[n].args[0]};
            std::unordered_set<int> seen;
            while (!stack.empty()) {
                int x = stack.back();
                stack.pop_back();
                if (seen.count(x)) continue;
                seen.insert(x);
                if (S[x].op == S_STORE) stack.push_back(S[x].args[0]);
                else if (S[x].op == S_ITE) { stack.push_back(S[x].args[1]); stack.push_back(S[x].args[2]); }
                else if (S[x].op == S_ARRAY) note(S[x].str, S[n].args[1]);
            }
        } else if (S[n].op == S_APPLY) {
            note(S[n].str, S[n].args[0]);
        }
    }
    OMap<std::string, std::vector<Big>> ck;
    for (auto& kv : out.items) {
        const auto* s = sym.find(kv.first);
        size_t ns = s ? s->size() : 0;
        if (!kv.second.empty() && (long long)ns * (long long)kv.second.size() <= max_links) {
            std::vector<Big> v = kv.second;
            std::sort(v.begin(), v.end());
            ck.put(kv.first, v);
        }
    }
    for (auto& kv : sym.items) sym_counts[kv.first] = (int)kv.second.size();
    return ck;
}

// ---------------------------------------------------------------------------
// search-mode inputs: candidate hints (model.harvest_hints) and ABI presets
// (abi.plan / Plan.view)
// ---------------------------------------------------------------------------
static void harvest_hints(const std::vector<Src>& S, const std::vector<int>& order, std::vector<U>& out) {
    U M256 = mask(256), low6 = ~U::of(63);
    for (int n : order) {                                 // topo(S, cons)
        if (S[n].op != S_BVNUM || S[n].width < 8) continue;
        U v = S[n].val.chunk(0);                         // (v + 63) & ~63, mod 2^256
        out.push_back((v + U::of(63)) & M256 & low6);
        const Big& b = S[n].val;
        if (!b.l.empty() && b.l.size() == 1) out.push_back(shl(U::of(b.l[0]), 224));
    }
}

struct Presets {
    std::vector<std::pair<std::string, U>> vars;                       // size var -> value
    std::vector<std::pair<std::string, std::vector<std::pair<int64_t, int>>>> arrays;   // offset -> byte
    std::vector<std::pair<int, U>> subst;                              // node -> numeral
};

// abi._split_add: k as base + constant (bvadd chains with numerals)
static bool split_add(const std::vector<Src>& S, int k, int& base, U& c) {
    base = -1;
    c = U();
    std::vector<int> stack{k};
    while (!stack.empty()) {
        int x = stack.back();
        stack.pop_back();
        if (S[x].op == S_BVNUM) c = c + S[x].val.low384();
        else if (S[x].op == S_BVADD) for (int a : S[x].args) stack.push_back(a);
        else if (base < 0) base = x;
        else return false;
    }
    if (base < 0) return false;
    c = c & mask(S[k].width);
    return true;
}

// abi._byte_cell: (offset, size var) of ite(p < size, A[p], 0) or A[p]
static bool byte_cell(const std::vector<Src>& S, int x, int arr, int64_t& off, int& size) {
    size = -1;
    if (S[x].op == S_ITE && S[S[x].args[2]].op == S_BVNUM && S[S[x].args[2]].val.l.empty()) {
        int c = S[x].args[0];
        if (S[c].op != S_BVSLT || S[S[c].args[0]].op != S_BVNUM || S[S[c].args[1]].op != S_VAR) return false;
        size = S[c].args[1];
        x = S[x].args[1];
    }
    if (S[x].op == S_SELECT && S[x].args[0] == arr && S[S[x].args[1]].op == S_BVNUM) {
        const Big& v = S[S[x].args[1]].val;
        if (v.l.size() > 2) return false;
        off = (int64_t)(v.l.empty() ? 0 : v.l[0]) | (v.l.size() > 1 ? (int64_t)v.l[1] << 32 : 0);
        return true;
    }
    return false;
}

// abi._word: (first byte offset, size var) when base is the 32-byte word of arr
static bool word_of(const std::vector<Src>& S, int base, int arr, int64_t& first, int& size) {
    std::vector<int> parts, stack{base};
    while (!stack.empty()) {
        int x = stack.back();
        stack.pop_back();
        if (S[x].op == S_CONCAT) for (size_t i = S[x].args.size(); i-- > 0;) stack.push_back(S[x].args[i]);
        else parts.push_back(x);
    }
    if (parts.size() != 32) return false;
    size = -1;
    std::vector<int64_t> offs;
    for (int p : parts) {
        int64_t o;
        int s;
        if (!byte_cell(S, p, arr, o, s) || (s >= 0 && size >= 0 && s != size)) return false;
        if (s >= 0) size = s;
        offs.push_back(o);
    }
    for (size_t i = 0; i < offs.size(); i++) if (offs[i] != offs[0] + (int64_t)i) return false;
    first = offs[0];
    return true;
}

static bool abi_plan(const std::vector<Src>& S, const std::vector<int>& nodes, Presets& out) {
    // nodes: topo(S, cons)
    struct Arr { int arr; std::vector<Big> consts; std::vector<int> sym; };
    OMap<int, Arr> by_arr;
    for (int n : nodes) {
        if (S[n].op != S_SELECT || S[S[n].args[0]].op != S_ARRAY) continue;
        int arr = S[n].args[0], k = S[n].args[1];
        Arr& d = by_arr.setdefault(arr, Arr{arr, {}, {}});
        if (S[k].op == S_BVNUM) {
            if (std::find(d.consts.begin(), d.consts.end(), S[k].val) == d.consts.end()) d.consts.push_back(S[k].val);
        } else {
            d.sym.push_back(k);
        }
    }
    for (auto& kv : by_arr.items) {
        const Arr& d = kv.second;
        if (d.sym.empty() || d.consts.empty()) continue;
        struct Base { int base; U lo, hi; int64_t off; std::vector<std::pair<int, U>> keys; int size; };
        OMap<int, Base> bases;
        bool ok = true;
        for (int k : d.sym) {
            int base;
            U c;
            if (!split_add(S, k, base, c) || nz(shr(c, 32))) { ok = false; break; }
            Base* r = bases.find(base);
            if (!r) {
                int64_t off = 0;
                int size = -1;
                if (!word_of(S, base, d.arr, off, size)) { ok = false; break; }
                r = &bases.setdefault(base, Base{base, c, c, off, {}, size});
            }
            r->lo = umin(r->lo, c);
            r->hi = umax(r->hi, c);
            r->keys.push_back({k, c});
        }
        if (!ok) continue;
        int size_var = -1;
        U nxt = std::max_element(d.consts.begin(), d.consts.end())->low384() + U::of(1);
        std::vector<std::pair<int64_t, int>> cells;           // insertion-ordered (dict)
        auto set_cell = [&](int64_t o, int b) {
            for (auto& c : cells) if (c.first == o) { c.second = b; return; }
            cells.push_back({o, b});
        };
        for (auto& bv : bases.items) {
            const Base& b = bv.second;
            U val = shl(sar(nxt - b.lo + U::of(31), 5), 5);    // 32-aligned, past nxt
            for (int i = 0; i < 32; i++) set_cell(b.off + i, (int)(sar(val, 8 * (31 - i)).w[0] & 0xFF));
            for (auto& kc : b.keys) out.subst.push_back({kc.first, (val + kc.second) & mask(S[kc.first].width)});
            nxt = val + b.hi + U::of(1);
            if (size_var < 0) size_var = b.size;
        }
        if (size_var >= 0) {
            out.vars.push_back({S[size_var].str, nxt});
            out.subst.push_back({size_var, nxt & mask(S[size_var].width)});
        }
        out.arrays.push_back({S[d.arr].str, cells});
        for (int n : nodes) {
            if (S[n].op != S_SELECT || S[n].args[0] != d.arr || S[S[n].args[1]].op != S_BVNUM) continue;
            const Big& v = S[S[n].args[1]].val;
            if (v.l.size() > 2) continue;
            int64_t o = (int64_t)(v.l.empty() ? 0 : v.l[0]) | (v.l.size() > 1 ? (int64_t)v.l[1] << 32 : 0);
            for (auto& c : cells)
                if (c.first == o) { out.subst.push_back({n, U::of((uint64_t)c.second) & mask(S[n].width)}); break; }
        }
    }
    return !out.arrays.empty();
}

// ---------------------------------------------------------------------------
// JSON output
// ---------------------------------------------------------------------------
static void jstr(std::string& o, const std::string& s) {
    o.push_back('"');
    for (unsigned char ch : s) {
        if (ch == '"' || ch == '\\') { o.push_back('\\'); o.push_back((char)ch); }
        else if (ch == '\n') o += "\\n";
        else if (ch == '\t') o += "\\t";
        else if (ch < 0x20) { char b[8]; std::snprintf(b, sizeof b, "\\u%04x", ch); o += b; }
        else o.push_back((char)ch);
    }
    o.push_back('"');
}

}  // namespace

struct mgc_result {
    std::string error;
    std::vector<uint32_t> code;
    std::vector<uint32_t> table;
    int32_t n_rows = 0, n_const_values = 0;
    std::string meta;
};

namespace {

static double now_us() {
    return std::chrono::duration<double, std::micro>(
        std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void compile(const mgc_input* in, mgc_result* res) {
    // phase boundaries (meta "t_us": decode, lower, solve, sinks, schedule,
    // allocate, pools + tables, metadata) — diagnostics for the get_model
    // compile latency, never part of the program
    double tp[9];
    tp[0] = now_us();
    // -- decode and check the source DAG ----------------------------------------
    // (the C ABI takes arrays from any caller: every index, count and width
    // is checked before use, so a malformed DAG is an error, never a wild
    // access — tests/fuzz_compile.cpp runs mutated inputs under ASan/UBSan)
    auto bad = [](const char* what) { throw std::runtime_error(what); };
    if (in->n_nodes < 0 || in->n_cons < 0 || in->n_probes < 0 || in->n_strings < 0 ||
        in->n_tables < 0 || in->n_extra < 0 || in->n_cval < 0 || in->n_string_bytes < 0)
        bad("negative count");
    if (in->n_nodes && (!in->op || !in->sort || !in->width || !in->dom || !in->id || !in->arg_off ||
                        !in->p0 || !in->p1 || !in->str || !in->cval_off))
        bad("missing node array");
    if ((in->n_cons && !in->cons) || (in->n_probes && !in->probes) ||
        (in->n_tables && (!in->table_name || !in->table_size)) || (in->n_extra && !in->extra) ||
        (in->n_cval && !in->cval) || (in->n_string_bytes && !in->strings))
        bad("missing array");
    if (in->nreg < 2 || in->nreg > 256 || in->default_entries < 0 || in->default_entries > 4096)
        bad("nreg / default_entries out of range");
    std::vector<std::string> strings;
    {
        const char* p = in->strings;
        const char* end = in->strings + in->n_string_bytes;
        for (int i = 0; i < in->n_strings; i++) {
            const char* z = p < end ? (const char*)std::memchr(p, 0, (size_t)(end - p)) : nullptr;
            if (!z) bad("string table overrun");
            strings.emplace_back(p, (size_t)(z - p));
            p = z + 1;
        }
    }
    if (in->n_nodes && in->arg_off[0] != 0) bad("arg_off[0] != 0");
    std::vector<Src> S(in->n_nodes);
    for (int i = 0; i < in->n_nodes; i++) {
        Src& s = S[i];
        s.op = in->op[i]; s.sort = in->sort[i]; s.width = in->width[i]; s.dom = in->dom[i];
        s.id = in->id[i];
        if (s.op < 0 || s.op > S_OTHER) bad("bad op code");
        if (s.sort < 0 || s.sort > MGC_SORT_ARRAY) bad("bad sort");
        if (s.width < 1 || s.width > MGC_MAX_SOURCE_WIDTH || s.dom < 0 || s.dom > MGC_MAX_SOURCE_WIDTH)
            bad("width out of range");
        if (in->arg_off[i + 1] < in->arg_off[i]) bad("arg_off not monotonic");
        if (in->arg_off[i + 1] > 0 && !in->args) bad("missing args array");
        for (int k = in->arg_off[i]; k < in->arg_off[i + 1]; k++) {
            int a = in->args[k];
            if (a < 0 || a >= i) bad("operand index out of order");
            s.args.push_back(a);
        }
        s.p0 = in->p0[i]; s.p1 = in->p1[i];
        if (in->str[i] >= 0) {
            if (in->str[i] >= in->n_strings) bad("string index out of range");
            s.str = strings[in->str[i]];
        }
        if (s.op == S_BVNUM) {
            int64_t nl = (s.width + 31) / 32;
            if (in->cval_off[i] < 0 || (int64_t)in->cval_off[i] + nl > in->n_cval) bad("numeral limbs out of range");
            s.val.l.assign(in->cval + in->cval_off[i], in->cval + in->cval_off[i] + nl);
            s.val.norm();
        }
        // operand counts the lowering reads (smt/node.py constructors' arities)
        size_t na = s.args.size(), need_min = 0, need_max = (size_t)-1;
        switch (s.op) {
        case S_BVNUM: case S_TRUE: case S_FALSE: case S_VAR: case S_ARRAY: need_max = 0; break;
        case S_BVNEG: case S_BVNOT: case S_NOT: case S_EXTRACT: case S_ZEXT: case S_SEXT: case S_K:
        case S_APPLY: need_min = need_max = 1; break;
        case S_BVSUB: case S_BVUDIV: case S_BVUREM: case S_BVSDIV: case S_BVSREM: case S_BVSMOD:
        case S_BVSHL: case S_BVLSHR: case S_BVASHR: case S_XOR: case S_IMPLIES: case S_BVULT:
        case S_BVULE: case S_BVUGT: case S_BVUGE: case S_BVSLT: case S_BVSLE: case S_BVSGT:
        case S_BVSGE: case S_UMULNO: case S_SELECT: need_min = need_max = 2; break;
        case S_ITE: case S_STORE: need_min = need_max = 3; break;
        case S_BVADD: case S_BVMUL: case S_BVAND: case S_BVOR: case S_BVXOR: case S_AND: case S_OR:
        case S_CONCAT: need_min = 1; break;
        case S_EQ: case S_DISTINCT: need_min = 2; break;
        default: break;
        }
        if (na < need_min || na > need_max) bad("operand count");
        if (s.op == S_EXTRACT && (s.p1 < 0 || s.p0 < s.p1 || s.p0 >= S[s.args[0]].width ||
                                  s.width != s.p0 - s.p1 + 1))
            bad("extract bounds");
        if ((s.op == S_ZEXT || s.op == S_SEXT) && (s.p0 < 0 || s.width != S[s.args[0]].width + s.p0))
            bad("extension width");
        if (s.op == S_APPLY && s.p0 != S[s.args[0]].width) bad("function domain");
    }
    std::vector<int> cons(in->cons, in->cons + in->n_cons);
    std::vector<int> probes(in->probes, in->probes + in->n_probes);
    for (int c : cons) if (c < 0 || c >= in->n_nodes) throw std::runtime_error("constraint index");
    for (int p : probes) if (p < 0 || p >= in->n_nodes) throw std::runtime_error("probe index");
    std::vector<int> all = cons;
    all.insert(all.end(), probes.begin(), probes.end());

    std::vector<U> hints;
    std::vector<int> cons_order;                         // one walk for both scans
    if (in->search_hints || in->abi_presets) cons_order = topo(S, cons);
    if (in->search_hints) harvest_hints(S, cons_order, hints);
    Presets presets;
    bool have_presets = in->abi_presets && abi_plan(S, cons_order, presets);
    if (have_presets) {
        // the query under the presets (Plan.view): each pinned node becomes
        // the numeral, keeping its id
        for (auto& su : presets.subst) {
            Src& s = S[su.first];
            s.op = S_BVNUM;
            s.args.clear();
            s.str.clear();
            s.p0 = s.p1 = 0;
            s.val = big_of(su.second);
        }
    }

    tp[1] = now_us();
    Lowerer lw(S, in->default_entries);
    for (int t = 0; t < in->n_tables; t++) {
        if (in->table_name[t] < 0 || in->table_name[t] >= in->n_strings || in->table_size[t] < 0 ||
            in->table_size[t] > 4096)
            bad("table entry out of range");
        lw.table_sizes.put(strings[in->table_name[t]], in->table_size[t]);
    }
    lw.solve = in->solve != 0;
    if (in->const_keys || in->solve) {
        std::unordered_map<std::string, int> sym_counts;
        const std::vector<int> all_order = topo(S, all);  // after the presets
        auto ck = scan_const_keys(S, all_order, in->solve ? 256 : 128, in->solve ? 8192 : 2048, sym_counts);
        if (in->const_keys) lw.table_ckeys = ck;
        if (in->solve) {
            for (int n : all_order) {
                if (S[n].op == S_ARRAY || S[n].op == S_APPLY) {
                    auto it = sym_counts.find(S[n].str);
                    if ((it == sym_counts.end() ? 0 : it->second) <= ARG_ENTRIES_CAP) lw.solve_tables.insert(S[n].str);
                }
            }
        }
    }
    Chunks roots;
    std::vector<int64_t> births;
    for (int c : cons) {
        if (!S[c].is_bool()) throw Unsupported("constraint is not Bool");
        roots.push_back(lw.lower(c)[0]);
        births.push_back(S[c].id);
    }
    tp[2] = now_us();
    std::vector<std::pair<int, int>> derived_nodes;
    Solver* solver = nullptr;
    std::unique_ptr<Solver> solver_own;
    if (lw.solve) {
        solver_own.reset(new Solver(lw));
        solver = solver_own.get();
        solver->run(roots, derived_nodes);
        if (solver->dead) {                 // a false root: that root alone
            births.resize(1);
            probes.clear();
        }
    }
    tp[3] = now_us();
    Memo probe_memo;
    Chunks sinks;
    for (size_t i = 0; i < roots.size(); i++) {
        lw.birth = births[i];
        sinks.push_back(lw.mk(MG_ROOT, 1, {roots[i]}));
    }
    int probe_chunks = 0;
    for (int p : probes) {
        if (S[p].is_array()) throw Unsupported("array probe");
        Chunks chs = lw.lower(p);
        for (int ch : chs) {
            if (solver) { lw.birth = 0; ch = solver->rewrite(ch, probe_memo); }
            lw.birth = S[p].id;
            sinks.push_back(lw.mki(MG_OUT, 1, {ch}, probe_chunks));
            probe_chunks++;
        }
    }
    int n_user_probes = probe_chunks;
    std::vector<std::pair<int, int>> derived;
    std::vector<std::pair<std::string, std::vector<std::vector<int>>>> entry_keys;
    if (solver) {
        auto out = [&](int n) {
            lw.birth = 0;
            sinks.push_back(lw.mki(MG_OUT, 1, {n}, probe_chunks));
            probe_chunks++;
            return probe_chunks - 1;
        };
        std::sort(derived_nodes.begin(), derived_nodes.end());
        for (auto& de : derived_nodes) derived.push_back({de.first, out(de.second)});
        Memo memo_e;
        lw.birth = 0;
        for (auto& te : lw.arg_entries.items) {
            if (solver->dead) break;
            std::vector<std::vector<int>> ks;
            for (auto& ent : te.second) {
                std::vector<int> row;
                for (int k : ent.first) row.push_back(out(solver->rewrite(k, memo_e)));
                ks.push_back(row);
            }
            entry_keys.push_back({te.first, ks});
        }
    }
    if (sinks.empty()) {
        int one = lw.cnst(1, 1);
        sinks.push_back(lw.mk(MG_ROOT, 1, {one}));
    }
    for (auto& n : lw.ln)
        if (is_pred(n.op)) { n.imm = U::of((uint64_t)n.width); n.has_imm = true; n.width = 1; }
    tp[4] = now_us();
    std::unordered_set<int> fused;
    std::vector<int> order = fuse_roots(lw.ln, schedule(lw.ln, sinks), fused);
    tp[5] = now_us();
    U M256 = mask(256);
    std::vector<U> const_values;
    for (int n : order) if (lw.ln[n].op == MG_CONST) const_values.push_back(lw.ln[n].imm & M256);
    for (int i = 0; i < in->n_extra; i++) {
        U v;
        for (int j = 0; j < 8; j++) v.w[j / 2] |= (uint64_t)in->extra[8 * i + j] << (32 * (j & 1));
        const_values.push_back(v);
    }
    for (auto& h : hints) const_values.push_back(h & M256);
    std::sort(const_values.begin(), const_values.end());
    const_values.erase(std::unique(const_values.begin(), const_values.end()), const_values.end());
    std::unordered_map<U, int, UHash> const_index;
    for (size_t i = 0; i < const_values.size(); i++) const_index[const_values[i]] = (int)i;
    Alloc al0(lw.ln, order, const_index, fused, in->nreg, in->remat_mode, in->remat_k,
              in->keep_clean != 0);
    al0.run();
    // eval form: the sink-driven order too when the source order keeps at
    // least SCHEDULE_MIN_SCRATCH spill slots in scratch, and the cheaper
    // allocation (ir.compile_constraints_py: scratch spill slots, then
    // spill + reload records, then instructions); search programs keep
    // source order
    const Alloc* alp = &al0;
    std::unordered_set<int> fused2;
    std::vector<int> order2;
    std::unique_ptr<Alloc> al2;
    if (!in->solve && !in->leaf_pools && al0.n_lds - LDS_TIER >= SCHEDULE_MIN_SCRATCH) {
        order2 = fuse_roots(lw.ln, schedule_demand(lw.ln, sinks), fused2);
        try {
            al2.reset(new Alloc(lw.ln, order2, const_index, fused2, in->nreg, in->remat_mode,
                                in->remat_k, in->keep_clean != 0));
            al2->run();
        } catch (const Unsupported&) {
            al2.reset();
        }
        auto cost = [](const Alloc& a) {
            return std::make_tuple(std::max(0, a.n_lds - LDS_TIER), a.n_spill + a.n_reload,
                                   (int)a.ins.size());
        };
        if (al2 && cost(*al2) < cost(al0)) alp = al2.get();
    }
    const Alloc& al = *alp;
    const std::vector<int>& ord = alp == &al0 ? order : order2;
    tp[6] = now_us();
    res->code.resize(4 * al.ins.size());
    for (size_t k = 0; k < al.ins.size(); k++) {
        const Ins& x = al.ins[k];
        res->code[4 * k] = x.op | (x.width << 8) | x.flags;
        res->code[4 * k + 1] = x.d | (x.a << 8) | (x.b << 16) | (x.c << 24);
        res->code[4 * k + 2] = x.imm;
        res->code[4 * k + 3] = 0;
    }
    // constant table: the CONST values, then every non-empty leaf pool,
    // written straight as limbs
    std::vector<std::pair<int, int>> pool_ranges;
    std::vector<std::vector<U>> pools;
    size_t n_rows = const_values.size();
    if (in->leaf_pools) {
        pools = leaf_pools(lw.ln, order, lw.leaves);
        for (size_t li = 0; li < pools.size(); li++) {
            if (!pools[li].empty()) {
                pool_ranges.push_back({(int)n_rows, (int)pools[li].size()});
                n_rows += pools[li].size();
            } else {
                pool_ranges.push_back({0, (int)const_values.size()});
            }
        }
    }
    res->n_rows = (int32_t)n_rows;
    res->n_const_values = (int32_t)const_values.size();
    res->table.resize(8 * n_rows);
    uint32_t* row = res->table.data();
    auto put = [&row](const U& u) {
        for (int j = 0; j < 8; j++) row[j] = (uint32_t)(u.w[j / 2] >> (32 * (j & 1)));
        row += 8;
    };
    for (const U& u : const_values) put(u);
    for (const auto& pl : pools)
        for (const U& u : pl) put(u);

    tp[7] = now_us();
    // -- metadata ---------------------------------------------------------------
    std::string& o = res->meta;
    // the leaves as ONE string, "name TAB width TAB kind TAB source TAB chunk
    // TAB entry" records separated by newlines: a big search group has
    // hundreds of leaves, and a caller that never unpacks a witness (a miss)
    // never needs more than their count and widths (ccompile.LeafRecords
    // splits it on first use); the widths also come as their own list
    bool plain = true;                       // no separator inside a name
    for (const Leaf& L : lw.leaves)
        plain = plain && L.name.find_first_of("\t\n") == std::string::npos &&
                L.source.find_first_of("\t\n") == std::string::npos;
    if (!plain) {
        o = "{\"leaves\":[";
        for (size_t i = 0; i < lw.leaves.size(); i++) {
            const Leaf& L = lw.leaves[i];
            if (i) o += ",";
            o += "[";
            jstr(o, L.name);
            o += "," + std::to_string(L.width) + ",";
            jstr(o, KIND_NAMES[L.kind]);
            o += ",";
            jstr(o, L.source);
            o += "," + std::to_string(L.chunk) + "," + std::to_string(L.entry) + "]";
        }
        o += "],\"leaves_rs\":null";
    } else {
        o = "{\"leaves_rs\":";
    }
    if (plain) {
        std::string rs;
        for (size_t i = 0; i < lw.leaves.size(); i++) {
            const Leaf& L = lw.leaves[i];
            if (i) rs += '\n';
            rs += L.name;
            rs += '\t';
            rs += std::to_string(L.width);
            rs += '\t';
            rs += KIND_NAMES[L.kind];
            rs += '\t';
            rs += L.source;
            rs += '\t';
            rs += std::to_string(L.chunk);
            rs += '\t';
            rs += std::to_string(L.entry);
        }
        jstr(o, rs);
    }
    o += ",\"leaf_widths\":[";
    for (size_t i = 0; i < lw.leaves.size(); i++) {
        if (i) o += ",";
        o += std::to_string(lw.leaves[i].width);
    }
    o += "],\"n_lds\":" + std::to_string(al.n_lds);
    o += ",\"n_probes\":" + std::to_string(probe_chunks);
    o += ",\"n_roots\":" + std::to_string(cons.size());
    // table sizes: solve tables report their argument-keyed entries
    o += ",\"table_sizes\":[";
    {
        bool first = true;
        for (auto& kv : lw.table_sizes.items) {
            int v = kv.second;
            if (lw.solve_tables.count(kv.first) && lw.table_kinds.has(kv.first)) {
                auto* ents = lw.arg_entries.find(kv.first);
                v = ents ? (int)ents->size() : 0;
            }
            if (!first) o += ",";
            first = false;
            o += "[";
            jstr(o, kv.first);
            o += "," + std::to_string(v) + "]";
        }
    }
    o += "],\"table_kinds\":[";
    for (size_t i = 0; i < lw.table_kinds.items.size(); i++) {
        if (i) o += ",";
        o += "[";
        jstr(o, lw.table_kinds.items[i].first);
        o += ",";
        jstr(o, lw.table_kinds.items[i].second);
        o += "]";
    }
    o += "],\"table_ckeys\":[";
    {
        bool first = true;
        for (auto& kv : lw.table_ckeys.items) {
            if (!lw.table_kinds.has(kv.first)) continue;
            if (!first) o += ",";
            first = false;
            o += "[";
            jstr(o, kv.first);
            o += ",[";
            for (size_t j = 0; j < kv.second.size(); j++) {
                if (j) o += ",";
                jstr(o, kv.second[j].hexs());
            }
            o += "]]";
        }
    }
    std::vector<int> hist(MG_NUM_OPS, 0);
    for (int n : ord) hist[lw.ln[n].op]++;
    o += "],\"lnodes\":" + std::to_string(ord.size());
    o += ",\"spills\":" + std::to_string(al.n_spill);
    o += ",\"reloads\":" + std::to_string(al.n_reload);
    o += ",\"hist\":[";
    {
        bool first = true;
        for (int op = 0; op < MG_NUM_OPS; op++) {
            if (!hist[op]) continue;
            if (!first) o += ",";
            first = false;
            o += "[" + std::to_string(op) + "," + std::to_string(hist[op]) + "]";
        }
    }
    o += "],\"hist_order\":[";
    {
        std::vector<char> seen(MG_NUM_OPS, 0);
        bool first = true;
        for (int n : ord) {
            int op = lw.ln[n].op;
            if (seen[op]) continue;
            seen[op] = 1;
            if (!first) o += ",";
            first = false;
            o += std::to_string(op);
        }
    }
    o += "],\"pool_ranges\":[";
    for (size_t i = 0; i < pool_ranges.size(); i++) {
        if (i) o += ",";
        o += "[" + std::to_string(pool_ranges[i].first) + "," + std::to_string(pool_ranges[i].second) + "]";
    }
    o += "],\"derived\":[";
    for (size_t i = 0; i < derived.size(); i++) {
        if (i) o += ",";
        o += "[" + std::to_string(derived[i].first) + "," + std::to_string(derived[i].second) + "]";
    }
    o += "],\"entry_keys\":[";
    for (size_t i = 0; i < entry_keys.size(); i++) {
        if (i) o += ",";
        o += "[";
        jstr(o, entry_keys[i].first);
        o += ",[";
        for (size_t j = 0; j < entry_keys[i].second.size(); j++) {
            if (j) o += ",";
            o += "[";
            for (size_t k = 0; k < entry_keys[i].second[j].size(); k++) {
                if (k) o += ",";
                o += std::to_string(entry_keys[i].second[j][k]);
            }
            o += "]";
        }
        o += "]]";
    }
    o += "],\"n_user_probes\":" + std::to_string(n_user_probes);
    tp[8] = now_us();
    o += ",\"t_us\":[";
    for (int k = 0; k < 8; k++) {
        char b[32];
        std::snprintf(b, sizeof b, "%s%.1f", k ? "," : "", tp[k + 1] - tp[k]);
        o += b;
    }
    o += "]";
    if (have_presets) {
        o += ",\"presets\":{\"vars\":[";
        for (size_t i = 0; i < presets.vars.size(); i++) {
            if (i) o += ",";
            o += "[";
            jstr(o, presets.vars[i].first);
            o += ",";
            jstr(o, (presets.vars[i].second.neg() ? "-" + hex(U() - presets.vars[i].second) : hex(presets.vars[i].second)));
            o += "]";
        }
        o += "],\"arrays\":[";
        for (size_t i = 0; i < presets.arrays.size(); i++) {
            if (i) o += ",";
            o += "[";
            jstr(o, presets.arrays[i].first);
            o += ",[";
            for (size_t j = 0; j < presets.arrays[i].second.size(); j++) {
                if (j) o += ",";
                o += "[" + std::to_string(presets.arrays[i].second[j].first) + "," +
                     std::to_string(presets.arrays[i].second[j].second) + "]";
            }
            o += "]]";
        }
        o += "]}";
    }
    o += "}";
}

}  // namespace

extern "C" {

const char* mgc_source_ops(void) { return SOP_NAMES; }

int mgc_compile(const mgc_input* in, mgc_result** out) {
    mgc_result* r = new mgc_result();
    *out = r;
    try {
        compile(in, r);
        return MGC_OK;
    } catch (Unsupported& e) {
        r->error = e.what();
        return MGC_UNSUPPORTED;
    } catch (BadShift& e) {
        r->error = e.what();
        return MGC_ERROR;
    } catch (std::exception& e) {
        r->error = e.what();
        return MGC_ERROR;
    } catch (MemoMiss&) {
        r->error = "operand lowered only as part of a pattern";
        return MGC_UNSUPPORTED;
    }
}

const char* mgc_error(const mgc_result* r) { return r->error.c_str(); }

const uint32_t* mgc_code(const mgc_result* r, int32_t* n_ins) {
    *n_ins = (int32_t)(r->code.size() / 4);
    return r->code.data();
}

const uint32_t* mgc_table(const mgc_result* r, int32_t* n_rows, int32_t* n_const_values) {
    *n_rows = r->n_rows;
    *n_const_values = r->n_const_values;
    return r->table.data();
}

const char* mgc_meta(const mgc_result* r) { return r->meta.c_str(); }

void mgc_free(mgc_result* r) { delete r; }

}  // extern "C"
