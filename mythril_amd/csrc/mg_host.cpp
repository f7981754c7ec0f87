// Host-only half of libmythgpu: program validation and the IR -> record
// translation of the assembly interpreter.  No HIP runtime calls, so this
// file also builds with plain g++ under ASan/UBSan (tests/test_host_sanitize.py
// fuzzes it with malformed programs): it is the safety boundary that keeps a
// kernel from indexing outside the register file, the spill area, the
// constant pool, the leaf table or the probe buffer.

#include <algorithm>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mg_host.h"

// LEAFD / RELOADD variants are the slot number, with MGA_V_WAITD as the wait
// flag above the slot bits (wait_vm below adds it to the handler id): more
// slots than that would alias slot d + 16 with slot d's WAITD handler
static_assert(MG_NREG <= MGA_V_WAITD, "register slots overlap the WAITD variant bit");

static int fail(std::string* err, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (err) *err = buf;
    return code;
}

// ---- IR -> assembly-interpreter records (8 words each) ----------------------
//
// w0 handler byte offset | w1 8*dst | w2 8*a | w3 8*b | w4 8*c / funnel index /
// leaf or probe index | w5 immediate (const / spill byte offset, funnel shift,
// source width) | w6 width | w7 byte offset of an 8- (SEXT: 16-) word mask
// entry appended to the constant table.  The record after a heavy op lives in
// bank A, otherwise banks alternate (asmgen.py: prefetch into the other bank).


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
static uint32_t slots_touched(uint32_t op, uint32_t d, uint32_t a, uint32_t b, uint32_t c,
                              uint32_t nreg) {
    switch (op) {
    case MG_NOP: return 0;
    case MG_CONST: case MG_LEAF: case MG_RELOAD: return 1u << d;
    case MG_SPILL: case MG_OUT: case MG_ROOT: return 1u << a;
    case MG_NOT: case MG_NEG: case MG_MOV: case MG_SEXT:
        return (1u << d) | (1u << a);
    // the funnel shifts read one slot beyond their operand (masked off, but
    // the registers are read): the next slot for EXTRACT, the previous one
    // for CONCAT's high part
    case MG_EXTRACT: return ((1u << d) | (3u << a)) & ((1u << nreg) - 1);
    case MG_CONCAT: return (1u << d) | (1u << a) | (a ? 1u << (a - 1) : 0u) | (1u << b);
    case MG_ITE: case MG_CDWE: case MG_CDWX: return (1u << d) | (1u << a) | (1u << b) | (1u << c);
    case MG_BCAST: return (1u << d) | (1u << a);
    default: return (1u << d) | (1u << a) | (1u << b);
    }
}

// slots an instruction reads (its destination only when it is also an operand)
static uint32_t slots_read(uint32_t op, uint32_t d, uint32_t a, uint32_t b, uint32_t c,
                           uint32_t nreg) {
    uint32_t m = slots_touched(op, d, a, b, c, nreg);
    switch (op) {
    case MG_NOP: case MG_CONST: case MG_LEAF: case MG_RELOAD: return 0;
    case MG_SPILL: case MG_OUT: case MG_ROOT: return m;
    default: break;
    }
    const bool d_operand = d == a || (op != MG_NOT && op != MG_NEG && op != MG_MOV &&
                                      op != MG_EXTRACT && op != MG_SEXT && op != MG_BCAST && d == b) ||
                           ((op == MG_ITE || op == MG_CDWE || op == MG_CDWX) && d == c) ||
                           (op == MG_EXTRACT && d == a + 1) ||
                           (op == MG_CONCAT && a && d == a - 1);
    return d_operand ? m : m & ~(1u << d);
}

// ---- spill placement ----------------------------------------------------------
//
// The compiler numbers spill slots lowest-free; the translator decides where
// each spilled VALUE lives (round 5).  An interval runs from a SPILL to the
// last RELOAD of its slot before the slot's next SPILL.  Placement packs the
// intervals into the n_lds LDS regions (8 KiB each: 8 dword positions per
// lane, [half][lane] x 16 B) greedily by scratch bytes saved per unit of LDS
// capacity x time: a 256-bit value takes a whole region for its interval, a
// one-limb value (Bool results, values of <= 32 bits: limbs 1..7 are zero,
// values being canonical) one dword position.  The rest goes to per-lane
// scratch, re-coloured lowest-free in start order (the fewest 32-byte
// scratch positions).  Every scratch spill is written back to HBM when its
// L2 line is evicted (profiles/r05: WRITE_SIZE ~ the static scratch store
// bytes) while reloads often hit L2, so what LDS takes off is mostly HBM
// writes.  A SPILL whose slot is never reloaded is dropped.
enum : uint32_t {
    PL_SPILLREL = 1u << 31,   // a SPILL / RELOAD with a placement
    PL_LDS = 1u << 30,        // in LDS (else scratch)
    PL_NARROW = 1u << 29,     // one dword (reload zeroes limbs 1..7)
    PL_DEAD = 1u << 28,       // a SPILL nobody reloads: emit nothing
    PL_OFF = (1u << 28) - 1,  // byte offset (LDS: region/half/dword; scratch: 32 * position)
};

static std::vector<uint32_t> place_spills(const uint32_t* code, uint32_t n_ins, uint32_t n_lds,
                                          uint32_t nreg, std::vector<uint32_t>& place2) {
    struct Iv { uint32_t start, end, reloads; bool narrow; uint32_t loc, loc2; };
    std::vector<uint32_t> place(n_ins, 0);
    std::vector<Iv> ivs;
    std::vector<int> open;                  // spill slot -> open interval (or -1)
    std::vector<int> owner(n_ins, -1);      // SPILL / RELOAD instruction -> interval
    bool narrow_reg[MG_NREG];
    for (int k = 0; k < MG_NREG; ++k) narrow_reg[k] = false;
    for (uint32_t i = 0; i < n_ins; ++i) {
        const uint32_t* in = code + 4 * i;
        const uint32_t op = in[0] & 0xFF, w = (in[0] >> 8) & 0x3FF, imm = in[2];
        const uint32_t d = in[1] & 0xFF, a = (in[1] >> 8) & 0xFF;
        if (op == MG_SPILL) {
            if (imm >= open.size()) open.resize(imm + 1, -1);
            open[imm] = (int)ivs.size();
            ivs.push_back({i, i, 0, a < nreg && narrow_reg[a], 0, 0});
            owner[i] = open[imm];
            continue;
        }
        if (op == MG_RELOAD) {
            const int k = imm < open.size() ? open[imm] : -1;
            if (k >= 0) {
                ivs[k].end = i;
                ivs[k].reloads++;
            }
            owner[i] = k;
            if (d < nreg) narrow_reg[d] = k >= 0 ? ivs[k].narrow : w <= 32;
            continue;
        }
        const bool writes = op != MG_NOP && op != MG_OUT && op != MG_ROOT;
        if (writes && d < nreg) narrow_reg[d] = is_compare(op) || w <= 32;
    }
    // LDS: 4-dword HALVES (half h: region h / 2, part h % 2, 4 KiB = 256
    // lanes x 16 B).  A 256-bit value takes two free halves (any two: the
    // record carries both offsets), a one-limb value one dword of a half.
    // With six regions a 13th half fills the CU (mg_lds_bytes).  Three
    // greedy orders (bytes saved per LDS capacity x time; bytes saved;
    // start), the one leaving the fewest scratch bytes wins.
    const uint32_t nhalf = mg_lds_halves(n_lds), npos = nhalf * 4;
    std::vector<uint32_t> cand;
    for (uint32_t k = 0; k < ivs.size(); ++k)
        if (ivs[k].reloads) cand.push_back(k);
    auto saved = [&](const Iv& v) { return (v.narrow ? 4.0 : 32.0) * (1.0 + v.reloads); };
    auto density = [&](const Iv& v) {
        return saved(v) / ((double)(v.end - v.start + 1) * (v.narrow ? 1.0 : 8.0));
    };
    std::vector<uint32_t> best_loc, best_loc2;
    double best_cost = -1.0;
    for (int pass = 0; pass < 3; ++pass) {
        std::vector<uint32_t> byprio = cand;
        if (pass == 0)
            std::stable_sort(byprio.begin(), byprio.end(), [&](uint32_t x, uint32_t y) {
                return density(ivs[x]) > density(ivs[y]);
            });
        else if (pass == 1)
            std::stable_sort(byprio.begin(), byprio.end(), [&](uint32_t x, uint32_t y) {
                return saved(ivs[x]) > saved(ivs[y]);
            });
        std::vector<std::vector<std::pair<uint32_t, uint32_t>>> used(npos);
        auto free_at = [&](uint32_t p, uint32_t s, uint32_t e) {
            for (auto& u : used[p])
                if (!(u.second < s || e < u.first)) return false;
            return true;
        };
        auto half_free = [&](uint32_t h, uint32_t s, uint32_t e) {
            for (uint32_t j = 0; j < 4; ++j)
                if (!free_at(h * 4 + j, s, e)) return false;
            return true;
        };
        auto half_load = [&](uint32_t h) {
            int load = 0;
            for (uint32_t j = 0; j < 4; ++j) load += (int)used[h * 4 + j].size();
            return load;
        };
        std::vector<uint32_t> loc(ivs.size(), 0), loc2(ivs.size(), 0);
        double cost = 0.0;
        for (uint32_t k : byprio) {
            const Iv& v = ivs[k];
            bool placed = false;
            if (!v.narrow) {
                // the two free halves with the fewest narrow tenants
                int h0 = -1, h1 = -1;
                for (uint32_t h = 0; h < nhalf; ++h) {
                    if (!half_free(h, v.start, v.end)) continue;
                    if (h0 < 0 || half_load(h) < half_load((uint32_t)h0)) { h1 = h0; h0 = (int)h; }
                    else if (h1 < 0 || half_load(h) < half_load((uint32_t)h1)) h1 = (int)h;
                }
                if (h0 >= 0 && h1 >= 0) {
                    for (uint32_t j = 0; j < 4; ++j) {
                        used[h0 * 4 + j].push_back({v.start, v.end});
                        used[h1 * 4 + j].push_back({v.start, v.end});
                    }
                    loc[k] = PL_LDS | mg_lds_half_offset((uint32_t)h0);
                    loc2[k] = mg_lds_half_offset((uint32_t)h1);
                    placed = true;
                }
            } else {
                // a free dword in the half already holding the most narrow
                // intervals (keeps whole halves free for 256-bit values)
                int best = -1, best_load = -1;
                for (uint32_t p = 0; p < npos; ++p) {
                    if (!free_at(p, v.start, v.end)) continue;
                    const int load = half_load(p / 4);
                    if (load > best_load) { best_load = load; best = (int)p; }
                }
                if (best >= 0) {
                    used[best].push_back({v.start, v.end});
                    loc[k] = PL_LDS | PL_NARROW |
                             (mg_lds_half_offset((uint32_t)best / 4) + ((uint32_t)best % 4) * 4u);
                    placed = true;
                }
            }
            if (!placed) cost += (v.narrow ? 4.0 : 32.0) * (1.0 + 0.5 * v.reloads);
        }
        if (best_cost < 0.0 || cost < best_cost) {
            best_cost = cost;
            best_loc = loc;
            best_loc2 = loc2;
        }
    }
    for (uint32_t k = 0; k < ivs.size(); ++k) {
        ivs[k].loc = best_loc.empty() ? 0u : best_loc[k];
        ivs[k].loc2 = best_loc2.empty() ? 0u : best_loc2[k];
    }
    // scratch: lowest free 32-byte position at each interval's start
    std::vector<uint32_t> scr_end;          // position -> end of its last interval
    for (uint32_t k = 0; k < ivs.size(); ++k) {
        Iv& v = ivs[k];
        if (!v.reloads) { v.loc = PL_DEAD; continue; }
        if (v.loc & PL_LDS) continue;
        uint32_t p = 0;
        while (p < scr_end.size() && scr_end[p] >= v.start) ++p;
        if (p == scr_end.size()) scr_end.push_back(0);
        scr_end[p] = v.end;
        v.loc = (v.narrow ? PL_NARROW : 0u) | p * 32u;
    }
    place2.assign(n_ins, 0);
    for (uint32_t i = 0; i < n_ins; ++i)
        if (owner[i] >= 0) {
            place[i] = PL_SPILLREL | ivs[owner[i]].loc;
            place2[i] = ivs[owner[i]].loc2;
        }
    return place;
}

void mg_translate_records(const uint32_t* hoff, const uint32_t* code, uint32_t n_ins, uint32_t n_consts,
                          uint32_t n_lds, uint32_t nreg, std::vector<uint32_t>& rec, MaskPool& pool) {
    pool.base = n_consts;
    const uint32_t ones = pool.add(mask_lt(256));
    rec.clear();
    rec.reserve((size_t)(n_ins + 4) * 8);
    // clean[s]: limbs 1..7 of slot s are known to be zero (its last value had
    // at most 32 bits); registers start uninitialised
    bool clean[MG_NREG];
    for (int k = 0; k < MG_NREG; ++k) clean[k] = false;
    // where every spilled value lives (LDS region / dword, or scratch), per
    // SPILL / RELOAD instruction (place_spills)
    std::vector<uint32_t> place2;           // a 256-bit LDS value's second half
    const std::vector<uint32_t> place = place_spills(code, n_ins, n_lds, nreg, place2);
    auto scratch_reload = [&](uint32_t i) {
        return (code[4 * i] & 0xFF) == MG_RELOAD && !(place[i] & PL_LDS);
    };
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
    uint32_t last_ld_hid = 0;               // its handler id, WAITD bit clear
    auto wait_vm = [&]() {
        if (last_ld != SIZE_MAX && last_ld + 8 == rec.size()) {
            // the LEAFD / RELOADD waits itself: its WAITD variant
            rec[last_ld] = hoff[last_ld_hid + 2 * MGA_V_WAITD];
            rec[last_ld + 6] = 1;
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
        if (!leafd && !scratch_reload(order[q])) continue;
        const uint32_t rd = in[1] & 0xFF, slot = leafd ? 0xFFFFFFFFu : in[2];
        uint32_t t = q;
        while (t > 0 && q - t < 24) {
            const uint32_t* p = code + 4 * order[t - 1];
            const uint32_t pop = p[0] & 0xFF;
            if (slots_touched(pop, p[1] & 0xFF, (p[1] >> 8) & 0xFF, (p[1] >> 16) & 0xFF,
                              (p[1] >> 24) & 0xFF, nreg) & (1u << rd))
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
    // A store-chain link: t = (a == b) of wide values, consumed only by the
    // next instruction, an ITE on t -> one EQSEL record.  Decided up front
    // (it depends on the order only): the dirty one-limb scan below must know
    // that such an ITE reads all eight limbs of its value operands (EQSEL
    // copies them), not limb 0 as a w <= 32 ITE does.
    std::vector<uint8_t> eqsel(n_ins + 1, 0), eqsel_ite(n_ins + 1, 0);
    for (uint32_t pc = 0; pc + 1 < n_ins; ++pc) {
        const uint32_t* in = code + 4 * order[pc];
        const uint32_t op = in[0] & 0xFF, w = (in[0] >> 8) & 0x3FF, d = in[1] & 0xFF;
        if (op != MG_EQ || w <= 32 || (in[0] & MG_ROOT_FLAG)) continue;
        const uint32_t* nx = code + 4 * order[pc + 1];
        const uint32_t na = (nx[1] >> 8) & 0xFF, nb = (nx[1] >> 16) & 0xFF, nc = (nx[1] >> 24) & 0xFF;
        bool fuse = (nx[0] & 0xFF) == MG_ITE && !(nx[0] & MG_ROOT_FLAG) && nc == d && na != d && nb != d;
        for (uint32_t q = pc + 2; fuse && q < n_ins; ++q) {     // is t dead after the ITE?
            const uint32_t* f = code + 4 * order[q];
            const uint32_t fop = f[0] & 0xFF, fd = f[1] & 0xFF, fa = (f[1] >> 8) & 0xFF,
                           fb = (f[1] >> 16) & 0xFF, fc = (f[1] >> 24) & 0xFF;
            if (slots_read(fop, fd, fa, fb, fc, nreg) & (1u << d)) fuse = false;
            else if (slots_touched(fop, fd, fa, fb, fc, nreg) & (1u << d)) break;   // rewritten
        }
        if (fuse) {
            eqsel[pc] = 1;
            eqsel_ite[pc + 1] = 1;
            ++pc;
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
        const uint32_t op = in[0] & 0xFF, w = (in[0] >> 8) & 0x3FF;
        const uint32_t pl = place[order[pc]];
        if (op == MG_SPILL && (pl & PL_DEAD)) continue;     // never reloaded
        const uint32_t d = in[1] & 0xFF, a = (in[1] >> 8) & 0xFF, b = (in[1] >> 16) & 0xFF,
                       c = (in[1] >> 24) & 0xFF;
        if (eqsel[pc]) {
            const uint32_t* nx = code + 4 * order[pc + 1];
            const uint32_t nd = nx[1] & 0xFF, na = (nx[1] >> 8) & 0xFF, nb = (nx[1] >> 16) & 0xFF,
                           nc = (nx[1] >> 24) & 0xFF;
            const uint32_t touch = slots_touched(op, d, a, b, c, nreg) | slots_touched(MG_ITE, nd, na, nb, nc, nreg);
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
        const bool leafd = op == MG_LEAF && w == 256;
        const bool reloadd = op == MG_RELOAD && !(pl & PL_LDS);
        if (pending && (slots_touched(op, d, a, b, c, nreg) & pending)) wait_vm();
        if (leafd || reloadd) pending |= 1u << d;
        uint32_t* r = emit();
        uint32_t var = (in[0] & MG_ROOT_FLAG) ? MGA_V_ROOT : 0;
        const bool writes = op != MG_NOP && op != MG_SPILL && op != MG_OUT && op != MG_ROOT;
        // result fits one limb: Bool results, or values of at most 32 bits
        // (a reload: the placement's view of the spilled value)
        const bool narrow = is_compare(op) || (writes && w <= 32) ||
                            (op == MG_RELOAD && (pl & PL_NARROW));
        const bool w32 = has_w32(op) && w <= 32;       // compares: w = operand width
        if (w32) var |= MGA_V_W32;
        // a one-limb result whose every reader (until the slot is written
        // again) reads limb 0 only — one-limb (W32) ops, an ITE's condition,
        // ROOT, a one-dword spill — need not zero limbs 1..7 either: the DC
        // handler (limb 0 only) serves, and the slot is then marked dirty
        // (round 5; the Bool results of compares are the common case)
        bool dirty = false;
        if (writes && narrow && !clean[d] && d < nreg) {
            dirty = true;
            bool read = false;
            for (uint32_t q = pc + 1; q < n_ins && dirty; ++q) {
                const uint32_t* f = code + 4 * order[q];
                const uint32_t fop = f[0] & 0xFF, fw = (f[0] >> 8) & 0x3FF, fd = f[1] & 0xFF,
                               fa = (f[1] >> 8) & 0xFF, fb = (f[1] >> 16) & 0xFF, fc = (f[1] >> 24) & 0xFF;
                const uint32_t rd = slots_read(fop, fd, fa, fb, fc, nreg);
                if (rd & (1u << d)) {
                    read = true;
                    const bool limb0 =
                        (has_w32(fop) && fw <= 32 && fop != MG_EXTRACT && !eqsel_ite[q]) ||
                        (fop == MG_ITE && fc == d && fa != d && fb != d && !eqsel_ite[q]) ||
                        fop == MG_ROOT ||
                        (fop == MG_SPILL && (place[order[q]] & PL_NARROW));
                    if (!limb0) dirty = false;
                }
                if (slots_touched(fop, fd, fa, fb, fc, nreg) & ~rd & (1u << d)) break;   // rewritten
            }
            (void)read;
        }
        if (writes && narrow && (clean[d] || dirty)) var |= MGA_V_DC;
        const uint32_t maskv = w32 ? (w < 32 ? MGA_V_MASK : 0) : ((w >= 1 && w < 256) ? MGA_V_MASK : 0);
        r[1] = 8 * d; r[2] = 8 * a; r[3] = 8 * b; r[4] = 8 * c; r[5] = 0; r[6] = w; r[7] = ones;
        int aop = MGA_NOP;
        switch (op) {
        case MG_NOP: aop = MGA_NOP; break;
        case MG_CONST: aop = MGA_CONST; r[5] = in[2] * 32u; break;
        case MG_LEAF:
            aop = MGA_LEAF; r[4] = in[2];
            if (leafd) { aop = MGA_LEAFD; var = d; }
            else if (maskv) { var |= MGA_V_MASK; r[7] = pool.add(mask_lt(w)); }
            break;
        case MG_SPILL:              // spills and reloads: the variant is the slot
        case MG_RELOAD: {           // (| NARROW: one dword, limbs 1..7 zero)
            const bool lds = pl & PL_LDS;
            const bool nf = pl & PL_NARROW;
            if (op == MG_SPILL) { aop = lds ? MGA_SPILL_LDS : MGA_SPILL_SCR; var = a; }
            else { aop = lds ? MGA_RELOAD_LDS : MGA_RELOADD; var = d; }
            if (nf) var |= MGA_V_NARROW;
            r[5] = (pl & PL_SPILLREL) ? (pl & PL_OFF) : 0u;
            if (lds && !nf) r[7] = place2[order[pc]];     // limbs 4..7 (second half)
            break;
        }
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
            const uint32_t q = in[2] >> 5, bs = in[2] & 31;
            var = q | (bs ? 8u : 0u);
            r[4] = 8 * a + 8 - q - (bs ? 1 : 0);
            r[5] = bs ? 32 - bs : 0;
            r[7] = ~((1u << bs) - 1u);              // limb q: bits >= bs from a
            break;
        }
        case MG_EXTRACT:            // R = (a >> imm) & mask(w)
            r[4] = 8 * a + (in[2] >> 5) + 8;
            r[5] = in[2] & 31;
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
            r[5] = in[2];
            std::vector<uint32_t> m = mask_lt(in[2]), m2 = mask_lt(w);
            m.insert(m.end(), m2.begin(), m2.end());
            r[7] = pool.add(m);
            break;
        }
        case MG_OUT: aop = MGA_OUT; r[4] = in[2]; break;
        case MG_ROOT: aop = MGA_ROOT; break;
        case MG_MOV: aop = MGA_MOV; break;
        case MG_BCAST: aop = MGA_BCAST; var = 0; break;
        case MG_CDWE: aop = MGA_CDWE; var = d == a ? MGA_V_IP : 0; break;
        case MG_CDWX: aop = MGA_CDWX; var = d == a ? MGA_V_IP : 0; break;
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
        // a ROOT-fused Bool nobody reads (the common case: a path condition):
        // the NW variant only updates the root and leaves the slot alone
        bool nw = false;
        if ((in[0] & MG_ROOT_FLAG) &&
            (aop == MGA_EQ || aop == MGA_ULT || aop == MGA_ULE || aop == MGA_SLT || aop == MGA_SLE ||
             ((aop == MGA_AND || aop == MGA_OR || aop == MGA_XOR) && (var & MGA_V_W32)))) {
            nw = true;
            for (uint32_t q = pc + 1; q < n_ins; ++q) {
                const uint32_t* f = code + 4 * order[q];
                const uint32_t fop = f[0] & 0xFF, fd = f[1] & 0xFF, fa = (f[1] >> 8) & 0xFF,
                               fb = (f[1] >> 16) & 0xFF, fc = (f[1] >> 24) & 0xFF;
                if (slots_read(fop, fd, fa, fb, fc, nreg) & (1u << d)) { nw = false; break; }
                if (slots_touched(fop, fd, fa, fb, fc, nreg) & (1u << d)) break;   // rewritten
            }
            if (nw) var = (var | MGA_V_NW) & ~MGA_V_DC;
        }
        r[0] = hoff[MGA_HID(aop, var, bank)];
        if (aop == MGA_LEAFD || aop == MGA_RELOADD) {
            r[6] = 0;
            last_ld = (size_t)(r - rec.data());
            last_ld_hid = MGA_HID(aop, var, bank);
        }
        if (writes && !nw) clean[d] = narrow && !dirty;
        bank = mga_is_heavy(aop) ? 0 : 1 - bank;
    }
}

int mg_validate(std::string* err, const uint32_t* code, uint32_t n_ins, uint32_t n_consts,
                const mg_leafgen* leaves, uint32_t n_leaves, uint32_t n_lds,
                uint32_t n_spill, uint32_t n_probes, uint32_t nreg) {
    if (!mg_find_layout(nreg)) return fail(err, MG_E_ARG, "no %u-slot register layout", nreg);
    if (n_lds > MG_MAX_LDS) return fail(err, MG_E_ARG, "too many LDS slots (%u)", n_lds);
    if (n_spill < n_lds || n_spill - n_lds > MG_MAX_PSLOTS)
        return fail(err, MG_E_ARG, "spill slots %u (LDS %u)", n_spill, n_lds);
    for (uint32_t i = 0; leaves && i < n_leaves; ++i) {
        const mg_leafgen& g = leaves[i];
        if (g.width < 1 || g.width > MG_MAX_WIDTH)
            return fail(err, MG_E_ARG, "leaf %u: width %u", i, g.width);
        if ((uint64_t)g.pool_off + g.pool_n > n_consts)
            return fail(err, MG_E_ARG, "leaf %u: pool outside const table", i);
        if (!(g.pct_uniform <= g.pct_small && g.pct_small <= g.pct_boundary &&
              g.pct_boundary <= 100))
            return fail(err, MG_E_ARG, "leaf %u: class thresholds", i);
    }
    for (uint32_t pc = 0; pc < n_ins; ++pc) {
        const uint32_t* in = code + 4 * pc;
        const uint32_t op = in[0] & 0xFF, w = (in[0] >> 8) & 0x3FF, imm0 = in[2];
        if (op >= MG_NUM_OPS) return fail(err, MG_E_ARG, "ins %u: bad opcode %u", pc, op);
        if ((in[0] & ~(0x3FFFFu | MG_ROOT_FLAG)) != 0)
            return fail(err, MG_E_ARG, "ins %u: reserved bits set", pc);
        for (int k = 0; k < 4; ++k)
            if (((in[1] >> (8 * k)) & 0xFF) >= nreg)
                return fail(err, MG_E_ARG, "ins %u: slot out of range", pc);
        const bool needs_w = op != MG_NOP && op != MG_SPILL && op != MG_OUT && op != MG_ROOT;
        if (needs_w && (w < 1 || w > MG_MAX_WIDTH))
            return fail(err, MG_E_ARG, "ins %u: width %u", pc, w);
        switch (op) {
        case MG_CONST:
            if (imm0 >= n_consts) return fail(err, MG_E_ARG, "ins %u: const %u", pc, imm0);
            break;
        case MG_LEAF:
            if (imm0 >= n_leaves) return fail(err, MG_E_ARG, "ins %u: leaf %u", pc, imm0);
            break;
        case MG_SPILL:
        case MG_RELOAD:
            if (imm0 >= n_spill) return fail(err, MG_E_ARG, "ins %u: spill slot %u", pc, imm0);
            break;
        case MG_OUT:
            if (imm0 >= n_probes) return fail(err, MG_E_ARG, "ins %u: probe %u", pc, imm0);
            break;
        case MG_CONCAT:
            if (imm0 < 1 || imm0 >= w) return fail(err, MG_E_ARG, "ins %u: concat split", pc);
            break;
        case MG_EXTRACT:
            if (imm0 + w > MG_MAX_WIDTH) return fail(err, MG_E_ARG, "ins %u: extract range", pc);
            break;
        case MG_SEXT:
            if (imm0 < 1 || imm0 > w) return fail(err, MG_E_ARG, "ins %u: sext width", pc);
            break;
        case MG_BCAST:
        case MG_CDWE:
        case MG_CDWX:          // their handlers write all eight limbs
            if (w != MG_MAX_WIDTH) return fail(err, MG_E_ARG, "ins %u: calldata word width %u", pc, w);
            if (in[0] & MG_ROOT_FLAG) return fail(err, MG_E_ARG, "ins %u: ROOT on a word", pc);
            break;
        default:
            break;
        }
    }
    return MG_OK;
}

// The register layouts this library holds an interpreter for (one kernel
// each, mg_interp_asm.hip): 16 slots at three waves per SIMD with six LDS
// spill regions (13 halves fill the CU), 11 slots in 128 VGPRs at four waves
// with five (40 KiB per block, four blocks per CU).
static const mg_layout_info kLayouts[] = {{MG_NREG, 3, 6}, {MG_NREG_W4, 4, 5}};

const mg_layout_info* mg_find_layout(uint32_t nreg) {
    for (const auto& l : kLayouts)
        if (l.nreg == nreg) return &l;
    return nullptr;
}

extern "C" {

int mg_layouts(uint32_t* out, uint32_t n) {
    if (!out && n) return MG_E_ARG;
    const uint32_t k = (uint32_t)(sizeof kLayouts / sizeof kLayouts[0]);
    for (uint32_t i = 0; i < k && 3 * i + 2 < n; ++i) {
        out[3 * i] = kLayouts[i].nreg;
        out[3 * i + 1] = kLayouts[i].waves;
        out[3 * i + 2] = kLayouts[i].lds_slots;
    }
    return (int)k;
}

int mg_translate(const uint32_t* code, uint32_t n_ins, uint32_t n_consts, uint32_t n_lds,
                 uint32_t nreg, const uint32_t* handler_off, uint32_t n_handlers,
                 uint32_t* records, uint32_t max_record_words, uint32_t* n_record_words,
                 uint32_t* masks, uint32_t max_mask_words, uint32_t* n_mask_words) {
    if ((n_ins && !code) || !handler_off || n_handlers != MGA_NUM_HANDLERS || !n_record_words ||
        !n_mask_words)
        return MG_E_ARG;
    // leaf and probe tables are not known here: only their indices' shape
    int rc = mg_validate(nullptr, code, n_ins, n_consts, nullptr, 0xFFFFFFFFu, MG_MAX_LDS,
                         MG_MAX_LDS + MG_MAX_PSLOTS, 0xFFFFFFFFu, nreg);
    if (rc) return rc;
    if (n_lds > MG_MAX_LDS) return MG_E_ARG;
    std::vector<uint32_t> rec;
    MaskPool pool;
    mg_translate_records(handler_off, code, n_ins, n_consts, n_lds, nreg, rec, pool);
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

int mg_version(void) { return MG_VERSION; }

}  // extern "C"
