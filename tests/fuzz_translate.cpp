// Fuzz driver for the host-only safety boundary of libmythgpu
// (mythril_amd/csrc/mg_host.cpp: mg_validate, mg_translate_records and the
// exported mg_translate).  Built with g++ -fsanitize=address,undefined by
// tests/test_host_sanitize.py; any sanitizer report or failed invariant
// aborts with a non-zero exit status.
//
// Programs: (a) random words — almost always rejected; (b) valid random
// straight-line programs — must be accepted and translated; (c) one field
// of a valid program mutated (slot, width, opcode, reserved bits, constant /
// leaf / spill / probe index, concat / extract / sext immediates) — must be
// either rejected or translated into in-range records.

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "mg_host.h"

#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            fprintf(stderr, "invariant failed: %s (%s:%d)\n", #c, __FILE__, \
                    __LINE__);                                            \
            abort();                                                      \
        }                                                                 \
    } while (0)

struct Prog {
    std::vector<uint32_t> code;
    uint32_t n_consts, n_leaves, n_lds, n_spill, n_probes;
    uint32_t nreg;                 // register layout: MG_NREG or MG_NREG_W4
};

static uint32_t ins_w0(uint32_t op, uint32_t w) { return op | (w << 8); }

static Prog valid_program(std::mt19937_64& rng) {
    Prog p;
    p.nreg = rng() % 2 ? MG_NREG : MG_NREG_W4;
    p.n_consts = 1 + rng() % 8;
    p.n_leaves = 1 + rng() % 8;
    p.n_spill = rng() % (MG_MAX_LDS + MG_MAX_PSLOTS + 1);
    p.n_lds = p.n_spill < MG_MAX_LDS ? p.n_spill : MG_MAX_LDS;
    p.n_probes = rng() % 4;
    const uint32_t n = 1 + rng() % 64;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t op = 1 + rng() % (MG_NUM_OPS - 1);
        uint32_t w = 1 + rng() % MG_MAX_WIDTH, imm = 0;
        const uint32_t d = rng() % p.nreg, a = rng() % p.nreg, b = rng() % p.nreg,
                       c = rng() % p.nreg;
        switch (op) {
        case MG_CONST: imm = rng() % p.n_consts; break;
        case MG_LEAF: imm = rng() % p.n_leaves; break;
        case MG_SPILL: case MG_RELOAD:
            if (!p.n_spill) op = MG_NOP; else imm = rng() % p.n_spill;
            break;
        case MG_OUT:
            if (!p.n_probes) op = MG_NOP; else imm = rng() % p.n_probes;
            break;
        case MG_CONCAT:
            if (w < 2) w = 2;
            imm = 1 + rng() % (w - 1);
            break;
        case MG_EXTRACT: imm = rng() % (MG_MAX_WIDTH - w + 1); break;
        case MG_SEXT: imm = 1 + rng() % w; break;
        case MG_BCAST: case MG_CDWE: case MG_CDWX: w = MG_MAX_WIDTH; break;   // words only
        default: break;
        }
        if (rng() % 8 == 0 && op != MG_OUT && op != MG_ROOT && op != MG_BCAST && op != MG_CDWE &&
            op != MG_CDWX)
            op |= MG_ROOT_FLAG;
        p.code.push_back(ins_w0(op & 0xFF, w) | (op & MG_ROOT_FLAG));
        p.code.push_back(MG_INS_W1(d, a, b, c));
        p.code.push_back(imm);
        p.code.push_back(0);
    }
    return p;
}

static void mutate(Prog& p, std::mt19937_64& rng) {
    const uint32_t n = (uint32_t)(p.code.size() / 4);
    uint32_t* in = p.code.data() + 4 * (rng() % n);
    switch (rng() % 8) {
    case 0: in[0] = (in[0] & ~0xFFu) | (uint32_t)(rng() % 256); break;           // opcode
    case 1: in[0] = (in[0] & 0xFFu) | ((uint32_t)(rng() % 1024) << 8); break;    // width
    case 2: in[0] |= 1u << (19 + rng() % 13); break;                            // reserved
    case 3: in[1] ^= 1u << (rng() % 32); break;                                  // a slot
    case 4: in[1] = (uint32_t)rng(); break;
    case 5: in[2] = (uint32_t)rng() % 300; break;                               // imm
    case 6: in[2] = (uint32_t)rng(); break;
    default: in[2] += 1; break;                                                 // off by one
    }
}

static void check_records(const Prog& p, const std::vector<uint32_t>& rec, const MaskPool& pool) {
    CHECK(rec.size() % 8 == 0);
    CHECK(rec.size() <= (2 * p.code.size() / 4 + 3) * 8);
    const uint32_t n_const_words = (p.n_consts + (uint32_t)(pool.words.size() / 8)) * 32;
    for (size_t r = 0; r < rec.size(); r += 8) {
        const uint32_t* w = rec.data() + r;
        if (w[0] == 0) {                          // the zeroed prefetch pad
            CHECK(r + 8 == rec.size());
            continue;
        }
        CHECK(w[0] >= 1 && w[0] <= MGA_NUM_HANDLERS);   // handler table index + 1
        CHECK(w[1] < 8 * p.nreg && w[2] < 8 * p.nreg);
        CHECK(w[1] % 8 == 0 && w[2] % 8 == 0);
    }
    CHECK(pool.words.size() % 8 == 0);
    (void)n_const_words;
}

static int run_one(const Prog& p, const uint32_t* hoff, bool must_accept) {
    const uint32_t n = (uint32_t)(p.code.size() / 4);
    std::vector<mg_leafgen> gens(p.n_leaves);
    for (uint32_t i = 0; i < p.n_leaves; ++i) gens[i] = {1 + i * 31 % 256, 0, p.n_consts, 20, 40, 60};
    std::string err;
    const int rc = mg_validate(&err, p.code.data(), n, p.n_consts, gens.data(), p.n_leaves,
                               p.n_lds, p.n_spill, p.n_probes, p.nreg);
    if (must_accept && rc != MG_OK) {
        fprintf(stderr, "valid program rejected: %s\n", err.c_str());
        abort();
    }
    if (rc != MG_OK) {
        CHECK(rc == MG_E_ARG && !err.empty());
        return 0;
    }
    std::vector<uint32_t> rec;
    MaskPool pool;
    mg_translate_records(hoff, p.code.data(), n, p.n_consts, p.n_lds < 6 ? p.n_lds : 6, p.nreg,
                         rec, pool);
    check_records(p, rec, pool);
    // the exported entry: exact-size buffers, then too-small ones
    uint32_t nw = 0, nm = 0;
    std::vector<uint32_t> out(rec.size() + 8), masks(pool.words.size() + 8);
    int rc2 = mg_translate(p.code.data(), n, p.n_consts, p.n_lds < 6 ? p.n_lds : 6, p.nreg, hoff,
                           MGA_NUM_HANDLERS, out.data(), (uint32_t)out.size(), &nw, masks.data(),
                           (uint32_t)masks.size(), &nm);
    CHECK(rc2 == MG_OK && nw == rec.size() && nm == pool.words.size());
    if (nw > 8) {
        rc2 = mg_translate(p.code.data(), n, p.n_consts, p.n_lds < 6 ? p.n_lds : 6, p.nreg, hoff,
                           MGA_NUM_HANDLERS, out.data(), nw - 8, &nw, masks.data(),
                           (uint32_t)masks.size(), &nm);
        CHECK(rc2 == MG_E_ARG);
    }
    return 1;
}

int main(int argc, char** argv) {
    const long iters = argc > 1 ? strtol(argv[1], nullptr, 10) : 20000;
    std::mt19937_64 rng(0x6D797468);
    std::vector<uint32_t> hoff(MGA_NUM_HANDLERS);
    for (uint32_t h = 0; h < MGA_NUM_HANDLERS; ++h) hoff[h] = h + 1;
    long accepted = 0, mutated_ok = 0, random_ok = 0;
    for (long it = 0; it < iters; ++it) {
        Prog p = valid_program(rng);
        accepted += run_one(p, hoff.data(), true);
        Prog m = p;
        for (int k = 0, nm = 1 + (int)(rng() % 3); k < nm; ++k) mutate(m, rng);
        mutated_ok += run_one(m, hoff.data(), false);
        Prog r = p;
        for (auto& x : r.code) x = (uint32_t)rng();
        random_ok += run_one(r, hoff.data(), false);
    }
    // null / degenerate arguments of the exported entry
    uint32_t nw, nm;
    CHECK(mg_translate(nullptr, 1, 0, 0, MG_NREG, hoff.data(), MGA_NUM_HANDLERS, nullptr, 0, &nw,
                       nullptr, 0, &nm) == MG_E_ARG);
    CHECK(mg_translate(nullptr, 0, 0, 0, MG_NREG, hoff.data(), MGA_NUM_HANDLERS - 1, nullptr, 0,
                       &nw, nullptr, 0, &nm) == MG_E_ARG);
    CHECK(mg_translate(nullptr, 0, 0, MG_MAX_LDS + 1, MG_NREG, hoff.data(), MGA_NUM_HANDLERS,
                       nullptr, 0, &nw, nullptr, 0, &nm) == MG_E_ARG);
    // a slot count no layout has, and a 16-slot program offered to the 11-slot layout
    CHECK(mg_translate(nullptr, 0, 0, 0, 12, hoff.data(), MGA_NUM_HANDLERS, nullptr, 0, &nw,
                       nullptr, 0, &nm) == MG_E_ARG);
    {
        const uint32_t code[4] = {ins_w0(MG_CONST, 8), 13u, 0u, 0u};   // dst slot 13
        std::vector<uint32_t> out(64), masks(64);
        CHECK(mg_translate(code, 1, 1, 0, MG_NREG_W4, hoff.data(), MGA_NUM_HANDLERS, out.data(),
                           64, &nw, masks.data(), 64, &nm) == MG_E_ARG);
        CHECK(mg_translate(code, 1, 1, 0, MG_NREG, hoff.data(), MGA_NUM_HANDLERS, out.data(),
                           64, &nw, masks.data(), 64, &nm) == MG_OK);
    }
    printf("{\"iterations\": %ld, \"valid_accepted\": %ld, \"mutated_accepted\": %ld, "
           "\"random_accepted\": %ld}\n", iters, accepted, mutated_ok, random_ok);
    return 0;
}
