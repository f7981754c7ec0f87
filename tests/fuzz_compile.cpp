// Fuzz driver for the native compiler's C ABI (include/mythcc.h), built with
// -fsanitize=address,undefined by tests/test_native_compiler.py: every input
// of a corpus file (written by the test from real DAGs) is compiled as is —
// it must succeed — and then under random mutations of its arrays and
// counts, which must end in MGC_OK / MGC_UNSUPPORTED / MGC_ERROR and never
// in an out-of-bounds access or undefined behaviour.
//
// usage: fuzz_compile <corpus.bin> <mutations per input>
// corpus: repeated records, little-endian:
//   int32 n_nodes n_strings n_cons n_probes n_tables default_entries nreg
//         n_extra leaf_pools const_keys solve remat_mode remat_k keep_clean
//         search_hints abi_presets n_cval n_string_bytes n_args
//   int32 op[n] sort[n] width[n] dom[n]; int64 id[n]; int32 arg_off[n+1]
//   int32 args[n_args]; int64 p0[n] p1[n]; int32 str[n] cval_off[n]
//   uint32 cval[n_cval]; char strings[n_string_bytes]; int32 cons[] probes[]
//   int32 table_name[] table_size[]; uint32 extra[8 n_extra]
#include "mythcc.h"

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

struct Rec {
    int32_t h[19];
    std::vector<int32_t> op, sort, width, dom, arg_off, args, str, cval_off, cons, probes, tname, tsize;
    std::vector<int64_t> id, p0, p1;
    std::vector<uint32_t> cval, extra;
    std::vector<char> strings;
};

template <class T> static bool rd(FILE* f, std::vector<T>& v, long n) {
    if (n < 0) return false;
    v.resize((size_t)n);
    return n == 0 || fread(v.data(), sizeof(T), (size_t)n, f) == (size_t)n;
}

static bool read_rec(FILE* f, Rec& r) {
    if (fread(r.h, sizeof r.h, 1, f) != 1) return false;
    long n = r.h[0];
    return rd(f, r.op, n) && rd(f, r.sort, n) && rd(f, r.width, n) && rd(f, r.dom, n) && rd(f, r.id, n) &&
           rd(f, r.arg_off, n + 1) && rd(f, r.args, r.h[18]) && rd(f, r.p0, n) && rd(f, r.p1, n) &&
           rd(f, r.str, n) && rd(f, r.cval_off, n) && rd(f, r.cval, r.h[16]) && rd(f, r.strings, r.h[17]) &&
           rd(f, r.cons, r.h[2]) && rd(f, r.probes, r.h[3]) && rd(f, r.tname, r.h[4]) &&
           rd(f, r.tsize, r.h[4]) && rd(f, r.extra, 8L * r.h[7]);
}

// the input as the caller hands it over; counts may disagree with the
// arrays' real lengths only downwards (the mutations shrink them)
static mgc_input view(Rec& r) {
    mgc_input in;
    std::memset(&in, 0, sizeof in);
    in.n_nodes = r.h[0]; in.n_strings = r.h[1]; in.n_cons = r.h[2]; in.n_probes = r.h[3];
    in.n_tables = r.h[4]; in.default_entries = r.h[5]; in.nreg = r.h[6]; in.n_extra = r.h[7];
    in.leaf_pools = r.h[8]; in.const_keys = r.h[9]; in.solve = r.h[10]; in.remat_mode = r.h[11];
    in.remat_k = r.h[12]; in.keep_clean = r.h[13]; in.search_hints = r.h[14]; in.abi_presets = r.h[15];
    in.n_cval = r.h[16]; in.n_string_bytes = r.h[17];
    in.op = r.op.data(); in.sort = r.sort.data(); in.width = r.width.data(); in.dom = r.dom.data();
    in.id = r.id.data(); in.arg_off = r.arg_off.data(); in.args = r.args.data(); in.p0 = r.p0.data();
    in.p1 = r.p1.data(); in.str = r.str.data(); in.cval_off = r.cval_off.data(); in.cval = r.cval.data();
    in.strings = r.strings.data(); in.cons = r.cons.data(); in.probes = r.probes.data();
    in.table_name = r.tname.data(); in.table_size = r.tsize.data(); in.extra = r.extra.data();
    return in;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<Rec> recs;
    Rec r;
    while (read_rec(f, r)) recs.push_back(r);
    fclose(f);
    int muts = atoi(argv[2]);
    std::mt19937_64 rng(0x6d797468);
    long ok = 0, unsup = 0, err = 0, valid_ok = 0;
    for (auto& base : recs) {
        mgc_input in = view(base);
        mgc_result* res;
        int rc = mgc_compile(&in, &res);
        valid_ok += rc == MGC_OK;
        mgc_free(res);
        for (int m = 0; m < muts; m++) {
            Rec x = base;
            int nm = 1 + (int)(rng() % 3);
            for (int k = 0; k < nm; k++) {
                long n = x.h[0];
                auto pick = [&](long lim) { return lim > 0 ? (long)(rng() % (uint64_t)lim) : 0L; };
                auto wild = [&]() { return (int32_t)((int64_t)(rng() % 140000) - 4000); };
                switch (rng() % 14) {
                case 0: if (n) x.op[pick(n)] = (int32_t)(rng() % 50) - 2; break;
                case 1: if (n) x.width[pick(n)] = wild(); break;
                case 2: if (!x.args.empty()) x.args[pick((long)x.args.size())] = (int32_t)pick(n + 4) - 2; break;
                case 3: if (n) x.arg_off[1 + pick(n)] = (int32_t)pick((long)x.args.size() + 1); break;
                case 4: if (n) x.p0[pick(n)] = (int64_t)wild(); break;
                case 5: if (n) x.p1[pick(n)] = (int64_t)wild(); break;
                case 6: if (n) x.str[pick(n)] = (int32_t)pick(x.h[1] + 3) - 1; break;
                case 7: if (n) x.cval_off[pick(n)] = (int32_t)pick(x.h[16] + 9) - 1; break;
                case 8: if (!x.cons.empty()) x.cons[pick((long)x.cons.size())] = (int32_t)pick(n + 3) - 1; break;
                case 9: x.h[16] = (int32_t)pick(x.h[16] + 1); break;                 // shorter cval
                case 10: x.h[17] = (int32_t)pick(x.h[17] + 1); break;                // shorter strings
                case 11: if (n) x.sort[pick(n)] = (int32_t)pick(5) - 1; break;
                case 12: if (n) x.dom[pick(n)] = wild(); break;
                default: x.h[6] = (int32_t)pick(40) - 4; break;                       // nreg
                }
            }
            // counts never exceed the arrays (the caller's contract)
            if (x.h[16] > (int32_t)x.cval.size()) x.h[16] = (int32_t)x.cval.size();
            if (x.h[17] > (int32_t)x.strings.size()) x.h[17] = (int32_t)x.strings.size();
            for (auto& o : x.arg_off) if (o > (int32_t)x.args.size()) o = (int32_t)x.args.size();
            mgc_input xi = view(x);
            rc = mgc_compile(&xi, &res);
            if (rc == MGC_OK) ok++;
            else if (rc == MGC_UNSUPPORTED) unsup++;
            else err++;
            (void)mgc_meta(res);
            mgc_free(res);
        }
    }
    printf("{\"inputs\": %zu, \"valid_ok\": %ld, \"mutated_ok\": %ld, \"mutated_unsupported\": %ld, "
           "\"mutated_error\": %ld}\n", recs.size(), valid_ok, ok, unsup, err);
    return 0;
}
