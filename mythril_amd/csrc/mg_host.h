// Host-only half of libmythgpu (mg_host.cpp): validation of uploaded IR and
// its translation into assembly-interpreter records.  No HIP types.
#ifndef MG_HOST_H
#define MG_HOST_H

#include <stdint.h>

#include <map>
#include <string>
#include <vector>

#include "mythgpu.h"
#include "mythgpu_ir.h"
#include "mg_asm_handlers.h"
#include "mg_device.h"

#define MG_VERSION 4

// Translator mask entries, appended to a program's constant table.
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

// 0 (MG_OK) or MG_E_ARG with a message in *err (may be NULL).  leaves may be
// NULL (n_leaves is then only the bound on LEAF indices).
// nreg: the register slots of the layout the program was compiled for
// (MG_NREG or MG_NREG_W4); every slot index must be below it.
int mg_validate(std::string* err, const uint32_t* code, uint32_t n_ins, uint32_t n_consts,
                const mg_leafgen* leaves, uint32_t n_leaves, uint32_t n_lds, uint32_t n_spill,
                uint32_t n_probes, uint32_t nreg);

// Records of a VALIDATED program (hoff: handler byte offsets, MGA_NUM_HANDLERS).
void mg_translate_records(const uint32_t* hoff, const uint32_t* code, uint32_t n_ins,
                          uint32_t n_consts, uint32_t n_lds, uint32_t nreg,
                          std::vector<uint32_t>& rec, MaskPool& pool);

// A register layout this library holds an interpreter for (slots, waves per
// SIMD, default LDS spill regions); nullptr for any other slot count.
struct mg_layout_info { uint32_t nreg, waves, lds_slots; };
const mg_layout_info* mg_find_layout(uint32_t nreg);

#endif
