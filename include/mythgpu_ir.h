/*
 * mythgpu IR — the compact postfix program the host compiler
 * (mythril_amd/ir.py) emits for one get_model constraint set.  The library
 * validates it and translates it into the records of the gfx950 assembly
 * interpreter (mythril_amd/asmgen.py, mg_interp_asm.hip), which executes it
 * per lane.
 *
 * One lane evaluates one candidate assignment.  Values are bit-vectors of
 * width 1..256 held as 8 little-endian 32-bit limbs, always canonical (bits
 * at and above the width are zero).  Bool is width 1.
 *
 * Instruction = 4 x uint32 (16 bytes, read by scalar loads, wave-uniform):
 *   w0 = op | width << 8 | flags         (width: result width, or operand
 *                                         width for comparisons / UMULNO;
 *                                         MG_ROOT_FLAG: result is a conjunct
 *                                         of the root, ROOT fused in)
 *   w1 = dst | a << 8 | b << 16 | c << 24 (register slots)
 *   w2 = imm0, w3 = imm1                 (per-op immediates, below)
 *
 * Register slots 0..nreg-1 of the context's register layout (16 slots:
 * MG_NREG, or 11: MG_NREG_W4; mg_layouts) live in VGPRs (per-limb
 * GPR-indexed vectors); slot nreg-1 also receives results nobody reads.  Values that do not fit are
 * spilled with SPILL/RELOAD: the first n_lds spill slots live in LDS, the
 * rest in per-lane scratch.  Every instruction writes `dst`.  The code array
 * is followed by 8 NOPs so the interpreter can prefetch ahead.
 *
 * The semantics of each op is SMT-LIB 2.6 FixedSizeBitVectors as z3 evaluates
 * it (bvudiv x 0 = ~0, bvurem x 0 = x, signed forms per the standard), the
 * theory the reference's get_model (mythril/support/model.py:15-49) hands to
 * z3.  Signed ops sign-extend their operands from `width` to 256 bits first.
 */
#ifndef MYTHGPU_IR_H
#define MYTHGPU_IR_H

#define MG_NREG 16           /* VGPR slots per lane (per-limb GPR-indexed
                                vectors) of the default register layout, and
                                the most any layout has: a context of the
                                four-wave layout holds MG_NREG_W4 (mg_layouts)
                                and its programs use slots 0..MG_NREG_W4-1   */
#define MG_NREG_W4 11        /* the four-wave layout (128 VGPRs)             */
#define MG_TRASH (MG_NREG - 1) /* result sink of the default layout           */
#define MG_LIMBS 8           /* 8 x 32-bit limbs = 256 bits                   */
#define MG_MAX_WIDTH 256
#define MG_MAX_LDS 10        /* LDS spill slots addressable by the IR; the
                                assembly kernel keeps the first 6 in LDS
                                (6 x 8 KiB per 256-lane block, 3 blocks per
                                CU) and the rest in per-lane scratch         */
#define MG_MAX_LDS_DS 8      /* LDS regions a context may use: compiled
                                programs address every half with a DS
                                instruction's 16-bit offset (16 halves x
                                4 KiB); more is refused when configured     */
#ifndef MG_MAX_PSLOTS        /* (A/B builds may override)                    */
#define MG_MAX_PSLOTS 240    /* further spill slots in per-lane scratch      */
#endif

enum mg_op {
    MG_NOP = 0,
    MG_CONST = 1,    /* dst = consts[imm0] (8 words)                          */
    MG_LEAF = 2,     /* dst = leaf value imm0 (input SoA or device generator) */
    MG_SPILL = 3,    /* spill[imm0] = R[a]  (imm0 < n_lds: LDS, else scratch) */
    MG_RELOAD = 4,   /* dst = spill[imm0]                                     */
    MG_ADD = 5,
    MG_SUB = 6,
    MG_MUL = 7,
    MG_UDIV = 8,
    MG_UREM = 9,
    MG_SDIV = 10,
    MG_SREM = 11,
    MG_SMOD = 12,
    MG_AND = 13,
    MG_OR = 14,
    MG_XOR = 15,
    MG_NOT = 16,     /* dst = ~a (masked)                                     */
    MG_SHL = 17,
    MG_LSHR = 18,
    MG_ASHR = 19,
    MG_EQ = 20,      /* Bool results; width = operand width                   */
    MG_ULT = 21,
    MG_ULE = 22,
    MG_SLT = 23,
    MG_SLE = 24,
    MG_UMULNO = 25,  /* a*b < 2^width                                         */
    MG_ITE = 26,     /* dst = R[c] ? R[a] : R[b]                              */
    MG_CONCAT = 27,  /* dst = R[a] << imm0 | R[b]   (imm0 = width of b)       */
    MG_EXTRACT = 28, /* dst = (R[a] >> imm0) masked to width                  */
    MG_SEXT = 29,    /* dst = sign_extend from imm0 bits to width             */
    MG_NEG = 30,
    MG_OUT = 31,     /* probe[imm0] = R[a]                                    */
    MG_ROOT = 32,    /* root &= R[a] & 1                                      */
    MG_MOV = 33,     /* dst = R[a]                                            */
    /* The calldata word LASER builds for CALLDATALOAD (reference
     * mythril/laser/ethereum/state/calldata.py:47-54,219-232):
     *   Concat_{i<32} If(off + i <s size, select(cd, off + i), 0)
     * over a free array read through its model table (entries (k_e, v_e) in
     * first-match order, then `else`), evaluated as one short chain instead
     * of 32 byte lookups (ir.py _calldata_word):
     *   w = BCAST(else); for e = E-1 .. 0: w = CDWE(w, k_e - off, v_e);
     *   word = CDWX(w, off, size)                                           */
    MG_BCAST = 34,   /* dst = byte 0 of R[a] in all 32 bytes (width 256)      */
    MG_CDWE = 35,    /* dst = R[a] with byte 31-d := R[c] & 0xff where        */
                     /*   d = R[b] < 32 (else R[a]); width 256                */
    MG_CDWX = 36,    /* dst = R[a] with byte 31-i := 0 for every i < 32 where */
                     /*   !(R[b] + i <s R[c]) (256-bit wrapping add); width 256 */
    MG_NUM_OPS = 37
};

#define MG_ROOT_FLAG (1u << 18)

#define MG_INS_W0(op, width) ((unsigned)(op) | ((unsigned)(width) << 8))
#define MG_INS_W1(d, a, b, c) \
    ((unsigned)(d) | ((unsigned)(a) << 8) | ((unsigned)(b) << 16) | ((unsigned)(c) << 24))

/* Device leaf generator classes (mg_leafgen.kind thresholds, percent). */
#define MG_GEN_UNIFORM 0
#define MG_GEN_SMALL 1
#define MG_GEN_BOUNDARY 2
#define MG_GEN_POOL 3

#endif
