"""Register layout per batch.

libmythgpu holds two interpreters (``mg_layouts``): 16 register slots at
three waves per SIMD with six LDS spill regions, and 11 slots in 128 VGPRs
at four waves with five.  A context runs one (``Engine(nreg=...)``), so a
batch picks its layout by the context it is loaded into — per launch, in one
process, no import-time switch.

Which layout wins depends on the programs.  The fourth wave fills VALU
issue slots, and the five fewer slots cost spills: a batch whose 16-slot
programs already keep values in per-lane scratch beyond the LDS tier gets
more of them at 11 slots, and scratch round trips are what such a batch
waits on.  Measured (alternated A/Bs on one box, ``profiles/r05/nreg/``,
round-5 compiler):

=========  ===========================================  ===================
workload   scratch spill slots per program at 16 slots  11 slots vs 16
=========  ===========================================  ===================
C2         1.80 (mean over the 4096 DAGs)               +3.7 %
C4         4.38                                          -1.5 %
C5         5.50                                          -11 %
C3         14.92                                         -11 %
=========  ===========================================  ===================

and the scratch count alone is not enough: with the round-6 schedule
choice C4's programs fell to 2.45 scratch slots at 16 (C2 1.77, C5 3.98,
C3 10.74: ``profiles/r06/r6p/`` ``config.layout_rule``; with the choice
gated on 10 scratch slots, C2 1.80, C4 4.00, C5 4.55, C3 10.96:
``profiles/r06/r6g/``), yet C4 on the four-wave layout lost 26-31 %
(``profiles/r06/sched/``).  What C2 has and
the query streams lack is heavy arithmetic: C2's programs are 8.5 % MUL /
division / umul_noovfl records (``ir.heavy_share``; every one of them at
least 1 %), C3 / C4 / C5 0.14 / 0 / 0.26 % — C2 is VALU-issue-bound (VALU
active 0.92 of SIMD cycles at three waves, 0.998 at four), the streams
wait on memory.  So the rule is: the four-wave layout when the batch's
16-slot programs average at least ``W4_MIN_HEAVY_SHARE`` heavy records AND
at most ``W4_MAX_SCRATCH_SLOTS`` scratch spill slots per program.  Both
statistics are static (the compiler's records and spill-slot count,
``Program.n_lds`` minus the 16-slot layout's LDS tier), known before
anything is launched.
"""

from typing import Sequence

from .ir import Program

DEFAULT = 16
FOUR_WAVES = 11
# mean scratch spill slots per 16-slot program at or below which a batch
# may run the four-wave layout (between C2's 1.80 and C4's 4.00, above)
W4_MAX_SCRATCH_SLOTS = 3.0
# mean share of heavy records (ir.heavy_share) at or above which it does
W4_MIN_HEAVY_SHARE = 0.02


def scratch_slots(p: Program) -> int:
    """Spill slots the program keeps in per-lane scratch at its layout (the
    compiler numbers spill slots lowest-free; those past the layout's LDS
    regions live in scratch)."""
    from .build import LAYOUT_LDS_SLOTS
    return max(0, p.n_lds - LAYOUT_LDS_SLOTS[p.nreg])


def mean_scratch_slots(progs: Sequence[Program]) -> float:
    return sum(scratch_slots(p) for p in progs) / max(1, len(progs))


def mean_heavy_share(progs: Sequence[Program]) -> float:
    from .ir import heavy_share
    return sum(heavy_share(p) for p in progs) / max(1, len(progs))


def choose(progs16: Sequence[Program]) -> int:
    """The register layout (slots) for a batch, from its programs compiled
    for the 16-slot layout."""
    if any(p.nreg != DEFAULT for p in progs16):
        raise ValueError("the rule reads 16-slot programs")
    if progs16 and mean_heavy_share(progs16) >= W4_MIN_HEAVY_SHARE and \
            mean_scratch_slots(progs16) <= W4_MAX_SCRATCH_SLOTS:
        return FOUR_WAVES
    return DEFAULT


def describe(nreg: int) -> str:
    from .build import LAYOUTS
    waves, lds = LAYOUTS[nreg]
    return "%d slots, %d waves/SIMD, %d LDS regions" % (nreg, waves, lds)
