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
waits on.  Measured (alternated A/B on one box, ``profiles/r05/nreg/``):

=========  ===========================================  ===================
workload   scratch spill slots per program at 16 slots  11 slots vs 16
=========  ===========================================  ===================
C2         1.80 (mean over the 4096 DAGs)               +3.7 %
C4         4.38                                          -1.5 %
C5         5.50                                          -11 %
C3         14.92                                         -11 %
=========  ===========================================  ===================

so the rule is: the four-wave layout when the batch's 16-slot programs hold
at most ``W4_MAX_SCRATCH_SLOTS`` scratch spill slots per program on average.
The statistic is static (the compiler's spill-slot count, ``Program.n_lds``
minus the 16-slot layout's LDS tier), known before anything is launched.
"""

from typing import Sequence

from .ir import Program

DEFAULT = 16
FOUR_WAVES = 11
# mean scratch spill slots per 16-slot program at or below which a batch
# runs the four-wave layout (between C2's 1.80 and C4's 4.38, above)
W4_MAX_SCRATCH_SLOTS = 3.0


def scratch_slots(p: Program) -> int:
    """Spill slots the program keeps in per-lane scratch at its layout (the
    compiler numbers spill slots lowest-free; those past the layout's LDS
    regions live in scratch)."""
    from .build import LAYOUT_LDS_SLOTS
    return max(0, p.n_lds - LAYOUT_LDS_SLOTS[p.nreg])


def mean_scratch_slots(progs: Sequence[Program]) -> float:
    return sum(scratch_slots(p) for p in progs) / max(1, len(progs))


def choose(progs16: Sequence[Program]) -> int:
    """The register layout (slots) for a batch, from its programs compiled
    for the 16-slot layout."""
    if any(p.nreg != DEFAULT for p in progs16):
        raise ValueError("the rule reads 16-slot programs")
    return FOUR_WAVES if progs16 and mean_scratch_slots(progs16) <= W4_MAX_SCRATCH_SLOTS \
        else DEFAULT


def describe(nreg: int) -> str:
    from .build import LAYOUTS
    waves, lds = LAYOUTS[nreg]
    return "%d slots, %d waves/SIMD, %d LDS regions" % (nreg, waves, lds)
