"""ctypes binding of libmythgpu (include/mythgpu.h).

The product path has no CPU evaluator: if the shared library or the GPU is
missing, :func:`get_engine` raises :class:`EngineUnavailable` and the caller
(``mythril_amd.model.get_model``) falls back to z3 — never to a host
re-implementation.
"""

from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .ir import Program


def _default_lib() -> str:
    from .build import LIB
    return LIB


# One library holds the interpreter of every register layout (build.LAYOUTS;
# a context runs one, Engine(nreg=...)).  MYTHGPU_LIB: an A/B build of the
# same ABI.
_LIB_PATH = os.environ.get("MYTHGPU_LIB") or _default_lib()

EXPORTS = ("mg_init", "mg_init_layout", "mg_layouts", "mg_free", "mg_last_error",
           "mg_device_info", "mg_load_program", "mg_free_program", "mg_eval", "mg_eval_gen",
           "mg_search", "mg_batch_create", "mg_batch_free", "mg_batch_eval_gen", "mg_batch_search",
           "mg_batch_search_probes", "mg_keccak256", "mg_version", "mg_config", "mg_translate",
           "mg_asm_digest", "mg_asm_digest_layout", "mg_last_kernel_ms", "mg_jit_attach",
           "mg_jit_detach", "mg_runtime_info")


def layouts() -> Dict[int, Tuple[int, int]]:
    """slots -> (waves per SIMD, default LDS spill regions) of every register
    layout the library holds (mg_layouts; build.LAYOUTS)."""
    lib = load_library(check_digest=False)
    buf = (C.c_uint32 * 24)()
    n = lib.mg_layouts(buf, 24)
    return {int(buf[3 * i]): (int(buf[3 * i + 1]), int(buf[3 * i + 2])) for i in range(n)}


def lds_slots_for(nreg: int) -> int:
    """LDS spill regions a context of the ``nreg``-slot layout uses (the
    compiled programs of a batch are rendered for the same): the layout's
    default, or ``MYTHGPU_LDS_SLOTS``."""
    from . import irdefs
    if "MYTHGPU_LDS_SLOTS" in os.environ:
        return irdefs.check_lds_slots(os.environ["MYTHGPU_LDS_SLOTS"])
    from .build import LAYOUT_LDS_SLOTS
    return LAYOUT_LDS_SLOTS[nreg]


class EngineUnavailable(RuntimeError):
    """No usable engine; ``slot`` > 0 when only an extra context of a device
    (model.DEVICES listing it again) could not be created."""

    def __init__(self, msg: str = "", slot: int = 0, device: int = 0):
        super().__init__(msg)
        self.slot = slot
        self.device = device


class EngineError(RuntimeError):
    pass


class LeafGen(C.Structure):
    _fields_ = [("width", C.c_uint32), ("pool_off", C.c_uint32), ("pool_n", C.c_uint32),
                ("pct_uniform", C.c_uint32), ("pct_small", C.c_uint32),
                ("pct_boundary", C.c_uint32)]


class Gen(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("first_index", C.c_uint64)]


_libs: Dict[str, object] = {}
_lib_lock = threading.Lock()


def load_library(path: str = _LIB_PATH, check_digest: bool = True):
    """Load libmythgpu.so (no GPU needed) and declare every export.  Other
    paths (A/B builds of the same ABI) load side by side."""
    with _lib_lock:
        if path in _libs:
            return _libs[path]
        if not os.path.exists(path):
            raise EngineUnavailable("libmythgpu.so not built (%s); run "
                                    "`python -m mythril_amd.build`" % path)
        try:
            lib = C.CDLL(path)
        except OSError as e:            # e.g. the HIP runtime it links is missing
            raise EngineUnavailable("cannot load %s: %s" % (path, e)) from e
        p, u32, u64, i64 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int64
        lib.mg_version.restype = C.c_int
        lib.mg_init.argtypes = [C.c_int, C.POINTER(p)]
        lib.mg_init_layout.argtypes = [C.c_int, u32, C.POINTER(p)]
        lib.mg_layouts.argtypes = [p, u32]
        lib.mg_asm_digest_layout.argtypes = [u32]
        lib.mg_asm_digest_layout.restype = C.c_char_p
        lib.mg_free.argtypes = [p]
        lib.mg_free.restype = None
        lib.mg_last_error.argtypes = [p]
        lib.mg_last_error.restype = C.c_char_p
        lib.mg_device_info.argtypes = [p, C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]
        lib.mg_load_program.argtypes = [p, p, u32, p, u32, p, u32, u32, u32, u64, C.POINTER(p)]
        lib.mg_free_program.argtypes = [p]
        lib.mg_free_program.restype = None
        lib.mg_eval.argtypes = [p, p, p, u64, p, p]
        lib.mg_eval_gen.argtypes = [p, p, C.POINTER(Gen), u64, p, p, p]
        lib.mg_search.argtypes = [p, p, C.POINTER(Gen), u64, C.POINTER(i64), p]
        lib.mg_batch_create.argtypes = [p, C.POINTER(p), u32, C.POINTER(p)]
        lib.mg_batch_free.argtypes = [p]
        lib.mg_batch_free.restype = None
        lib.mg_batch_eval_gen.argtypes = [p, p, u64, u64, u64, p, p, p]
        lib.mg_batch_search.argtypes = [p, p, C.POINTER(Gen), u64, p, p, u32]
        lib.mg_batch_search_probes.argtypes = [p, p, C.POINTER(Gen), u64, p, p, u32, p, u32]
        lib.mg_keccak256.argtypes = [p, p, p, p, u32, p]
        lib.mg_config.argtypes = [p, u32]
        lib.mg_asm_digest.restype = C.c_char_p
        lib.mg_last_kernel_ms.argtypes = [p]
        lib.mg_last_kernel_ms.restype = C.c_float
        lib.mg_jit_attach.argtypes = [p, C.POINTER(p), u32, p, C.c_size_t, C.POINTER(p)]
        lib.mg_jit_detach.argtypes = [p]
        lib.mg_jit_detach.restype = None
        lib.mg_runtime_info.argtypes = [C.POINTER(C.c_int), C.c_char_p, C.c_size_t]
        pu32 = C.POINTER(u32)
        lib.mg_translate.argtypes = [p, u32, u32, u32, u32, p, u32, p, u32, pu32, p, u32, pu32]
        for name in EXPORTS:
            getattr(lib, name)
        if check_digest:
            # every layout's interpreter must be the one this generator
            # makes (a stale build is refused; ADVICE r5: and the slot count
            # the compiler allocates must be a layout the library holds)
            from . import asmgen
            from .build import LAYOUTS
            for nreg in sorted(LAYOUTS):
                with asmgen.layout(nreg):
                    want = asmgen.digest()
                got = lib.mg_asm_digest_layout(nreg)
                got = got.decode() if got else None
                if got != want:
                    raise EngineUnavailable(
                        "%s was built from a different assembly interpreter for %d slots "
                        "(digest %s, generator %s); rebuild with `python -m mythril_amd.build`"
                        % (path, nreg, got, want))
            _libs[path] = lib
        return lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def default_leafgen(program: Program, pct=(50, 70, 85)) -> List[LeafGen]:
    """C2 value distribution: 50 % uniform, 20 % < 2^64, 15 %
    boundary values, 15 % DAG constants +-1 (pool = the program's constants)."""
    n_c = len(program.const_values)
    widths = getattr(program.leaves, "widths", None) or [l.width for l in program.leaves]
    return [LeafGen(w, 0, n_c, pct[0], pct[1], pct[2]) for w in widths]


class LoadedProgram:
    def __init__(self, engine: "Engine", program: Program, handle):
        self.engine = engine
        self.program = program
        self.handle = handle

    def __del__(self):
        try:
            if self.handle and self.engine._ctx:
                self.engine.lib.mg_free_program(self.handle)
        except Exception:
            pass
        self.handle = None


class Engine:
    """One HIP device context (one per host thread)."""

    def __init__(self, device: int = 0, lib_path: str = _LIB_PATH, nreg: Optional[int] = None):
        """A context on ``device`` running the ``nreg``-slot register layout
        (default: the process's, ``irdefs.NREG``; 16, or 11 for four waves
        per SIMD): programs compiled for that many slots load into it."""
        # an A/B build elsewhere may carry another assembly interpreter
        self.lib = load_library(lib_path, check_digest=lib_path == _LIB_PATH)
        ctx = C.c_void_p()
        from . import irdefs
        self.nreg = irdefs.NREG if nreg is None else int(nreg)
        try:
            self.lds_slots = lds_slots_for(self.nreg)     # (mg_init refuses a bad one too)
        except (KeyError, ValueError) as e:
            raise EngineUnavailable("register layout %d / MYTHGPU_LDS_SLOTS: %s"
                                    % (self.nreg, e)) from e
        rc = self.lib.mg_init_layout(device, self.nreg, C.byref(ctx))
        if rc != 0:
            raise EngineUnavailable("mg_init_layout(%d, %d) failed with %d (no usable GPU?)"
                                    % (device, self.nreg, rc))
        self._ctx = ctx
        name = C.create_string_buffer(256)
        cus = C.c_int()
        self.lib.mg_device_info(ctx, name, 256, C.byref(cus))
        self.device_name = name.value.decode()
        self.n_cus = cus.value

    def close(self):
        if self._ctx:
            self.lib.mg_free(self._ctx)
            self._ctx = None

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise EngineError("%s failed (%d): %s" % (what, rc,
                              self.lib.mg_last_error(self._ctx).decode(errors="replace")))

    def runtime_info(self) -> dict:
        """The HIP runtime the library runs on in this process (version,
        libamdhip64 file)."""
        v = C.c_int()
        path = C.create_string_buffer(1024)
        self.lib.mg_runtime_info(C.byref(v), path, 1024)
        return {"hip_runtime_version": v.value, "libamdhip64": path.value.decode()}

    def last_kernel_ms(self) -> float:
        """Device time of the last synchronous eval / search call."""
        return float(self.lib.mg_last_kernel_ms(self._ctx))

    def load(self, program: Program, leafgen: Optional[Sequence[LeafGen]] = None,
             prog_seed: int = 0) -> LoadedProgram:
        if program.nreg != self.nreg:
            raise EngineError("program compiled for %d register slots, this context runs the "
                              "%d-slot layout" % (program.nreg, self.nreg))
        code = np.ascontiguousarray(program.code, dtype=np.uint32)
        consts = np.ascontiguousarray(program.consts, dtype=np.uint32)
        gens = list(leafgen) if leafgen is not None else default_leafgen(program)
        garr = (LeafGen * max(1, len(gens)))(*gens)
        h = C.c_void_p()
        rc = self.lib.mg_load_program(self._ctx, _ptr(code), code.shape[0], _ptr(consts),
                                      consts.shape[0], C.cast(garr, C.c_void_p), len(gens),
                                      program.n_lds, program.n_probes, prog_seed & (2**64 - 1),
                                      C.byref(h))
        self._check(rc, "mg_load_program")
        return LoadedProgram(self, program, h)

    def eval(self, lp: LoadedProgram, leaves_soa: np.ndarray, want_probes: bool = False):
        """leaves_soa: (n_leaves, 8, n) uint32.  Returns (root bool array,
        probes (n_probes, 8, n) uint32 or None)."""
        prog = lp.program
        leaves_soa = np.ascontiguousarray(leaves_soa, dtype=np.uint32)
        n = leaves_soa.shape[2] if leaves_soa.ndim == 3 else 0
        if leaves_soa.shape[:2] != (len(prog.leaves), 8):
            raise ValueError("leaves_soa must be (n_leaves, 8, n)")
        bits = np.zeros((n + 63) // 64, dtype=np.uint64)
        probes = np.zeros((prog.n_probes, 8, n), dtype=np.uint32) if want_probes else None
        rc = self.lib.mg_eval(self._ctx, lp.handle, _ptr(leaves_soa), n, _ptr(bits), _ptr(probes))
        self._check(rc, "mg_eval")
        return unpack_bits(bits, n), probes

    def eval_gen(self, lp: LoadedProgram, seed: int, first_index: int, n: int,
                 want_probes: bool = False, want_leaves: bool = False):
        prog = lp.program
        bits = np.zeros((n + 63) // 64, dtype=np.uint64)
        probes = np.zeros((prog.n_probes, 8, n), dtype=np.uint32) if want_probes else None
        leaves = np.zeros((len(prog.leaves), 8, n), dtype=np.uint32) if want_leaves else None
        g = Gen(seed & (2**64 - 1), first_index)
        rc = self.lib.mg_eval_gen(self._ctx, lp.handle, C.byref(g), n, _ptr(bits), _ptr(probes),
                                  _ptr(leaves))
        self._check(rc, "mg_eval_gen")
        return unpack_bits(bits, n), probes, leaves

    def search(self, lp: LoadedProgram, seed: int, n_cand: int,
               first_index: int = 0) -> Tuple[int, Optional[np.ndarray]]:
        prog = lp.program
        first = C.c_int64(-1)
        wit = np.zeros((max(1, len(prog.leaves)), 8), dtype=np.uint32)
        g = Gen(seed & (2**64 - 1), first_index)
        rc = self.lib.mg_search(self._ctx, lp.handle, C.byref(g), n_cand, C.byref(first),
                                _ptr(wit))
        self._check(rc, "mg_search")
        if first.value < 0:
            return -1, None
        return first.value, wit[:len(prog.leaves)]

    def witness(self, lp: LoadedProgram, seed: int, index: int):
        """Leaves and probe values of candidate ``index`` (one lane): what a
        solve-mode program's model needs besides the generated leaves."""
        _, probes, leaves = self.eval_gen(lp, seed, index, 1, want_probes=True, want_leaves=True)
        return leaves[:, :, 0], (probes[:, :, 0] if probes is not None else None)

    def keccak256(self, msgs: Sequence[bytes]) -> List[bytes]:
        n = len(msgs)
        if n == 0:
            return []
        lens = np.array([len(m) for m in msgs], dtype=np.uint32)
        offs = np.zeros(n, dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        data = np.frombuffer(b"".join(msgs) or b"\0", dtype=np.uint8).copy()
        out = np.zeros((n, 32), dtype=np.uint8)
        rc = self.lib.mg_keccak256(self._ctx, _ptr(data), _ptr(offs), _ptr(lens), n, _ptr(out))
        self._check(rc, "mg_keccak256")
        return [bytes(out[i]) for i in range(n)]

    # corpus batches (device pointers; used by bench.py)
    def batch_create(self, loaded: Sequence[LoadedProgram]):
        arr = (C.c_void_p * len(loaded))(*[lp.handle for lp in loaded])
        h = C.c_void_p()
        rc = self.lib.mg_batch_create(self._ctx, arr, len(loaded), C.byref(h))
        self._check(rc, "mg_batch_create")
        return h

    def batch_free(self, h):
        self.lib.mg_batch_free(h)

    def jit_attach(self, loaded: Sequence[LoadedProgram], image: bytes):
        """Point the programs at their compiled code (``jit.compile_batch``
        of the same programs, leaf generators and seeds, in order); returns
        the handle for :meth:`jit_detach`.  Attach before ``batch_create``."""
        arr = (C.c_void_p * len(loaded))(*[lp.handle for lp in loaded])
        buf = C.create_string_buffer(image, len(image))
        h = C.c_void_p()
        rc = self.lib.mg_jit_attach(self._ctx, arr, len(loaded), C.cast(buf, C.c_void_p),
                                    len(image), C.byref(h))
        self._check(rc, "mg_jit_attach")
        return h

    def jit_detach(self, h):
        self.lib.mg_jit_detach(h)

    def batch_eval_gen(self, h, seed: int, first_index: int, n_assign: int,
                       d_root_bits: int = 0, d_first_sat: int = 0, stream: int = 0):
        rc = self.lib.mg_batch_eval_gen(self._ctx, h, seed & (2**64 - 1), first_index, n_assign,
                                        C.c_void_p(d_root_bits or None),
                                        C.c_void_p(d_first_sat or None), C.c_void_p(stream or None))
        self._check(rc, "mg_batch_eval_gen")


    def batch_search(self, loaded: Sequence[LoadedProgram], seed: int, n_cand: int,
                     first_index: int = 0, want_probes: bool = False) -> List[tuple]:
        """Witness search over many programs in shared launches
        (mg_batch_search, witnesses regenerated in one launch); per program
        (index, leaves) or (-1, None) — with ``want_probes`` (index, leaves,
        probes) or (-1, None, None), the probe values coming from the same
        regeneration launch (mg_batch_search_probes)."""
        if not loaded:
            return []
        h = self.batch_create(loaded)
        max_leaves = max(1, max(len(lp.program.leaves) for lp in loaded))
        max_probes = max(1, max(lp.program.n_probes for lp in loaded))
        try:
            first = np.full(len(loaded), -1, dtype=np.int64)
            wit = np.zeros((len(loaded), max_leaves, 8), dtype=np.uint32)
            g = Gen(seed & (2**64 - 1), first_index)
            if want_probes:
                prb = np.zeros((len(loaded), max_probes, 8), dtype=np.uint32)
                rc = self.lib.mg_batch_search_probes(self._ctx, h, C.byref(g), n_cand, _ptr(first),
                                                     _ptr(wit), max_leaves, _ptr(prb), max_probes)
                self._check(rc, "mg_batch_search_probes")
            else:
                rc = self.lib.mg_batch_search(self._ctx, h, C.byref(g), n_cand, _ptr(first),
                                              _ptr(wit), max_leaves)
                self._check(rc, "mg_batch_search")
        finally:
            self.batch_free(h)
        out = []
        for k, (lp, f) in enumerate(zip(loaded, first.tolist())):
            if not want_probes:
                out.append((-1, None) if f < 0 else (f, wit[k, :len(lp.program.leaves)].copy()))
            else:
                out.append((-1, None, None) if f < 0 else
                           (f, wit[k, :len(lp.program.leaves)].copy(),
                            prb[k, :lp.program.n_probes].copy()))
        return out


def translate_records(program: Program, lds_slots: Optional[int] = None):
    """Host-only (no GPU): the records ``mg_load_program`` would upload for
    ``program`` with handler IDS in word 0 (the translator run with an
    identity offset table; the last record is the zeroed prefetch pad), and
    the number of mask entries the translator appended to the constant
    table.  ``lds_slots`` is the context's LDS spill tier (``lds_slots_for``
    the program's layout).  The translator is the one of the program's
    register layout (``Program.nreg``)."""
    from . import asmgen
    if lds_slots is None:
        lds_slots = lds_slots_for(program.nreg)
    lib = load_library()
    code = np.ascontiguousarray(program.code, dtype=np.uint32)
    n_ins = code.shape[0]
    ident = np.arange(asmgen.NUM_HANDLERS, dtype=np.uint32)
    max_rec = (2 * n_ins + 3) * 8
    max_mask = (2 * n_ins + 4) * 16
    rec = np.zeros(max_rec, dtype=np.uint32)
    masks = np.zeros(max_mask, dtype=np.uint32)
    nrw, nmw = C.c_uint32(), C.c_uint32()
    rc = lib.mg_translate(_ptr(code), n_ins, program.consts.shape[0],
                          min(program.n_lds, lds_slots), program.nreg, _ptr(ident),
                          asmgen.NUM_HANDLERS,
                          C.cast(rec.ctypes.data, C.POINTER(C.c_uint32)), max_rec, C.byref(nrw),
                          _ptr(masks), max_mask, C.byref(nmw))
    if rc != 0:
        raise EngineError("mg_translate failed (%d)" % rc)
    return rec[:nrw.value], nmw.value // 8


def record_handlers(program: Program, lds_slots: Optional[int] = None) -> List[int]:
    """The assembly-interpreter handler id of every record, in order."""
    rec, _ = translate_records(program, lds_slots)
    return [int(h) for h in rec[::8][:-1]]       # the last record is a zeroed pad


def handler_variants(program: Program, lds_slots: Optional[int] = None):
    """The set of (family, canonical variant) the program executes (every
    record runs on every lane: programs are straight-line)."""
    from . import asmgen
    out = set()
    hs = record_handlers(program, lds_slots)
    with asmgen.layout(program.nreg):
        for h in hs:
            c = asmgen.canonical(h)
            aop, var = c // (2 * asmgen.NVAR), (c // 2) % asmgen.NVAR
            out.add((asmgen.AOPS[aop], var))
    return out


def unpack_bits(bits: np.ndarray, n: int) -> np.ndarray:
    b = np.unpackbits(bits.view(np.uint8), bitorder="little")
    return b[:n].astype(bool)


def int_to_limbs(v: int) -> List[int]:
    return [(v >> (32 * j)) & 0xFFFFFFFF for j in range(8)]


def limbs_to_int(limbs) -> int:
    v = 0
    for j in reversed(range(8)):
        v = (v << 32) | int(limbs[j])
    return v


_engines: Dict[Tuple[int, int, int], Engine] = {}
_failed: Dict[Tuple[int, int], str] = {}
_engines_lock = threading.Lock()


def get_engine(device: int = 0, slot: int = 0, nreg: Optional[int] = None) -> Engine:
    """The engine (one HIP context) of ``device`` running the ``nreg``-slot
    register layout (default: the process's); ``slot`` > 0 gives further
    independent contexts on the same device (a device listed twice in
    ``MYTHRIL_GPU_DEVICES`` is searched from two host threads, and a context
    serves one thread at a time).  An initialisation failure is remembered
    per (device, slot), so later calls raise EngineUnavailable at once
    instead of retrying mg_init; a failed extra slot (e.g. out of memory for
    one more context) does not mark the device's first context failed, and
    the exception carries ``slot`` so callers can tell the two apart."""
    from . import irdefs
    nreg = irdefs.NREG if nreg is None else int(nreg)
    with _engines_lock:
        e = _engines.get((device, slot, nreg))
        if e is None:
            for key in ((device, 0), (device, slot)):
                if key in _failed:
                    raise EngineUnavailable(_failed[key], slot=key[1], device=device)
            try:
                e = Engine(device, nreg=nreg)
            except EngineUnavailable as x:
                _failed[(device, slot)] = str(x)
                raise EngineUnavailable(str(x), slot=slot, device=device) from x
            except Exception as x:  # noqa: BLE001 - any init failure means no engine
                _failed[(device, slot)] = "%s: %s" % (type(x).__name__, x)
                raise EngineUnavailable(_failed[(device, slot)], slot=slot, device=device) from x
            _engines[(device, slot, nreg)] = e
        return e


def device_slots(devices) -> List[Tuple[int, int]]:
    """(device, slot) per entry of a device list: the k-th repeat of a device
    gets slot k, its own context."""
    seen: Dict[int, int] = {}
    out = []
    for d in devices:
        out.append((d, seen.get(d, 0)))
        seen[d] = seen.get(d, 0) + 1
    return out
