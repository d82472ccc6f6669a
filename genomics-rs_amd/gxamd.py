"""gxamd -- Python mirror of the reference's alignment interface over the C ABI.

nlaha/genomics-rs exposes (src/lib.rs:3-6):
  sequence::{Sequence, SequenceContainer, SequenceOperations::{from_fasta, is_match}}
  config::{Scores, Config, get_config}
  alignment::algo::{alignment_table, retrace, AlignmentChoice, AlignedSequences}
This module offers the same names with the same argument meaning, backed by
libgx_amd.so (HIP kernels for gfx950 + C ABI declared in include/gx.h).

There is no CPU fallback: if libgx_amd.so is missing or no HIP device is
present, calls raise GxError.
"""
from __future__ import annotations

import ctypes
import enum
import logging
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence as Seq, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_log = logging.getLogger("gxamd")
LIB_PATH = os.environ.get("GX_LIB", os.path.join(_HERE, "libgx_amd.so"))

GX_TABLE_PLANES = 1
GX_TABLE_MATCHES = 2
GX_ALIGN_MAX_CELL = 4
GX_STAGED_PLANE_SUMS = 8
GX_STAGED_ALTERNATE = 16   # gx.h: pass k runs the k % 2 half of the staged pairs
GX_STAGED_KEEP_PLANES = 32   # gx.h: the last pass's planes stay on the device (gx_staged_table)

# status codes (include/gx.h)
_CODES = {0: "GX_OK", 1: "GX_EINVAL", 2: "GX_ESEQ", 3: "GX_ERANGE", 4: "GX_ENOMEM", 5: "GX_EHIP",
          6: "GX_EPANIC", 7: "GX_ECAP", 8: "GX_EIO", 9: "GX_EPARSE"}


class GxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{_CODES.get(code, code)}: {msg}")
        self.code = code


class CScores(ctypes.Structure):
    _fields_ = [("s_match", ctypes.c_int64), ("s_mismatch", ctypes.c_int64),
                ("g", ctypes.c_int64), ("h", ctypes.c_int64)]


class CCell(ctypes.Structure):
    _fields_ = [("insert_score", ctypes.c_int64), ("delete_score", ctypes.c_int64), ("sub_score", ctypes.c_int64),
                ("insert_matches", ctypes.c_uint64), ("delete_matches", ctypes.c_uint64),
                ("sub_matches", ctypes.c_uint64)]


class CStep(ctypes.Structure):
    _fields_ = [("choice", ctypes.c_uint8), ("pad", ctypes.c_uint8 * 7),
                ("i", ctypes.c_uint64), ("j", ctypes.c_uint64)]


class CResult(ctypes.Structure):
    _fields_ = [("score", ctypes.c_int64), ("matches", ctypes.c_uint64), ("mismatches", ctypes.c_uint64),
                ("gap_extensions", ctypes.c_uint64), ("opening_gaps", ctypes.c_uint64),
                ("n_steps", ctypes.c_uint64), ("start_i", ctypes.c_uint64), ("start_j", ctypes.c_uint64),
                ("max_cell_i", ctypes.c_uint64), ("max_cell_j", ctypes.c_uint64),
                ("matches_at_max", ctypes.c_uint64), ("fill_us", ctypes.c_int64), ("retrace_us", ctypes.c_int64)]


CELL_DTYPE = np.dtype([("insert_score", "<i8"), ("delete_score", "<i8"), ("sub_score", "<i8"),
                       ("insert_matches", "<u8"), ("delete_matches", "<u8"), ("sub_matches", "<u8")])
STEP_DTYPE = np.dtype([("choice", "u1"), ("pad", "u1", (7,)), ("i", "<u8"), ("j", "<u8")])

# exported symbols (include/gx.h) -- checked by tests/test_abi.py
EXPORTED = ["gx_last_error", "gx_version", "gx_context_create", "gx_context_destroy", "gx_context_trim",
            "gx_alignment_table", "gx_table_info", "gx_table_export", "gx_table_export_plane", "gx_table_export_rows",
            "gx_table_plane_sums", "gx_retrace", "gx_table_free", "gx_align", "gx_align_batch", "gx_align_batch_multi",
            "gx_stage_pairs",
            "gx_run_staged", "gx_run_staged_steps", "gx_staged_plane_sums", "gx_staged_steps",
            "gx_staged_pass_results", "gx_fill_info", "gx_batch_chunks", "gx_fill_twin", "gx_fill_groups", "gx_fill_plane_bits", "gx_plane_bytes_per_cell", "gx_twin_admission",
            "gx_twin_admission_mode", "gx_plan_layout", "gx_staged_table",
            "gx_fasta_load",
            "gx_config_load", "gx_format_alignment", "gx_format_table"]

_lib = None


def lib():
    """Load libgx_amd.so (raises if absent: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GxError(5, f"{LIB_PATH} not built (run `make -C genomics-rs_amd` or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, u8p = ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint8)
    L.gx_last_error.restype = ctypes.c_char_p
    L.gx_version.restype = ctypes.c_char_p
    L.gx_context_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.gx_context_destroy.argtypes = [vp]
    L.gx_context_destroy.restype = None
    L.gx_context_trim.argtypes = [vp]
    L.gx_alignment_table.argtypes = [vp, vp, sz, vp, sz, ctypes.POINTER(CScores), ctypes.c_int, ctypes.c_int,
                                     ctypes.c_uint32, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_uint64)]
    L.gx_table_info.argtypes = [vp] + [ctypes.POINTER(ctypes.c_uint64)] * 4 + [ctypes.POINTER(ctypes.c_int64)]
    L.gx_table_export.argtypes = [vp, vp, sz]
    L.gx_table_export_plane.argtypes = [vp, ctypes.c_int, vp, sz, ctypes.c_int]
    L.gx_table_export_rows.argtypes = [vp, ctypes.c_int, sz, sz, vp, sz]
    L.gx_table_plane_sums.argtypes = [vp, vp]
    L.gx_staged_plane_sums.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
    L.gx_staged_steps.argtypes = [vp, sz, vp, sz, ctypes.POINTER(sz)]
    L.gx_staged_pass_results.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
    L.gx_retrace.argtypes = [vp, ctypes.c_int, vp, sz, ctypes.POINTER(CResult)]
    L.gx_table_free.argtypes = [vp]
    L.gx_table_free.restype = None
    L.gx_align.argtypes = [vp, vp, sz, vp, sz, ctypes.POINTER(CScores), ctypes.c_int, ctypes.c_int,
                           ctypes.c_uint32, vp, sz, ctypes.POINTER(CResult)]
    L.gx_align_batch.argtypes = [vp, vp, vp, vp, vp, sz, ctypes.POINTER(CScores), ctypes.c_int, ctypes.c_uint32,
                                 vp, vp, vp]
    L.gx_align_batch_multi.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, sz, ctypes.POINTER(CScores), ctypes.c_int,
                                       ctypes.c_uint32, vp, vp, vp]
    L.gx_stage_pairs.argtypes = [vp, vp, vp, vp, vp, sz]
    L.gx_run_staged.argtypes = [vp, ctypes.POINTER(CScores), ctypes.c_int, ctypes.c_int, ctypes.c_uint32, vp,
                                ctypes.POINTER(ctypes.c_double)]
    L.gx_run_staged_steps.argtypes = [vp, ctypes.POINTER(CScores), ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                      ctypes.c_int, vp, ctypes.POINTER(ctypes.c_double)]
    L.gx_fill_info.argtypes = [vp] + [ctypes.POINTER(ctypes.c_int)] * 3
    L.gx_batch_chunks.argtypes = [vp]
    L.gx_fill_twin.argtypes = [vp]
    L.gx_fill_groups.argtypes = [vp]
    if hasattr(L, "gx_fill_plane_bits"):   # (absent from pre-12-bit builds run for A/B timing)
        L.gx_fill_plane_bits.argtypes = [vp]
    L.gx_plane_bytes_per_cell.argtypes = [ctypes.POINTER(CScores), ctypes.c_int]
    L.gx_twin_admission.argtypes = [ctypes.POINTER(CScores), ctypes.c_int, ctypes.c_int64,
                                    ctypes.POINTER(ctypes.c_int64)]
    L.gx_twin_admission_mode.argtypes = [ctypes.POINTER(CScores), ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                         ctypes.POINTER(ctypes.c_int64)]
    L.gx_staged_table.argtypes = [vp, sz, ctypes.POINTER(vp)]
    L.gx_plan_layout.argtypes = [ctypes.POINTER(CScores), ctypes.c_int, ctypes.POINTER(ctypes.c_int64),
                                 ctypes.POINTER(ctypes.c_int64), sz, ctypes.c_int, ctypes.c_int]
    L.gx_fasta_load.argtypes = [ctypes.c_char_p, vp, sz, vp, vp, vp, vp, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)]
    L.gx_config_load.argtypes = [ctypes.c_char_p, ctypes.POINTER(CScores)]
    L.gx_format_alignment.argtypes = [vp, sz, vp, sz, vp, sz, ctypes.POINTER(CResult), vp, sz, ctypes.POINTER(sz)]
    L.gx_format_table.argtypes = [vp, sz, vp, sz, vp, sz, vp, vp, vp, ctypes.c_int, vp, sz, ctypes.POINTER(sz)]
    _lib = L
    return L


def _check(rc: int):
    if rc != 0:
        raise GxError(rc, lib().gx_last_error().decode(errors="replace"))


def _buf(b: bytes):
    """Keep-alive numpy view of bytes and its address."""
    a = np.frombuffer(b, dtype=np.uint8) if len(b) else np.zeros(1, np.uint8)
    return a, a.ctypes.data


# ---------------------------------------------------------------------------
# config.rs

@dataclass
class Scores:
    """config::Scores (config.rs:6-13)."""
    s_match: int = 1
    s_mismatch: int = -2
    g: int = -1
    h: int = -5

    def c(self) -> CScores:
        return CScores(self.s_match, self.s_mismatch, self.g, self.h)


@dataclass
class Config:
    scores: Scores


def get_config(filepath: str) -> Config:
    """config::get_config (config.rs:21-40).  The reference exit(1)s on a read
    or parse error; this raises GxError (GX_EIO / GX_EPARSE) instead."""
    s = CScores()
    _check(lib().gx_config_load(filepath.encode(), ctypes.byref(s)))
    return Config(Scores(s.s_match, s.s_mismatch, s.g, s.h))


# ---------------------------------------------------------------------------
# sequence.rs

@dataclass
class Sequence:
    name: str
    sequence: str

    def __str__(self):  # sequence.rs:14-18
        return f"{self.name}: {self.sequence}"


@dataclass
class SequenceContainer:
    sequences: List[Sequence] = field(default_factory=list)

    def from_fasta(self, filepath: str) -> None:
        """from_fasta (sequence.rs:45-95): appends the file's records."""
        L = lib()
        nrec = ctypes.c_size_t(0)
        need = ctypes.c_size_t(0)
        # size query: the loader reports bytes/records needed when given no room
        rc = L.gx_fasta_load(filepath.encode(), None, 0, None, None, None, None, 0, ctypes.byref(nrec),
                             ctypes.byref(need))
        if rc not in (0, 7):
            _check(rc)
        k, nb = nrec.value, need.value
        if k == 0:
            return
        buf = np.zeros(max(nb, 1), np.uint8)
        arrs = [np.zeros(k, np.uint64) for _ in range(4)]
        _check(L.gx_fasta_load(filepath.encode(), buf.ctypes.data, buf.size, *[a.ctypes.data for a in arrs], k,
                               ctypes.byref(nrec), ctypes.byref(need)))
        raw = buf.tobytes()
        no, nl, so, sl = arrs
        for r in range(nrec.value):
            name = raw[int(no[r]):int(no[r] + nl[r])].decode("utf-8")
            seq = raw[int(so[r]):int(so[r] + sl[r])].decode("utf-8")
            self.sequences.append(Sequence(name, seq))

    def is_match(self, i: int, j: int, reverse_sequences: bool) -> bool:
        """is_match (sequence.rs:102-115), host-side (the fill evaluates it on the GPU)."""
        a = self.sequences[0].sequence.encode()
        b = self.sequences[1].sequence.encode()
        ip, jp = (len(b) - i, len(a) - j) if reverse_sequences else (i, j)
        x = a[ip] if 0 <= ip < len(a) else None
        y = b[jp] if 0 <= jp < len(b) else None
        return x == y


# ---------------------------------------------------------------------------
# alignment/algo.rs

class AlignmentChoice(enum.IntEnum):
    """#[repr(u8)] AlignmentChoice (algo.rs:124-133)."""
    Match = 0
    Mismatch = 1
    Insert = 2
    Delete = 3
    OpenInsert = 4
    OpenDelete = 5


@dataclass
class AlignedSequences:
    """algo.rs:135-146."""
    s1: Sequence
    s2: Sequence
    alignment: List[Tuple[AlignmentChoice, int, int]]
    score: int
    matches: int
    mismatches: int
    gap_extensions: int
    opening_gaps: int
    # beyond the reference struct: where the walk started, timings
    start: Tuple[int, int] = (0, 0)
    max_cell: Tuple[int, int] = (0, 0)
    matches_at_max: int = 0
    fill_us: int = 0
    retrace_us: int = 0
    _steps: Optional[np.ndarray] = None

    def __str__(self):
        """Display for AlignedSequences (display.rs:9-127)."""
        L = lib()
        a, pa = _buf(self.s1.sequence.encode())
        b, pb = _buf(self.s2.sequence.encode())
        steps = self._steps if self._steps is not None else _steps_array(self.alignment)
        res = CResult(self.score, self.matches, self.mismatches, self.gap_extensions, self.opening_gaps,
                      len(steps), 0, 0, 0, 0, 0, 0, 0)
        need = ctypes.c_size_t(0)
        L.gx_format_alignment(pa, len(self.s1.sequence.encode()), pb, len(self.s2.sequence.encode()),
                              steps.ctypes.data, len(steps), ctypes.byref(res), None, 0, ctypes.byref(need))
        out = ctypes.create_string_buffer(need.value)
        _check(L.gx_format_alignment(pa, len(self.s1.sequence.encode()), pb, len(self.s2.sequence.encode()),
                                     steps.ctypes.data, len(steps), ctypes.byref(res), out, need.value, None))
        return out.value.decode("utf-8")


def _steps_array(alignment) -> np.ndarray:
    arr = np.zeros(len(alignment), STEP_DTYPE)
    for k, (c, i, j) in enumerate(alignment):
        arr[k]["choice"] = int(c)
        arr[k]["i"] = i
        arr[k]["j"] = j
    return arr


def plane_bytes_per_cell(scores: "Scores", is_local: bool) -> int:
    """Score-plane bytes per cell of a batch launch with these scores: 3
    (compact byte differences) or 12 (int32 planes); gx_plane_bytes_per_cell.
    An upper bound: a launch that takes the twin fill writes 2 (its plane
    codes; Context.fill_info reports the launch's figure)."""
    r = lib().gx_plane_bytes_per_cell(ctypes.byref(scores.c()), int(is_local))
    if r < 0:
        raise GxError(3, "invalid scores")
    return r


def plan_layout(scores: "Scores", is_local: bool, shapes: Seq[Tuple[int, int]], track: bool = False,
                grid_cap: int = 0) -> int:
    """The fill layout a launch of these (n, m) pair shapes would take
    (gx_plan_layout; host rule only, no device): 0 anti-diagonal 128-row
    strips, 1 the column step, 3 the skewed 64-row strips; -1 invalid."""
    k = len(shapes)
    n = (ctypes.c_int64 * max(k, 1))(*[a for a, _ in shapes])
    m = (ctypes.c_int64 * max(k, 1))(*[b for _, b in shapes])
    return lib().gx_plan_layout(ctypes.byref(scores.c()), int(bool(is_local)), n, m, k, int(bool(track)),
                                int(grid_cap))


def twin_admission(scores: "Scores", band_waves: int, col_gap: int = 0, is_local: bool = False) -> Tuple[bool, int]:
    """The twin fill's int16 admission rule (gx_twin_admission_mode): (admitted,
    bound), bound = the largest |value - base| a band of `band_waves` strips
    can reach when a twin's pairs differ by up to col_gap columns."""
    b = ctypes.c_int64(0)
    r = lib().gx_twin_admission_mode(ctypes.byref(scores.c()), int(bool(is_local)), int(band_waves), int(col_gap),
                                     ctypes.byref(b))
    if r < 0:
        raise GxError(3, "invalid scores")
    return bool(r), int(b.value)


class Context:
    """One GPU: device-memory cache and stream (gx_context)."""

    def __init__(self, device: int = 0):
        p = ctypes.c_void_p()
        _check(lib().gx_context_create(device, ctypes.byref(p)))
        self.ptr = p
        self.device = device

    def close(self):
        if self.ptr:
            lib().gx_context_destroy(self.ptr)
            self.ptr = None

    def trim(self):
        _check(lib().gx_context_trim(self.ptr))

    def fill_info(self) -> dict:
        """The last fill launch: layout, band width, score-plane bytes per cell (gx_fill_info)."""
        v = [ctypes.c_int() for _ in range(3)]
        _check(lib().gx_fill_info(self.ptr, *[ctypes.byref(x) for x in v]))
        bits = lib().gx_fill_plane_bits(self.ptr) if hasattr(lib(), "gx_fill_plane_bits") else 8 * v[2].value
        return {"layout": v[0].value, "band_waves": v[1].value,
                "plane_bytes_per_cell": bits // 8 if bits % 8 == 0 else bits / 8,   # (twin codes: 1.5)
                "chunks": lib().gx_batch_chunks(self.ptr), "twin": lib().gx_fill_twin(self.ptr),
                "groups": lib().gx_fill_groups(self.ptr)}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx: dict = {}


def device_for_rank(local_rank: int) -> int:
    """HIP device of a local rank: GX_DEVICE_MAP="d0,d1,..." maps rank r to
    map[r % len] (several ranks may share one GPU, e.g. "0,0" to run the
    two-rank path on a one-GPU box); otherwise the rank itself."""
    dm = os.environ.get("GX_DEVICE_MAP", "")
    devs = [int(x) for x in dm.split(",") if x.strip()]
    return devs[local_rank % len(devs)] if devs else local_rank


def default_context(device: Optional[int] = None) -> Context:
    if device is None:
        device = device_for_rank(int(os.environ.get("LOCAL_RANK", "0"))) if "GX_DEVICE" not in os.environ \
            else int(os.environ["GX_DEVICE"])
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


class AlignmentTable:
    """A device-resident Array2<AlignmentCell> (gx_table).  Consumed by retrace()."""

    def __init__(self, ptr, s1: bytes, s2: bytes, flags: int):
        self.ptr = ptr
        self.s1, self.s2 = s1, s2
        self.flags = flags

    @property
    def shape(self):
        return (len(self.s1) + 1, len(self.s2) + 1)

    def info(self):
        v = [ctypes.c_uint64() for _ in range(4)]
        us = ctypes.c_int64()
        _check(lib().gx_table_info(self.ptr, *[ctypes.byref(x) for x in v], ctypes.byref(us)))
        return {"shape": (v[0].value, v[1].value), "max_cell": (v[2].value, v[3].value), "fill_us": us.value}

    def export(self) -> np.ndarray:
        """The full table as the reference's column-major Array2 (structured
        numpy array of shape (n+1, m+1), Fortran order, dtype == AlignmentCell)."""
        n1, m1 = self.shape
        out = np.zeros(n1 * m1, CELL_DTYPE)
        _check(lib().gx_table_export(self.ptr, out.ctypes.data, out.size))
        return out.reshape((n1, m1), order="F")

    def plane(self, which: int) -> np.ndarray:
        """int64 plane (0 insert, 1 delete, 2 sub), row-major (n+1, m+1)."""
        n1, m1 = self.shape
        out = np.zeros((n1, m1), np.int64)
        _check(lib().gx_table_export_plane(self.ptr, which, out.ctypes.data, out.size, 0))
        return out

    def rows(self, which: int, row0: int, nrows: int) -> np.ndarray:
        """int64 rows row0 .. row0+nrows-1 of plane `which`, shape (nrows, m+1)."""
        m1 = self.shape[1]
        out = np.zeros((nrows, m1), np.int64)
        _check(lib().gx_table_export_rows(self.ptr, which, row0, nrows, out.ctypes.data, out.size))
        return out

    def plane_sums(self) -> List[int]:
        """Device-side checksums of the I, D, S planes (gx_table_plane_sums):
        sum over interior cells of value * (1 + i*0x9E3779B1 + j*0x85EBCA77) mod 2^64."""
        out = np.zeros(3, np.uint64)
        _check(lib().gx_table_plane_sums(self.ptr, out.ctypes.data))
        return [int(x) for x in out]

    def free(self):
        if self.ptr:
            lib().gx_table_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _first_two(sc: SequenceContainer) -> Tuple[Sequence, Sequence]:
    if len(sc.sequences) < 2:
        # the reference panics with index out of bounds (algo.rs:169)
        raise GxError(2, "index out of bounds: fewer than two sequences in the container")
    return sc.sequences[0], sc.sequences[1]


def alignment_table(sequence_container: SequenceContainer, scores: Scores, is_local: bool,
                    reverse_sequences: bool, flags: int = GX_TABLE_PLANES,
                    ctx: Optional[Context] = None, max_cell: bool = True) -> Tuple[AlignmentTable, int]:
    """alignment_table (algo.rs:151-282) on the GPU -> (table, matches_at_max).

    max_cell=False skips the running max cell and matches_at_max (returned as
    0): the untracked fill, whose score planes are kept in the compact
    byte format (gx_api_plan.cpp d8_planes_ok) when the table is built on layout 0."""
    a, b = _first_two(sequence_container)
    if len(sequence_container.sequences) > 2:   # algo.rs:161-163
        _log.warning("More than two sequences found. Only the first two will be used.")
    s1, s2 = a.sequence.encode(), b.sequence.encode()
    ctx = ctx or default_context()
    x, px = _buf(s1)
    y, py = _buf(s2)
    t = ctypes.c_void_p()
    mam = ctypes.c_uint64()
    _check(lib().gx_alignment_table(ctx.ptr, px, len(s1), py, len(s2), ctypes.byref(scores.c()), int(is_local),
                                    int(reverse_sequences), flags, ctypes.byref(t),
                                    ctypes.byref(mam) if max_cell else None))
    return AlignmentTable(t, s1, s2, flags), int(mam.value)


DISP_MAX_WIDTH = 200  # display.rs:7


def _stdout_color() -> bool:
    """The `colored` crate's decision: a terminal, unless NO_COLOR / CLICOLOR=0
    (CLICOLOR_FORCE forces colour)."""
    import sys
    if os.environ.get("CLICOLOR_FORCE", "0") != "0":
        return True
    if os.environ.get("NO_COLOR") or os.environ.get("CLICOLOR") == "0":
        return False
    return sys.stdout.isatty()


def format_alignment_table(aligned: "AlignedSequences", planes, color: bool = False) -> str:
    """Text of print_alignment_table (display.rs:131-181) with its three
    print_scores_table blocks (display.rs:183-220).  `planes` = (insert,
    delete, sub) int64 row-major (n+1, m+1) arrays (AlignmentTable.plane);
    "" when the table is too large to visualise (display.rs:139-144)."""
    a = aligned.s1.sequence.encode()
    b = aligned.s2.sequence.encode()
    x, pa = _buf(a)
    y, pb = _buf(b)
    steps = aligned._steps if aligned._steps is not None else _steps_array(aligned.alignment)
    small = len(a) < DISP_MAX_WIDTH and len(b) < DISP_MAX_WIDTH * 10
    pl = [np.ascontiguousarray(p, dtype=np.int64) for p in planes] if small else [None, None, None]
    ptrs = [p.ctypes.data if p is not None else None for p in pl]
    need = ctypes.c_size_t(0)
    L = lib()
    L.gx_format_table(pa, len(a), pb, len(b), steps.ctypes.data, len(steps), *ptrs, int(color), None, 0,
                      ctypes.byref(need))
    out = ctypes.create_string_buffer(need.value)
    _check(L.gx_format_table(pa, len(a), pb, len(b), steps.ctypes.data, len(steps), *ptrs, int(color), out,
                             need.value, None))
    return out.value.decode("utf-8")


def print_alignment_table(aligned: "AlignedSequences", planes) -> None:
    """print_alignment_table (display.rs:131-181) to stdout."""
    import sys
    sys.stdout.write(format_alignment_table(aligned, planes, _stdout_color()))


def retrace(sequence_container: SequenceContainer, table: AlignmentTable, is_local: bool) -> AlignedSequences:
    """retrace (algo.rs:287-441).  Consumes `table`.  Like the reference
    (algo.rs:438) it ends by printing the sequence table for small inputs
    (tables filled with GX_TABLE_PLANES; set GX_NO_TABLE_PRINT=1 to skip)."""
    a, b = _first_two(sequence_container)
    cap = len(table.s1) + len(table.s2) + 2
    steps = np.zeros(cap, STEP_DTYPE)
    r = CResult()
    small = len(table.s1) < DISP_MAX_WIDTH and len(table.s2) < DISP_MAX_WIDTH * 10
    planes = None
    if small and (table.flags & GX_TABLE_PLANES) and not os.environ.get("GX_NO_TABLE_PRINT"):
        planes = [table.plane(k) for k in range(3)]   # before the table is consumed
    ptr, table.ptr = table.ptr, None
    _check(lib().gx_retrace(ptr, int(is_local), steps.ctypes.data, cap, ctypes.byref(r)))
    out = _aligned(a, b, steps[: r.n_steps], r)
    if planes is not None:
        print_alignment_table(out, planes)
    return out


def _aligned(a: Sequence, b: Sequence, steps: np.ndarray, r: CResult) -> AlignedSequences:
    ch = steps["choice"]
    ii = steps["i"]
    jj = steps["j"]
    alignment = [(AlignmentChoice(int(c)), int(i), int(j)) for c, i, j in zip(ch, ii, jj)]
    return AlignedSequences(a, b, alignment, r.score, r.matches, r.mismatches, r.gap_extensions, r.opening_gaps,
                            (r.start_i, r.start_j), (r.max_cell_i, r.max_cell_j), r.matches_at_max, r.fill_us,
                            r.retrace_us, steps)


def align_raw(s1: bytes, s2: bytes, scores: Scores, is_local: bool, reverse_sequences: bool = False,
              ctx: Optional[Context] = None, max_cell: bool = True):
    """Fused alignment_table + retrace on bytes -> (steps structured array, CResult).
    max_cell: also report alignment_table's max cell / matches_at_max."""
    ctx = ctx or default_context()
    x, px = _buf(s1)
    y, py = _buf(s2)
    cap = len(s1) + len(s2) + 2
    steps = np.zeros(cap, STEP_DTYPE)
    r = CResult()
    _check(lib().gx_align(ctx.ptr, px, len(s1), py, len(s2), ctypes.byref(scores.c()), int(is_local),
                          int(reverse_sequences), GX_ALIGN_MAX_CELL if max_cell else 0, steps.ctypes.data, cap,
                          ctypes.byref(r)))
    return steps[: r.n_steps], r


def align_batch(pairs: Seq[Tuple[bytes, bytes]], scores: Scores, is_local: bool, with_steps: bool = True,
                ctx: Optional[Context] = None, max_cell: bool = True):
    """Many independent pairs in one device launch -> list of (steps, CResult)."""
    ctx = ctx or default_context()
    P = len(pairs)
    keep = [(_buf(a), _buf(b)) for a, b in pairs]
    s1p = (ctypes.c_void_p * P)(*[k[0][1] for k in keep])
    s2p = (ctypes.c_void_p * P)(*[k[1][1] for k in keep])
    n = (ctypes.c_size_t * P)(*[len(a) for a, _ in pairs])
    m = (ctypes.c_size_t * P)(*[len(b) for _, b in pairs])
    res = (CResult * P)()
    steps_arr = [np.zeros(len(a) + len(b) + 2, STEP_DTYPE) for a, b in pairs] if with_steps else None
    stp = (ctypes.c_void_p * P)(*[s.ctypes.data for s in steps_arr]) if with_steps else None
    caps = (ctypes.c_size_t * P)(*[s.size for s in steps_arr]) if with_steps else None
    _check(lib().gx_align_batch(ctx.ptr, s1p, n, s2p, m, P, ctypes.byref(scores.c()), int(is_local),
                                GX_ALIGN_MAX_CELL if max_cell else 0, stp, caps, res))
    out = []
    for p in range(P):
        st = steps_arr[p][: res[p].n_steps] if with_steps else None
        out.append((st, res[p]))
    return out


def align_batch_multi(pairs: Seq[Tuple[bytes, bytes]], scores: Scores, is_local: bool, ctxs: Seq[Context],
                      with_steps: bool = True, max_cell: bool = True):
    """align_batch over several GPUs (gx_align_batch_multi): one context per
    device, the pairs shared out by longest-processing-time on n*m cells, one
    host thread per context -> list of (steps, CResult) in pair order."""
    P = len(pairs)
    keep = [(_buf(a), _buf(b)) for a, b in pairs]
    s1p = (ctypes.c_void_p * P)(*[k[0][1] for k in keep])
    s2p = (ctypes.c_void_p * P)(*[k[1][1] for k in keep])
    n = (ctypes.c_size_t * P)(*[len(a) for a, _ in pairs])
    m = (ctypes.c_size_t * P)(*[len(b) for _, b in pairs])
    res = (CResult * P)()
    steps_arr = [np.zeros(len(a) + len(b) + 2, STEP_DTYPE) for a, b in pairs] if with_steps else None
    stp = (ctypes.c_void_p * P)(*[s.ctypes.data for s in steps_arr]) if with_steps else None
    caps = (ctypes.c_size_t * P)(*[s.size for s in steps_arr]) if with_steps else None
    cp = (ctypes.c_void_p * len(ctxs))(*[c.ptr.value for c in ctxs])
    _check(lib().gx_align_batch_multi(cp, len(ctxs), s1p, n, s2p, m, P, ctypes.byref(scores.c()), int(is_local),
                                      GX_ALIGN_MAX_CELL if max_cell else 0, stp, caps, res))
    return [(steps_arr[p][: res[p].n_steps] if with_steps else None, res[p]) for p in range(P)]


class StagedPairs:
    """Pairs kept resident in HBM for repeated hot-path runs (bench.py)."""

    def __init__(self, pairs: Seq[Tuple[bytes, bytes]], ctx: Optional[Context] = None):
        self.ctx = ctx or default_context()
        self.P = len(pairs)
        self._keep = [(_buf(a), _buf(b)) for a, b in pairs]
        self._lens = [(len(a), len(b)) for a, b in pairs]
        s1p = (ctypes.c_void_p * self.P)(*[k[0][1] for k in self._keep])
        s2p = (ctypes.c_void_p * self.P)(*[k[1][1] for k in self._keep])
        n = (ctypes.c_size_t * self.P)(*[len(a) for a, _ in pairs])
        m = (ctypes.c_size_t * self.P)(*[len(b) for _, b in pairs])
        _check(lib().gx_stage_pairs(self.ctx.ptr, s1p, n, s2p, m, self.P))

    def run(self, scores: Scores, is_local: bool, keep_planes: bool = True, max_cell: bool = False,
            steps: int = 1, plane_sums: bool = False, alternate: bool = False, keep: bool = False):
        """`steps` back-to-back passes (pipelined one pass deep when > 1) ->
        (the last pass's results, mean fill ms).  plane_sums: also checksum
        every pass's score planes on the device (self.plane_sums()).
        alternate: pass k runs the k % 2 half of the staged pairs
        (GX_STAGED_ALTERNATE; the halves hold pairs of equal shapes).
        keep: the last pass's planes stay on the device (GX_STAGED_KEEP_PLANES)
        for self.table(p)."""
        res = (CResult * self.P)()
        fms = ctypes.c_double(0)
        flags = ((GX_ALIGN_MAX_CELL if max_cell else 0) | (GX_STAGED_PLANE_SUMS if plane_sums else 0)
                 | (GX_STAGED_ALTERNATE if alternate else 0) | (GX_STAGED_KEEP_PLANES if keep else 0))
        _check(lib().gx_run_staged_steps(self.ctx.ptr, ctypes.byref(scores.c()), int(is_local), int(keep_planes),
                                         flags, int(steps), res, ctypes.byref(fms)))
        return list(res), fms.value

    def table(self, pair: int) -> "AlignmentTable":
        """Staged pair `pair`'s score planes from the last run(keep=True), as
        an AlignmentTable (exports and checksums decode the batch format;
        gx_staged_table).  Its alignment is self.steps(pair)."""
        t = ctypes.c_void_p()
        _check(lib().gx_staged_table(self.ctx.ptr, pair, ctypes.byref(t)))
        (a, _), (b, _) = self._keep[pair]
        n, m = self._lens[pair]
        return AlignmentTable(t, bytes(a[:n]), bytes(b[:m]), GX_TABLE_PLANES)

    def plane_sums(self) -> np.ndarray:
        """uint64 [passes, pairs, 3] plane checksums of the last run(plane_sums=True)."""
        n = ctypes.c_size_t(0)
        _check(lib().gx_staged_plane_sums(self.ctx.ptr, None, 0, ctypes.byref(n)))
        out = np.zeros(max(n.value, 1), np.uint64)
        _check(lib().gx_staged_plane_sums(self.ctx.ptr, out.ctypes.data, out.size, ctypes.byref(n)))
        return out[: n.value].reshape(-1, self.P, 3)

    def pass_results(self) -> List[List["CResult"]]:
        """Every pass's per-pair results of the last run, [pass][pair] (gx_staged_pass_results)."""
        n = ctypes.c_size_t(0)
        _check(lib().gx_staged_pass_results(self.ctx.ptr, None, 0, ctypes.byref(n)))
        out = (CResult * max(n.value, 1))()
        _check(lib().gx_staged_pass_results(self.ctx.ptr, out, n.value, ctypes.byref(n)))
        rows = list(out)[: n.value]
        return [rows[k * self.P:(k + 1) * self.P] for k in range(n.value // max(self.P, 1))]

    def steps(self, pair: int) -> np.ndarray:
        """The alignment of staged pair `pair` from the last pass of the last run (STEP_DTYPE array)."""
        n = ctypes.c_size_t(0)
        _check(lib().gx_staged_steps(self.ctx.ptr, pair, None, 0, ctypes.byref(n)))
        out = np.zeros(max(n.value, 1), STEP_DTYPE)
        _check(lib().gx_staged_steps(self.ctx.ptr, pair, out.ctypes.data, out.size, ctypes.byref(n)))
        return out[: n.value]


# ---------------------------------------------------------------------------
# all-vs-all (BASELINE config 4)

def lpt_partition(weights: Seq[float], parts: int) -> List[List[int]]:
    """Longest-processing-time assignment of items (weight = n*m cells) to
    `parts` GPUs; each bin sorted.  Deterministic, so every rank computes the
    same plan without communicating."""
    order = sorted(range(len(weights)), key=lambda k: (-weights[k], k))
    bins: List[List[int]] = [[] for _ in range(parts)]
    load = [0.0] * parts
    for k in order:
        b = min(range(parts), key=lambda x: (load[x], x))
        bins[b].append(k)
        load[b] += weights[k]
    return [sorted(b) for b in bins]


def all_pairs(k: int, with_self: bool = True) -> List[Tuple[int, int]]:
    """(i, j) with i <= j (i < j without self pairs), in the reference compare
    matrix's fill order: row j, column i (main.rs:253-264)."""
    return [(i, j) for j in range(k) for i in range(j + 1) if i < j or with_self]


PAIR_FIELDS = ("score", "matches", "mismatches", "gap_extensions", "opening_gaps", "n_steps")


def _batch_stats(pairs, scores, is_local, ctx):
    """Product aligner for one rank's share: one gx_align_batch launch."""
    res = align_batch(pairs, scores, is_local, with_steps=False, ctx=ctx, max_cell=False)
    return [[getattr(r, f) for f in PAIR_FIELDS] for _, r in res]


def _pack(seqs: List[bytes]):
    lens = np.array([len(s) for s in seqs], np.int64)
    buf = np.frombuffer(b"".join(seqs), np.uint8) if lens.sum() else np.zeros(0, np.uint8)
    return lens, buf


def _broadcast_bytes_list(dist, items, device: str) -> List[bytes]:
    """Rank 0's list of byte strings on every rank (count + lengths, then the
    packed bytes: three broadcasts)."""
    import torch
    meta = torch.zeros(2, dtype=torch.int64, device=device)
    if dist.get_rank() == 0:
        lens, buf = _pack(items)
        meta[0], meta[1] = len(items), int(lens.sum())
    dist.broadcast(meta, 0)
    k, tot = int(meta[0]), int(meta[1])
    tl = torch.zeros(max(k, 1), dtype=torch.int64, device=device)
    tb = torch.zeros(max(tot, 1), dtype=torch.uint8, device=device)
    if dist.get_rank() == 0:
        if k:
            tl[:k].copy_(torch.from_numpy(lens))
        if tot:
            tb[:tot].copy_(torch.from_numpy(buf.copy()))
    dist.broadcast(tl, 0)
    dist.broadcast(tb, 0)
    lens = tl.cpu().numpy()[:k]
    raw = tb.cpu().numpy().tobytes()
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    return [raw[int(offs[x]):int(offs[x + 1])] for x in range(k)]


def all_vs_all(sequence_container: SequenceContainer, scores: Scores, is_local: bool = False,
               with_self: bool = True, ctx: Optional[Context] = None, dist=None, device: str = "cpu",
               align_fn=None) -> dict:
    """Align every pair (i <= j) of the container's sequences.

    dist = None: one GPU (ctx), one batched launch.  dist = torch.distributed
    (one process per GPU): rank 0's container is broadcast to every rank (the
    scatter; ≈30 KB per genome), each rank aligns its longest-processing-time
    share of the pairs, and the fixed-size per-pair records are all-gathered
    (RCCL over xGMI for backend "nccl", `device` = "cuda"; gloo on CPU).  No
    collective touches the DP data.  align_fn(pairs, scores, is_local) -> rows
    replaces the GPU aligner (tests of the plumbing only).

    Returns {"names", "lengths", "pairs", "records"}: records[p] = PAIR_FIELDS
    of pairs[p]; matrix(...) renders the reference's TSV layout."""
    align_fn = align_fn or (lambda prs, sc, loc: _batch_stats(prs, sc, loc, ctx or default_context()))
    seqs = [s.sequence.encode() for s in sequence_container.sequences]
    names = [s.name for s in sequence_container.sequences]
    if dist is not None:
        rank, world = dist.get_rank(), dist.get_world_size()
        # scatter: broadcast rank 0's packed sequences and names (utf-8)
        seqs = _broadcast_bytes_list(dist, seqs if rank == 0 else None, device)
        names = [x.decode("utf-8") for x in
                 _broadcast_bytes_list(dist, [x.encode("utf-8") for x in names] if rank == 0 else None, device)]
    else:
        rank, world = 0, 1
    pairs = all_pairs(len(seqs), with_self)
    weights = [float(len(seqs[i])) * len(seqs[j]) for i, j in pairs]
    mine = lpt_partition(weights, world)[rank]
    rows = align_fn([(seqs[pairs[p][0]], seqs[pairs[p][1]]) for p in mine], scores, is_local) if mine else []
    local = np.array([[p] + list(r) for p, r in zip(mine, rows)], np.int64).reshape(-1, 1 + len(PAIR_FIELDS))
    if dist is not None:
        import torch
        # gather: fixed-size records, padded to the largest share
        cap = max(len(b) for b in lpt_partition(weights, world))
        t = torch.full((cap, local.shape[1]), -1, dtype=torch.int64, device=device)
        if len(local):
            t[: len(local)].copy_(torch.from_numpy(local))
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        local = np.concatenate([x.cpu().numpy() for x in parts])
        local = local[local[:, 0] >= 0]
    records: List[Optional[List[int]]] = [None] * len(pairs)
    for row in local:
        records[int(row[0])] = [int(x) for x in row[1:]]
    if any(r is None for r in records):
        raise GxError(1, "all_vs_all: missing pair records after gather")
    return {"names": names, "lengths": [len(s) for s in seqs], "pairs": pairs, "records": records}


def similarity_tsv(result: dict, field: str = "score", blank_header: bool = False) -> str:
    """The reference compare writer's layout (main.rs:333-359): a header row of
    sequence indices, then row r = "r\\t" + one value per column; cells (r, c)
    with c <= r hold the pair's value, the rest 0 (never computed)."""
    k = len(result["lengths"])
    f = PAIR_FIELDS.index(field)
    cell = {(j, i): rec[f] for (i, j), rec in zip(result["pairs"], result["records"])}
    out = [(" \t" if blank_header else "\t") + "".join(f"{i}\t" for i in range(k)) + "\n"]
    for r in range(k):
        out.append(f"{r}\t" + "".join(f"{cell.get((r, c), 0)}\t" for c in range(k)) + "\n")
    return "".join(out)
