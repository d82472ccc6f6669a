"""ctypes wrapper for the CPU oracle (oracle/gx_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product (genomics-rs_amd/).

Mirrors the reference's alignment path (nlaha/genomics-rs):
  alignment_table  src/alignment/algo.rs:151-282
  retrace          src/alignment/algo.rs:287-441
  is_match         src/sequence.rs:102-115
  from_fasta       src/sequence.rs:45-95
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

CHOICE_NAMES = ["Match", "Mismatch", "Insert", "Delete", "OpenInsert", "OpenDelete"]


class OResult(ctypes.Structure):
    _fields_ = [
        ("score", ctypes.c_int64),
        ("matches", ctypes.c_uint64),
        ("mismatches", ctypes.c_uint64),
        ("gap_extensions", ctypes.c_uint64),
        ("opening_gaps", ctypes.c_uint64),
        ("n_steps", ctypes.c_uint64),
        ("start_i", ctypes.c_uint64),
        ("start_j", ctypes.c_uint64),
        ("max_cell_i", ctypes.c_uint64),
        ("max_cell_j", ctypes.c_uint64),
        ("matches_at_max", ctypes.c_uint64),
        ("status", ctypes.c_int32),
        ("pad", ctypes.c_int32),
    ]


_lib = None


def build(native: bool = False, out: str | None = None) -> str:
    """Compile the oracle.  native=True builds an -march=native copy (the
    CPU-baseline build, mirroring .cargo/config.toml:2) at `out`."""
    src = os.path.join(HERE, "gx_oracle.c")
    if not native:
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
        return LIB_PATH
    out = out or os.path.join(HERE, "liboracle_native.so")
    subprocess.run(["gcc", "-O3", "-march=native", "-fPIC", "-std=c11", "-D_GNU_SOURCE",
                    "-shared", "-o", out, src], check=True)
    return out


def load(path: str | None = None):
    global _lib
    if path is None and _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        build()
    lib = ctypes.CDLL(p)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    lib.oracle_align.restype = ctypes.c_int
    lib.oracle_align.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t,
                                 ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                 ctypes.POINTER(OResult)]
    lib.oracle_align_lean.restype = ctypes.c_int
    lib.oracle_align_lean.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t,
                                      ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.POINTER(OResult), ctypes.c_void_p]
    lib.oracle_ref_layout_fill_rows.restype = ctypes.c_uint64
    lib.oracle_ref_layout_fill_rows.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t,
                                                ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                                ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64)]
    lib.oracle_fasta_parse.restype = ctypes.c_int
    lib.oracle_fasta_parse.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_size_t]
    if path is None:
        _lib = lib
    return lib


def _u8(b: bytes):
    arr = np.frombuffer(b, dtype=np.uint8) if len(b) else np.zeros(1, np.uint8)
    return arr, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


@dataclass
class OracleAlignment:
    score: int
    matches: int
    mismatches: int
    gap_extensions: int
    opening_gaps: int
    start: tuple
    max_cell: tuple
    matches_at_max: int
    choices: np.ndarray          # uint8, traceback order (end -> start)
    steps_i: np.ndarray          # uint64
    steps_j: np.ndarray          # uint64
    status: int
    planes: np.ndarray | None = None   # int64 [3, n+1, m+1]: I, D, S (row-major)
    lcs: np.ndarray | None = None      # uint64 [n+1, m+1]: max_matches()
    extra: dict = field(default_factory=dict)

    def alignment(self):
        """[(choice_name, i, j), ...] as in AlignedSequences.alignment."""
        return [(CHOICE_NAMES[c], int(i), int(j))
                for c, i, j in zip(self.choices, self.steps_i, self.steps_j)]


def align(s1: bytes, s2: bytes, scores=(1, -2, -1, -5), is_local=False, rev=False,
          layout: int = 0, want_planes=False, want_lcs=False) -> OracleAlignment:
    lib = load()
    n, m = len(s1), len(s2)
    a1, p1 = _u8(s1)
    a2, p2 = _u8(s2)
    cap = n + m + 2
    ch = np.zeros(cap, np.uint8)
    si = np.zeros(cap, np.uint64)
    sj = np.zeros(cap, np.uint64)
    planes = np.zeros((3, n + 1, m + 1), np.int64) if want_planes else None
    lcs = np.zeros((n + 1, m + 1), np.uint64) if want_lcs else None
    r = OResult()
    sm, smm, g, h = scores
    rc = lib.oracle_align(p1, n, p2, m, sm, smm, g, h, int(is_local), int(rev), layout,
                          planes.ctypes.data if planes is not None else None,
                          lcs.ctypes.data if lcs is not None else None,
                          ch.ctypes.data, si.ctypes.data, sj.ctypes.data, cap, ctypes.byref(r))
    if rc != 0:
        raise MemoryError("oracle_align failed")
    k = int(r.n_steps)
    return OracleAlignment(int(r.score), int(r.matches), int(r.mismatches), int(r.gap_extensions),
                           int(r.opening_gaps), (int(r.start_i), int(r.start_j)),
                           (int(r.max_cell_i), int(r.max_cell_j)), int(r.matches_at_max),
                           ch[:k].copy(), si[:k].copy(), sj[:k].copy(), int(r.status), planes, lcs)


def align_lean(s1: bytes, s2: bytes, scores=(1, -2, -1, -5), is_local=False) -> OracleAlignment:
    """Rolling-row restatement for large pairs (O(nm) bytes).  extra['plane_sums']
    holds the weighted checksums of the I, D, S planes."""
    lib = load()
    n, m = len(s1), len(s2)
    a1, p1 = _u8(s1)
    a2, p2 = _u8(s2)
    cap = n + m + 2
    ch = np.zeros(cap, np.uint8)
    si = np.zeros(cap, np.uint64)
    sj = np.zeros(cap, np.uint64)
    sums = np.zeros(3, np.uint64)
    r = OResult()
    sm, smm, g, h = scores
    rc = lib.oracle_align_lean(p1, n, p2, m, sm, smm, g, h, int(is_local), ch.ctypes.data, si.ctypes.data,
                               sj.ctypes.data, cap, ctypes.byref(r), sums.ctypes.data)
    if rc != 0:
        raise MemoryError("oracle_align_lean failed")
    k = int(r.n_steps)
    return OracleAlignment(int(r.score), int(r.matches), int(r.mismatches), int(r.gap_extensions),
                           int(r.opening_gaps), (int(r.start_i), int(r.start_j)),
                           (int(r.max_cell_i), int(r.max_cell_j)), int(r.matches_at_max),
                           ch[:k].copy(), si[:k].copy(), sj[:k].copy(), int(r.status),
                           extra={"plane_sums": [int(x) for x in sums]})


def ref_layout_fill_rows(s1: bytes, s2: bytes, rows: int, scores=(1, -2, -1, -5), is_local=False,
                         lib_path: str | None = None):
    """Time-able fill of the first `rows` rows in the reference's own layout.
    Returns (cells_updated, checksum)."""
    lib = load(lib_path) if lib_path else load()
    a1, p1 = _u8(s1)
    a2, p2 = _u8(s2)
    ck = ctypes.c_uint64(0)
    sm, smm, g, h = scores
    cells = lib.oracle_ref_layout_fill_rows(p1, len(s1), p2, len(s2), sm, smm, g, h, int(is_local),
                                            rows, ctypes.byref(ck))
    return int(cells), int(ck.value)


def fasta_parse(data: bytes):
    """from_fasta restatement on the bytes of one file -> [(name, seq), ...]."""
    lib = load()
    a, p = _u8(data)
    cap = len(data) + 16
    out = np.zeros(cap, np.uint8)
    rec_cap = data.count(b">") + 1
    no = np.zeros(rec_cap, np.uint64)
    nl = np.zeros(rec_cap, np.uint64)
    so = np.zeros(rec_cap, np.uint64)
    sl = np.zeros(rec_cap, np.uint64)
    k = lib.oracle_fasta_parse(p, len(data), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), cap,
                               no.ctypes.data, nl.ctypes.data, so.ctypes.data, sl.ctypes.data, rec_cap)
    if k < 0:
        raise ValueError("fasta parse capacity exceeded")
    ob = out.tobytes()
    res = []
    for r in range(k):
        res.append((ob[int(no[r]):int(no[r] + nl[r])], ob[int(so[r]):int(so[r] + sl[r])]))
    return res


def processed_bytes(s1: bytes, s2: bytes, rev: bool = False):
    """The bytes is_match compares (sequence.rs:102-115) as int arrays, None
    (an index past the end, incl. the usize wrap of len - i) as -1: row k of
    the table (k = i - 1) reads s1[len(s2) - k], column k reads s2[len(s1) - k]
    when rev, else s1[k] / s2[k]."""
    a = np.frombuffer(s1, np.uint8).astype(np.int32)
    b = np.frombuffer(s2, np.uint8).astype(np.int32)
    if not rev:
        return a, b
    n, m = len(a), len(b)
    c1 = np.full(n, -1, np.int32)
    c2 = np.full(m, -1, np.int32)
    for k in range(n):
        if k <= m and m - k < n:
            c1[k] = a[m - k]
    for k in range(m):
        if k <= n and n - k < m:
            c2[k] = b[n - k]
    return c1, c2


def lcs_rows(s1: bytes, s2: bytes, rows, rev: bool = False) -> dict:
    """max_matches(cell(i, j)) for every i in `rows` (a dict i -> int32 row
    of m + 1 values): the recurrence of algo.rs:250-256 (max of
    max_matches(i, j-1), max_matches(i-1, j), max_matches(i-1, j-1) +
    is_match), 0 on row 0 and column 0 (algo.rs:195-220).  Row by row in
    numpy: L(i, j) = max over k <= j of max(L(i-1, k), L(i-1, k-1) + is_match),
    the prefix max carrying the L(i, j-1) term."""
    c1, c2 = processed_bytes(s1, s2, rev)
    want = set(int(i) for i in rows)
    out = {}
    prev = np.zeros(len(c2) + 1, np.int32)
    if 0 in want:
        out[0] = prev.copy()
    top = max(want) if want else 0
    for i in range(1, top + 1):
        mt = (c2 == c1[i - 1]).astype(np.int32)
        t = np.maximum(prev[1:], prev[:-1] + mt)
        cur = np.empty_like(prev)
        cur[0] = 0
        np.maximum.accumulate(t, out=cur[1:])
        prev = cur
        if i in want:
            out[i] = cur.copy()
    return out
