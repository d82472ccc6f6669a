/*
 * gx.h -- C ABI of genomics-rs_amd: an MI355X (gfx950) drop-in for the
 * affine-gap alignment path of nlaha/genomics-rs.
 *
 * Every entry point replaces one item of the reference's public Rust API
 * (src/lib.rs:3-6 re-exports alignment, config, sequence).  A Rust shim binds
 * these 1:1 with `extern "C"`.  Plain pointers and sizes
 * only; host memory unless a name says `_device`.  All calls return 0 on
 * success or a GX_E* code; gx_last_error() (thread-local) describes the last
 * failure.  The library never aborts the process.
 */
#ifndef GX_H
#define GX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
#define GX_OK 0
#define GX_EINVAL 1       /* bad argument (NULL, size mismatch)                        */
#define GX_ESEQ 2         /* fewer than 2 sequences: the reference panics (algo.rs:169) */
#define GX_ERANGE 3       /* scores/lengths outside the exact int32 device range        */
#define GX_ENOMEM 4       /* device or host allocation failed                           */
#define GX_EHIP 5         /* HIP runtime error                                          */
#define GX_EPANIC 6       /* the reference would panic (retrace, algo.rs:407-408)       */
#define GX_ECAP 7         /* caller buffer too small (needed size reported)             */
#define GX_EIO 8          /* file could not be read                                     */
#define GX_EPARSE 9       /* config could not be parsed                                 */

/* ---- config.rs:6-13  Scores ------------------------------------------ */
typedef struct gx_scores {
    int64_t s_match;
    int64_t s_mismatch;
    int64_t g; /* per-residue gap */
    int64_t h; /* gap opening     */
} gx_scores;

/* ---- algo.rs:25-35  #[repr(C)] AlignmentCell (48 B, same field order) - */
typedef struct gx_cell {
    int64_t insert_score;
    int64_t delete_score;
    int64_t sub_score;
    uint64_t insert_matches;
    uint64_t delete_matches;
    uint64_t sub_matches;
} gx_cell;

/* ---- algo.rs:124-133  #[repr(u8)] AlignmentChoice ---------------------- */
enum {
    GX_MATCH = 0,
    GX_MISMATCH = 1,
    GX_INSERT = 2,
    GX_DELETE = 3,
    GX_OPEN_INSERT = 4,
    GX_OPEN_DELETE = 5
};

/* one element of AlignedSequences.alignment: (AlignmentChoice, usize, usize) */
typedef struct gx_step {
    uint8_t choice;
    uint8_t pad[7];
    uint64_t i;
    uint64_t j;
} gx_step;

/* ---- algo.rs:135-146  AlignedSequences stats (+ where the walk started) - */
typedef struct gx_result {
    int64_t score;
    uint64_t matches;
    uint64_t mismatches;
    uint64_t gap_extensions;
    uint64_t opening_gaps;
    uint64_t n_steps;        /* alignment.len()                                  */
    uint64_t start_i;        /* retrace start cell (algo.rs:306-323)             */
    uint64_t start_j;
    uint64_t max_cell_i;     /* alignment_table's running max cell (algo.rs:258) */
    uint64_t max_cell_j;
    uint64_t matches_at_max; /* alignment_table's second return (algo.rs:279)    */
    int64_t fill_us;         /* device fill time (µs), for the info! log lines    */
    int64_t retrace_us;      /* traceback time (µs)                              */
} gx_result;

typedef struct gx_context gx_context; /* one per GPU (device memory cache + stream) */
typedef struct gx_table gx_table;     /* a device-resident Array2<AlignmentCell>     */

const char* gx_last_error(void);
const char* gx_version(void);

/* Create a context on HIP device `device`. */
int gx_context_create(int device, gx_context** out);
void gx_context_destroy(gx_context* ctx);
/* Release cached device buffers (they are otherwise reused across calls). */
int gx_context_trim(gx_context* ctx);

/* ---- alignment_table (algo.rs:151-156) --------------------------------
 * Fills the table of the first two sequences on the GPU.  The table stays in
 * HBM (the reference's (n+1)x(m+1) 48 B cells need 42.9 GB at 30k).  The
 * three score planes take 12 B/cell as int32, or 3 B/cell as exact per-cell
 * byte differences (untracked tables on the anti-diagonal layout whose scores
 * pass the range proof, gx_plane_bytes_per_cell; untracked global tables also
 * keep values shifted by (i + j) g on the device).  Every export decodes them
 * to the reference's int64 values.  `reverse_sequences` has the semantics of
 * is_match(.., true) (sequence.rs:102-115).  On success *table_out owns the
 * table and *matches_at_max holds the second tuple element.  Passing
 * matches_at_max = NULL skips the running-max/LCS tracking (gx_table_info
 * then reports max cell (0, 0)) unless GX_TABLE_MATCHES is set.
 * flags: GX_TABLE_PLANES keeps the three score planes (needed for export);
 *        GX_TABLE_MATCHES additionally keeps the LCS plane so that the
 *        *_matches fields can be exported (full AlignmentCell fidelity).   */
#define GX_TABLE_PLANES 1u
#define GX_TABLE_MATCHES 2u
int gx_alignment_table(gx_context* ctx, const uint8_t* s1, size_t n, const uint8_t* s2, size_t m,
                       const gx_scores* scores, int is_local, int reverse_sequences, uint32_t flags,
                       gx_table** table_out, uint64_t* matches_at_max);

/* Shape and running-max bookkeeping of a table. */
int gx_table_info(const gx_table* t, uint64_t* n_rows /* n+1 */, uint64_t* n_cols /* m+1 */,
                  uint64_t* max_cell_i, uint64_t* max_cell_j, int64_t* fill_us);

/* Copy the whole table into caller memory as the reference's Array2
 * (column-major `.f()`, element (i,j) at i + j*(n+1), algo.rs:172).
 * Requires GX_TABLE_PLANES (and GX_TABLE_MATCHES for the *_matches fields,
 * which are otherwise written as 0). */
int gx_table_export(const gx_table* t, gx_cell* out, size_t out_cells);

/* Copy one score plane (0 = insert, 1 = delete, 2 = sub) as int64, row-major
 * (i*(m+1)+j) when colmajor = 0, column-major otherwise. */
int gx_table_export_plane(const gx_table* t, int which, int64_t* out, size_t out_cells, int colmajor);

/* Rows row0 .. row0+rows-1 of one score plane as int64, row-major rows x (m+1)
 * (a slice of the table: a 30k x 30k plane is 7.2 GB as int64).  Row 0 and
 * column 0 are the reference's boundary cells (algo.rs:195-220).  which = 3:
 * max_matches of each cell (AlignmentCell::max_matches, algo.rs:113-121; 0 on
 * the boundary), for tables built with GX_TABLE_MATCHES.  No reference
 * counterpart (the reference materialises the whole Array2). */
int gx_table_export_rows(const gx_table* t, int which, size_t row0, size_t rows, int64_t* out, size_t out_cells);

/* Checksums of the three score planes, computed on the device from the
 * stored planes: sums[k] = sum over interior cells (i, j >= 1) of plane k's
 * value * (1 + i*0x9E3779B1 + j*0x85EBCA77) mod 2^64 (k = 0 insert, 1 delete,
 * 2 sub; oracle/gx_oracle.c oracle_align_lean folds the same sums).  Requires
 * GX_TABLE_PLANES.  Verification at sizes where exporting is impractical. */
int gx_table_plane_sums(const gx_table* t, uint64_t sums[3]);

/* ---- retrace (algo.rs:287-291) -----------------------------------------
 * Walks the table and consumes it (the reference moves the Array2 in); the
 * handle is invalid afterwards whatever the return code.  steps[] receives
 * AlignedSequences.alignment in the reference's order (end -> start);
 * cap = n + m + 1 always suffices.  GX_ECAP reports out->n_steps needed.  */
int gx_retrace(gx_table* t, int is_local, gx_step* steps, size_t cap, gx_result* out);

/* Frees a table without retracing. */
void gx_table_free(gx_table* t);

/* ---- fused alignment_table + retrace (main.rs:143-150) ----------------
 * main.rs discards alignment_table's matches_at_max, so the fused paths do
 * not track the running max cell unless asked: with GX_ALIGN_MAX_CELL in
 * `flags` the result's max_cell_i/j and matches_at_max are filled as
 * gx_alignment_table would; otherwise they are 0.                         */
#define GX_ALIGN_MAX_CELL 4u
int gx_align(gx_context* ctx, const uint8_t* s1, size_t n, const uint8_t* s2, size_t m,
             const gx_scores* scores, int is_local, int reverse_sequences, uint32_t flags, gx_step* steps,
             size_t cap, gx_result* out);

/* ---- many independent pairs in one device launch -----------------------
 * Pair p aligns s1[p] (n[p]) with s2[p] (m[p]).  Score planes are not kept
 * (only the traceback codes), so the batch fits HBM.  steps may be NULL
 * (stats only); otherwise steps[p] has caps[p] entries.  flags as gx_align. */
int gx_align_batch(gx_context* ctx, const uint8_t* const* s1, const size_t* n, const uint8_t* const* s2,
                   const size_t* m, size_t npairs, const gx_scores* scores, int is_local, uint32_t flags,
                   gx_step* const* steps, const size_t* caps, gx_result* out);

/* The same over several GPUs: ctxs[0..nctx-1] are contexts created with
 * gx_context_create (one per device; two contexts on one device are allowed).
 * The pairs are shared out by longest-processing-time on n[p] * m[p] cells and
 * each share runs as one gx_align_batch on its own host thread; results land
 * at their pair's index.  SURVEY.md 8(b)'s gx_align_batch(..., ndev) shape; the
 * reference's multi-worker driver is the rayon pool of main.rs:245-261. */
int gx_align_batch_multi(gx_context* const* ctxs, int nctx, const uint8_t* const* s1, const size_t* n,
                         const uint8_t* const* s2, const size_t* m, size_t npairs, const gx_scores* scores,
                         int is_local, uint32_t flags, gx_step* const* steps, const size_t* caps, gx_result* out);

/* ---- device-resident benchmarking path ---------------------------------
 * Stage one pair per slot in HBM once (gx_stage_pairs), then run the hot
 * path (fill with score planes + traceback) on the staged inputs with no
 * host->device traffic.  Used by bench.py; results and flags as gx_align.
 * Batches larger than the free HBM run in chunks (gx_batch_chunks). */
int gx_stage_pairs(gx_context* ctx, const uint8_t* const* s1, const size_t* n, const uint8_t* const* s2,
                   const size_t* m, size_t npairs);
int gx_run_staged(gx_context* ctx, const gx_scores* scores, int is_local, int keep_planes, uint32_t flags,
                  gx_result* out, double* fill_ms_out);
/* nsteps back-to-back passes over the staged pairs, pipelined one pass deep
 * (pass k's traceback labelling on the host overlaps pass k+1's fill on the
 * device).  out = the last pass's results; *fill_ms_out = mean fill time. */
int gx_run_staged_steps(gx_context* ctx, const gx_scores* scores, int is_local, int keep_planes, uint32_t flags,
                        int nsteps, gx_result* out, double* fill_ms_out);
/* flags bit for gx_run_staged(_steps) with keep_planes: after every pass's
 * fill, the plane checksums of gx_table_plane_sums are computed for every
 * staged pair (before the planes are reused); gx_staged_plane_sums returns
 * them as [pass][pair][3] (nsteps * npairs * 3 values).  Verification only. */
#define GX_STAGED_PLANE_SUMS 8u
int gx_staged_plane_sums(const gx_context* ctx, uint64_t* out, size_t cap, size_t* n_values);
/* flags bit for gx_run_staged_steps: the staged pairs are two sets of equal
 * size -- pairs 0 .. P/2-1 and P/2 .. P-1, pair p and p + P/2 of the same
 * shape -- and pass k runs set k % 2 through the same pipeline, so that every
 * pass's device buffers once held the other set's data (a pass that read a
 * previous pass's planes or records would see different values).  Pass k's
 * results, plane sums and (for the last pass of each set) walks land at its
 * set's pair indices; the other set's row of pass k is zero.  The sets must
 * fit one chunk (else GX_EINVAL).  Verification only. */
#define GX_STAGED_ALTERNATE 16u
/* flags bit for gx_run_staged_steps with keep_planes: the last pass's score
 * planes stay on the device, in the format the batch launch stored them
 * (twin plane codes 2 B/cell, compact bytes 3 B/cell or int32; DESIGN.md
 * 4.2, 4.4), until the next staged run and the last gx_staged_table of them
 * is freed.  One chunk only (else GX_EINVAL); such a run does not take the
 * overlapped two-group pipeline, whose buffers alternate. */
#define GX_STAGED_KEEP_PLANES 32u
/* A table of staged pair `pair` from the last GX_STAGED_KEEP_PLANES run: the
 * reference hands alignment_table's Array2 to its caller (algo.rs:172, 281),
 * and this hands over a batch's planes the same way -- gx_table_info,
 * gx_table_export, gx_table_export_plane, gx_table_export_rows and
 * gx_table_plane_sums decode them to the reference's values.  Its alignment
 * is the run's (gx_staged_steps): gx_retrace returns GX_EINVAL.  Free with
 * gx_table_free. */
int gx_staged_table(gx_context* ctx, size_t pair, gx_table** table_out);
/* The alignment (AlignedSequences.alignment) of staged pair `pair` from the
 * last pass of the last gx_run_staged(_steps) call; *n_steps = its length
 * (steps may be NULL to query it). */
int gx_staged_steps(const gx_context* ctx, size_t pair, gx_step* steps, size_t cap, size_t* n_steps);
/* Every pass's results of the last gx_run_staged(_steps) call, [pass][pair]
 * (nsteps * npairs records; `out` of that call is the last pass's row), so
 * that each timed pass can be checked, not only the last.  Verification only. */
int gx_staged_pass_results(const gx_context* ctx, gx_result* out, size_t cap, size_t* n_values);
/* The last fill launch on ctx: its layout (0: anti-diagonal 128-row strips,
 * 1: column step over 64-row strips, 2: the same as core + side waves,
 * 3: anti-diagonal 64-row strips with one row per lane, the latency fill of
 * untracked single pairs), band width (strips per workgroup) and
 * score-plane bytes written per cell (0: none, 12: int32 planes, 3: compact
 * planes -- per-cell byte differences, decoded exactly by the exports, 2:
 * the twin fill's plane codes -- 12 bits a cell since round 6, DESIGN.md
 * 4.4, batches only; reported rounded up: gx_fill_plane_bits gives the exact
 * figure).  No reference counterpart (measurement only). */
int gx_fill_info(const gx_context* ctx, int* layout, int* band_waves, int* plane_bytes_per_cell);
/* Score-plane bits written per cell by the last fill launch (0, 12: twin
 * plane codes, 24: compact bytes, 96: int32 planes, 192: int64 planes), or
 * -1 without a context.  No reference counterpart (measurement only). */
int gx_fill_plane_bits(const gx_context* ctx);
/* Chunks of the last gx_run_staged(_steps) / gx_align_batch call: a batch
 * whose device footprint (planes, codes, skeleton) exceeds the free HBM runs
 * as contiguous chunks of pairs through the same device buffers
 * (GX_CHUNK_BYTES overrides the per-chunk byte budget).  Measurement only. */
int gx_batch_chunks(const gx_context* ctx);
/* 1 when the last fill launch on ctx was the twin fill (two pairs per band,
 * one per 16-bit half, packed arithmetic), else 0.
 * Measurement only (GX_TWIN=0 disables it, GX_TWIN=1 forces it where the
 * range bound admits it; by default deep band queues take it). */
int gx_fill_twin(const gx_context* ctx);

/* Fill launches per pass of the last staged / batch call: 2 when the pairs
 * ran as two groups whose walks overlap the next pass's fills (a batch of
 * long pairs on the twin fill), else 1. */
int gx_fill_groups(const gx_context* ctx);
/* Score-plane bytes per cell a batch launch (layout 0, no max tracking)
 * writes with these scores: 3 when the compact format's range proof holds
 * (global mode, g, h <= 0, differences within a signed byte), else 12; -1 on
 * invalid scores.  An upper bound: a launch that takes the twin fill with
 * its plane codes writes 2 (gx_fill_info reports the
 * launch's own figure). */
int gx_plane_bytes_per_cell(const gx_scores* scores, int is_local);

/* The twin fill's int16 admission rule for global batches:
 * *bound receives the largest |value - base| a band of `band_waves` strips can
 * reach with these scores when a twin's two pairs differ by up to col_gap
 * columns; returns 1 when the global twin fill admits the band (bound <
 * 30,000 < 2^15), 0 when it does not, -1 on invalid scores.  Diagnostic
 * (tests/test_twin_bound.py checks the rule against brute-force spreads).
 * No reference counterpart. */
int gx_twin_admission(const gx_scores* scores, int band_waves, int64_t col_gap, int64_t* bound);
/* The same rule for either mode: local batches (is_local = 1) keep plain
 * values relative to the same per-block bases, with the neighbour difference
 * max(|h + g|, U) of the unshifted values and the floor's constants
 * (DESIGN.md 6.7).  Same returns as gx_twin_admission. */
int gx_twin_admission_mode(const gx_scores* scores, int is_local, int band_waves, int64_t col_gap, int64_t* bound);
/* The fill layout a launch of these pair shapes would take (host rule only,
 * no device): 0 = anti-diagonal 128-row strips (batches), 1 = the column
 * step, 3 = skewed 64-row strips (the latency layouts);
 * `track` = an alignment_table call that keeps max_cell / matches_at_max
 * (algo.rs:258-262, 279).  grid_cap = the device's CU count (0: 256).  -1 on
 * invalid arguments.  Diagnostic; no reference counterpart. */
int gx_plan_layout(const gx_scores* scores, int is_local, const int64_t* n, const int64_t* m, size_t npairs,
                   int track, int grid_cap);

/* ---- sequence.rs / config.rs mirrors ----------------------------------- */
/* from_fasta (sequence.rs:45-95) on a file: records are appended to the
 * caller's buffers.  Returns GX_OK and sets *n_records; names/sequences are
 * concatenated into `buf` (cap bytes) with offsets/lengths in the arrays
 * (rec_cap entries).  An unreadable file logs and yields 0 records (the
 * reference swallows the error, sequence.rs:84-86). */
int gx_fasta_load(const char* path, uint8_t* buf, size_t cap, uint64_t* name_off, uint64_t* name_len,
                  uint64_t* seq_off, uint64_t* seq_len, size_t rec_cap, size_t* n_records, size_t* bytes_needed);
/* get_config (config.rs:21-40): reads [scores] s_match, s_mismatch, g, h. */
int gx_config_load(const char* path, gx_scores* out);

/* Display for AlignedSequences (display.rs:9-127) into `out` (NUL-terminated).
 * *needed receives the full length + 1. */
int gx_format_alignment(const uint8_t* s1, size_t n, const uint8_t* s2, size_t m, const gx_step* steps,
                        size_t n_steps, const gx_result* res, char* out, size_t cap, size_t* needed);

/* print_alignment_table + print_scores_table (display.rs:131-220), which the
 * reference's retrace prints to stdout with the table it consumed
 * (algo.rs:438).  Planes are int64 row-major (n+1)x(m+1), as
 * gx_table_export_plane(.., colmajor = 0) writes them (export them before
 * gx_retrace consumes the table).  Empty output when n >= 200 or m >= 2000
 * (the reference only warns then).  color != 0: ANSI styles of the `colored`
 * crate (the reference colours only when stdout is a terminal).  GX_EPANIC
 * where the reference's chars().nth().unwrap() panics (non-ASCII input). */
int gx_format_table(const uint8_t* s1, size_t n, const uint8_t* s2, size_t m, const gx_step* steps, size_t n_steps,
                    const int64_t* insert_plane, const int64_t* delete_plane, const int64_t* sub_plane, int color,
                    char* out, size_t cap, size_t* needed);

#ifdef __cplusplus
}
#endif

#endif /* GX_H */
