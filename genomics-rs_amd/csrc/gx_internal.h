// gx_internal.h -- structures shared by the HIP kernels and the C++ host code.
//
// Device data layout (DESIGN.md "HBM layout"):
//   A pair (s1: n rows, s2: m columns) is cut into STRIPS of 128 interior rows
//   (strip k = rows 128k+1 .. 128k+128; lane l owns rows 128k+2l+1 and
//   128k+2l+2, "row-in-lane" h = 0, 1).  One wave sweeps a strip along the
//   anti-diagonal skew: at step t lane l computes column j = t - l + 1 for both
//   its rows, so a strip takes T = m + 64 steps.  W strips (W from
//   kFillWidths, chosen per launch) form a BAND, processed by one workgroup
//   (one wave per strip + one I/O wave).
//
//   Score planes (int32, one each for insert/delete/sub score):
//       plane[strip][t/4][h][lane][t%4]     (16 B per lane per row per 4 steps)
//   so each wave stores 1 KiB contiguous per plane and row every 4 steps.
//   Traceback direction codes (2 bit/cell), two bit-planes per word:
//       codes[strip][t/16][row-in-strip]  (row-in-strip = 2l + h; uint32; for
//       k = t%16 bit 31-k = "delete beats insert and sub", bit 15-k = "insert
//       beats sub"; decode D ? 2 : I ? 1 : 0)
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace gx {

constexpr int kWave = 64;
constexpr int kNeg = -(1 << 30);   // int32 stand-in for negative_inf (algo.rs:166)
#ifndef GX_RING
#define GX_RING 256
#endif
constexpr int kRing = GX_RING;     // LDS ring records per strip boundary (power of two)
constexpr int kSub = 16;           // steps per flow-control sub-block (multiple of 16)
constexpr int kIoChunk = 16;       // columns per I/O-wave transfer (layout 0)
constexpr int kIoChunk1 = 4;       // columns per I/O-wave transfer (layout 1)
constexpr int kRowsPerLane = 2;    // a lane owns rows 2l+1, 2l+2 of its strip
constexpr int kStripRows = kWave * kRowsPerLane;   // 128 rows per strip
// Plane layout (ints): plane[strip][t/4][row-in-lane][lane][t%4]; one 4-step
// group of one row is 1 KiB contiguous per wave.
constexpr int kGroupInts = kRowsPerLane * kWave * 4;
// twin plane codes (gx_fill_pk.hip PLANES 2): one 12-bit code per cell and
// pair (round 6; 16 bits before), a lane's 4 steps of one row for both pairs
// of a twin in a 12-B record (gx_device.h w12_pack); a 4-step group of a
// strip = [row][lane] records
constexpr int kTwinRec = 12;
constexpr int kTwinGroupBytes = kRowsPerLane * kWave * kTwinRec;
// Column-step layout (layout 1): 64-row strips, lane l owns row 64s + l + 1,
// step t = column t + 1 for every lane (no skew); planes
// plane[strip][t/4][lane][t%4] (1 KiB per wave per plane every 4 columns),
// codes[strip][t/16][lane].  The vertical delete chain is a prefix max over
// the wave (gx_kernels.hip, compute_wave_cs).
constexpr int kGroupInts1 = kWave * 4;
constexpr int kStripRows1 = kWave;
// Layout 3 (gx_skew.hip, the latency fill): 64-row strips like layout 1, lane
// l owns row 64s + l + 1, but on the anti-diagonal skew like layout 0 (step t
// = column t - l + 1); planes plane[strip][t/4][lane][t%4], codes
// codes[strip][t/16][lane], both indexed by step; skeleton E + 64 per column.
inline int strip_rows(int lay) { return lay ? kStripRows1 : kStripRows; }
// Compute waves per band (workgroup = W compute waves + 1 I/O wave).  The
// host picks the narrowest width whose bands fit one workgroup per CU (a
// single pair: 3, one compute wave per SIMD, so a strip's own speed sets the
// time; a batch: wider bands, all strips in flight from the start).  The
// launcher instantiates these widths (must match GX_W_ALL / GX_W_TRACK in
// gx_kernels.hip); the tracked and local variants carry more state per row
// (256-VGPR builds) and stop at 8-wave workgroups.
constexpr int kFillWidths[] = {3, 4, 6, 8, 11, 15};
constexpr int kFillWidthsTrack[] = {3, 7};

// Scores narrowed to int32 after the host range guard (DESIGN.md "Integer range").
struct Scores32 {
    int sm;      // s_match
    int smm;     // s_mismatch
    int g;       // per-residue gap
    int h;       // gap open
    int hg;      // h + g
    int floor_;  // local ? 0 : kNeg  (the 4th lane of score_max, algo.rs:103)
    int dbg;     // GX_DEBUG_FLAGS: bit0 = rolled (ramp) path only
    int shift;   // layout-0 untracked global launches: values kept as V - (i + j) g (sm, smm hold s - 2g)
    int sym[4];  // small-alphabet launches: the job's distinct processed bytes (code k = sym[k])
    int koff;    // local twin fill (gx_fill_pk.hip): K = max(0, -min(sm, smm)) added to sm / smm (score tables >= 0)
};

// One inter-strip record: the bottom-row cell (r, j) of a strip, as needed by
// the strip below.  dd = its delete-successor max(max(I,S)+h+g, D+g, floor),
// sm = score_max(cell), c2 = s2[j-1], l = max_matches(cell) (only with LCS
// tracking; the three leading words are then one ds_read_b96).
struct __attribute__((aligned(16))) Rec {
    int dd, sm, c2, l;
};

// Bit-parallel LCS rows of layout-3 tracked fills (gx_lcs.h): a word holds
// kLcsBits columns (bit k of word w: column kLcsBits w + k + 1); steps a strip of the sweep takes
// for rows of `words` words (a multiple of 32, the sweep's unrolling: lane 63
// finishes word words - 1 at step words + 62), and the index (in words) of word w of row i (1-based)
// in PairDev.lbits, [strip][step][lane].
constexpr int kLcsBits = 64;
constexpr int kLcsMaskPad = 64;         // zero words before (and after) each mask row
constexpr int lcs_steps(int words) { return (words + 64 + 31) & ~31; }
constexpr size_t lcs_word_index(int i, int w, int words) {
    return ((size_t)((i - 1) / 64) * (size_t)lcs_steps(words) + (size_t)(w + (i - 1) % 64)) * 64 + (size_t)((i - 1) % 64);
}

struct __attribute__((aligned(16))) StripRes {
    int best, bi, bj, bl;      // first max of score_max in row-major order + LCS there
    int lbest, li, lj, lE;     // last max (local start search) + its landing column
};

// Landing column E(i, j): the traceback path from cell (i, j) leaves its
// strip through the strip's top boundary row 128s at column E (E >= 0), or
// reaches column 0 inside the strip at local row -E (E < 0).  The fill
// propagates it with the traceback codes; each strip's bottom row is stored
// as the traceback skeleton.
struct __attribute__((aligned(16))) PairRes {
    int max_val, max_i, max_j, mam;       // first max over interior (algo.rs:258-262, 279)
    int lmax_val, lmax_i, lmax_j, nstrips;// last max over interior (algo.rs:310-322)
    int end_SM, end_E, lmax_E, pad2;      // score_max and E of cell (n, m); E of the last max
};

// Optional per-strip timeline (GX_TRACE_FILE): s_memrealtime ticks (100 MHz)
// and spin iterations, for the diagnostic runs behind DESIGN.md's numbers.
constexpr int kTraceQ = 7;   // progress stamps per strip (at k/8 of the sweep)
constexpr int kTraceTL = 64; // layout 3: dense timeline stamps per strip (every 1,024 steps)
struct __attribute__((aligned(16))) StripTrace {
    long long t_start;   // wave starts the strip
    long long t_first;   // first input sub-block available
    long long t_end;     // strip done
    int wait_in;         // spin iterations waiting for the row above
    int wait_out;        // spin iterations waiting for ring space below
    long long clk;       // shader-clock ticks (s_memtime) from t_first to t_end
    long long t_q[kTraceQ];   // when the sweep passed k/8 of its steps (k = 1..7)
    long long tl[kTraceTL];   // layout 3: when the core wave reached step 1024 k (a dense timeline)
    long long tc[kTraceTL];   // ... and the shader clock (s_memtime) then
    long long ts[kTraceTL];   // layout 3: when the side wave reached step 1024 k
};

struct __attribute__((aligned(16))) PairDev {   // 16-B multiple: the pinned staging puts PairRes (aligned 16) after P of these
    const uint8_t* c1;   // processed row chars, n   (is_match row operand)
    const uint8_t* c2;   // processed col chars, m
    int n, m;
    int strips;          // ceil(n / 64)
    int bands;           // ceil(strips / W)
    int t4;              // plane step-groups per strip (multiple of 4)
    int t16;             // code words per lane per strip
    int band_base;       // global index of this pair's band 0
    int strip_base;      // index of this pair's strip 0 in the StripRes array
    int32_t* pI;         // planes (nullptr: score-only)
    int32_t* pD;
    int32_t* pS;
    int32_t* pL;         // optional LCS plane (full AlignmentCell export)
    uint32_t* codes;     // traceback codes (nullptr: none)
    Rec* feed;           // [bands-1][feed_stride] band-boundary rows
    int* progress;       // [bands-1][kProgStride] columns published per boundary (one per 256 B)
    StripTrace* trace;   // per strip, or nullptr
    int* skel;           // [strips][skel_stride] landing column E of each strip's bottom row
    int feed_stride;
    int skel_stride;
    int twin_half;       // twin fill: this pair's 16-bit half (0 low, 1 high) in its twin's shared buffers
    const int* ccodes;   // layout 3: the column symbols as int32 (code * 8 with score tables), 64 zeros
                         // before and after (index j - 1 + 64 for column j; gx_skew.hip)
    // layout-3 tracked fills: max_matches as bit-parallel LCS rows (gx_lcs.h),
    // computed beside the fill by the launch's leading workgroups
    unsigned long long* lbits;   // row i's LCS difference bits V_i (bit k of word w: column 64 w + k + 1),
                                 // [strip][step][lane] (gx_lcs.h lcs_word_index), or each strip's last row
    unsigned long long* lmask;   // [256][lwords + 128] match masks of each byte against s2 (zeroed before the launch)
    unsigned long long* llink;   // [strips][lcs_steps][2] the strips' bottom rows, tagged halves (zeroed before the launch)
    unsigned long long* ltrace;  // diagnostics (GX_LCS_TRACE): [strip][4] s_memrealtime stamps, or nullptr
    int lwords;                  // words per bit row, ceil(m / kLcsBits); 0 = no LCS rows
    int lcs_waves;               // sweeping waves per LCS workgroup | (workgroups << 8) | (every row << 16)
    int lcs_base;                // the pair's first LCS workgroup (blockIdx.x)
    int lcs_pad;
};
static_assert(sizeof(PairDev) % 16 == 0, "PairDev staging keeps the PairRes that follow it 16-B aligned");

struct TbDev {           // per-pair traceback job
    const uint32_t* codes;
    const int* skel;
    int skel_stride;
    int n, m, t16, strips;
    int start_i, start_j;  // interior start cell (1-based), or 0 = nothing to walk
    int start_E;           // landing column of the start cell (PairRes.end_E / lmax_E)
    const int* start_E_dev;// or, when non-null, read on the device (the fill's PairRes.end_E: no host round trip)
    int srows;             // rows per strip: 128 (layout 0, anti-diagonal) or 64 (layouts 1 and 3)
    int skew;              // layout 3 (gx_skew.hip): 64-row strips on the anti-diagonal skew, one row per lane
    int skel_half;         // -1: int32 skeleton; 0 / 1: the low / high int16 of a twin fill's packed skeleton
    int* seg;              // out: [strips][4] {entry_i, entry_j, records, active} per strip on the path
    uint32_t* recs;        // out: [strips][kStripRows] one record per row, (insert run << 2) | kind
    int* end_ij;           // out: [4] {i, j} where the walk leaves the interior, first strip, rounds
    // twin fill without code words (gx_fill_pk.hip, twin plane codes): the
    // traceback derives the code words of the strips on the path from the
    // plane codes first (tb_w16_codes_kernel); nullptr: the fill wrote them
    const uint8_t* w16;    // the twin's code plane (strip 0), [strip][t/4][row-in-lane][lane][t%4] dwords
    int w16_half;          // this pair's 16-bit half of each dword
    int t4;                // 4-step groups per strip
    const int* start_ij_dev;// local twin fill in the overlapped pipeline: the start cell {i, j} read on the device
                           // (PairRes.lmax_i / lmax_j after finalize_kernel: no host round trip); tb_seq_kernel only
};

// ---- wide (int64) fill (gx_wide.hip): jobs outside the exact-int32 range --
struct WideScores {
    long long sm, smm, g, h;
    long long neg_inf;   // i64::MIN + |g + h| (algo.rs:166)
};
struct __attribute__((aligned(8))) WideRow {   // one cell of a strip's bottom row, for the strip below
    long long dd, sm;    // delete successor score_max(hg, hg, g), score_max(0, 0, 0)
    unsigned lm, pad;    // max_matches
};
struct WideRes {
    long long max_val, lmax_val, end_SM;
    unsigned long long mam;
    int max_i, max_j, lmax_i, lmax_j, lmax_E, end_E, pad0, pad1;
};
struct WideDev {
    const uint8_t* c1;
    const uint8_t* c2;
    int n, m, strips, t16;
    long long* pI;       // int64 planes, row-major n x m interior (nullptr: not kept)
    long long* pD;
    long long* pS;
    unsigned* pL;        // LCS plane (max_matches), or nullptr
    uint32_t* codes;     // codes[strip][t16][64] (layout-1 format)
    int* skel;           // [strips][skel_stride]: landing column + 64 of the strip's bottom row
    WideRow* rows;       // [strips][m + 1] bottom rows
    int skel_stride, pad;
};

// Band-boundary progress counters sit 256 B apart: every I/O wave polls its
// own, and neighbouring counters in one cache line would put all of a
// batch's polls on one L2 channel.
constexpr int kProgStride = 64;

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

}  // namespace gx
