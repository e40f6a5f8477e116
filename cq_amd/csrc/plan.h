// plan.h -- compiled SELECT plan shared by the host executor and the kernels.
#pragma once
#include <stdint.h>
#include "cell.h"

namespace cq {

constexpr int MAX_NEED = 8;     // distinct CSV columns one scan parses
constexpr int MAX_PROG = 128;   // predicate instructions
constexpr int MAX_CONST = 48;   // literal cells
constexpr int MAX_ACC = 8;      // accumulators (one per aggregate SELECT item)
constexpr int MAX_GPART = 64;   // composite GROUP BY parts (the reference's list grows without bound)
// distinct columns of a plan, a join side or a projection on the cells path: plans
// over more than MAX_NEED columns ("wide") read their cells from the parsed cell
// tables (scan.hip PairView) instead of registers
constexpr int MAX_WIDE = 256;
constexpr int VM_STACK = 8;

// predicate bytecode (WHERE tree of evaluator_conditions.c:62-164 and
// evaluator_expressions.c:23-263, flattened in post-order)
enum : uint8_t {
    OP_COL = 0,    // push cells[a]
    OP_CONST,      // push consts[b]
    OP_NULLV,      // push NULL (unresolvable identifier, unsupported expression value)
    OP_ARITH,      // a = AR_*; pop r, l; push arith(l, r)
    OP_NEG,        // unary minus
    OP_CMP,        // a = CMP_*; pop r, l; push bool
    OP_IN,         // b = item count, a = negate; pops items then left
    OP_LIKE,       // a = case-sensitive
    OP_NOT,
    OP_AND,
    OP_OR,
    OP_BOOL,       // push bool a
};
enum : uint8_t { CMP_EQ = 0, CMP_NE, CMP_LT, CMP_GT, CMP_LE, CMP_GE };

struct Insn {
    uint8_t op;
    uint8_t a;
    uint16_t b;
};

// accumulator kinds
enum : uint8_t { ACC_SUM = 0, ACC_MIN = 1, ACC_MAX = 2 };

struct AccSpec {
    uint8_t kind;   // ACC_*
    uint8_t slot;   // need slot of the argument column
    uint8_t cls;    // MIN/MAX over the pair path: only cells of these value classes (class_bit; 0 = all)
    uint8_t pos_only;   // MIN over the pair path: every qualifying cell counts as equal (first position)
};

struct ScanPlan {
    uint64_t n;            // bytes in the table
    uint64_t data_begin;   // first byte a data record may start at
    uint64_t range_begin;  // records are owned by [range_begin, range_end)
    uint64_t range_end;
    uint32_t delim;
    uint32_t quote;
    int32_t nneed;
    int32_t max_col;
    int16_t need_col[MAX_NEED];
    int32_t nprog;         // 0: no WHERE
    Insn prog[MAX_PROG];
    int32_t nconst;
    Cell consts[MAX_CONST];
    int32_t group_slot;    // -1: one group (aggregate query without GROUP BY)
    // composite / expression GROUP BY (evaluator.c:113-212, evaluator_aggregates.c:179-250):
    // ngpart > 0 replaces group_slot; part k is need slot gpart_slot[k] (>= 0), the
    // expression prog[gcode_off[k], gcode_off[k + 1]) (-1, after the WHERE program) or
    // a column the composite path cannot resolve (-2: the text "NULL")
    int32_t ngpart;
    int16_t gpart_slot[MAX_GPART];
    uint16_t gcode_off[MAX_GPART + 1];
    int32_t nacc;
    AccSpec acc[MAX_ACC];
    int32_t want_rows;     // 1: also emit matching record offsets (row-returning)
    uint32_t lean_ws;      // lean_kernel window stride (0: the largest, lean::WS)
    uint32_t lean_k16;     // lean_kernel GROUP BY tags of 16 key bytes (the column's sampled fields exceed 8)
    uint64_t fast_seed;    // fast_kernel: device address of the GROUP BY column's seeded LDS tags (0: none)
    uint64_t fast_wide_cols;   // bit c: sampled fields of column c over 4 bytes (bit 63: columns >= 63)
    uint32_t test_digest_bits;   // test knob CQGPU_TEST_DIGEST_BITS: composite digests cut to this many bits (0: all 128)
};

// projection of a row-returning SELECT (device pointers): ncols CSV columns
// parsed per record (ascending), nout programs code[off[k], off[k+1])
struct ProjDesc {
    const int16_t* cols;
    const Insn* code;
    const uint32_t* off;
    const Cell* consts;
    int32_t ncols;
    int32_t nout;
    uint32_t delim;
    uint32_t quote;
};

// finish_kernel (scan.hip): what to gather for every compacted group
struct FinishDesc {
    int16_t cols[MAX_WIDE];   // representative columns, ascending
    int32_t ncols;
    uint32_t delim;
    uint32_t quote;
    int32_t nacc;
    uint32_t sb;              // inline STRING bytes per cell
    uint32_t first_shift;     // the record offset is first >> first_shift (a join's pair key: 32)
};

// INNER JOIN (evaluator_joins.c:63-181) on the device: columns of one side parsed
// per record into a row-major cell array (ncols cells per row)
struct ColsDesc {
    int16_t cols[MAX_WIDE];   // CSV columns, ascending
    int32_t ncols;
    uint32_t delim;
    uint32_t quote;
};
// where each need slot of a plan over the joined row lives: side 0 = left cells,
// 1 = right cells, col = index within that side's row of cells
struct JoinMap {
    int8_t side[MAX_WIDE];
    int16_t col[MAX_WIDE];
    int32_t n;
    uint32_t lstride, rstride;
};

// one slot of a join's hash table of right-side keys: the key (code, value
// class) and, once the rows are sorted by slot, the slot's run [start, end) in
// sidx -- one 24-byte record, so a build or a probe touches one line, not five
struct HSlot {
    unsigned long long code;
    uint32_t st;                        // 0 empty, 1 claimed, 2 + class published
    uint32_t start, end;
    uint32_t pad;
};
static_assert(sizeof(HSlot) == 24, "24-byte hash slots");

// the right side of a join (scan.hip join_count_kernel / join_emit_kernel)
struct JoinRight {
    // open-addressing hash table of the right side's distinct keys (value class, code)
    const HSlot* hslot;
    uint32_t hcap;                      // slots, a power of two
    const uint32_t* sidx;               // right rows grouped by key slot, row order within a slot
    const uint32_t* ridx_c;             // rows grouped by class, row order within a class
    const Cell* cells;
    uint32_t stride, kcol;
    uint32_t seg[5];                    // class segment bounds (0 NULL, 1 number, 2 string, 3 date)
};

// the same table while it is built (hash_build_kernel)
struct JoinHashW {
    HSlot* slot;
    uint32_t cap;
};

// scan statistics written by the kernel (one per launch)
struct ScanStats {
    unsigned long long records;     // data records seen
    unsigned long long passed;      // records passing WHERE
    unsigned long long short_rows;  // records too short for a needed column
    unsigned long long lds_spills;  // records aggregated straight into the global table
    unsigned long long overflow;    // global table full: host must retry larger
    unsigned long long rows_emitted;
    unsigned int acc_classes[MAX_ACC];  // OR of value classes seen per accumulator (1 num, 2 str, 4 date)
    unsigned long long slow_records;    // records the fast field walk handed to the general parser
    unsigned long long clk[8];          // profiling builds (CQ_CLOCKS): shader cycles per phase, summed over waves
    unsigned int key_flags;             // composite GROUP BY: 2 = a joined text that could not render (never: every cell renders)
};

// a MIN/MAX candidate published by one block (or wave) for one group
struct ExtCand {
    Cell c;
    unsigned long long pos;
    unsigned long long pad;
};

// global (HBM) group table, structure of arrays, capacity `cap` (power of two)
struct GroupTable {
    uint32_t cap;
    uint32_t* tag;                 // 0 empty, 1 being written, else hash tag
    uint32_t* clslen;              // key class << 16 | text length
    uint64_t* w0;                  // key words (cell.h GKey)
    uint64_t* w1;
    unsigned long long* cnt;
    unsigned long long* first;     // min record byte offset
    double* sum[MAX_ACC];          // ACC_SUM: sum of numeric cells
    unsigned long long* num[MAX_ACC];  // ACC_SUM: numeric cell count
    Cell* ext[MAX_ACC];            // ACC_MIN/MAX: extreme cell
    unsigned long long* extpos[MAX_ACC];
    uint32_t* lock[MAX_ACC];
    // lock-free MIN/MAX merge across blocks: extref holds the index of the best
    // published candidate (~0: none); candidate slot = block * cand_stride + LDS slot
    unsigned long long* extref[MAX_ACC];
    ExtCand* cand[MAX_ACC];
    uint32_t cand_stride;
    uint32_t* used;                // number of occupied slots
};

// dense group record handed back to the host
struct GroupOut {
    uint32_t clslen, pad;
    uint64_t w0, w1;
    unsigned long long cnt;
    unsigned long long first;
    double sum[MAX_ACC];
    unsigned long long num[MAX_ACC];
    Cell ext[MAX_ACC];
    unsigned long long extpos[MAX_ACC];
};

// gather-merge of range partials (multi-GPU, scan.hip gm_pack_kernel -> merge.hip
// gm_*): per rank a GM_HDR-byte header, then up to maxg group records of
// gm_rec_bytes(nacc, R): clslen u32, pad, w0, w1, COUNT, first (local offset),
// per accumulator (SUM f64, numeric count), then R + 1 cells of GM_CELL bytes
// (kind u32, len u32, bits, GM_TEXT bytes of STRING text; the last one is a long
// key's text)
constexpr uint32_t GM_HDR = 64, GM_CELL = 64, GM_TEXT = 48;
enum : uint32_t { GM_OK = 0, GM_FAILED = 1, GM_DECLINE = 2 };
struct GmHdr {
    uint32_t status;        // GM_OK / GM_FAILED / GM_DECLINE
    uint32_t ng;            // groups in this rank's records
    uint64_t base;          // the rank's whole-file byte offset
    uint64_t records, passed, slow_records, lds_spills;
    uint64_t pad[2];
};
static_assert(sizeof(GmHdr) == GM_HDR, "gather-merge header");
#if defined(__HIPCC__)
__host__ __device__
#endif
constexpr uint32_t gm_rec_bytes(int nacc, uint32_t R) {
    return 40u + 16u * (uint32_t)nacc + GM_CELL * (R + 1u);
}

}  // namespace cq
