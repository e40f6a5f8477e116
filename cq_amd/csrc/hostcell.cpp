// hostcell.cpp -- cell.h's typing (parse_value / infer_type restatement) compiled
// for the host, so the executor types SQL literals without a device round trip.
// Same source as the kernels' parser (cell.h), built by g++ without __HIPCC__.
#include <cstring>
#include "cell.h"

extern "C" cq::Cell cq_host_parse_cell(const uint8_t* text, uint32_t len) { return cq::parse_cell(text, len); }
// create_groups' canonical key of a cell (the typed join exchange's tags, on the host)
extern "C" cq::GKey cq_host_group_key(cq::Cell c) { return cq::group_key(c); }

#include "plan.h"

// evaluate_expression (evaluator_expressions.c:23-263) on the host over one row of
// cells: a non-aggregate expression item of an aggregate SELECT, evaluated on the
// group's first row (build_aggregated_result, evaluator_aggregates.c:669-677).
// OP_COL b indexes `cols`, OP_CONST b indexes `consts`.
extern "C" cq::Cell cq_host_eval(const cq::Insn* code, uint32_t n, const cq::Cell* cols, const cq::Cell* consts) {
    using namespace cq;
    Cell st[VM_STACK + 1];
    int sp = 0;
    for (uint32_t pc = 0; pc < n; pc++) {
        const Insn in = code[pc];
        if (sp > VM_STACK) return cell_null();
        switch (in.op) {
            case OP_COL: st[sp++] = cols[in.b]; break;
            case OP_CONST: st[sp++] = consts[in.b]; break;
            case OP_ARITH: {
                if (sp < 2) return cell_null();
                const Cell r = st[--sp], l = st[--sp];
                st[sp++] = arith(in.a, l, r);
                break;
            }
            case OP_NEG: {
                if (sp < 1) return cell_null();
                const Cell x = st[--sp];
                st[sp++] = negate(x);
                break;
            }
            default: st[sp++] = cell_null(); break;
        }
    }
    return sp > 0 ? st[sp - 1] : cell_null();
}

// a DOUBLE cell's composite-key part text (cell.h joined_text_add: "%.6f", the first
// 255 bytes) into out (256 bytes); its length.  Checked on the CPU against Python's
// correctly rounded formatting (tests/test_key_text.py).
namespace {
struct HostSink {
    char* p;
    uint32_t n;
    void byte(uint8_t c) { if (n < 255) p[n] = (char)c; n++; }
    void bytes(const uint8_t* q, uint32_t k) { for (uint32_t i = 0; i < k; i++) byte(q[i]); }
    void dec(uint64_t v, int mind) {
        uint8_t t[20];
        int k = 0;
        do { t[k++] = (uint8_t)('0' + v % 10); v /= 10; } while (v);
        while (k < mind) t[k++] = '0';
        while (k) byte(t[--k]);
    }
};
}  // namespace
extern "C" uint32_t cq_host_double_key_text(uint64_t bits, char* out) {
    HostSink h{out, 0};
    cq::Cell c;
    c.kind = cq::K_DBL;
    c.len = 0;
    c.bits = bits;
    cq::joined_text_add(h, c, true);
    return h.n < 255 ? h.n : 255;
}
