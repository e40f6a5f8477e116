// Host build of cq_amd/csrc/cell.h (the exact code the gfx950 kernels run) for
// unit tests against glibc strtod/strtoll/sscanf/printf -- test infrastructure.
#include <cstdint>
#include <cstring>
#include "../../cq_amd/csrc/cell.h"

extern "C" {
// parse one field (bytes must be followed by readable padding, like the device buffer)
void cell_parse(const uint8_t* f, uint32_t len, uint32_t* kind, uint32_t* slen, uint64_t* bits,
                int64_t* str_off) {
    cq::Cell c = cq::parse_cell(f, len);
    *kind = c.kind;
    *slen = c.len;
    *bits = c.bits;
    *str_off = c.kind == cq::K_STR ? (int64_t)((const uint8_t*)(uintptr_t)c.bits - f) : -1;
}
double cell_to_dbl(const uint8_t* s) { return cq::to_dbl(s); }
int64_t cell_to_int(const uint8_t* s) { return cq::to_int(s); }
int cell_parse_date(const char* s, int* y, int* m, int* d) { return cq::parse_date(s, *y, *m, *d); }
// group-key identity: (class, payload)
void cell_dbl_key(double x, uint32_t* cls, uint64_t* v) {
    cq::GKey k = cq::group_key(cq::cell_dbl(x));
    *cls = k.cls;
    *v = k.v;
}
}
