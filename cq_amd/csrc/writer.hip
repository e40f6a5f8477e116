// writer.hip -- the `-o` CSV writer on the GPU (replaces write_csv_file, reference
// utils.c:220-289, for results of the executor).
//
// The result's cells are packed once (kind, length, payload; string bytes in one
// arena) and uploaded; one thread per row formats its row twice -- a counting pass
// for the row's byte length, then, after an exclusive scan of the lengths
// (prim.hip), the writing pass into one output buffer that goes back to the host
// in a single copy and is written with one fwrite.  Formats follow the reference's
// fprintf calls exactly: INTEGER "%lld", DOUBLE "%.2f" (glibc: the exact binary
// value rounded half-to-even at the second decimal, "-0.00" for negative values
// that round to zero, every digit of huge values, "inf" / "nan"), DATE
// "%04d-%02d-%02d", STRING quoted (quotes doubled) when it holds the delimiter, a
// quote, '\n' or '\r', NULL as nothing.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/cqgpu.h"

extern "C" {
size_t cq_scan_scratch_bytes(uint64_t n, int elem_bytes);
hipError_t cq_scan_u64(const unsigned long long* in, unsigned long long* out, uint64_t n, void* scratch,
                       unsigned long long* total, hipStream_t s);
}

namespace cq {
namespace wr {

enum : uint32_t { W_NULL = 0, W_INT = 1, W_DBL = 2, W_STR = 3, W_DATE = 4 };

struct WCell {            // 16 bytes
    uint32_t kind;
    uint32_t len;         // STRING: bytes (up to the C string's NUL)
    uint64_t bits;        // INT value, DOUBLE bits, DATE y << 32 | m << 16 | d (as unsigned 16-bit fields
                          // of the signed ints), STRING: arena offset
};

struct Counter {
    uint64_t n = 0;
    __device__ __forceinline__ void put(uint8_t) { n++; }
    __device__ __forceinline__ void put(const uint8_t*, uint32_t k) { n += k; }
};
struct Writer {
    uint8_t* p;
    __device__ __forceinline__ void put(uint8_t c) { *p++ = c; }
    __device__ __forceinline__ void put(const uint8_t* s, uint32_t k) {
        for (uint32_t i = 0; i < k; i++) p[i] = s[i];
        p += k;
    }
};

// decimal digits of v (v > 0 or the single digit 0)
template <class S>
__device__ void put_u64(S& s, uint64_t v) {
    uint8_t b[20];
    int k = 0;
    do { b[k++] = (uint8_t)('0' + v % 10); v /= 10; } while (v);
    while (k) s.put(b[--k]);
}

// "%d" of a signed int with at least `w` digits, zero padded ("%04d", "%02d")
template <class S>
__device__ void put_int_w(S& s, int32_t v, int w) {
    uint32_t u = v < 0 ? (uint32_t)(-(int64_t)v) : (uint32_t)v;
    uint8_t b[12];
    int k = 0;
    do { b[k++] = (uint8_t)('0' + u % 10); u /= 10; } while (u);
    if (v < 0) { s.put('-'); w--; }          // the width counts the sign: "%04d" of -5 is "-005"
    for (int i = k; i < w; i++) s.put('0');
    while (k) s.put(b[--k]);
}

// "%.2f" of a finite double
template <class S>
__device__ void put_f2(S& s, double x) {
    uint64_t bits;
    memcpy(&bits, &x, 8);
    const bool neg = (bits >> 63) != 0;
    const uint32_t ex = (uint32_t)(bits >> 52) & 0x7FF;
    uint64_t m = bits & ((1ULL << 52) - 1);
    if (ex == 0x7FF) {                                   // inf / nan
        if (neg) s.put('-');
        const uint8_t* t = (const uint8_t*)(m ? "nan" : "inf");
        s.put(t, 3);
        return;
    }
    int32_t e;
    if (ex == 0) e = -1074;
    else { m |= 1ULL << 52; e = (int32_t)ex - 1075; }
    if (neg) s.put('-');
    if (e >= 0) {
        // an integer m * 2^e: exact digits by a multi-limb number (<= 1024 bits), then ".00"
        uint32_t lim[33];
        int nl = 0;
        lim[nl++] = (uint32_t)m;
        lim[nl++] = (uint32_t)(m >> 32);
        for (int32_t k = 0; k < e; k++) {             // times 2, e times (e <= 971)
            uint32_t carry = 0;
            for (int i = 0; i < nl; i++) {
                const uint32_t v = lim[i];
                lim[i] = (v << 1) | carry;
                carry = v >> 31;
            }
            if (carry) lim[nl++] = carry;
        }
        while (nl > 1 && lim[nl - 1] == 0) nl--;
        uint32_t chunks[36];                          // base 10^9, least significant first
        int nc = 0;
        while (nl > 1 || lim[0] != 0) {
            uint64_t r = 0;
            for (int i = nl - 1; i >= 0; i--) {
                const uint64_t cur = (r << 32) | lim[i];
                lim[i] = (uint32_t)(cur / 1000000000u);
                r = cur % 1000000000u;
            }
            chunks[nc++] = (uint32_t)r;
            while (nl > 1 && lim[nl - 1] == 0) nl--;
        }
        if (nc == 0) s.put('0');
        else {
            put_u64(s, chunks[nc - 1]);
            for (int i = nc - 2; i >= 0; i--) {
                uint32_t v = chunks[i];
                uint8_t b[9];
                for (int k = 8; k >= 0; k--) { b[k] = (uint8_t)('0' + v % 10); v /= 10; }
                s.put(b, 9);
            }
        }
        s.put('.'); s.put('0'); s.put('0');
        return;
    }
    // |x| = m / 2^sh: q = round-half-even(m * 100 / 2^sh) in 128 bits
    const uint32_t sh = (uint32_t)(-e);
    const unsigned __int128 p = (unsigned __int128)m * 100u;
    uint64_t q;
    bool round_up;
    if (sh >= 128) { q = 0; round_up = false; }
    else {
        const unsigned __int128 qq = p >> sh;
        const unsigned __int128 rem = p - (qq << sh);
        const unsigned __int128 half = (unsigned __int128)1 << (sh - 1);
        q = (uint64_t)qq;
        round_up = rem > half || (rem == half && (q & 1));
    }
    if (round_up) q++;
    put_u64(s, q / 100);
    s.put('.');
    s.put((uint8_t)('0' + (q / 10) % 10));
    s.put((uint8_t)('0' + q % 10));
}

template <class S>
__device__ void put_cell(S& s, const WCell& c, const uint8_t* arena, uint8_t delim) {
    switch (c.kind) {
        case W_INT: {
            const int64_t v = (int64_t)c.bits;
            if (v < 0) { s.put('-'); put_u64(s, 0 - (uint64_t)v); }
            else put_u64(s, (uint64_t)v);
            break;
        }
        case W_DBL: {
            double d;
            memcpy(&d, &c.bits, 8);
            put_f2(s, d);
            break;
        }
        case W_DATE:
            put_int_w(s, (int32_t)(c.bits >> 32), 4); s.put('-');
            put_int_w(s, (int32_t)(int16_t)((c.bits >> 16) & 0xFFFF), 2); s.put('-');
            put_int_w(s, (int32_t)(int16_t)(c.bits & 0xFFFF), 2);
            break;
        case W_STR: {
            const uint8_t* p = arena + c.bits;
            bool q = false;
            for (uint32_t i = 0; i < c.len && !q; i++) q = p[i] == delim || p[i] == '"' || p[i] == '\n' || p[i] == '\r';
            if (!q) { s.put(p, c.len); break; }
            s.put('"');
            for (uint32_t i = 0; i < c.len; i++) {
                if (p[i] == '"') s.put('"');
                s.put(p[i]);
            }
            s.put('"');
            break;
        }
        default: break;
    }
}

template <class S>
__device__ void put_row(S& s, const WCell* cells, uint32_t nc, const uint8_t* arena, uint8_t delim) {
    for (uint32_t j = 0; j < nc; j++) {
        if (j) s.put(delim);
        put_cell(s, cells[j], arena, delim);
    }
    s.put('\n');
}

__global__ void row_len_kernel(const WCell* __restrict__ cells, const uint64_t* __restrict__ row_cell,
                               uint32_t nrows, const uint8_t* __restrict__ arena, uint8_t delim,
                               unsigned long long* __restrict__ len) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    Counter c;
    put_row(c, cells + row_cell[r], (uint32_t)(row_cell[r + 1] - row_cell[r]), arena, delim);
    len[r] = c.n;
}

__global__ void row_write_kernel(const WCell* __restrict__ cells, const uint64_t* __restrict__ row_cell,
                                 uint32_t nrows, const uint8_t* __restrict__ arena, uint8_t delim,
                                 const unsigned long long* __restrict__ off, uint8_t* __restrict__ out) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    Writer w{out + off[r]};
    put_row(w, cells + row_cell[r], (uint32_t)(row_cell[r + 1] - row_cell[r]), arena, delim);
}

}  // namespace wr
}  // namespace cq

namespace {
struct Dev {                                 // device allocations of one write, freed on every exit
    std::vector<void*> p;
    void* get(size_t n) {
        void* q = nullptr;
        if (hipMalloc(&q, n < 16 ? 16 : n) != hipSuccess) return nullptr;
        p.push_back(q);
        return q;
    }
    ~Dev() {
        for (void* q : p) (void)hipFree(q);
    }
};
}  // namespace

extern "C" {

// write_csv_file (reference utils.c:220-289) for any result table: the header by
// the host, every row formatted on the GPU.  Same messages as the reference.
// Returns 0, or -1 (message on stderr) when the file or the device fails.
int cqgpu_write_csv(const char* filename, const cq_table* result, char delimiter) {
    using namespace cq::wr;
    FILE* f = fopen(filename, "w");
    if (!f) {
        fprintf(stderr, "Error: Cannot open output file '%s'\n", filename);
        return -1;
    }
    for (int i = 0; i < result->ncols; i++) {
        if (i > 0) fputc(delimiter, f);
        fputs(result->columns[i].name ? result->columns[i].name : "(null)", f);
    }
    fputc('\n', f);
    const uint32_t nrows = result->nrows > 0 ? (uint32_t)result->nrows : 0u;
    int rc = 0;
    if (nrows) {
        // pack: cells row-major (each row's own column count), strings in one arena
        std::vector<uint64_t> row_cell(nrows + 1, 0);
        std::vector<WCell> cells;
        std::vector<uint8_t> arena;
        for (uint32_t r = 0; r < nrows; r++) {
            const cq_row& row = result->rows[r];
            for (int j = 0; j < row.ncols; j++) {
                const cq_value& v = row.values[j];
                WCell w{W_NULL, 0, 0};
                switch (v.kind) {
                    case CQ_V_INT: w.kind = W_INT; w.bits = (uint64_t)v.u.i; break;
                    case CQ_V_DOUBLE: w.kind = W_DBL; memcpy(&w.bits, &v.u.f, 8); break;
                    case CQ_V_DATE:
                        w.kind = W_DATE;
                        w.bits = ((uint64_t)(uint32_t)v.u.date.y << 32) | ((uint64_t)(uint16_t)v.u.date.m << 16) |
                                 (uint16_t)v.u.date.d;
                        break;
                    case CQ_V_STRING: {
                        const char* sv = v.u.s ? v.u.s : "";
                        const size_t n = strlen(sv);
                        w.kind = W_STR;
                        w.len = (uint32_t)n;
                        w.bits = arena.size();
                        arena.insert(arena.end(), (const uint8_t*)sv, (const uint8_t*)sv + n);
                        break;
                    }
                    default: break;
                }
                cells.push_back(w);
            }
            row_cell[r + 1] = cells.size();
        }
        hipStream_t s = nullptr;
        Dev d;
        const size_t scr = cq_scan_scratch_bytes(nrows, 8);
        WCell* dc = (WCell*)d.get(cells.size() * sizeof(WCell));
        uint64_t* drc = (uint64_t*)d.get(row_cell.size() * 8);
        uint8_t* da = (uint8_t*)d.get(arena.size());
        unsigned long long* dlen = (unsigned long long*)d.get((size_t)nrows * 8);
        unsigned long long* doff = (unsigned long long*)d.get((size_t)nrows * 8);
        unsigned long long* dtot = (unsigned long long*)d.get(8);
        void* dscr = d.get(scr);
        unsigned long long total = 0;
        hipError_t e = (dc && drc && da && dlen && doff && dtot && dscr) ? hipSuccess : hipErrorOutOfMemory;
        if (e == hipSuccess && !cells.empty())
            e = hipMemcpyAsync(dc, cells.data(), cells.size() * sizeof(WCell), hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(drc, row_cell.data(), row_cell.size() * 8, hipMemcpyHostToDevice, s);
        if (e == hipSuccess && !arena.empty())
            e = hipMemcpyAsync(da, arena.data(), arena.size(), hipMemcpyHostToDevice, s);
        const uint32_t grid = (nrows + 255) / 256;
        if (e == hipSuccess) {
            hipLaunchKernelGGL(row_len_kernel, dim3(grid), dim3(256), 0, s, dc, drc, nrows, da, (uint8_t)delimiter, dlen);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = cq_scan_u64(dlen, doff, nrows, dscr, dtot, s);
        if (e == hipSuccess) e = hipMemcpyAsync(&total, dtot, 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        uint8_t* dout = nullptr;
        if (e == hipSuccess) {
            dout = (uint8_t*)d.get(total);
            if (!dout) e = hipErrorOutOfMemory;
        }
        std::vector<uint8_t> host(total);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(row_write_kernel, dim3(grid), dim3(256), 0, s, dc, drc, nrows, da, (uint8_t)delimiter,
                               doff, dout);
            e = hipGetLastError();
        }
        if (e == hipSuccess && total) e = hipMemcpyAsync(host.data(), dout, total, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            fprintf(stderr, "cq_amd: CSV writer: %s\n", hipGetErrorString(e));
            rc = -1;
        } else if (total && fwrite(host.data(), 1, total, f) != total) {
            fprintf(stderr, "Error: Cannot write output file '%s'\n", filename);
            rc = -1;
        }
    }
    fclose(f);
    if (rc == 0) printf("Result written to '%s'\n", filename);
    return rc;
}

}  // extern "C"
