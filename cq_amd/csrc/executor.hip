// executor.hip -- host side of libcqgpu: the drop-in evaluate_query, resident
// tables, plan compilation from the reference AST, kernel launches, result
// materialisation and the small host post-ops the reference also runs on its
// (small) result (HAVING, ORDER BY, DISTINCT, LIMIT).
//
// The SELECT orchestration mirrors evaluate_query_internal (reference
// evaluator.c:26-287); names below cite the reference function each piece
// replaces.  Every per-row operation runs on the GPU (scan.hip); the host only
// compiles the plan and shapes the few result rows.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cerrno>
#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <map>
#include <functional>
#include <set>
#include <memory>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

#include <fcntl.h>
#include <link.h>
#include <malloc.h>
#include <strings.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <rccl/rccl.h>

#include "../../include/cqgpu.h"
#include "plan.h"

using namespace cq;

extern "C" {
uint32_t cq_lean_pick_ws(const uint8_t* data, uint64_t n);
uint64_t cq_lean_long_cols(const uint8_t* data, uint64_t n, uint32_t delim);
uint64_t cq_cols_longer_than(const uint8_t* data, uint64_t n, uint32_t delim, uint32_t limit);
uint32_t cq_scan_cand_stride(const ScanPlan* P, int grouped);
size_t cq_scan_lds_bytes(const ScanPlan* P, int grouped);
int cq_scan_occupancy(const ScanPlan* P, int grouped);
hipError_t cq_launch_scan(const uint8_t* g, const ScanPlan* P, const GroupTable* gt, const GroupTable* rt,
                          ScanStats* stats, unsigned long long* row_out, unsigned long long row_cap, int grouped,
                          int grid, hipStream_t s, Cell* cells_out, unsigned long long* slow_list,
                          unsigned long long slow_cap);
hipError_t cq_launch_finish_pack(const uint8_t* g, uint64_t n, const GroupOut* out, const unsigned long long* ofirst,
                                 const unsigned int* count, unsigned int cap_out, const FinishDesc* D, uint8_t* dst,
                                 const ScanStats* stats, uint8_t* hdr, hipStream_t s);
unsigned int cq_finish_pack_max();
hipError_t cq_launch_compact(const GroupTable* gt, const ScanPlan* P, GroupOut* out, unsigned int* count,
                             unsigned int cap_out, hipStream_t s, unsigned long long* ofirst);
hipError_t cq_launch_comp_text(const cq::Cell* cells, uint32_t n, uint32_t cap, uint8_t* out, uint32_t* lens,
                               hipStream_t s);
hipError_t cq_launch_gather(const uint8_t* g, const ScanPlan* P, const unsigned long long* recs,
                            uint32_t nrec, Cell* out, hipStream_t s);
hipError_t cq_launch_copy_strings(const Cell* cells, uint32_t n, const unsigned long long* offs,
                                  uint8_t* out, hipStream_t s);
cq::Cell cq_host_parse_cell(const uint8_t* text, uint32_t len);
cq::GKey cq_host_group_key(cq::Cell c);
cq::Cell cq_host_eval(const cq::Insn* code, uint32_t n, const cq::Cell* cols, const cq::Cell* consts);
hipError_t cq_launch_cells(const uint8_t* g, uint64_t tn, const unsigned long long* recs, uint32_t n,
                           const cq::ColsDesc* D, cq::Cell* out, hipStream_t s);
hipError_t cq_launch_join_code(const cq::Cell* cells, uint32_t stride, uint32_t kcol, uint32_t n,
                               unsigned long long* codes, uint32_t* cls, uint32_t* idx, unsigned int* per_class,
                               hipStream_t s);
hipError_t cq_launch_gather_codes(const unsigned long long* codes, const uint32_t* idx, uint32_t n,
                                  unsigned long long* out, hipStream_t s);
hipError_t cq_launch_dict_build(const void* all, const void* text, uint32_t n, uint32_t* state, uint32_t* rec_of,
                                uint32_t* first_of, uint32_t cap, uint32_t* slot_of, unsigned int* err, hipStream_t s);
hipError_t cq_launch_dict_flag(const uint32_t* slot_of, const uint32_t* first_of, uint32_t n, uint32_t* flag,
                               hipStream_t s);
hipError_t cq_launch_rebase(void* recs, uint32_t n, uint64_t add, hipStream_t s);
hipError_t cq_launch_fill_rows(unsigned long long* dst, uint64_t g, uint32_t w, const unsigned long long* row,
                               hipStream_t s);
hipError_t cq_launch_dict_scatter(const uint32_t* slot_of, const uint32_t* first_of, const uint32_t* dense_of,
                                  uint32_t mine, uint32_t m, const unsigned long long* st_sum,
                                  const unsigned long long* st_min, const unsigned long long* st_priv, uint32_t W,
                                  uint32_t P, uint32_t Q, unsigned long long* dsum, unsigned long long* dmin,
                                  unsigned long long* dpriv, uint32_t* dense_id, hipStream_t s);
hipError_t cq_launch_ext_mask(const unsigned long long* dmin, const unsigned long long* dpriv, uint64_t g, uint32_t P,
                              uint32_t Q, uint32_t nmm, unsigned long long* dext, hipStream_t s);
hipError_t cq_launch_cell_mask(const unsigned long long* dmin, const unsigned long long* dext,
                               const unsigned long long* dpriv, const double* dsum, uint64_t g, uint32_t P, uint32_t Q,
                               uint32_t W, uint32_t nmm, uint32_t R, uint32_t nv, uint32_t vsum0,
                               unsigned long long* dcell, double* dvla, hipStream_t s);
hipError_t cq_launch_class_mask(const cq::Cell* cells, uint32_t stride, uint32_t kcol, uint32_t n, unsigned int* mask,
                                hipStream_t s);
hipError_t cq_launch_run_bounds(const uint32_t* ssid, uint32_t n, cq::HSlot* slots, hipStream_t s);
hipError_t cq_launch_hash_build(const unsigned long long* codes, const uint32_t* cls, uint32_t n, const cq::JoinHashW* H,
                                uint32_t* sid, unsigned long long* overflow, hipStream_t s);
hipError_t cq_sort_u32(void* temp, size_t* temp_bytes, const unsigned int* kin, unsigned int* kout,
                       const unsigned int* vin, unsigned int* vout, size_t n, int bits, hipStream_t s);
hipError_t cq_launch_join_count(const cq::Cell* L, uint32_t ls, uint32_t lk, uint32_t nL, const cq::JoinRight* J,
                                int outer_left, uint32_t* lo, unsigned long long* cnt, hipStream_t s);
hipError_t cq_launch_join_emit(const cq::Cell* L, uint32_t ls, uint32_t lk, uint32_t nL, const cq::JoinRight* J,
                               const uint32_t* lo, const unsigned long long* cnt, const unsigned long long* offs,
                               uint2* pairs, unsigned int* rmatched, hipStream_t s);
hipError_t cq_launch_route_runs(const uint32_t* dest, const uint32_t* len, uint32_t n, uint32_t nw, uint32_t nranks,
                                unsigned long long* rcnt, unsigned long long* rbytes, hipStream_t s);
hipError_t cq_launch_typed_summary(const unsigned int* roffs, const unsigned int* rcnt, const unsigned int* wbase,
                                   const unsigned int* wcount, uint64_t nw, uint32_t nranks, const uint32_t* ctl,
                                   uint32_t* out, hipStream_t s);
hipError_t cq_launch_route_dest_mode(const uint32_t* cls, uint32_t n, uint32_t nranks, uint32_t rep, uint32_t fixed,
                                    uint32_t* dest, hipStream_t s);
hipError_t cq_launch_pair_rep_flags(const uint2* pairs, unsigned long long np, const cq::Cell* L, uint32_t ls,
                                    uint32_t lk, const cq::Cell* R, uint32_t rs, uint32_t rk, uint32_t major,
                                    unsigned int* flags, hipStream_t s);
hipError_t cq_launch_route_run_starts(const unsigned long long* cbase, const unsigned long long* bbase,
                                     const unsigned long long* rcnt, const unsigned long long* rbytes, uint32_t nw,
                                     uint32_t nranks, unsigned long long* starts, hipStream_t s);
hipError_t cq_launch_route_scatter(const uint8_t* g, const unsigned long long* recs, const uint32_t* dest,
                                   const uint32_t* len, uint32_t n, uint32_t nw, uint32_t nranks, uint64_t end,
                                   const unsigned long long* cbase, const unsigned long long* bbase, uint64_t gid_base,
                                   uint8_t* out, unsigned long long* gids, hipStream_t s);
hipError_t cq_launch_pack_first_gid(uint8_t* pk, const unsigned int* count, uint32_t cap, uint32_t rec,
                                    const unsigned long long* starts, unsigned long long n,
                                    const unsigned long long* gids, hipStream_t s);
hipError_t cq_launch_gid_narrow(const unsigned long long* in, uint64_t n, uint32_t* out, hipStream_t s);
hipError_t cq_launch_gid_widen(const uint32_t* in, uint64_t n, unsigned long long* out, hipStream_t s);
hipError_t cq_launch_outer_global(unsigned int* unm, uint32_t n, const uint8_t* gset, uint32_t emit, uint8_t* matched_out,
                                  hipStream_t s);
hipError_t cq_launch_join_fill(const unsigned int* flags, const unsigned int* pos, uint32_t n, unsigned long long base,
                               int right_side, uint2* pairs, hipStream_t s);
hipError_t cq_launch_join_gather(const uint2* pairs, unsigned long long np, const cq::JoinMap* M, const cq::Cell* L,
                                 const cq::Cell* R, cq::Cell* out, hipStream_t s);
hipError_t cq_sort_classes(void* temp, size_t* temp_bytes, const unsigned int* kin, unsigned int* kout,
                           const unsigned int* vin, unsigned int* vout, size_t n, hipStream_t s);
hipError_t cq_launch_join_agg(const uint2* pairs, unsigned long long np, const cq::JoinMap* M, const cq::Cell* L,
                              const cq::Cell* R, const cq::ScanPlan* P, const cq::GroupTable* gt,
                              cq::ScanStats* stats, int grouped, hipStream_t s);
hipError_t cq_launch_join_filter(const uint2* pairs, unsigned long long np, const cq::JoinMap* M, const cq::Cell* L,
                                 const cq::Cell* R, const cq::ScanPlan* P, unsigned int* flags, hipStream_t s);
hipError_t cq_launch_join_project(const uint2* pairs, unsigned long long np, const unsigned int* flags,
                                  const unsigned int* pos, unsigned long long lo, uint32_t m, const cq::JoinMap* M,
                                  const cq::Cell* L, const cq::Cell* R, const cq::Insn* code, const uint32_t* off,
                                  int nout, const cq::Cell* consts, cq::Cell* scratch, cq::Cell* out, hipStream_t s);
hipError_t cq_launch_join_finish(const cq::GroupOut* out, const unsigned int* count, unsigned int cap_out,
                                 const uint2* pairs, const cq::JoinMap* M, const cq::Cell* L, const cq::Cell* R,
                                 int nacc, uint32_t sb, cq::Cell* cells, uint8_t* bytes, hipStream_t s);
size_t cq_join_sum_lds(int nacc);
hipError_t cq_launch_comp_verify(const uint2* pairs, unsigned long long np, const cq::JoinMap* M, const cq::Cell* L,
                                 const cq::Cell* R, const cq::ScanPlan* P, const cq::GroupTable* gt, unsigned int* bad,
                                 hipStream_t s);
hipError_t cq_launch_join_sum(const uint2* pairs, unsigned long long np, const cq::JoinMap* M, const cq::Cell* L,
                              const cq::Cell* R, const cq::ScanPlan* P, const cq::GroupTable* gt,
                              cq::ScanStats* stats, int ncu, hipStream_t s);
hipError_t cq_launch_vla_pair_prep(const uint2* pairs, uint32_t n, const cq::JoinMap* M, const cq::JoinMap* V,
                                   const cq::Cell* L, const cq::Cell* R, const cq::ScanPlan* P, int grouped,
                                   unsigned long long* kw0, unsigned long long* kw1, unsigned long long* kcl,
                                   unsigned long long* vkey, unsigned int* flag, hipStream_t s);
hipError_t cq_launch_vla_prep(const cq::Cell* cells, uint32_t n, uint32_t nc, int gslot, uint32_t vslot,
                              unsigned long long* kw0, unsigned long long* kw1, unsigned long long* kcl,
                              unsigned long long* vkey, unsigned int* flag, hipStream_t s);
hipError_t cq_launch_vla_compact(const unsigned int* flag, const unsigned int* pos, uint32_t n, unsigned int* perm,
                                 hipStream_t s);
hipError_t cq_launch_vla_gather(const unsigned long long* a, const unsigned int* perm, uint32_t m,
                                unsigned long long* out, hipStream_t s);
hipError_t cq_launch_vla_heads(const unsigned long long* kw0, const unsigned long long* kw1,
                               const unsigned long long* kcl, const unsigned int* perm, uint32_t m, unsigned int* head,
                               hipStream_t s);
hipError_t cq_launch_vla_starts(const unsigned int* head, const unsigned int* sid, uint32_t m, unsigned int* start,
                                hipStream_t s);
hipError_t cq_launch_vla_reduce(const unsigned long long* vkey, const unsigned long long* kw0,
                                const unsigned long long* kw1, const unsigned long long* kcl, const unsigned int* perm,
                                const unsigned int* start, uint32_t nseg, uint32_t m, int kind, unsigned long long* out,
                                double* aux, hipStream_t s);
hipError_t cq_sort_codes(void* temp, size_t* temp_bytes, const unsigned long long* kin, unsigned long long* kout,
                         const unsigned int* vin, unsigned int* vout, size_t n, hipStream_t s);
hipError_t cq_excl_sum_u64(void* temp, size_t* temp_bytes, const unsigned long long* in, unsigned long long* out,
                           size_t n, hipStream_t s);
hipError_t cq_excl_sum_u32(void* temp, size_t* temp_bytes, const unsigned int* in, unsigned int* out, size_t n,
                           hipStream_t s);
size_t cq_pack_result_bytes(unsigned int ng, int nacc, uint32_t ncell, uint32_t sb);
hipError_t cq_launch_gm_pack(const cq::GroupOut* out, const unsigned int* count, unsigned int cap_out, int nacc,
                             uint32_t R, const cq::Cell* cells, const uint8_t* bytes, uint32_t sb, uint32_t maxg,
                             uint8_t* dst, const cq::ScanStats* stats, uint8_t* hdr, hipStream_t s);
size_t cq_gm_scan_bytes(uint32_t T);
hipError_t cq_launch_gm_merge(const uint8_t* buf, uint64_t B, uint32_t N, uint32_t maxg, int nacc, uint32_t R,
                              int grouped, uint32_t sb, uint32_t* state, uint32_t* rec_of, uint32_t* first_of, uint32_t cap,
                              uint32_t* slot_of, uint32_t* flag, uint32_t* dense, uint32_t* idx, void* scan_temp,
                              size_t scan_temp_bytes, unsigned int* err, uint8_t* dst, unsigned int* gcount,
                              uint8_t* mail, hipStream_t s);
int cq_fast_ext_plan(const cq::ScanPlan* P, int grouped);
hipError_t cq_launch_raw_merge(const cq::GroupTable* gt, const cq::GroupTable* rt, int nacc, cq::ScanStats* stats,
                               hipStream_t s, uint32_t max_mask = 0, const uint8_t* g = nullptr,
                               int pk_acc = -1, uint32_t pk_col = 0, uint32_t delim = ',');
hipError_t cq_launch_join_cross(uint32_t na, uint32_t nb, uint2* pairs, hipStream_t s);
uint64_t cq_jx_windows(uint64_t lo, uint64_t hi, uint32_t ws);
hipError_t cq_jx_extract(const uint8_t* g, uint64_t lo, uint64_t hi, uint32_t ws, uint32_t delim, uint32_t quote,
                         int kcol, int pcol, int build, int pass, unsigned long long* key, unsigned long long* pay,
                         uint32_t* off, unsigned int* wcount, const unsigned int* wbase, unsigned int cap,
                         unsigned int* flag, unsigned long long* krange, int grid, hipStream_t s);
hipError_t cq_jx_build(const unsigned long long* key, uint32_t n, void* table, uint64_t tcap, unsigned int* flag,
                       int grid, hipStream_t s);
size_t cq_jx_entry_bytes();
hipError_t cq_jx_build_direct(const unsigned long long* key, const unsigned long long* pay, const uint32_t* off,
                              uint32_t n, unsigned long long kmin, unsigned long long range, void* D,
                              unsigned int* flag, int grid, hipStream_t s);
size_t cq_jx_direct_bytes();
hipError_t cq_jx_star_extract(const uint8_t* g, uint64_t lo, uint64_t hi, uint32_t ws, uint32_t delim, uint32_t quote,
                              int kcol, int pcol, int build, unsigned long long kmin, unsigned long long range,
                              uint32_t stride, uint16_t* d16, uint32_t* l32, unsigned long long* ttab,
                              unsigned long long* gsum, unsigned long long* counter, unsigned int* flag,
                              unsigned long long* krange, uint32_t* notmono, unsigned long long* wfl,
                              uint32_t* gminix, int rp, int grid, hipStream_t s, unsigned long long* pent = nullptr,
                              uint32_t* pcnt = nullptr, uint32_t np = 0, uint32_t pcap = 0, uint32_t psh = 0);
hipError_t cq_jx_part_probe(const unsigned long long* pent, const uint32_t* pcnt, uint32_t nsrc, uint32_t np,
                            uint32_t pcap, unsigned long long range, uint16_t* d16, const uint32_t* notmono,
                            unsigned long long* gsum, uint32_t* gminix, unsigned long long* npairs, int grid,
                            hipStream_t s);
hipError_t cq_jx_star_order(const unsigned long long* wfl, unsigned long long nwin, uint32_t* notmono, hipStream_t s);
hipError_t cq_jx_star_init(void* d16, size_t d16_bytes, void* small, size_t small_bytes, uint32_t ff0, uint32_t ff1,
                           uint32_t ffw, const void* seed, size_t seed_bytes, int grid, hipStream_t s);
hipError_t cq_jx_star_first(const uint16_t* d16, const uint32_t* l32, unsigned long long range, const uint32_t* notmono,
                            uint32_t* gfirst, unsigned long long* nocc, int grid, hipStream_t s);
hipError_t cq_jx_star_flush(int grouped, int value, const unsigned long long* ttab, const unsigned long long* gsum,
                            const uint32_t* gfirst, const uint32_t* gminix, const uint32_t* l32, const uint32_t* notmono,
                            const unsigned long long* cnts, const cq::GroupTable* rt, int nacc, cq::ScanStats* stats,
                            unsigned int* flag, hipStream_t s);
uint32_t cq_jx_star_groups();
uint32_t cq_jx_rchunk();
hipError_t cq_jx_route(const uint8_t* g, uint64_t lo, uint64_t hi, uint32_t ws, uint32_t delim, uint32_t quote,
                       int kcol, int pcol, int build, int rp, int pass, uint32_t nranks, unsigned long long qbase,
                       unsigned long long gbase, unsigned int* rcnt, unsigned int* wcount, const unsigned int* roffs,
                       const unsigned int* wbase, void* rent, uint32_t cap, unsigned int* flag,
                       unsigned long long* krange, int grid, hipStream_t s);
hipError_t cq_jx_ent_build(const void* ent, unsigned long long n, uint32_t qoff, unsigned long long range, uint16_t* d16,
                           uint32_t* l32, unsigned long long* ttab, unsigned long long* nplaced, unsigned int* flag,
                           int grid, hipStream_t s, int ungrouped, uint32_t* notmono);
hipError_t cq_jx_ent_first(const uint32_t* gminix, const uint32_t* l32, const uint32_t* notmono, uint32_t* gfirst,
                           hipStream_t s);
hipError_t cq_jx_ent_part(const void* ent, unsigned long long n, uint32_t qoff, unsigned long long range, uint32_t np,
                          uint32_t pcap, uint32_t psh, unsigned long long* pent, uint32_t* pcnt, unsigned int* flag,
                          int grid, hipStream_t s);
hipError_t cq_jx_ent_probe(const void* ent, unsigned long long n, uint32_t qoff, unsigned long long range, uint16_t* d16,
                           unsigned long long* gsum, unsigned long long* npairs, int grid, hipStream_t s,
                           const uint32_t* notmono, uint32_t* gminix);
hipError_t cq_jx_probe(int grouped, int value, int direct, const unsigned long long* pkey,
                       const unsigned long long* ppay, const uint32_t* poff, uint32_t n, unsigned long long kmin,
                       const void* table, uint64_t tcap, const unsigned long long* bpay, const uint32_t* boff,
                       const cq::GroupTable* rt, int nacc, cq::ScanStats* stats, unsigned int* flag, int grid,
                       hipStream_t s);
hipError_t cq_launch_mail_copy(const void* src, const unsigned int* count, unsigned int cap_out, int nacc, uint32_t ncell,
                               uint32_t sb, void* dst, hipStream_t s);
hipError_t cq_launch_pack_result(const cq::GroupOut* out, const unsigned int* count, unsigned int cap_out, int nacc,
                                 const cq::Cell* cells, const uint8_t* bytes, uint32_t ncell, uint32_t sb,
                                 uint8_t* dst, const cq::ScanStats* stats, uint8_t* hdr, int order, hipStream_t s);
unsigned int cq_pack_order_max();
hipError_t cq_launch_finish(const uint8_t* g, uint64_t n, const cq::GroupOut* out, const unsigned int* count,
                            unsigned int cap_out, const cq::FinishDesc* D, cq::Cell* cells, uint8_t* bytes,
                            hipStream_t s);
hipError_t cq_launch_parse_literals(const uint8_t* text, const unsigned int* offs,
                                    const unsigned int* lens, uint32_t n, Cell* out, hipStream_t s);
hipError_t cq_launch_project(const uint8_t* g, const unsigned long long* recs, uint32_t nrec,
                             const ProjDesc* D, Cell* scratch, Cell* out, hipStream_t s);
int cq_set_scan_mode(int mode);
int cq_scan_uses_lean(const cq::ScanPlan* P, int with_cells);
int cq_fast_eligible(const cq::ScanPlan* P, int grouped, int want_rows);
int cq_scan_kernel_kind(const cq::ScanPlan* P, int grouped, int want_rows, int with_cells);
uint32_t cq_fast_seed(const uint8_t* data, uint64_t n, uint32_t delim, uint32_t quote, uint32_t col,
                      unsigned long long* tags);
size_t cq_fast_seed_slots();
hipError_t cq_sort_offsets(void* temp, size_t* temp_bytes, const unsigned long long* in,
                           unsigned long long* out, size_t n, int bits, hipStream_t s);
hipError_t cq_launch_route_len(const uint8_t* g, const unsigned long long* recs, uint32_t n,
                               const unsigned long long* codes, const uint32_t* cls, uint32_t nranks, uint32_t* len,
                               uint32_t* dest, hipStream_t s);
uint32_t cq_rs_blocks(uint64_t n);
hipError_t cq_launch_rs_count(const uint8_t* g, uint64_t lo, uint64_t n, unsigned long long* counts, hipStream_t s);
hipError_t cq_launch_rs_write(const uint8_t* g, uint64_t lo, uint64_t n, const unsigned long long* base,
                              unsigned long long* out, hipStream_t s);
hipError_t cq_launch_route_bounds(const uint32_t* dsorted, const unsigned long long* off,
                                  const unsigned long long* lens, uint32_t n, uint32_t nranks,
                                  unsigned long long* starts, hipStream_t s);
hipError_t cq_sort_codes(void* temp, size_t* temp_bytes, const unsigned long long* kin, unsigned long long* kout,
                         const unsigned int* vin, unsigned int* vout, size_t n, hipStream_t s);
hipError_t cq_sort_dest(void* temp, size_t* temp_bytes, const unsigned int* kin, unsigned int* kout,
                        const unsigned int* vin, unsigned int* vout, size_t n, int bits, hipStream_t s);
hipError_t cq_launch_iota_u64(uint32_t n, unsigned long long* out, hipStream_t s);
hipError_t cq_launch_gather_len(const uint32_t* len, const uint32_t* order, uint32_t n, unsigned long long* out,
                                hipStream_t s);
hipError_t cq_launch_route_project(const uint8_t* g, const unsigned long long* recs, uint32_t n, uint64_t end,
                                   uint64_t mask, uint32_t last_keep, uint32_t delim, uint32_t quote,
                                   const unsigned long long* codes, const uint32_t* cls, uint32_t nranks, uint32_t* len,
                                   uint32_t* dest, uint8_t* proj, hipStream_t s);
hipError_t cq_launch_route_copy(const uint8_t* g, const unsigned long long* recs, const uint32_t* order,
                                const uint32_t* len, const unsigned long long* off, uint32_t n, uint64_t gid_base,
                                uint8_t* out, unsigned long long* gids, hipStream_t s);
hipError_t cq_launch_chain_key(const uint2* pairs, unsigned long long np, const unsigned long long* prev,
                               unsigned long long prev_none, unsigned long long radix, const unsigned long long* rg,
                               unsigned long long r_none, unsigned long long* out, hipStream_t s);
hipError_t cq_launch_key_pick(const unsigned long long* key, const unsigned long long* pidx, uint32_t n,
                              unsigned long long* out, hipStream_t s);
hipError_t cq_launch_offset_gid(const unsigned long long* starts, unsigned long long n, const unsigned long long* q,
                               uint32_t nq, const unsigned long long* gids, unsigned long long* out, hipStream_t s);
hipError_t cq_launch_key_flagged(const unsigned long long* key, unsigned long long np, const unsigned int* flags,
                                 const unsigned int* pos, unsigned long long* out, hipStream_t s);
hipError_t cq_launch_pair_gid(const uint2* pairs, const unsigned long long* pidx, uint32_t n,
                              const unsigned long long* lg, const unsigned long long* rg, unsigned long long* out,
                              hipStream_t s);
hipError_t cq_launch_pair_gid_flagged(const uint2* pairs, unsigned long long np, const unsigned int* flags,
                                      const unsigned int* pos, const unsigned long long* lg,
                                      const unsigned long long* rg, unsigned long long* out, hipStream_t s);
}

// reference evaluator.c:23
cq_csv_config global_csv_config = {',', '"', true};

namespace {

constexpr uint64_t PAD_BEFORE = 256;   // byte 0 lands 256-aligned: lean_kernel windows are 128-byte aligned
constexpr uint64_t PAD_AFTER = 32768 + 2048 + 256;   // >= WIN + MARGIN of the scan
constexpr uint64_t NOPOS = ~0ULL;

std::string g_err, g_inel;
cqgpu_stats g_stats;
unsigned long long g_clk[8];     // profiling builds: ScanStats.clk of the last scan
cqgpu_fallback_fn g_fallback = nullptr;

void set_err(const char* fmt, ...) {
    char b[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(b, sizeof b, fmt, ap);
    va_end(ap);
    g_err = b;
    fprintf(stderr, "%s\n", b);
}

struct HipError {
    std::string msg;
};
#define HIPCHECK(x)                                                                   \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess)                                                         \
            throw HipError{std::string(#x) + ": " + hipGetErrorString(e_)};          \
    } while (0)

struct Ineligible {
    std::string why;
};
// a MIN/MAX argument mixes value classes: the fused scans hand the plan to the
// cells path, whose pair aggregation folds such extremes exactly
struct MixedExtremes : Ineligible {
    MixedExtremes() : Ineligible{"MIN/MAX over a column mixing numbers, strings and dates"} {}
};

// ------------------------------------------------------------------ per-device context
struct DevCtx {
    int device = -1;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int ncu = 0;
    // reusable workspace
    void* ws = nullptr;
    size_t ws_size = 0;
    void* pinned = nullptr;
    size_t pinned_size = 0;
    uint8_t* mail = nullptr;           // host-mapped, coherent: kernels write results here directly
    size_t mail_size = 0;
    // per-query scratch (literals, gathers, string fetches): a bump region reset at
    // the start of every query, so the query path makes no hipMalloc / hipFree
    uint8_t* bump = nullptr;
    size_t bump_size = 0, bump_used = 0;
    uint64_t query_gen = 1;            // bumped at every query (literal cache lifetimes)
};
DevCtx g_ctx[64];

// Two HIP runtimes in one process (e.g. /opt/rocm's, pulled in by this library, and
// the copy a torch wheel ships, loaded afterwards) each own a device state and free
// the shared one twice at exit: refused at the first device use, with the fix named
int count_hip_runtime(struct dl_phdr_info* info, size_t, void* data) {
    const char* n = info->dlpi_name;
    if (n && strstr(n, "libamdhip64.so")) {
        char buf[4096];
        const char* r = realpath(n, buf);
        ((std::set<std::string>*)data)->insert(r ? r : n);
    }
    return 0;
}
void check_one_hip_runtime() {
    std::set<std::string> seen;
    dl_iterate_phdr(count_hip_runtime, &seen);
    if (seen.size() > 1) {
        std::string all;
        for (auto& s : seen) all += " " + s;
        throw HipError{"two HIP runtimes are loaded in this process (" + all.substr(1) +
                       "): load the host framework's HIP (e.g. import torch) before libcqgpu.so"};
    }
}

DevCtx& ctx() {
    int dev = 0;
    HIPCHECK(hipGetDevice(&dev));
    DevCtx& c = g_ctx[dev & 63];
    if (c.device != dev) {
        check_one_hip_runtime();
        c.device = dev;
        HIPCHECK(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
        HIPCHECK(hipEventCreate(&c.ev0));
        HIPCHECK(hipEventCreate(&c.ev1));
        hipDeviceProp_t prop;
        HIPCHECK(hipGetDeviceProperties(&prop, dev));
        c.ncu = prop.multiProcessorCount;
    }
    return c;
}

void* workspace(DevCtx& c, size_t bytes) {
    if (bytes > c.ws_size) {
        if (c.ws) HIPCHECK(hipFree(c.ws));
        size_t sz = std::max(bytes, c.ws_size * 2);
        HIPCHECK(hipMalloc(&c.ws, sz));
        c.ws_size = sz;
    }
    return c.ws;
}

// per-query device scratch: from the context's bump region when it fits, else an
// owned allocation freed with the object
constexpr size_t BUMP_BYTES = 8u << 20;
void bump_reset(DevCtx& c) { c.bump_used = 0; c.query_gen++; }
struct Scratch {
    uint8_t* p = nullptr;
    bool owned = false;
    Scratch() = default;
    Scratch(DevCtx& c, size_t bytes) { get(c, bytes); }
    void get(DevCtx& c, size_t bytes) {
        release();
        bytes = (std::max<size_t>(bytes, 16) + 255) & ~(size_t)255;
        if (!c.bump) {
            HIPCHECK(hipMalloc(&c.bump, BUMP_BYTES));
            c.bump_size = BUMP_BYTES;
            c.bump_used = 0;
        }
        if (c.bump_used + bytes <= c.bump_size) {
            p = c.bump + c.bump_used;
            c.bump_used += bytes;
            owned = false;
        } else {
            HIPCHECK(hipMalloc(&p, bytes));
            owned = true;
        }
    }
    void release() {
        if (p && owned) (void)hipFree(p);
        p = nullptr;
        owned = false;
    }
    Scratch(const Scratch&) = delete;
    Scratch& operator=(const Scratch&) = delete;
    ~Scratch() { release(); }
};

// owned device allocation
// Device scratch blocks are recycled instead of hipFree'd: hipFree synchronises
// the device and cost ~140 us per call (74 calls per repartitioned-join step,
// ~10 ms).  Every kernel and copy of the library runs on its device's one DevCtx
// stream, so a block released here and handed out again ON THE SAME DEVICE is only
// touched by work enqueued after everything that used it before: the idle lists
// are per device, and a block goes back to the list of the device it was
// allocated on.  Released blocks are kept up to DEVPOOL_KEEP bytes per device; a
// failed hipMalloc empties that device's list and retries.
constexpr size_t DEVPOOL_KEEP = 8ull << 30;
constexpr int DEVPOOL_MAXDEV = 64;
struct DevPool {
    std::multimap<size_t, void*> idle[DEVPOOL_MAXDEV];
    size_t idle_bytes[DEVPOOL_MAXDEV] = {};
    std::unordered_map<void*, std::pair<size_t, int>> live;     // block -> (size class, device)
};
DevPool& devpool() {
    static DevPool* P = new DevPool;      // never destroyed: blocks outlive static teardown
    return *P;
}
int devpool_device() {
    int d = 0;
    HIPCHECK(hipGetDevice(&d));
    if (d < 0 || d >= DEVPOOL_MAXDEV) throw HipError{"device index beyond the scratch pool"};
    return d;
}
size_t devpool_class(size_t n) {          // 4 size classes per power of two
    n = std::max<size_t>(n, 256);
    if (n <= 4096) return (n + 255) & ~(size_t)255;
    int k = 63 - __builtin_clzll((unsigned long long)n);
    const size_t step = (size_t)1 << (k - 2);
    return (n + step - 1) & ~(step - 1);
}
void devpool_trim(int dev, size_t keep) {   // frees blocks of `dev` (the current device)
    DevPool& P = devpool();
    while (P.idle_bytes[dev] > keep && !P.idle[dev].empty()) {
        auto it = std::prev(P.idle[dev].end());   // largest first
        P.idle_bytes[dev] -= it->first;
        (void)hipFree(it->second);
        P.idle[dev].erase(it);
    }
}
void* devpool_get(size_t bytes) {
    DevPool& P = devpool();
    const int dev = devpool_device();
    const size_t sz = devpool_class(bytes);
    auto it = P.idle[dev].find(sz);
    void* p = nullptr;
    if (it != P.idle[dev].end()) {
        p = it->second;
        P.idle[dev].erase(it);
        P.idle_bytes[dev] -= sz;
    } else if (hipMalloc(&p, sz) != hipSuccess) {
        (void)hipGetLastError();
        devpool_trim(dev, 0);
        HIPCHECK(hipMalloc(&p, sz));
    }
    P.live[p] = {sz, dev};
    return p;
}
void devpool_put(void* p) {
    DevPool& P = devpool();
    auto it = P.live.find(p);
    if (it == P.live.end()) { (void)hipFree(p); return; }
    const size_t sz = it->second.first;
    const int dev = it->second.second;
    P.live.erase(it);
    P.idle[dev].emplace(sz, p);
    P.idle_bytes[dev] += sz;
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur == dev) devpool_trim(dev, DEVPOOL_KEEP);
}

struct DevBuf {
    void* p = nullptr;
    DevBuf() = default;
    explicit DevBuf(size_t bytes) { p = devpool_get(bytes); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { if (p) devpool_put(p); }
    template <class T> T* as() const { return (T*)p; }
};

void* pinned(DevCtx& c, size_t bytes) {
    if (bytes > c.pinned_size) {
        if (c.pinned) HIPCHECK(hipHostFree(c.pinned));
        size_t sz = std::max(bytes, std::max<size_t>(c.pinned_size * 2, 1 << 20));
        HIPCHECK(hipHostMalloc(&c.pinned, sz, hipHostMallocDefault));
        c.pinned_size = sz;
    }
    return c.pinned;
}

// the result mailbox: host memory the device writes over PCIe (fine-grained,
// coherent), read by the host after the stream's one synchronisation
uint8_t* mailbox(DevCtx& c, size_t bytes) {
    if (bytes > c.mail_size) {
        if (c.mail) HIPCHECK(hipHostFree(c.mail));
        c.mail = nullptr;
        size_t sz = std::max(bytes, std::max<size_t>(c.mail_size * 2, 4 << 20));
        HIPCHECK(hipHostMalloc((void**)&c.mail, sz, hipHostMallocMapped | hipHostMallocCoherent));
        c.mail_size = sz;
    }
    return c.mail;
}

double as_dbl(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
uint64_t dbl_bits(double d) { uint64_t b; memcpy(&b, &d, 8); return b; }

// C-locale helpers
bool is_space(int c) { return c == ' ' || (c >= 9 && c <= 13); }
const char* ci_find(const char* hay, const char* needle) {   // cq_strcasestr
    size_t n = strlen(needle);
    for (const char* p = hay; *p; p++)
        if (strncasecmp(p, needle, n) == 0) return p;
    return nullptr;
}
std::string rtrim(std::string s) {
    while (!s.empty() && is_space((unsigned char)s.back())) s.pop_back();
    return s;
}

}  // namespace

// ------------------------------------------------------------------ resident table
// join-key repartition state of a shard between cqgpu_route_plan and cqgpu_route_fill
struct RouteState {
    DevBuf recs, order, len, off;
    DevBuf proj;                   // the projected records at their source offsets (keep != ~0)
    // nranks <= 64: the destination-run layout (route.hip route_runs_kernel) -- each
    // record's destination, and every (destination, wave) run's record / byte base
    DevBuf dest, cbase, bbase;
    uint32_t nw = 0, nranks = 0;
    bool runs = false;
    uint32_t n = 0;
    uint64_t bytes = 0;
    uint64_t keep = ~0ull;         // columns sent (route_keep_mask; ~0: whole records)
    uint32_t last_keep = ~0u;
};

// the typed join exchange's send side of one table (cqgpu_typed_count / _send): the
// count pass's per (destination, window) entry counts and their scan, then the entries,
// destination d's in [rstart[d], rstart[d + 1]) (16 B build, 8 B probe)
struct TypedSend {
    uint32_t N = 0, ws = 0;
    int rp = 2;
    uint64_t qbase = 0, nwin = 0;
    DevBuf rcnt, roffs, wcount, wbase;
    std::vector<uint64_t> counts, rstart;
    uint64_t nrec = 0;                              // (build) the table's records
    uint32_t flags = 0;
    unsigned long long krange[2] = {~0ull, 0ull};   // the build side's keys' min, max (every non-NULL one)
    DevBuf ent;
    uint64_t esize = 0;
    bool emitted = false;
    bool one_pass = false;                          // (probe) entries written by the count (ROUTE 3)
    uint32_t eflags = 0;                            // one pass: the emit pass's flags (512)
};

constexpr uint64_t SAMPLE_BYTES = 256u << 10;   // bytes a table keeps for plan-time sampling

// the device byte ranges of the live tables: a group's STRING cells (representative,
// MIN/MAX and long-key cells) address table bytes, checked before the copy kernel
// dereferences them (a kernel bug becomes an error, never an out-of-bounds read)
std::map<uintptr_t, uintptr_t> g_table_ranges;   // begin -> end
void note_table_bytes(const uint8_t* p, size_t n) { if (p) g_table_ranges[(uintptr_t)p] = (uintptr_t)p + n; }
void forget_table_bytes(const uint8_t* p) { if (p) g_table_ranges.erase((uintptr_t)p); }
bool in_some_table(uint64_t a, uint32_t len) {
    auto it = g_table_ranges.upper_bound((uintptr_t)a);
    if (it == g_table_ranges.begin()) return false;
    --it;
    return a >= it->first && a + len <= it->second;
}

struct cqgpu_table {
    uint8_t* dbuf = nullptr;
    const uint8_t* g = nullptr;      // device byte 0
    uint64_t n = 0;
    uint64_t base_offset = 0;
    cq_csv_config cfg{',', '"', true};
    std::vector<std::string> names;
    std::string header_rec;          // the header record's bytes (routed tables rebuilt on a rank reuse it)
    uint64_t data_begin = 0;
    int device = 0;
    uint32_t lean_ws = 0;            // lean_kernel window stride for this file's record lengths
    uint64_t long_cols = ~0ull;      // columns with sampled fields over 8 bytes (cq_lean_long_cols)
    uint64_t wide4_cols = ~0ull;     // columns with sampled fields over 4 bytes (fast_kernel's numerals)
    std::string sample;              // the first data bytes (plan-time sampling: fast_kernel's key seed)
    std::map<int, std::unique_ptr<DevBuf>> fast_seed;   // per GROUP BY column: seeded LDS tags (device)
    // per join-key column: its canonical INTEGER keys' [min, max], learned by a STAR
    // join's build pass (the table is immutable) -- the next build sizes its arrays by it
    std::map<int, std::pair<uint64_t, uint64_t>> key_range;
    // routed tables (cqgpu_table_set_key_stride): the canonical INTEGER join keys were
    // routed by key mod key_stride, so this rank's keys are one residue class -- a
    // STAR join indexes them by (key - kmin) / key_stride
    uint32_t key_stride = 1;
    unsigned long long* gids = nullptr;   // routed tables: global record id of each record (device)
    uint64_t ngids = 0;
    uint64_t gid_total = 0;               // routed tables: records of the whole input (every rank's share)
    std::unique_ptr<RouteState> route;    // pending repartition (cqgpu_route_plan)
    // a routed side's replication (cqgpu_table_set_replicated): rep_major 1-3: every
    // non-NULL key of another value class went to every rank; bcast: every record of
    // this side is on every rank (a JOIN without ON); rep_owner: this rank keeps what
    // every rank finds (pairs of two replicated records, a cross join's unmatched rows)
    uint32_t rep_major = 0;
    bool bcast = false;
    bool rep_owner = true;
    std::unique_ptr<DevBuf> rec_starts;   // record start offsets, file order (built on first need; immutable table)
    uint32_t nrec_starts = 0;
    // the typed join exchange (cqgpu_typed_*): this table's counts and pending entries
    std::unique_ptr<TypedSend> tsend;
    uint64_t est_records = 0;        // the sample's record count scaled to the table (0: not yet)
};

namespace {

// parse_line's field split for the header record (reference csv_reader.c:278-357)
std::vector<std::string> split_header(const char* p, const char* end, char delim, char quote,
                                      bool has_header) {
    std::vector<std::pair<const char*, size_t>> fs;
    while (p < end) {
        while (p < end && is_space((unsigned char)*p) && *p != '\n' && *p != '\r') p++;
        if (p >= end) break;
        const char* s = p;
        size_t len = 0;
        if (*p == quote) {
            p++;
            s = p;
            bool closed = false;
            while (p < end) {
                if (*p == quote) {
                    if (p + 1 < end && p[1] == quote) { p += 2; len += 2; }
                    else { len = (size_t)(p - s); p++; closed = true; break; }
                } else p++;
            }
            (void)closed;
            while (p < end && *p != delim && *p != '\n' && *p != '\r') p++;
        } else {
            while (p < end && *p != delim && *p != '\n' && *p != '\r') p++;
            len = (size_t)(p - s);
        }
        fs.emplace_back(s, len);
        if (p < end && *p == delim) p++;
    }
    std::vector<std::string> names;
    for (size_t i = 0; i < fs.size(); i++) {
        if (has_header && fs[i].second > 0) {
            // cq_strndup stops at NUL, then trim_whitespace
            std::string nm(fs[i].first, strnlen(fs[i].first, fs[i].second));
            size_t a = 0;
            while (a < nm.size() && is_space((unsigned char)nm[a])) a++;
            size_t b = nm.size();
            while (b > a && is_space((unsigned char)nm[b - 1])) b--;
            names.push_back(nm.substr(a, b - a));
        } else {
            names.push_back("$" + std::to_string(i));
        }
    }
    return names;
}

// `fd` >= 0: the bytes are the file's [fd_off, fd_off + n) and the bulk copy reads them
// with pread() straight into the pinned chunks (`host`, the file's mapping, then only
// serves the header and the 256 KiB plan sample): on the bench host that ingests at
// 44-49 GB/s against 19-22 GB/s for memcpy out of the mapping, whose page faults the
// copy threads otherwise take (scripts/micro/ingest.cpp, gpurun_out/r6a/ingest.txt)
cqgpu_table* upload(const uint8_t* host, size_t n, cq_csv_config cfg, uint64_t base_offset,
                    const char* header, size_t header_len, int fd = -1, uint64_t fd_off = 0) {
    DevCtx& c = ctx();
    cqgpu_table* t = new cqgpu_table;
    t->cfg = cfg;
    t->n = n;
    t->base_offset = base_offset;
    HIPCHECK(hipGetDevice(&t->device));
    // names and the first data byte (csv_load: first non-empty record is the header)
    if (header) {
        const char* e = header + header_len;
        const char* p = header;
        while (p < e && (*p == '\n' || *p == '\r')) p++;
        const char* ls = p;
        while (p < e && *p != '\n' && *p != '\r') p++;
        t->names = split_header(ls, p, cfg.delimiter, cfg.quote, cfg.has_header);
        t->header_rec.assign(ls, (size_t)(p - ls));
        t->data_begin = 0;
    } else {
        const char* d = (const char*)host;
        const char* e = d + n;
        const char* p = d;
        while (p < e && (*p == '\n' || *p == '\r')) p++;
        const char* ls = p;
        while (p < e && *p != '\n' && *p != '\r') p++;
        if (p > ls) t->names = split_header(ls, p, cfg.delimiter, cfg.quote, cfg.has_header);
        if (cfg.has_header) t->header_rec.assign(ls, (size_t)(p - ls));
        t->data_begin = cfg.has_header ? (uint64_t)(p - d) : 0;
    }
    t->lean_ws = cq_lean_pick_ws(host + t->data_begin, n - std::min<uint64_t>(n, t->data_begin));
    t->long_cols = cq_lean_long_cols(host + t->data_begin, n - std::min<uint64_t>(n, t->data_begin),
                                     (uint8_t)cfg.delimiter);
    t->wide4_cols = cq_cols_longer_than(host + t->data_begin, n - std::min<uint64_t>(n, t->data_begin),
                                        (uint8_t)cfg.delimiter, 4);
    {
        const uint64_t db = std::min<uint64_t>(n, t->data_begin);
        t->sample.assign((const char*)host + db, (size_t)std::min<uint64_t>(n - db, SAMPLE_BYTES));
    }
    size_t total = PAD_BEFORE + n + PAD_AFTER;
    HIPCHECK(hipMalloc(&t->dbuf, total));
    note_table_bytes(t->dbuf, total);
    HIPCHECK(hipMemsetAsync(t->dbuf, '\n', PAD_BEFORE, c.stream));
    HIPCHECK(hipMemsetAsync(t->dbuf + PAD_BEFORE + n, '\n', PAD_AFTER, c.stream));
    // stream the bytes through a ring of S pinned slots: P host threads claim chunks in
    // order and fill them (pread from the file, or memcpy out of the mapping) -- one
    // thread's copy runs at ~10 GB/s, far below the host-to-device link -- while this
    // thread issues each filled chunk's DMA in order and records its slot's event; a
    // thread reuses a slot once the DMA of the chunk before it in that slot is done.
    // Continuous: the link never waits for a whole group, only the first chunk's fill
    // and the last chunk's DMA are exposed (CQGPU_UPLOAD_THREADS, CQGPU_UPLOAD_CHUNK_MB)
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const char* up_env = getenv("CQGPU_UPLOAD_THREADS");
    const char* ch_env = getenv("CQGPU_UPLOAD_CHUNK_MB");
    const size_t P = up_env ? (size_t)std::min(std::max(atoi(up_env), 1), 64)
                            : std::min<size_t>(8, std::max(1u, hw / 2));
    const size_t CH = (ch_env ? (size_t)std::min(std::max(atoi(ch_env), 1), 256) : 32) << 20;
    const size_t nch = (n + CH - 1) / CH;
    const size_t S = std::max<size_t>(2 * P, 4);
    const size_t slot = std::min(CH, std::max<size_t>(n, 1));
    uint8_t* st = (uint8_t*)pinned(c, S * slot);
    std::vector<hipEvent_t> ev(S, nullptr);
    for (auto& e : ev) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    struct EvFree {
        std::vector<hipEvent_t>& v;
        ~EvFree() { for (auto e : v) if (e) (void)hipEventDestroy(e); }
    } ev_free_{ev};
    std::atomic<size_t> next{0}, issued{0};
    std::atomic<int> rerr{0};
    std::unique_ptr<std::atomic<uint8_t>[]> filled(new std::atomic<uint8_t>[nch ? nch : 1]);
    for (size_t k = 0; k < nch; k++) filled[k].store(0, std::memory_order_relaxed);
    auto worker = [&]() {
        for (;;) {
            const size_t k = next.fetch_add(1);
            if (k >= nch || rerr.load()) return;
            if (k >= S) {                      // the slot's previous chunk: issued, then copied
                while (issued.load(std::memory_order_acquire) <= k - S) {
                    if (rerr.load()) return;
                    std::this_thread::yield();
                }
                if (hipEventSynchronize(ev[k % S]) != hipSuccess) { rerr.store(EIO); return; }
            }
            uint8_t* dst = st + (k % S) * slot;
            const size_t off = k * CH, len = std::min(CH, n - off);
            if (fd < 0) {
                memcpy(dst, host + off, len);
            } else {
                size_t got = 0;
                while (got < len) {
                    const ssize_t r = pread(fd, dst + got, len - got, (off_t)(fd_off + off + got));
                    if (r < 0 && errno == EINTR) continue;
                    if (r <= 0) { rerr.store(r < 0 ? errno : EIO); return; }
                    got += (size_t)r;
                }
            }
            filled[k].store(1, std::memory_order_release);
        }
    };
    std::vector<std::thread> th;
    for (size_t k = 0; k < std::min(P, nch); k++) th.emplace_back(worker);
    hipError_t herr = hipSuccess;
    for (size_t k = 0; k < nch && herr == hipSuccess; k++) {
        while (!filled[k].load(std::memory_order_acquire) && !rerr.load()) std::this_thread::yield();
        if (rerr.load()) break;
        const size_t off = k * CH;
        herr = hipMemcpyAsync(t->dbuf + PAD_BEFORE + off, st + (k % S) * slot, std::min(CH, n - off),
                              hipMemcpyHostToDevice, c.stream);
        if (herr == hipSuccess) herr = hipEventRecord(ev[k % S], c.stream);
        issued.store(k + 1, std::memory_order_release);
    }
    if (herr != hipSuccess && !rerr.load()) rerr.store(EIO);
    for (auto& x : th) x.join();
    if (rerr.load()) {
        (void)hipStreamSynchronize(c.stream);
        forget_table_bytes(t->dbuf);
        (void)hipFree(t->dbuf);
        delete t;
        throw HipError{herr != hipSuccess ? std::string("upload: ") + hipGetErrorString(herr)
                                          : std::string("upload: pread: ") + strerror(rerr.load())};
    }
    HIPCHECK(hipStreamSynchronize(c.stream));
    t->g = t->dbuf + PAD_BEFORE;
    return t;
}

int col_index(const cqgpu_table* t, const char* name) {      // csv_get_column_index
    if (!name) return -1;
    for (size_t i = 0; i < t->names.size(); i++)
        if (strcasecmp(t->names[i].c_str(), name) == 0) return (int)i;
    return -1;
}
int col_index_fallback(const cqgpu_table* t, const char* name) {   // find_column_index_with_fallback
    int c = col_index(t, name);
    if (c < 0 && name) {
        const char* dot = strchr(name, '.');
        if (dot) c = col_index(t, dot + 1);
    }
    return c;
}

// ------------------------------------------------------------------ host cells
struct HCell {
    uint32_t kind = K_NULL;
    uint64_t bits = 0;
    std::string s;
};

int hcompare(const HCell& a, const HCell& b) {     // value_compare over host cells
    if (a.kind == K_NULL && b.kind == K_NULL) return 0;
    if (a.kind == K_NULL) return -1;
    if (b.kind == K_NULL) return 1;
    if (a.kind == K_DATE && b.kind == K_DATE) {
        int ay = (int)(a.bits >> 32), by = (int)(b.bits >> 32);
        if (ay != by) return ay - by;
        int am = (int)((a.bits >> 16) & 0xffff), bm = (int)((b.bits >> 16) & 0xffff);
        if (am != bm) return am - bm;
        return (int)(a.bits & 0xffff) - (int)(b.bits & 0xffff);
    }
    auto num = [](const HCell& c) { return c.kind == K_INT ? (double)(int64_t)c.bits : as_dbl(c.bits); };
    bool an = a.kind == K_INT || a.kind == K_DBL, bn = b.kind == K_INT || b.kind == K_DBL;
    if (an && bn) {
        double x = num(a), y = num(b);
        return x < y ? -1 : (x > y ? 1 : 0);
    }
    if (a.kind == K_STR && b.kind == K_STR) return strcmp(a.s.c_str(), b.s.c_str());
    return 0;
}

cq_value to_value(const HCell& h) {
    cq_value v;
    memset(&v, 0, sizeof v);
    v.kind = (int)h.kind;
    switch (h.kind) {
        case K_INT: v.u.i = (long long)h.bits; break;
        case K_DBL: v.u.f = as_dbl(h.bits); break;
        case K_DATE:
            v.u.date.y = (int)(h.bits >> 32);
            v.u.date.m = (int)((h.bits >> 16) & 0xffff);
            v.u.date.d = (int)(h.bits & 0xffff);
            break;
        case K_STR: v.u.s = strdup(h.s.c_str()); break;
        default: v.kind = CQ_V_NULL; break;
    }
    return v;
}

HCell from_value(const cq_value& v) {              // to_value's inverse (result rows -> blob cells)
    HCell h;
    h.kind = (uint32_t)v.kind;
    switch (v.kind) {
        case K_INT: h.bits = (uint64_t)v.u.i; break;
        case K_DBL: h.bits = dbl_bits(v.u.f); break;
        case K_DATE: h.bits = ((uint64_t)(uint32_t)v.u.date.y << 32) | ((uint64_t)(v.u.date.m & 0xffff) << 16) |
                              (uint64_t)(v.u.date.d & 0xffff); break;
        case K_STR: h.s = v.u.s ? v.u.s : ""; break;
        default: h.kind = K_NULL; break;
    }
    return h;
}

// device cells -> host cells (strings copied back with one kernel); `table_cells`:
// every STRING must lie in a live table's bytes
std::vector<HCell> fetch_cells(DevCtx& c, const std::vector<Cell>& cells, bool table_cells = false) {
    std::vector<HCell> out(cells.size());
    std::vector<unsigned long long> offs(cells.size(), 0);
    unsigned long long total = 0;
    for (size_t i = 0; i < cells.size(); i++) {
        out[i].kind = cells[i].kind;
        out[i].bits = cells[i].bits;
        offs[i] = total;
        if (cells[i].kind == K_STR) total += cells[i].len;
        if (table_cells && cells[i].kind == K_STR && cells[i].len && !in_some_table(cells[i].bits, cells[i].len)) {
            char b[160];
            snprintf(b, sizeof b, "internal: a group's STRING cell %zu of %zu (address 0x%llx, %u bytes) is outside every table",
                     i, cells.size(), (unsigned long long)cells[i].bits, cells[i].len);
            throw HipError{b};
        }
    }
    if (total == 0 && std::none_of(cells.begin(), cells.end(), [](const Cell& x) { return x.kind == K_STR; }))
        return out;
    size_t n = cells.size();
    size_t need = n * sizeof(Cell) + n * 8 + total + 16;
    Scratch sc(c, need);
    uint8_t* d = sc.p;
    Cell* dc = (Cell*)d;
    unsigned long long* doffs = (unsigned long long*)(d + n * sizeof(Cell));
    uint8_t* dout = d + n * sizeof(Cell) + n * 8;
    HIPCHECK(hipMemcpyAsync(dc, cells.data(), n * sizeof(Cell), hipMemcpyHostToDevice, c.stream));
    HIPCHECK(hipMemcpyAsync(doffs, offs.data(), n * 8, hipMemcpyHostToDevice, c.stream));
    HIPCHECK(cq_launch_copy_strings(dc, (uint32_t)n, doffs, dout, c.stream));
    std::vector<char> hb(total + 1, 0);
    if (total) HIPCHECK(hipMemcpyAsync(hb.data(), dout, total, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    for (size_t i = 0; i < n; i++)
        if (cells[i].kind == K_STR) out[i].s.assign(hb.data() + offs[i], cells[i].len);
    return out;
}

// ------------------------------------------------------------------ compiled plan
enum OutKind { OUT_COUNT, OUT_SUM, OUT_AVG, OUT_EXT, OUT_REP, OUT_CONST, OUT_NULL, OUT_VLA, OUT_HEXPR };
struct OutCol {
    OutKind kind = OUT_NULL;
    int acc = -1;          // accumulator index for SUM/AVG/EXT
    int rep = -1;          // rep slot
    int lit = -1;          // literal index (OUT_CONST)
};

struct Compiled {
    ScanPlan P;
    bool grouped = false;            // GROUP BY present
    bool group_missing = false;      // GROUP BY column not found: zero groups
    std::vector<int> need_cols;      // csv column per need slot
    std::vector<std::string> lits;   // literal texts (const index)
    std::vector<OutCol> outs;
    std::vector<std::string> names;
    std::vector<int> rep_cols;       // csv column per rep slot
    int max_depth = 0;
    int group_col = -1;              // csv column of the GROUP BY key
    std::vector<std::pair<int, int>> vla;   // STDDEV (0) / MEDIAN (1) and their csv column
    int where_len = -1;              // WHERE program length when group expressions follow it
    // expression items evaluated on the host over each group's first-row cells:
    // OP_COL b = rep slot, OP_CONST b = literal index (C.lits)
    std::vector<std::vector<Insn>> hexpr;
    // more than MAX_NEED distinct columns: the fused scans (registers per need slot)
    // cannot take the plan; it runs on the cells path (parsed cell tables + PairView)
    bool wide = false;
};

struct Compiler {
    const cqgpu_table* t;
    cq_node* q;
    const char* alias;               // FROM alias ("main" default)
    Compiled& C;
    std::vector<Insn> code;
    int depth = 0, bdepth = 0;
    int need_cap = MAX_WIDE;         // distinct columns one plan may reference (> MAX_NEED: the cells path)
    int lit_cap = MAX_CONST;

    int need(int col) {
        auto it = std::find(C.need_cols.begin(), C.need_cols.end(), col);
        if (it != C.need_cols.end()) return (int)(it - C.need_cols.begin());
        if ((int)C.need_cols.size() >= need_cap)
            throw Ineligible{"more than " + std::to_string(need_cap) + " referenced columns"};
        C.need_cols.push_back(col);
        return (int)C.need_cols.size() - 1;
    }
    int lit(const char* text) {
        C.lits.push_back(text ? text : "");
        if ((int)C.lits.size() > lit_cap) throw Ineligible{"too many literals"};
        return (int)C.lits.size() - 1;
    }
    void emit(uint8_t op, int a = 0, int b = 0) {
        if ((int)code.size() >= MAX_PROG) throw Ineligible{"WHERE clause too long"};
        Insn in;
        in.op = op;
        in.a = (uint8_t)a;
        in.b = (uint16_t)b;
        code.push_back(in);
    }
    void push(int n = 1) {
        depth += n;
        C.max_depth = std::max(C.max_depth, depth);
        if (depth > VM_STACK) throw Ineligible{"expression too deep"};
    }
    void bpush() {
        if (++bdepth > 30) throw Ineligible{"condition too deep"};
    }

    // resolve_column for WHERE (reference evaluator_core.c:70-167, one table)
    // returns csv column, or -2 when the name is a SELECT alias handled by caller
    int resolve(const char* name, cq_node** alias_expr) {
        *alias_expr = nullptr;
        if (!name) return -1;
        const char* dot = strchr(name, '.');
        if (dot) {
            int c = col_index(t, name);
            if (c >= 0) return c;
            std::string al(name, (size_t)(dot - name));
            if (strcasecmp(al.c_str(), alias) != 0) return -1;
            return col_index(t, dot + 1);
        }
        int c = col_index(t, name);
        if (c >= 0) return c;
        cq_node* sel = q->u.q.select;
        if (sel && sel->kind == CQ_N_SELECT && sel->u.sel.exprs) {
            for (int i = 0; i < sel->u.sel.count; i++) {
                const char* cs = sel->u.sel.texts[i];
                if (!cs) continue;
                const char* as = ci_find(cs, " AS ");
                if (!as) continue;
                const char* a = as + 4;
                while (*a && is_space((unsigned char)*a)) a++;
                if (strcasecmp(a, name) == 0) { *alias_expr = sel->u.sel.exprs[i]; return -2; }
            }
        }
        return -1;
    }

    // evaluate_expression (evaluator_expressions.c:23-263)
    void expr(cq_node* e, int nest = 0) {
        if (nest > 16) throw Ineligible{"recursive SELECT alias"};
        if (!e) { emit(OP_NULLV); push(); return; }
        switch (e->kind) {
            case CQ_N_LITERAL: emit(OP_CONST, 0, lit(e->u.text)); push(); return;
            case CQ_N_IDENTIFIER: {
                cq_node* ae;
                int c = resolve(e->u.text, &ae);
                if (c >= 0) { need(c); emit(OP_COL, 0, c); push(); }
                else if (c == -2) expr(ae, nest + 1);
                else { emit(OP_NULLV); push(); }
                return;
            }
            case CQ_N_BINARY_OP: {
                const char* op = e->u.bin.op ? e->u.bin.op : "";
                if (!e->u.bin.lhs || !e->u.bin.rhs) {
                    cq_node* only = e->u.bin.lhs ? e->u.bin.lhs : e->u.bin.rhs;
                    if (!only) { emit(OP_NULLV); push(); return; }
                    if (!strcmp(op, "-")) { expr(only, nest); emit(OP_NEG); return; }
                    if (!strcmp(op, "+")) { expr(only, nest); return; }
                    emit(OP_NULLV); push();
                    return;
                }
                int ar;
                if (!strcmp(op, "+")) ar = AR_ADD;
                else if (!strcmp(op, "-")) ar = AR_SUB;
                else if (!strcmp(op, "*")) ar = AR_MUL;
                else if (!strcmp(op, "/")) ar = AR_DIV;
                else if (!strcmp(op, "%")) ar = AR_MOD;
                else if (!strcmp(op, "&")) ar = AR_AND;
                else if (!strcmp(op, "|")) ar = AR_OR;
                else if (!strcmp(op, "^")) ar = AR_XOR;
                else throw Ineligible{std::string("arithmetic operator ") + op};
                expr(e->u.bin.lhs, nest);
                expr(e->u.bin.rhs, nest);
                emit(OP_ARITH, ar);
                depth--;
                return;
            }
            default:
                throw Ineligible{"expression kind " + std::to_string(e->kind) +
                                 " (function/CASE/subquery)"};
        }
    }

    // evaluate_condition (evaluator_conditions.c:62-164)
    void cond(cq_node* n) {
        if (!n) { emit(OP_BOOL, 1); bpush(); return; }
        if (n->kind != CQ_N_CONDITION) { emit(OP_BOOL, 0); bpush(); return; }
        const char* op = n->u.bin.op ? n->u.bin.op : "";
        if (!strcasecmp(op, "NOT")) { cond(n->u.bin.lhs); emit(OP_NOT); return; }
        if (!strcasecmp(op, "AND") || !strcasecmp(op, "OR")) {
            cond(n->u.bin.lhs);
            cond(n->u.bin.rhs);
            emit(!strcasecmp(op, "AND") ? OP_AND : OP_OR);
            bdepth--;
            return;
        }
        int cmp = -1;
        if (!strcmp(op, "=")) cmp = CMP_EQ;
        else if (!strcmp(op, "!=") || !strcmp(op, "<>")) cmp = CMP_NE;
        else if (!strcmp(op, ">")) cmp = CMP_GT;
        else if (!strcmp(op, "<")) cmp = CMP_LT;
        else if (!strcmp(op, ">=")) cmp = CMP_GE;
        else if (!strcmp(op, "<=")) cmp = CMP_LE;
        if (cmp >= 0) {
            expr(n->u.bin.lhs);
            expr(n->u.bin.rhs);
            emit(OP_CMP, cmp);
            depth -= 2;
            bpush();
            return;
        }
        if (!strcasecmp(op, "IN") || !strcasecmp(op, "NOT IN")) {
            bool neg = !strcasecmp(op, "NOT IN");
            cq_node* r = n->u.bin.rhs;
            if (r && r->kind == CQ_N_SUBQUERY) throw Ineligible{"IN subquery"};
            if (r && r->kind == CQ_N_LIST) {
                expr(n->u.bin.lhs);
                int items = r->u.list.nitems;
                for (int i = 0; i < items; i++) expr(r->u.list.items[i]);
                emit(OP_IN, neg ? 1 : 0, items);
                depth -= items + 1;
                bpush();
                return;
            }
            emit(OP_BOOL, neg ? 1 : 0);
            bpush();
            return;
        }
        if (!strcasecmp(op, "LIKE") || !strcasecmp(op, "ILIKE")) {
            expr(n->u.bin.lhs);
            expr(n->u.bin.rhs);
            emit(OP_LIKE, !strcasecmp(op, "LIKE") ? 1 : 0);
            depth -= 2;
            bpush();
            return;
        }
        emit(OP_BOOL, 0);
        bpush();
    }
};

bool is_agg_name(const std::string& f) {          // is_aggregate_function
    const char* s = f.c_str();
    return !strcasecmp(s, "COUNT") || !strcasecmp(s, "SUM") || !strcasecmp(s, "AVG") ||
           !strcasecmp(s, "MIN") || !strcasecmp(s, "MAX") || !strcasecmp(s, "STDDEV") ||
           !strcasecmp(s, "STDDEV_POP") || !strcasecmp(s, "MEDIAN");
}

bool has_aggregates(cq_node* sel) {               // has_aggregate_functions (:55-106)
    if (!sel || sel->kind != CQ_N_SELECT) return false;
    if (sel->u.sel.exprs) {
        for (int i = 0; i < sel->u.sel.count; i++) {
            cq_node* n = sel->u.sel.exprs[i];
            if (!n || n->kind != CQ_N_FUNCTION || !n->u.fn.name) continue;
            const char* f = n->u.fn.name;
            if (!strcasecmp(f, "COUNT") || !strcasecmp(f, "SUM") || !strcasecmp(f, "AVG") ||
                !strcasecmp(f, "MIN") || !strcasecmp(f, "MAX") || !strcasecmp(f, "STDDEV") ||
                !strcasecmp(f, "MEDIAN"))
                return true;
        }
        return false;
    }
    for (int i = 0; i < sel->u.sel.count; i++) {
        const char* cs = sel->u.sel.texts[i];
        if ((strstr(cs, "COUNT(") || strstr(cs, "SUM(") || strstr(cs, "AVG(") || strstr(cs, "MIN(") ||
             strstr(cs, "MAX(") || strstr(cs, "STDDEV(") || strstr(cs, "MEDIAN(")) &&
            !ci_find(cs, "OVER"))
            return true;
    }
    return false;
}

// result column names of build_aggregated_result (evaluator_aggregates.c:546-593)
std::string agg_display_name(const char* cs) {
    const char* as = ci_find(cs, " AS ");
    if (as) return std::string(as + 4);
    const char* par = strchr(cs, '(');
    if (par) {
        std::string fn(cs, (size_t)(par - cs));
        const char* pc = strchr(par, ')');
        std::string arg = pc ? std::string(par + 1, (size_t)(pc - par - 1)) : std::string(par + 1);
        if (arg.size() > 127) arg.resize(127);
        size_t dot = arg.find('.');
        std::string an = dot == std::string::npos ? arg : arg.substr(dot + 1);
        std::string r = fn + "(" + an + ")";
        if (r.size() > 255) r.resize(255);
        return r;
    }
    const char* dot = strchr(cs, '.');
    return std::string(dot ? dot + 1 : cs);
}

// order the need slots by column so one left-to-right pass parses them all,
// and fill the table-dependent plan fields

// fast_kernel's LDS table seed for GROUP BY column `col` of table t: the distinct
// keys of the table's sample placed by cq_fast_seed (fast.hip), built on first use
// and kept with the table (const: a cache, not table state)
const void* fast_seed_of(const cqgpu_table* tc, int col) {
    cqgpu_table* t = const_cast<cqgpu_table*>(tc);
    auto it = t->fast_seed.find(col);
    if (it != t->fast_seed.end()) return it->second->p;
    if (t->sample.empty()) return nullptr;
    std::vector<unsigned long long> tags(cq_fast_seed_slots());
    cq_fast_seed((const uint8_t*)t->sample.data(), t->sample.size(), (uint8_t)t->cfg.delimiter, (uint8_t)t->cfg.quote,
                 (uint32_t)col, tags.data());
    std::unique_ptr<DevBuf> b(new DevBuf(tags.size() * 8));
    DevCtx& c = ctx();
    HIPCHECK(hipMemcpyAsync(b->p, tags.data(), tags.size() * 8, hipMemcpyHostToDevice, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    const void* r = b->p;
    t->fast_seed[col] = std::move(b);
    return r;
}

void finish_plan(const cqgpu_table* t, Compiled& C, Compiler& cc) {
    std::vector<int> order(C.need_cols.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = (int)i;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return C.need_cols[a] < C.need_cols[b]; });
    std::vector<int> remap(order.size());
    for (size_t i = 0; i < order.size(); i++) remap[order[i]] = (int)i;
    std::vector<int> sorted(order.size());
    for (size_t i = 0; i < order.size(); i++) sorted[remap[i]] = C.need_cols[i];
    C.P.nneed = (int)sorted.size();
    C.wide = C.P.nneed > MAX_NEED;
    if (C.wide) g_stats.wide = 1;
    for (int i = 0; i < C.P.nneed && i < MAX_NEED; i++) C.P.need_col[i] = (int16_t)sorted[i];
    C.P.max_col = C.P.nneed ? sorted.back() : -1;
    for (auto& in : cc.code) {
        if (in.op == OP_COL) {
            auto it = std::find(C.need_cols.begin(), C.need_cols.end(), (int)in.b);
            in.a = (uint8_t)remap[it - C.need_cols.begin()];
        }
    }
    for (int a = 0; a < C.P.nacc; a++) C.P.acc[a].slot = (uint8_t)remap[C.P.acc[a].slot];
    if (C.P.group_slot >= 0) C.P.group_slot = remap[C.P.group_slot];
    for (int g = 0; g < C.P.ngpart; g++)
        if (C.P.gpart_slot[g] >= 0) C.P.gpart_slot[g] = (int16_t)remap[C.P.gpart_slot[g]];
    C.need_cols = sorted;
    C.P.nprog = C.where_len >= 0 ? C.where_len : (int)cc.code.size();
    std::copy(cc.code.begin(), cc.code.end(), C.P.prog);
    C.P.nconst = (int)C.lits.size();
    C.P.delim = (uint8_t)t->cfg.delimiter;
    C.P.quote = (uint8_t)t->cfg.quote;
    C.P.n = t->n;
    C.P.data_begin = t->data_begin;
    C.P.range_begin = 0;
    C.P.range_end = t->n;
    C.P.lean_ws = t->lean_ws;
    C.P.fast_wide_cols = t->wide4_cols;
    C.P.fast_seed = 0;
    if (C.P.group_slot >= 0 && !C.wide) {
        const int gc = C.P.need_col[C.P.group_slot];
        C.P.lean_k16 = (uint32_t)((t->long_cols >> (gc < 63 ? gc : 63)) & 1);
        if (!C.P.lean_k16) C.P.fast_seed = (uint64_t)(uintptr_t)fast_seed_of(t, gc);
    }
}

// compile the aggregate SELECT (evaluator.c:69-258 + build_aggregated_result)
void compile_aggregate(const cqgpu_table* t, cq_node* q, Compiled& C) {
    memset(&C.P, 0, sizeof C.P);
    const char* alias = (q->u.q.from && q->u.q.from->u.from.alias) ? q->u.q.from->u.from.alias : "main";
    Compiler cc{t, q, alias, C};
    if (q->u.q.where) {
        cc.cond(q->u.q.where);
    }
    C.where_len = (int)cc.code.size();
    cq_node* gb = q->u.q.group_by;
    C.grouped = gb && gb->kind == CQ_N_GROUP_BY && gb->u.grp.keys && gb->u.grp.nkeys > 0;
    C.P.group_slot = -1;
    C.P.ngpart = 0;
    if (C.grouped) {
        // a GROUP BY name matching a SELECT alias groups by that item's expression
        // (evaluator.c:71-98)
        const int nk = gb->u.grp.nkeys;
        if (nk > MAX_GPART) throw Ineligible{"GROUP BY of more than " + std::to_string(MAX_GPART) + " parts"};
        std::vector<cq_node*> gexpr(nk, nullptr);
        cq_node* sel = q->u.q.select;
        for (int g = 0; g < nk; g++) {
            const char* key = gb->u.grp.keys[g];
            if (!key || !sel || sel->kind != CQ_N_SELECT || !sel->u.sel.exprs) continue;
            for (int i = 0; i < sel->u.sel.count; i++) {
                const char* cs = sel->u.sel.texts[i];
                if (!cs) continue;
                const char* as = ci_find(cs, " AS ");
                if (!as) continue;
                const char* a = as + 4;
                while (*a && is_space((unsigned char)*a)) a++;
                if (!strcasecmp(a, key)) { gexpr[g] = sel->u.sel.exprs[i]; break; }
            }
        }
        if (nk == 1 && !gexpr[0]) {                     // create_groups (find_column_index_with_fallback)
            int gc = col_index_fallback(t, gb->u.grp.keys[0]);
            C.group_col = gc;
            if (gc < 0) C.group_missing = true;
            else C.P.group_slot = cc.need(gc);
        } else {
            // create_groups_by_expression, or the composite key: expressions by the
            // WHERE VM (code after the WHERE program), columns by csv_get_column_index
            // -- no table-prefix fallback on this path (evaluator.c:152), a missing
            // column is the part "NULL"
            C.P.ngpart = nk;
            if (const char* e = getenv("CQGPU_TEST_DIGEST_BITS")) C.P.test_digest_bits = (uint32_t)std::min(atoi(e), 63);
            for (int g = 0; g < nk; g++) {
                C.P.gcode_off[g] = (uint16_t)cc.code.size();
                if (gexpr[g]) {
                    const int d0 = cc.depth;
                    cc.expr(gexpr[g]);
                    cc.depth = d0;
                    C.P.gpart_slot[g] = -1;
                } else {
                    const int col = col_index(t, gb->u.grp.keys[g]);
                    C.P.gpart_slot[g] = (int16_t)(col >= 0 ? cc.need(col) : -2);
                }
            }
            C.P.gcode_off[nk] = (uint16_t)cc.code.size();
        }
    }
    cq_node* sel = q->u.q.select;
    int nsel = sel ? sel->u.sel.count : 0;
    if (nsel > MAX_ACC) throw Ineligible{"more than 8 SELECT items"};
    for (int i = 0; i < nsel; i++) {
        const char* cs = sel->u.sel.texts[i];
        C.names.push_back(agg_display_name(cs));
        std::string cn;
        const char* as = ci_find(cs, " AS ");
        cn = as ? std::string(cs, (size_t)(as - cs)) : std::string(cs);
        cn = rtrim(cn);
        OutCol oc;
        size_t par = cn.find('(');
        if (par != std::string::npos) {
            std::string fn = cn.substr(0, par);
            if (!is_agg_name(fn)) throw Ineligible{"scalar function in an aggregate SELECT"};
            size_t pc = cn.find(')', par + 1);
            std::string arg = pc != std::string::npos ? cn.substr(par + 1, pc - par - 1) : cn;
            const char* f = fn.c_str();
            const bool is_vla = !strcasecmp(f, "STDDEV") || !strcasecmp(f, "STDDEV_POP") || !strcasecmp(f, "MEDIAN");
            if (!strcasecmp(f, "COUNT") && arg == "*") { oc.kind = OUT_COUNT; C.outs.push_back(oc); continue; }
            int col = col_index_fallback(t, arg.c_str());
            if (col < 0) { oc.kind = OUT_NULL; C.outs.push_back(oc); continue; }
            if (is_vla) {          // value-list aggregates: compute_vla after the scan
                const std::pair<int, int> v{!strcasecmp(f, "MEDIAN") ? 1 : 0, col};
                auto it = std::find(C.vla.begin(), C.vla.end(), v);
                oc.acc = (int)(it - C.vla.begin());
                if (it == C.vla.end()) {
                    if (C.vla.size() >= (size_t)MAX_ACC) throw Ineligible{"too many STDDEV/MEDIAN"};
                    C.vla.push_back(v);
                }
                oc.kind = OUT_VLA;
                C.outs.push_back(oc);
                continue;
            }
            if (!strcasecmp(f, "COUNT")) { oc.kind = OUT_COUNT; C.outs.push_back(oc); continue; }
            uint8_t kind = (!strcasecmp(f, "SUM") || !strcasecmp(f, "AVG")) ? ACC_SUM
                         : (!strcasecmp(f, "MIN") ? ACC_MIN : ACC_MAX);
            int slot = cc.need(col);
            int acc = -1;
            for (int a = 0; a < C.P.nacc; a++)
                if (C.P.acc[a].kind == kind && C.P.acc[a].slot == slot) acc = a;
            if (acc < 0) {
                if (C.P.nacc >= MAX_ACC) throw Ineligible{"too many aggregates"};
                acc = C.P.nacc++;
                C.P.acc[acc].kind = kind;
                C.P.acc[acc].slot = (uint8_t)slot;
            }
            oc.acc = acc;
            oc.kind = kind == ACC_SUM ? (!strcasecmp(f, "SUM") ? OUT_SUM : OUT_AVG) : OUT_EXT;
            C.outs.push_back(oc);
            continue;
        }
        cq_node* node = sel->u.sel.exprs ? sel->u.sel.exprs[i] : nullptr;
        if (node && node->kind != CQ_N_IDENTIFIER) {
            if (node->kind == CQ_N_LITERAL) { oc.kind = OUT_CONST; oc.lit = cc.lit(node->u.text); C.outs.push_back(oc); continue; }
            // an expression on the group's first row (evaluator_aggregates.c:669-677):
            // compiled by a scratch compiler, its columns become representative cells
            Compiled T;
            Compiler tc{t, q, alias, T};
            tc.lit_cap = MAX_CONST - (int)C.lits.size();
            tc.need_cap = MAX_WIDE;
            tc.expr(node);
            std::vector<Insn> code = tc.code;
            for (auto& in : code) {
                if (in.op == OP_COL) {
                    const int col = in.b;
                    auto it = std::find(C.rep_cols.begin(), C.rep_cols.end(), col);
                    if (it == C.rep_cols.end()) { C.rep_cols.push_back(col); in.b = (uint16_t)(C.rep_cols.size() - 1); }
                    else in.b = (uint16_t)(it - C.rep_cols.begin());
                } else if (in.op == OP_CONST) {
                    in.b = (uint16_t)cc.lit(T.lits[in.b].c_str());
                }
            }
            oc.kind = OUT_HEXPR;
            oc.acc = (int)C.hexpr.size();
            C.hexpr.push_back(std::move(code));
            C.outs.push_back(oc);
            continue;
        }
        int col = col_index_fallback(t, cn.c_str());
        if (col < 0) { oc.kind = OUT_NULL; C.outs.push_back(oc); continue; }
        oc.kind = OUT_REP;
        auto it = std::find(C.rep_cols.begin(), C.rep_cols.end(), col);
        if (it == C.rep_cols.end()) { C.rep_cols.push_back(col); oc.rep = (int)C.rep_cols.size() - 1; }
        else oc.rep = (int)(it - C.rep_cols.begin());
        C.outs.push_back(oc);
    }
    finish_plan(t, C, cc);
}

// ------------------------------------------------------------------ host groups
// vla_prep_kernel's order-preserving value key back to the double (scan.hip vla_value)
inline double vkey_value(unsigned long long k) {
    const uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFULL) : ~k;
    double d;
    memcpy(&d, &b, 8);
    return d;
}

struct HGroup {
    uint32_t kcls = 0, klen = 0;        // cell.h GKey class and text length
    uint64_t kw0 = 0, kw1 = 0;          // key words (GK_LONG: w1 = content hash)
    std::string kbytes;                 // text-class key bytes
    unsigned long long cnt = 0, first = NOPOS;   // first: whole-file byte offset
    double sum[MAX_ACC] = {};
    unsigned long long num[MAX_ACC] = {};
    HCell ext[MAX_ACC];
    unsigned long long extpos[MAX_ACC] = {NOPOS, NOPOS, NOPOS, NOPOS, NOPOS, NOPOS, NOPOS, NOPOS};
    std::vector<HCell> reps;            // representative cells (first row)
    double vla[MAX_ACC] = {};           // STDDEV / MEDIAN results
    bool vla_ok[MAX_ACC] = {};          // false: no numeric value (NULL)
    // across partials, STDDEV's state: sum, squared deviations from the partial's
    // mean and the numeric count (merged exactly by the parallel-variance rule)
    double vsum[MAX_ACC] = {}, vm2[MAX_ACC] = {}, vn[MAX_ACC] = {};
    // across partials, MEDIAN's state: the group's numeric values as order-preserving
    // keys, ascending (mvals[v] for value-list aggregate v; empty for STDDEV)
    std::vector<std::vector<unsigned long long>> mvals;
    // MIN/MAX over several value classes: per class (0 number, 1 string, 2 date) the
    // extreme with its position and the class's first position, so range partials
    // can fold the whole file's row order (aggregate_pairs' class-split pass)
    struct ClassSplit {
        int acc = 0;
        HCell ext[3];
        unsigned long long extpos[3] = {NOPOS, NOPOS, NOPOS}, first[3] = {NOPOS, NOPOS, NOPOS};
    };
    std::vector<ClassSplit> split;
};

// little-endian byte writer / reader of the partial-aggregation blobs
struct Blob {
    std::vector<uint8_t> d;
    void raw(const void* p, size_t n) { const uint8_t* b = (const uint8_t*)p; d.insert(d.end(), b, b + n); }
    void u32(uint32_t v) { raw(&v, 4); }
    void u64(uint64_t v) { raw(&v, 8); }
    void f64(double v) { raw(&v, 8); }
    void str(const std::string& s) { u32((uint32_t)s.size()); raw(s.data(), s.size()); }
    void cell(const HCell& h) { u32(h.kind); u64(h.bits); str(h.s); }
    void split(const std::vector<HGroup::ClassSplit>& v) {
        u32((uint32_t)v.size());
        for (const HGroup::ClassSplit& cs : v) {
            u32((uint32_t)cs.acc);
            for (int k = 0; k < 3; k++) { cell(cs.ext[k]); u64(cs.extpos[k]); u64(cs.first[k]); }
        }
    }
    void mvals(const std::vector<unsigned long long>* v) {
        u64(v ? v->size() : 0);
        if (v && !v->empty()) raw(v->data(), v->size() * 8);
    }
};
struct Reader {
    const uint8_t* p;
    size_t n, o;
    void raw(void* dst, size_t k) {
        if (o + k > n) throw HipError{"truncated partial blob"};
        memcpy(dst, p + o, k);
        o += k;
    }
    uint32_t u32() { uint32_t v; raw(&v, 4); return v; }
    uint64_t u64() { uint64_t v; raw(&v, 8); return v; }
    double f64() { double v; raw(&v, 8); return v; }
    std::string str() {
        const uint32_t k = u32();
        if (o + k > n) throw HipError{"truncated partial blob"};
        std::string s((const char*)p + o, k);
        o += k;
        return s;
    }
    HCell cell() { HCell h; h.kind = u32(); h.bits = u64(); h.s = str(); return h; }
};

// literal cells parsed on the device with the same parser as the data
struct Literals {
    Scratch dev;
    Cell* dcells = nullptr;           // device copy of `cells`
    std::vector<Cell> cells;          // STRING bits: device addresses
    std::vector<HCell> host;          // the same cells with host strings
};

// A query's literals repeat from step to step: their typed cells and device copy are
// kept per device (up to LIT_CACHE entries) and reused when the texts are the same.
// An entry that some Literals of the running query uses is never replaced.
constexpr size_t LIT_CACHE = 8;
struct LitEntry {
    std::string key;
    uint8_t* dev = nullptr;
    size_t cap = 0;
    std::vector<Cell> cells;
    std::vector<HCell> host;
    size_t cell_off = 0;
    uint64_t gen = 0;                  // the last query that used it
};
std::vector<LitEntry> g_litcache[64];

// typed on the host by cell.h's parser (hostcell.cpp, the kernels' own typing
// code); STRING literals get a device copy of their bytes for the kernels
void parse_literals(DevCtx& c, const std::vector<std::string>& texts, Literals& L) {
    size_t n = texts.size();
    L.dev.release();
    L.dcells = nullptr;
    L.cells.clear();
    L.host.clear();
    if (!n) return;
    std::string key;
    for (size_t i = 0; i < n; i++) {
        const uint32_t k = (uint32_t)texts[i].size();
        key.append((const char*)&k, 4);
        key += texts[i];
    }
    std::vector<LitEntry>& cache = g_litcache[c.device & 63];
    for (LitEntry& e : cache) {
        if (e.dev && e.key == key) {
            e.gen = c.query_gen;
            L.cells = e.cells;
            L.host = e.host;
            L.dcells = (Cell*)(e.dev + e.cell_off);
            return;
        }
    }
    std::vector<size_t> offs(n);
    std::string blob;
    for (size_t i = 0; i < n; i++) {
        offs[i] = blob.size();
        blob += texts[i];
        blob.append(16, '\0');            // strtoll/strtod stop at the C string's NUL
    }
    L.cells.resize(n);
    L.host.resize(n);
    for (size_t i = 0; i < n; i++) {
        const uint8_t* t = (const uint8_t*)blob.data() + offs[i];
        Cell x = cq_host_parse_cell(t, (uint32_t)texts[i].size());
        L.host[i].kind = x.kind;
        L.host[i].bits = x.bits;
        if (x.kind == K_STR) {
            const size_t off = (size_t)((const uint8_t*)(uintptr_t)x.bits - (const uint8_t*)blob.data());
            L.host[i].s.assign(blob.data() + off, x.len);
            x.bits = off;                  // relocated to the device copy below
        }
        L.cells[i] = x;
    }
    const size_t cell_off = (blob.size() + 15) & ~(size_t)15;
    const size_t bytes = cell_off + n * sizeof(Cell);
    // a cache entry no Literals of this query holds (else the query's scratch)
    LitEntry* slot = nullptr;
    if (cache.size() < LIT_CACHE) {
        cache.emplace_back();
        slot = &cache.back();
    } else {
        for (LitEntry& e : cache)
            if (e.gen < c.query_gen && (!slot || e.gen < slot->gen)) slot = &e;
    }
    uint8_t* dst;
    if (slot) {
        if (slot->cap < bytes) {
            if (slot->dev) HIPCHECK(hipFree(slot->dev));
            slot->dev = nullptr;
            slot->cap = 0;
            HIPCHECK(hipMalloc((void**)&slot->dev, std::max<size_t>(bytes, 4096)));
            slot->cap = std::max<size_t>(bytes, 4096);
        }
        dst = slot->dev;
    } else {
        L.dev.get(c, bytes);
        dst = L.dev.p;
    }
    for (size_t i = 0; i < n; i++)
        if (L.cells[i].kind == K_STR) L.cells[i].bits += (uint64_t)(uintptr_t)dst;
    std::vector<uint8_t> up(bytes, 0);
    memcpy(up.data(), blob.data(), blob.size());
    memcpy(up.data() + cell_off, L.cells.data(), n * sizeof(Cell));
    HIPCHECK(hipMemcpyAsync(dst, up.data(), up.size(), hipMemcpyHostToDevice, c.stream));
    L.dcells = (Cell*)(dst + cell_off);
    HIPCHECK(hipStreamSynchronize(c.stream));   // the staging vector goes out of scope
    if (slot) {
        slot->key = key;
        slot->cells = L.cells;
        slot->host = L.host;
        slot->cell_off = cell_off;
        slot->gen = c.query_gen;
    }
}

// group table arena in the device workspace
struct TableArena {
    GroupTable gt;
    GroupTable rt;                     // raw-byte keys of lean_kernel (lean.hip), merged into gt
    ScanStats* stats;
    GroupOut* out;
    unsigned int* out_count;
    unsigned long long* slow_list;     // records the fast scan declines (scan.hip slow_kernel)
    unsigned long long slow_cap;
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// one launch initialises an arena: bytes [0, n) zero except the 0xff regions
// (every region 256-byte aligned; the slow list past n needs no initialisation)
constexpr int ARENA_FILLS = 32;
struct ArenaFills {
    uint32_t n;
    uint64_t off[ARENA_FILLS], end[ARENA_FILLS];
};
__global__ void arena_init_kernel(uint4* __restrict__ base, uint64_t n16, ArenaFills F) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b = i * 16;
        bool ff = false;
        for (uint32_t k = 0; k < F.n; k++) ff |= (b >= F.off[k]) & (b < F.end[k]);
        const uint32_t v = ff ? 0xffffffffu : 0u;
        base[i] = make_uint4(v, v, v, v);
    }
}

TableArena make_arena(DevCtx& c, const ScanPlan& P, uint32_t cap, size_t out_cap, size_t cand_blocks = 0,
                      uint32_t cand_stride = 16, unsigned long long slow_cap = 1ull << 20) {
    TableArena A;
    memset(&A.gt, 0, sizeof A.gt);
    memset(&A.rt, 0, sizeof A.rt);
    A.slow_cap = slow_cap;
    A.rt.cap = cap;
    A.rt.cand_stride = cand_stride;
    A.gt.cap = cap;
    A.gt.cand_stride = cand_stride;
    struct Part { void** p; size_t bytes; int fill; };
    std::vector<Part> parts;
    parts.push_back({(void**)&A.gt.tag, cap * 4ull, 0});
    parts.push_back({(void**)&A.gt.clslen, cap * 4ull, 0});
    parts.push_back({(void**)&A.gt.w0, cap * 8ull, 0});
    parts.push_back({(void**)&A.gt.w1, cap * 8ull, 0});
    parts.push_back({(void**)&A.gt.cnt, cap * 8ull, 0});
    parts.push_back({(void**)&A.gt.first, cap * 8ull, 0xff});
    for (int a = 0; a < P.nacc; a++) {
        if (P.acc[a].kind == ACC_SUM) {
            parts.push_back({(void**)&A.gt.sum[a], cap * 8ull, 0});
            parts.push_back({(void**)&A.gt.num[a], cap * 8ull, 0});
        } else {
            parts.push_back({(void**)&A.gt.ext[a], cap * (size_t)sizeof(Cell), 0});
            parts.push_back({(void**)&A.gt.extpos[a], cap * 8ull, 0xff});
            parts.push_back({(void**)&A.gt.lock[a], cap * 4ull, 0});
            parts.push_back({(void**)&A.gt.extref[a], cap * 8ull, 0xff});
            parts.push_back({(void**)&A.gt.cand[a], std::max<size_t>(cand_blocks, 1) * cand_stride * sizeof(ExtCand), 0});
        }
    }
    parts.push_back({(void**)&A.gt.used, 256, 0});
    bool sums_only = true;
    for (int a = 0; a < P.nacc; a++) sums_only = sums_only && P.acc[a].kind == ACC_SUM;
    // lean_kernel / fast_kernel plans: the raw-key table (with extreme cells for a
    // fast_kernel MIN / MAX build, cq_fast_ext_plan)
    if (sums_only || cq_fast_ext_plan(&P, 1) || cq_fast_ext_plan(&P, 0)) {
        parts.push_back({(void**)&A.rt.tag, cap * 4ull, 0});
        parts.push_back({(void**)&A.rt.clslen, cap * 4ull, 0});
        parts.push_back({(void**)&A.rt.w0, cap * 8ull, 0});
        parts.push_back({(void**)&A.rt.w1, cap * 8ull, 0});
        parts.push_back({(void**)&A.rt.cnt, cap * 8ull, 0});
        parts.push_back({(void**)&A.rt.first, cap * 8ull, 0xff});
        for (int a = 0; a < P.nacc; a++) {
            if (P.acc[a].kind == ACC_SUM) {
                parts.push_back({(void**)&A.rt.sum[a], cap * 8ull, 0});
                parts.push_back({(void**)&A.rt.num[a], cap * 8ull, 0});
            } else {
                parts.push_back({(void**)&A.rt.ext[a], cap * (size_t)sizeof(Cell), 0});
                parts.push_back({(void**)&A.rt.extpos[a], cap * 8ull, 0xff});
                parts.push_back({(void**)&A.rt.lock[a], cap * 4ull, 0});
            }
        }
        parts.push_back({(void**)&A.rt.used, 256, 0});
    }
    parts.push_back({(void**)&A.stats, 256, 0});
    parts.push_back({(void**)&A.out_count, 256, 0});
    parts.push_back({(void**)&A.out, out_cap * sizeof(GroupOut), 0});
    parts.push_back({(void**)&A.slow_list, slow_cap * 8ull, 0});
    size_t total = 0;
    for (auto& p : parts) total += align256(p.bytes);
    uint8_t* base = (uint8_t*)workspace(c, total);
    size_t off = 0;
    ArenaFills F;
    F.n = 0;
    bool fits = true;
    for (auto& p : parts) {
        *p.p = base + off;
        if (p.fill) {
            if (p.fill != 0xff || F.n == ARENA_FILLS) fits = false;
            else { F.off[F.n] = off; F.end[F.n] = off + align256(p.bytes); F.n++; }
        }
        off += align256(p.bytes);
    }
    const size_t init = total - align256(slow_cap * 8ull);   // the slow list is the last part
    if (fits) {
        const uint64_t n16 = init / 16;
        const unsigned grid = (unsigned)std::min<uint64_t>((n16 + 255) / 256, 2048);
        hipLaunchKernelGGL(arena_init_kernel, dim3(std::max(grid, 1u)), dim3(256), 0, c.stream, (uint4*)base, n16, F);
        HIPCHECK(hipGetLastError());
    } else {             // zero everything in one memset, then the fill regions
        HIPCHECK(hipMemsetAsync(base, 0, init, c.stream));
        off = 0;
        for (auto& p : parts) {
            if (p.fill) HIPCHECK(hipMemsetAsync(base + off, p.fill, p.bytes, c.stream));
            off += align256(p.bytes);
        }
    }
    return A;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// CQ_AMD_TIMING=1: host-side phase times of each aggregate query on stderr
struct PhaseClock {
    bool on;
    double t;
    std::string line;
    PhaseClock() : on(getenv("CQ_AMD_TIMING") != nullptr), t(on ? now_ms() : 0.0) {}
    void mark(const char* what) {
        if (!on) return;
        const double n = now_ms();
        char b[64];
        snprintf(b, sizeof b, " %s %.3f", what, n - t);
        line += b;
        t = n;
    }
    ~PhaseClock() { if (on && !line.empty()) fprintf(stderr, "cq_amd timing ms:%s\n", line.c_str()); }
};
PhaseClock* g_phase = nullptr;
#define PHASE(x) do { if (g_phase) g_phase->mark(x); } while (0)

// compacted groups + finish output -> host groups in first-appearance order
// (create_groups appends groups in row order); `limit`: first positions are below it
std::vector<HGroup> make_groups(DevCtx& c, const Compiled& C, uint64_t limit, uint64_t base_offset,
                                std::vector<GroupOut>& outs, std::vector<Cell>& fcells, std::vector<uint8_t>& fbytes,
                                int nrep_sorted, const std::vector<int>& rep_ord, uint32_t SB,
                                bool presorted = false) {
    std::vector<HGroup> groups;
    const uint32_t ncell = (uint32_t)nrep_sorted + (uint32_t)C.P.nacc + 1;
    // single group: always present (evaluator.c:232-247), even with no rows
    if (!C.grouped && outs.empty()) {
        GroupOut z;
        memset(&z, 0, sizeof z);
        z.clslen = (uint32_t)GK_ALL << 16;   // the kernels' key of the one group (partials merge by it)
        z.first = NOPOS;
        for (int a = 0; a < MAX_ACC; a++) z.extpos[a] = NOPOS;
        outs.push_back(z);
        fcells.assign(ncell, Cell{K_NULL, 0, 0});
        fbytes.assign((size_t)ncell * SB, 0);
    }
    // never let a kernel bug turn into an out-of-bounds gather below
    for (auto& o : outs)
        if (o.first != NOPOS && o.first >= limit) throw HipError{"scan kernel: group first-row offset out of range"};
    // host cells of the finish output; STRINGs longer than SB fetched in one batch
    std::vector<HCell> hcells(fcells.size());
    std::vector<Cell> longs;
    std::vector<size_t> long_at;
    for (size_t k = 0; k < fcells.size(); k++) {
        hcells[k].kind = fcells[k].kind;
        hcells[k].bits = fcells[k].bits;
        if (fcells[k].kind != K_STR) continue;
        if (fcells[k].len <= SB) {
            hcells[k].s.assign((const char*)fbytes.data() + k * SB, fcells[k].len);
        } else {
            longs.push_back(fcells[k]);
            long_at.push_back(k);
        }
    }
    if (getenv("CQGPU_DEBUG_GROUPS")) {   // the groups as the device returned them
        fprintf(stderr, "make_groups: %zu groups, %u cells each\n", outs.size(), ncell);
        for (size_t i = 0; i < outs.size() && i < 16; i++) {
            const GroupOut& o = outs[i];
            fprintf(stderr, "  g%zu cls %u len %u w0 0x%llx w1 0x%llx cnt %llu first %llu\n", i, o.clslen >> 16,
                    o.clslen & 0xffff, (unsigned long long)o.w0, (unsigned long long)o.w1, (unsigned long long)o.cnt,
                    (unsigned long long)o.first);
            for (uint32_t k = 0; k < ncell && (i + 1) * ncell <= fcells.size(); k++)
                fprintf(stderr, "    cell %u kind %u len %u bits 0x%llx\n", k, fcells[i * ncell + k].kind,
                        fcells[i * ncell + k].len, (unsigned long long)fcells[i * ncell + k].bits);
        }
        for (auto& r : g_table_ranges)
            fprintf(stderr, "  table bytes [0x%llx, 0x%llx)\n", (unsigned long long)r.first, (unsigned long long)r.second);
    }
    if (!longs.empty()) {
        std::vector<HCell> hl = fetch_cells(c, longs, true);
        for (size_t i = 0; i < longs.size(); i++) hcells[long_at[i]] = hl[i];
    }
    PHASE("hcells");
    // first-appearance order (create_groups appends groups in row order)
    std::vector<uint32_t> order(outs.size());
    if (presorted) {                       // pack_result_kernel placed them in this order
        for (size_t i = 0; i < order.size(); i++) order[i] = (uint32_t)i;
    } else {
        std::vector<std::pair<unsigned long long, uint32_t>> fo(outs.size());
        for (size_t i = 0; i < fo.size(); i++) fo[i] = {outs[i].first, (uint32_t)i};
        std::sort(fo.begin(), fo.end());   // (first, index): ties keep the index order
        for (size_t i = 0; i < fo.size(); i++) order[i] = fo[i].second;
    }
    const size_t nrep = C.rep_cols.size();
    PHASE("order");
    groups.reserve(order.size());
    for (uint32_t gi : order) {
        const GroupOut& o = outs[gi];
        const HCell* cs = hcells.data() + (size_t)gi * ncell;
        groups.emplace_back();
        HGroup& h = groups.back();
        h.kcls = o.clslen >> 16;
        h.klen = o.clslen & 0xffff;
        h.kw0 = o.w0;
        h.kw1 = o.w1;
        if (h.kcls == GK_LONG) {
            h.kbytes = cs[nrep_sorted + C.P.nacc].s;
        } else if (h.kcls == GK_STR) {
            for (uint32_t i = 0; i < h.klen; i++)
                h.kbytes.push_back((char)((i < 8 ? o.w0 >> (8 * i) : o.w1 >> (8 * (i - 8))) & 0xff));
        }
        h.cnt = o.cnt;
        h.first = o.first == NOPOS ? NOPOS : o.first + base_offset;
        for (int a = 0; a < MAX_ACC; a++) {
            h.sum[a] = o.sum[a];
            h.num[a] = o.num[a];
            if (a < C.P.nacc) {
                h.ext[a] = cs[nrep_sorted + a];
                h.extpos[a] = o.extpos[a] == NOPOS ? NOPOS : o.extpos[a] + base_offset;
            }
        }
        h.reps.resize(nrep);
        for (size_t i = 0; i < rep_ord.size(); i++) h.reps[rep_ord[i]] = cs[i];
    }
    PHASE("groups");
    return groups;
}

// Result-table blocks allocated while the device works: the host waits ~1 ms in the
// stream synchronisation of every scan, and the result rows csv_free releases
// (reference csv_reader.c:467-490: every row's values array and every string is its
// own malloc block) cost ~50 us of calloc / malloc per 1,000 groups after it.  The
// pool keeps calloc'd value arrays and malloc'd string blocks of POOL_STR bytes,
// refilled during the wait to the previous result's size; build_direct takes from
// it (any malloc block of the needed size is what csv_free expects).
struct RowPool {
    int ncols = -1;
    std::vector<cq_value*> vals;
    std::vector<char*> strs;
    uint32_t hint = 0;                 // rows of the last direct result
};
constexpr size_t POOL_STR = 32;
thread_local RowPool g_rowpool;
const bool g_rowpool_off = getenv("CQGPU_NO_ROWPOOL") != nullptr;   // A/B knob
void rowpool_fill(int ncols, uint32_t nstr_per_row) {
    if (g_rowpool_off) return;
    RowPool& P = g_rowpool;
    if (P.ncols != ncols) {
        for (cq_value* v : P.vals) free(v);
        P.vals.clear();
        P.ncols = ncols;
    }
    const size_t want = std::min<size_t>(P.hint, 1u << 16);
    while (P.vals.size() < want) P.vals.push_back((cq_value*)calloc(std::max(ncols, 1), sizeof(cq_value)));
    const size_t ws = std::min<size_t>(want * nstr_per_row, 1u << 17);
    while (P.strs.size() < ws) P.strs.push_back((char*)malloc(POOL_STR));
}
cq_value* rowpool_vals(int ncols) {
    RowPool& P = g_rowpool;
    if (P.ncols == ncols && !P.vals.empty()) {
        cq_value* v = P.vals.back();
        P.vals.pop_back();
        return v;
    }
    return (cq_value*)calloc(std::max(ncols, 1), sizeof(cq_value));
}
char* rowpool_str(size_t bytes) {
    RowPool& P = g_rowpool;
    if (bytes <= POOL_STR && !P.strs.empty()) {
        char* s = P.strs.back();
        P.strs.pop_back();
        return s;
    }
    return (char*)malloc(bytes);
}

// run the fused scan (with regrowth on overflow) and return the groups
// row_out (optional): offsets of the records passing WHERE, unordered; entries
// past row_cap are counted in ScanStats.rows_emitted but not written
cq_table* build_direct(const Compiled& C, const uint8_t* hp, uint32_t ng, uint32_t ncell, uint32_t SB,
                       const std::vector<int>& rep_ord, const Literals& L, uint64_t limit);

// gather-merge output of one rank (dist_query): its groups packed in the GM
// layout (plan.h) into `dst` (header first; the caller zeroes the header's status)
struct GmSend {
    uint8_t* dst = nullptr;
    uint32_t maxg = 0;
    uint32_t ng = 0;                 // out: the rank's groups (may exceed maxg: declined)
};

// direct (optional): for plans build_direct handles, the result table built straight
// from the packed result (no HGroup per group); the returned vector is then empty.
// gm (optional): the groups packed for the gather-merge instead, nothing returned
std::vector<HGroup> run_aggregate(DevCtx& c, const cqgpu_table* t, Compiled& C, Literals& L,
                                  ScanStats* stats_out, unsigned long long* row_out = nullptr,
                                  unsigned long long row_cap = 0, cq_table** direct = nullptr,
                                  GmSend* gm = nullptr) {
    parse_literals(c, C.lits, L);
    for (size_t i = 0; i < L.cells.size(); i++) C.P.consts[i] = L.cells[i];
    PHASE("literals");
    std::vector<HGroup> groups;
    if (C.group_missing) return groups;    // create_groups: unknown column -> no groups
    const int grouped = C.grouped ? 1 : 0;
    uint32_t cap = grouped ? 8192 : 64;
    int retries = 0;
    const uint64_t windows = (t->n + 31679) / 31680;   // scan.hip WSTRIDE
    int per_cu = cq_scan_occupancy(&C.P, grouped);
    int grid = (int)std::min<uint64_t>(std::max<uint64_t>(windows, 1), (uint64_t)c.ncu * per_cu);
    ScanStats st;
    std::vector<GroupOut> outs;
    // what finish_kernel gathers per group: representative cells (ascending columns),
    // MIN/MAX cells, the long-key text; STRING bytes inline up to SB
    constexpr uint32_t SB = 48;
    FinishDesc FD;
    memset(&FD, 0, sizeof FD);
    std::vector<int> rep_ord(C.rep_cols.size());
    for (size_t i = 0; i < rep_ord.size(); i++) rep_ord[i] = (int)i;
    std::sort(rep_ord.begin(), rep_ord.end(), [&](int a, int b) { return C.rep_cols[a] < C.rep_cols[b]; });
    if (C.wide) throw HipError{"internal: a wide plan reached the fused scan"};
    if (rep_ord.size() > (size_t)MAX_WIDE) throw Ineligible{"too many representative columns"};
    FD.ncols = (int32_t)rep_ord.size();
    for (size_t i = 0; i < rep_ord.size(); i++) FD.cols[i] = (int16_t)C.rep_cols[rep_ord[i]];
    FD.delim = C.P.delim;
    FD.quote = C.P.quote;
    FD.nacc = C.P.nacc;
    FD.sb = SB;
    const uint32_t ncell = (uint32_t)FD.ncols + (uint32_t)FD.nacc + 1;
    std::vector<Cell> fcells;
    std::vector<uint8_t> fbytes;
    uint64_t chunk = 0;          // 0: the whole table in one launch
    bool presorted = false;
    while (true) {
        // test knob CQGPU_SLOW_CAP: a smaller slow-record list, to force the chunked rescan
        unsigned long long slow_cap = 1ull << 20;
        if (const char* e = getenv("CQGPU_SLOW_CAP"))
            if (atoll(e) >= 64) slow_cap = std::min<unsigned long long>(slow_cap, (unsigned long long)atoll(e));
        TableArena A = make_arena(c, C.P, cap, cap / 2 + 1, (size_t)grid, cq_scan_cand_stride(&C.P, grouped), slow_cap);
        const unsigned int cap_out = cap / 2 + 1;
        Scratch fin(c, (size_t)cap_out * ncell * (sizeof(Cell) + SB) + 64);
        Cell* dcells = (Cell*)fin.p;
        uint8_t* dbytes = fin.p + (size_t)cap_out * ncell * sizeof(Cell);
        // the mailbox: scan statistics and group count, then the packed result
        constexpr size_t MAIL_HDR = 1024;
        static_assert(sizeof(ScanStats) + 4 <= MAIL_HDR, "mailbox header");
        uint8_t* mail = mailbox(c, MAIL_HDR + cq_pack_result_bytes(cap_out, C.P.nacc, ncell, SB) + 64);
        Scratch pk, ofs;                          // the packed result in HBM (until the sync below)
        bool is_packed = false;
        memset(&st, 0, sizeof st);
        unsigned long long last_clk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        float ms_total = 0;
        bool slow_over = false, finished = false;
        unsigned int ng = 0;
        const uint64_t step = chunk ? chunk : std::max<uint64_t>(t->n, 1);
        for (uint64_t b = 0; b < std::max<uint64_t>(t->n, 1); b += step) {
            ScanPlan P = C.P;
            P.range_begin = b;
            P.range_end = std::min<uint64_t>(b + step, t->n);
            const uint64_t wins = (P.range_end - P.range_begin + 31679) / 31680 + 1;
            const int g2 = chunk ? (int)std::min<uint64_t>(grid, wins) : grid;
            HIPCHECK(hipEventRecord(c.ev0, c.stream));
            const unsigned long long done = st.rows_emitted;
            HIPCHECK(cq_launch_scan(t->g, &P, &A.gt, A.rt.tag ? &A.rt : nullptr, A.stats, row_out ? row_out + std::min(done, row_cap) : nullptr,
                                    row_cap > done ? row_cap - done : 0, grouped, g2, c.stream, nullptr,
                                    A.slow_list, A.slow_cap));
            HIPCHECK(hipEventRecord(c.ev1, c.stream));
            // finish + pack in one launch (finish_pack_kernel) for the mailbox path
            const bool fp = !chunk && !gm && cap_out <= cq_finish_pack_max() && !getenv("CQGPU_PACK_MAPPED") &&
                            !getenv("CQGPU_NO_FINISH_PACK");
            if (fp) {
                ofs.get(c, (size_t)cap_out * 8 + 64);
                pk.get(c, cq_pack_result_bytes(cap_out, C.P.nacc, ncell, SB) + 64);
                HIPCHECK(cq_launch_compact(&A.gt, &C.P, A.out, A.out_count, cap_out, c.stream,
                                           (unsigned long long*)ofs.p));
                HIPCHECK(cq_launch_finish_pack(t->g, t->n, A.out, (const unsigned long long*)ofs.p, A.out_count,
                                               cap_out, &FD, pk.p, A.stats, mail, c.stream));
                HIPCHECK(cq_launch_mail_copy(pk.p, A.out_count, cap_out, C.P.nacc, ncell, SB, mail + MAIL_HDR, c.stream));
                finished = true;
                is_packed = true;
            } else if (!chunk) {      // one launch: compact and finish speculatively, one sync for all
                HIPCHECK(cq_launch_compact(&A.gt, &C.P, A.out, A.out_count, cap_out, c.stream, nullptr));
                HIPCHECK(cq_launch_finish(t->g, t->n, A.out, A.out_count, cap_out, &FD, dcells, dbytes, c.stream));
                if (gm) {                            // the rank's records for the root (header: mailbox)
                    HIPCHECK(cq_launch_gm_pack(A.out, A.out_count, cap_out, C.P.nacc, (uint32_t)FD.ncols, dcells,
                                               dbytes, SB, gm->maxg, gm->dst, A.stats, mail, c.stream));
                } else if (getenv("CQGPU_PACK_MAPPED")) {   // A/B knob: pack straight into the mapped mailbox
                    HIPCHECK(cq_launch_pack_result(A.out, A.out_count, cap_out, C.P.nacc, dcells, dbytes, ncell, SB,
                                                   mail + MAIL_HDR, A.stats, mail, 1, c.stream));
                } else {                             // pack in HBM, then coalesced copy into the mailbox
                    pk.get(c, cq_pack_result_bytes(cap_out, C.P.nacc, ncell, SB) + 64);
                    HIPCHECK(cq_launch_pack_result(A.out, A.out_count, cap_out, C.P.nacc, dcells, dbytes, ncell, SB,
                                                   pk.p, A.stats, mail, 1, c.stream));
                    HIPCHECK(cq_launch_mail_copy(pk.p, A.out_count, cap_out, C.P.nacc, ncell, SB, mail + MAIL_HDR,
                                                 c.stream));
                }
                finished = true;
                is_packed = !gm;
            }
            // the group count and the scan statistics through pinned memory, one sync
            // (one launch: pack_result_kernel wrote both into the mailbox)
            uint8_t* hs = finished ? mail : (uint8_t*)pinned(c, sizeof(ScanStats) + 16);
            if (!finished) HIPCHECK(hipMemcpyAsync(hs, A.stats, sizeof(ScanStats), hipMemcpyDeviceToHost, c.stream));
            PHASE("launch");
            if (direct && finished && C.grouped) {      // the result's blocks, while the device works
                uint32_t nstr = 0;
                for (const OutCol& o : C.outs) nstr += o.kind == OUT_REP || o.kind == OUT_CONST;
                rowpool_fill((int)C.outs.size(), nstr);
                PHASE("pool");
            }
            HIPCHECK(hipStreamSynchronize(c.stream));
            PHASE("scan+finish");
            ScanStats s1;
            memcpy(&s1, hs, sizeof s1);
            if (finished) memcpy(&ng, hs + sizeof(ScanStats), 4);
            float ms = 0;
            HIPCHECK(hipEventElapsedTime(&ms, c.ev0, c.ev1));
            ms_total += ms;
            for (int i = 0; i < 8; i++) last_clk[i] = s1.clk[i];
            st.records += s1.records;
            st.passed += s1.passed;
            st.short_rows += s1.short_rows;
            st.lds_spills += s1.lds_spills;
            st.rows_emitted += s1.rows_emitted;
            st.slow_records += s1.slow_records;
            st.overflow = std::max(st.overflow, s1.overflow);
            for (int a = 0; a < MAX_ACC; a++) st.acc_classes[a] |= s1.acc_classes[a];
            if (s1.slow_records > A.slow_cap) { slow_over = true; break; }
            if (chunk) HIPCHECK(hipMemsetAsync(A.stats, 0, sizeof(ScanStats), c.stream));
        }
        g_stats.scan_ms = ms_total;
        g_stats.grid = grid;
        g_stats.scan_kernel = cq_scan_kernel_kind(&C.P, grouped, row_out != nullptr, 0);
        for (int i = 0; i < 8; i++) g_clk[i] = last_clk[i];
        if (st.overflow >= 2)   // a bounded spin gave up: a kernel bug, never a data property
            throw HipError{st.overflow == 2 ? "scan kernel: MIN/MAX lock timeout" : "scan kernel: group insert timeout"};
        if (slow_over) {        // too many records for the general kernel's list: rescan in chunks
            if (chunk) throw HipError{"scan: slow-record list overflow"};
            chunk = A.slow_cap;
            continue;
        }
        if (st.overflow) {
            if (cap >= (1u << 30)) throw HipError{"group table overflow"};
            cap *= 8;
            retries++;
            continue;
        }
        if (!finished) {
            HIPCHECK(cq_launch_compact(&A.gt, &C.P, A.out, A.out_count, cap_out, c.stream, nullptr));
            HIPCHECK(cq_launch_finish(t->g, t->n, A.out, A.out_count, cap_out, &FD, dcells, dbytes, c.stream));
            if (gm)
                HIPCHECK(cq_launch_gm_pack(A.out, A.out_count, cap_out, C.P.nacc, (uint32_t)FD.ncols, dcells, dbytes,
                                           SB, gm->maxg, gm->dst, A.stats, nullptr, c.stream));
            HIPCHECK(hipMemcpyAsync(&ng, A.out_count, 4, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
        }
        ng = std::min(ng, cap_out);
        if (gm) {                   // packed for the root: statistics only
            gm->ng = ng;
            g_stats.retries = retries;
            g_stats.records = st.records;
            g_stats.lds_spills = st.lds_spills;
            g_stats.slow_records = st.slow_records;
            g_stats.passed = st.passed;
            g_stats.scan_bytes = t->n;
            if (stats_out) *stats_out = st;
            return {};
        }
        if (direct && is_packed && ng && ng <= cq_pack_order_max() && C.grouped) {
            // the stats checks below run first; then the table straight from the mailbox
            for (int a = 0; a < C.P.nacc; a++) {
                if (C.P.acc[a].kind == ACC_SUM) continue;
                unsigned m = st.acc_classes[a];
                if (m & (m - 1)) throw MixedExtremes{};
            }
            // (one sequential copy out of the PCIe-written mailbox, then cached reads)
            static thread_local std::vector<uint8_t> hbuf;
            const size_t pb = cq_pack_result_bytes(ng, C.P.nacc, ncell, SB);
            if (hbuf.size() < pb) hbuf.resize(pb);
            memcpy(hbuf.data(), mail + MAIL_HDR, pb);
            PHASE("mcopy");
            *direct = build_direct(C, hbuf.data(), ng, ncell, SB, rep_ord, L, t->n);
            if (*direct) {
                g_stats.retries = retries;
                g_stats.records = st.records;
                g_stats.lds_spills = st.lds_spills;
                g_stats.slow_records = st.slow_records;
                g_stats.passed = st.passed;
                g_stats.scan_bytes = t->n;
                g_stats.groups = ng;
                if (stats_out) *stats_out = st;
                PHASE("direct");
                return {};
            }
        }
        outs.resize(ng);
        fcells.resize((size_t)ng * ncell);
        fbytes.resize((size_t)ng * ncell * SB);
        if (ng && is_packed) {   // one copy of the packed result (pack_result_kernel's layout)
            const size_t rec = 40 + 40 * (size_t)C.P.nacc, b1 = fcells.size() * sizeof(Cell), b2 = fbytes.size();
            const uint8_t* hp = mail + MAIL_HDR;   // written by pack_result_kernel, synchronised above
            memset(outs.data(), 0, ng * sizeof(GroupOut));
            for (unsigned int i = 0; i < ng; i++) {
                const uint8_t* r = hp + i * rec;
                GroupOut& o = outs[i];
                o.clslen = ((const uint32_t*)r)[0];
                o.w0 = ((const uint64_t*)r)[1];
                o.w1 = ((const uint64_t*)r)[2];
                o.cnt = ((const unsigned long long*)r)[3];
                o.first = ((const unsigned long long*)r)[4];
                const uint64_t* q = (const uint64_t*)(r + 40);
                for (int a = 0; a < C.P.nacc; a++) {
                    o.sum[a] = as_dbl(q[5 * a]);
                    o.num[a] = q[5 * a + 1];
                    o.ext[a].kind = (uint32_t)q[5 * a + 2];
                    o.ext[a].len = (uint32_t)(q[5 * a + 2] >> 32);
                    o.ext[a].bits = q[5 * a + 3];
                    o.extpos[a] = q[5 * a + 4];
                }
            }
            memcpy(fcells.data(), hp + ng * rec, b1);
            memcpy(fbytes.data(), hp + ng * rec + b1, b2);
        } else if (ng) {   // through the pinned staging buffer: three async copies, one sync
            const size_t b0 = ng * sizeof(GroupOut), b1 = fcells.size() * sizeof(Cell), b2 = fbytes.size();
            uint8_t* hp = (uint8_t*)pinned(c, b0 + b1 + b2);
            HIPCHECK(hipMemcpyAsync(hp, A.out, b0, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipMemcpyAsync(hp + b0, dcells, b1, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipMemcpyAsync(hp + b0 + b1, dbytes, b2, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
            memcpy(outs.data(), hp, b0);
            memcpy(fcells.data(), hp + b0, b1);
            memcpy(fbytes.data(), hp + b0 + b1, b2);
        }
        presorted = is_packed && ng <= cq_pack_order_max();
        PHASE("copies");
        break;
    }
    g_stats.retries = retries;
    g_stats.records = st.records;
    g_stats.lds_spills = st.lds_spills;
    g_stats.slow_records = st.slow_records;
    g_stats.passed = st.passed;
    g_stats.scan_bytes = t->n;
    if (stats_out) *stats_out = st;
    // MIN/MAX over a column mixing value classes depends on row order in the
    // reference (incomparable cells compare equal): the cells path folds it
    for (int a = 0; a < C.P.nacc; a++) {
        if (C.P.acc[a].kind == ACC_SUM) continue;
        unsigned m = st.acc_classes[a];
        if (m & (m - 1)) throw MixedExtremes{};
    }
    return make_groups(c, C, t->n, t->base_offset, outs, fcells, fbytes, FD.ncols, rep_ord, SB,
                       presorted);
}

// ------------------------------------------------------------------ result tables
cq_table* new_result(const std::vector<std::string>& names) {
    cq_table* r = (cq_table*)calloc(1, sizeof(cq_table));
    r->filename = strdup("query_result");
    r->data = nullptr;
    r->fd = -1;
    r->has_header = true;
    r->delimiter = ',';
    r->quote = '"';
    r->ncols = (int)names.size();
    r->columns = (cq_column*)malloc(sizeof(cq_column) * std::max<size_t>(names.size(), 1));
    for (size_t i = 0; i < names.size(); i++) {
        r->columns[i].name = strdup(names[i].c_str());
        r->columns[i].inferred_kind = CQ_V_STRING;
    }
    return r;
}

void free_row(cq_row& row) {
    for (int j = 0; j < row.ncols; j++)
        if (row.values[j].kind == CQ_V_STRING) free(row.values[j].u.s);
    free(row.values);
}

// build_aggregated_result rows (evaluator_aggregates.c:596-693)
// order (optional): row g is groups[(*order)[g]] (a merge's first-pair order without
// moving the groups)
cq_table* build_groups(const Compiled& C, const std::vector<HGroup>& groups, const Literals& L,
                       DevCtx& c, const std::vector<uint32_t>* order = nullptr) {
    cq_table* r = new_result(C.names);
    r->nrows = r->row_capacity = (int)groups.size();
    r->rows = (cq_row*)malloc(sizeof(cq_row) * std::max<size_t>(groups.size(), 1));
    std::vector<HCell> litcells;
    if (!L.cells.empty()) litcells = L.host;
    for (size_t g = 0; g < groups.size(); g++) {
        const HGroup& h = groups[order ? (*order)[g] : g];
        cq_row& row = r->rows[g];
        row.ncols = r->ncols;
        row.values = (cq_value*)calloc(std::max(r->ncols, 1), sizeof(cq_value));
        for (int i = 0; i < r->ncols; i++) {
            const OutCol& o = C.outs[i];
            HCell v;
            switch (o.kind) {
                case OUT_COUNT: v.kind = K_INT; v.bits = (uint64_t)h.cnt; break;
                case OUT_SUM: v.kind = K_DBL; v.bits = dbl_bits(h.num[o.acc] ? h.sum[o.acc] : 0.0); break;
                case OUT_AVG:
                    v.kind = K_DBL;
                    v.bits = dbl_bits(h.num[o.acc] ? h.sum[o.acc] / (double)h.num[o.acc] : 0.0);
                    break;
                case OUT_EXT: if (h.extpos[o.acc] != NOPOS) v = h.ext[o.acc]; break;
                case OUT_VLA:
                    if (h.vla_ok[o.acc]) { v.kind = K_DBL; v.bits = dbl_bits(h.vla[o.acc]); }
                    break;
                case OUT_REP: if (h.cnt > 0 && o.rep < (int)h.reps.size()) v = h.reps[o.rep]; break;
                case OUT_CONST: if (h.cnt > 0) v = litcells[o.lit]; break;
                case OUT_HEXPR:
                    if (h.cnt > 0) {
                        // host cells -> cells whose STRING bits point at the host strings
                        std::vector<Cell> cols(h.reps.size()), consts(litcells.size());
                        auto to_cell = [](const HCell& x) {
                            Cell y;
                            y.kind = x.kind; y.len = (uint32_t)x.s.size(); y.bits = x.bits;
                            if (x.kind == K_STR) y.bits = (uint64_t)(uintptr_t)x.s.c_str();
                            return y;
                        };
                        for (size_t k = 0; k < cols.size(); k++) cols[k] = to_cell(h.reps[k]);
                        for (size_t k = 0; k < consts.size(); k++) consts[k] = to_cell(litcells[k]);
                        const auto& code = C.hexpr[o.acc];
                        const Cell r = cq_host_eval(code.data(), (uint32_t)code.size(), cols.data(), consts.data());
                        v.kind = r.kind;
                        v.bits = r.bits;
                        if (r.kind == K_STR) v.s.assign((const char*)(uintptr_t)r.bits, r.len);
                    }
                    break;
                default: break;
            }
            row.values[i] = to_value(v);
        }
    }
    return r;
}

// build_groups' rows straight from pack_result_kernel's output in first-appearance
// order, for plans whose items are COUNT / SUM / AVG / representative cells /
// constants and whose STRING cells are inline: one calloc per row and one strdup
// per string, nothing else per group.  nullptr: the plan or the data needs
// make_groups + build_groups.
cq_table* build_direct(const Compiled& C, const uint8_t* hp, uint32_t ng, uint32_t ncell, uint32_t SB,
                       const std::vector<int>& rep_ord, const Literals& L, uint64_t limit) {
    for (const OutCol& o : C.outs)
        if (o.kind != OUT_COUNT && o.kind != OUT_SUM && o.kind != OUT_AVG && o.kind != OUT_REP &&
            o.kind != OUT_CONST && o.kind != OUT_NULL)
            return nullptr;
    const int nacc = C.P.nacc;
    const size_t rec = 40 + 40 * (size_t)nacc;
    const Cell* cells = (const Cell*)(hp + (size_t)ng * rec);
    const uint8_t* bytes = (const uint8_t*)(cells + (size_t)ng * ncell);
    std::vector<int> rep_at(C.rep_cols.size(), -1);   // rep slot -> finish cell index
    for (size_t i = 0; i < rep_ord.size(); i++) rep_at[rep_ord[i]] = (int)i;
    for (uint32_t g = 0; g < ng; g++) {
        const unsigned long long first = ((const unsigned long long*)(hp + g * rec))[4];
        if (first != NOPOS && first >= limit) throw HipError{"scan kernel: group first-row offset out of range"};
        for (const OutCol& o : C.outs) {
            if (o.kind != OUT_REP || o.rep < 0 || o.rep >= (int)rep_at.size()) continue;
            const Cell& x = cells[(size_t)g * ncell + rep_at[o.rep]];
            if (x.kind == K_STR && x.len > SB) return nullptr;          // long text: fetched by make_groups
        }
    }
    PHASE("dcheck");
    cq_table* r = new_result(C.names);
    r->nrows = r->row_capacity = (int)ng;
    r->rows = (cq_row*)malloc(sizeof(cq_row) * std::max<size_t>(ng, 1));
    g_rowpool.hint = ng;
    for (uint32_t g = 0; g < ng; g++) {
        const uint8_t* rp = hp + g * rec;
        const unsigned long long cnt = ((const unsigned long long*)rp)[3];
        const uint64_t* q = (const uint64_t*)(rp + 40);
        cq_row& row = r->rows[g];
        row.ncols = r->ncols;
        row.values = rowpool_vals(r->ncols);
        for (int i = 0; i < r->ncols; i++) {
            const OutCol& o = C.outs[i];
            cq_value& v = row.values[i];
            v.kind = CQ_V_NULL;
            switch (o.kind) {
                case OUT_COUNT: v.kind = K_INT; v.u.i = (long long)cnt; break;
                case OUT_SUM: {
                    const unsigned long long num = q[5 * o.acc + 1];
                    v.kind = K_DBL;
                    v.u.f = num ? as_dbl(q[5 * o.acc]) : 0.0;
                    break;
                }
                case OUT_AVG: {
                    const unsigned long long num = q[5 * o.acc + 1];
                    v.kind = K_DBL;
                    v.u.f = num ? as_dbl(q[5 * o.acc]) / (double)num : 0.0;
                    break;
                }
                case OUT_REP:
                    if (cnt > 0 && o.rep >= 0 && o.rep < (int)rep_at.size()) {
                        const size_t k = (size_t)g * ncell + rep_at[o.rep];
                        const Cell& x = cells[k];
                        if (x.kind == K_STR) {             // to_value's strdup: up to the first NUL
                            const char* src = (const char*)bytes + k * SB;
                            const size_t n = strnlen(src, x.len);
                            char* d = rowpool_str(n + 1);
                            memcpy(d, src, n);
                            d[n] = 0;
                            v.kind = K_STR;
                            v.u.s = d;
                        } else {
                            HCell h;
                            h.kind = x.kind;
                            h.bits = x.bits;
                            v = to_value(h);
                        }
                    }
                    break;
                case OUT_CONST: if (cnt > 0) v = to_value(L.host[o.lit]); break;
                default: break;
            }
        }
    }
    return r;
}

// ------------------------------------------------------------------ host post-ops
// value_compare on result cells
int vcompare(const cq_value& a, const cq_value& b) {
    if (a.kind == CQ_V_NULL && b.kind == CQ_V_NULL) return 0;
    if (a.kind == CQ_V_NULL) return -1;
    if (b.kind == CQ_V_NULL) return 1;
    if (a.kind == CQ_V_DATE && b.kind == CQ_V_DATE) {
        if (a.u.date.y != b.u.date.y) return a.u.date.y - b.u.date.y;
        if (a.u.date.m != b.u.date.m) return a.u.date.m - b.u.date.m;
        return a.u.date.d - b.u.date.d;
    }
    bool an = a.kind == CQ_V_INT || a.kind == CQ_V_DOUBLE, bn = b.kind == CQ_V_INT || b.kind == CQ_V_DOUBLE;
    if (an && bn) {
        double x = a.kind == CQ_V_INT ? (double)a.u.i : a.u.f;
        double y = b.kind == CQ_V_INT ? (double)b.u.i : b.u.f;
        return x < y ? -1 : (x > y ? 1 : 0);
    }
    if (a.kind == CQ_V_STRING && b.kind == CQ_V_STRING) return strcmp(a.u.s, b.u.s);
    return 0;
}

// apply_having_filter (evaluator_aggregates.c:417-530); literal operands are
// parsed on the device like every other cell
struct Having {
    const cq_table* r;
    cq_node* sel;
    std::vector<std::pair<cq_node*, HCell>> lit;
    bool get(cq_node* e, int ri, cq_value& out) {
        memset(&out, 0, sizeof out);
        if (!e) return false;
        if (e->kind == CQ_N_LITERAL) {
            for (auto& p : lit)
                if (p.first == e) { out = to_value(p.second); return true; }
            return false;
        }
        if (e->kind == CQ_N_FUNCTION) {
            std::string fs = std::string(e->u.fn.name ? e->u.fn.name : "") + "(";
            for (int i = 0; i < e->u.fn.nargs; i++) {
                if (i > 0) fs += ", ";
                cq_node* a = e->u.fn.args[i];
                if (a && (a->kind == CQ_N_IDENTIFIER || a->kind == CQ_N_LITERAL)) fs += a->u.text;
            }
            fs += ")";
            if (fs.size() > 255) fs.resize(255);
            for (int c = 0; c < r->ncols; c++) {
                if (!strcasecmp(r->columns[c].name, fs.c_str()) ||
                    (sel && c < sel->u.sel.count && !strncasecmp(sel->u.sel.texts[c], fs.c_str(), fs.size()))) {
                    out = r->rows[ri].values[c];
                    if (out.kind == CQ_V_STRING) out.u.s = strdup(out.u.s);
                    return true;
                }
            }
        }
        if (e->kind == CQ_N_IDENTIFIER) {
            for (int c = 0; c < r->ncols; c++)
                if (!strcasecmp(r->columns[c].name, e->u.text)) {
                    out = r->rows[ri].values[c];
                    if (out.kind == CQ_V_STRING) out.u.s = strdup(out.u.s);
                    return true;
                }
        }
        return false;
    }
    bool cond(cq_node* n, int ri) {
        if (!n) return true;
        if (n->kind != CQ_N_CONDITION) return false;
        const char* op = n->u.bin.op ? n->u.bin.op : "";
        if (!strcasecmp(op, "AND")) return cond(n->u.bin.lhs, ri) && cond(n->u.bin.rhs, ri);
        if (!strcasecmp(op, "OR")) return cond(n->u.bin.lhs, ri) || cond(n->u.bin.rhs, ri);
        cq_value a, b;
        get(n->u.bin.lhs, ri, a);
        get(n->u.bin.rhs, ri, b);
        int c = vcompare(a, b);
        bool res = false;
        if (!strcmp(op, "=")) res = c == 0;
        else if (!strcmp(op, "!=") || !strcmp(op, "<>")) res = c != 0;
        else if (!strcmp(op, ">")) res = c > 0;
        else if (!strcmp(op, "<")) res = c < 0;
        else if (!strcmp(op, ">=")) res = c >= 0;
        else if (!strcmp(op, "<=")) res = c <= 0;
        if (a.kind == CQ_V_STRING) free(a.u.s);
        if (b.kind == CQ_V_STRING) free(b.u.s);
        return res;
    }
};

void collect_literals(cq_node* n, std::vector<cq_node*>& out) {
    if (!n) return;
    if (n->kind == CQ_N_LITERAL) { out.push_back(n); return; }
    if (n->kind == CQ_N_CONDITION || n->kind == CQ_N_BINARY_OP) {
        collect_literals(n->u.bin.lhs, out);
        collect_literals(n->u.bin.rhs, out);
    }
}

void apply_having(DevCtx& c, cq_table* r, cq_node* having, cq_node* sel) {
    if (!having || r->nrows == 0) return;
    Having H{r, sel, {}};
    std::vector<cq_node*> lits;
    collect_literals(having, lits);
    if (!lits.empty()) {
        std::vector<std::string> texts;
        for (auto* n : lits) texts.push_back(n->u.text ? n->u.text : "");
        Literals L;
        parse_literals(c, texts, L);
        std::vector<HCell> hc = L.host;
        for (size_t i = 0; i < lits.size(); i++) H.lit.emplace_back(lits[i], hc[i]);
    }
    int w = 0;
    for (int i = 0; i < r->nrows; i++) {
        if (H.cond(having, i)) r->rows[w++] = r->rows[i];
        else free_row(r->rows[i]);
    }
    r->nrows = w;
}

std::string norm_spec(const char* spec) {     // FUNC(col) / col with table prefixes stripped
    const char* par = strchr(spec, '(');
    if (par) {
        std::string fn(spec, (size_t)(par - spec));
        if (fn.size() > 63) fn.resize(63);
        const char* pc = strchr(par + 1, ')');
        if (!pc) return std::string();
        std::string arg(par + 1, (size_t)(pc - par - 1));
        if (arg.size() > 127) arg.resize(127);
        size_t dot = arg.find('.');
        return fn + "(" + (dot == std::string::npos ? arg : arg.substr(dot + 1)) + ")";
    }
    const char* dot = strchr(spec, '.');
    return std::string(dot ? dot + 1 : spec);
}

// sort_result (evaluator_utils.c:579-700); glibc qsort on these sizes is a stable merge sort
void sort_result(cq_table* r, cq_node* sel, const char* spec, bool desc) {
    if (!r || r->nrows == 0 || !spec) return;
    std::string look = norm_spec(spec);
    int ci = -1;
    for (int i = 0; i < r->ncols; i++)
        if (!strcasecmp(r->columns[i].name, look.c_str())) { ci = i; break; }
    if (ci < 0 && sel) {
        for (int i = 0; i < sel->u.sel.count; i++) {
            const char* cs = sel->u.sel.texts[i];
            const char* as = ci_find(cs, " AS ");
            std::string eb = as ? std::string(cs, (size_t)(as - cs)) : std::string(cs);
            if (eb.size() > 255) eb.resize(255);
            eb = rtrim(eb);
            if (!strcasecmp(norm_spec(eb.c_str()).c_str(), look.c_str())) { ci = i; break; }
        }
    }
    if (ci < 0) {
        fprintf(stderr, "warning: cannot sort by unknown column '%s' (looked for '%s')\n", spec, look.c_str());
        return;
    }
    std::stable_sort(r->rows, r->rows + r->nrows, [&](const cq_row& a, const cq_row& b) {
        if (ci >= a.ncols) return false;
        int cmp = vcompare(a.values[ci], b.values[ci]);
        return desc ? cmp > 0 : cmp < 0;
    });
}

void apply_distinct(cq_table* r) {            // apply_distinct (evaluator_utils.c:868-932)
    if (r->nrows <= 1) return;
    std::vector<char> keep(r->nrows, 0);
    for (int i = 0; i < r->nrows; i++) {
        bool dup = false;
        for (int j = 0; j < i && !dup; j++) {
            if (!keep[j]) continue;
            bool eq = true;
            for (int c = 0; c < r->ncols && eq; c++)
                if (vcompare(r->rows[i].values[c], r->rows[j].values[c]) != 0) eq = false;
            dup = eq;
        }
        keep[i] = !dup;
    }
    int w = 0;
    for (int i = 0; i < r->nrows; i++) {
        if (keep[i]) r->rows[w++] = r->rows[i];
        else free_row(r->rows[i]);
    }
    r->nrows = w;
}

void apply_limit(cq_table* r, int limit, int offset) {    // apply_limit_offset (:703-733)
    if (limit < 0 && offset < 0) return;
    int off = offset >= 0 ? offset : 0;
    int lim = limit >= 0 ? limit : r->nrows;
    if (off >= r->nrows) {
        for (int i = 0; i < r->nrows; i++) free_row(r->rows[i]);
        r->nrows = 0;
        return;
    }
    int cnt = lim;
    if (off + cnt > r->nrows) cnt = r->nrows - off;
    for (int i = 0; i < off; i++) free_row(r->rows[i]);
    for (int i = off + cnt; i < r->nrows; i++) free_row(r->rows[i]);
    if (off > 0 && cnt > 0) memmove(r->rows, r->rows + off, sizeof(cq_row) * (size_t)cnt);
    r->nrows = cnt;
}

void post_ops(DevCtx& c, cq_table* res, cq_node* q, bool rows = false, bool limited = false) {
    cq_node* sel = q->u.q.select;
    if (q->u.q.having && !rows) apply_having(c, res, q->u.q.having, sel);   // grouped paths only
    cq_node* ob = q->u.q.order_by;
    if (ob && ob->kind == CQ_N_ORDER_BY && ob->u.ord.key) sort_result(res, sel, ob->u.ord.key, ob->u.ord.desc);
    if (sel && sel->u.sel.distinct) apply_distinct(res);
    if (!limited) apply_limit(res, q->u.q.limit, q->u.q.offset);
}

// ------------------------------------------------------------------ row-returning SELECT
// projection of build_result (evaluator_utils.c:249-549): one program per output
// column; `*` expands to every table column (:263-295), other items evaluate their
// AST node with evaluate_expression (:345-371, :502-506)
struct RowPlan {
    std::vector<std::string> names;
    std::vector<int> cols;            // CSV columns parsed per record, ascending
    std::vector<Insn> code;           // OP_COL b = index into cols
    std::vector<uint32_t> off;        // program k = code[off[k], off[k+1])
    std::vector<std::string> lits;
};

std::string row_display_name(const char* cs) {
    const char* as = ci_find(cs, " AS ");
    if (as) return std::string(as + 4);                       // extract_column_alias (:57-63)
    if (strchr(cs, '(')) return std::string(cs);
    const char* dot = strchr(cs, '.');
    return std::string(dot ? dot + 1 : cs);
}

void compile_rows(const cqgpu_table* t, cq_node* q, Compiled& C, RowPlan& R) {
    memset(&C.P, 0, sizeof C.P);
    const char* alias = (q->u.q.from && q->u.q.from->u.from.alias) ? q->u.q.from->u.from.alias : "main";
    Compiler cc{t, q, alias, C};
    if (q->u.q.where) cc.cond(q->u.q.where);
    C.P.group_slot = -1;
    finish_plan(t, C, cc);
    cq_node* sel = q->u.q.select;
    R.off.push_back(0);
    if (!sel || sel->kind != CQ_N_SELECT) return;         // build_result: no SELECT -> no columns
    Compiled PC;
    Compiler pc{t, q, alias, PC};
    pc.need_cap = 32767;
    pc.lit_cap = 1 << 20;
    bool star = false;
    for (int i = 0; i < sel->u.sel.count; i++)
        if (sel->u.sel.texts[i] && !strcmp(sel->u.sel.texts[i], "*")) star = true;
    auto close = [&]() {
        R.code.insert(R.code.end(), pc.code.begin(), pc.code.end());
        R.off.push_back((uint32_t)R.code.size());
        pc.code.clear();
        pc.depth = 0;
    };
    for (int i = 0; i < sel->u.sel.count; i++) {
        const char* cs = sel->u.sel.texts[i] ? sel->u.sel.texts[i] : "";
        if (star && !strcmp(cs, "*")) {
            for (int j = 0; j < (int)t->names.size(); j++) {
                R.names.push_back(t->names[j]);
                pc.need(j);
                pc.emit(OP_COL, 0, j);
                close();
            }
            continue;
        }
        R.names.push_back(row_display_name(cs));
        cq_node* node = sel->u.sel.exprs ? sel->u.sel.exprs[i] : nullptr;
        if (node) {
            pc.expr(node);                                     // throws on subquery/window/function
        } else {
            // evaluate_column_expression (:194-246) on the spec text
            std::string cn = cs;
            const char* as = ci_find(cs, " AS ");
            if (as) cn.assign(cs, (size_t)(as - cs));
            if (cn.find('(') != std::string::npos) throw Ineligible{"scalar function in SELECT"};
            int col = col_index_fallback(t, cn.c_str());
            if (col >= 0) { pc.need(col); pc.emit(OP_COL, 0, col); }
            else pc.emit(OP_NULLV);
        }
        close();
    }
    // parse the referenced columns in one ascending pass; OP_COL b -> position
    R.cols = PC.need_cols;
    std::sort(R.cols.begin(), R.cols.end());
    for (auto& in : R.code)
        if (in.op == OP_COL)
            in.b = (uint16_t)(std::lower_bound(R.cols.begin(), R.cols.end(), (int)in.b) - R.cols.begin());
    R.lits = PC.lits;
}

// convert projected device cells of `n` rows into result rows [at, at + n)
void append_rows(DevCtx& c, cq_table* r, int at, const std::vector<Cell>& cells, int nout, int n) {
    std::vector<HCell> h = fetch_cells(c, cells);
    for (int i = 0; i < n; i++) {
        cq_row& row = r->rows[at + i];
        row.ncols = nout;
        row.values = (cq_value*)calloc(std::max(nout, 1), sizeof(cq_value));
        for (int k = 0; k < nout; k++) row.values[k] = to_value(h[(size_t)i * nout + k]);
    }
}

uint32_t all_records(DevCtx& c, const cqgpu_table* t, DevBuf& out);
struct JoinSide;
void load_side(DevCtx& c, const cqgpu_table* t, JoinSide& S);

// filter_rows (evaluator_utils.c:986-1006) for a WHERE over more than MAX_NEED
// columns: the byte offsets of the passing records, in file order, into `out`
unsigned long long wide_filter(DevCtx& c, const cqgpu_table* t, Compiled& C, DevBuf& out);

// keys: when given (a range partial, cqgpu_query_partial), the rank's rows are all
// kept in file order -- OFFSET is global, so only the first OFFSET+LIMIT rows of the
// shard can matter -- and each row's whole-file byte position is returned with it
cq_table* run_rows(DevCtx& c, const cqgpu_table* t, Compiled& C, RowPlan& R, cq_node* q, bool* limited,
                   std::vector<unsigned long long>* keys = nullptr) {
    const int nout = (int)R.names.size();
    *limited = false;
    // 1. scan: WHERE over every record, matching record offsets out (unordered)
    Literals L;
    ScanStats st;
    // test knobs: CQGPU_ROW_CAP0 (first-pass offset capacity), CQGPU_ROW_BATCH (projection batch)
    const char* cap_env = getenv("CQGPU_ROW_CAP0");
    unsigned long long cap = std::min<unsigned long long>(t->n / 2 + 2, 1ull << 24);
    if (cap_env && atoll(cap_env) > 0) cap = std::min<unsigned long long>(cap, (unsigned long long)atoll(cap_env));
    DevBuf rows(8), sorted(8);
    unsigned long long n = 0;
    if (C.wide) {
        // a WHERE over more than MAX_NEED columns: every record's needed cells, the
        // WHERE per record (join_filter over identity pairs), the passing records'
        // offsets compacted in file order -- no sort
        n = wide_filter(c, t, C, sorted);
    } else {
        DevBuf r0(cap * 8);
        std::swap(rows.p, r0.p);
        (void)run_aggregate(c, t, C, L, &st, rows.as<unsigned long long>(), cap);
        if (st.rows_emitted > cap) {          // exact count known now: rescan into a buffer that fits
            cap = st.rows_emitted;
            DevBuf bigger(cap * 8);
            std::swap(rows.p, bigger.p);
            (void)run_aggregate(c, t, C, L, &st, rows.as<unsigned long long>(), cap);
            if (st.rows_emitted != cap) throw HipError{"row scan: matching-row count changed between passes"};
        }
        n = st.rows_emitted;
        DevBuf s0(n * 8);
        std::swap(sorted.p, s0.p);
    }
    if (n > (unsigned long long)INT32_MAX) throw Ineligible{"more than 2^31-1 result rows"};
    g_stats.groups = n;
    // 2. file order: radix sort of the byte offsets
    if (C.wide) {
    } else if (n > 1) {
        int bits = 1;
        while (bits < 64 && (1ull << bits) <= t->n) bits++;
        size_t tb = 0;
        HIPCHECK(cq_sort_offsets(nullptr, &tb, rows.as<unsigned long long>(), sorted.as<unsigned long long>(), n,
                                 bits, c.stream));
        DevBuf temp(tb);
        HIPCHECK(cq_sort_offsets(temp.p, &tb, rows.as<unsigned long long>(), sorted.as<unsigned long long>(), n,
                                 bits, c.stream));
    } else if (n == 1) {
        HIPCHECK(hipMemcpyAsync(sorted.p, rows.p, 8, hipMemcpyDeviceToDevice, c.stream));
    }
    // LIMIT/OFFSET without ORDER BY or DISTINCT keeps a contiguous run of rows:
    // project only that run (apply_limit_offset, evaluator_utils.c:703-733)
    unsigned long long lo = 0, hi = n;
    cq_node* sel = q->u.q.select;
    cq_node* ob = q->u.q.order_by;
    const bool ordered = ob && ob->kind == CQ_N_ORDER_BY && ob->u.ord.key;
    const bool distinct = sel && sel->u.sel.distinct;
    if (!ordered && !distinct && (q->u.q.limit >= 0 || q->u.q.offset >= 0)) {
        const unsigned long long off = q->u.q.offset >= 0 ? (unsigned long long)q->u.q.offset : 0;
        const unsigned long long lim = q->u.q.limit >= 0 ? (unsigned long long)q->u.q.limit : n;
        if (keys) {
            hi = std::min(n, off + std::min(lim, n));
        } else {
            lo = std::min(off, n);
            hi = std::min(n, lo + lim);
            *limited = true;
        }
    }
    cq_table* r = new_result(R.names);
    const int nr = (int)(hi - lo);
    if (keys) {
        keys->resize(hi - lo);
        if (hi > lo) {
            HIPCHECK(hipMemcpyAsync(keys->data(), sorted.as<unsigned long long>() + lo, (hi - lo) * 8,
                                    hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
        }
        for (auto& k : *keys) k += t->base_offset;
    }
    r->nrows = r->row_capacity = nr;
    r->rows = (cq_row*)calloc(std::max(nr, 1), sizeof(cq_row));
    if (!nr || !nout) {
        for (int i = 0; i < nr; i++) { r->rows[i].ncols = nout; r->rows[i].values = (cq_value*)calloc(1, sizeof(cq_value)); }
        return r;
    }
    // 3. projection on the device, in batches
    Literals LP;
    parse_literals(c, R.lits, LP);
    const int ncols = (int)R.cols.size();
    std::vector<int16_t> cols16(R.cols.begin(), R.cols.end());
    DevBuf dcols(cols16.size() * 2), dcode(R.code.size() * sizeof(Insn)), doff(R.off.size() * 4);
    if (!cols16.empty())
        HIPCHECK(hipMemcpyAsync(dcols.p, cols16.data(), cols16.size() * 2, hipMemcpyHostToDevice, c.stream));
    if (!R.code.empty())
        HIPCHECK(hipMemcpyAsync(dcode.p, R.code.data(), R.code.size() * sizeof(Insn), hipMemcpyHostToDevice, c.stream));
    HIPCHECK(hipMemcpyAsync(doff.p, R.off.data(), R.off.size() * 4, hipMemcpyHostToDevice, c.stream));
    ProjDesc D;
    D.cols = dcols.as<int16_t>();
    D.code = dcode.as<Insn>();
    D.off = doff.as<uint32_t>();
    D.consts = LP.dcells;
    D.ncols = ncols;
    D.nout = nout;
    D.delim = (uint8_t)t->cfg.delimiter;
    D.quote = (uint8_t)t->cfg.quote;
    const size_t per = (size_t)(ncols + nout) * sizeof(Cell);
    int batch = (int)std::max<size_t>(1024, std::min<size_t>(1u << 20, (512u << 20) / per));
    const char* batch_env = getenv("CQGPU_ROW_BATCH");
    if (batch_env && atoi(batch_env) > 0) batch = std::min(batch, atoi(batch_env));
    DevBuf scratch((size_t)batch * std::max(ncols, 1) * sizeof(Cell)), dout((size_t)batch * nout * sizeof(Cell));
    std::vector<Cell> hcells;
    for (int b = 0; b < nr; b += batch) {
        const int m = std::min(batch, nr - b);
        HIPCHECK(cq_launch_project(t->g, sorted.as<unsigned long long>() + lo + b, (uint32_t)m, &D,
                                   scratch.as<Cell>(), dout.as<Cell>(), c.stream));
        hcells.resize((size_t)m * nout);
        HIPCHECK(hipMemcpyAsync(hcells.data(), dout.p, hcells.size() * sizeof(Cell), hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        append_rows(c, r, b, hcells, nout, m);
    }
    return r;
}

// STDDEV / MEDIAN (evaluate_aggregate, evaluator_aggregates.c:328-411): per passing
// row its group key words and the value as an order-preserving key (vla_prep /
// vla_pair_prep), sorted on the device by (key, value), reduced per group (scan.hip
// vla_* kernels), matched back to the aggregation's groups by key.
using VlaAt = std::map<std::tuple<uint64_t, uint64_t, uint64_t>, size_t>;
VlaAt vla_index(const Compiled& C, const std::vector<HGroup>& groups) {
    VlaAt at;                            // GK_LONG keys by content hash, as the kernels key them
    for (size_t g = 0; g < groups.size(); g++) {
        const HGroup& h = groups[g];
        const uint64_t cl = C.grouped ? ((uint64_t)h.kcls << 16 | h.klen) : ((uint64_t)GK_ALL << 16);
        const uint64_t w0 = !C.grouped || h.kcls == GK_LONG ? 0 : h.kw0;
        const uint64_t w1 = C.grouped ? h.kw1 : 0;
        at[std::make_tuple(cl, w0, w1)] = g;
    }
    return at;
}
struct VlaRows {                         // one row per candidate: key words, value key, numeric flag
    DevBuf kw0, kw1, kcl, vkey, flag;
    explicit VlaRows(size_t n) : kw0(n * 8), kw1(n * 8), kcl(n * 8), vkey(n * 8), flag(n * 4) {}
};
// sort + segment + reduce one value-list aggregate (index vi, kind 0 STDDEV / 1 MEDIAN)
void vla_finish(DevCtx& c, const VlaAt& at, bool grouped, std::vector<HGroup>& groups, size_t vi, int kind,
                VlaRows& V, uint32_t n, bool partial = false) {
    if (!n) return;
    const size_t N = n;
    DevBuf pos(N * 4), perm(N * 4), perm2(N * 4), keys(N * 8), keys2(N * 8), head(N * 4), sid(N * 4), start(N * 4),
        out(N * 32);
    uint32_t m = 0;
    {
        size_t tb = 0;
        HIPCHECK(cq_excl_sum_u32(nullptr, &tb, V.flag.as<unsigned int>(), pos.as<unsigned int>(), n, c.stream));
        DevBuf temp(tb);
        HIPCHECK(cq_excl_sum_u32(temp.p, &tb, V.flag.as<unsigned int>(), pos.as<unsigned int>(), n, c.stream));
        unsigned int last[2] = {0, 0};
        HIPCHECK(hipMemcpyAsync(&last[0], pos.as<unsigned int>() + n - 1, 4, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipMemcpyAsync(&last[1], V.flag.as<unsigned int>() + n - 1, 4, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        m = last[0] + last[1];
    }
    if (!m) return;                      // no numeric value anywhere: every group NULL
    HIPCHECK(cq_launch_vla_compact(V.flag.as<unsigned int>(), pos.as<unsigned int>(), n, perm.as<unsigned int>(),
                                   c.stream));
    // LSD: value, then the key words (stable sorts keep the value order inside a key)
    const unsigned long long* passes[4] = {V.vkey.as<unsigned long long>(), V.kcl.as<unsigned long long>(),
                                           V.kw1.as<unsigned long long>(), V.kw0.as<unsigned long long>()};
    for (int ps = 0; ps < 4; ps++) {
        if (ps > 0 && !grouped) break;
        HIPCHECK(cq_launch_vla_gather(passes[ps], perm.as<unsigned int>(), m, keys.as<unsigned long long>(), c.stream));
        size_t tb = 0;
        HIPCHECK(cq_sort_codes(nullptr, &tb, keys.as<unsigned long long>(), keys2.as<unsigned long long>(),
                               perm.as<unsigned int>(), perm2.as<unsigned int>(), m, c.stream));
        DevBuf temp(tb);
        HIPCHECK(cq_sort_codes(temp.p, &tb, keys.as<unsigned long long>(), keys2.as<unsigned long long>(),
                               perm.as<unsigned int>(), perm2.as<unsigned int>(), m, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        std::swap(perm.p, perm2.p);
    }
    HIPCHECK(cq_launch_vla_heads(V.kw0.as<unsigned long long>(), V.kw1.as<unsigned long long>(),
                                 V.kcl.as<unsigned long long>(), perm.as<unsigned int>(), m, head.as<unsigned int>(),
                                 c.stream));
    size_t tb = 0;
    HIPCHECK(cq_excl_sum_u32(nullptr, &tb, head.as<unsigned int>(), sid.as<unsigned int>(), m, c.stream));
    DevBuf temp(tb);
    HIPCHECK(cq_excl_sum_u32(temp.p, &tb, head.as<unsigned int>(), sid.as<unsigned int>(), m, c.stream));
    unsigned int last[2] = {0, 0};
    HIPCHECK(hipMemcpyAsync(&last[0], sid.as<unsigned int>() + m - 1, 4, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipMemcpyAsync(&last[1], head.as<unsigned int>() + m - 1, 4, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    const uint32_t nseg = last[0] + last[1];
    HIPCHECK(cq_launch_vla_starts(head.as<unsigned int>(), sid.as<unsigned int>(), m, start.as<unsigned int>(), c.stream));
    // a partial's MEDIAN keeps every value: the (key, value)-sorted value keys and the
    // segment starts come back, each group's run becomes its mvals
    const bool values = partial && kind == 1;
    const bool moments = partial && kind == 0;
    DevBuf aux(moments ? (size_t)nseg * 16 : 16);
    HIPCHECK(cq_launch_vla_reduce(V.vkey.as<unsigned long long>(), V.kw0.as<unsigned long long>(),
                                  V.kw1.as<unsigned long long>(), V.kcl.as<unsigned long long>(), perm.as<unsigned int>(),
                                  start.as<unsigned int>(), nseg, m, moments ? 2 : kind, out.as<unsigned long long>(),
                                  aux.as<double>(), c.stream));
    std::vector<unsigned long long> h((size_t)nseg * 4);
    std::vector<double> ha(moments ? (size_t)nseg * 2 : 0);
    std::vector<unsigned long long> hv(values ? m : 0);
    std::vector<unsigned int> hs(values ? nseg : 0);
    HIPCHECK(hipMemcpyAsync(h.data(), out.p, h.size() * 8, hipMemcpyDeviceToHost, c.stream));
    if (moments) HIPCHECK(hipMemcpyAsync(ha.data(), aux.p, ha.size() * 8, hipMemcpyDeviceToHost, c.stream));
    if (values) {
        HIPCHECK(cq_launch_vla_gather(V.vkey.as<unsigned long long>(), perm.as<unsigned int>(), m,
                                      keys.as<unsigned long long>(), c.stream));
        HIPCHECK(hipMemcpyAsync(hv.data(), keys.p, (size_t)m * 8, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipMemcpyAsync(hs.data(), start.p, (size_t)nseg * 4, hipMemcpyDeviceToHost, c.stream));
    }
    HIPCHECK(hipStreamSynchronize(c.stream));
    for (uint32_t sg = 0; sg < nseg; sg++) {
        auto it = at.find(std::make_tuple((uint64_t)h[4 * sg], (uint64_t)h[4 * sg + 1], (uint64_t)h[4 * sg + 2]));
        if (it == at.end()) continue;
        HGroup& g = groups[it->second];
        if (values) {
            const uint32_t e = sg + 1 < nseg ? hs[sg + 1] : m;
            if (g.mvals.size() <= vi) g.mvals.resize(vi + 1);
            g.mvals[vi].assign(hv.begin() + hs[sg], hv.begin() + e);
            g.vla_ok[vi] = true;
            continue;
        }
        if (moments) {
            g.vsum[vi] = as_dbl(h[4 * sg + 3]);
            g.vm2[vi] = ha[2 * sg];
            g.vn[vi] = ha[2 * sg + 1];
            g.vla_ok[vi] = true;
            continue;
        }
        g.vla[vi] = as_dbl(h[4 * sg + 3]);
        g.vla_ok[vi] = true;
    }
}

// single table, single-column (or no) GROUP BY: the WHERE-passing records' key and
// value cells from their byte offsets
void compute_vla(DevCtx& c, const cqgpu_table* t, const Compiled& C, std::vector<HGroup>& groups,
                 bool partial = false) {
    if (C.vla.empty() || groups.empty()) return;
    const cqgpu_stats saved = g_stats;
    Compiled W = C;                          // the WHERE alone, matching records out
    W.grouped = false;
    W.P.group_slot = -1;
    W.P.nacc = 0;
    W.rep_cols.clear();
    W.vla.clear();
    Literals L;
    ScanStats st;
    const unsigned long long cap = t->n / 2 + 2;
    DevBuf rows(cap * 8);
    (void)run_aggregate(c, t, W, L, &st, rows.as<unsigned long long>(), cap);
    const unsigned long long n64 = st.rows_emitted;
    g_stats = saved;
    if (n64 > cap) throw HipError{"STDDEV/MEDIAN: record count exceeds the offset buffer"};
    if (n64 >= (1ull << 31)) throw Ineligible{"STDDEV/MEDIAN over more than 2^31 rows"};
    const uint32_t n = (uint32_t)n64;
    std::vector<int> cols;
    if (C.grouped) cols.push_back(C.group_col);
    for (auto& v : C.vla) cols.push_back(v.second);
    std::sort(cols.begin(), cols.end());
    cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
    ColsDesc D;
    memset(&D, 0, sizeof D);
    D.ncols = (int)cols.size();
    for (int k = 0; k < D.ncols; k++) D.cols[k] = (int16_t)cols[k];
    D.delim = (uint8_t)t->cfg.delimiter;
    D.quote = (uint8_t)t->cfg.quote;
    auto slot = [&](int col) { return (int)(std::find(cols.begin(), cols.end(), col) - cols.begin()); };
    DevBuf cells((size_t)std::max<uint32_t>(n, 1) * D.ncols * sizeof(Cell));
    HIPCHECK(cq_launch_cells(t->g, t->n, rows.as<unsigned long long>(), n, &D, cells.as<Cell>(), c.stream));
    const VlaAt at = vla_index(C, groups);
    VlaRows V(std::max<uint32_t>(n, 1));
    for (size_t vi = 0; vi < C.vla.size(); vi++) {
        HIPCHECK(cq_launch_vla_prep(cells.as<Cell>(), n, (uint32_t)D.ncols, C.grouped ? slot(C.group_col) : -1,
                                    (uint32_t)slot(C.vla[vi].second), V.kw0.as<unsigned long long>(),
                                    V.kw1.as<unsigned long long>(), V.kcl.as<unsigned long long>(),
                                    V.vkey.as<unsigned long long>(), V.flag.as<unsigned int>(), c.stream));
        vla_finish(c, at, C.grouped, groups, vi, C.vla[vi].first, V, n, partial);
    }
}

// over (l, r) pairs of parsed cells (joins; composite / expression keys over identity
// pairs): MA the plan's need slots, VM[vi] the value column of C.vla[vi]
void compute_vla_pairs(DevCtx& c, const Compiled& C, const JoinMap& MA, const std::vector<JoinMap>& VM,
                       const uint2* pairs, unsigned long long np, const Cell* Lc, const Cell* Rc,
                       std::vector<HGroup>& groups, bool partial = false) {
    if (C.vla.empty() || groups.empty()) return;
    if (np >= (1ull << 31)) throw Ineligible{"STDDEV/MEDIAN over more than 2^31 rows"};
    const uint32_t n = (uint32_t)np;
    const VlaAt at = vla_index(C, groups);
    VlaRows V(std::max<uint32_t>(n, 1));
    for (size_t vi = 0; vi < C.vla.size(); vi++) {
        HIPCHECK(cq_launch_vla_pair_prep(pairs, n, &MA, &VM[vi], Lc, Rc, &C.P, C.grouped ? 1 : 0,
                                         V.kw0.as<unsigned long long>(), V.kw1.as<unsigned long long>(),
                                         V.kcl.as<unsigned long long>(), V.vkey.as<unsigned long long>(),
                                         V.flag.as<unsigned int>(), c.stream));
        vla_finish(c, at, C.grouped, groups, vi, C.vla[vi].first, V, n, partial);
    }
}

void check_plan_shape(cq_node* q, const cqgpu_table* t, bool join_ok);
bool is_row_query(cq_node* q);

// ------------------------------------------------------------------ INNER JOIN
// process_joins + perform_join (reference evaluator_joins.c:237-274, :63-181) for
// one INNER JOIN with an `ident = ident` ON: both sides' needed columns parsed on
// the device, the right side sorted by key code, (l, r) pairs in nested-loop
// order, then WHERE / GROUP BY / aggregates or the projection over the pairs.

// every data record of t, file order (csv_load's rows)
uint32_t all_records(DevCtx& c, const cqgpu_table* t, DevBuf& out) {
    // record starts in file order (route.hip rs_*: count, scan, write; no atomics)
    const uint32_t nb = cq_rs_blocks(t->n);
    DevBuf counts((size_t)nb * 8), base((size_t)nb * 8);
    HIPCHECK(cq_launch_rs_count(t->g, t->data_begin, t->n, counts.as<unsigned long long>(), c.stream));
    size_t tb = 0;
    HIPCHECK(cq_excl_sum_u64(nullptr, &tb, counts.as<unsigned long long>(), base.as<unsigned long long>(), nb, c.stream));
    DevBuf temp(tb);
    HIPCHECK(cq_excl_sum_u64(temp.p, &tb, counts.as<unsigned long long>(), base.as<unsigned long long>(), nb, c.stream));
    unsigned long long last[2] = {0, 0};
    HIPCHECK(hipMemcpyAsync(&last[0], base.as<unsigned long long>() + nb - 1, 8, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipMemcpyAsync(&last[1], counts.as<unsigned long long>() + nb - 1, 8, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    const unsigned long long n = last[0] + last[1];
    if (n >= (1ull << 32)) throw Ineligible{"join side over 2^32 rows"};
    DevBuf recs(std::max<unsigned long long>(n, 1) * 8);
    HIPCHECK(cq_launch_rs_write(t->g, t->data_begin, t->n, base.as<unsigned long long>(), recs.as<unsigned long long>(),
                                c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    std::swap(out.p, recs.p);
    return (uint32_t)n;
}

// record starts through the general scan path (kept for cqgpu_debug_all_records'
// cross-check against the two-pass kernels)
uint32_t all_records_scan(DevCtx& c, const cqgpu_table* t, DevBuf& out) {
    Compiled C;
    memset(&C.P, 0, sizeof C.P);
    C.P.group_slot = -1;
    C.P.delim = (uint8_t)t->cfg.delimiter;
    C.P.quote = (uint8_t)t->cfg.quote;
    C.P.n = t->n;
    C.P.data_begin = t->data_begin;
    C.P.range_end = t->n;
    Literals L;
    ScanStats st;
    unsigned long long cap = std::max<unsigned long long>(t->n / 2 + 2, 16);
    DevBuf rows(cap * 8);
    (void)run_aggregate(c, t, C, L, &st, rows.as<unsigned long long>(), cap);
    const unsigned long long n = st.rows_emitted;
    if (n > cap) throw HipError{"join: record count exceeds the offset buffer"};
    if (n >= (1ull << 32)) throw Ineligible{"join side over 2^32 rows"};
    DevBuf sorted(n * 8);
    if (n > 1) {
        int bits = 1;
        while (bits < 64 && (1ull << bits) <= t->n) bits++;
        size_t tb = 0;
        HIPCHECK(cq_sort_offsets(nullptr, &tb, rows.as<unsigned long long>(), sorted.as<unsigned long long>(), n, bits,
                                 c.stream));
        DevBuf temp(tb);
        HIPCHECK(cq_sort_offsets(temp.p, &tb, rows.as<unsigned long long>(), sorted.as<unsigned long long>(), n, bits,
                                 c.stream));
    } else if (n == 1) {
        HIPCHECK(hipMemcpyAsync(sorted.p, rows.p, 8, hipMemcpyDeviceToDevice, c.stream));
    }
    std::swap(out.p, sorted.p);
    return (uint32_t)n;
}

// join_match's column lookup (evaluator_joins.c:40-60 via resolve_column): the
// name is looked up in its own side's table, else by alias in either table --
// and the value is then read from its own side's row at that index
int join_on_index(const char* name, const cqgpu_table* own, const cqgpu_table* L, const char* la,
                  const cqgpu_table* R, const char* ra) {
    if (!name) return -1;
    int idx = col_index(own, name);
    if (idx >= 0) return idx;
    const char* dot = strchr(name, '.');
    if (!dot) return -1;
    std::string al(name, (size_t)(dot - name));
    if (!strcasecmp(la, al.c_str())) return col_index(L, dot + 1);
    if (!strcasecmp(ra, al.c_str())) return col_index(R, dot + 1);
    return -1;
}

struct JoinSide {
    DevBuf recs, cells;
    uint32_t n = 0;
    std::vector<int> cols;            // CSV columns parsed, ascending
    int slot(int col) const { return (int)(std::find(cols.begin(), cols.end(), col) - cols.begin()); }
};

void load_side(DevCtx& c, const cqgpu_table* t, JoinSide& S) {
    std::sort(S.cols.begin(), S.cols.end());
    S.cols.erase(std::unique(S.cols.begin(), S.cols.end()), S.cols.end());
    if ((int)S.cols.size() > MAX_WIDE) throw Ineligible{"join: more than " + std::to_string(MAX_WIDE) + " columns of one side"};
    S.n = all_records(c, t, S.recs);
    ColsDesc D;
    memset(&D, 0, sizeof D);
    D.ncols = (int)S.cols.size();
    for (int k = 0; k < D.ncols; k++) D.cols[k] = (int16_t)S.cols[k];
    D.delim = (uint8_t)t->cfg.delimiter;
    D.quote = (uint8_t)t->cfg.quote;
    DevBuf cells((size_t)std::max<uint32_t>(S.n, 1) * std::max(D.ncols, 1) * sizeof(Cell));
    std::swap(S.cells.p, cells.p);
    HIPCHECK(cq_launch_cells(t->g, t->n, S.recs.as<unsigned long long>(), S.n, &D, S.cells.as<Cell>(), c.stream));
}

// joined column -> (side, cell index)
JoinMap join_map(const std::vector<int>& jcols, int nl, const JoinSide& A, const JoinSide& B) {
    JoinMap M;
    memset(&M, 0, sizeof M);
    if ((int)jcols.size() > MAX_WIDE) throw Ineligible{"join: more than " + std::to_string(MAX_WIDE) + " joined columns"};
    M.n = (int)jcols.size();
    for (int k = 0; k < M.n; k++) {
        const int j = jcols[k];
        M.side[k] = j < nl ? 0 : 1;
        M.col[k] = (int16_t)(j < nl ? A.slot(j) : B.slot(j - nl));
    }
    M.lstride = (uint32_t)std::max<size_t>(A.cols.size(), 1);
    M.rstride = (uint32_t)std::max<size_t>(B.cols.size(), 1);
    return M;
}

// JoinPartial::lmask bit: the partial's sides were routed with the minority key
// classes replicated (cqgpu_route_plan2), so cross-class pairs need no refusal
constexpr uint32_t REP_ROUTED = 0x10u;

// per-rank state of a repartitioned join (cqgpu_query_partial over routed tables)
struct JoinPartial {
    std::vector<std::string> names;   // joined schema (alias.col)
    std::vector<HGroup> groups;       // first / extpos: (global left id << 32) | global right id
    uint32_t acc_classes[MAX_ACC] = {};
    uint32_t lmask = 0, rmask = 0;    // bit k: a key of value class k (1 number, 2 string, 3 date)
    // row-returning joins: the projected rows of the passing pairs, in local pair
    // order, with their global order keys ((global left id << 32) | global right id)
    cq_table* rows = nullptr;
    std::vector<unsigned long long> row_keys;
    // the joined plan's shape (run_join's compile): accumulators, representative
    // cells, STDDEV / MEDIAN states -- the blob's header, without a second compile
    int nacc = -1;
    uint32_t nrep = 0, nvla = 0;
    // the fused join's groups serialised straight from the packed result (no HGroup
    // objects): `ng` records in the blob's group format, `first_at[i]` the byte offset
    // of group i's first-pair key (patched to its global id by run_fast_join)
    bool direct = false;
    uint64_t ng = 0;
    std::vector<uint8_t> gblob;
    std::vector<size_t> first_at;
    // cqgpu_join_outer_matched: run the chain up to this level, keep its right side's
    // locally matched records (one byte each) and stop
    int probe_level = -1;
    std::vector<uint8_t> probe_out;
    ~JoinPartial() { if (rows) cqgpu_result_free(rows); }
};

// A chain's later RIGHT / FULL level across partials (perform_join's unmatched right
// rows, evaluator_joins.c:143-171, chained through process_joins :268-270): the
// level's table is whole on every rank, and its unmatched records are the ones no
// rank's joined rows matched.  Per level: the OR over the ranks of their matched
// flags (cqgpu_join_outer_set), and whether this rank's partial carries the
// unmatched records (exactly one rank does).
struct OuterSet {
    std::vector<uint8_t> matched;
    bool emit = false;
};
std::map<int, OuterSet> g_outer_sets;

// global record ids of a join side: the routed ids, or the local row index
void side_gids(DevCtx& c, const cqgpu_table* t, uint32_t n, DevBuf& own, const unsigned long long** out) {
    if (t->gids) {
        if (t->ngids != n) throw HipError{"routed table: record count differs from its ids"};
        *out = t->gids;
        return;
    }
    DevBuf b((size_t)std::max<uint32_t>(n, 1) * 8);
    std::swap(own.p, b.p);
    HIPCHECK(cq_launch_iota_u64(n, own.as<unsigned long long>(), c.stream));
    *out = own.as<unsigned long long>();
}

// WHERE + GROUP BY + aggregates over (l, r) pairs of parsed cells (join_agg_kernel),
// then compaction and the representative cells of each group's first pair
// (join_finish_kernel): groups in first-pair order, `first` / `extpos` = pair indexes
std::vector<HGroup> aggregate_pairs(DevCtx& c, Compiled& C, const JoinMap& MA, const JoinMap& MR, const uint2* pairs,
                                    unsigned long long np, const Cell* Lc, const Cell* Rc, ScanStats& st,
                                    bool all_splits = false) {
    const int grouped = C.grouped ? 1 : 0;
    constexpr uint32_t SB = 48;
    const uint32_t ncell = (uint32_t)MR.n + (uint32_t)C.P.nacc + 1;
    uint32_t cap = grouped ? 8192 : 64;
    std::vector<GroupOut> outs;
    std::vector<Cell> fcells;
    std::vector<uint8_t> fbytes;
    while (true) {
        TableArena Ar = make_arena(c, C.P, cap, cap / 2 + 1, 1, cq_scan_cand_stride(&C.P, grouped));
        const unsigned int cap_out = cap / 2 + 1;
        Scratch fin(c, (size_t)cap_out * ncell * (sizeof(Cell) + SB) + 64);
        Cell* dcells = (Cell*)fin.p;
        uint8_t* dbytes = fin.p + (size_t)cap_out * ncell * sizeof(Cell);
        bool sums_only = grouped && !getenv("CQ_AMD_NO_JOIN_PREAGG");
        for (int a = 0; a < C.P.nacc; a++) sums_only = sums_only && C.P.acc[a].kind == ACC_SUM;
        HIPCHECK(hipEventRecord(c.ev0, c.stream));
        if (sums_only)   // COUNT / SUM / AVG by group: block-local LDS pre-aggregation
            HIPCHECK(cq_launch_join_sum(pairs, np, &MA, Lc, Rc, &C.P, &Ar.gt, Ar.stats, c.ncu, c.stream));
        else
            HIPCHECK(cq_launch_join_agg(pairs, np, &MA, Lc, Rc, &C.P, &Ar.gt, Ar.stats, grouped, c.stream));
        HIPCHECK(hipEventRecord(c.ev1, c.stream));
        // composite keys: every pair's parts against its group's first pair's parts
        const bool verify = grouped && C.P.ngpart > 1;
        DevBuf vbad(64);
        if (verify) {
            HIPCHECK(hipMemsetAsync(vbad.p, 0, 4, c.stream));
            HIPCHECK(cq_launch_comp_verify(pairs, np, &MA, Lc, Rc, &C.P, &Ar.gt, vbad.as<unsigned int>(), c.stream));
        }
        HIPCHECK(cq_launch_compact(&Ar.gt, &C.P, Ar.out, Ar.out_count, cap_out, c.stream, nullptr));
        HIPCHECK(cq_launch_join_finish(Ar.out, Ar.out_count, cap_out, pairs, &MR, Lc, Rc, C.P.nacc, SB, dcells, dbytes,
                                       c.stream));
        unsigned int ng = 0, bad = 0;
        HIPCHECK(hipMemcpyAsync(&ng, Ar.out_count, 4, hipMemcpyDeviceToHost, c.stream));
        if (verify) HIPCHECK(hipMemcpyAsync(&bad, vbad.p, 4, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipMemcpyAsync(&st, Ar.stats, sizeof st, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        float ms = 0;
        HIPCHECK(hipEventElapsedTime(&ms, c.ev0, c.ev1));
        g_stats.scan_ms = ms;
        if (st.overflow >= 2) throw HipError{"join aggregate: lock / insert timeout"};
        if (st.overflow) {
            if (cap >= (1u << 30)) throw HipError{"group table overflow"};
            cap *= 8;
            continue;
        }
        if (bad) throw HipError{"composite GROUP BY: two different part lists share a 128-bit key digest"};
        ng = std::min(ng, cap_out);
        outs.resize(ng);
        fcells.resize((size_t)ng * ncell);
        fbytes.resize((size_t)ng * ncell * SB);
        if (ng) {
            HIPCHECK(hipMemcpyAsync(outs.data(), Ar.out, ng * sizeof(GroupOut), hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipMemcpyAsync(fcells.data(), dcells, fcells.size() * sizeof(Cell), hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipMemcpyAsync(fbytes.data(), dbytes, fbytes.size(), hipMemcpyDeviceToHost, c.stream));
        }
        HIPCHECK(hipStreamSynchronize(c.stream));
        PHASE("copies");
        break;
    }
    g_stats.passed = st.passed;
    if (st.key_flags & 2u) throw HipError{"internal: a composite key part the joined text could not render"};
    std::vector<int> rep_ord(C.rep_cols.size());
    for (size_t i = 0; i < rep_ord.size(); i++) rep_ord[i] = (int)i;
    std::vector<HGroup> groups =
        make_groups(c, C, std::max<unsigned long long>(np, 1), 0, outs, fcells, fbytes, MR.n, rep_ord, SB);
    // MIN/MAX over cells of several value classes (evaluator_aggregates.c:311-326):
    // a row-order fold under value_compare, where cells of different classes compare
    // "equal", so the result keeps the class of the group's first non-NULL cell and
    // is the first occurrence of that class's extreme.  One more pass per such
    // accumulator computes, per class, the extreme (with its first position) and the
    // first position of any cell of the class; groups come out in the same order.
    // all_splits (a join partial): also for one class, since another rank may hold
    // cells of another class and the merge then needs this rank's first position of
    // each class, not its extreme's
    for (int a = 0; a < C.P.nacc; a++) {
        if (C.P.acc[a].kind == ACC_SUM || C.P.acc[a].cls) continue;   // (a class-split pass itself)
        const unsigned m = st.acc_classes[a];
        if (!m || (!all_splits && !(m & (m - 1)))) continue;
        Compiled C2 = C;
        C2.P.nacc = 6;
        for (int k = 0; k < 3; k++) {
            AccSpec& e = C2.P.acc[k];
            e.kind = C.P.acc[a].kind; e.slot = C.P.acc[a].slot; e.cls = (uint8_t)(1u << k); e.pos_only = 0;
            AccSpec& f = C2.P.acc[3 + k];
            f.kind = ACC_MIN; f.slot = C.P.acc[a].slot; f.cls = (uint8_t)(1u << k); f.pos_only = 1;
        }
        ScanStats st2;
        const std::vector<HGroup> split = aggregate_pairs(c, C2, MA, MR, pairs, np, Lc, Rc, st2);
        if (split.size() != groups.size()) throw HipError{"mixed MIN/MAX: class-split pass disagrees on the groups"};
        for (size_t g = 0; g < groups.size(); g++) {
            int best = -1;
            for (int k = 0; k < 3; k++)
                if (split[g].extpos[3 + k] != NOPOS && (best < 0 || split[g].extpos[3 + k] < split[g].extpos[3 + best]))
                    best = k;
            groups[g].ext[a] = best >= 0 ? split[g].ext[best] : HCell();
            groups[g].extpos[a] = best >= 0 ? split[g].extpos[best] : NOPOS;
            HGroup::ClassSplit cs;
            cs.acc = a;
            for (int k = 0; k < 3; k++) {
                cs.ext[k] = split[g].ext[k];
                cs.extpos[k] = split[g].extpos[k];
                cs.first[k] = split[g].extpos[3 + k];
            }
            groups[g].split.push_back(cs);
        }
    }
    return groups;
}

// key value classes present in a side's key column (bit k: class k, 1 number,
// 2 string, 3 date): a repartitioned join's ranks report them so the merge can
// refuse cross-class keys, which value_compare calls "equal" (csv_reader.c:128)
uint32_t key_class_mask(DevCtx& c, const JoinSide& S, int kcol) {
    if (!S.n) return 0;
    const uint32_t stride = (uint32_t)S.cols.size(), k = (uint32_t)S.slot(kcol);
    DevBuf dm(64);
    HIPCHECK(hipMemsetAsync(dm.p, 0, 4, c.stream));
    HIPCHECK(cq_launch_class_mask(S.cells.as<Cell>(), stride, k, S.n, dm.as<unsigned int>(), c.stream));
    unsigned int m = 0;
    HIPCHECK(hipMemcpyAsync(&m, dm.p, 4, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    return m & 0xEu;                                   // classes 1-3 (NULL keys match only NULL)
}

// (l, r) pairs of one join level in the nested loop's order (perform_join,
// evaluator_joins.c:63-181): left rows ascending, each with its matching right
// rows ascending; LEFT / FULL put an unmatched left row (l, -) in its place,
// RIGHT / FULL append the unmatched right rows (-, r) in row order.  kl / kr:
// the ON operands' columns of A / B (keyed: both resolved).
// gset (device, one byte per right record; with outer_right): the records some rank
// matched -- the unmatched rows appended are the others, and only when gemit;
// matched_out (device, with outer_right): this call's matched flags of the right side
unsigned long long build_pairs(DevCtx& c, JoinSide& A, JoinSide& B, int kl, int kr, bool keyed, bool outer_left,
                               bool outer_right, DevBuf& pairs, bool cross = false, const uint8_t* gset = nullptr,
                               bool gemit = true, uint8_t* matched_out = nullptr) {
    unsigned long long np = 0;
    const bool global_right = outer_right && (gset || matched_out);
    if (cross && A.n && B.n) {
        // JOIN without ON: evaluate_join_condition is true for a NULL condition
        // (evaluator_joins.c:42), so every (l, r) pair matches, in the nested loops'
        // order, and no row of either side is unmatched
        np = (unsigned long long)A.n * B.n;
        if (np >= (1ull << 31)) throw Ineligible{"JOIN without ON: a cross product of 2^31 or more pairs"};
        DevBuf pb(np * 8);
        std::swap(pairs.p, pb.p);
        HIPCHECK(cq_launch_join_cross(A.n, B.n, pairs.as<uint2>(), c.stream));
        if (matched_out) HIPCHECK(hipMemsetAsync(matched_out, 1, B.n, c.stream));
        return np;
    }
    if (keyed && A.n && B.n) {
        const uint32_t ls = (uint32_t)A.cols.size(), rs = (uint32_t)B.cols.size();
        const uint32_t lk = (uint32_t)A.slot(kl), rk = (uint32_t)B.slot(kr);
        // right side: codes and classes; rows grouped by class (the cross-class
        // streams); the hash table of distinct keys and the rows sorted by key slot
        DevBuf rcodes((size_t)B.n * 8), rcls((size_t)B.n * 4), ridx((size_t)B.n * 4), ridx_c, pc(64);
        HIPCHECK(hipMemsetAsync(pc.p, 0, 64, c.stream));
        HIPCHECK(cq_launch_join_code(B.cells.as<Cell>(), rs, rk, B.n, rcodes.as<unsigned long long>(),
                                     rcls.as<uint32_t>(), ridx.as<uint32_t>(), pc.as<unsigned int>(), c.stream));
        unsigned int per[4] = {0, 0, 0, 0};
        HIPCHECK(hipMemcpyAsync(per, pc.p, 16, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        // rows grouped by class, row order within a class: with one class present that
        // is the identity ridx (join_code's idx), so the class sort runs only for mixes
        const int nclass = (per[0] != 0) + (per[1] != 0) + (per[2] != 0) + (per[3] != 0);
        if (nclass > 1) {
            DevBuf ccls((size_t)B.n * 4), rc((size_t)B.n * 4);
            size_t tb = 0;
            HIPCHECK(cq_sort_classes(nullptr, &tb, rcls.as<unsigned int>(), ccls.as<unsigned int>(),
                                     ridx.as<unsigned int>(), rc.as<unsigned int>(), B.n, c.stream));
            DevBuf temp(tb);
            HIPCHECK(cq_sort_classes(temp.p, &tb, rcls.as<unsigned int>(), ccls.as<unsigned int>(),
                                     ridx.as<unsigned int>(), rc.as<unsigned int>(), B.n, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));   // (temp / ccls freed on scope exit)
            std::swap(ridx_c.p, rc.p);
        }
        const uint32_t* ridx_cp = nclass > 1 ? ridx_c.as<uint32_t>() : ridx.as<uint32_t>();
        int hbits = 6;
        while (hbits < 31 && (1ull << hbits) < 2ull * B.n) hbits++;
        const uint32_t cap = 1u << hbits;
        DevBuf hslot((size_t)cap * sizeof(HSlot)), sid((size_t)B.n * 4), ssid((size_t)B.n * 4), sidx((size_t)B.n * 4);
        HIPCHECK(hipMemsetAsync(hslot.p, 0, (size_t)cap * sizeof(HSlot), c.stream));
        JoinHashW HW;
        HW.slot = hslot.as<HSlot>();
        HW.cap = cap;
        unsigned long long* dovf = (unsigned long long*)((uint8_t*)pc.p + 32);
        HIPCHECK(hipMemsetAsync(dovf, 0, 8, c.stream));
        HIPCHECK(cq_launch_hash_build(rcodes.as<unsigned long long>(), rcls.as<uint32_t>(), B.n, &HW, sid.as<uint32_t>(),
                                      dovf, c.stream));
        size_t tbr = 0;
        HIPCHECK(cq_sort_u32(nullptr, &tbr, sid.as<unsigned int>(), ssid.as<unsigned int>(), ridx.as<unsigned int>(),
                             sidx.as<unsigned int>(), B.n, hbits, c.stream));
        DevBuf temp1(tbr);
        HIPCHECK(cq_sort_u32(temp1.p, &tbr, sid.as<unsigned int>(), ssid.as<unsigned int>(), ridx.as<unsigned int>(),
                             sidx.as<unsigned int>(), B.n, hbits, c.stream));
        HIPCHECK(cq_launch_run_bounds(ssid.as<uint32_t>(), B.n, hslot.as<HSlot>(), c.stream));
        unsigned long long ovf = 0;
        HIPCHECK(hipMemcpyAsync(&ovf, dovf, 8, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        if (ovf) throw HipError{"join hash build: table full or insert timeout"};
        JoinRight JR;
        memset(&JR, 0, sizeof JR);
        JR.seg[0] = 0;
        for (int k = 0; k < 4; k++) JR.seg[k + 1] = JR.seg[k] + per[k];
        JR.hslot = hslot.as<HSlot>();
        JR.hcap = cap;
        JR.sidx = sidx.as<uint32_t>();
        JR.ridx_c = ridx_cp;
        JR.cells = B.cells.as<Cell>();
        JR.stride = rs;
        JR.kcol = rk;
        DevBuf lo((size_t)A.n * 4), cnt((size_t)A.n * 8), offs((size_t)A.n * 8);
        HIPCHECK(cq_launch_join_count(A.cells.as<Cell>(), ls, lk, A.n, &JR, outer_left ? 1 : 0, lo.as<uint32_t>(),
                                      cnt.as<unsigned long long>(), c.stream));
        size_t tb2 = 0;
        HIPCHECK(cq_excl_sum_u64(nullptr, &tb2, cnt.as<unsigned long long>(), offs.as<unsigned long long>(), A.n,
                                 c.stream));
        DevBuf temp2(tb2);
        HIPCHECK(cq_excl_sum_u64(temp2.p, &tb2, cnt.as<unsigned long long>(), offs.as<unsigned long long>(), A.n,
                                 c.stream));
        unsigned long long last[2] = {0, 0};
        HIPCHECK(hipMemcpyAsync(&last[0], offs.as<unsigned long long>() + A.n - 1, 8, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipMemcpyAsync(&last[1], cnt.as<unsigned long long>() + A.n - 1, 8, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        const unsigned long long nleft = last[0] + last[1];
        // RIGHT / FULL: right rows no left row matched, appended in row order
        DevBuf unm(outer_right ? (size_t)B.n * 4 : 4), upos(outer_right ? (size_t)B.n * 4 : 4);
        if (outer_right) HIPCHECK(hipMemsetD32Async((hipDeviceptr_t)unm.p, 1u, B.n, c.stream));
        DevBuf pb((nleft + (outer_right ? B.n : 0)) * 8);
        std::swap(pairs.p, pb.p);
        HIPCHECK(cq_launch_join_emit(A.cells.as<Cell>(), ls, lk, A.n, &JR, lo.as<uint32_t>(),
                                     cnt.as<unsigned long long>(), offs.as<unsigned long long>(), pairs.as<uint2>(),
                                     outer_right ? unm.as<unsigned int>() : nullptr, c.stream));
        np = nleft;
        if (global_right)
            HIPCHECK(cq_launch_outer_global(unm.as<unsigned int>(), B.n, gset, gemit ? 1u : 0u, matched_out, c.stream));
        if (outer_right) {
            size_t tb3 = 0;
            HIPCHECK(cq_excl_sum_u32(nullptr, &tb3, unm.as<unsigned int>(), upos.as<unsigned int>(), B.n, c.stream));
            DevBuf temp3(tb3);
            HIPCHECK(cq_excl_sum_u32(temp3.p, &tb3, unm.as<unsigned int>(), upos.as<unsigned int>(), B.n, c.stream));
            unsigned int ul[2] = {0, 0};
            HIPCHECK(hipMemcpyAsync(&ul[0], upos.as<unsigned int>() + B.n - 1, 4, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipMemcpyAsync(&ul[1], unm.as<unsigned int>() + B.n - 1, 4, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(cq_launch_join_fill(unm.as<unsigned int>(), upos.as<unsigned int>(), B.n, nleft, 1,
                                         pairs.as<uint2>(), c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
            np += (unsigned long long)ul[0] + ul[1];
        }
        HIPCHECK(hipStreamSynchronize(c.stream));        // before the scratch buffers of this block are freed
    }
    else if (global_right && B.n) {
        // nothing matches on this rank: the left rows (LEFT / FULL) NULL-padded, then
        // the right records no rank matched (on the emitting rank)
        const unsigned long long nl2 = outer_left ? A.n : 0;
        DevBuf unm((size_t)B.n * 4), upos((size_t)B.n * 4);
        HIPCHECK(hipMemsetD32Async((hipDeviceptr_t)unm.p, 1u, B.n, c.stream));
        HIPCHECK(cq_launch_outer_global(unm.as<unsigned int>(), B.n, gset, gemit ? 1u : 0u, matched_out, c.stream));
        size_t tb3 = 0;
        HIPCHECK(cq_excl_sum_u32(nullptr, &tb3, unm.as<unsigned int>(), upos.as<unsigned int>(), B.n, c.stream));
        DevBuf temp3(tb3);
        HIPCHECK(cq_excl_sum_u32(temp3.p, &tb3, unm.as<unsigned int>(), upos.as<unsigned int>(), B.n, c.stream));
        unsigned int ul[2] = {0, 0};
        HIPCHECK(hipMemcpyAsync(&ul[0], upos.as<unsigned int>() + B.n - 1, 4, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipMemcpyAsync(&ul[1], unm.as<unsigned int>() + B.n - 1, 4, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        const unsigned long long nr2 = (unsigned long long)ul[0] + ul[1];
        DevBuf pb(std::max<unsigned long long>(nl2 + nr2, 1) * 8);
        std::swap(pairs.p, pb.p);
        if (nl2) HIPCHECK(cq_launch_join_fill(nullptr, nullptr, (uint32_t)nl2, 0, 0, pairs.as<uint2>(), c.stream));
        if (nr2) HIPCHECK(cq_launch_join_fill(unm.as<unsigned int>(), upos.as<unsigned int>(), B.n, nl2, 1,
                                              pairs.as<uint2>(), c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        np = nl2 + nr2;
    }
    else if (outer_left || outer_right) {
        // nothing matches: every row of the outer side(s), NULL-padded
        const unsigned long long nl2 = outer_left ? A.n : 0, nr2 = outer_right ? B.n : 0;
        DevBuf pb(std::max<unsigned long long>(nl2 + nr2, 1) * 8);
        std::swap(pairs.p, pb.p);
        if (nl2) HIPCHECK(cq_launch_join_fill(nullptr, nullptr, (uint32_t)nl2, 0, 0, pairs.as<uint2>(), c.stream));
        if (nr2) HIPCHECK(cq_launch_join_fill(nullptr, nullptr, (uint32_t)nr2, nl2, 1, pairs.as<uint2>(), c.stream));
        np = nl2 + nr2;
    }
    return np;
}

// The canonical INTEGER keys (jx_key's shape) of column `col` in the table's sampled
// bytes: their [min, max] widened to cover the records the whole table is estimated to
// hold (a guess: a key outside it only costs the STAR join a second round).  S: the
// table's key stride (1, or N on a rank of a key-mod-N repartition): the keys are one
// residue class mod S, so the estimated records span est * S key units, and kmin
// stays in the sampled keys' class
bool sample_key_range(const cqgpu_table* t, int col, uint64_t S, uint64_t* kmin, uint64_t* kmax, uint64_t* est) {
    const std::string& s = t->sample;
    const char delim = (char)t->cfg.delimiter;
    uint64_t lo = ~0ull, hi = 0, nrec = 0, used = 0;
    size_t i = 0;
    while (i < s.size()) {
        while (i < s.size() && (s[i] == '\n' || s[i] == '\r')) i++;
        const size_t rs = i;
        while (i < s.size() && s[i] != '\n' && s[i] != '\r') i++;
        if (i >= s.size()) break;                    // a record cut by the sample's end
        nrec++;
        used = i;
        size_t f = rs;
        for (int k = 0; k < col && f < i; k++) {
            while (f < i && s[f] != delim) f++;
            if (f < i) f++;
        }
        size_t e = f;
        while (e < i && s[e] != delim) e++;
        const size_t len = e - f;
        if (len == 0 || len > 15 || (len >= 8 && len <= 10) || (s[f] == '0' && len > 1)) continue;
        uint64_t v = 0;
        bool ok = true;
        for (size_t k = f; k < e; k++) {
            const unsigned dg = (unsigned)(unsigned char)s[k] - '0';
            ok = ok && dg < 10;
            v = v * 10 + dg;
        }
        if (!ok) continue;
        lo = std::min(lo, v);
        hi = std::max(hi, v);
    }
    if (!nrec || lo > hi || !used || S == 0) return false;
    const uint64_t n = t->n > t->data_begin ? t->n - t->data_begin : 0;
    *est = (uint64_t)((double)n * (double)nrec / (double)used) + 1;
    const uint64_t span = std::max<uint64_t>(hi - lo, *est * S);
    const uint64_t pad = (span / 8 / S + 16) * S;
    *kmin = lo > pad ? lo - pad : lo % S;
    *kmax = std::max(hi, *kmin + span + span / 4 + 1024 * S);
    return true;
}

// average record bytes of a table's sampled data (records and their terminators)
double sample_record_bytes(const cqgpu_table* t) {
    const std::string& s = t->sample;
    size_t i = 0, nrec = 0, used = 0;
    while (i < s.size()) {
        while (i < s.size() && (s[i] == '\n' || s[i] == '\r')) i++;
        while (i < s.size() && s[i] != '\n' && s[i] != '\r') i++;
        if (i >= s.size()) break;
        nrec++;
        used = i;
    }
    return nrec ? (double)used / (double)nrec : 64.0;
}

// The fused aggregate join: one INNER JOIN on `ident = ident`
// without WHERE, COUNT / SUM / AVG of one probe-side (right) column, GROUP BY one
// build-side (left) column or none, every other item a left column.  No record-start
// pass, no cell tables, no pair array: both sides stream through jx_extract_kernel
// (ON key + one payload per record), the left side's keys go into an HBM hash table,
// and every right record probes it and aggregates its pairs into LDS group tables
// (jx_probe_kernel), then raw_merge / compact / finish (the group's first pair's left
// record) / pack as run_aggregate.  Same groups, order and cells as aggregate_pairs:
// a pair's order key is (left byte offset, right byte offset), the nested loop's
// (l, r) order.  nullptr: outside this shape, or the data (a quote, a short row, a key
// that is not a canonical INTEGER below 10^15 or NULL, a wider numeral) needs the
// general pipeline.
// test knob CQ_AMD_JX_DEBUG: why a fused join handed a query on (stderr)
#define JXDBG(...) do { if (getenv("CQ_AMD_JX_DEBUG")) fprintf(stderr, "cq_amd jx: " __VA_ARGS__); } while (0)
// run_fast_join's answer when it filled a JoinPartial (a range / routed partial)
cq_table* const JOIN_PART_DONE = reinterpret_cast<cq_table*>(uintptr_t(1));

cq_table* run_fast_join(DevCtx& c, cq_node* q, Compiled& C, const cqgpu_table* L, const cqgpu_table* R, int kl,
                        int kr, int nl, JoinPartial* part = nullptr, const std::vector<std::string>* jnames = nullptr) {
    if (getenv("CQ_AMD_NO_FAST_JOIN")) return nullptr;
    if (part && !C.grouped) return nullptr;  // (an ungrouped partial reports its one group even when empty)
    if (C.group_missing || C.P.nprog != 0 || C.P.ngpart != 0 || !C.vla.empty()) return nullptr;
    if (L->n >= (1ull << 32) - 4096 || R->n >= (1ull << 32) - 4096) return nullptr;
    if (L->cfg.delimiter != R->cfg.delimiter || L->cfg.quote != R->cfg.quote) return nullptr;
    const uint32_t d = (uint8_t)L->cfg.delimiter;
    if ((d - '0') < 10u || d == '.' || ((d | 32) >= 'a' && (d | 32) <= 'z') || d == '+' || d == '-' || d <= ' ')
        return nullptr;
    if ((uint8_t)L->cfg.quote == d || L->cfg.quote == '\n' || L->cfg.quote == '\r') return nullptr;
    const bool grouped = C.grouped;
    int gcol = -1, vcol = -1;
    if (grouped) {
        if (C.P.group_slot < 0) return nullptr;
        gcol = C.need_cols[C.P.group_slot];
        if (gcol >= nl) return nullptr;
    }
    for (int a = 0; a < C.P.nacc; a++) {
        if (C.P.acc[a].kind != ACC_SUM) return nullptr;
        const int col = C.need_cols[C.P.acc[a].slot];
        if (col < nl) return nullptr;
        if (vcol >= 0 && col - nl != vcol) return nullptr;
        vcol = col - nl;
    }
    for (int rc : C.rep_cols)
        if (rc >= nl) return nullptr;
    for (const OutCol& o : C.outs)
        if (o.kind != OUT_COUNT && o.kind != OUT_SUM && o.kind != OUT_AVG && o.kind != OUT_REP && o.kind != OUT_CONST &&
            o.kind != OUT_NULL)
            return nullptr;
    if (C.wide || C.rep_cols.size() > (size_t)MAX_WIDE) return nullptr;
    const uint32_t ws = L->lean_ws ? L->lean_ws : 3968u, wsr = R->lean_ws ? R->lean_ws : 3968u;
    const int xgrid = c.ncu;
    const uint8_t dq = (uint8_t)L->cfg.quote;
    Literals Lit;
    parse_literals(c, C.lits, Lit);
    // finish: the representative (left) columns of each group's first pair's left record
    constexpr uint32_t SB = 48;
    FinishDesc FD;
    memset(&FD, 0, sizeof FD);
    std::vector<int> rep_ord(C.rep_cols.size());
    for (size_t i = 0; i < rep_ord.size(); i++) rep_ord[i] = (int)i;
    std::sort(rep_ord.begin(), rep_ord.end(), [&](int a, int b) { return C.rep_cols[a] < C.rep_cols[b]; });
    FD.ncols = (int32_t)rep_ord.size();
    for (size_t i = 0; i < rep_ord.size(); i++) FD.cols[i] = (int16_t)C.rep_cols[rep_ord[i]];
    FD.delim = d;
    FD.quote = (uint8_t)L->cfg.quote;
    FD.nacc = C.P.nacc;
    FD.sb = SB;
    FD.first_shift = 32;
    const uint32_t ncell = (uint32_t)FD.ncols + (uint32_t)FD.nacc + 1;
    // the groups `fill` puts into an arena's table (raw tags when grouped) -> the result:
    // raw_merge / compact / finish / pack, one synchronisation; *fallback when the
    // flags at dflag ask for another path (nothing returned then)
    // a STAR partial: the packed groups' first pairs mapped to global left ids on the
    // device before the mailbox copy (route.hip pack_first_gid_kernel); `first_mapped`
    // says the result holds ids
    const unsigned long long* map_starts = nullptr;
    const unsigned long long* map_gids = nullptr;
    unsigned long long map_n = 0;
    bool first_mapped = false;
    auto results = [&](const std::function<void(TableArena&)>& fill, const unsigned int* dflag, uint64_t records,
                       int kind, bool* fallback) -> cq_table* {
        *fallback = false;
        uint32_t cap = grouped ? 8192 : 64;
        for (int attempt = 0; attempt < 4; attempt++, cap *= 8) {
            TableArena A = make_arena(c, C.P, cap, cap / 2 + 1, 1, 16);
            const unsigned int cap_out = cap / 2 + 1;
            Scratch fin(c, (size_t)cap_out * ncell * (sizeof(Cell) + SB) + 64);
            Cell* dcells = (Cell*)fin.p;
            uint8_t* dbytes = fin.p + (size_t)cap_out * ncell * sizeof(Cell);
            fill(A);
            if (grouped) HIPCHECK(cq_launch_raw_merge(&A.gt, &A.rt, C.P.nacc, A.stats, c.stream));
            HIPCHECK(hipEventRecord(c.ev1, c.stream));
            constexpr size_t MAIL_HDR = 1024;
            uint8_t* mail = mailbox(c, MAIL_HDR + cq_pack_result_bytes(cap_out, C.P.nacc, ncell, SB) + 64);
            Scratch pk, ofs;
            if (cap_out <= cq_finish_pack_max()) {      // finish + pack in one launch, then the mailbox copy
                ofs.get(c, (size_t)cap_out * 8 + 64);
                pk.get(c, cq_pack_result_bytes(cap_out, C.P.nacc, ncell, SB) + 64);
                HIPCHECK(cq_launch_compact(&A.gt, &C.P, A.out, A.out_count, cap_out, c.stream,
                                           (unsigned long long*)ofs.p));
                HIPCHECK(cq_launch_finish_pack(L->g, L->n, A.out, (const unsigned long long*)ofs.p, A.out_count,
                                               cap_out, &FD, pk.p, A.stats, mail, c.stream));
                if (map_starts) {
                    HIPCHECK(cq_launch_pack_first_gid(pk.p, A.out_count, cap_out, 40u + 40u * (uint32_t)C.P.nacc,
                                                      map_starts, map_n, map_gids, c.stream));
                    first_mapped = true;
                }
                HIPCHECK(cq_launch_mail_copy(pk.p, A.out_count, cap_out, C.P.nacc, ncell, SB, mail + MAIL_HDR,
                                             c.stream));
            } else {
                first_mapped = false;
                HIPCHECK(cq_launch_compact(&A.gt, &C.P, A.out, A.out_count, cap_out, c.stream, nullptr));
                HIPCHECK(cq_launch_finish(L->g, L->n, A.out, A.out_count, cap_out, &FD, dcells, dbytes, c.stream));
                HIPCHECK(cq_launch_pack_result(A.out, A.out_count, cap_out, C.P.nacc, dcells, dbytes, ncell, SB,
                                               mail + MAIL_HDR, A.stats, mail, 1, c.stream));
            }
            // the flags through pinned memory (a pageable destination would block here);
            // the result rows' pool refilled while the device works
            unsigned int* hfl = (unsigned int*)pinned(c, 16);
            HIPCHECK(hipMemcpyAsync(hfl, dflag, 4, hipMemcpyDeviceToHost, c.stream));
            PHASE("results launch");
            if (grouped) {
                uint32_t nstr = 0;
                for (const OutCol& o : C.outs) nstr += o.kind == OUT_REP || o.kind == OUT_CONST;
                rowpool_fill((int)C.outs.size(), nstr);
                PHASE("pool");
            }
            HIPCHECK(hipStreamSynchronize(c.stream));
            const unsigned int fl = *hfl;
            PHASE("sync");
            if (fl) { JXDBG("flags %#x\n", fl); *fallback = true; return nullptr; }
            ScanStats st;
            memcpy(&st, mail, sizeof st);
            unsigned int ng = 0;
            memcpy(&ng, mail + sizeof(ScanStats), 4);
            if (st.overflow >= 2) throw HipError{"fused join: group insert timeout"};
            if (st.overflow) continue;
            float ms = 0;
            HIPCHECK(hipEventElapsedTime(&ms, c.ev0, c.ev1));
            g_stats.scan_ms = ms;
            g_stats.records = records;
            g_stats.passed = st.passed;
            g_stats.scan_kernel = kind;
            ng = std::min(ng, cap_out);
            const bool presorted = ng <= cq_pack_order_max();
            static thread_local std::vector<uint8_t> hbuf;
            const size_t pb = cq_pack_result_bytes(ng, C.P.nacc, ncell, SB);
            if (hbuf.size() < pb + 8) hbuf.resize(pb + 8);
            memcpy(hbuf.data(), mail + MAIL_HDR, pb);
            PHASE("mcopy");
            cq_table* res = nullptr;
            if (!part && grouped && presorted && ng) res = build_direct(C, hbuf.data(), ng, ncell, SB, rep_ord, Lit, ~0ull);
            PHASE("direct");
            if (part && presorted && C.vla.empty()) {
                // the partial's groups in the blob's group format, straight from the packed
                // records (cqgpu_query_partial's "CQJ1" writer, field for field); any STRING
                // cell longer than the inline bytes takes the HGroup path below
                const size_t rec = 40 + 40 * (size_t)C.P.nacc;
                const Cell* cells = (const Cell*)(hbuf.data() + ng * rec);
                const uint8_t* sbytes = hbuf.data() + ng * rec + (size_t)ng * ncell * sizeof(Cell);
                bool inline_ok = true;
                for (size_t k = 0; k < (size_t)ng * ncell; k++)
                    inline_ok = inline_ok && !(cells[k].kind == K_STR && cells[k].len > SB);
                if (inline_ok) {
                    const uint32_t nrep = (uint32_t)C.rep_cols.size();
                    // sized once for the worst case (every cell a SB-byte string), written
                    // through a raw cursor, trimmed at the end
                    const size_t cell_max = 16 + SB;
                    const size_t per = 4 + 4 + 8 + 8 + 4 + 16 + 8 + 8 + (size_t)C.P.nacc * (24 + cell_max) +
                                       (size_t)nrep * cell_max + 4 + cell_max;
                    std::vector<uint8_t>& gb = part->gblob;
                    gb.resize((size_t)ng * per);
                    uint8_t* w = gb.data();
                    auto u32 = [&](uint32_t v) { memcpy(w, &v, 4); w += 4; };
                    auto u64 = [&](uint64_t v) { memcpy(w, &v, 8); w += 8; };
                    auto bytes = [&](const void* src, uint32_t n) { u32(n); memcpy(w, src, n); w += n; };
                    part->first_at.clear();
                    part->first_at.reserve(ng);
                    auto cell_out = [&](size_t k) {
                        const Cell& x = cells[k];
                        u32(x.kind);
                        u64(x.bits);
                        bytes(sbytes + k * SB, x.kind == K_STR ? x.len : 0u);
                    };
                    std::vector<int> rep_at(nrep, -1);          // h.reps[rep_ord[i]] = cs[i]
                    for (size_t i = 0; i < rep_ord.size(); i++) rep_at[rep_ord[i]] = (int)i;
                    for (unsigned int i = 0; i < ng; i++) {
                        const uint8_t* r = hbuf.data() + i * rec;
                        const uint32_t cl = ((const uint32_t*)r)[0];
                        const uint64_t w0 = ((const uint64_t*)r)[1], w1 = ((const uint64_t*)r)[2];
                        const uint32_t kcls = cl >> 16, klen = cl & 0xffff;
                        u32(kcls);
                        u32(klen);
                        u64(w0);
                        u64(w1);
                        if (kcls == GK_LONG) {
                            const size_t k = (size_t)i * ncell + FD.ncols + C.P.nacc;
                            bytes(sbytes + k * SB, cells[k].kind == K_STR ? cells[k].len : 0u);
                        } else if (kcls == GK_STR) {
                            uint8_t kb[16];
                            const uint32_t n = std::min<uint32_t>(klen, 16);
                            for (uint32_t j = 0; j < n; j++) kb[j] = (uint8_t)((j < 8 ? w0 >> (8 * j) : w1 >> (8 * (j - 8))) & 0xff);
                            bytes(kb, n);
                        } else {
                            u32(0);
                        }
                        u64(((const unsigned long long*)r)[3]);          // COUNT
                        part->first_at.push_back((size_t)(w - gb.data()));
                        u64(((const unsigned long long*)r)[4]);          // first pair (patched)
                        const uint64_t* qq = (const uint64_t*)(r + 40);
                        for (int a = 0; a < C.P.nacc; a++) {
                            u64(qq[5 * a]);                              // SUM (f64 bits)
                            u64(qq[5 * a + 1]);                          // numeric count
                            u64(NOPOS);                                  // (SUM plans: no extreme)
                            cell_out((size_t)i * ncell + FD.ncols + a);
                        }
                        for (uint32_t rr = 0; rr < nrep; rr++) {
                            if (rep_at[rr] >= 0) cell_out((size_t)i * ncell + rep_at[rr]);
                            else { u32(K_NULL); u64(0); u32(0); }
                        }
                        u32(0);                                          // no class splits
                    }
                    gb.resize((size_t)(w - gb.data()));
                    part->direct = true;
                    part->ng = ng;
                    g_stats.groups = ng;
                    PHASE("serialize");
                    return JOIN_PART_DONE;
                }
            }
            if (!res) {
                std::vector<GroupOut> outs(ng);
                std::vector<Cell> fcells((size_t)ng * ncell);
                std::vector<uint8_t> fbytes((size_t)ng * ncell * SB);
                const size_t rec = 40 + 40 * (size_t)C.P.nacc;
                memset(outs.data(), 0, ng * sizeof(GroupOut));
                for (unsigned int i = 0; i < ng; i++) {
                    const uint8_t* r = hbuf.data() + i * rec;
                    GroupOut& o = outs[i];
                    o.clslen = ((const uint32_t*)r)[0];
                    o.w0 = ((const uint64_t*)r)[1];
                    o.w1 = ((const uint64_t*)r)[2];
                    o.cnt = ((const unsigned long long*)r)[3];
                    o.first = ((const unsigned long long*)r)[4];
                    const uint64_t* qq = (const uint64_t*)(r + 40);
                    for (int a = 0; a < C.P.nacc; a++) {
                        o.sum[a] = as_dbl(qq[5 * a]);
                        o.num[a] = qq[5 * a + 1];
                        o.extpos[a] = NOPOS;
                    }
                }
                memcpy(fcells.data(), hbuf.data() + ng * rec, fcells.size() * sizeof(Cell));
                memcpy(fbytes.data(), hbuf.data() + ng * rec + fcells.size() * sizeof(Cell), fbytes.size());
                std::vector<HGroup> groups = make_groups(c, C, ~0ull, 0, outs, fcells, fbytes, FD.ncols, rep_ord, SB,
                                                         presorted);
                g_stats.groups = groups.size();
                if (part) {                       // the groups themselves; run_fast_join globalises them
                    part->groups = std::move(groups);
                    return JOIN_PART_DONE;
                }
                res = build_groups(C, groups, Lit, c);
            } else {
                g_stats.groups = ng;
            }
            post_ops(c, res, q);
            return res;
        }
        *fallback = true;
        return nullptr;
    };

    // ---- STAR: the build side's keys span a dense range (a primary key): both sides
    // stream once, the build records straight into key-indexed arrays (group id + 1,
    // byte offset), every probe record looks its key up, marks it and adds its pair
    // into per-block group sums; no record arrays, no count pass (fast.hip jx_star_*).
    // The range comes from the table's learned key range, else the sampled bytes; a
    // key outside it, a NULL or repeated build key, or more than JX_G GROUP BY values
    // sends the query on to the record-array path below.
    if (!getenv("CQ_AMD_NO_STAR_JOIN")) {
        cqgpu_table* Lm = const_cast<cqgpu_table*>(L);
        bool no_part = getenv("CQ_AMD_NO_PART_PROBE") != nullptr;
        if (part && !getenv("CQGPU_HOST_FIRST_IDS")) {
            // the partial's first pairs become global left ids on the device: the left
            // table's file-order record starts (once per table: it is immutable)
            if (!Lm->rec_starts) {
                std::unique_ptr<DevBuf> b(new DevBuf());
                Lm->nrec_starts = all_records(c, L, *b);
                Lm->rec_starts = std::move(b);
            }
            if (L->gids && L->ngids != Lm->nrec_starts) throw HipError{"routed table: record count differs from its ids"};
            map_starts = Lm->rec_starts->as<unsigned long long>();
            map_n = Lm->nrec_starts;
            map_gids = L->gids;
        }
        for (int round = 0; round < 3; round++) {
            uint64_t kmin = 0, kmax = 0, est = 0;
            const uint64_t S = L->key_stride ? L->key_stride : 1;
            auto it = Lm->key_range.find(kl);
            // (CQGPU_NO_LEARNED_RANGE: every call as a fresh table's first -- a routed
            //  table rebuilt per step, as the multi-GPU join does)
            const bool learned = it != Lm->key_range.end() && !getenv("CQGPU_NO_LEARNED_RANGE");
            if (learned) {
                kmin = it->second.first;
                kmax = it->second.second;
                est = kmax >= kmin ? (kmax - kmin) / S + 1 : 0;
            } else if (!sample_key_range(L, kl, S, &kmin, &kmax, &est)) {
                JXDBG("star: no sampled keys\n");
                break;
            }
            // key slots: kmin, kmin + S, ... (the table's keys are one residue class mod S)
            const uint64_t range = kmax >= kmin ? (kmax - kmin) / S + 1 : 0;
            JXDBG("star round %d: keys [%llu, %llu] stride %llu slots %llu est %llu learned %d\n", round,
                  (unsigned long long)kmin, (unsigned long long)kmax, (unsigned long long)S, (unsigned long long)range,
                  (unsigned long long)est, (int)learned);
            if (kmax < kmin || range >= (1ull << 31) || range * S >= (1ull << 32) || range > 4 * est + 1024) break;
            const size_t b16 = (range * 2 + 15) & ~(size_t)15;
            DevBuf big(b16), l32(range * 4 + 16);
            const uint32_t G = cq_jx_star_groups();
            // ttab | gsum | gfirst | gminix | control words; the build windows' first / last keys
            // (control words: [0] flags, [8..32) placed / pairs / occupied, [32..48) the build
            // keys' min (0xFF..) and max, [48..52) not-rising)
            const size_t o_gsum = (size_t)G * 8, o_first = o_gsum + (size_t)G * 24, o_minix = o_first + (size_t)G * 4,
                         o_ctl = o_minix + (size_t)G * 4;
            DevBuf small(o_ctl + 64);
            // records averaging under ~33 bytes (a sampled stride below the largest):
            // three records per lane pass over windows of the largest stride (fast_kernel's rule)
            const bool rp2 = getenv("CQGPU_FAST_RP2") != nullptr;
            const int rpl = ws < 3968u && !rp2 ? 3 : 2, rpr = wsr < 3968u && !rp2 ? 3 : 2;
            const uint32_t wsl3 = rpl == 3 ? 3968u : ws, wsr3 = rpr == 3 ? 3968u : wsr;
            const uint64_t nwb = cq_jx_windows(L->data_begin, L->n, wsl3);
            DevBuf wfl(std::max<uint64_t>(nwb, 1) * 16);
            uint16_t* d16 = big.as<uint16_t>();
            unsigned long long* ttab = small.as<unsigned long long>();
            unsigned long long* gsum = (unsigned long long*)(small.as<uint8_t>() + o_gsum);
            uint32_t* gfirst = (uint32_t*)(small.as<uint8_t>() + o_first);
            uint32_t* gminix = (uint32_t*)(small.as<uint8_t>() + o_minix);
            unsigned int* sflag = (unsigned int*)(small.as<uint8_t>() + o_ctl);
            unsigned long long* cnts = (unsigned long long*)(small.as<uint8_t>() + o_ctl + 8);   // placed, pairs, occupied
            unsigned long long* skr = cnts + 3;                                                  // build keys' min, max
            uint32_t* snotmono = (uint32_t*)(skr + 2);
            PHASE("star setup");
            // one launch: d16 zero, gfirst / gminix and the keys' min 0xFF.., the rest of
            // the small block zero, the GROUP BY tag table seeded with the build side's
            // sampled tags (fast_kernel's placement: the build's lookups hit without walking)
            const void* seed = grouped ? fast_seed_of(L, gcol) : nullptr;
            HIPCHECK(cq_jx_star_init(big.p, b16, small.p, o_ctl + 64, (uint32_t)o_first, (uint32_t)o_ctl,
                                     (uint32_t)o_ctl + 32, seed, seed ? (size_t)G * 8 : 0, c.ncu * 4, c.stream));
            HIPCHECK(hipEventRecord(c.ev0, c.stream));
            HIPCHECK(cq_jx_star_extract(L->g, L->data_begin, L->n, wsl3, d, dq, kl, grouped ? gcol : -1, 1, kmin, range, (uint32_t)S, d16,
                                        l32.as<uint32_t>(), ttab, gsum, cnts, sflag, skr, snotmono,
                                        wfl.as<unsigned long long>(), nullptr, rpl, xgrid, c.stream));
            HIPCHECK(cq_jx_star_order(wfl.as<unsigned long long>(), nwb, snotmono, c.stream));
            // the probe: when d16 (2 bytes per key slot) outgrows one XCD's 4 MiB L2, in two
            // passes -- every probe record's (slot, payload) appended to its key partition
            // (2 MiB d16 slices), then each partition looked up by the blocks of one XCD
            // (fast.hip jx_part_probe_kernel); else one pass with the lookups in place
            // (test knobs: CQGPU_PART_PROBE_MIN slots above which it partitions, default 2^21;
            //  CQGPU_PART_PROBE_SHIFT log2 slots per partition, default 20)
            const char* pm_env = getenv("CQGPU_PART_PROBE_MIN");
            const char* ps_env = getenv("CQGPU_PART_PROBE_SHIFT");
            const uint64_t part_min = pm_env ? strtoull(pm_env, nullptr, 10) : (2ull << 20);
            const uint32_t PSH = ps_env ? (uint32_t)std::min(std::max(atoi(ps_env), 4), 24) : 20u;
            const uint64_t np64 = (range + (1ull << PSH) - 1) >> PSH;
            const bool pprobe = !no_part && range > part_min && np64 <= 4096 && xgrid >= 8;
            DevBuf pent, pcnt;
            if (pprobe) {
                const uint64_t rb = R->n > R->data_begin ? R->n - R->data_begin : 0;
                const uint64_t est_r = (uint64_t)((double)rb / std::max(1.0, sample_record_bytes(R))) + 1;
                // (a sampled range is padded past the keys: the probe keys fill the
                // partitions of about `est` slots, not all np64 of them)
                const uint64_t np_eff = std::max<uint64_t>(1, std::min<uint64_t>(range, est) >> PSH);
                const uint64_t per = est_r / ((uint64_t)xgrid * std::min<uint64_t>(np64, np_eff));
                const uint32_t pcap = (uint32_t)std::min<uint64_t>(per + per / 4 + 256, 1u << 30);
                DevBuf a((size_t)xgrid * np64 * pcap * 8), b((size_t)xgrid * np64 * 4);
                std::swap(pent.p, a.p);
                std::swap(pcnt.p, b.p);
                // (two records per lane pass here, whatever the record length: the partition
                // append holds more state per record, and the three-record build measured
                // 0.92 vs 0.72 ms on config 5's 33-byte orders, same box)
                const char* prp = getenv("CQGPU_PART_RP");
                const int rpp = prp ? (atoi(prp) == 3 ? 3 : 2) : 2;
                HIPCHECK(cq_jx_star_extract(R->g, R->data_begin, R->n, 3968u, d, dq, kr, vcol, 0, kmin, range, (uint32_t)S,
                                            d16, l32.as<uint32_t>(), ttab, gsum, cnts + 1, sflag, nullptr, snotmono,
                                            nullptr, gminix, rpp, xgrid, c.stream, pent.as<unsigned long long>(),
                                            pcnt.as<uint32_t>(), (uint32_t)np64, pcap, PSH));
                HIPCHECK(cq_jx_part_probe(pent.as<unsigned long long>(), pcnt.as<uint32_t>(), (uint32_t)xgrid,
                                          (uint32_t)np64, pcap, range, d16, snotmono, gsum, gminix, cnts + 1,
                                          std::max(8, (c.ncu / 8) * 8), c.stream));
            } else {
                HIPCHECK(cq_jx_star_extract(R->g, R->data_begin, R->n, wsr3, d, dq, kr, vcol, 0, kmin, range, (uint32_t)S,
                                            d16, l32.as<uint32_t>(), ttab, gsum, cnts + 1, sflag, nullptr, snotmono,
                                            nullptr, gminix, rpr, xgrid, c.stream));
            }
            HIPCHECK(cq_jx_star_first(d16, l32.as<uint32_t>(), range, snotmono, gfirst, cnts + 2, c.ncu * 4, c.stream));
            PHASE("star launch");
            bool fb = false;
            cq_table* res = results([&](TableArena& A) {
                HIPCHECK(cq_jx_star_flush(grouped ? 1 : 0, vcol >= 0 ? 1 : 0, ttab, gsum, gfirst, gminix,
                                          l32.as<uint32_t>(), snotmono, cnts, grouped ? &A.rt : &A.gt, C.P.nacc,
                                          A.stats, sflag, c.stream));
            }, sflag, 0, 4, &fb);
            if (res == JOIN_PART_DONE) {
                // a partial: each group's first pair as (global left id << 32) -- the left
                // record's byte offset to its row (binary search over the table's record
                // starts) to its global id; the right id is left 0: a left record belongs
                // to one group and lives on one rank, so the left id alone orders groups,
                // here and in the merge
                cqgpu_table* Lw = const_cast<cqgpu_table*>(L);
                if (!Lw->rec_starts) {
                    std::unique_ptr<DevBuf> b(new DevBuf());
                    Lw->nrec_starts = all_records(c, L, *b);
                    Lw->rec_starts = std::move(b);
                }
                if (L->gids && L->ngids != Lw->nrec_starts) throw HipError{"routed table: record count differs from its ids"};
                PHASE("recs");
                std::vector<unsigned long long> qo;
                std::vector<size_t> qat;                 // (direct blob: where each first lives)
                if (first_mapped) {                      // ids already (pack_first_gid_kernel)
                    auto check = [](unsigned long long f) {
                        if (f != NOPOS && (f >> 32) == 0xFFFFFFFFull)
                            throw HipError{"fused join partial: left id out of range"};
                    };
                    if (part->direct) {
                        for (size_t at : part->first_at) {
                            unsigned long long f;
                            memcpy(&f, part->gblob.data() + at, 8);
                            check(f);
                        }
                    } else {
                        for (const HGroup& h : part->groups) check(h.first);
                    }
                } else if (part->direct) {
                    for (size_t at : part->first_at) {
                        unsigned long long f;
                        memcpy(&f, part->gblob.data() + at, 8);
                        if (f != NOPOS) { qo.push_back(f >> 32); qat.push_back(at); }
                    }
                } else {
                    for (const HGroup& h : part->groups)
                        if (h.first != NOPOS) qo.push_back(h.first >> 32);
                }
                if (!qo.empty()) {
                    // (through the pinned staging buffer and the bump scratch: pageable
                    // copies and fresh device buffers cost more than the lookup itself)
                    const size_t qb = qo.size() * 8;
                    Scratch dqk(c, 2 * qb + 64);
                    unsigned long long* dq = (unsigned long long*)dqk.p;
                    unsigned long long* dk = dq + qo.size();
                    unsigned long long* hq = (unsigned long long*)pinned(c, qb);
                    memcpy(hq, qo.data(), qb);
                    HIPCHECK(hipMemcpyAsync(dq, hq, qb, hipMemcpyHostToDevice, c.stream));
                    HIPCHECK(cq_launch_offset_gid(Lw->rec_starts->as<unsigned long long>(), Lw->nrec_starts, dq,
                                                  (uint32_t)qo.size(), L->gids, dk, c.stream));
                    HIPCHECK(hipMemcpyAsync(hq, dk, qb, hipMemcpyDeviceToHost, c.stream));
                    PHASE("gid launch");
                    HIPCHECK(hipStreamSynchronize(c.stream));
                    PHASE("gid sync");
                    memcpy(qo.data(), hq, qb);
                    for (unsigned long long g : qo)
                        if (g >= (1ull << 32)) throw HipError{"fused join partial: left id out of range"};
                    if (part->direct) {
                        for (size_t k = 0; k < qo.size(); k++) {
                            const unsigned long long f = qo[k] << 32;
                            memcpy(part->gblob.data() + qat[k], &f, 8);
                        }
                    } else {
                        size_t k = 0;
                        for (HGroup& h : part->groups) {
                            if (h.first == NOPOS) continue;
                            h.first = qo[k++] << 32;
                        }
                    }
                }
                PHASE("gids");
                if (jnames) part->names = *jnames;
                for (int a = 0; a < MAX_ACC; a++) part->acc_classes[a] = 0;    // SUM only
                // key classes (bit 1: numbers): every build key is a canonical INTEGER (else the
                // STAR flags declined); the probe side reported as numbers whenever it has rows
                part->lmask |= Lw->nrec_starts ? 2u : 0u;
                part->rmask |= R->n > R->data_begin ? 2u : 0u;
            }
            if (res || !fb) {
                if (res && !learned) {           // the exact range, for the next query on this table
                    unsigned long long kr2[2] = {~0ull, 0ull};
                    HIPCHECK(hipMemcpyAsync(kr2, skr, 16, hipMemcpyDeviceToHost, c.stream));
                    HIPCHECK(hipStreamSynchronize(c.stream));
                    if (kr2[0] <= kr2[1]) Lm->key_range[kl] = {kr2[0], kr2[1]};
                }
                return res;
            }
            unsigned int fl = 0;
            unsigned long long kr2[2] = {~0ull, 0ull};
            HIPCHECK(hipMemcpyAsync(&fl, sflag, 4, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipMemcpyAsync(kr2, skr, 16, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
            // a full partition region (skewed probe keys) or a wide payload: again, unpartitioned
            if (fl == 128u && !no_part) {
                no_part = true;
                continue;
            }
            // only a range miss is worth a second round (with the range the build saw)
            if (fl != 16u || kr2[0] > kr2[1] || learned) break;
            Lm->key_range[kl] = {kr2[0], kr2[1]};
        }
    }

    if (part) return nullptr;              // (partials: the general join below the caller)
    // pass 0: records per window; exclusive scans give every window's first record index
    const uint64_t nwl = cq_jx_windows(L->data_begin, L->n, ws), nwr = cq_jx_windows(R->data_begin, R->n, wsr);
    if (nwl >= (1ull << 31) || nwr >= (1ull << 31)) return nullptr;
    DevBuf wcl(std::max<size_t>(nwl, 1) * 4), wbl(std::max<size_t>(nwl, 1) * 4);
    DevBuf wcr(std::max<size_t>(nwr, 1) * 4), wbr(std::max<size_t>(nwr, 1) * 4), ctl(256);
    unsigned int* dctl = ctl.as<unsigned int>();      // [2] extract flags, [3] direct-build flags
    unsigned long long* krange = (unsigned long long*)(dctl + 4);   // build keys' min, max; [2..3] probe's
    HIPCHECK(hipMemsetAsync(ctl.p, 0, 256, c.stream));
    HIPCHECK(hipMemsetAsync(krange, 0xff, 8, c.stream));
    HIPCHECK(hipMemsetAsync(krange + 2, 0xff, 8, c.stream));
    HIPCHECK(hipEventRecord(c.ev0, c.stream));
    HIPCHECK(cq_jx_extract(L->g, L->data_begin, L->n, ws, d, dq, kl, gcol, 1, 0, nullptr, nullptr, nullptr,
                           wcl.as<unsigned int>(), nullptr, 0, dctl + 2, krange, xgrid, c.stream));
    HIPCHECK(cq_jx_extract(R->g, R->data_begin, R->n, wsr, d, dq, kr, vcol, 0, 0, nullptr, nullptr, nullptr,
                           wcr.as<unsigned int>(), nullptr, 0, dctl + 2, krange + 2, xgrid, c.stream));
    size_t tbl = 0, tbr = 0;
    HIPCHECK(cq_excl_sum_u32(nullptr, &tbl, wcl.as<unsigned int>(), wbl.as<unsigned int>(), nwl, c.stream));
    HIPCHECK(cq_excl_sum_u32(nullptr, &tbr, wcr.as<unsigned int>(), wbr.as<unsigned int>(), nwr, c.stream));
    DevBuf tmp(std::max(tbl, tbr) + 16);
    if (nwl) HIPCHECK(cq_excl_sum_u32(tmp.p, &tbl, wcl.as<unsigned int>(), wbl.as<unsigned int>(), nwl, c.stream));
    if (nwr) HIPCHECK(cq_excl_sum_u32(tmp.p, &tbr, wcr.as<unsigned int>(), wbr.as<unsigned int>(), nwr, c.stream));
    unsigned int tail[4] = {0, 0, 0, 0};
    if (nwl) {
        HIPCHECK(hipMemcpyAsync(&tail[0], wbl.as<unsigned int>() + nwl - 1, 4, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipMemcpyAsync(&tail[1], wcl.as<unsigned int>() + nwl - 1, 4, hipMemcpyDeviceToHost, c.stream));
    }
    if (nwr) {
        HIPCHECK(hipMemcpyAsync(&tail[2], wbr.as<unsigned int>() + nwr - 1, 4, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipMemcpyAsync(&tail[3], wcr.as<unsigned int>() + nwr - 1, 4, hipMemcpyDeviceToHost, c.stream));
    }
    HIPCHECK(hipStreamSynchronize(c.stream));
    const uint64_t nL = (uint64_t)tail[0] + tail[1], nR = (uint64_t)tail[2] + tail[3];
    if (nL >= (1ull << 31) || nR >= (1ull << 31)) return nullptr;
    // pass 1: the records, in file order
    DevBuf lkey(std::max<size_t>(nL, 1) * 8), lpay(std::max<size_t>(nL, 1) * 8), loff(std::max<size_t>(nL, 1) * 4);
    DevBuf rkey(std::max<size_t>(nR, 1) * 8), rpay(std::max<size_t>(nR, 1) * 8), roff(std::max<size_t>(nR, 1) * 4);
    HIPCHECK(cq_jx_extract(L->g, L->data_begin, L->n, ws, d, dq, kl, gcol, 1, 1, lkey.as<unsigned long long>(),
                           lpay.as<unsigned long long>(), loff.as<uint32_t>(), nullptr, wbl.as<unsigned int>(),
                           (unsigned int)nL, dctl + 2, krange, xgrid, c.stream));
    HIPCHECK(cq_jx_extract(R->g, R->data_begin, R->n, wsr, d, dq, kr, vcol, 0, 1, rkey.as<unsigned long long>(),
                           rpay.as<unsigned long long>(), roff.as<uint32_t>(), nullptr, wbr.as<unsigned int>(),
                           (unsigned int)nR, dctl + 2, krange + 2, xgrid, c.stream));
    unsigned long long kr2[2] = {~0ull, 0ull};
    unsigned int fl0 = 0;
    HIPCHECK(hipMemcpyAsync(&fl0, dctl + 2, 4, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipMemcpyAsync(kr2, krange, 16, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    if (fl0) { JXDBG("record arrays: extract flags %#x\n", fl0); return nullptr; }
    // the build side's keys: a direct array over a dense key range (primary keys), else
    // the hash table
    DevBuf table(8);
    uint64_t tcap = 0;
    bool direct = false;
    if (nL && kr2[0] <= kr2[1] && kr2[1] - kr2[0] < 4 * nL + 1024) {
        tcap = kr2[1] - kr2[0] + 1;
        DevBuf t2(tcap * cq_jx_direct_bytes());
        std::swap(table.p, t2.p);
        HIPCHECK(hipMemsetAsync(table.p, 0, tcap * cq_jx_direct_bytes(), c.stream));
        HIPCHECK(cq_jx_build_direct(lkey.as<unsigned long long>(), lpay.as<unsigned long long>(), loff.as<uint32_t>(),
                                    (uint32_t)nL, kr2[0], tcap, table.p, dctl + 3, c.ncu * 8, c.stream));
        unsigned int fl1 = 0;
        HIPCHECK(hipMemcpyAsync(&fl1, dctl + 3, 4, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        direct = fl1 == 0;                  // (a NULL or repeated key: the hash table)
    }
    if (!direct) {
        tcap = 1024;
        while (tcap < 2 * nL) tcap <<= 1;
        DevBuf t2((size_t)tcap * cq_jx_entry_bytes());
        std::swap(table.p, t2.p);
        HIPCHECK(hipMemsetAsync(table.p, 0, (size_t)tcap * cq_jx_entry_bytes(), c.stream));
        HIPCHECK(cq_jx_build(lkey.as<unsigned long long>(), (uint32_t)nL, table.p, tcap, dctl + 2, c.ncu * 8, c.stream));
    }
    bool fb = false;
    return results([&](TableArena& A) {
        HIPCHECK(cq_jx_probe(grouped ? 1 : 0, vcol >= 0 ? 1 : 0, direct ? 1 : 0, rkey.as<unsigned long long>(),
                             rpay.as<unsigned long long>(), roff.as<uint32_t>(), (uint32_t)nR, kr2[0], table.p, tcap,
                             lpay.as<unsigned long long>(), loff.as<uint32_t>(), grouped ? &A.rt : &A.gt, C.P.nacc,
                             A.stats, dctl + 2, c.ncu * 2, c.stream));
    }, dctl + 2, nL + nR, 3, &fb);
}

// One JOIN, or a chain of them (process_joins, evaluator_joins.c:237-274): join
// j's left side is the table joined so far, named "joined" with columns
// "<alias>.<col>" of the previous level (so a second level names "joined.u.id").
// Every level runs on the device; between levels only the columns later levels,
// the WHERE, the groups and the SELECT read are gathered into a cell table of the
// joined rows (NULL cells for an outer join's missing side).
// The columns of join side `side` (0: FROM, 1: the first JOIN's table) that a
// repartitioned join reads -- the first level's needs as run_join plans them
// (ON keys, and every column the WHERE, SELECT, GROUP BY, aggregates, HAVING /
// ORDER BY and the chain's later levels read) -- as route.hip's keep mask: bit c
// for column c, bit 63 for every column from 63 on.  ~0 (whole records): a plan
// this cannot plan (the route or the join itself then reports it), CQGPU_NO_ROUTE_PROJECT.
uint64_t route_keep_mask(cq_node* q, cqgpu_table* const* tables, int ntables, int side, uint32_t* last_keep) {
    *last_keep = ~0u;
    if (getenv("CQGPU_NO_ROUTE_PROJECT")) return ~0ull;
    try {
        const int nj = q->u.q.join_count;
        if (nj < 1 || ntables < nj + 1) return ~0ull;
        std::vector<std::string> wnames = tables[0]->names;
        std::string wa = (q->u.q.from && q->u.q.from->u.from.alias) ? q->u.q.from->u.from.alias : "main";
        std::vector<int> nleft(nj), kl(nj, -1), kr(nj, -1);
        for (int j = 0; j < nj; j++) {
            cq_node* jn = q->u.q.joins[j];
            const cqgpu_table* R = tables[j + 1];
            if (!jn || jn->kind != CQ_N_JOIN || !R) return ~0ull;
            const std::string ra = jn->u.join.alias ? jn->u.join.alias : "right";
            cqgpu_table W;
            W.names = wnames;
            cq_node* on = jn->u.join.on;
            if (on && on->kind == CQ_N_CONDITION && on->u.bin.op && !strcmp(on->u.bin.op, "=") && on->u.bin.lhs &&
                on->u.bin.rhs && on->u.bin.lhs->kind == CQ_N_IDENTIFIER && on->u.bin.rhs->kind == CQ_N_IDENTIFIER) {
                kl[j] = join_on_index(on->u.bin.lhs->u.text, &W, &W, wa.c_str(), R, ra.c_str());
                kr[j] = join_on_index(on->u.bin.rhs->u.text, R, &W, wa.c_str(), R, ra.c_str());
            }
            nleft[j] = (int)wnames.size();
            std::vector<std::string> nn;
            for (auto& nm : wnames) nn.push_back(wa + "." + nm);
            for (auto& nm : R->names) nn.push_back(ra + "." + nm);
            wnames.swap(nn);
            wa = "joined";
        }
        cqgpu_table J;
        J.cfg = tables[0]->cfg;
        J.names = wnames;
        Compiled C;
        RowPlan RP;
        if (is_row_query(q)) compile_rows(&J, q, C, RP);
        else compile_aggregate(&J, q, C);
        std::set<int> cur(C.need_cols.begin(), C.need_cols.end());
        cur.insert(C.rep_cols.begin(), C.rep_cols.end());
        for (auto& v : C.vla) cur.insert(v.second);
        cur.insert(RP.cols.begin(), RP.cols.end());
        std::set<int> lneed, rneed;
        for (int j = nj - 1; j >= 0; j--) {
            lneed.clear();
            rneed.clear();
            for (int f : cur) {
                if (f < nleft[j]) lneed.insert(f);
                else rneed.insert(f - nleft[j]);
            }
            if (kl[j] >= 0 && kr[j] >= 0) { lneed.insert(kl[j]); rneed.insert(kr[j]); }
            cur = lneed;
        }
        const std::set<int>& need = side == 0 ? lneed : rneed;
        const int ncols = (int)tables[side]->names.size();
        if (need.empty() || (int)need.size() >= ncols) return ~0ull;
        uint64_t m = 0;
        int last = 0;
        for (int f : need) {
            if (f < 0) return ~0ull;
            m |= 1ull << (f < 63 ? f : 63);
            last = std::max(last, f);
        }
        *last_keep = (m >> 63) ? ~0u : (uint32_t)last;
        return m;
    } catch (...) {
        *last_keep = ~0u;
        return ~0ull;
    }
}

cq_table* run_join(DevCtx& c, cq_node* q, const cqgpu_table* L, const cqgpu_table* const* rights, int nrights,
                   JoinPartial* part = nullptr) {
    const int nj = q->u.q.join_count;
    if (nj < 1) throw HipError{"run_join without a JOIN"};
    PhaseClock pc;
    PhaseClock* const outer_phase = g_phase;
    g_phase = &pc;
    struct Unset { PhaseClock* o; ~Unset() { g_phase = o; } } unset_{outer_phase};
    if (nrights < nj) throw Ineligible{"join table not given"};
    // across partials the first level runs on the key-routed sides; a chain's later
    // levels join each rank's joined rows with the whole next table (every joined
    // row lives on one rank, so INNER and LEFT need nothing global; the unmatched
    // right rows of a later RIGHT / FULL level are the records no rank matched:
    // g_outer_sets, cqgpu_join_outer_matched / cqgpu_join_outer_set)
    const bool chain = part && nj > 1;
    struct Level {
        const cqgpu_table* R;
        std::string ra;
        bool outer_left, outer_right, keyed, cross;
        int kl, kr, nleft;
        std::set<int> lneed, rneed;
    };
    std::vector<Level> lv(nj);
    std::vector<std::string> wnames = L->names;
    std::string wa = (q->u.q.from && q->u.q.from->u.from.alias) ? q->u.q.from->u.from.alias : "main";
    for (int j = 0; j < nj; j++) {
        cq_node* jn = q->u.q.joins[j];
        if (!jn || jn->kind != CQ_N_JOIN) throw Ineligible{"malformed JOIN"};
        Level& v = lv[j];
        const int kind = jn->u.join.kind;
        v.outer_left = kind == CQ_JOIN_LEFT || kind == CQ_JOIN_FULL;
        v.outer_right = kind == CQ_JOIN_RIGHT || kind == CQ_JOIN_FULL;
        v.R = rights[j];
        if (!v.R) throw Ineligible{"join table failed to load"};
        cq_node* on = jn->u.join.on;
        v.cross = on == nullptr;              // JOIN without ON: the cross product (evaluator_joins.c:42)
        // across partials the first level's JOIN table must be on every rank
        // (cqgpu_route_plan2's cross routing, marked by cqgpu_table_set_replicated)
        if (v.cross && part && j == 0 && !v.R->bcast) throw Ineligible{"JOIN without ON across partials"};
        v.ra = jn->u.join.alias ? jn->u.join.alias : "right";
        cqgpu_table W;                       // the left side's schema at this level
        W.names = wnames;
        // ON operands (anything but `ident = ident` matches no pair)
        v.kl = v.kr = -1;
        if (on && on->kind == CQ_N_CONDITION && on->u.bin.op && !strcmp(on->u.bin.op, "=") && on->u.bin.lhs &&
            on->u.bin.rhs && on->u.bin.lhs->kind == CQ_N_IDENTIFIER && on->u.bin.rhs->kind == CQ_N_IDENTIFIER) {
            v.kl = join_on_index(on->u.bin.lhs->u.text, &W, &W, wa.c_str(), v.R, v.ra.c_str());
            v.kr = join_on_index(on->u.bin.rhs->u.text, v.R, &W, wa.c_str(), v.R, v.ra.c_str());
        }
        v.keyed = v.kl >= 0 && v.kr >= 0;
        if (part && j == 0 && !v.keyed && !v.cross) throw Ineligible{"JOIN without an `ident = ident` ON across partials"};
        if (part && j == 0 && (L->rep_major || v.R->rep_major)) {
            // keys of several value classes, the minority classes replicated to every
            // rank (cqgpu_route_plan2): INNER pairs are exact once the pairs of two
            // replicated records are kept on one rank; an outer join's unmatched rows
            // would need every rank's matches
            if (L->rep_major != v.R->rep_major || !v.keyed) throw HipError{"join sides routed in different modes"};
            if (v.outer_left || v.outer_right)
                throw Ineligible{"an outer JOIN over keys of different value classes across partials"};
        }
        if (part && j > 0 && v.R->gids) throw HipError{"join chain across partials: a later level's table must be whole"};
        v.nleft = (int)wnames.size();
        std::vector<std::string> nn;        // copy_columns_with_prefix (evaluator_joins.c:30-37)
        for (auto& nm : wnames) nn.push_back(wa + "." + nm);
        for (auto& nm : v.R->names) nn.push_back(v.ra + "." + nm);
        wnames.swap(nn);
        wa = "joined";
    }
    // the final joined table's schema
    cqgpu_table J;
    J.cfg = L->cfg;
    J.names = wnames;
    const bool rows = is_row_query(q);
    Compiled C;
    RowPlan RP;
    if (rows) compile_rows(&J, q, C, RP);
    else compile_aggregate(&J, q, C);
    if (part && !rows) {
        part->nacc = C.P.nacc;
        part->nrep = (uint32_t)C.rep_cols.size();
        part->nvla = (uint32_t)C.vla.size();
    }
    if (!rows && nj == 1 && lv[0].keyed && !lv[0].outer_left && !lv[0].outer_right && !L->rep_major &&
        !(part && getenv("CQ_AMD_NO_PART_FAST_JOIN"))) {
        // (partials: the STAR form only, its groups globalised into *part)
        cq_table* fj = run_fast_join(c, q, C, L, lv[0].R, lv[0].kl, lv[0].kr, lv[0].nleft, part, &J.names);
        if (fj == JOIN_PART_DONE) return nullptr;
        if (fj) return fj;
    }
    // columns each level needs, from the last level back
    {
        std::set<int> cur(C.need_cols.begin(), C.need_cols.end());
        cur.insert(C.rep_cols.begin(), C.rep_cols.end());
        for (auto& v : C.vla) cur.insert(v.second);
        cur.insert(RP.cols.begin(), RP.cols.end());
        for (int j = nj - 1; j >= 0; j--) {
            Level& v = lv[j];
            for (int f : cur) {
                if (f < v.nleft) v.lneed.insert(f);
                else v.rneed.insert(f - v.nleft);
            }
            if (v.keyed) { v.lneed.insert(v.kl); v.rneed.insert(v.kr); }
            cur = v.lneed;
        }
    }
    // level 0's left side: the FROM table's columns
    std::unique_ptr<JoinSide> Ap(new JoinSide);
    Ap->cols.assign(lv[0].lneed.begin(), lv[0].lneed.end());
    if (Ap->cols.empty()) Ap->cols.push_back(0);
    load_side(c, L, *Ap);
    std::unique_ptr<JoinSide> Bp;
    DevBuf pairs(8);
    unsigned long long np = 0;
    DevBuf ckey;                             // chain across partials: each joined row's order key
    unsigned long long kspace = 0;           // one past every key of the level so far
    for (int j = 0; j < nj; j++) {
        Level& v = lv[j];
        Bp.reset(new JoinSide);
        Bp->cols.assign(v.rneed.begin(), v.rneed.end());
        if (Bp->cols.empty()) Bp->cols.push_back(0);
        load_side(c, v.R, *Bp);
        // a later RIGHT / FULL level across partials: the ranks' matched records
        const bool probe_here = part && part->probe_level == j;
        const OuterSet* os = nullptr;
        DevBuf gdev, mdev;
        if (part && j > 0 && v.outer_right && !probe_here) {
            auto it = g_outer_sets.find(j);
            if (it == g_outer_sets.end())
                throw Ineligible{"RIGHT/FULL JOIN after the first level across partials without the ranks' matched "
                                 "records (cqgpu_join_outer_set)"};
            if (it->second.matched.size() != Bp->n)
                throw HipError{"join_outer_set: " + std::to_string(it->second.matched.size()) +
                               " flags for a level of " + std::to_string(Bp->n) + " records"};
            os = &it->second;
            DevBuf g(std::max<size_t>(Bp->n, 1));
            std::swap(gdev.p, g.p);
            if (Bp->n)
                HIPCHECK(hipMemcpyAsync(gdev.p, os->matched.data(), Bp->n, hipMemcpyHostToDevice, c.stream));
        }
        if (probe_here) {
            DevBuf mb(std::max<size_t>(Bp->n, 1));
            std::swap(mdev.p, mb.p);
        }
        DevBuf pb(8);
        // a cross join's first level across partials: the JOIN table is whole on every
        // rank, so its unmatched rows (RIGHT / FULL) exist only when the FROM table is
        // empty on every rank, and one rank emits them
        const bool right_rows = !(part && j == 0 && v.cross) || (L->gid_total == 0 && v.R->rep_owner);
        np = build_pairs(c, *Ap, *Bp, v.kl, v.kr, v.keyed, v.outer_left, (v.outer_right && right_rows) || probe_here,
                         pb, v.cross, os ? gdev.as<uint8_t>() : nullptr, os ? os->emit : true,
                         probe_here ? mdev.as<uint8_t>() : nullptr);
        if (part && j == 0 && v.keyed && L->rep_major && !L->rep_owner && np) {
            // pairs of two replicated records: every rank found them, the owner keeps them
            DevBuf fl(np * 4), pos(np * 4), kept(np * 8);
            HIPCHECK(cq_launch_pair_rep_flags(pb.as<uint2>(), np, Ap->cells.as<Cell>(), (uint32_t)Ap->cols.size(),
                                              (uint32_t)Ap->slot(v.kl), Bp->cells.as<Cell>(), (uint32_t)Bp->cols.size(),
                                              (uint32_t)Bp->slot(v.kr), L->rep_major, fl.as<unsigned int>(), c.stream));
            size_t tb = 0;
            HIPCHECK(cq_excl_sum_u32(nullptr, &tb, fl.as<unsigned int>(), pos.as<unsigned int>(), np, c.stream));
            DevBuf temp(tb);
            HIPCHECK(cq_excl_sum_u32(temp.p, &tb, fl.as<unsigned int>(), pos.as<unsigned int>(), np, c.stream));
            HIPCHECK(cq_launch_key_flagged(pb.as<unsigned long long>(), np, fl.as<unsigned int>(), pos.as<unsigned int>(),
                                           kept.as<unsigned long long>(), c.stream));
            unsigned int last[2] = {0, 0};
            HIPCHECK(hipMemcpyAsync(&last[0], pos.as<unsigned int>() + np - 1, 4, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipMemcpyAsync(&last[1], fl.as<unsigned int>() + np - 1, 4, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
            np = (unsigned long long)last[0] + last[1];
            std::swap(pb.p, kept.p);
        }
        if (probe_here) {
            part->probe_out.assign(Bp->n, 0);
            if (Bp->n)
                HIPCHECK(hipMemcpyAsync(part->probe_out.data(), mdev.p, Bp->n, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
            return nullptr;
        }
        HIPCHECK(hipStreamSynchronize(c.stream));       // (gdev is released at the end of this level)
        std::swap(pairs.p, pb.p);
        if (part && j == 0 && v.keyed) {     // even when one side is empty on this rank
            part->lmask |= key_class_mask(c, *Ap, v.kl);
            part->rmask |= key_class_mask(c, *Bp, v.kr);
            if (L->rep_major) part->lmask |= REP_ROUTED;   // the cross-class pairs are exact (replicated)
        }
        if (chain) {                         // route.hip chain_key_kernel
            DevBuf nk((size_t)std::max<unsigned long long>(np, 1) * 8);
            if (j == 0) {
                if ((L->gids && !L->gid_total) || (v.R->gids && !v.R->gid_total))
                    throw HipError{"routed join side without its record total (cqgpu_table_set_record_total)"};
                const unsigned long long nl0 = L->gids ? L->gid_total : Ap->n;
                const unsigned long long nr0 = v.R->gids ? v.R->gid_total : Bp->n;
                if ((unsigned __int128)(nl0 + 1) * (nr0 + 1) >= ((unsigned __int128)1 << 64))
                    throw Ineligible{"join chain across partials: order keys over 64 bits"};
                DevBuf lown, rown;
                const unsigned long long *lg = nullptr, *rg = nullptr;
                side_gids(c, L, Ap->n, lown, &lg);
                side_gids(c, v.R, Bp->n, rown, &rg);
                HIPCHECK(cq_launch_chain_key(pairs.as<uint2>(), np, lg, nl0, nr0 + 1, rg, nr0,
                                             nk.as<unsigned long long>(), c.stream));
                HIPCHECK(hipStreamSynchronize(c.stream));     // lown / rown go out of scope
                kspace = (nl0 + 1) * (nr0 + 1);
            } else {
                const unsigned long long nr = Bp->n;
                if ((unsigned __int128)(kspace + 1) * (nr + 1) >= ((unsigned __int128)1 << 64))
                    throw Ineligible{"join chain across partials: order keys over 64 bits"};
                HIPCHECK(cq_launch_chain_key(pairs.as<uint2>(), np, ckey.as<unsigned long long>(), kspace, nr + 1,
                                             nullptr, nr, nk.as<unsigned long long>(), c.stream));
                HIPCHECK(hipStreamSynchronize(c.stream));     // the previous keys are released below
                kspace = (kspace + 1) * (nr + 1);
            }
            std::swap(ckey.p, nk.p);
        }
        if (j + 1 == nj) break;
        // the joined rows' cells the next levels read: the next left side
        if (np >= (1ull << 32)) throw Ineligible{"intermediate join over 2^32 rows"};
        std::unique_ptr<JoinSide> Wn(new JoinSide);
        Wn->cols.assign(lv[j + 1].lneed.begin(), lv[j + 1].lneed.end());
        if (Wn->cols.empty()) Wn->cols.push_back(0);
        if ((int)Wn->cols.size() > MAX_WIDE) throw Ineligible{"join: more than " + std::to_string(MAX_WIDE) + " columns of one side"};
        Wn->n = (uint32_t)np;
        const JoinMap M = join_map(Wn->cols, v.nleft, *Ap, *Bp);
        DevBuf cells((size_t)std::max<unsigned long long>(np, 1) * Wn->cols.size() * sizeof(Cell));
        std::swap(Wn->cells.p, cells.p);
        if (np) HIPCHECK(cq_launch_join_gather(pairs.as<uint2>(), np, &M, Ap->cells.as<Cell>(), Bp->cells.as<Cell>(),
                                               Wn->cells.as<Cell>(), c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        Ap = std::move(Wn);
    }
    JoinSide& A = *Ap;
    JoinSide& B = *Bp;
    const int nl = lv[nj - 1].nleft;
    const cqgpu_table* R = lv[nj - 1].R;
    g_stats.records = np;
    Literals Lit;
    parse_literals(c, C.lits, Lit);
    for (size_t i = 0; i < Lit.cells.size(); i++) C.P.consts[i] = Lit.cells[i];
    if (rows) {
        // WHERE flags -> output positions -> projection of the window LIMIT keeps
        const JoinMap MW = join_map(C.need_cols, nl, A, B);
        const JoinMap MP = join_map(RP.cols, nl, A, B);
        DevBuf flags(std::max<unsigned long long>(np, 1) * 4), pos(std::max<unsigned long long>(np, 1) * 4);
        unsigned long long npass = 0;
        if (np) {
            HIPCHECK(cq_launch_join_filter(pairs.as<uint2>(), np, &MW, A.cells.as<Cell>(), B.cells.as<Cell>(), &C.P,
                                           flags.as<unsigned int>(), c.stream));
            size_t tb = 0;
            HIPCHECK(cq_excl_sum_u32(nullptr, &tb, flags.as<unsigned int>(), pos.as<unsigned int>(), np, c.stream));
            DevBuf temp(tb);
            HIPCHECK(cq_excl_sum_u32(temp.p, &tb, flags.as<unsigned int>(), pos.as<unsigned int>(), np, c.stream));
            unsigned int last[2] = {0, 0};
            HIPCHECK(hipMemcpyAsync(&last[0], pos.as<unsigned int>() + np - 1, 4, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipMemcpyAsync(&last[1], flags.as<unsigned int>() + np - 1, 4, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
            npass = (unsigned long long)last[0] + last[1];
        }
        if (npass > (unsigned long long)INT32_MAX) throw Ineligible{"more than 2^31-1 result rows"};
        g_stats.groups = npass;
        std::vector<unsigned long long> keys;
        if (part) {   // every passing row with its global order key; the merge sorts, ORDER / LIMIT after
            DevBuf lown, rown, dk(std::max<unsigned long long>(npass, 1) * 8);
            if (chain) {
                HIPCHECK(cq_launch_key_flagged(ckey.as<unsigned long long>(), np, flags.as<unsigned int>(),
                                               pos.as<unsigned int>(), dk.as<unsigned long long>(), c.stream));
            } else {
                const unsigned long long *lg = nullptr, *rg = nullptr;
                side_gids(c, L, A.n, lown, &lg);
                side_gids(c, R, B.n, rown, &rg);
                HIPCHECK(cq_launch_pair_gid_flagged(pairs.as<uint2>(), np, flags.as<unsigned int>(),
                                                    pos.as<unsigned int>(), lg, rg, dk.as<unsigned long long>(),
                                                    c.stream));
            }
            keys.resize(npass);
            if (npass) HIPCHECK(hipMemcpyAsync(keys.data(), dk.p, npass * 8, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
        }
        unsigned long long lo = 0, hi = npass;
        cq_node* sel = q->u.q.select;
        cq_node* ob = q->u.q.order_by;
        const bool ordered = ob && ob->kind == CQ_N_ORDER_BY && ob->u.ord.key;
        const bool distinct = sel && sel->u.sel.distinct;
        bool limited = false;
        if (!part && !ordered && !distinct && (q->u.q.limit >= 0 || q->u.q.offset >= 0)) {
            const unsigned long long off = q->u.q.offset >= 0 ? (unsigned long long)q->u.q.offset : 0;
            const unsigned long long lim = q->u.q.limit >= 0 ? (unsigned long long)q->u.q.limit : npass;
            lo = std::min(off, npass);
            hi = std::min(npass, lo + lim);
            limited = true;
        }
        const int nout = (int)RP.names.size();
        cq_table* res = new_result(RP.names);
        const int nr = (int)(hi - lo);
        res->nrows = res->row_capacity = nr;
        res->rows = (cq_row*)calloc(std::max(nr, 1), sizeof(cq_row));
        if (!nr || !nout) {
            for (int i = 0; i < nr; i++) { res->rows[i].ncols = nout; res->rows[i].values = (cq_value*)calloc(1, sizeof(cq_value)); }
        } else {
            Literals LP;
            parse_literals(c, RP.lits, LP);
            DevBuf dcode(std::max<size_t>(RP.code.size(), 1) * sizeof(Insn)), doff(RP.off.size() * 4);
            if (!RP.code.empty())
                HIPCHECK(hipMemcpyAsync(dcode.p, RP.code.data(), RP.code.size() * sizeof(Insn), hipMemcpyHostToDevice, c.stream));
            HIPCHECK(hipMemcpyAsync(doff.p, RP.off.data(), RP.off.size() * 4, hipMemcpyHostToDevice, c.stream));
            const int batch = 1 << 20;
            DevBuf scratch((size_t)std::min(nr, batch) * std::max(MP.n, 1) * sizeof(Cell));
            DevBuf dout((size_t)std::min(nr, batch) * nout * sizeof(Cell));
            std::vector<Cell> hcells;
            for (int b = 0; b < nr; b += batch) {
                const int m = std::min(batch, nr - b);
                HIPCHECK(cq_launch_join_project(pairs.as<uint2>(), np, flags.as<unsigned int>(), pos.as<unsigned int>(),
                                                lo + b, (uint32_t)m, &MP, A.cells.as<Cell>(), B.cells.as<Cell>(),
                                                dcode.as<Insn>(), doff.as<uint32_t>(), nout, LP.dcells,
                                                scratch.as<Cell>(), dout.as<Cell>(), c.stream));
                hcells.resize((size_t)m * nout);
                HIPCHECK(hipMemcpyAsync(hcells.data(), dout.p, hcells.size() * sizeof(Cell), hipMemcpyDeviceToHost, c.stream));
                HIPCHECK(hipStreamSynchronize(c.stream));
                append_rows(c, res, b, hcells, nout, m);
            }
        }
        if (part) {
            part->names = RP.names;
            part->rows = res;
            part->row_keys.swap(keys);
            return nullptr;
        }
        post_ops(c, res, q, true, limited);
        return res;
    }
    // aggregates over the pairs
    std::vector<HGroup> groups;
    if (!C.group_missing) {
        const JoinMap MA = join_map(C.need_cols, nl, A, B);
        const JoinMap MR = join_map(C.rep_cols, nl, A, B);
        ScanStats st;
        groups = aggregate_pairs(c, C, MA, MR, pairs.as<uint2>(), np, A.cells.as<Cell>(), B.cells.as<Cell>(), st,
                                 part != nullptr);
        if (!C.vla.empty()) {
            std::vector<JoinMap> VM;
            for (auto& v : C.vla) VM.push_back(join_map(std::vector<int>{v.second}, nl, A, B));
            compute_vla_pairs(c, C, MA, VM, pairs.as<uint2>(), np, A.cells.as<Cell>(), B.cells.as<Cell>(), groups,
                              part != nullptr);
        }
        if (part) {
            for (int a = 0; a < C.P.nacc; a++) part->acc_classes[a] = st.acc_classes[a];
            // pair positions -> global (left id, right id) order keys
            std::vector<unsigned long long> pidx;
            for (const HGroup& h : groups) {
                if (h.first != NOPOS) pidx.push_back(h.first);
                for (int a = 0; a < C.P.nacc; a++)
                    if (h.extpos[a] != NOPOS) pidx.push_back(h.extpos[a]);
                for (const HGroup::ClassSplit& cs : h.split)     // (per-class MIN/MAX state)
                    for (int k = 0; k < 3; k++) {
                        if (cs.extpos[k] != NOPOS) pidx.push_back(cs.extpos[k]);
                        if (cs.first[k] != NOPOS) pidx.push_back(cs.first[k]);
                    }
            }
            for (unsigned long long p : pidx)
                if (p >= np) throw HipError{"join partial: pair position out of range"};
            if (!pidx.empty()) {
                DevBuf lown, rown;
                DevBuf dp(pidx.size() * 8), dk(pidx.size() * 8);
                HIPCHECK(hipMemcpyAsync(dp.p, pidx.data(), pidx.size() * 8, hipMemcpyHostToDevice, c.stream));
                if (chain) {
                    HIPCHECK(cq_launch_key_pick(ckey.as<unsigned long long>(), dp.as<unsigned long long>(),
                                                (uint32_t)pidx.size(), dk.as<unsigned long long>(), c.stream));
                } else {
                    const unsigned long long *lg = nullptr, *rg = nullptr;
                    side_gids(c, L, A.n, lown, &lg);
                    side_gids(c, R, B.n, rown, &rg);
                    HIPCHECK(cq_launch_pair_gid(pairs.as<uint2>(), dp.as<unsigned long long>(), (uint32_t)pidx.size(),
                                                lg, rg, dk.as<unsigned long long>(), c.stream));
                }
                std::vector<unsigned long long> keys(pidx.size());
                HIPCHECK(hipMemcpyAsync(keys.data(), dk.p, keys.size() * 8, hipMemcpyDeviceToHost, c.stream));
                HIPCHECK(hipStreamSynchronize(c.stream));
                size_t k = 0;
                for (HGroup& h : groups) {
                    if (h.first != NOPOS) h.first = keys[k++];
                    for (int a = 0; a < C.P.nacc; a++)
                        if (h.extpos[a] != NOPOS) h.extpos[a] = keys[k++];
                    for (HGroup::ClassSplit& cs : h.split)
                        for (int j = 0; j < 3; j++) {
                            if (cs.extpos[j] != NOPOS) cs.extpos[j] = keys[k++];
                            if (cs.first[j] != NOPOS) cs.first[j] = keys[k++];
                        }
                }
            }
        }
    }
    if (part) {
        // a rank that saw no groups still reports the plan's single group (COUNT = 0 ...)
        part->names = J.names;
        part->groups = std::move(groups);
        return nullptr;
    }
    g_stats.groups = groups.size();
    cq_table* res = build_groups(C, groups, Lit, c);
    post_ops(c, res, q);
    return res;
}

// Aggregates the fused scan kernels do not cover (composite and expression GROUP
// BY, evaluator.c:113-212 / evaluator_aggregates.c:179-250): every record's needed
// columns parsed into cells (record-start kernels + cells_kernel), then the pair
// aggregation with one "pair" (row, -) per record.  Groups come back in
// first-appearance order with whole-file byte offsets, like run_aggregate's.
// Range partials of a composite GROUP BY: each group's key becomes its joined key
// text (scan.hip comp_text_kernel, from the group's first record), carried as a
// text key (GK_LONG class) so the dense and blob merges across ranks group by the
// text byte for byte -- create_groups' own identity (evaluator.c:113-212) -- instead
// of by the 128-bit part digest each rank computed (exact even for a digest
// collision between ranks).  Every key of such a plan is composite, so no
// single-column text key can meet these.
void comp_key_texts(DevCtx& c, const cqgpu_table* t, const Compiled& C, std::vector<HGroup>& groups) {
    if (C.P.ngpart < 2 || groups.empty()) return;
    constexpr uint32_t CAP = 4096;
    const uint32_t n = (uint32_t)groups.size();
    std::vector<unsigned long long> recs(n);
    for (uint32_t i = 0; i < n; i++) {
        const HGroup& h = groups[i];
        if (h.first == NOPOS || h.first < t->base_offset || h.first - t->base_offset >= t->n)
            throw HipError{"composite key text: a group without its first record"};
        recs[i] = h.first - t->base_offset;
    }
    const uint32_t nneed = (uint32_t)std::max(C.P.nneed, 1);
    DevBuf drecs((size_t)n * 8), dcells((size_t)n * nneed * sizeof(Cell)), dtext((size_t)n * CAP), dlen((size_t)n * 4);
    HIPCHECK(hipMemcpyAsync(drecs.p, recs.data(), (size_t)n * 8, hipMemcpyHostToDevice, c.stream));
    HIPCHECK(cq_launch_gather(t->g, &C.P, drecs.as<unsigned long long>(), n, dcells.as<Cell>(), c.stream));
    HIPCHECK(cq_launch_comp_text(dcells.as<Cell>(), n, CAP, dtext.as<uint8_t>(), dlen.as<uint32_t>(), c.stream));
    std::vector<uint32_t> lens(n);
    std::vector<uint8_t> text((size_t)n * CAP);
    HIPCHECK(hipMemcpyAsync(lens.data(), dlen.p, (size_t)n * 4, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipMemcpyAsync(text.data(), dtext.p, text.size(), hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    for (uint32_t i = 0; i < n; i++) {
        if (lens[i] == 0xFFFFFFFFu)
            throw Ineligible{"composite GROUP BY across partials: a key text over 4 KiB"};
        HGroup& h = groups[i];
        h.kcls = GK_LONG;
        h.klen = lens[i];
        h.kbytes.assign((const char*)text.data() + (size_t)i * CAP, lens[i]);
        h.kw0 = 0;
        h.kw1 = 0;
    }
}

std::vector<HGroup> run_cells_aggregate(DevCtx& c, const cqgpu_table* t, Compiled& C, Literals& Lit,
                                        ScanStats* st_out = nullptr, bool partial = false) {
    parse_literals(c, C.lits, Lit);
    for (size_t i = 0; i < Lit.cells.size(); i++) C.P.consts[i] = Lit.cells[i];
    std::vector<HGroup> groups;
    if (C.group_missing) return groups;
    JoinSide A, B;
    for (int j : C.need_cols) A.cols.push_back(j);
    for (int j : C.rep_cols) A.cols.push_back(j);
    for (auto& v : C.vla) A.cols.push_back(v.second);
    std::sort(A.cols.begin(), A.cols.end());
    A.cols.erase(std::unique(A.cols.begin(), A.cols.end()), A.cols.end());
    if (A.cols.empty()) A.cols.push_back(0);
    load_side(c, t, A);
    const unsigned long long np = A.n;
    DevBuf pairs(std::max<unsigned long long>(np, 1) * 8), bcells(sizeof(Cell));
    if (np) HIPCHECK(cq_launch_join_fill(nullptr, nullptr, (uint32_t)np, 0, 0, pairs.as<uint2>(), c.stream));
    const int nl = (int)t->names.size();
    const JoinMap MA = join_map(C.need_cols, nl, A, B);
    const JoinMap MR = join_map(C.rep_cols, nl, A, B);
    ScanStats st;
    groups = aggregate_pairs(c, C, MA, MR, pairs.as<uint2>(), np, A.cells.as<Cell>(), bcells.as<Cell>(), st);
    if (!C.vla.empty()) {
        std::vector<JoinMap> VM;
        for (auto& v : C.vla) VM.push_back(join_map(std::vector<int>{v.second}, nl, A, B));
        compute_vla_pairs(c, C, MA, VM, pairs.as<uint2>(), np, A.cells.as<Cell>(), bcells.as<Cell>(), groups, partial);
    }
    if (st_out) *st_out = st;
    g_stats.records = np;
    g_stats.scan_bytes = t->n;
    // row indexes -> whole-file byte offsets of the records
    std::vector<uint32_t> idx;
    for (const HGroup& h : groups) {
        if (h.first != NOPOS) idx.push_back((uint32_t)h.first);
        for (int a = 0; a < C.P.nacc; a++)
            if (h.extpos[a] != NOPOS) idx.push_back((uint32_t)h.extpos[a]);
        for (const HGroup::ClassSplit& cs : h.split)
            for (int k = 0; k < 3; k++) {
                if (cs.extpos[k] != NOPOS) idx.push_back((uint32_t)cs.extpos[k]);
                if (cs.first[k] != NOPOS) idx.push_back((uint32_t)cs.first[k]);
            }
    }
    for (uint32_t i : idx)
        if (i >= np) throw HipError{"cells aggregate: row index out of range"};
    if (!idx.empty()) {
        DevBuf di(idx.size() * 4), dof(idx.size() * 8);
        HIPCHECK(hipMemcpyAsync(di.p, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, c.stream));
        HIPCHECK(cq_launch_gather_codes(A.recs.as<unsigned long long>(), di.as<uint32_t>(), (uint32_t)idx.size(),
                                        dof.as<unsigned long long>(), c.stream));
        std::vector<unsigned long long> off(idx.size());
        HIPCHECK(hipMemcpyAsync(off.data(), dof.p, off.size() * 8, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        size_t k = 0;
        for (HGroup& h : groups) {
            if (h.first != NOPOS) h.first = off[k++] + t->base_offset;
            for (int a = 0; a < C.P.nacc; a++)
                if (h.extpos[a] != NOPOS) h.extpos[a] = off[k++] + t->base_offset;
            for (HGroup::ClassSplit& cs : h.split)
                for (int j = 0; j < 3; j++) {
                    if (cs.extpos[j] != NOPOS) cs.extpos[j] = off[k++] + t->base_offset;
                    if (cs.first[j] != NOPOS) cs.first[j] = off[k++] + t->base_offset;
                }
        }
    }
    return groups;
}

unsigned long long wide_filter(DevCtx& c, const cqgpu_table* t, Compiled& C, DevBuf& out) {
    Literals Lit;
    parse_literals(c, C.lits, Lit);
    for (size_t i = 0; i < Lit.cells.size(); i++) C.P.consts[i] = Lit.cells[i];
    JoinSide A, B;
    A.cols = C.need_cols;
    if (A.cols.empty()) A.cols.push_back(0);
    load_side(c, t, A);
    const uint32_t n = A.n;
    g_stats.records = n;
    g_stats.scan_bytes = t->n;
    g_stats.scan_kernel = 0;
    if (!n) return 0;
    DevBuf pairs((size_t)n * 8), bcells(sizeof(Cell)), flags((size_t)n * 4), pos((size_t)n * 4);
    HIPCHECK(cq_launch_join_fill(nullptr, nullptr, n, 0, 0, pairs.as<uint2>(), c.stream));
    const JoinMap MW = join_map(C.need_cols, (int)t->names.size(), A, B);
    HIPCHECK(cq_launch_join_filter(pairs.as<uint2>(), n, &MW, A.cells.as<Cell>(), bcells.as<Cell>(), &C.P,
                                   flags.as<unsigned int>(), c.stream));
    size_t tb = 0;
    HIPCHECK(cq_excl_sum_u32(nullptr, &tb, flags.as<unsigned int>(), pos.as<unsigned int>(), n, c.stream));
    DevBuf temp(tb);
    HIPCHECK(cq_excl_sum_u32(temp.p, &tb, flags.as<unsigned int>(), pos.as<unsigned int>(), n, c.stream));
    unsigned int last[2] = {0, 0};
    HIPCHECK(hipMemcpyAsync(&last[0], pos.as<unsigned int>() + n - 1, 4, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipMemcpyAsync(&last[1], flags.as<unsigned int>() + n - 1, 4, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    const uint32_t npass = last[0] + last[1];
    g_stats.passed = npass;
    DevBuf perm((size_t)std::max(npass, 1u) * 4), o((size_t)std::max(npass, 1u) * 8);
    if (npass) {
        HIPCHECK(cq_launch_vla_compact(flags.as<unsigned int>(), pos.as<unsigned int>(), n, perm.as<unsigned int>(),
                                       c.stream));
        HIPCHECK(cq_launch_gather_codes(A.recs.as<unsigned long long>(), perm.as<uint32_t>(), npass,
                                        o.as<unsigned long long>(), c.stream));
    }
    HIPCHECK(hipStreamSynchronize(c.stream));
    std::swap(out.p, o.p);
    return npass;
}

// ------------------------------------------------------------------ query dispatch
void check_plan_shape(cq_node* q, const cqgpu_table* t, bool join_ok = false) {
    if (!q || q->kind != CQ_N_QUERY) throw Ineligible{"not a SELECT query"};
    cq_node* f = q->u.q.from;
    if (!f || f->kind != CQ_N_FROM) throw Ineligible{"no FROM clause"};
    if (f->u.from.subquery) throw Ineligible{"FROM subquery"};
    if (q->u.q.join_count > 0 && !join_ok) throw Ineligible{"JOIN"};
    char d = t->cfg.delimiter;
    if (d == '\n' || d == '\r' || is_space((unsigned char)d) || d == t->cfg.quote || d == 0)
        throw Ineligible{"whitespace/quote delimiter"};
}

bool is_row_query(cq_node* q) {      // evaluator.c:259-262: neither GROUP BY nor aggregates
    cq_node* gb = q->u.q.group_by;
    bool grouped = gb && gb->kind == CQ_N_GROUP_BY && gb->u.grp.keys && gb->u.grp.nkeys > 0;
    return !grouped && !has_aggregates(q->u.q.select);
}

cq_table* query_impl(cq_node* q, cqgpu_table* const* tables, int ntables) {
    bump_reset(ctx());
    DevCtx& c = ctx();
    if (ntables < 1 || !tables[0]) throw HipError{"no table"};
    const cqgpu_table* t = tables[0];
    if (q && q->kind == CQ_N_QUERY && q->u.q.join_count > 0) {
        check_plan_shape(q, t, true);
        if (ntables < 2) throw Ineligible{"join table not given"};
        for (int j = 1; j < ntables; j++)
            if (tables[j]) check_plan_shape(q, tables[j], true);
        return run_join(c, q, t, tables + 1, ntables - 1);
    }
    check_plan_shape(q, t);
    if (is_row_query(q)) {
        Compiled C;
        RowPlan R;
        compile_rows(t, q, C, R);
        bool limited = false;
        cq_table* res = run_rows(c, t, C, R, q, &limited);
        post_ops(c, res, q, true, limited);
        return res;
    }
    PhaseClock pc;
    PhaseClock* const outer_phase = g_phase;
    g_phase = &pc;
    struct Unset { PhaseClock* o; ~Unset() { g_phase = o; } } unset_{outer_phase};
    Compiled C;
    compile_aggregate(t, q, C);
    PHASE("compile");
    Literals L;
    std::vector<HGroup> groups;
    if (C.P.ngpart > 0 || C.wide) {
        groups = run_cells_aggregate(c, t, C, L);
    } else {
        try {
            cq_table* direct = nullptr;
            groups = run_aggregate(c, t, C, L, nullptr, nullptr, 0, &direct);
            if (direct) {
                post_ops(c, direct, q);
                PHASE("post");
                return direct;
            }
            compute_vla(c, t, C, groups);
        } catch (MixedExtremes&) {
            groups = run_cells_aggregate(c, t, C, L);
        }
    }
    PHASE("groups");
    g_stats.groups = groups.size();
    cq_table* res = build_groups(C, groups, L, c);
    PHASE("build");
    post_ops(c, res, q);
    PHASE("post");
    return res;
}

cqgpu_table* open_table(const char* path, cq_csv_config cfg) {
    int fd = open(path, O_RDONLY);
    if (fd < 0) return nullptr;
    struct stat sb;
    if (fstat(fd, &sb) < 0 || sb.st_size == 0) { close(fd); return nullptr; }   // mmap.c:80-95
    size_t n = (size_t)sb.st_size;
    void* d = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (d == MAP_FAILED) { close(fd); return nullptr; }
    cqgpu_table* t = nullptr;
    try {
        t = upload((const uint8_t*)d, n, cfg, 0, nullptr, 0, fd, 0);     // bulk bytes by pread
    } catch (...) {
        munmap(d, n);
        close(fd);
        throw;
    }
    munmap(d, n);
    close(fd);
    return t;
}

// ---- range partition (multi-GPU scans) -----------------
bool is_term(uint8_t b) { return b == '\n' || b == '\r'; }

// header record [hl, hh) (csv_load: first non-empty line, csv_reader.c:411-419) and
// the first byte after it and its terminator run (the data region's start)
void header_span(const uint8_t* d, uint64_t n, uint64_t* hl, uint64_t* hh, uint64_t* data0) {
    uint64_t p = 0;
    while (p < n && is_term(d[p])) p++;
    *hl = p;
    while (p < n && !is_term(d[p])) p++;
    *hh = p;
    while (p < n && is_term(d[p])) p++;
    *data0 = p;
}

// the record start at or after the nominal cut c: the byte after the next
// terminator run (c itself when the byte before it ends a record)
uint64_t snap_cut(const uint8_t* d, uint64_t n, uint64_t c) {
    if (c >= n) return n;
    uint64_t s = c;
    if (!(s > 0 && is_term(d[s - 1])))
        while (s < n && !is_term(d[s])) s++;
    while (s < n && is_term(d[s])) s++;
    return s;
}

void range_bounds(const uint8_t* d, uint64_t n, const cq_csv_config& cfg, int rank, int nranks, uint64_t* lo,
                  uint64_t* hi, uint64_t* hl, uint64_t* hh) {
    uint64_t data0;
    header_span(d, n, hl, hh, &data0);
    if (!cfg.has_header) data0 = 0;          // every line is data; the first one still names the columns
    const uint64_t span = n - data0;
    auto cut = [&](int r) -> uint64_t {
        if (r <= 0) return 0;
        if (r >= nranks) return n;
        const uint64_t c = data0 + (uint64_t)((unsigned __int128)span * (unsigned)r / (unsigned)nranks);
        return std::max(snap_cut(d, n, c), data0);
    };
    *lo = cut(rank);
    *hi = cut(rank + 1);
    if (*hi < *lo) *hi = *lo;
}

// ---- device-resident table cache of the drop-in entry point -----------------
// The reference re-reads and re-parses the file on every query (csv_load per
// evaluate_query, evaluator_joins.c:219 for joins).  evaluate_query keeps the
// uploaded bytes resident in HBM between calls instead, keyed by path and the
// file's identity (device, inode, size, mtime in ns) plus the CSV config; a
// changed file misses and is re-uploaded, so results equal a fresh load.
// LRU within a byte budget (CQGPU_TABLE_CACHE_BYTES, default 32 GiB of the 288 GB
// HBM; 0 disables).
struct CacheEnt {
    std::string path;
    uint64_t dev = 0, ino = 0, size = 0;
    int64_t mtime_ns = 0;
    char delim = ',', quote = '"';
    bool header = true;
    cqgpu_table* t = nullptr;
    uint64_t tick = 0;
};
std::vector<CacheEnt> g_cache;
uint64_t g_cache_tick = 0, g_cache_hits = 0;
long long g_cache_limit = -1;           // -1: not read from the environment yet

uint64_t cache_limit() {
    if (g_cache_limit < 0) {
        const char* e = getenv("CQGPU_TABLE_CACHE_BYTES");
        g_cache_limit = e ? (long long)strtoull(e, nullptr, 10) : (32ll << 30);
    }
    return (uint64_t)g_cache_limit;
}

void cache_drop(size_t i) {
    cqgpu_table* t = g_cache[i].t;
    g_cache.erase(g_cache.begin() + (long)i);
    forget_table_bytes(t->dbuf);
    if (t->dbuf) (void)hipFree(t->dbuf);
    if (t->gids) (void)hipFree(t->gids);
    delete t;
}

// *owned: the caller frees the table (not cached)
cqgpu_table* cached_open(const char* path, cq_csv_config cfg, bool* owned) {
    *owned = true;
    const uint64_t lim = cache_limit();
    if (!lim) return open_table(path, cfg);
    struct stat sb;
    if (stat(path, &sb) != 0) return open_table(path, cfg);
    const int64_t mt = (int64_t)sb.st_mtim.tv_sec * 1000000000ll + sb.st_mtim.tv_nsec;
    int dev = 0;
    (void)hipGetDevice(&dev);
    for (size_t i = 0; i < g_cache.size(); i++) {
        CacheEnt& e = g_cache[i];
        if (e.path != path) continue;
        if (e.dev == (uint64_t)sb.st_dev && e.ino == (uint64_t)sb.st_ino && e.size == (uint64_t)sb.st_size &&
            e.mtime_ns == mt && e.delim == cfg.delimiter && e.quote == cfg.quote && e.header == cfg.has_header &&
            e.t->device == dev) {
            e.tick = ++g_cache_tick;
            g_cache_hits++;
            *owned = false;
            return e.t;
        }
        if (e.dev != (uint64_t)sb.st_dev || e.ino != (uint64_t)sb.st_ino || e.size != (uint64_t)sb.st_size ||
            e.mtime_ns != mt) {
            cache_drop(i);          // the file changed: its bytes are stale
            i--;
        }
    }
    cqgpu_table* t = open_table(path, cfg);
    if (!t || t->n > lim) return t;
    uint64_t used = 0;
    for (auto& e : g_cache) used += e.t->n;
    while (!g_cache.empty() && used + t->n > lim) {
        size_t v = 0;
        for (size_t i = 1; i < g_cache.size(); i++)
            if (g_cache[i].tick < g_cache[v].tick) v = i;
        used -= g_cache[v].t->n;
        cache_drop(v);
    }
    CacheEnt e;
    e.path = path;
    e.dev = (uint64_t)sb.st_dev;
    e.ino = (uint64_t)sb.st_ino;
    e.size = (uint64_t)sb.st_size;
    e.mtime_ns = mt;
    e.delim = cfg.delimiter;
    e.quote = cfg.quote;
    e.header = cfg.has_header;
    e.t = t;
    e.tick = ++g_cache_tick;
    g_cache.push_back(e);
    *owned = false;
    return t;
}

}  // namespace

// ================================================================== C ABI
extern "C" {

void cqgpu_cache_clear(void) {
    while (!g_cache.empty()) cache_drop(g_cache.size() - 1);
}

long long cqgpu_set_cache_limit(long long bytes) {
    const long long prev = (long long)cache_limit();
    g_cache_limit = bytes < 0 ? 0 : bytes;
    uint64_t used = 0;
    for (auto& e : g_cache) used += e.t->n;
    while (!g_cache.empty() && used > (uint64_t)g_cache_limit) {
        size_t v = 0;
        for (size_t i = 1; i < g_cache.size(); i++)
            if (g_cache[i].tick < g_cache[v].tick) v = i;
        used -= g_cache[v].t->n;
        cache_drop(v);
    }
    return prev;
}

int cqgpu_cache_info(uint64_t* entries, uint64_t* bytes, uint64_t* hits) {
    uint64_t used = 0;
    for (auto& e : g_cache) used += e.t->n;
    if (entries) *entries = g_cache.size();
    if (bytes) *bytes = used;
    if (hits) *hits = g_cache_hits;
    return 0;
}

cqgpu_table* cqgpu_table_open(const char* path, cq_csv_config cfg) {
    try {
        cqgpu_table* t = open_table(path, cfg);
        if (!t) set_err("Error loading file: %s", path);
        return t;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return nullptr;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return nullptr;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return nullptr;
    }
}

cqgpu_table* cqgpu_table_from_bytes(const void* data, size_t n, cq_csv_config cfg, uint64_t base_offset,
                                    const char* header, size_t header_len) {
    try {
        return upload((const uint8_t*)data, n, cfg, base_offset, header, header_len);
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return nullptr;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return nullptr;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return nullptr;
    }
}

int cqgpu_range_bounds(const void* data, size_t n, cq_csv_config cfg, int rank, int nranks, uint64_t* lo,
                       uint64_t* hi, uint64_t* hdr_lo, uint64_t* hdr_hi) {
    if ((!data && n) || nranks < 1 || rank < 0 || rank >= nranks || !lo || !hi) return -1;
    uint64_t hl, hh;
    range_bounds((const uint8_t*)data, n, cfg, rank, nranks, lo, hi, &hl, &hh);
    if (hdr_lo) *hdr_lo = hl;
    if (hdr_hi) *hdr_hi = hh;
    return 0;
}

cqgpu_table* cqgpu_table_open_range(const char* path, cq_csv_config cfg, int rank, int nranks) {
    g_err.clear();
    if (nranks < 1 || rank < 0 || rank >= nranks) {
        set_err("cq_amd: bad range %d of %d", rank, nranks);
        return nullptr;
    }
    int fd = open(path, O_RDONLY);
    if (fd < 0) { set_err("Error loading file: %s", path); return nullptr; }
    struct stat sb;
    if (fstat(fd, &sb) < 0 || sb.st_size == 0) { close(fd); set_err("Error loading file: %s", path); return nullptr; }
    const size_t n = (size_t)sb.st_size;
    void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) { close(fd); set_err("Error loading file: %s", path); return nullptr; }
    const uint8_t* d = (const uint8_t*)m;
    uint64_t lo, hi, hl, hh;
    range_bounds(d, n, cfg, rank, nranks, &lo, &hi, &hl, &hh);
    madvise((void*)d, n, MADV_NORMAL);
    cqgpu_table* t = nullptr;
    struct CloseFd { int fd; ~CloseFd() { close(fd); } } close_fd{fd};
    try {
        // (the bulk bytes by pread from the range's file offset, upload())
        if (lo == 0) t = upload(d, hi, cfg, 0, nullptr, 0, fd, 0);
        else t = upload(d + lo, hi - lo, cfg, lo, (const char*)d + hl, hh - hl, fd, lo);
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        t = nullptr;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        t = nullptr;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        t = nullptr;
    }
    munmap(m, n);
    return t;
}

uint64_t cqgpu_table_base_offset(const cqgpu_table* t) { return t ? t->base_offset : 0; }

// ---- join-key repartition (multi-GPU JOIN) -----------------------------------
namespace {
// cqgpu_route_plan / cqgpu_route_plan2: rank < 0 = the caller's rank unknown (a JOIN
// without ON is refused); mode 0 = key routing, 1-3 = non-NULL keys of other classes
// to every rank; class_counts (optional): this side's keys per class (NULL, number,
// string, date)
void route_plan_impl(cq_node* q, cqgpu_table* const* tables, int ntables, int side, int nranks, int rank,
                     uint32_t mode, uint64_t* bytes_per_rank, uint64_t* recs_per_rank, uint64_t* class_counts) {
    DevCtx& c = ctx();
    bump_reset(c);
    if (ntables < 2 || !tables[0] || !tables[1] || (side != 0 && side != 1)) throw HipError{"route: bad tables"};
    if (nranks < 1 || nranks > 4096) throw HipError{"route: bad rank count"};
    if (rank >= nranks || mode > 3) throw HipError{"route: bad rank or mode"};
    // the first JOIN's ON keys route both its sides; a chain's later tables stay whole
    if (!q || q->kind != CQ_N_QUERY || q->u.q.join_count < 1 || !q->u.q.joins[0]) throw Ineligible{"no JOIN"};
    check_plan_shape(q, tables[0], true);
    cq_node* jn = q->u.q.joins[0];
    cq_node* on = jn->u.join.on;
    const cqgpu_table* L = tables[0];
    const cqgpu_table* R = tables[1];
    const char* la = (q->u.q.from && q->u.q.from->u.from.alias) ? q->u.q.from->u.from.alias : "main";
    const char* ra = jn->u.join.alias ? jn->u.join.alias : "right";
    int k = -1;
    if (on && on->kind == CQ_N_CONDITION && on->u.bin.op && !strcmp(on->u.bin.op, "=") && on->u.bin.lhs &&
        on->u.bin.rhs && on->u.bin.lhs->kind == CQ_N_IDENTIFIER && on->u.bin.rhs->kind == CQ_N_IDENTIFIER) {
        // same operand binding as run_join (evaluator_joins.c:49-52)
        k = side == 0 ? join_on_index(on->u.bin.lhs->u.text, L, L, la, R, ra)
                      : join_on_index(on->u.bin.rhs->u.text, R, L, la, R, ra);
    }
    // a JOIN without ON (evaluator_joins.c:41: every pair matches): the FROM side
    // stays on its rank, the JOIN side goes to every rank
    const bool cross = on == nullptr && rank >= 0;
    if (k < 0 && !cross) throw Ineligible{"JOIN without an `ident = ident` ON across partials"};
    const bool special = cross || mode != 0;
    if (special && (nranks > 64 || getenv("CQGPU_ROUTE_SORT")))
        throw Ineligible{"replicated join routing over more than 64 ranks"};
    cqgpu_table* t = tables[side];
    auto st = std::make_unique<RouteState>();
    JoinSide S;
    S.cols.push_back(k >= 0 ? k : 0);
    load_side(c, t, S);
    std::swap(st->recs.p, S.recs.p);
    const uint32_t n = S.n;
    st->n = n;
    st->keep = route_keep_mask(q, tables, ntables, side, &st->last_keep);
    std::vector<unsigned long long> per(2 * (size_t)nranks, 0);
    if (n) {
        DevBuf codes((size_t)n * 8), cls((size_t)n * 4), dest((size_t)n * 4), idx((size_t)n * 4),
            len((size_t)n * 4), dst((2 * (size_t)nranks + 2) * 8), pcls(64);
        HIPCHECK(hipMemsetAsync(pcls.p, 0, 16, c.stream));
        HIPCHECK(cq_launch_join_code(S.cells.as<Cell>(), 1, 0, n, codes.as<unsigned long long>(), cls.as<uint32_t>(),
                                     idx.as<uint32_t>(), class_counts && !cross ? pcls.as<unsigned int>() : nullptr,
                                     c.stream));
        if (class_counts && !cross) {
            unsigned int pc4[4] = {0, 0, 0, 0};
            HIPCHECK(hipMemcpyAsync(pc4, pcls.p, 16, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
            for (int j = 0; j < 4; j++) class_counts[j] = pc4[j];
        }
        if (st->keep != ~0ull) {
            DevBuf proj(t->n + 64);
            HIPCHECK(cq_launch_route_project(t->g, st->recs.as<unsigned long long>(), n, t->n, st->keep,
                                             st->last_keep, (uint8_t)t->cfg.delimiter, (uint8_t)t->cfg.quote,
                                             codes.as<unsigned long long>(), cls.as<uint32_t>(), (uint32_t)nranks,
                                             len.as<uint32_t>(), dest.as<uint32_t>(), proj.as<uint8_t>(),
                                             c.stream));
            std::swap(st->proj.p, proj.p);
        } else {
            HIPCHECK(cq_launch_route_len(t->g, st->recs.as<unsigned long long>(), n, codes.as<unsigned long long>(),
                                         cls.as<uint32_t>(), (uint32_t)nranks, len.as<uint32_t>(),
                                         dest.as<uint32_t>(), c.stream));
        }
        if (special)
            HIPCHECK(cq_launch_route_dest_mode(cls.as<uint32_t>(), n, (uint32_t)nranks, cross ? 0u : mode,
                                               cross ? (side == 0 ? (uint32_t)rank : (uint32_t)nranks) : ~0u,
                                               dest.as<uint32_t>(), c.stream));
        if (nranks <= 64 && !getenv("CQGPU_ROUTE_SORT")) {
            // destination runs: per (destination, wave) counts, one exclusive scan each
            // (dest == nranks: the record's copy in every destination's run)
            const uint32_t nw = (uint32_t)(((uint64_t)n + 63) / 64);
            const size_t nrun = (size_t)nranks * nw;
            DevBuf rc(nrun * 8), rbt(nrun * 8), cb(nrun * 8), bb(nrun * 8);
            HIPCHECK(hipMemsetAsync(rc.p, 0, nrun * 8, c.stream));
            HIPCHECK(hipMemsetAsync(rbt.p, 0, nrun * 8, c.stream));
            HIPCHECK(cq_launch_route_runs(dest.as<uint32_t>(), len.as<uint32_t>(), n, nw, (uint32_t)nranks,
                                          rc.as<unsigned long long>(), rbt.as<unsigned long long>(), c.stream));
            size_t tr = 0;
            HIPCHECK(cq_excl_sum_u64(nullptr, &tr, rc.as<unsigned long long>(), cb.as<unsigned long long>(), nrun,
                                     c.stream));
            DevBuf tmp(tr);
            HIPCHECK(cq_excl_sum_u64(tmp.p, &tr, rc.as<unsigned long long>(), cb.as<unsigned long long>(), nrun,
                                     c.stream));
            HIPCHECK(cq_excl_sum_u64(tmp.p, &tr, rbt.as<unsigned long long>(), bb.as<unsigned long long>(), nrun,
                                     c.stream));
            HIPCHECK(cq_launch_route_run_starts(cb.as<unsigned long long>(), bb.as<unsigned long long>(),
                                                rc.as<unsigned long long>(), rbt.as<unsigned long long>(), nw,
                                                (uint32_t)nranks, dst.as<unsigned long long>(), c.stream));
            std::vector<unsigned long long> starts(2 * (size_t)nranks + 2);
            HIPCHECK(hipMemcpyAsync(starts.data(), dst.p, starts.size() * 8, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
            for (int r = 0; r < nranks; r++) {
                per[nranks + r] = starts[r + 1] - starts[r];
                per[r] = starts[nranks + 2 + r] - starts[nranks + 1 + r];
            }
            st->runs = true;
            st->nw = nw;
            st->nranks = (uint32_t)nranks;
            std::swap(st->dest.p, dest.p);
            std::swap(st->len.p, len.p);
            std::swap(st->cbase.p, cb.p);
            std::swap(st->bbase.p, bb.p);
        } else {
        DevBuf dsorted((size_t)n * 4), order((size_t)n * 4), lens((size_t)n * 8), off((size_t)n * 8);
        int bits = 1;
        while ((1 << bits) < nranks) bits++;
        size_t tb = 0;
        HIPCHECK(cq_sort_dest(nullptr, &tb, dest.as<unsigned int>(), dsorted.as<unsigned int>(), idx.as<unsigned int>(),
                              order.as<unsigned int>(), n, bits, c.stream));
        DevBuf temp(tb);
        HIPCHECK(cq_sort_dest(temp.p, &tb, dest.as<unsigned int>(), dsorted.as<unsigned int>(), idx.as<unsigned int>(),
                              order.as<unsigned int>(), n, bits, c.stream));
        HIPCHECK(cq_launch_gather_len(len.as<uint32_t>(), order.as<uint32_t>(), n, lens.as<unsigned long long>(),
                                      c.stream));
        size_t tb2 = 0;
        HIPCHECK(cq_excl_sum_u64(nullptr, &tb2, lens.as<unsigned long long>(), off.as<unsigned long long>(), n,
                                 c.stream));
        DevBuf temp2(tb2);
        HIPCHECK(cq_excl_sum_u64(temp2.p, &tb2, lens.as<unsigned long long>(), off.as<unsigned long long>(), n,
                                 c.stream));
        HIPCHECK(cq_launch_route_bounds(dsorted.as<uint32_t>(), off.as<unsigned long long>(),
                                        lens.as<unsigned long long>(), n, (uint32_t)nranks,
                                        dst.as<unsigned long long>(), c.stream));
        std::vector<unsigned long long> starts(2 * (size_t)nranks + 2);
        HIPCHECK(hipMemcpyAsync(starts.data(), dst.p, starts.size() * 8, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        for (int r = 0; r < nranks; r++) {
            per[nranks + r] = starts[r + 1] - starts[r];
            per[r] = starts[nranks + 2 + r] - starts[nranks + 1 + r];
        }
        std::swap(st->order.p, order.p);
        std::swap(st->len.p, len.p);
        std::swap(st->off.p, off.p);
        }
    }
    st->bytes = 0;
    for (int r = 0; r < nranks; r++) {
        st->bytes += per[r];
        if (bytes_per_rank) bytes_per_rank[r] = per[r];
        if (recs_per_rank) recs_per_rank[r] = per[nranks + r];
    }
    if (class_counts && (!n || cross))
        for (int j = 0; j < 4; j++) class_counts[j] = 0;
    t->route = std::move(st);
}
}  // namespace

int cqgpu_route_plan(cq_node* q, cqgpu_table* const* tables, int ntables, int side, int nranks,
                     uint64_t* bytes_per_rank, uint64_t* recs_per_rank) {
    return cqgpu_route_plan2(q, tables, ntables, side, nranks, -1, 0, bytes_per_rank, recs_per_rank, nullptr) < 0 ? -1
                                                                                                               : 0;
}

int64_t cqgpu_route_plan2(cq_node* q, cqgpu_table* const* tables, int ntables, int side, int nranks, int rank,
                          uint32_t mode, uint64_t* bytes_per_rank, uint64_t* recs_per_rank, uint64_t* class_counts) {
    g_inel.clear();
    g_err.clear();
    try {
        route_plan_impl(q, tables, ntables, side, nranks, rank, mode, bytes_per_rank, recs_per_rank, class_counts);
        return (int64_t)tables[side]->route->n;
    } catch (Ineligible& e) {
        g_inel = e.why;
        set_err("cq_amd: query outside the GPU executor's subset: %s", e.why.c_str());
        return -1;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return -1;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return -1;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return -1;
    }
}

int cqgpu_route_fill(cqgpu_table* t, uint64_t gid_base, void* dev_bytes, uint64_t* dev_gids) {
    g_err.clear();
    try {
        DevCtx& c = ctx();
        if (!t || !t->route) throw HipError{"route_fill without route_plan"};
        RouteState& st = *t->route;
        if (gid_base + st.n >= (1ull << 32)) throw HipError{"route: 2^32 - 1 or more records on a join side"};
        if (st.n) {
            if (!dev_bytes || !dev_gids) throw HipError{"route_fill: null output buffer"};
            const uint8_t* src = st.keep != ~0ull ? st.proj.as<uint8_t>() : t->g;
            if (st.runs)
                HIPCHECK(cq_launch_route_scatter(src, st.recs.as<unsigned long long>(), st.dest.as<uint32_t>(),
                                                 st.len.as<uint32_t>(), st.n, st.nw, st.nranks, t->n,
                                                 st.cbase.as<unsigned long long>(),
                                                 st.bbase.as<unsigned long long>(), gid_base, (uint8_t*)dev_bytes,
                                                 (unsigned long long*)dev_gids, c.stream));
            else
                HIPCHECK(cq_launch_route_copy(src, st.recs.as<unsigned long long>(), st.order.as<uint32_t>(),
                                              st.len.as<uint32_t>(), st.off.as<unsigned long long>(), st.n, gid_base,
                                              (uint8_t*)dev_bytes, (unsigned long long*)dev_gids, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
        }
        t->route.reset();
        return 0;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return -1;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return -1;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return -1;
    }
}

cqgpu_table* cqgpu_table_from_routed(const void* dev_bytes, size_t n, const uint64_t* dev_gids, size_t nrec,
                                     cq_csv_config cfg, const char* header, size_t header_len) {
    g_err.clear();
    cqgpu_table* t = nullptr;
    try {
        DevCtx& c = ctx();
        if (!header) throw HipError{"routed table needs the header record"};
        if ((n && !dev_bytes) || (nrec && !dev_gids)) throw HipError{"routed table: null buffer"};
        t = upload(nullptr, 0, cfg, 0, header, header_len);
        // replace the empty upload with the received bytes (records already '\n'-terminated)
        forget_table_bytes(t->dbuf);
        (void)hipFree(t->dbuf);
        t->dbuf = nullptr;
        HIPCHECK(hipMalloc(&t->dbuf, PAD_BEFORE + n + PAD_AFTER));
        note_table_bytes(t->dbuf, PAD_BEFORE + n + PAD_AFTER);
        HIPCHECK(hipMemsetAsync(t->dbuf, '\n', PAD_BEFORE, c.stream));
        HIPCHECK(hipMemsetAsync(t->dbuf + PAD_BEFORE + n, '\n', PAD_AFTER, c.stream));
        if (n) HIPCHECK(hipMemcpyAsync(t->dbuf + PAD_BEFORE, dev_bytes, n, hipMemcpyDeviceToDevice, c.stream));
        t->g = t->dbuf + PAD_BEFORE;
        t->n = n;
        HIPCHECK(hipMalloc((void**)&t->gids, std::max<size_t>(nrec, 1) * 8));
        if (nrec) HIPCHECK(hipMemcpyAsync(t->gids, dev_gids, nrec * 8, hipMemcpyDeviceToDevice, c.stream));
        t->ngids = nrec;
        // the plan-time sample (a STAR join's key range guess and tag seed)
        if (n) {
            t->sample.resize((size_t)std::min<uint64_t>(n, SAMPLE_BYTES));
            HIPCHECK(hipMemcpyAsync(&t->sample[0], dev_bytes, t->sample.size(), hipMemcpyDeviceToHost, c.stream));
        }
        HIPCHECK(hipStreamSynchronize(c.stream));
        if (n) {   // the scan plans' sampled record shape, as upload() takes it from a file's bytes
            const uint8_t* sp = (const uint8_t*)t->sample.data();
            const uint64_t sn = t->sample.size();
            t->lean_ws = cq_lean_pick_ws(sp, sn);
            t->long_cols = cq_lean_long_cols(sp, sn, (uint8_t)cfg.delimiter);
            t->wide4_cols = cq_cols_longer_than(sp, sn, (uint8_t)cfg.delimiter, 4);
        }
        return t;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        cqgpu_table_free(t);
        return nullptr;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        cqgpu_table_free(t);
        return nullptr;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        cqgpu_table_free(t);
        return nullptr;
    }
}

int cqgpu_table_set_key_stride(cqgpu_table* t, uint32_t stride) {
    g_err.clear();
    if (!t || stride == 0) {
        set_err("cq_amd: %s", "key stride must be at least 1");
        return -1;
    }
    t->key_stride = stride;
    t->key_range.clear();                   // learned ranges assumed the old stride
    return 0;
}

int cqgpu_table_set_replicated(cqgpu_table* t, uint32_t mode, int owner) {
    g_err.clear();
    if (!t || mode > 4) {
        set_err("cq_amd: %s", "table_set_replicated: mode 0-4");
        return -1;
    }
    t->rep_major = mode <= 3 ? mode : 0u;
    t->bcast = mode == 4;
    t->rep_owner = owner != 0;
    return 0;
}

uint32_t cqgpu_route_major(const uint64_t* lcounts, const uint64_t* rcounts) {
    // value_compare (csv_reader.c:126-129): non-NULL keys of different classes are
    // "equal", so such a pair exists iff the sides hold some classes x != y
    bool mixed = false;
    for (int x = 1; x < 4; x++)
        for (int y = 1; y < 4; y++) mixed = mixed || (x != y && lcounts[x] && rcounts[y]);
    if (!mixed) return 0;
    uint32_t best = 1;                     // the class most records hold routes by key
    for (uint32_t k = 2; k < 4; k++)
        if (lcounts[k] + rcounts[k] > lcounts[best] + rcounts[best]) best = k;
    return best;
}

int cqgpu_table_set_record_total(cqgpu_table* t, uint64_t total) {
    g_err.clear();
    if (!t || total < t->ngids) {
        set_err("cq_amd: %s", "record total below the table's own records");
        return -1;
    }
    t->gid_total = total;
    return 0;
}

void cqgpu_table_free(cqgpu_table* t) {
    if (!t) return;
    forget_table_bytes(t->dbuf);
    if (t->dbuf) (void)hipFree(t->dbuf);
    if (t->gids) (void)hipFree(t->gids);
    delete t;
}

size_t cqgpu_table_bytes(const cqgpu_table* t) { return t ? t->n : 0; }
int cqgpu_table_ncols(const cqgpu_table* t) { return t ? (int)t->names.size() : 0; }

void cqgpu_result_free(cq_table* r) {
    if (!r) return;
    // rows and short strings back into this thread's pool (build_direct takes them
    // again: no free / malloc per group and step); the rest to free()
    RowPool& P = g_rowpool;
    for (int i = 0; i < r->nrows; i++) {
        cq_row& row = r->rows[i];
        if (g_rowpool_off || row.ncols != P.ncols || P.vals.size() >= (1u << 16)) {
            free_row(row);
            continue;
        }
        for (int j = 0; j < row.ncols; j++) {
            if (row.values[j].kind != CQ_V_STRING) continue;
            char* sp = row.values[j].u.s;
            if (sp && P.strs.size() < (1u << 17) && malloc_usable_size(sp) >= POOL_STR) P.strs.push_back(sp);
            else free(sp);
        }
        memset(row.values, 0, sizeof(cq_value) * (size_t)std::max(row.ncols, 1));
        P.vals.push_back(row.values);
    }
    free(r->rows);
    for (int i = 0; i < r->ncols; i++) free(r->columns[i].name);
    free(r->columns);
    free(r->filename);
    free(r);
}

cq_table* cqgpu_query(cq_node* q, cqgpu_table* const* tables, int ntables) {
    double t0 = now_ms();
    memset(&g_stats, 0, sizeof g_stats);
    g_inel.clear();
    g_err.clear();
    try {
        cq_table* r = query_impl(q, tables, ntables);
        g_stats.path = 1;
        g_stats.total_ms = now_ms() - t0;
        return r;
    } catch (Ineligible& e) {
        g_inel = e.why;
        if (g_fallback) {
            g_stats.path = 2;
            return g_fallback(q);
        }
        set_err("cq_amd: query outside the GPU executor's subset: %s", e.why.c_str());
        return nullptr;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return nullptr;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return nullptr;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return nullptr;
    }
}

cq_table* evaluate_query(cq_node* q) {
    if (!q) return nullptr;
    if (q->kind != CQ_N_QUERY) {                // DML/DDL/set operations: not the SELECT path
        g_inel = "not a SELECT query";
        if (g_fallback) { g_stats.path = 2; return g_fallback(q); }
        set_err("cq_amd: statement kind %d is outside the GPU executor's subset", q->kind);
        return nullptr;
    }
    cq_node* f = q->u.q.from;
    if (!f || f->kind != CQ_N_FROM) {
        fprintf(stderr, "Error: FROM clause is required\n");
        return nullptr;
    }
    if (!f->u.from.path) {
        g_inel = "FROM subquery";
        if (g_fallback) { g_stats.path = 2; return g_fallback(q); }
        set_err("cq_amd: FROM subquery is outside the GPU executor's subset");
        return nullptr;
    }
    std::vector<cqgpu_table*> tables;
    std::vector<bool> owned;
    std::vector<std::string> paths;
    auto open_one = [&](const char* path) -> cqgpu_table* {
        // a path named twice (FROM and JOIN, or two JOINs) is opened once: a second
        // cache lookup could drop the first entry if the file changed in between
        for (size_t i = 0; i < paths.size(); i++) {
            if (paths[i] == path && tables[i]) {
                tables.push_back(tables[i]);
                owned.push_back(false);
                paths.push_back(path);
                return tables[i];
            }
        }
        paths.push_back(path);
        bool own = true;
        cqgpu_table* t = nullptr;
        try {
            t = cached_open(path, global_csv_config, &own);
        } catch (HipError& e) {
            set_err("cq_amd: %s", e.msg.c_str());
            t = nullptr;
        } catch (std::exception& e) {
            set_err("cq_amd: %s", e.what());
            t = nullptr;
        } catch (...) {
            set_err("cq_amd: %s", "unexpected C++ exception");
            t = nullptr;
        }
        if (!t) set_err("Error loading file: %s", path);
        tables.push_back(t);
        owned.push_back(own);
        return t;
    };
    if (!open_one(f->u.from.path)) {
        fprintf(stderr, "Failed to load table from '%s'\n", f->u.from.path);
        return nullptr;
    }
    for (int j = 0; j < q->u.q.join_count; j++) {
        cq_node* jn = q->u.q.joins[j];
        if (jn && jn->u.join.path) open_one(jn->u.join.path);
        else { tables.push_back(nullptr); owned.push_back(true); paths.push_back(""); }
    }
    cq_table* r = cqgpu_query(q, tables.data(), (int)tables.size());
    for (size_t i = 0; i < tables.size(); i++)
        if (owned[i]) cqgpu_table_free(tables[i]);
    return r;
}

// profiling builds (-DCQ_CLOCKS): per-phase shader cycles of the last scan
int cqgpu_debug_clocks(unsigned long long* out8) {
    for (int i = 0; i < 8; i++) out8[i] = g_clk[i];
    return 0;
}

int cqgpu_last_stats(cqgpu_stats* out) {
    if (!out) return -1;
    *out = g_stats;
    return 0;
}
const char* cqgpu_last_error(void) { return g_err.c_str(); }
const char* cqgpu_last_ineligible(void) { return g_inel.c_str(); }
void cqgpu_set_fallback(cqgpu_fallback_fn fn) { g_fallback = fn; }
int cqgpu_set_scan_kernel(int mode) { return cq_set_scan_mode(mode); }

// plan explanation for a header line, no device needed (planner unit tests)
int cqgpu_explain(cq_node* q, const char* header, cq_csv_config cfg, char* out, size_t cap) {
    try {
        cqgpu_table t;
        t.cfg = cfg;
        size_t hl = strlen(header);
        t.names = split_header(header, header + hl, cfg.delimiter, cfg.quote, cfg.has_header);
        t.wide4_cols = 0;           // (no sample: every field taken as narrow, keys as <= 8 bytes)
        t.long_cols = 0;
        check_plan_shape(q, &t);
        Compiled C;
        std::string s;
        if (is_row_query(q)) {
            RowPlan R;
            compile_rows(&t, q, C, R);
            s = "rows\nneed:";
            for (int col : C.need_cols) s += " " + std::to_string(col);
            s += "\ncols:";
            for (int cidx : R.cols) s += " " + std::to_string(cidx);
            s += "\nnames:";
            for (auto& n : R.names) s += " [" + n + "]";
            s += "\nprogs:";
            for (size_t k = 0; k + 1 < R.off.size(); k++) {
                s += " [";
                for (uint32_t i = R.off[k]; i < R.off[k + 1]; i++)
                    s += (i > R.off[k] ? " " : "") + std::to_string(R.code[i].op) + "/" +
                         std::to_string(R.code[i].a) + "/" + std::to_string(R.code[i].b);
                s += "]";
            }
            s += "\n";
            snprintf(out, cap, "%s", s.c_str());
            return 0;
        }
        compile_aggregate(&t, q, C);
        s = "need:";
        for (int col : C.need_cols) s += " " + std::to_string(col);
        s += "\nprog:";
        for (int i = 0; i < C.P.nprog; i++)
            s += " " + std::to_string(C.P.prog[i].op) + "/" + std::to_string(C.P.prog[i].a) + "/" +
                 std::to_string(C.P.prog[i].b);
        s += "\ngroup_slot: " + std::to_string(C.P.group_slot) + (C.group_missing ? " missing" : "");
        // (the literals typed on the host, as parse_literals types them for a launch)
        for (size_t i = 0; i < C.lits.size() && i < (size_t)MAX_CONST; i++)
            C.P.consts[i] = cq_host_parse_cell((const uint8_t*)C.lits[i].data(), (uint32_t)C.lits[i].size());
        s += "\nfast: " + std::to_string(cq_fast_eligible(&C.P, C.grouped ? 1 : 0, 0));
        s += "\nacc:";
        for (int a = 0; a < C.P.nacc; a++)
            s += " " + std::to_string(C.P.acc[a].kind) + "@" + std::to_string(C.P.acc[a].slot);
        s += "\nouts:";
        for (auto& o : C.outs)
            s += " " + std::to_string((int)o.kind) + ":" + std::to_string(o.acc) + ":" + std::to_string(o.rep);
        s += "\nnames:";
        for (auto& n : C.names) s += " [" + n + "]";
        s += "\nlits:";
        for (auto& l : C.lits) s += " [" + l + "]";
        s += "\n";
        snprintf(out, cap, "%s", s.c_str());
        return 0;
    } catch (Ineligible& e) {
        snprintf(out, cap, "ineligible: %s\n", e.why.c_str());
        return 1;
    } catch (HipError& e) {
        snprintf(out, cap, "error: %s\n", e.msg.c_str());
        return 2;
    } catch (std::exception& e) {
        snprintf(out, cap, "error: %s\n", e.what());
        return 2;
    } catch (...) {
        snprintf(out, cap, "error: %s\n", "unexpected C++ exception");
        return 2;
    }
}

// record start offsets of every data record, in file order (tokenizer check)
size_t cqgpu_debug_all_records(cqgpu_table* t, int method, unsigned long long* out, size_t cap) {
    g_err.clear();
    try {
        DevCtx& c = ctx();
        if (!t) throw HipError{"no table"};
        DevBuf recs;
        const uint32_t n = method == 1 ? all_records_scan(c, t, recs) : all_records(c, t, recs);
        const size_t m = std::min<size_t>(n, cap);
        if (m && out) {
            HIPCHECK(hipMemcpyAsync(out, recs.p, m * 8, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
        }
        return n;
    } catch (Ineligible& e) {
        set_err("cq_amd: %s", e.why.c_str());
        return (size_t)-1;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return (size_t)-1;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return (size_t)-1;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return (size_t)-1;
    }
}

size_t cqgpu_debug_records(cqgpu_table* t, unsigned long long* out, size_t cap) {
    try {
        DevCtx& c = ctx();
        ScanPlan P;
        memset(&P, 0, sizeof P);
        P.delim = (uint8_t)t->cfg.delimiter;
        P.quote = (uint8_t)t->cfg.quote;
        P.n = t->n;
        P.data_begin = t->data_begin;
        P.range_end = t->n;
        P.group_slot = -1;
        TableArena A = make_arena(c, P, 64, 2, 0, 16, t->n + 1);
        unsigned long long* d;
        HIPCHECK(hipMalloc(&d, std::max<size_t>(cap, 1) * 8));
        uint64_t windows = (t->n + 31679) / 31680;
        int grid = (int)std::min<uint64_t>(std::max<uint64_t>(windows, 1), (uint64_t)c.ncu * cq_scan_occupancy(&P, 0));
        HIPCHECK(cq_launch_scan(t->g, &P, &A.gt, A.rt.tag ? &A.rt : nullptr, A.stats, d, cap, 0, grid, c.stream, nullptr, A.slow_list,
                                A.slow_cap));
        ScanStats st;
        HIPCHECK(hipMemcpyAsync(&st, A.stats, sizeof st, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        size_t n = std::min<size_t>(st.rows_emitted, cap);
        HIPCHECK(hipMemcpy(out, d, n * 8, hipMemcpyDeviceToHost));
        HIPCHECK(hipFree(d));
        std::sort(out, out + n);
        return (size_t)st.rows_emitted;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return 0;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return 0;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return 0;
    }
}

// the fused scan kernel's own parsed cells for columns `cols` (scan-path check);
// rows come back in arbitrary order with their record offsets in recs_out
cq_table* cqgpu_debug_scan_cells(cqgpu_table* t, const int* cols, int ncols, unsigned long long* recs_out,
                                 size_t cap) {
    try {
        DevCtx& c = ctx();
        ScanPlan P;
        memset(&P, 0, sizeof P);
        P.delim = (uint8_t)t->cfg.delimiter;
        P.quote = (uint8_t)t->cfg.quote;
        P.n = t->n;
        P.data_begin = t->data_begin;
        P.range_end = t->n;
        P.group_slot = -1;
        if (ncols > MAX_NEED || ncols < 1) throw HipError{"bad column count"};
        P.nneed = ncols;
        for (int i = 0; i < ncols; i++) P.need_col[i] = (int16_t)cols[i];   // ascending expected
        TableArena A = make_arena(c, P, 64, 2, 0, 16, t->n + 1);
        unsigned long long* d;
        Cell* dc;
        HIPCHECK(hipMalloc(&d, std::max<size_t>(cap, 1) * 8));
        HIPCHECK(hipMalloc(&dc, std::max<size_t>(cap, 1) * ncols * sizeof(Cell)));
        uint64_t windows = (t->n + 31679) / 31680;
        int grid = (int)std::min<uint64_t>(std::max<uint64_t>(windows, 1), (uint64_t)c.ncu * cq_scan_occupancy(&P, 0));
        HIPCHECK(cq_launch_scan(t->g, &P, &A.gt, A.rt.tag ? &A.rt : nullptr, A.stats, d, cap, 0, grid, c.stream, dc, A.slow_list,
                                A.slow_cap));
        ScanStats st;
        HIPCHECK(hipMemcpyAsync(&st, A.stats, sizeof st, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        size_t n = std::min<size_t>(st.rows_emitted, cap);
        std::vector<Cell> got(n * ncols);
        HIPCHECK(hipMemcpy(recs_out, d, n * 8, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(got.data(), dc, got.size() * sizeof(Cell), hipMemcpyDeviceToHost));
        std::vector<HCell> h = fetch_cells(c, got);
        HIPCHECK(hipFree(d));
        HIPCHECK(hipFree(dc));
        std::vector<std::string> names(ncols, "c");
        cq_table* r = new_result(names);
        r->nrows = r->row_capacity = (int)n;
        r->rows = (cq_row*)malloc(sizeof(cq_row) * std::max<size_t>(n, 1));
        for (size_t i = 0; i < n; i++) {
            r->rows[i].ncols = ncols;
            r->rows[i].values = (cq_value*)calloc(ncols, sizeof(cq_value));
            for (int j = 0; j < ncols; j++) r->rows[i].values[j] = to_value(h[i * ncols + j]);
        }
        return r;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return nullptr;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return nullptr;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return nullptr;
    }
}

// typed cells of columns `cols` at the given records (parse_value check)
cq_table* cqgpu_debug_cells(cqgpu_table* t, const int* cols, int ncols, const unsigned long long* recs,
                            size_t nrec) {
    try {
        DevCtx& c = ctx();
        ScanPlan RP;
        memset(&RP, 0, sizeof RP);
        RP.delim = (uint8_t)t->cfg.delimiter;
        RP.quote = (uint8_t)t->cfg.quote;
        RP.n = t->n;
        if (ncols > MAX_NEED || ncols < 1) throw HipError{"bad column count"};
        std::vector<int> ord(ncols);
        for (int i = 0; i < ncols; i++) ord[i] = i;
        std::sort(ord.begin(), ord.end(), [&](int a, int b) { return cols[a] < cols[b]; });
        RP.nneed = ncols;
        for (int i = 0; i < ncols; i++) RP.need_col[i] = (int16_t)cols[ord[i]];
        std::vector<Cell> got(std::max<size_t>(nrec, 1) * ncols);
        if (nrec) {
            uint8_t* d;
            HIPCHECK(hipMalloc(&d, nrec * 8 + got.size() * sizeof(Cell) + 64));
            unsigned long long* drecs = (unsigned long long*)d;
            Cell* dcells = (Cell*)(d + ((nrec * 8 + 15) & ~15ull));
            HIPCHECK(hipMemcpyAsync(drecs, recs, nrec * 8, hipMemcpyHostToDevice, c.stream));
            HIPCHECK(cq_launch_gather(t->g, &RP, drecs, (uint32_t)nrec, dcells, c.stream));
            HIPCHECK(hipMemcpyAsync(got.data(), dcells, nrec * ncols * sizeof(Cell), hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
            HIPCHECK(hipFree(d));
        }
        got.resize(nrec * ncols);
        std::vector<HCell> h = fetch_cells(c, got);
        std::vector<std::string> names;
        for (int i = 0; i < ncols; i++) names.push_back(cols[i] < (int)t->names.size() ? t->names[cols[i]] : "?");
        cq_table* r = new_result(names);
        r->nrows = r->row_capacity = (int)nrec;
        r->rows = (cq_row*)malloc(sizeof(cq_row) * std::max<size_t>(nrec, 1));
        for (size_t i = 0; i < nrec; i++) {
            r->rows[i].ncols = ncols;
            r->rows[i].values = (cq_value*)calloc(ncols, sizeof(cq_value));
            for (int j = 0; j < ncols; j++) r->rows[i].values[ord[j]] = to_value(h[i * ncols + j]);
        }
        return r;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return nullptr;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return nullptr;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return nullptr;
    }
}

// ---- partial aggregation across ranks (range-partitioned tables)
// Blob: "CQP1", column names, per-accumulator value classes, then per group its
// key, COUNT, first-row offset (whole-file), SUM/AVG state, MIN/MAX extreme with
// its offset, and representative cells.  Merging is order-free: counts and sums
// add, first offsets and extremes take the (value, offset) minimum, and the
// representative row is the one of the smallest first offset -- what
// create_groups / evaluate_aggregate give on the whole file.
// a chain's later RIGHT / FULL level across partials (include/cqgpu.h)
int cqgpu_join_outer_matched(cq_node* q, cqgpu_table* const* tables, int ntables, int level, const uint8_t** flags,
                             uint64_t* n) {
    g_inel.clear();
    g_err.clear();
    memset(&g_stats, 0, sizeof g_stats);
    static thread_local std::vector<uint8_t> out;
    if (flags) *flags = nullptr;
    if (n) *n = 0;
    try {
        if (!q || q->kind != CQ_N_QUERY || level < 1 || level >= q->u.q.join_count) return 0;
        cq_node* jn = q->u.q.joins[level];
        if (!jn || jn->kind != CQ_N_JOIN) throw Ineligible{"malformed JOIN"};
        if (jn->u.join.kind != CQ_JOIN_RIGHT && jn->u.join.kind != CQ_JOIN_FULL) return 0;
        if (ntables < 2 || !tables || !tables[0]) throw HipError{"no table"};
        DevCtx& c = ctx();
        bump_reset(c);
        check_plan_shape(q, tables[0], true);
        JoinPartial jp;
        jp.probe_level = level;
        (void)run_join(c, q, tables[0], tables + 1, ntables - 1, &jp);
        out.swap(jp.probe_out);
        if (flags) *flags = out.data();
        if (n) *n = out.size();
        return 1;
    } catch (Ineligible& e) {
        g_inel = e.why;
        set_err("cq_amd: query outside the GPU executor's subset: %s", e.why.c_str());
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
    }
    return -1;
}

int cqgpu_join_outer_set(int level, const uint8_t* matched, uint64_t n, int emit) {
    g_err.clear();
    if (level < 1 || (n && !matched)) {
        set_err("cq_amd: %s", "join_outer_set: bad arguments");
        return -1;
    }
    OuterSet& o = g_outer_sets[level];
    o.matched.assign(matched, matched + n);
    o.emit = emit != 0;
    return 0;
}

void cqgpu_join_outer_clear(void) { g_outer_sets.clear(); }

}  // extern "C"

namespace {
// a join partial's "CQJ1" blob (cqgpu_query_partial; the typed exchange's partials too)
void join_blob(const JoinPartial& jp, Blob& b) {
    if (jp.nacc < 0) throw HipError{"join partial: the plan's shape was not recorded"};
    const int nacc = jp.nacc;
    const uint32_t nrep = jp.nrep, nvla = jp.nvla;
    b.d.reserve(256 + (jp.direct ? jp.gblob.size() : jp.groups.size() * (64 + 48 * (size_t)nacc + 24 * (size_t)nrep)));
    b.u32(0x314a5143u);                      // "CQJ1"
    b.u32((uint32_t)jp.names.size());
    for (auto& nm : jp.names) b.str(nm);
    b.u32((uint32_t)nacc);
    for (int a = 0; a < nacc; a++) b.u32(jp.acc_classes[a]);
    b.u32(nrep);
    b.u32(nvla);
    b.u32(jp.lmask);
    b.u32(jp.rmask);
    if (jp.direct) {                          // (run_fast_join wrote the groups already)
        b.u64(jp.ng);
        b.raw(jp.gblob.data(), jp.gblob.size());
    } else {
        b.u64(jp.groups.size());
    }
    for (const HGroup& h : jp.groups) {
        b.u32(h.kcls); b.u32(h.klen); b.u64(h.kw0); b.u64(h.kw1); b.str(h.kbytes);
        b.u64(h.cnt); b.u64(h.first);
        for (int a = 0; a < nacc; a++) {
            b.f64(h.sum[a]); b.u64(h.num[a]); b.u64(h.extpos[a]); b.cell(h.ext[a]);
        }
        for (uint32_t r = 0; r < nrep; r++) b.cell(r < h.reps.size() ? h.reps[r] : HCell());
        for (size_t v = 0; v < nvla; v++) {
            b.f64(h.vsum[v]); b.f64(h.vm2[v]); b.f64(h.vn[v]);
            b.mvals(v < h.mvals.size() ? &h.mvals[v] : nullptr);
        }
        b.split(h.split);
    }
}
}  // namespace

extern "C" {

size_t cqgpu_query_partial(cq_node* q, cqgpu_table* const* tables, int ntables, void** blob_out) {
    if (blob_out) *blob_out = nullptr;
    g_inel.clear();
    g_err.clear();
    memset(&g_stats, 0, sizeof g_stats);     // per call: a caller reads this call's path / kernel kind
    try {
        DevCtx& c = ctx();
        bump_reset(c);
        if (ntables < 1 || !tables[0]) throw HipError{"no table"};
        const cqgpu_table* t = tables[0];
        if (q && q->kind == CQ_N_QUERY && q->u.q.join_count > 0) {
            // repartitioned INNER JOIN: this rank's routed sides (cqgpu_route_* + cqgpu_table_from_routed)
            check_plan_shape(q, t, true);
            if (ntables < 2 || !tables[1]) throw Ineligible{"join table not given"};
            PhaseClock pc;
            g_phase = &pc;
            struct Unset { ~Unset() { g_phase = nullptr; } } unset_;
            JoinPartial jp;
            (void)run_join(c, q, t, tables + 1, ntables - 1, &jp);
            PHASE("join");
            if (jp.rows) {                           // "CQR1": names, then per row its order key and cells
                Blob b;
                b.u32(0x31525143u);
                b.u32((uint32_t)jp.names.size());
                for (auto& nm : jp.names) b.str(nm);
                b.u32(jp.lmask);
                b.u32(jp.rmask);
                const cq_table* r = jp.rows;
                b.u64((uint64_t)r->nrows);
                for (int i = 0; i < r->nrows; i++) {
                    b.u64(jp.row_keys[i]);
                    for (int k = 0; k < r->ncols; k++) b.cell(from_value(r->rows[i].values[k]));
                }
                void* out = malloc(std::max<size_t>(b.d.size(), 1));
                if (!out) throw HipError{"out of host memory"};
                memcpy(out, b.d.data(), b.d.size());
                *blob_out = out;
                return b.d.size();
            }
            Blob b;
            join_blob(jp, b);
            PHASE("serialize");
            void* out = malloc(std::max<size_t>(b.d.size(), 1));
            if (!out) throw HipError{"out of host memory"};
            memcpy(out, b.d.data(), b.d.size());
            *blob_out = out;
            PHASE("blob");
            return b.d.size();
        }
        check_plan_shape(q, t);
        if (is_row_query(q)) {
            // "CQR1" as for joins: this shard's projected rows in file order, each keyed
            // by its record's whole-file byte position; cqgpu_merge_partials orders all
            // ranks' rows by that key (the whole file's record order, build_result's
            // row order) before ORDER BY / DISTINCT / LIMIT
            Compiled C;
            RowPlan R;
            compile_rows(t, q, C, R);
            bool limited = false;
            std::vector<unsigned long long> keys;
            cq_table* r = run_rows(c, t, C, R, q, &limited, &keys);
            struct Free { cq_table* r; ~Free() { cqgpu_result_free(r); } } free_{r};
            Blob b;
            b.u32(0x31525143u);
            b.u32((uint32_t)R.names.size());
            for (auto& nm : R.names) b.str(nm);
            b.u32(0);
            b.u32(0);
            b.u64((uint64_t)r->nrows);
            for (int i = 0; i < r->nrows; i++) {
                b.u64(keys[i]);
                for (int k = 0; k < (int)R.names.size(); k++) b.cell(from_value(r->rows[i].values[k]));
            }
            void* out = malloc(std::max<size_t>(b.d.size(), 1));
            if (!out) throw HipError{"out of host memory"};
            memcpy(out, b.d.data(), b.d.size());
            *blob_out = out;
            return b.d.size();
        }
        Compiled C;
        compile_aggregate(t, q, C);
        Literals L;
        ScanStats st;
        memset(&st, 0, sizeof st);
        std::vector<HGroup> groups;
        if (C.P.ngpart > 0 || C.wide) {
            groups = run_cells_aggregate(c, t, C, L, &st, true);
        } else {
            try {
                groups = run_aggregate(c, t, C, L, &st);
                compute_vla(c, t, C, groups, true);
            } catch (MixedExtremes&) {
                groups = run_cells_aggregate(c, t, C, L, &st, true);
            }
        }
        comp_key_texts(c, t, C, groups);             // (composite keys: their joined texts)
        Blob b;
        b.u32(0x31505143u);                          // "CQP1"
        b.u32((uint32_t)t->names.size());
        for (auto& nm : t->names) b.str(nm);
        b.u32((uint32_t)C.P.nacc);
        for (int a = 0; a < C.P.nacc; a++) b.u32(st.acc_classes[a]);
        const uint32_t nrep = (uint32_t)C.rep_cols.size();
        b.u32(nrep);
        b.u32((uint32_t)C.vla.size());
        b.u64(groups.size());
        for (const HGroup& h : groups) {
            b.u32(h.kcls); b.u32(h.klen); b.u64(h.kw0); b.u64(h.kw1); b.str(h.kbytes);
            b.u64(h.cnt); b.u64(h.first);
            for (int a = 0; a < C.P.nacc; a++) {
                b.f64(h.sum[a]); b.u64(h.num[a]); b.u64(h.extpos[a]); b.cell(h.ext[a]);
            }
            for (uint32_t r = 0; r < nrep; r++) b.cell(r < h.reps.size() ? h.reps[r] : HCell());
            for (size_t v = 0; v < C.vla.size(); v++) {
                b.f64(h.vsum[v]); b.f64(h.vm2[v]); b.f64(h.vn[v]);
                b.mvals(v < h.mvals.size() ? &h.mvals[v] : nullptr);
            }
            b.split(h.split);
        }
        void* out = malloc(std::max<size_t>(b.d.size(), 1));
        if (!out) throw HipError{"out of host memory"};
        memcpy(out, b.d.data(), b.d.size());
        *blob_out = out;
        return b.d.size();
    } catch (Ineligible& e) {
        g_inel = e.why;
        set_err("cq_amd: query outside the GPU executor's subset: %s", e.why.c_str());
        return 0;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return 0;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return 0;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return 0;
    }
}

cq_table* cqgpu_merge_partials(cq_node* q, const void* const* blobs, const size_t* sizes, int nblobs) {
    memset(&g_stats, 0, sizeof g_stats);
    g_inel.clear();
    g_err.clear();
    PhaseClock pc;
    PhaseClock* const outer_phase = g_phase;
    g_phase = &pc;
    struct Unset { PhaseClock* o; ~Unset() { g_phase = o; } } unset_{outer_phase};
    try {
        DevCtx& c = ctx();
        if (nblobs < 1) throw HipError{"no partials"};
        struct Part {
            std::vector<std::string> names;
            std::vector<uint32_t> classes;
        };
        std::vector<Part> parts(nblobs);
        uint32_t nacc = 0, nrep = 0, nvla = 0, magic0 = 0, lmask = 0, rmask = 0;
        uint32_t rep_all = REP_ROUTED;    // every partial's sides routed with replication
        if (sizes[0] >= 4 && *(const uint32_t*)blobs[0] == 0x31525143u) {
            // "CQR1": a row-returning join's rows from every rank, merged in the
            // reference's nested-loop order by their global (left id, right id) keys
            std::vector<std::string> names;
            struct Row { unsigned long long key; std::vector<HCell> cells; };
            std::vector<Row> all;
            for (int bi = 0; bi < nblobs; bi++) {
                Reader r{(const uint8_t*)blobs[bi], sizes[bi], 0};
                if (r.u32() != 0x31525143u) throw HipError{"partials from different plans"};
                std::vector<std::string> nm(r.u32());
                for (auto& x : nm) x = r.str();
                if (bi == 0) names = nm;
                else if (nm != names) throw HipError{"partials from different plans"};
                const uint32_t lm = r.u32();
                lmask |= lm;
                rep_all &= lm;
                rmask |= r.u32();
                const uint64_t nr = r.u64();
                for (uint64_t i = 0; i < nr; i++) {
                    Row row;
                    row.key = r.u64();
                    row.cells.resize(names.size());
                    for (auto& cc : row.cells) cc = r.cell();
                    all.push_back(std::move(row));
                }
            }
            for (int x = 1; x < 4; x++)           // value_compare's cross-class "equal" (csv_reader.c:128)
                for (int y = 1; y < 4; y++)
                    if (x != y && (lmask >> x & 1) && (rmask >> y & 1) && !rep_all)
                        throw Ineligible{"join keys of different value classes across partials"};
            if (all.size() > (size_t)INT32_MAX) throw Ineligible{"more than 2^31-1 result rows"};
            std::stable_sort(all.begin(), all.end(), [](const Row& a, const Row& b) { return a.key < b.key; });
            cq_table* res = new_result(names);
            res->nrows = res->row_capacity = (int)all.size();
            res->rows = (cq_row*)calloc(std::max<size_t>(all.size(), 1), sizeof(cq_row));
            for (size_t i = 0; i < all.size(); i++) {
                res->rows[i].ncols = (int)names.size();
                res->rows[i].values = (cq_value*)calloc(std::max<size_t>(names.size(), 1), sizeof(cq_value));
                for (size_t k = 0; k < names.size(); k++) res->rows[i].values[k] = to_value(all[i].cells[k]);
            }
            post_ops(c, res, q, true, false);
            g_stats.path = 1;
            return res;
        }
        // headers first (the plan, the accumulators' classes); every blob's groups are
        // then parsed straight into the merge, one scratch group at a time
        std::vector<size_t> gat(nblobs, 0);
        std::vector<uint64_t> gcount(nblobs, 0);
        for (int bi = 0; bi < nblobs; bi++) {
            Reader r{(const uint8_t*)blobs[bi], sizes[bi], 0};
            const uint32_t magic = r.u32();
            if (magic != 0x31505143u && magic != 0x314a5143u) throw HipError{"bad partial blob"};
            if (bi == 0) magic0 = magic;
            else if (magic != magic0) throw HipError{"partials from different plans"};
            Part& pt = parts[bi];
            pt.names.resize(r.u32());
            for (auto& nm : pt.names) nm = r.str();
            const uint32_t na = r.u32();
            for (uint32_t a = 0; a < na; a++) pt.classes.push_back(r.u32());
            const uint32_t nr = r.u32();
            const uint32_t nv = r.u32();
            if (magic == 0x314a5143u) {
                const uint32_t lm = r.u32();
                lmask |= lm;
                rep_all &= lm;
                rmask |= r.u32();
            }
            if (bi == 0) { nacc = na; nrep = nr; nvla = nv; }
            else if (pt.names != parts[0].names || na != nacc || nr != nrep || nv != nvla)
                throw HipError{"partials from different plans"};
            if (nv > (uint32_t)MAX_ACC || na > (uint32_t)MAX_ACC) throw HipError{"bad partial blob"};
            gcount[bi] = r.u64();
            gat[bi] = r.o;
        }
        PHASE("merge parse");
        // the plan binds columns by name: compile it against the shards' header
        const bool joined = magic0 == 0x314a5143u;
        if (joined) {
            // value_compare calls keys of different non-NULL classes equal (csv_reader.c:128):
            // such pairs span ranks after a plain hash repartition, so the plan is refused
            // unless every partial's sides were routed with replication (cqgpu_route_plan2)
            for (int x = 1; x < 4; x++)
                for (int y = 1; y < 4; y++)
                    if (x != y && (lmask >> x & 1) && (rmask >> y & 1) && !rep_all)
                        throw Ineligible{"join keys of different value classes across partials"};
        }
        cqgpu_table meta;
        meta.names = parts[0].names;
        check_plan_shape(q, &meta, joined);
        if (is_row_query(q)) throw Ineligible{"row-returning SELECT across partials"};
        Compiled C;
        compile_aggregate(&meta, q, C);
        if ((uint32_t)C.P.nacc != nacc || (uint32_t)C.rep_cols.size() != nrep)
            throw HipError{"partials do not match the plan"};
        // MIN/MAX over several value classes: value_compare calls cells of different
        // classes "equal" (csv_reader.c:128), so the row-order fold keeps the class of
        // the first non-NULL cell and that class's first extreme.  Range partials carry
        // per class the extreme and first position (HGroup::split); a partial that saw
        // one class has that class's extreme only, whose position stands in for the
        // class's first -- ranges are disjoint and ordered, so only the order between
        // partials matters there.  Join partials interleave positions across ranks, so
        // each carries every class's true first position (aggregate_pairs all_splits),
        // as global (left id, right id) order keys.
        bool mixed[MAX_ACC] = {};
        for (uint32_t a = 0; a < nacc; a++) {
            if (C.P.acc[a].kind == ACC_SUM) continue;
            uint32_t m = 0;
            for (auto& pt : parts) m |= pt.classes[a];
            mixed[a] = (m & (m - 1)) != 0;
        }
        auto split_of = [](HGroup& h, int a) -> HGroup::ClassSplit& {
            for (auto& cs : h.split)
                if (cs.acc == a) return cs;
            HGroup::ClassSplit cs;
            cs.acc = a;
            if (h.extpos[a] != NOPOS) {
                const int k = h.ext[a].kind == K_STR ? 1 : h.ext[a].kind == K_DATE ? 2 : 0;
                cs.ext[k] = h.ext[a];
                cs.extpos[k] = cs.first[k] = h.extpos[a];
            }
            h.split.push_back(cs);
            return h.split.back();
        };
        auto better_ext = [&](int a, const HCell& x, unsigned long long xp, const HCell& y, unsigned long long yp) {
            if (xp == NOPOS) return false;
            if (yp == NOPOS) return true;
            const int cv = hcompare(x, y);     // first strictly better wins (evaluator_aggregates.c:311-326)
            return (C.P.acc[a].kind == ACC_MIN ? cv < 0 : cv > 0) || (cv == 0 && xp < yp);
        };
        std::vector<HGroup> merged;
        uint64_t total_groups = 0;
        for (int bi = 0; bi < nblobs; bi++) total_groups += gcount[bi];
        merged.reserve((size_t)std::min<uint64_t>(total_groups, 1u << 22));
        // group identity: class + text for text keys, both words for composite digests,
        // the first word otherwise (raw bytes of a fixed-width key, no decimal formatting);
        // an open-addressing table of merged indexes over the identity's hash
        auto text_key = [](const HGroup& h) { return h.kcls == GK_STR || h.kcls == GK_LONG; };
        auto key_hash = [&](const HGroup& h) {
            uint64_t x = (uint64_t)h.kcls * 0x9E3779B97F4A7C15ull;
            if (text_key(h)) {
                uint64_t f = 1469598103934665603ull;     // FNV-1a of the text
                for (unsigned char ch : h.kbytes) f = (f ^ ch) * 1099511628211ull;
                x ^= f;
            } else {
                x ^= h.kw0 + 0x632BE59BD9B4E019ull;
                if (h.kcls == GK_COMP) x ^= h.kw1 * 0xC2B2AE3D27D4EB4Full;
            }
            x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29;
            return x;
        };
        auto same_key = [&](const HGroup& a, const HGroup& b) {
            if (a.kcls != b.kcls) return false;
            if (text_key(a)) return a.kbytes == b.kbytes;
            return a.kw0 == b.kw0 && (a.kcls != GK_COMP || a.kw1 == b.kw1);
        };
        uint64_t cap = 64;
        while (cap < 2 * std::min<uint64_t>(total_groups, 1ull << 30) + 2) cap <<= 1;
        std::vector<uint32_t> slot_of((size_t)cap, 0u);          // merged index + 1
        HGroup h;                                                // the scratch group
        for (int bi = 0; bi < nblobs; bi++) {
            Reader r{(const uint8_t*)blobs[bi], sizes[bi], gat[bi]};
            for (uint64_t gi = 0; gi < gcount[bi]; gi++) {
                h.kcls = r.u32(); h.klen = r.u32(); h.kw0 = r.u64(); h.kw1 = r.u64(); h.kbytes = r.str();
                h.cnt = r.u64(); h.first = r.u64();
                for (uint32_t a = 0; a < nacc; a++) {
                    h.sum[a] = r.f64(); h.num[a] = r.u64(); h.extpos[a] = r.u64(); h.ext[a] = r.cell();
                }
                h.reps.clear();
                for (uint32_t k = 0; k < nrep; k++) h.reps.push_back(r.cell());
                for (auto& mv : h.mvals) mv.clear();
                for (uint32_t v = 0; v < nvla; v++) {
                    h.vsum[v] = r.f64(); h.vm2[v] = r.f64(); h.vn[v] = r.f64();
                    const uint64_t nv = r.u64();
                    if (nv > (r.n - r.o) / 8) throw HipError{"truncated partial blob"};
                    if (nv) {
                        if (h.mvals.size() <= v) h.mvals.resize(v + 1);
                        h.mvals[v].resize(nv);
                        for (auto& x : h.mvals[v]) x = r.u64();
                    }
                }
                h.split.clear();
                const uint32_t ns = r.u32();
                if (ns > nacc) throw HipError{"bad partial blob"};
                for (uint32_t j = 0; j < ns; j++) {
                    HGroup::ClassSplit cs;
                    cs.acc = (int)r.u32();
                    if (cs.acc < 0 || cs.acc >= (int)nacc) throw HipError{"bad partial blob"};
                    for (int k = 0; k < 3; k++) { cs.ext[k] = r.cell(); cs.extpos[k] = r.u64(); cs.first[k] = r.u64(); }
                    h.split.push_back(cs);
                }
                for (uint32_t a = 0; a < nacc; a++)
                    if (mixed[a]) (void)split_of(h, (int)a);
                uint64_t at = key_hash(h) & (cap - 1);
                while (slot_of[at] && !same_key(merged[slot_of[at] - 1], h)) at = (at + 1) & (cap - 1);
                if (!slot_of[at]) {
                    if (merged.size() >= (size_t)UINT32_MAX - 1) throw Ineligible{"too many groups to merge"};
                    slot_of[at] = (uint32_t)merged.size() + 1;
                    merged.push_back(std::move(h));
                    // (no fresh HGroup: every field the next group uses is parsed over, the
                    // moved-from containers are cleared -- a default HGroup is ~1 KiB to build)
                    h.kbytes.clear();
                    h.reps.clear();
                    h.mvals.clear();
                    h.split.clear();
                    continue;
                }
                HGroup& m = merged[slot_of[at] - 1];
                m.cnt += h.cnt;
                if (h.first < m.first) { m.first = h.first; m.reps = h.reps; }
                for (uint32_t a = 0; a < nacc; a++) {
                    m.sum[a] += h.sum[a];
                    m.num[a] += h.num[a];
                    if (C.P.acc[a].kind == ACC_SUM) continue;
                    if (mixed[a]) {
                        HGroup::ClassSplit& ms = split_of(m, (int)a);
                        const HGroup::ClassSplit& hs = split_of(h, (int)a);
                        for (int k = 0; k < 3; k++) {
                            ms.first[k] = std::min(ms.first[k], hs.first[k]);
                            if (better_ext((int)a, hs.ext[k], hs.extpos[k], ms.ext[k], ms.extpos[k])) {
                                ms.ext[k] = hs.ext[k];
                                ms.extpos[k] = hs.extpos[k];
                            }
                        }
                        continue;
                    }
                    if (better_ext((int)a, h.ext[a], h.extpos[a], m.ext[a], m.extpos[a])) {
                        m.ext[a] = h.ext[a];
                        m.extpos[a] = h.extpos[a];
                    }
                }
                for (uint32_t v = 0; v < nvla; v++) {   // MEDIAN: every value
                    if (v >= h.mvals.size() || h.mvals[v].empty()) continue;
                    if (m.mvals.size() <= v) m.mvals.resize(v + 1);
                    m.mvals[v].insert(m.mvals[v].end(), h.mvals[v].begin(), h.mvals[v].end());
                }
                for (uint32_t v = 0; v < nvla; v++) {   // parallel variance: counts, sums, squared deviations
                    if (h.vn[v] == 0) continue;
                    if (m.vn[v] == 0) { m.vsum[v] = h.vsum[v]; m.vm2[v] = h.vm2[v]; m.vn[v] = h.vn[v]; continue; }
                    const double na = m.vn[v], nb = h.vn[v], n = na + nb;
                    const double d = h.vsum[v] / nb - m.vsum[v] / na;
                    m.vm2[v] += h.vm2[v] + d * d * (na * nb / n);
                    m.vsum[v] += h.vsum[v];
                    m.vn[v] = n;
                }
            }
        }
        for (HGroup& h : merged)           // the mixed-class fold: the first class's extreme
            for (uint32_t a = 0; a < nacc; a++) {
                if (!mixed[a]) continue;
                const HGroup::ClassSplit& cs = split_of(h, (int)a);
                int best = -1;
                for (int k = 0; k < 3; k++)
                    if (cs.first[k] != NOPOS && (best < 0 || cs.first[k] < cs.first[best])) best = k;
                h.ext[a] = best >= 0 ? cs.ext[best] : HCell();
                h.extpos[a] = best >= 0 ? cs.extpos[best] : NOPOS;
            }
        // one group without GROUP BY, present even with no rows
        if (!C.grouped && merged.size() > 1) throw HipError{"partials disagree on the single group"};
        if (C.vla.size() != nvla) throw HipError{"partials do not match the plan"};
        for (HGroup& h : merged)           // population STDDEV / MEDIAN of the merged state
            for (uint32_t v = 0; v < nvla; v++) {
                if (C.vla[v].first == 1) {      // vla_reduce_kernel's MEDIAN over all ranks' values
                    std::vector<unsigned long long> e;
                    if (v < h.mvals.size()) e.swap(h.mvals[v]);
                    std::sort(e.begin(), e.end());
                    const size_t n = e.size();
                    h.vla_ok[v] = n > 0;
                    h.vla[v] = !n ? 0.0 : (n & 1) ? vkey_value(e[n / 2])
                                                  : (vkey_value(e[n / 2 - 1]) + vkey_value(e[n / 2])) / 2.0;
                    continue;
                }
                h.vla_ok[v] = h.vn[v] > 0;
                h.vla[v] = h.vn[v] > 0 ? sqrt(h.vm2[v] / h.vn[v]) : 0.0;
            }
        PHASE("merge groups");
        // first-pair order, by index (an HGroup is large to move; the rows are built in it)
        std::vector<uint32_t> ord(merged.size());
        {
            std::vector<std::pair<unsigned long long, uint32_t>> fk(merged.size());
            for (size_t i = 0; i < fk.size(); i++) fk[i] = {merged[i].first, (uint32_t)i};
            std::sort(fk.begin(), fk.end());             // (ties by index: a stable order)
            for (size_t i = 0; i < fk.size(); i++) ord[i] = fk[i].second;
        }
        PHASE("merge sort");
        Literals L;
        parse_literals(c, C.lits, L);
        PHASE("merge literals");
        g_stats.groups = merged.size();
        cq_table* res = build_groups(C, merged, L, c, &ord);
        PHASE("merge build");
        post_ops(c, res, q);
        PHASE("merge post");
        g_stats.path = 1;
        return res;
    } catch (Ineligible& e) {
        g_inel = e.why;
        set_err("cq_amd: query outside the GPU executor's subset: %s", e.why.c_str());
        return nullptr;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return nullptr;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return nullptr;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return nullptr;
    }
}


// ---- device-side GROUP BY merge for range-partitioned scans (merge.hip) -------
// SURVEY.md section 8e, "RCCL reduce for the final aggregate merge".  The library
// drives the merge as a fixed sequence of collectives that the caller runs over
// RCCL (cqgpu_partial_next / cqgpu_partial_put, cqgpu.h); the sequence depends on
// the plan only, so every rank issues the same collectives.
//   KEYS  all_gather of [m][m key records][long key texts]   -> dictionary (G groups)
//   MIN   all_reduce MIN of the MIN plane  (first positions, per-class firsts, order keys)
//   SUM   all_reduce SUM of the SUM plane  (STDDEV plans: ranks need the global means)
//   STRS  all_gather of the string extremes of groups whose MIN/MAX keeps the string
//         class (text has no fixed-width order key: every rank picks the winner)
//   EXT   all_reduce MIN of masked extreme positions      (MIN/MAX plans)
//   CELL  reduce SUM of the owners' cells to rank 0         (representative / extreme cells)
//   VLA   reduce SUM of the pooled squared deviations      (STDDEV plans)
//   SUMR  reduce SUM of the SUM plane to rank 0            (plans without STDDEV)
//   SIDE  all_gather of the owners' cell texts over 8 bytes (plans with cells)
// Out of this path (blob merge instead): MEDIAN (needs every value), more than 2^29 keys.
namespace {
constexpr uint32_t KEYREC = 32;
struct HKeyRec { uint32_t clslen, pad; uint64_t w0, w1, pad2; };
constexpr unsigned long long ABS64 = 0x7FFFFFFFFFFFFFFFull;        // merge.hip ABSENT
constexpr unsigned long long CELL_PRESENT = 1ull << 63, CELL_LONG = 1ull << 62;
enum : int32_t { COLL_DONE = 0, COLL_ALLGATHER = 1, COLL_ALLREDUCE_MIN_I64 = 2, COLL_ALLREDUCE_SUM_F64 = 3,
                 COLL_REDUCE_SUM_I64 = 4, COLL_REDUCE_SUM_F64 = 5, COLL_DECLINE = 6 };
enum Stage { ST_KEYS, ST_MIN, ST_SUM, ST_STRS, ST_EXT, ST_CELL, ST_VLA, ST_SUMR, ST_SIDE };

// two independent hashes of a long key's bytes (the dictionary's filter before the
// byte compare; identical on every rank)
uint64_t text_hash(const uint8_t* b, uint32_t n, uint64_t seed) {
    uint64_t h = seed ^ n;
    for (uint32_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001B3ull + (h >> 29);
    h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33;
    return h;
}

static int cell_class(const HCell& x) { return x.kind == K_STR ? 1 : x.kind == K_DATE ? 2 : 0; }

// per-class state of MIN/MAX accumulator a (HGroup::split, or the one class a
// single-class partial saw, whose extreme position stands in for its first)
static HGroup::ClassSplit class_split(const HGroup& h, int a) {
    for (const auto& cs : h.split)
        if (cs.acc == a) return cs;
    HGroup::ClassSplit cs;
    cs.acc = a;
    if (h.extpos[a] != NOPOS) {
        const int k = cell_class(h.ext[a]);
        cs.ext[k] = h.ext[a];
        cs.extpos[k] = cs.first[k] = h.extpos[a];
    }
    return cs;
}

// MIN-reduce order key of an extreme cell: value_compare's order within its class
// (numbers as doubles, dates by (y, m, d)), negated for MAX, as a signed 64-bit
// integer.  Strings get a constant: their winner is picked from the gathered texts.
unsigned long long ext_order_key(const HCell& x, bool is_max) {
    const unsigned long long SIGN = 1ull << 63;
    unsigned long long ku = 0;
    switch (cell_class(x)) {
        case 0: {
            double d = x.kind == K_INT ? (double)(long long)x.bits : as_dbl(x.bits);
            if (d == 0) d = 0.0;                             // -0 and 0 compare equal
            const unsigned long long u = dbl_bits(d);
            ku = (u >> 63) ? ~u : (u | SIGN);
            break;
        }
        case 1: return 0;
        default: ku = x.bits; break;                         // (y << 32) | (m << 16) | d
    }
    if (is_max) ku = ~ku;
    return ku ^ SIGN;
}

void enc_cell(const HCell& x, std::string& ltext, unsigned long long* w) {
    const uint64_t len = x.kind == K_STR ? x.s.size() : 0;
    w[0] = CELL_PRESENT | x.kind | (len << 8);
    w[1] = x.bits;
    if (x.kind == K_STR) {
        w[1] = 0;
        if (len <= 8) {
            for (size_t i = 0; i < len; i++) w[1] |= (unsigned long long)(uint8_t)x.s[i] << (8 * i);
        } else {
            w[0] |= CELL_LONG;
            w[1] = ltext.size();
            ltext += x.s;
        }
    }
}
}  // namespace

struct cqgpu_partial {
    Compiled C;
    std::vector<int> mm;                 // MIN/MAX accumulator indexes
    uint32_t W = 1, P = 1, Q = 1, R = 0, NV = 0, VS0 = 0;
    uint32_t m = 0;                      // this rank's groups
    std::vector<uint8_t> keyblob;        // [u64 m][m key records][long key texts]
    std::string ltext;                   // this rank's cell texts over 8 bytes
    DevBuf st_sum, st_min, st_priv;      // this rank's planes, m rows
    std::vector<Stage> stages;
    size_t at = 0;                       // stages[at] is the next to issue
    int32_t op = COLL_DONE;
    uint64_t count = 0;
    bool masked = false;
    // the dictionary (from the gathered key blobs)
    uint32_t nall = 0, G = 0;
    DevBuf all, text, slot_of, first_of, dense_of, flag;
    uint64_t text_bytes = 0;
    DevBuf dsum, dmin, dpriv, dext, dcell, dvla;
    std::vector<uint8_t> side;           // [u32 d][u32 cell][u32 len][bytes] of owned long cells
    std::vector<uint8_t> side_all;       // everyone's, gathered
    std::vector<std::string> mystr;      // per local group and MIN/MAX: its string-class extreme
    std::vector<unsigned long long> mystrpos;
    std::vector<uint32_t> dense_id;      // per local group: its dense id
    std::vector<uint8_t> strs;           // [u32 d][u32 i][u32 len][u64 pos][bytes] candidates
    std::unordered_map<uint64_t, unsigned long long> str_best;   // d * nmm + i -> winner position
};

cqgpu_partial* cqgpu_partial_new(cq_node* q, cqgpu_table* const* tables, int ntables) {
    memset(&g_stats, 0, sizeof g_stats);
    g_inel.clear();
    g_err.clear();
    std::unique_ptr<cqgpu_partial> p(new cqgpu_partial);
    PhaseClock pc;
    PhaseClock* const outer_phase = g_phase;
    g_phase = &pc;
    struct Unset { PhaseClock* o; ~Unset() { g_phase = o; } } unset_{outer_phase};
    try {
        DevCtx& c = ctx();
        bump_reset(c);
        if (ntables < 1 || !tables[0]) throw HipError{"no table"};
        const cqgpu_table* t = tables[0];
        check_plan_shape(q, t);
        if (is_row_query(q)) throw Ineligible{"dense merge: row-returning SELECT"};
        Compiled& C = p->C;
        compile_aggregate(t, q, C);
        for (auto& v : C.vla)
            if (v.first != 0) throw Ineligible{"dense merge: MEDIAN (needs every value)"};
        for (int a = 0; a < C.P.nacc; a++)
            if (C.P.acc[a].kind != ACC_SUM) p->mm.push_back(a);
        const uint32_t nacc = (uint32_t)C.P.nacc, nmm = (uint32_t)p->mm.size();
        p->R = (uint32_t)C.rep_cols.size();
        p->NV = (uint32_t)C.vla.size();
        p->VS0 = 1 + 2 * nacc;
        p->W = p->VS0 + 2 * p->NV;
        p->P = 1 + 6 * nmm;
        p->Q = 1 + 12 * nmm + 2 * p->R + 3 * p->NV;
        Literals L;
        ScanStats st;
        memset(&st, 0, sizeof st);
        std::vector<HGroup> groups;
        if (C.P.ngpart > 0 || C.wide) {
            groups = run_cells_aggregate(c, t, C, L, &st, true);
        } else {
            try {
                groups = run_aggregate(c, t, C, L, &st);
                compute_vla(c, t, C, groups, true);
            } catch (MixedExtremes&) {
                groups = run_cells_aggregate(c, t, C, L, &st, true);
            }
        }
        comp_key_texts(c, t, C, groups);             // (composite keys: their joined texts)
        PHASE("partial scan");
        const uint32_t m = (uint32_t)groups.size();
        p->m = m;
        const uint32_t W = p->W, P = p->P, Q = p->Q, R = p->R, NV = p->NV;
        std::vector<HKeyRec> k(m);
        std::string ktext;
        std::vector<unsigned long long> hs((size_t)m * W), hm((size_t)m * P), hp((size_t)m * Q);
        p->mystr.assign((size_t)m * nmm, std::string());
        p->mystrpos.assign((size_t)m * nmm, NOPOS);
        for (uint32_t j = 0; j < m; j++) {
            const HGroup& h = groups[j];
            // identity as cqgpu_merge_partials': class + text for text keys, class +
            // first word for numbers; long text keys carry their bytes in the blob
            if (h.kcls == GK_LONG) {
                const uint8_t* b = (const uint8_t*)h.kbytes.data();
                const uint32_t n = (uint32_t)h.kbytes.size();
                k[j] = HKeyRec{(GK_LONG << 16) | n, 0, text_hash(b, n, 0x9E3779B97F4A7C15ull), text_hash(b, n, 0x2545F4914F6CDD1Dull),
                               8 + (uint64_t)m * KEYREC + ktext.size()};
                ktext += h.kbytes;
            } else {
                const bool txt = h.kcls == GK_STR || h.kcls == GK_COMP;
                k[j] = HKeyRec{(h.kcls << 16) | (txt ? h.klen : 0u), 0, h.kw0, txt ? h.kw1 : 0ull, 0};
            }
            unsigned long long* s = &hs[(size_t)j * W];
            s[0] = dbl_bits((double)h.cnt);
            for (uint32_t a = 0; a < nacc; a++) {
                s[1 + 2 * a] = dbl_bits(h.sum[a]);
                s[2 + 2 * a] = dbl_bits((double)h.num[a]);
            }
            for (uint32_t v = 0; v < NV; v++) {
                s[p->VS0 + 2 * v] = dbl_bits(h.vn[v]);
                s[p->VS0 + 2 * v + 1] = dbl_bits(h.vsum[v]);
            }
            unsigned long long* mn = &hm[(size_t)j * P];
            unsigned long long* pv = &hp[(size_t)j * Q];
            mn[0] = pv[0] = h.first == NOPOS ? ABS64 : h.first;
            for (uint32_t i = 0; i < nmm; i++) {
                const int a = p->mm[i];
                const HGroup::ClassSplit cs = class_split(h, a);
                for (int kk = 0; kk < 3; kk++) {
                    const bool here = cs.extpos[kk] != NOPOS;
                    const unsigned long long key = here ? ext_order_key(cs.ext[kk], C.P.acc[a].kind == ACC_MAX) : ABS64;
                    mn[1 + 6 * i + kk] = cs.first[kk] == NOPOS ? ABS64 : cs.first[kk];
                    mn[1 + 6 * i + 3 + kk] = key;
                    pv[1 + 12 * i + kk] = key;
                    pv[1 + 12 * i + 3 + kk] = here ? cs.extpos[kk] : ABS64;
                    if (here) enc_cell(cs.ext[kk], p->ltext, &pv[1 + 12 * i + 6 + 2 * kk]);
                    if (here && kk == 1) {
                        p->mystr[(size_t)j * nmm + i] = cs.ext[1].s;
                        p->mystrpos[(size_t)j * nmm + i] = cs.extpos[1];
                    }
                }
            }
            for (uint32_t r = 0; r < R; r++)
                if (r < h.reps.size()) enc_cell(h.reps[r], p->ltext, &pv[1 + 12 * nmm + 2 * r]);
            for (uint32_t v = 0; v < NV; v++) {
                pv[1 + 12 * nmm + 2 * R + 3 * v] = dbl_bits(h.vn[v]);
                pv[1 + 12 * nmm + 2 * R + 3 * v + 1] = dbl_bits(h.vsum[v]);
                pv[1 + 12 * nmm + 2 * R + 3 * v + 2] = dbl_bits(h.vm2[v]);
            }
        }
        p->keyblob.resize(8 + (size_t)m * KEYREC + ktext.size());
        const uint64_t m64 = m;
        memcpy(p->keyblob.data(), &m64, 8);
        if (m) memcpy(p->keyblob.data() + 8, k.data(), (size_t)m * KEYREC);
        if (!ktext.empty()) memcpy(p->keyblob.data() + 8 + (size_t)m * KEYREC, ktext.data(), ktext.size());
        DevBuf a(std::max<size_t>(hs.size() * 8, 64)), b(std::max<size_t>(hm.size() * 8, 64)),
            r(std::max<size_t>(hp.size() * 8, 64));
        std::swap(p->st_sum.p, a.p); std::swap(p->st_min.p, b.p); std::swap(p->st_priv.p, r.p);
        if (m) {
            HIPCHECK(hipMemcpyAsync(p->st_sum.p, hs.data(), hs.size() * 8, hipMemcpyHostToDevice, c.stream));
            HIPCHECK(hipMemcpyAsync(p->st_min.p, hm.data(), hm.size() * 8, hipMemcpyHostToDevice, c.stream));
            HIPCHECK(hipMemcpyAsync(p->st_priv.p, hp.data(), hp.size() * 8, hipMemcpyHostToDevice, c.stream));
        }
        HIPCHECK(hipStreamSynchronize(c.stream));
        PHASE("partial planes");
        p->stages = {ST_KEYS, ST_MIN};
        if (NV) p->stages.push_back(ST_SUM);
        if (nmm) p->stages.push_back(ST_STRS);
        if (nmm) p->stages.push_back(ST_EXT);
        if (R + nmm) p->stages.push_back(ST_CELL);
        if (NV) p->stages.push_back(ST_VLA);
        if (!NV) p->stages.push_back(ST_SUMR);
        if (R + nmm) p->stages.push_back(ST_SIDE);
        return p.release();
    } catch (Ineligible& e) {
        g_inel = e.why;
        set_err("cq_amd: query outside the dense merge: %s", e.why.c_str());
        return nullptr;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return nullptr;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return nullptr;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return nullptr;
    }
}

namespace {
// the dictionary from the gathered key blobs: records compacted in rank order,
// long-key text offsets rebased into the concatenation, then merge.hip's build
// (dense id = rank of a key's first occurrence) and this rank's planes scattered
// into G-row dense planes (rows of absent groups hold the planes' identities)
bool build_dictionary(DevCtx& c, cqgpu_partial* p, const uint8_t* cat, const uint64_t* sizes, int rank, int world) {
    std::vector<uint64_t> off(world + 1, 0), ms(world, 0);
    for (int r = 0; r < world; r++) off[r + 1] = off[r] + sizes[r];
    for (int r = 0; r < world; r++) {
        if (sizes[r] < 8) throw HipError{"partial_next: bad key blob"};
        HIPCHECK(hipMemcpyAsync(&ms[r], cat + off[r], 8, hipMemcpyDeviceToHost, c.stream));
    }
    HIPCHECK(hipStreamSynchronize(c.stream));
    uint64_t nall = 0, mine = 0;
    for (int r = 0; r < world; r++) {
        if (8 + ms[r] * KEYREC > sizes[r]) throw HipError{"partial_next: bad key blob"};
        if (r < rank) mine += ms[r];
        nall += ms[r];
    }
    if (ms[rank] != p->m) throw HipError{"partial_next: the gathered blob of this rank is not its own"};
    // the table holds 2 * nall slots of 32-bit indexes
    if (nall >= (1ull << 29)) return false;
    const uint32_t n = (uint32_t)nall;
    DevBuf all(std::max<size_t>((size_t)n * KEYREC, 64)), text(std::max<uint64_t>(off[world], 64));
    HIPCHECK(hipMemcpyAsync(text.p, cat, off[world], hipMemcpyDeviceToDevice, c.stream));
    uint64_t at = 0;
    for (int r = 0; r < world; r++) {
        if (!ms[r]) continue;
        uint8_t* dst = all.as<uint8_t>() + at * KEYREC;
        HIPCHECK(hipMemcpyAsync(dst, cat + off[r] + 8, ms[r] * KEYREC, hipMemcpyDeviceToDevice, c.stream));
        HIPCHECK(cq_launch_rebase(dst, (uint32_t)ms[r], off[r], c.stream));
        at += ms[r];
    }
    uint64_t cap = 64;
    while (cap < 2 * (uint64_t)n) cap <<= 1;
    DevBuf st((size_t)cap * 4), ro((size_t)cap * 4), fo((size_t)cap * 4), so(std::max<size_t>((size_t)n * 4, 4)),
        fl(std::max<size_t>((size_t)n * 4, 4)), de(std::max<size_t>((size_t)n * 4, 4)), err(64);
    HIPCHECK(hipMemsetAsync(st.p, 0, (size_t)cap * 4, c.stream));
    HIPCHECK(hipMemsetAsync(fo.p, 0xFF, (size_t)cap * 4, c.stream));
    HIPCHECK(hipMemsetAsync(err.p, 0, 4, c.stream));
    HIPCHECK(cq_launch_dict_build(all.p, text.p, n, st.as<uint32_t>(), ro.as<uint32_t>(), fo.as<uint32_t>(),
                                  (uint32_t)cap, so.as<uint32_t>(), err.as<unsigned int>(), c.stream));
    HIPCHECK(cq_launch_dict_flag(so.as<uint32_t>(), fo.as<uint32_t>(), n, fl.as<uint32_t>(), c.stream));
    size_t tb = 0;
    HIPCHECK(cq_excl_sum_u32(nullptr, &tb, fl.as<unsigned int>(), de.as<unsigned int>(), n, c.stream));
    DevBuf temp(std::max<size_t>(tb, 16));
    HIPCHECK(cq_excl_sum_u32(temp.p, &tb, fl.as<unsigned int>(), de.as<unsigned int>(), n, c.stream));
    unsigned int e = 0, last[2] = {0, 0};
    HIPCHECK(hipMemcpyAsync(&e, err.p, 4, hipMemcpyDeviceToHost, c.stream));
    if (n) {
        HIPCHECK(hipMemcpyAsync(&last[0], de.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipMemcpyAsync(&last[1], fl.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, c.stream));
    }
    HIPCHECK(hipStreamSynchronize(c.stream));
    if (e) throw HipError{"partial_next: key table full or insert timeout"};
    const uint32_t G = last[0] + last[1];
    p->nall = n;
    p->G = G;
    p->text_bytes = off[world];
    std::swap(p->all.p, all.p); std::swap(p->text.p, text.p); std::swap(p->slot_of.p, so.p);
    std::swap(p->first_of.p, fo.p); std::swap(p->dense_of.p, de.p); std::swap(p->flag.p, fl.p);
    // G-row planes: identities first, then this rank's rows
    const uint32_t W = p->W, P = p->P, Q = p->Q, nmm = (uint32_t)p->mm.size(), C = p->R + nmm;
    DevBuf ds(std::max<size_t>((size_t)G * W * 8, 64)), dm(std::max<size_t>((size_t)G * P * 8, 64)),
        dp(std::max<size_t>((size_t)G * Q * 8, 64)), dx(std::max<size_t>((size_t)G * nmm * 8, 64)),
        dc(std::max<size_t>((size_t)G * C * 16, 64)), dv(std::max<size_t>((size_t)G * p->NV * 8, 64));
    std::vector<unsigned long long> rows(W + P + Q, 0);
    for (uint32_t w = 0; w < P; w++) rows[W + w] = ABS64;
    rows[W + P] = ABS64;                                     // private: first, then per MIN/MAX keys
    for (uint32_t i = 0; i < nmm; i++)                       // and positions absent, cells / moments 0
        for (int kk = 0; kk < 6; kk++) rows[W + P + 1 + 12 * i + kk] = ABS64;
    DevBuf drow(rows.size() * 8), did(std::max<size_t>((size_t)p->m * 4, 64));
    HIPCHECK(hipMemcpyAsync(drow.p, rows.data(), rows.size() * 8, hipMemcpyHostToDevice, c.stream));
    HIPCHECK(cq_launch_fill_rows(ds.as<unsigned long long>(), G, W, drow.as<unsigned long long>(), c.stream));
    HIPCHECK(cq_launch_fill_rows(dm.as<unsigned long long>(), G, P, drow.as<unsigned long long>() + W, c.stream));
    HIPCHECK(cq_launch_fill_rows(dp.as<unsigned long long>(), G, Q, drow.as<unsigned long long>() + W + P, c.stream));
    HIPCHECK(cq_launch_dict_scatter(p->slot_of.as<uint32_t>(), p->first_of.as<uint32_t>(), p->dense_of.as<uint32_t>(),
                                    (uint32_t)mine, p->m, p->st_sum.as<unsigned long long>(),
                                    p->st_min.as<unsigned long long>(), p->st_priv.as<unsigned long long>(), W, P, Q,
                                    ds.as<unsigned long long>(), dm.as<unsigned long long>(),
                                    dp.as<unsigned long long>(), did.as<uint32_t>(), c.stream));
    p->dense_id.resize(p->m);
    if (p->m)
        HIPCHECK(hipMemcpyAsync(p->dense_id.data(), did.p, (size_t)p->m * 4, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    std::swap(p->dsum.p, ds.p); std::swap(p->dmin.p, dm.p); std::swap(p->dpriv.p, dp.p);
    std::swap(p->dext.p, dx.p); std::swap(p->dcell.p, dc.p); std::swap(p->dvla.p, dv.p);
    return true;
}

// the owners' cells and STDDEV terms (merge.hip cell_mask_kernel), and the side blob
// of this rank's owned cell texts over 8 bytes
void mask_cells(DevCtx& c, cqgpu_partial* p) {
    if (p->masked) return;
    const uint32_t nmm = (uint32_t)p->mm.size(), C = p->R + nmm;
    HIPCHECK(cq_launch_cell_mask(p->dmin.as<unsigned long long>(), p->dext.as<unsigned long long>(),
                                 p->dpriv.as<unsigned long long>(), p->dsum.as<double>(), p->G, p->P, p->Q, p->W, nmm,
                                 p->R, p->NV, p->VS0, p->dcell.as<unsigned long long>(), p->dvla.as<double>(),
                                 c.stream));
    std::vector<unsigned long long> cells((size_t)p->G * C * 2);
    if (!cells.empty())
        HIPCHECK(hipMemcpyAsync(cells.data(), p->dcell.p, cells.size() * 8, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    p->side.clear();
    auto u32 = [&](uint32_t v) { p->side.insert(p->side.end(), (uint8_t*)&v, (uint8_t*)&v + 4); };
    for (size_t i = 0; i < cells.size() / 2; i++) {
        const unsigned long long w0 = cells[2 * i], w1 = cells[2 * i + 1];
        if (!(w0 & CELL_PRESENT) || !(w0 & CELL_LONG)) continue;
        const uint32_t len = (uint32_t)((w0 >> 8) & 0xFFFFFFFFull);
        if (w1 + len > p->ltext.size()) throw HipError{"partial_next: bad cell text offset"};
        u32((uint32_t)(i / C));
        u32((uint32_t)(i % C));
        u32(len);
        p->side.insert(p->side.end(), p->ltext.begin() + w1, p->ltext.begin() + w1 + len);
    }
    p->masked = true;
}
}  // namespace

namespace {
// this rank's string-class extremes of the (group, MIN/MAX) pairs whose result keeps
// the string class (the class whose first cell comes first, from the global MIN plane)
void string_candidates(DevCtx& c, cqgpu_partial* p) {
    const uint32_t nmm = (uint32_t)p->mm.size(), P = p->P;
    std::vector<unsigned long long> mn((size_t)p->G * P);
    if (!mn.empty()) HIPCHECK(hipMemcpyAsync(mn.data(), p->dmin.p, mn.size() * 8, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    p->strs.clear();
    for (uint32_t j = 0; j < p->m; j++)
        for (uint32_t i = 0; i < nmm; i++) {
            if (p->mystrpos[(size_t)j * nmm + i] == NOPOS) continue;
            const uint32_t d = p->dense_id[j];
            const unsigned long long* cf = &mn[(size_t)d * P + 1 + 6 * i];
            int best = -1;
            for (int k = 0; k < 3; k++)
                if (cf[k] != ABS64 && (best < 0 || (long long)cf[k] < (long long)cf[best])) best = k;
            if (best != 1) continue;
            const std::string& t = p->mystr[(size_t)j * nmm + i];
            const uint32_t h[3] = {d, i, (uint32_t)t.size()};
            const unsigned long long pos = p->mystrpos[(size_t)j * nmm + i];
            p->strs.insert(p->strs.end(), (const uint8_t*)h, (const uint8_t*)h + 12);
            p->strs.insert(p->strs.end(), (const uint8_t*)&pos, (const uint8_t*)&pos + 8);
            p->strs.insert(p->strs.end(), t.begin(), t.end());
        }
}

// every rank's candidates -> per (group, MIN/MAX) the winner: strcmp order (value_compare
// on strings), the first position among equals (evaluator_aggregates.c:311-326)
void string_winners(cqgpu_partial* p, const uint8_t* all, size_t n) {
    const uint32_t nmm = (uint32_t)p->mm.size();
    struct Best { HCell v; unsigned long long pos; };
    std::unordered_map<uint64_t, Best> best;
    for (size_t o = 0; o + 20 <= n;) {
        uint32_t h[3];
        unsigned long long pos;
        memcpy(h, all + o, 12);
        memcpy(&pos, all + o + 12, 8);
        o += 20;
        if (o + h[2] > n || h[0] >= p->G || h[1] >= nmm) throw HipError{"partial_next: bad string candidates"};
        HCell x;
        x.kind = K_STR;
        x.s.assign((const char*)all + o, h[2]);
        o += h[2];
        const bool is_max = p->C.P.acc[p->mm[h[1]]].kind == ACC_MAX;
        const uint64_t key = (uint64_t)h[0] * nmm + h[1];
        auto it = best.find(key);
        if (it == best.end()) { best.emplace(key, Best{x, pos}); continue; }
        const int cv = hcompare(x, it->second.v);
        if ((is_max ? cv > 0 : cv < 0) || (cv == 0 && pos < it->second.pos)) it->second = Best{x, pos};
    }
    p->str_best.clear();
    for (auto& kv : best) p->str_best[kv.first] = kv.second.pos;
}
}  // namespace

int cqgpu_partial_next(cqgpu_partial* p, const void* result, const uint64_t* result_sizes, int rank, int world,
                       cqgpu_coll* next) {
    g_err.clear();
    try {
        if (!p || !next || world < 1 || rank < 0 || rank >= world) throw HipError{"partial_next: bad arguments"};
        DevCtx& c = ctx();
        const uint32_t G = p->G, nmm = (uint32_t)p->mm.size(), C = p->R + nmm;
        // 1. take the result of the collective issued last
        if (p->at > 0) {
            const Stage done = p->stages[p->at - 1];
            const size_t bytes = p->count * (done == ST_KEYS || done == ST_SIDE || done == ST_STRS ? 1 : 8);
            if (!result && bytes) throw HipError{"partial_next: no result buffer"};
            DevBuf* into = nullptr;
            switch (done) {
                case ST_KEYS:
                    if (!result_sizes) throw HipError{"partial_next: no gathered sizes"};
                    if (!build_dictionary(c, p, (const uint8_t*)result, result_sizes, rank, world)) {
                        next->op = COLL_DECLINE;
                        next->count = 0;
                        p->op = COLL_DECLINE;
                        return 0;
                    }
                    break;
                case ST_MIN: into = &p->dmin; break;
                case ST_SUM: case ST_SUMR: into = &p->dsum; break;
                case ST_EXT: into = &p->dext; break;
                case ST_CELL: into = &p->dcell; break;
                case ST_VLA: into = &p->dvla; break;
                case ST_STRS: {
                    if (!result_sizes) throw HipError{"partial_next: no gathered sizes"};
                    uint64_t tot = 0;
                    for (int r = 0; r < world; r++) tot += result_sizes[r];
                    std::vector<uint8_t> h(tot);
                    if (tot) HIPCHECK(hipMemcpyAsync(h.data(), result, tot, hipMemcpyDeviceToHost, c.stream));
                    HIPCHECK(hipStreamSynchronize(c.stream));
                    string_winners(p, h.data(), h.size());
                    break;
                }
                case ST_SIDE: {
                    if (!result_sizes) throw HipError{"partial_next: no gathered sizes"};
                    uint64_t tot = 0;
                    for (int r = 0; r < world; r++) tot += result_sizes[r];
                    p->side_all.resize(tot);
                    if (tot) HIPCHECK(hipMemcpyAsync(p->side_all.data(), result, tot, hipMemcpyDeviceToHost, c.stream));
                    HIPCHECK(hipStreamSynchronize(c.stream));
                    break;
                }
            }
            if (into && bytes) {
                HIPCHECK(hipMemcpyAsync(into->p, result, bytes, hipMemcpyDeviceToDevice, c.stream));
                HIPCHECK(hipStreamSynchronize(c.stream));
            }
        }
        // 2. the next collective
        if (p->at >= p->stages.size()) {
            p->op = next->op = COLL_DONE;
            p->count = next->count = 0;
            return 0;
        }
        const uint32_t g = p->G;
        (void)G;
        switch (p->stages[p->at]) {
            case ST_KEYS: p->op = COLL_ALLGATHER; p->count = p->keyblob.size(); break;
            case ST_MIN: p->op = COLL_ALLREDUCE_MIN_I64; p->count = (uint64_t)g * p->P; break;
            case ST_SUM: p->op = COLL_ALLREDUCE_SUM_F64; p->count = (uint64_t)g * p->W; break;
            case ST_STRS:
                string_candidates(c, p);
                p->op = COLL_ALLGATHER;
                p->count = p->strs.size();
                break;
            case ST_EXT:
                HIPCHECK(cq_launch_ext_mask(p->dmin.as<unsigned long long>(), p->dpriv.as<unsigned long long>(), g, p->P,
                                            p->Q, nmm, p->dext.as<unsigned long long>(), c.stream));
                if (!p->str_best.empty()) {       // string winners: every rank already knows the position
                    std::vector<unsigned long long> ex((size_t)g * nmm);
                    HIPCHECK(hipMemcpyAsync(ex.data(), p->dext.p, ex.size() * 8, hipMemcpyDeviceToHost, c.stream));
                    HIPCHECK(hipStreamSynchronize(c.stream));
                    for (auto& kv : p->str_best) ex[kv.first] = kv.second;
                    HIPCHECK(hipMemcpyAsync(p->dext.p, ex.data(), ex.size() * 8, hipMemcpyHostToDevice, c.stream));
                }
                HIPCHECK(hipStreamSynchronize(c.stream));
                p->op = COLL_ALLREDUCE_MIN_I64;
                p->count = (uint64_t)g * nmm;
                break;
            case ST_CELL: mask_cells(c, p); p->op = COLL_REDUCE_SUM_I64; p->count = (uint64_t)g * C * 2; break;
            case ST_VLA: mask_cells(c, p); p->op = COLL_REDUCE_SUM_F64; p->count = (uint64_t)g * p->NV; break;
            case ST_SUMR: p->op = COLL_REDUCE_SUM_F64; p->count = (uint64_t)g * p->W; break;
            case ST_SIDE: mask_cells(c, p); p->op = COLL_ALLGATHER; p->count = p->side.size(); break;
        }
        p->at++;
        next->op = p->op;
        next->count = p->count;
        return 0;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return -1;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return -1;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return -1;
    }
}

int cqgpu_partial_put(cqgpu_partial* p, void* dev_dst) {
    g_err.clear();
    try {
        if (!p || p->at == 0 || p->op == COLL_DONE || p->op == COLL_DECLINE) throw HipError{"partial_put: nothing pending"};
        if (!p->count) return 0;
        if (!dev_dst) throw HipError{"partial_put: no buffer"};
        DevCtx& c = ctx();
        const void* src = nullptr;
        hipMemcpyKind kind = hipMemcpyDeviceToDevice;
        switch (p->stages[p->at - 1]) {
            case ST_KEYS: src = p->keyblob.data(); kind = hipMemcpyHostToDevice; break;
            case ST_SIDE: src = p->side.data(); kind = hipMemcpyHostToDevice; break;
            case ST_STRS: src = p->strs.data(); kind = hipMemcpyHostToDevice; break;
            case ST_MIN: src = p->dmin.p; break;
            case ST_SUM: case ST_SUMR: src = p->dsum.p; break;
            case ST_EXT: src = p->dext.p; break;
            case ST_CELL: src = p->dcell.p; break;
            case ST_VLA: src = p->dvla.p; break;
        }
        const size_t bytes = p->count * (p->op == COLL_ALLGATHER ? 1 : 8);
        HIPCHECK(hipMemcpyAsync(dev_dst, src, bytes, kind, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        return 0;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return -1;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return -1;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return -1;
    }
}

cq_table* cqgpu_partial_result(cqgpu_partial* p, cq_node* q) {
    g_inel.clear();
    g_err.clear();
    PhaseClock pc;
    PhaseClock* const outer_phase = g_phase;
    g_phase = &pc;
    struct Unset { PhaseClock* o; ~Unset() { g_phase = o; } } unset_{outer_phase};
    try {
        if (!p || p->op != COLL_DONE || p->at != p->stages.size()) throw HipError{"partial_result: merge not finished"};
        DevCtx& c = ctx();
        const uint32_t G = p->G, n = p->nall, W = p->W, P = p->P, nmm = (uint32_t)p->mm.size(), R = p->R;
        const uint32_t C = R + nmm, NV = p->NV;
        std::vector<HKeyRec> all(n);
        std::vector<uint32_t> flag(n);
        std::vector<uint8_t> text(p->text_bytes);
        std::vector<double> sm((size_t)G * W), vla((size_t)G * NV);
        std::vector<unsigned long long> mn((size_t)G * P), ex((size_t)G * nmm), cells((size_t)G * C * 2);
        // every plane into one pinned staging buffer (pageable copies are staged one
        // by one by the runtime), one sync, then host copies out
        struct Piece { void* dst; const void* src; size_t bytes; size_t at; };
        Piece pieces[] = {{all.data(), p->all.p, n ? (size_t)n * KEYREC : 0, 0},
                          {flag.data(), p->flag.p, n ? (size_t)n * 4 : 0, 0},
                          {text.data(), p->text.p, text.size(), 0},
                          {sm.data(), p->dsum.p, sm.size() * 8, 0},
                          {vla.data(), p->dvla.p, vla.size() * 8, 0},
                          {mn.data(), p->dmin.p, mn.size() * 8, 0},
                          {ex.data(), p->dext.p, ex.size() * 8, 0},
                          {cells.data(), p->dcell.p, cells.size() * 8, 0}};
        size_t tot = 0;
        for (Piece& pc2 : pieces) { pc2.at = tot; tot += (pc2.bytes + 15) & ~(size_t)15; }
        uint8_t* stage = (uint8_t*)pinned(c, std::max<size_t>(tot, 16));
        for (Piece& pc2 : pieces)
            if (pc2.bytes) HIPCHECK(hipMemcpyAsync(stage + pc2.at, pc2.src, pc2.bytes, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        for (Piece& pc2 : pieces)
            if (pc2.bytes) memcpy(pc2.dst, stage + pc2.at, pc2.bytes);
        PHASE("result copies");
        // the owners' texts over 8 bytes
        std::unordered_map<uint64_t, std::string> longs;
        for (size_t o = 0; o + 12 <= p->side_all.size();) {
            uint32_t h[3];
            memcpy(h, p->side_all.data() + o, 12);
            o += 12;
            if (o + h[2] > p->side_all.size() || h[0] >= G || h[1] >= C) throw HipError{"partial_result: bad side blob"};
            longs[(uint64_t)h[0] * C + h[1]].assign((const char*)p->side_all.data() + o, h[2]);
            o += h[2];
        }
        auto dec = [&](uint64_t d, uint32_t ci) {
            HCell x;
            const unsigned long long w0 = cells[(d * C + ci) * 2], w1 = cells[(d * C + ci) * 2 + 1];
            if (!(w0 & CELL_PRESENT)) return x;
            x.kind = (uint32_t)(w0 & 0xff);
            x.bits = w1;
            if (x.kind == K_STR) {
                const uint32_t len = (uint32_t)((w0 >> 8) & 0xFFFFFFFFull);
                x.bits = 0;
                if (w0 & CELL_LONG) {
                    auto it = longs.find(d * C + ci);
                    if (it == longs.end()) throw HipError{"partial_result: a long cell's text is missing"};
                    x.s = it->second;
                } else {
                    for (uint32_t i = 0; i < len; i++) x.s.push_back((char)((w1 >> (8 * i)) & 0xff));
                }
            }
            return x;
        };
        const Compiled& Cp = p->C;
        // dense id d <-> its key record r (the d-th flagged record), then the groups
        // built straight in first-row order (a stable sort of (first, d) pairs instead
        // of moving whole HGroups)
        std::vector<uint32_t> rec_of;
        rec_of.reserve(G);
        for (uint32_t r = 0; r < n && rec_of.size() < G; r++)
            if (flag[r]) rec_of.push_back(r);
        std::vector<std::pair<unsigned long long, uint32_t>> ord(rec_of.size());
        for (uint32_t d = 0; d < (uint32_t)rec_of.size(); d++) {
            const unsigned long long f = mn[(size_t)d * P];
            ord[d] = {f == ABS64 ? NOPOS : f, d};
        }
        std::sort(ord.begin(), ord.end());      // (first, d): ties keep dense order, as the stable sort did
        std::vector<HGroup> groups(ord.size());
        for (size_t gi = 0; gi < ord.size(); gi++) {
            const uint32_t d = ord[gi].second, r = rec_of[d];
            const HKeyRec& k = all[r];
            HGroup& h = groups[gi];
            h.kcls = k.clslen >> 16;
            h.klen = k.clslen & 0xffff;
            h.kw0 = k.w0;
            h.kw1 = k.w1;
            if (h.kcls == GK_STR) {
                char kb[16];
                for (uint32_t i = 0; i < h.klen && i < 16; i++)
                    kb[i] = (char)((i < 8 ? k.w0 >> (8 * i) : k.w1 >> (8 * (i - 8))) & 0xff);
                h.kbytes.assign(kb, std::min<uint32_t>(h.klen, 16));
            }
            if (h.kcls == GK_LONG) {
                if (k.pad2 + h.klen > text.size()) throw HipError{"partial_result: bad key text offset"};
                h.kbytes.assign((const char*)text.data() + k.pad2, h.klen);
            }
            h.cnt = (unsigned long long)sm[(size_t)d * W];
            for (int a = 0; a < Cp.P.nacc; a++) {
                h.sum[a] = sm[(size_t)d * W + 1 + 2 * a];
                h.num[a] = (unsigned long long)sm[(size_t)d * W + 2 + 2 * a];
            }
            h.first = mn[(size_t)d * P] == ABS64 ? NOPOS : mn[(size_t)d * P];
            for (uint32_t r2 = 0; r2 < R; r2++) h.reps.push_back(dec(d, r2));
            for (uint32_t i = 0; i < nmm; i++) {
                const int a = p->mm[i];
                const unsigned long long pos = ex[(size_t)d * nmm + i];
                if (pos == ABS64) continue;
                h.ext[a] = dec(d, R + i);
                h.extpos[a] = pos;
            }
            for (uint32_t v = 0; v < NV; v++) {
                const double nv = sm[(size_t)d * W + p->VS0 + 2 * v];
                h.vla_ok[v] = nv > 0;
                h.vla[v] = nv > 0 ? sqrt(vla[(size_t)d * NV + v] / nv) : 0.0;
            }
        }
        if (!Cp.grouped && groups.size() > 1) throw HipError{"partials disagree on the single group"};
        PHASE("result groups");
        Compiled C2 = Cp;
        Literals L;
        parse_literals(c, C2.lits, L);
        PHASE("result literals");
        g_stats.groups = groups.size();
        cq_table* res = build_groups(C2, groups, L, c);
        post_ops(c, res, q);
        PHASE("result table");
        g_stats.path = 1;
        return res;
    } catch (Ineligible& e) {
        g_inel = e.why;
        set_err("cq_amd: query outside the GPU executor's subset: %s", e.why.c_str());
        return nullptr;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return nullptr;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return nullptr;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return nullptr;
    }
}

void cqgpu_partial_free(cqgpu_partial* p) { delete p; }

}  // extern "C"

// ==================================================================== typed join exchange
// SURVEY.md section 8e's (key, row id, payload) entries for the repartitioned JOIN: the
// sender types every record once (fast.hip jx_extract_kernel ROUTE: the ON key as a
// canonical INTEGER, the build side's GROUP BY bytes or the probe side's SUM argument
// as 10^-3 fixed point) and writes a fixed-size entry into its destination's region
// (key mod N) -- 16 bytes {key / N - qbase, global record id, tag} per build record,
// 8 bytes {key / N - qbase, payload} per probe record -- instead of CSV text; the
// receiver's STAR join reads the entries (jx_ent_*) instead of re-parsing.  Plans:
// one INNER JOIN `l.k = r.k` without WHERE, COUNT / SUM / AVG of one right column,
// GROUP BY one left column (its value the only other item) or no GROUP BY.  Anything
// the entries cannot carry exactly (a quote, a key that is not a canonical INTEGER or
// NULL, a GROUP BY value over 8 bytes, a wider numeral, a NULL or repeated build key,
// more than JX_G groups, a sparse key range) sends every rank back to the CSV-record
// exchange together.
namespace {

struct TypedJoin {
    Compiled C;
    std::vector<std::string> names;   // the joined schema (alias.col)
    int kl = -1, kr = -1;             // ON key columns of the left / right table
    int gcol = -1;                    // GROUP BY column (left table; -1: no GROUP BY)
    int vcol = -1;                    // SUM / AVG argument (right table; -1: none)
};

bool typed_join_plan(cq_node* q, const cqgpu_table* L, const cqgpu_table* R, TypedJoin& tj, std::string& why) {
    why.clear();
    if (getenv("CQGPU_NO_TYPED_JOIN")) { why = "disabled"; return false; }
    if (!q || q->kind != CQ_N_QUERY || q->u.q.join_count != 1 || !L || !R) { why = "not one JOIN"; return false; }
    cq_node* jn = q->u.q.joins[0];
    if (!jn || jn->kind != CQ_N_JOIN || jn->u.join.kind != CQ_JOIN_INNER) { why = "not an INNER JOIN"; return false; }
    if (L->cfg.delimiter != ',' || L->cfg.quote != '"' || R->cfg.delimiter != ',' || R->cfg.quote != '"') {
        why = "CSV dialect";
        return false;
    }
    try {
        check_plan_shape(q, L, true);
        cq_node* on = jn->u.join.on;
        const std::string la = (q->u.q.from && q->u.q.from->u.from.alias) ? q->u.q.from->u.from.alias : "main";
        const std::string ra = jn->u.join.alias ? jn->u.join.alias : "right";
        cqgpu_table W;
        W.names = L->names;
        if (on && on->kind == CQ_N_CONDITION && on->u.bin.op && !strcmp(on->u.bin.op, "=") && on->u.bin.lhs &&
            on->u.bin.rhs && on->u.bin.lhs->kind == CQ_N_IDENTIFIER && on->u.bin.rhs->kind == CQ_N_IDENTIFIER) {
            tj.kl = join_on_index(on->u.bin.lhs->u.text, &W, &W, la.c_str(), R, ra.c_str());
            tj.kr = join_on_index(on->u.bin.rhs->u.text, R, &W, la.c_str(), R, ra.c_str());
        }
        if (tj.kl < 0 || tj.kr < 0) { why = "ON"; return false; }
        tj.names.clear();
        for (auto& nm : L->names) tj.names.push_back(la + "." + nm);
        for (auto& nm : R->names) tj.names.push_back(ra + "." + nm);
        cqgpu_table J;
        J.cfg = L->cfg;
        J.names = tj.names;
        if (is_row_query(q)) { why = "row-returning"; return false; }
        compile_aggregate(&J, q, tj.C);
    } catch (Ineligible& e) {
        why = e.why;
        return false;
    }
    const Compiled& C = tj.C;
    const int nl = (int)L->names.size();
    if (C.group_missing || C.P.nprog != 0 || C.P.ngpart != 0 || !C.vla.empty() || C.wide) { why = "plan"; return false; }
    if (C.grouped) {
        if (C.P.group_slot < 0) { why = "GROUP BY"; return false; }
        tj.gcol = C.need_cols[C.P.group_slot];
        if (tj.gcol >= nl) { why = "GROUP BY a right column"; return false; }
    }
    for (int a = 0; a < C.P.nacc; a++) {
        if (C.P.acc[a].kind != ACC_SUM) { why = "MIN / MAX"; return false; }
        const int col = C.need_cols[C.P.acc[a].slot];
        if (col < nl || (tj.vcol >= 0 && col - nl != tj.vcol)) { why = "aggregate columns"; return false; }
        tj.vcol = col - nl;
    }
    for (int rc : C.rep_cols)
        if (rc != tj.gcol) { why = "an item other than the GROUP BY column"; return false; }
    for (const OutCol& o : C.outs)
        if (o.kind != OUT_COUNT && o.kind != OUT_SUM && o.kind != OUT_AVG && o.kind != OUT_REP && o.kind != OUT_CONST &&
            o.kind != OUT_NULL) {
            why = "items";
            return false;
        }
    return true;
}

// the window stride and records per lane pass of a side (run_fast_join's rule)
void typed_stride(const cqgpu_table* t, uint32_t* ws, int* rp) {
    const uint32_t w = t->lean_ws ? t->lean_ws : 3968u;
    *rp = w < 3968u && !getenv("CQGPU_FAST_RP2") ? 3 : 2;
    *ws = *rp == 3 ? 3968u : w;
}

// a first qbase guess: the build side's sampled keys' minimum (sample_key_range pads it
// down) / N -- a key below it flags the send (16) and the retry takes the exact minimum
uint64_t typed_sample_kmin(const cqgpu_table* t, int kcol) {
    uint64_t kmin = 0, kmax = 0, est = 0;
    if (!sample_key_range(t, kcol, 1, &kmin, &kmax, &est)) return 0;
    return kmin;
}

// the count pass over one side (jx_extract_kernel ROUTE 1): per (destination, window)
// the entries, their destination-major exclusive scan (every entry's region position
// base) and per destination the entries; build: the records per window and their scan
// (the global ids); flags 1 (a key the entries cannot carry: the CSV exchange), 8, 16.
// The probe side (pcol: its SUM column or -1) at N <= 8 takes one pass instead
// (typed_one_pass); CQGPU_TYPED_TWO_PASS=1 keeps the count + emit passes.
bool typed_one_pass(DevCtx& c, cqgpu_table* t, int kcol, int pcol, TypedSend& ts);
TypedSend& typed_count_pass(DevCtx& c, cqgpu_table* t, bool build, int kcol, int N, uint64_t qbase, int pcol = -1) {
    std::unique_ptr<TypedSend> ts(new TypedSend);
    typed_stride(t, &ts->ws, &ts->rp);
    ts->N = (uint32_t)N;
    ts->qbase = qbase;
    const uint64_t nw = cq_jx_windows(t->data_begin, t->n, ts->ws);
    if (nw * (uint64_t)N >= (1ull << 31)) throw Ineligible{"typed exchange: too many windows"};
    ts->nwin = nw;
    if (!build && N <= 8 && nw && !getenv("CQGPU_TYPED_TWO_PASS") && typed_one_pass(c, t, kcol, pcol, *ts)) {
        t->tsend = std::move(ts);
        return *t->tsend;
    }
    const uint64_t nn = std::max<uint64_t>(nw * (uint64_t)N, 1);
    {
        DevBuf a(nn * 4), b(nn * 4 + 16);
        std::swap(ts->rcnt.p, a.p);
        std::swap(ts->roffs.p, b.p);
        if (build) {
            DevBuf x(std::max<uint64_t>(nw, 1) * 4), y(std::max<uint64_t>(nw, 1) * 4 + 16);
            std::swap(ts->wcount.p, x.p);
            std::swap(ts->wbase.p, y.p);
        }
    }
    DevBuf ctl(64);
    unsigned int* flag = ctl.as<unsigned int>();
    unsigned long long* kr = (unsigned long long*)(ctl.as<uint8_t>() + 16);
    HIPCHECK(hipMemsetAsync(ctl.p, 0, 64, c.stream));
    HIPCHECK(hipMemsetAsync(kr, 0xff, 8, c.stream));
    if (!nw) HIPCHECK(hipMemsetAsync(ts->rcnt.p, 0, nn * 4, c.stream));
    HIPCHECK(cq_jx_route(t->g, t->data_begin, t->n, ts->ws, (uint8_t)t->cfg.delimiter, (uint8_t)t->cfg.quote, kcol, -1,
                         build ? 1 : 0, ts->rp, 1, (uint32_t)N, qbase, 0, ts->rcnt.as<unsigned int>(),
                         build ? ts->wcount.as<unsigned int>() : nullptr, nullptr, nullptr, nullptr, 0u, flag, kr,
                         c.ncu, c.stream));
    size_t tb = 0;
    HIPCHECK(cq_excl_sum_u32(nullptr, &tb, ts->rcnt.as<unsigned int>(), ts->roffs.as<unsigned int>(), nn, c.stream));
    if (build && nw) {
        size_t tb2 = 0;
        HIPCHECK(cq_excl_sum_u32(nullptr, &tb2, ts->wcount.as<unsigned int>(), ts->wbase.as<unsigned int>(), nw, c.stream));
        tb = std::max(tb, tb2);
    }
    DevBuf tmp(tb + 16);
    HIPCHECK(cq_excl_sum_u32(tmp.p, &tb, ts->rcnt.as<unsigned int>(), ts->roffs.as<unsigned int>(), nn, c.stream));
    if (build && nw)
        HIPCHECK(cq_excl_sum_u32(tmp.p, &tb, ts->wcount.as<unsigned int>(), ts->wbase.as<unsigned int>(), nw, c.stream));
    // back to the host in one copy (typed_summary_kernel): the flags and key range, every
    // destination's first position, the totals
    DevBuf dsum(4 * (12 + (size_t)N));
    HIPCHECK(cq_launch_typed_summary(ts->roffs.as<unsigned int>(), ts->rcnt.as<unsigned int>(),
                                     build && nw ? ts->wbase.as<unsigned int>() : nullptr,
                                     build && nw ? ts->wcount.as<unsigned int>() : nullptr, nw, (uint32_t)N,
                                     (const uint32_t*)ctl.p, dsum.as<uint32_t>(), c.stream));
    uint8_t* h = (uint8_t*)pinned(c, 4 * (12 + (size_t)N));
    HIPCHECK(hipMemcpyAsync(h, dsum.p, 4 * (12 + (size_t)N), hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    uint32_t* hstart = (uint32_t*)(h + 32);
    uint32_t* htail = hstart + N;                    // [0] last roffs, [1] last rcnt, [2] last wbase, [3] last wcount
    memcpy(&ts->flags, h, 4);
    memcpy(ts->krange, h + 16, 16);
    ts->rstart.assign((size_t)N + 1, 0);
    ts->counts.assign(N, 0);
    if (nw) {
        for (int d = 0; d < N; d++) ts->rstart[d] = hstart[d];
        ts->rstart[N] = (uint64_t)htail[0] + htail[1];
        ts->nrec = build ? (uint64_t)htail[2] + htail[3] : 0;
    }
    for (int d = 0; d < N; d++) ts->counts[d] = ts->rstart[d + 1] - ts->rstart[d];
    t->tsend = std::move(ts);
    return *t->tsend;
}

// the probe side's single pass (jx_extract_kernel ROUTE 3): entries written while they
// are counted, destination d's region [d cap, (d + 1) cap) filled in chunks from its
// cursor with holes at the waves' chunk tails (the receivers skip them); the region
// capacity is twice the sampled share plus a chunk per wave with a window.  False (nothing kept):
// no sample, or a region overflowed (skewed keys) -- the caller runs the two passes.
bool typed_one_pass(DevCtx& c, cqgpu_table* t, int kcol, int pcol, TypedSend& ts) {
    if (!t->est_records) {                            // (once per table: the sample is fixed)
        uint64_t skmin = 0, skmax = 0, est = 0;
        if (!sample_key_range(t, kcol, 1, &skmin, &skmax, &est)) return false;
        t->est_records = est;
    }
    const uint64_t est = t->est_records;
    const uint32_t N = ts.N;
    const char* ce = getenv("CQGPU_TEST_ONE_PASS_CAP");     // test knob: the region capacity
    const uint64_t cap64 = ce ? strtoull(ce, nullptr, 10)
                              : 2 * est / N + std::min<uint64_t>(ts.nwin, (uint64_t)c.ncu * 16) * cq_jx_rchunk() + 4096;
    if (cap64 == 0 || cap64 >= (1ull << 31)) return false;
    const uint32_t cap = (uint32_t)cap64;
    {
        DevBuf e((size_t)N * cap * 8 + 16);
        std::swap(ts.ent.p, e.p);
    }
    const size_t hb = 64 + (size_t)N * 256;           // flags, key range, then the cursors (stride 256 B)
    DevBuf ctl(hb);
    unsigned int* flag = ctl.as<unsigned int>();
    unsigned long long* kr = (unsigned long long*)(ctl.as<uint8_t>() + 16);
    unsigned int* cur = (unsigned int*)(ctl.as<uint8_t>() + 64);
    HIPCHECK(hipMemsetAsync(ctl.p, 0, hb, c.stream));
    HIPCHECK(cq_jx_route(t->g, t->data_begin, t->n, ts.ws, (uint8_t)t->cfg.delimiter, (uint8_t)t->cfg.quote, kcol, pcol,
                         0, ts.rp, 3, N, ts.qbase, 0, cur, nullptr, nullptr, nullptr, ts.ent.p, cap, flag, kr, c.ncu,
                         c.stream));
    uint8_t* h = (uint8_t*)pinned(c, hb);
    HIPCHECK(hipMemcpyAsync(h, ctl.p, hb, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    uint32_t fl = 0;
    memcpy(&fl, h, 4);
    bool over = (fl & 1024u) != 0;
    ts.rstart.assign((size_t)N + 1, 0);
    ts.counts.assign(N, 0);
    for (uint32_t d = 0; d < N; d++) {
        uint32_t n = 0;
        memcpy(&n, h + 64 + 256 * (size_t)d, 4);
        over = over || n > cap;
        ts.rstart[d] = (uint64_t)d * cap;
        ts.counts[d] = n;
    }
    ts.rstart[N] = (uint64_t)N * cap;
    if (over) {
        DevBuf drop;
        std::swap(ts.ent.p, drop.p);
        ts.rstart.clear();
        ts.counts.clear();
        return false;
    }
    ts.flags = fl & ~512u;
    ts.eflags = fl & 512u;
    ts.esize = 8;
    ts.one_pass = true;
    return true;
}

// the emit pass (jx_extract_kernel ROUTE 2) after typed_count_pass: every entry at its
// position; flags 1 (a payload the entries cannot carry), 512
uint32_t typed_emit_pass(DevCtx& c, cqgpu_table* t, bool build, int kcol, int pcol, uint64_t gbase) {
    if (!t->tsend) throw HipError{"typed exchange: send without a count"};
    TypedSend& ts = *t->tsend;
    if (ts.one_pass) {                                    // (written by the count pass)
        ts.emitted = true;
        ts.flags |= ts.eflags;
        return ts.eflags;
    }
    ts.esize = build ? 16 : 8;
    const uint64_t total = ts.rstart[ts.N];
    {
        DevBuf e(std::max<uint64_t>(total, 1) * ts.esize + 16);
        std::swap(ts.ent.p, e.p);
    }
    DevBuf ctl(64);
    unsigned int* flag = ctl.as<unsigned int>();
    unsigned long long* kr = (unsigned long long*)(ctl.as<uint8_t>() + 16);
    HIPCHECK(hipMemsetAsync(ctl.p, 0, 64, c.stream));
    HIPCHECK(cq_jx_route(t->g, t->data_begin, t->n, ts.ws, (uint8_t)t->cfg.delimiter, (uint8_t)t->cfg.quote, kcol, pcol,
                         build ? 1 : 0, ts.rp, 2, ts.N, ts.qbase, gbase, nullptr, nullptr, ts.roffs.as<unsigned int>(),
                         build ? ts.wbase.as<unsigned int>() : nullptr, ts.ent.p, 0u, flag, kr, c.ncu, c.stream));
    uint32_t* h = (uint32_t*)pinned(c, 16);
    HIPCHECK(hipMemcpyAsync(h, flag, 4, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    ts.emitted = true;
    ts.flags |= h[0];
    return h[0];
}

// the receiving rank: STAR over the entries -> this rank's groups in `part`; returns
// the flags (0: done; 16 / 32 / 64: the entries do not fit the STAR form)
uint32_t typed_receive(DevCtx& c, const TypedJoin& tj, const void* ub, uint64_t nu, const void* ob, uint64_t no,
                       uint64_t qoff, uint64_t range, JoinPartial& part, bool allow_part = true) {
    PhaseClock pc;
    PhaseClock* const outer_phase = g_phase;
    g_phase = &pc;
    struct Unset { PhaseClock* o; ~Unset() { g_phase = o; } } unset_{outer_phase};
    const uint32_t G = cq_jx_star_groups();
    const bool grouped = tj.gcol >= 0;
    if (range >= (1ull << 31) || qoff >= (1ull << 32)) return 16u;
    const size_t b16 = (range * 2 + 15) & ~(size_t)15;
    DevBuf d16(b16 + 16), l32(range * 4 + 16);
    // small: tags, per group sums, first ids, smallest matched slots (both ~0 at the
    // start), flags and counts
    const size_t o_gsum = (size_t)G * 8, o_first = o_gsum + (size_t)G * 24, o_minix = o_first + (size_t)G * 4,
                 o_ctl = o_minix + (size_t)G * 4;
    DevBuf small(o_ctl + 64);
    unsigned long long* ttab = small.as<unsigned long long>();
    unsigned long long* gsum = (unsigned long long*)(small.as<uint8_t>() + o_gsum);
    uint32_t* gfirst = (uint32_t*)(small.as<uint8_t>() + o_first);
    uint32_t* gminix = (uint32_t*)(small.as<uint8_t>() + o_minix);
    unsigned int* flag = (unsigned int*)(small.as<uint8_t>() + o_ctl);
    unsigned long long* cnts = (unsigned long long*)(small.as<uint8_t>() + o_ctl + 8);   // placed, pairs, occupied
    uint32_t* notmono = (uint32_t*)(small.as<uint8_t>() + o_ctl + 32);
    HIPCHECK(cq_jx_star_init(d16.p, b16, small.p, o_ctl + 64, (uint32_t)o_first, (uint32_t)o_ctl,
                             (uint32_t)o_ctl + 48, nullptr, 0, c.ncu * 4, c.stream));
    // notmono (zeroed by star_init): the build sets it unless the slots rise along the
    // entries (global-id order); rising, the probe keeps each group's smallest matched
    // slot (no d16 match flags, no jx_star_first scan); CQGPU_TYPED_FLAGS=1 forces the
    // matched-flag form
    if (getenv("CQGPU_TYPED_FLAGS")) HIPCHECK(hipMemsetAsync(notmono, 1, 4, c.stream));
    HIPCHECK(hipEventRecord(c.ev0, c.stream));
    // (ungrouped: no tag lookup, every build entry in group 0)
    HIPCHECK(cq_jx_ent_build(ub, nu, (uint32_t)qoff, range, d16.as<uint16_t>(), l32.as<uint32_t>(), ttab, cnts, flag,
                             c.ncu * 4, c.stream, grouped ? 0 : 1, notmono));
    // the probe: when d16 outgrows an XCD's L2, in two passes -- the entries into 2 MiB
    // key partitions (jx_ent_part_kernel), then each partition looked up by one XCD's
    // blocks (jx_part_probe_kernel, the CSV STAR's pass 2); a full segment (skewed keys)
    // reruns the whole receive unpartitioned.  CQGPU_TYPED_NO_PART=1: one pass; test
    // knobs as the CSV STAR's: CQGPU_PART_PROBE_MIN (slots above which it partitions,
    // default 2^21; also the probe entries' floor, 2^20 by default), CQGPU_PART_PROBE_SHIFT
    const char* pm_env = getenv("CQGPU_PART_PROBE_MIN");
    const char* ps_env = getenv("CQGPU_PART_PROBE_SHIFT");
    const uint64_t part_min = pm_env ? strtoull(pm_env, nullptr, 10) : (2ull << 20);
    const uint32_t PSH = ps_env ? (uint32_t)std::min(std::max(atoi(ps_env), 4), 24) : 20u;
    const uint64_t np64 = (range + (1ull << PSH) - 1) >> PSH;
    const uint32_t pgrid = (uint32_t)c.ncu;
    const bool pprobe = allow_part && !getenv("CQGPU_TYPED_NO_PART") && range > part_min && np64 <= 4096 &&
                        no >= std::min<uint64_t>(part_min / 2, 1ull << 20) && pgrid >= 8;
    DevBuf pent, pcnt;
    if (pprobe) {
        const uint64_t per = no / ((uint64_t)pgrid * np64) + 1;
        const uint32_t pcap = (uint32_t)std::min<uint64_t>(per + per / 4 + 256, 1u << 30);
        DevBuf a((size_t)pgrid * np64 * pcap * 8), b((size_t)pgrid * np64 * 4);
        std::swap(pent.p, a.p);
        std::swap(pcnt.p, b.p);
        HIPCHECK(cq_jx_ent_part(ob, no, (uint32_t)qoff, range, (uint32_t)np64, pcap, PSH, pent.as<unsigned long long>(),
                                pcnt.as<uint32_t>(), flag, (int)pgrid, c.stream));
        HIPCHECK(cq_jx_part_probe(pent.as<unsigned long long>(), pcnt.as<uint32_t>(), pgrid, (uint32_t)np64, pcap, range,
                                  d16.as<uint16_t>(), notmono, gsum, gminix, cnts + 1, std::max(8, (c.ncu / 8) * 8),
                                  c.stream));
    } else {
        HIPCHECK(cq_jx_ent_probe(ob, no, (uint32_t)qoff, range, d16.as<uint16_t>(), gsum, cnts + 1, c.ncu * 4, c.stream,
                                 notmono, gminix));
    }
    HIPCHECK(cq_jx_ent_first(gminix, l32.as<uint32_t>(), notmono, gfirst, c.stream));   // (rising keys only)
    HIPCHECK(cq_jx_star_first(d16.as<uint16_t>(), l32.as<uint32_t>(), range, notmono, gfirst, cnts + 2, c.ncu * 4,
                              c.stream));
    HIPCHECK(hipEventRecord(c.ev1, c.stream));
    PHASE("typed launch");
    std::vector<uint8_t> h(o_ctl + 64);
    uint8_t* hp = (uint8_t*)pinned(c, h.size());
    HIPCHECK(hipMemcpyAsync(hp, small.p, h.size(), hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    PHASE("typed kernels");
    memcpy(h.data(), hp, h.size());
    float ms = 0;
    HIPCHECK(hipEventElapsedTime(&ms, c.ev0, c.ev1));
    g_stats.scan_ms = ms;
    uint32_t fl = 0;
    memcpy(&fl, h.data() + o_ctl, 4);
    if (fl & 128u) {                                     // a partition segment overflowed
        HIPCHECK(hipStreamSynchronize(c.stream));         // (the partition buffers go out of scope)
        return typed_receive(c, tj, ub, nu, ob, no, qoff, range, part, false);
    }
    unsigned long long cn[3];
    memcpy(cn, h.data() + o_ctl + 8, 24);
    uint32_t nm = 0;
    memcpy(&nm, h.data() + o_ctl + 32, 4);
    if (nm && cn[0] != cn[2]) fl |= 64u;                 // a repeated build key (rising keys are distinct)
    if (fl) return fl;
    g_stats.records = nu + no;
    g_stats.passed = cn[1];
    g_stats.scan_kernel = 5;                             // the typed STAR join
    const unsigned long long* ht = (const unsigned long long*)h.data();
    const unsigned long long* hs = (const unsigned long long*)(h.data() + o_gsum);
    const uint32_t* hf = (const uint32_t*)(h.data() + o_first);
    const int nacc = tj.C.P.nacc;
    const uint32_t nrep = (uint32_t)tj.C.rep_cols.size();
    std::vector<HGroup> groups;
    groups.reserve(G);
    struct KeyHash {
        size_t operator()(const std::tuple<uint64_t, uint64_t, uint64_t>& k) const {
            uint64_t x = std::get<0>(k) * 0x9E3779B97F4A7C15ull ^ std::get<1>(k) ^ (std::get<2>(k) * 0xC2B2AE3D27D4EB4Full);
            x ^= x >> 29;
            return (size_t)(x * 0xBF58476D1CE4E5B9ull);
        }
    };
    std::unordered_map<std::tuple<uint64_t, uint64_t, uint64_t>, size_t, KeyHash> at;
    at.reserve(2 * (size_t)G);
    auto fill = [&](HGroup& x, uint32_t s) {
        x.cnt = hs[3 * s];
        x.first = hf[s] == ~0u ? NOPOS : ((unsigned long long)hf[s] << 32);
        for (int a = 0; a < nacc; a++) {
            x.sum[a] = hs[3 * s + 2] ? (double)(long long)hs[3 * s + 1] / 1000.0 : 0.0;
            x.num[a] = hs[3 * s + 2];
        }
    };
    for (uint32_t s = 0; s < G; s++) {
        if (!hs[3 * s]) continue;
        HGroup x;
        fill(x, s);
        if (grouped) {
            // the tag's bytes (fast_kernel's tag: zero padded, (1 << 32) for the empty field)
            const unsigned long long tag = ht[s];
            uint8_t b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            uint32_t len = 0;
            if (tag != (1ull << 32)) {
                for (uint32_t j = 0; j < 8; j++) {
                    b[j] = (uint8_t)(tag >> (8 * j));
                    if (b[j]) len = j + 1;
                }
            }
            const Cell cell = cq_host_parse_cell(b, len);
            const GKey k = cq_host_group_key(cell);
            x.kcls = k.cls;
            x.klen = k.len;
            x.kw0 = k.w0;
            x.kw1 = k.w1;
            if (k.cls == GK_STR) {                      // the key's text (a NULL key's is "NULL")
                char kt[16];
                for (uint32_t j = 0; j < 16; j++) kt[j] = (char)((j < 8 ? k.w0 >> (8 * j) : k.w1 >> (8 * (j - 8))) & 0xFF);
                x.kbytes.assign(kt, std::min<uint32_t>(k.len, 16));
            }
            HCell rep;
            rep.kind = cell.kind;
            rep.bits = cell.kind == K_STR ? 0 : cell.bits;
            if (cell.kind == K_STR) rep.s.assign((const char*)(uintptr_t)cell.bits, cell.len);
            for (uint32_t r = 0; r < nrep; r++) x.reps.push_back(rep);
        } else {
            x.kcls = GK_ALL;
        }
        // raw tags of one canonical key (e.g. "1.0" and "1.00") are one group: counts and
        // sums add, the first pair is the smaller, its row gives the representative cells
        const auto kk = std::make_tuple((uint64_t)x.kcls << 32 | x.klen, x.kw0, x.kw1);
        auto it = at.find(kk);
        if (it == at.end()) {
            at.emplace(kk, groups.size());
            groups.push_back(std::move(x));
            continue;
        }
        HGroup* same = &groups[it->second];
        same->cnt += x.cnt;
        for (int a = 0; a < nacc; a++) { same->sum[a] += x.sum[a]; same->num[a] += x.num[a]; }
        if (x.first < same->first) { same->first = x.first; same->reps = x.reps; }
    }
    part.groups = std::move(groups);
    part.names = tj.names;
    part.nacc = nacc;
    part.nrep = nrep;
    part.nvla = 0;
    for (int a = 0; a < MAX_ACC; a++) part.acc_classes[a] = 0;   // SUM only
    part.lmask |= nu ? 2u : 0u;                                    // (canonical INTEGER keys: numbers)
    part.rmask |= no ? 2u : 0u;
    g_stats.groups = part.groups.size();
    PHASE("typed groups");
    return 0;
}

}  // namespace

extern "C" {

int cqgpu_typed_plan(cq_node* q, cqgpu_table* const* tables, int ntables) {
    g_inel.clear();
    g_err.clear();
    if (ntables != 2 || !tables || !tables[0] || !tables[1]) return 0;
    TypedJoin tj;
    std::string why;
    const bool ok = typed_join_plan(q, tables[0], tables[1], tj, why);
    if (!ok) g_inel = why;
    return ok ? 1 : 0;
}

uint64_t cqgpu_typed_sample_kmin(cq_node* q, cqgpu_table* const* tables, int ntables) {
    TypedJoin tj;
    std::string why;
    if (ntables != 2 || !tables || !tables[0] || !tables[1] || !typed_join_plan(q, tables[0], tables[1], tj, why))
        return ~0ull;
    return tables[0]->n > tables[0]->data_begin ? typed_sample_kmin(tables[0], tj.kl) : ~0ull;
}

int64_t cqgpu_typed_count(cq_node* q, cqgpu_table* const* tables, int ntables, int side, int nranks, uint64_t qbase,
                          uint64_t* counts, uint64_t* krange, uint32_t* flags) {
    g_err.clear();
    try {
        TypedJoin tj;
        std::string why;
        if (ntables != 2 || (side != 0 && side != 1) || nranks < 1 || nranks > 64 ||
            !typed_join_plan(q, tables[0], tables[1], tj, why))
            throw Ineligible{"typed exchange: " + why};
        DevCtx& c = ctx();
        const TypedSend& ts = typed_count_pass(c, tables[side], side == 0, side == 0 ? tj.kl : tj.kr, nranks, qbase,
                                               side == 0 ? -1 : tj.vcol);
        for (int d = 0; d < nranks; d++) if (counts) counts[d] = ts.counts[d];
        if (krange) { krange[0] = ts.krange[0]; krange[1] = ts.krange[1]; }
        if (flags) *flags = ts.flags;
        uint64_t sent = 0;
        for (int d = 0; d < nranks; d++) sent += ts.counts[d];
        return (int64_t)(side == 0 ? ts.nrec : sent);
    } catch (Ineligible& e) {
        g_inel = e.why;
        set_err("cq_amd: %s", e.why.c_str());
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
    }
    return -1;
}

int cqgpu_typed_send(cq_node* q, cqgpu_table* const* tables, int ntables, int side, uint64_t gid_base, uint32_t* flags) {
    g_err.clear();
    try {
        TypedJoin tj;
        std::string why;
        if (ntables != 2 || (side != 0 && side != 1) || !typed_join_plan(q, tables[0], tables[1], tj, why))
            throw Ineligible{"typed exchange: " + why};
        DevCtx& c = ctx();
        const uint32_t f = typed_emit_pass(c, tables[side], side == 0, side == 0 ? tj.kl : tj.kr,
                                           side == 0 ? tj.gcol : tj.vcol, gid_base);
        if (flags) *flags = f;
        return 0;
    } catch (Ineligible& e) {
        g_inel = e.why;
        set_err("cq_amd: %s", e.why.c_str());
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
    }
    return -1;
}

void cqgpu_typed_reset(cqgpu_table* t) {
    if (t) t->tsend.reset();
}

const void* cqgpu_typed_region(const cqgpu_table* t, int dest, uint64_t* entries, uint64_t* entry_bytes) {
    if (!t || !t->tsend || !t->tsend->emitted || dest < 0 || (uint32_t)dest >= t->tsend->N) return nullptr;
    const TypedSend& ts = *t->tsend;
    if (entries) *entries = ts.counts[dest];
    if (entry_bytes) *entry_bytes = ts.esize;
    return ts.ent.as<uint8_t>() + ts.rstart[dest] * ts.esize;
}

int64_t cqgpu_typed_gather(cqgpu_table* const* senders, int nsenders, int dest, void* dev_out, uint64_t cap_entries) {
    g_err.clear();
    try {
        DevCtx& c = ctx();
        uint64_t at = 0, esize = 0;
        for (int r = 0; r < nsenders; r++) {
            uint64_t n = 0, eb = 0;
            const void* p = cqgpu_typed_region(senders[r], dest, &n, &eb);
            if (!p) throw HipError{"typed_gather: a sender has no entries"};
            if (esize && eb != esize) throw HipError{"typed_gather: entries of different sides"};
            esize = eb;
            if (at + n > cap_entries) throw HipError{"typed_gather: the output is too small"};
            if (n) HIPCHECK(hipMemcpyAsync((uint8_t*)dev_out + at * eb, p, n * eb, hipMemcpyDeviceToDevice, c.stream));
            at += n;
        }
        HIPCHECK(hipStreamSynchronize(c.stream));
        return (int64_t)at;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
    }
    return -1;
}

size_t cqgpu_typed_partial(cq_node* q, cqgpu_table* const* tables, int ntables, const void* dev_build, uint64_t nbuild,
                           const void* dev_probe, uint64_t nprobe, uint64_t qoff, uint64_t range, void** blob_out) {
    if (blob_out) *blob_out = nullptr;
    g_inel.clear();
    g_err.clear();
    memset(&g_stats, 0, sizeof g_stats);
    try {
        TypedJoin tj;
        std::string why;
        if (ntables != 2 || !typed_join_plan(q, tables[0], tables[1], tj, why)) throw Ineligible{"typed exchange: " + why};
        DevCtx& c = ctx();
        bump_reset(c);
        JoinPartial jp;
        const uint32_t fl = typed_receive(c, tj, dev_build, nbuild, dev_probe, nprobe, qoff, range, jp);
        if (fl) {
            char b[96];
            snprintf(b, sizeof b, "typed exchange: the entries do not fit the STAR join (flags %#x)", fl);
            throw Ineligible{b};
        }
        Blob b;
        join_blob(jp, b);
        void* out = malloc(std::max<size_t>(b.d.size(), 1));
        if (!out) throw HipError{"out of host memory"};
        memcpy(out, b.d.data(), b.d.size());
        *blob_out = out;
        g_stats.path = 1;
        return b.d.size();
    } catch (Ineligible& e) {
        g_inel = e.why;
        set_err("cq_amd: %s", e.why.c_str());
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
    }
    return 0;
}

}  // extern "C"

// ==================================================================== N > 1 over RCCL
// The whole range-partitioned step inside the library (cqgpu.h cqgpu_dist_query):
// one communicator per device, every collective on the device context's stream,
// rank-local failures carried as status words in the payloads.  Three merges, chosen
// from the plan alone (so every rank takes the same one):
//   gather-merge  COUNT / SUM / AVG / group columns / constants over <= 1 GROUP BY
//                 column: each rank's groups (first-appearance order) to rank 0 in
//                 one grouped send / recv, merged by merge.hip gm_* on its device;
//                 then rank 0's status to every rank (ncclBroadcast)
//   dense         other aggregates but MEDIAN: the cqgpu_partial stage sequence
//                 (KEYS all_gather, MIN / SUM all-reduces, SUM reduces to rank 0)
//   blobs         MEDIAN, row-returning SELECT: cqgpu_query_partial blobs to rank 0
// A gather-merge the data declines (more than GM_MAXG groups on a rank, texts over
// GM_TEXT bytes) falls to the dense merge, a dense merge over 2^29 keys to blobs.
namespace {

#define NCCLCHECK(x)                                                                  \
    do {                                                                              \
        ncclResult_t r_ = (x);                                                        \
        if (r_ != ncclSuccess) throw HipError{std::string(#x) + ": " + ncclGetErrorString(r_)}; \
    } while (0)

// The collectives the N > 1 step issues, behind one table.  The product backend is
// RCCL over the library's own communicator (RcclColl).  The test backend (HostColl,
// cqgpu_comm_init_host) stages every buffer through host memory and hands it to a
// caller-supplied function -- the tests run the very same dist_gm / dist_dense /
// dist_blob / dist_join code at world size 2 and 3 over torch.distributed gloo, with
// several processes sharing one GPU (RCCL refuses two ranks on one device).
enum CollDt { CD_U8 = 0, CD_U32 = 1, CD_U64 = 2, CD_I64 = 3, CD_F64 = 4 };
enum CollRed { CR_SUM = 0, CR_MIN = 1, CR_MAX = 2 };
size_t coll_elem(CollDt t) { return t == CD_U8 ? 1 : (t == CD_U32 ? 4 : 8); }

struct Coll {
    virtual ~Coll() {}
    // in place
    virtual void all_reduce(void* buf, size_t n, CollDt t, CollRed o, hipStream_t s) = 0;
    // recv = every rank's n elements of send, in rank order (send may lie inside recv)
    virtual void all_gather(const void* send, void* recv, size_t n, CollDt t, hipStream_t s) = 0;
    // in place; the result on `root` only
    virtual void reduce(void* buf, size_t n, CollDt t, CollRed o, int root, hipStream_t s) = 0;
    // root's send into every rank's recv
    virtual void broadcast(const void* send, void* recv, size_t n, CollDt t, int root, hipStream_t s) = 0;
    // point to point between group_start and group_end (all of one group run together)
    virtual void group_start() = 0;
    virtual void send(const void* buf, size_t n, CollDt t, int peer, hipStream_t s) = 0;
    virtual void recv(void* buf, size_t n, CollDt t, int peer, hipStream_t s) = 0;
    virtual void group_end(hipStream_t s) = 0;
};

ncclDataType_t nccl_dt(CollDt t) {
    switch (t) {
        case CD_U8: return ncclUint8;
        case CD_U32: return ncclUint32;
        case CD_U64: return ncclUint64;
        case CD_I64: return ncclInt64;
        default: return ncclFloat64;
    }
}
ncclRedOp_t nccl_op(CollRed o) { return o == CR_SUM ? ncclSum : (o == CR_MIN ? ncclMin : ncclMax); }

struct RcclColl : Coll {
    ncclComm_t comm = nullptr;
    ~RcclColl() override {
        if (comm) (void)ncclCommDestroy(comm);
    }
    void all_reduce(void* buf, size_t n, CollDt t, CollRed o, hipStream_t s) override {
        NCCLCHECK(ncclAllReduce(buf, buf, n, nccl_dt(t), nccl_op(o), comm, s));
    }
    void all_gather(const void* send, void* recv, size_t n, CollDt t, hipStream_t s) override {
        NCCLCHECK(ncclAllGather(send, recv, n, nccl_dt(t), comm, s));
    }
    void reduce(void* buf, size_t n, CollDt t, CollRed o, int root, hipStream_t s) override {
        NCCLCHECK(ncclReduce(buf, buf, n, nccl_dt(t), nccl_op(o), root, comm, s));
    }
    void broadcast(const void* send, void* recv, size_t n, CollDt t, int root, hipStream_t s) override {
        NCCLCHECK(ncclBroadcast(send, recv, n, nccl_dt(t), root, comm, s));
    }
    void group_start() override { NCCLCHECK(ncclGroupStart()); }
    void send(const void* buf, size_t n, CollDt t, int peer, hipStream_t s) override {
        NCCLCHECK(ncclSend(buf, n, nccl_dt(t), peer, comm, s));
    }
    void recv(void* buf, size_t n, CollDt t, int peer, hipStream_t s) override {
        NCCLCHECK(ncclRecv(buf, n, nccl_dt(t), peer, comm, s));
    }
    void group_end(hipStream_t) override { NCCLCHECK(ncclGroupEnd()); }
};

// test backend: device buffers staged through host memory, each collective one call of
// the caller's function (cqgpu.h cqgpu_coll_fn), synchronous on the library's stream
struct HostColl : Coll {
    cqgpu_coll_fn fn = nullptr;
    void* user = nullptr;
    int world = 1;
    struct Pending {
        void* dev;
        std::vector<uint8_t> host;
    };
    std::vector<std::vector<uint8_t>> sends;   // alive until group_end
    std::vector<Pending> recvs;
    void call(int op, CollDt t, CollRed o, int peer, const void* sb, void* rb, size_t n) {
        if (fn(user, op, (int)t, (int)o, peer, sb, rb, (uint64_t)n) != 0)
            throw HipError{"host collective backend: operation " + std::to_string(op) + " failed"};
    }
    std::vector<uint8_t> down(const void* dev, size_t bytes, hipStream_t s) {
        std::vector<uint8_t> h(std::max<size_t>(bytes, 1));
        if (bytes) HIPCHECK(hipMemcpyAsync(h.data(), dev, bytes, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        return h;
    }
    void up(void* dev, const uint8_t* h, size_t bytes, hipStream_t s) {
        if (bytes) HIPCHECK(hipMemcpyAsync(dev, h, bytes, hipMemcpyHostToDevice, s));
        HIPCHECK(hipStreamSynchronize(s));
    }
    void all_reduce(void* buf, size_t n, CollDt t, CollRed o, hipStream_t s) override {
        std::vector<uint8_t> h = down(buf, n * coll_elem(t), s);
        call(CQGPU_HC_ALLREDUCE, t, o, -1, h.data(), h.data(), n);
        up(buf, h.data(), n * coll_elem(t), s);
    }
    void all_gather(const void* send, void* recv, size_t n, CollDt t, hipStream_t s) override {
        const size_t b = n * coll_elem(t);
        std::vector<uint8_t> h = down(send, b, s), r(std::max<size_t>(b * world, 1));
        call(CQGPU_HC_ALLGATHER, t, CR_SUM, -1, h.data(), r.data(), n);
        up(recv, r.data(), b * world, s);
    }
    void reduce(void* buf, size_t n, CollDt t, CollRed o, int root, hipStream_t s) override {
        std::vector<uint8_t> h = down(buf, n * coll_elem(t), s);
        call(CQGPU_HC_REDUCE, t, o, root, h.data(), h.data(), n);
        up(buf, h.data(), n * coll_elem(t), s);
    }
    void broadcast(const void* send, void* recv, size_t n, CollDt t, int root, hipStream_t s) override {
        std::vector<uint8_t> h = down(send ? send : recv, n * coll_elem(t), s);
        call(CQGPU_HC_BROADCAST, t, CR_SUM, root, h.data(), h.data(), n);
        up(recv, h.data(), n * coll_elem(t), s);
    }
    void group_start() override {
        sends.clear();
        recvs.clear();
    }
    void send(const void* buf, size_t n, CollDt t, int peer, hipStream_t s) override {
        sends.push_back(down(buf, n * coll_elem(t), s));
        call(CQGPU_HC_SEND, t, CR_SUM, peer, sends.back().data(), nullptr, n);
    }
    void recv(void* buf, size_t n, CollDt t, int peer, hipStream_t s) override {
        recvs.push_back(Pending{buf, std::vector<uint8_t>(std::max<size_t>(n * coll_elem(t), 1))});
        call(CQGPU_HC_RECV, t, CR_SUM, peer, nullptr, recvs.back().host.data(), n);
        recvs.back().host.resize(n * coll_elem(t));
    }
    void group_end(hipStream_t s) override {
        call(CQGPU_HC_GROUP_END, CD_U8, CR_SUM, -1, nullptr, nullptr, 0);
        for (Pending& p : recvs) up(p.dev, p.host.data(), p.host.size(), s);
        sends.clear();
        recvs.clear();
    }
};

struct DistComm {
    std::unique_ptr<Coll> be;            // RcclColl, or HostColl in the tests
    int rank = 0, world = 1;
};
DistComm g_comm[64];

DistComm& dist_comm() {
    int dev = 0;
    HIPCHECK(hipGetDevice(&dev));
    DistComm& m = g_comm[dev & 63];
    if (!m.be) throw HipError{"dist_query: no communicator on this device (cqgpu_comm_init)"};
    return m;
}

// a rank-local step failed on some rank: every rank throws it after the same collectives
struct PeerFail {
    std::string msg;
};

constexpr uint32_t GM_MAXG = 4096;      // groups one rank may send (above: the dense merge)
constexpr uint32_t GM_SB = 48;          // finish_kernel's inline string bytes (run_aggregate SB)
constexpr size_t DIST_MAIL_HDR = 1024;

enum DistPath { DP_GM = 1, DP_DENSE = 2, DP_BLOB = 3 };

bool gm_eligible(const Compiled& C) {
    if (C.wide || C.P.ngpart > 0 || !C.vla.empty()) return false;
    for (int a = 0; a < C.P.nacc; a++)
        if (C.P.acc[a].kind != ACC_SUM) return false;
    for (const OutCol& o : C.outs)
        if (o.kind != OUT_COUNT && o.kind != OUT_SUM && o.kind != OUT_AVG && o.kind != OUT_REP && o.kind != OUT_CONST &&
            o.kind != OUT_NULL)
            return false;
    return true;
}
bool dense_eligible(const Compiled& C) {
    for (auto& v : C.vla)
        if (v.first != 0) return false;      // MEDIAN needs every value
    return true;
}

// per-device buffers of the N > 1 step, kept across steps (grown as needed)
struct DistBufs {
    DevBuf send, recv, scratch, word;
    size_t send_b = 0, recv_b = 0, scratch_b = 0;
    uint32_t* hword = nullptr;           // pinned: status words read back
};
DistBufs g_dbuf[64];
DistBufs& dist_bufs() {
    int dev = 0;
    HIPCHECK(hipGetDevice(&dev));
    DistBufs& b = g_dbuf[dev & 63];
    if (!b.word.p) {
        DevBuf w(256);
        std::swap(b.word.p, w.p);
        HIPCHECK(hipHostMalloc((void**)&b.hword, 256, hipHostMallocDefault));
    }
    return b;
}
uint8_t* grow(DevBuf& b, size_t& have, size_t need) {
    if (need > have || !b.p) {
        DevBuf nb(std::max<size_t>(need, 256));
        std::swap(b.p, nb.p);
        have = std::max<size_t>(need, 256);
    }
    return (uint8_t*)b.p;
}

// one MAX all-reduce of this rank's flag (0 / 1); true when any rank set it
bool agree_any(DevCtx& c, DistComm& m, bool bad) {
    DistBufs& b = dist_bufs();
    b.hword[0] = bad ? 1u : 0u;
    uint32_t* dw = b.word.as<uint32_t>();
    HIPCHECK(hipMemcpyAsync(dw, b.hword, 4, hipMemcpyHostToDevice, c.stream));
    m.be->all_reduce(dw, 1, CD_U32, CR_MAX, c.stream);
    HIPCHECK(hipMemcpyAsync(b.hword + 1, dw, 4, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    return b.hword[1] != 0;
}

// rank 0's status word (device, `dsrc` on rank 0) to every rank; returns it
uint32_t bcast_status(DevCtx& c, DistComm& m, const uint32_t* dsrc) {
    DistBufs& b = dist_bufs();
    uint32_t* dw = b.word.as<uint32_t>() + 4;
    m.be->broadcast(m.rank == 0 ? (const void*)dsrc : (const void*)dw, dw, 1, CD_U32, 0, c.stream);
    HIPCHECK(hipMemcpyAsync(b.hword + 2, dw, 4, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    return b.hword[2];
}

// ---- gather-merge
uint64_t gm_rank_bytes(const Compiled& C) {
    const uint64_t B = GM_HDR + (uint64_t)GM_MAXG * gm_rec_bytes(C.P.nacc, (uint32_t)C.rep_cols.size());
    return (B + 255) & ~255ull;
}

// this rank's scan packed into dst (header + records); GM_OK or GM_FAILED (the
// header says which either way)
uint32_t gm_local_part(DevCtx& c, const cqgpu_table* t, Compiled& C, uint8_t* dst, std::string& err) {
    GmHdr h;
    memset(&h, 0, sizeof h);
    try {
        HIPCHECK(hipMemsetAsync(dst, 0, GM_HDR, c.stream));
        Literals L;
        ScanStats st;
        memset(&st, 0, sizeof st);   // run_aggregate returns early (group_missing) without writing it
        GmSend gs;
        gs.dst = dst;
        gs.maxg = GM_MAXG;
        (void)run_aggregate(c, t, C, L, &st, nullptr, 0, nullptr, &gs);
        h.base = t->base_offset;
        h.records = st.records;
        h.passed = st.passed;
        h.slow_records = st.slow_records;
        h.lds_spills = st.lds_spills;
        // bytes [8, 48): base and statistics (status and ng are gm_pack_kernel's)
        HIPCHECK(hipMemcpyAsync(dst + 8, (const uint8_t*)&h + 8, 40, hipMemcpyHostToDevice, c.stream));
        return GM_OK;
    } catch (HipError& e) {
        err = e.msg;
    } catch (Ineligible& e) {
        err = e.why;
    } catch (std::exception& e) {
        err = e.what();
    }
    (void)hipGetLastError();
    memset(&h, 0, sizeof h);
    h.status = GM_FAILED;
    (void)hipMemcpyAsync(dst, &h, GM_HDR, hipMemcpyHostToDevice, c.stream);
    return GM_FAILED;
}

struct GmRoot {
    uint32_t* dstatus = nullptr;         // device: the merge's status word
    uint8_t* mail = nullptr;
};
// rank 0: the merge kernels over N ranks' records, the result into the mailbox
GmRoot gm_merge_launch(DevCtx& c, const Compiled& C, const uint8_t* recv, uint64_t B, uint32_t N) {
    DistBufs& db = dist_bufs();
    const uint32_t T = N * GM_MAXG;
    uint32_t cap = 64;
    while (cap < 2 * T) cap <<= 1;
    const uint32_t R = (uint32_t)C.rep_cols.size(), nacc = (uint32_t)C.P.nacc, ncell = R + nacc + 1;
    const size_t scan_b = cq_gm_scan_bytes(T);
    const size_t out_b = cq_pack_result_bytes(T, (int)nacc, ncell, GM_SB);
    size_t off = 0;
    auto part = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    const size_t o_state = part((size_t)cap * 4), o_first = part((size_t)cap * 4), o_idx = part((size_t)N * T * 4);
    const size_t o_rec = part((size_t)cap * 4), o_slot = part((size_t)T * 4), o_flag = part((size_t)T * 4),
                 o_dense = part((size_t)T * 4), o_err = part(64), o_scan = part(scan_b), o_out = part(out_b);
    uint8_t* S = grow(db.scratch, db.scratch_b, off);
    // zero: state, err; 0xFF: first_of, idx (contiguous: one memset each)
    HIPCHECK(hipMemsetAsync(S + o_state, 0, o_first - o_state, c.stream));
    HIPCHECK(hipMemsetAsync(S + o_first, 0xFF, o_rec - o_first, c.stream));
    HIPCHECK(hipMemsetAsync(S + o_err, 0, 64, c.stream));
    GmRoot g;
    g.mail = mailbox(c, DIST_MAIL_HDR + out_b + 64);
    unsigned int* gcount = (unsigned int*)(S + o_err + 16);
    HIPCHECK(cq_launch_gm_merge(recv, B, N, GM_MAXG, (int)nacc, R, C.grouped ? 1 : 0, GM_SB, (uint32_t*)(S + o_state),
                                (uint32_t*)(S + o_rec), (uint32_t*)(S + o_first), cap, (uint32_t*)(S + o_slot),
                                (uint32_t*)(S + o_flag), (uint32_t*)(S + o_dense), (uint32_t*)(S + o_idx), S + o_scan,
                                scan_b, (unsigned int*)(S + o_err), S + o_out, gcount, g.mail, c.stream));
    HIPCHECK(cq_launch_mail_copy(S + o_out, gcount, T, (int)nacc, ncell, GM_SB, g.mail + DIST_MAIL_HDR, c.stream));
    g.dstatus = gcount + 1;
    return g;
}

// rank 0, after the stream's sync: the result table from the mailbox
cq_table* gm_finish_root(DevCtx& c, cq_node* q, Compiled& C, const uint8_t* mail) {
    ScanStats st;
    memcpy(&st, mail, sizeof st);
    uint32_t G = 0;
    memcpy(&G, mail + sizeof(ScanStats), 4);
    const uint32_t R = (uint32_t)C.rep_cols.size(), ncell = R + (uint32_t)C.P.nacc + 1;
    std::vector<int> rep_ord(R);
    for (uint32_t i = 0; i < R; i++) rep_ord[i] = (int)i;
    std::sort(rep_ord.begin(), rep_ord.end(), [&](int a, int b) { return C.rep_cols[a] < C.rep_cols[b]; });
    Literals L;
    parse_literals(c, C.lits, L);
    static thread_local std::vector<uint8_t> hbuf;
    const size_t pb = cq_pack_result_bytes(G, C.P.nacc, ncell, GM_SB);
    if (hbuf.size() < pb + 8) hbuf.resize(pb + 8);
    memcpy(hbuf.data(), mail + DIST_MAIL_HDR, pb);
    g_stats.records = st.records;
    g_stats.passed = st.passed;
    g_stats.slow_records = st.slow_records;
    g_stats.lds_spills = st.lds_spills;
    g_stats.groups = G;
    cq_table* res = build_direct(C, hbuf.data(), G, ncell, GM_SB, rep_ord, L, ~0ull);
    if (!res) throw HipError{"gather-merge: a result cell is not inline"};
    post_ops(c, res, q);
    g_stats.path = 1;
    return res;
}

// the gather-merge step; returns GM_OK (rank 0: *res), GM_DECLINE, or throws PeerFail.
// `D` is the plan-only compile of dist_path -- identical on every rank -- so every
// rank derives the same per-rank send size B from it (a rank whose own compile threw
// partway still sends and receives exactly B bytes).  Rank 0 runs the merge AND
// builds the result before it broadcasts its final status, so a throw anywhere on
// rank 0 (merge launch, literals, result table, post-ops) becomes GM_FAILED on every
// rank after the same collectives, never a hang or a one-sided failure.
uint32_t dist_gm(DevCtx& c, DistComm& m, cq_node* q, const cqgpu_table* t, const Compiled& D, cq_table** res) {
    Compiled C;
    std::string err;
    uint32_t mine = GM_OK;
    try {
        compile_aggregate(t, q, C);
        if (C.P.nacc != D.P.nacc || C.rep_cols.size() != D.rep_cols.size())
            throw HipError{"gather-merge: the table's compile differs from the plan's"};
    } catch (Ineligible& e) {
        err = e.why;
        mine = GM_FAILED;
    } catch (HipError& e) {
        err = e.msg;
        mine = GM_FAILED;
    }
    const uint32_t N = (uint32_t)m.world;
    const uint64_t B = gm_rank_bytes(D);
    DistBufs& db = dist_bufs();
    uint8_t* recv = m.rank == 0 ? grow(db.recv, db.recv_b, B * N) : nullptr;
    uint8_t* dst = m.rank == 0 ? recv : grow(db.send, db.send_b, B);
    if (mine == GM_OK && getenv("CQGPU_TEST_GM_FAIL_PART")) {      // test knob: this rank's part fails
        err = "gather-merge: injected local failure (CQGPU_TEST_GM_FAIL_PART)";
        mine = GM_FAILED;
    }
    if (mine == GM_OK) {
        mine = gm_local_part(c, t, C, dst, err);
    } else {
        GmHdr h;
        memset(&h, 0, sizeof h);
        h.status = GM_FAILED;
        HIPCHECK(hipMemcpyAsync(dst, &h, GM_HDR, hipMemcpyHostToDevice, c.stream));
    }
    m.be->group_start();
    if (m.rank == 0) {
        for (uint32_t r = 1; r < N; r++) m.be->recv(recv + r * B, B, CD_U8, (int)r, c.stream);
    } else {
        m.be->send(dst, B, CD_U8, 0, c.stream);
    }
    m.be->group_end(c.stream);
    uint32_t fin = GM_OK;                               // rank 0: the final status
    std::string rerr;
    if (m.rank == 0) {
        try {
            GmRoot g = gm_merge_launch(c, D, recv, B, N);   // (D: every rank's layout, even if C threw)
            HIPCHECK(hipStreamSynchronize(c.stream));
            memcpy(&fin, g.mail + sizeof(ScanStats) + 4, 4);   // the merge's status word (mailbox)
            if (fin == GM_OK) {
                if (getenv("CQGPU_TEST_GM_FAIL_FINISH")) throw HipError{"gather-merge: injected finish failure"};
                *res = gm_finish_root(c, q, C, g.mail);
            } else if (fin != GM_DECLINE) {
                fin = GM_FAILED;
                rerr = mine == GM_FAILED ? err : std::string("a peer rank failed");
            }
        } catch (HipError& e) {
            fin = GM_FAILED;
            rerr = e.msg;
        } catch (Ineligible& e) {
            fin = GM_FAILED;
            rerr = e.why;
        } catch (std::exception& e) {
            fin = GM_FAILED;
            rerr = e.what();
        }
        (void)hipGetLastError();
        if (fin != GM_OK && *res) { cqgpu_result_free(*res); *res = nullptr; }
        db.hword[8] = fin;
        HIPCHECK(hipMemcpyAsync(db.word.as<uint32_t>() + 12, db.hword + 8, 4, hipMemcpyHostToDevice, c.stream));
    }
    const uint32_t st = bcast_status(c, m, db.word.as<uint32_t>() + 12);
    if (st == GM_FAILED) {
        if (*res) { cqgpu_result_free(*res); *res = nullptr; }
        throw PeerFail{m.rank == 0 ? rerr : (mine == GM_FAILED ? err : std::string("a peer rank failed"))};
    }
    if (st == GM_DECLINE) return GM_DECLINE;
    return GM_OK;
}

// ---- dense merge: the cqgpu_partial stage sequence issued here over RCCL
// the collective a rank that failed mid-loop still issues at stage `at` (counts of
// the reduces follow from G, known on every rank after the KEYS agreement; its
// all-gathers send nothing and report the failure in the size exchange)
cqgpu_coll expected_coll(const cqgpu_partial* p, size_t at) {
    cqgpu_coll x;
    memset(&x, 0, sizeof x);
    if (!p || at >= p->stages.size()) { x.op = COLL_DONE; return x; }
    const uint64_t g = p->G, nmm = p->mm.size(), C = p->R + nmm;
    switch (p->stages[at]) {
        case ST_KEYS: case ST_STRS: case ST_SIDE: x.op = COLL_ALLGATHER; x.count = 0; break;
        case ST_MIN: x.op = COLL_ALLREDUCE_MIN_I64; x.count = g * p->P; break;
        case ST_SUM: x.op = COLL_ALLREDUCE_SUM_F64; x.count = g * p->W; break;
        case ST_EXT: x.op = COLL_ALLREDUCE_MIN_I64; x.count = g * nmm; break;
        case ST_CELL: x.op = COLL_REDUCE_SUM_I64; x.count = g * C * 2; break;
        case ST_VLA: x.op = COLL_REDUCE_SUM_F64; x.count = g * p->NV; break;
        case ST_SUMR: x.op = COLL_REDUCE_SUM_F64; x.count = g * p->W; break;
    }
    return x;
}

// all-gather of a variable-length device byte buffer: sizes (with this rank's failure
// flag) first -- the one host synchronisation a data-dependent size needs -- then
// the payloads padded to the largest; *out holds them concatenated in rank order
bool allgather_var(DevCtx& c, DistComm& m, const void* buf, uint64_t n, bool bad, DevBuf& out,
                   std::vector<uint64_t>& sizes) {
    const int N = m.world;
    DevBuf pair((size_t)N * 16 + 16);
    uint64_t* dp = pair.as<uint64_t>();
    uint64_t mine[2] = {bad ? 0 : n, bad ? 1ull : 0ull};
    HIPCHECK(hipMemcpyAsync(dp + 2 * N, mine, 16, hipMemcpyHostToDevice, c.stream));
    m.be->all_gather(dp + 2 * N, dp, 2, CD_U64, c.stream);
    std::vector<uint64_t> all((size_t)2 * N);
    HIPCHECK(hipMemcpyAsync(all.data(), dp, all.size() * 8, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    bool any = false;
    uint64_t mx = 1, tot = 0;
    sizes.assign(N, 0);
    for (int r = 0; r < N; r++) {
        any = any || all[2 * r + 1] != 0;
        sizes[r] = all[2 * r];
        mx = std::max(mx, sizes[r]);
        tot += sizes[r];
    }
    if (any) return false;
    DevBuf pad(mx), gathered(mx * N);
    if (n) HIPCHECK(hipMemcpyAsync(pad.p, buf, n, hipMemcpyDeviceToDevice, c.stream));
    m.be->all_gather(pad.p, gathered.p, mx, CD_U8, c.stream);
    DevBuf cat(std::max<uint64_t>(tot, 16));
    uint64_t at = 0;
    for (int r = 0; r < N; r++) {
        if (sizes[r])
            HIPCHECK(hipMemcpyAsync(cat.as<uint8_t>() + at, gathered.as<uint8_t>() + (uint64_t)r * mx, sizes[r],
                                    hipMemcpyDeviceToDevice, c.stream));
        at += sizes[r];
    }
    std::swap(out.p, cat.p);
    HIPCHECK(hipStreamSynchronize(c.stream));      // before pad / gathered go back to the pool
    return true;
}

// returns 0 (rank 0: *res), 1 declined (blobs); throws PeerFail
int dist_dense(DevCtx& c, DistComm& m, cq_node* q, cqgpu_table* t, cq_table** res) {
    std::string err;
    cqgpu_partial* p = cqgpu_partial_new(q, &t, 1);
    const bool inel = !p && !g_inel.empty();
    bool bad = !p && !inel;
    if (bad) err = g_err;
    // entry: did any rank fail, is any rank off the dense path (one MAX all-reduce of two words)
    {
        DistBufs& b = dist_bufs();
        b.hword[0] = bad ? 1u : 0u;
        b.hword[1] = inel ? 1u : 0u;
        uint32_t* dw = b.word.as<uint32_t>() + 8;
        HIPCHECK(hipMemcpyAsync(dw, b.hword, 8, hipMemcpyHostToDevice, c.stream));
        m.be->all_reduce(dw, 2, CD_U32, CR_MAX, c.stream);
        HIPCHECK(hipMemcpyAsync(b.hword + 4, dw, 8, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        if (b.hword[4]) {
            if (p) cqgpu_partial_free(p);
            throw PeerFail{bad ? err : std::string("a peer rank failed")};
        }
        if (b.hword[5]) {
            if (p) cqgpu_partial_free(p);
            return 1;
        }
    }
    std::unique_ptr<cqgpu_partial> own(p);
    DevBuf result;
    std::vector<uint64_t> sizes;
    bool have_sizes = false, have_result = false;
    size_t cur = 0;
    while (true) {
        cqgpu_coll nx;
        memset(&nx, 0, sizeof nx);
        const size_t before = cur;
        if (!bad) {
            if (cqgpu_partial_next(p, have_result ? result.p : nullptr, have_sizes ? sizes.data() : nullptr, m.rank,
                                   m.world, &nx) != 0) {
                bad = true;
                err = g_err;
            }
        }
        if (bad) nx = expected_coll(p, before);
        cur = before + 1;
        // the KEYS result just built the dictionary (G): agree before counts depend on it
        if (before == 1 && agree_any(c, m, bad)) throw PeerFail{bad ? err : std::string("a peer rank failed")};
        if (nx.op == COLL_DONE) break;
        if (nx.op == COLL_DECLINE) return 1;            // (every rank: it depends on the gathered keys)
        const size_t elem = nx.op == COLL_ALLGATHER ? 1 : 8;
        DevBuf buf(std::max<size_t>(nx.count * elem, 16));
        if (!bad && nx.count && cqgpu_partial_put(p, buf.p) != 0) {
            bad = true;
            err = g_err;
        }
        have_sizes = false;
        if (nx.op == COLL_ALLGATHER) {
            if (!allgather_var(c, m, buf.p, bad ? 0 : nx.count, bad, result, sizes))
                throw PeerFail{bad ? err : std::string("a peer rank failed")};
            have_sizes = true;
        } else {
            if (nx.count) {
                const CollDt ty = (nx.op == COLL_ALLREDUCE_SUM_F64 || nx.op == COLL_REDUCE_SUM_F64) ? CD_F64 : CD_I64;
                if (nx.op == COLL_ALLREDUCE_MIN_I64 || nx.op == COLL_ALLREDUCE_SUM_F64)
                    m.be->all_reduce(buf.p, nx.count, ty, nx.op == COLL_ALLREDUCE_MIN_I64 ? CR_MIN : CR_SUM, c.stream);
                else
                    m.be->reduce(buf.p, nx.count, ty, CR_SUM, 0, c.stream);
            }
            std::swap(result.p, buf.p);
        }
        have_result = true;
    }
    if (agree_any(c, m, bad)) throw PeerFail{bad ? err : std::string("a peer rank failed")};
    // rank 0's result, then its status to every rank
    DistBufs& b = dist_bufs();
    std::string rerr;
    if (m.rank == 0) {
        *res = cqgpu_partial_result(p, q);
        if (!*res) rerr = g_err;
        b.hword[8] = *res ? 0u : 1u;
        HIPCHECK(hipMemcpyAsync(b.word.as<uint32_t>() + 12, b.hword + 8, 4, hipMemcpyHostToDevice, c.stream));
    }
    if (bcast_status(c, m, b.word.as<uint32_t>() + 12)) {
        if (*res) { cqgpu_result_free(*res); *res = nullptr; }
        throw PeerFail{m.rank == 0 ? rerr : std::string("rank 0 failed to finish the merge")};
    }
    return 0;
}

// ---- blobs: every rank's cqgpu_query_partial to rank 0, merged there
// (blob: this rank's partial, malloc'd -- freed here; n == 0: this rank failed with err)
void dist_blob_send(DevCtx& c, DistComm& m, cq_node* q, void* blob, size_t n, const std::string& err_in,
                    cq_table** res);
void dist_blob(DevCtx& c, DistComm& m, cq_node* q, cqgpu_table* const* tabs, int ntabs, cq_table** res,
               bool bad_in = false, const std::string& err_in = std::string()) {
    void* blob = nullptr;
    const size_t n = bad_in ? 0 : cqgpu_query_partial(q, tabs, ntabs, &blob);
    const std::string err = bad_in ? err_in : (n == 0 ? (g_err.empty() ? g_inel : g_err) : std::string());
    dist_blob_send(c, m, q, blob, n, err, res);
}
void dist_blob_send(DevCtx& c, DistComm& m, cq_node* q, void* blob, size_t n, const std::string& err_in,
                    cq_table** res) {
    const bool bad = n == 0;
    const std::string err = err_in;
    struct Free { void* b; ~Free() { free(b); } } fr{blob};
    const int N = m.world;
    DevBuf pair((size_t)N * 16 + 16), dblob(std::max<size_t>(n, 16));
    uint64_t* dp = pair.as<uint64_t>();
    uint64_t mine[2] = {bad ? 0 : (uint64_t)n, bad ? 1ull : 0ull};
    HIPCHECK(hipMemcpyAsync(dp + 2 * N, mine, 16, hipMemcpyHostToDevice, c.stream));
    m.be->all_gather(dp + 2 * N, dp, 2, CD_U64, c.stream);
    std::vector<uint64_t> all((size_t)2 * N);
    HIPCHECK(hipMemcpyAsync(all.data(), dp, all.size() * 8, hipMemcpyDeviceToHost, c.stream));
    if (n) HIPCHECK(hipMemcpyAsync(dblob.p, blob, n, hipMemcpyHostToDevice, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
    for (int r = 0; r < N; r++)
        if (all[2 * r + 1]) throw PeerFail{bad ? err : std::string("a peer rank failed")};
    std::vector<uint64_t> off(N + 1, 0);
    for (int r = 0; r < N; r++) off[r + 1] = off[r] + all[2 * r];
    DevBuf gathered(m.rank == 0 ? std::max<uint64_t>(off[N], 16) : 16);
    m.be->group_start();
    if (m.rank == 0) {
        for (int r = 1; r < N; r++)
            if (all[2 * r]) m.be->recv(gathered.as<uint8_t>() + off[r], all[2 * r], CD_U8, r, c.stream);
    } else {
        m.be->send(dblob.p, n, CD_U8, 0, c.stream);
    }
    m.be->group_end(c.stream);
    DistBufs& b = dist_bufs();
    std::string rerr;
    if (m.rank == 0) {
        std::vector<uint8_t> h(off[N]);
        if (off[N] > off[1])
            HIPCHECK(hipMemcpyAsync(h.data() + off[1], gathered.as<uint8_t>() + off[1], off[N] - off[1],
                                    hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        memcpy(h.data(), blob, n);
        std::vector<const void*> ptrs(N);
        std::vector<size_t> sz(N);
        for (int r = 0; r < N; r++) { ptrs[r] = h.data() + off[r]; sz[r] = all[2 * r]; }
        *res = cqgpu_merge_partials(q, ptrs.data(), sz.data(), N);
        if (!*res) rerr = g_err;
        b.hword[8] = *res ? 0u : 1u;
        HIPCHECK(hipMemcpyAsync(b.word.as<uint32_t>() + 12, b.hword + 8, 4, hipMemcpyHostToDevice, c.stream));
    }
    if (bcast_status(c, m, b.word.as<uint32_t>() + 12)) {
        if (*res) { cqgpu_result_free(*res); *res = nullptr; }
        throw PeerFail{m.rank == 0 ? rerr : std::string("rank 0 failed to finish the merge")};
    }
}

// ---- the repartitioned JOIN step (cqgpu_dist_join): per side the device routing
// (cqgpu_route_plan: whole keys by key mod N, others by hash), every rank's per-
// destination byte / record counts in one all-gather (with each rank's failure flag),
// the records and their global ids in one grouped send / recv per side over the
// communicator, the received records rebuilt as this rank's side (file order, global
// ids, key stride N, whole-input record total), then the join partials as blobs to
// rank 0 (dist_blob).  No host round trip carries data; the host reads only counts.
// ---- the typed exchange inside cqgpu_dist_join (see "typed join exchange" above):
// every rank decides the same at every step -- from the plan, then from flags and
// counts every rank has gathered -- so the ranks take it, retry it or leave it for the
// CSV-record exchange together.  Returns true when *res / the status is final.
bool g_join_typed = false;             // the last cqgpu_dist_join took the typed exchange
bool dist_join_typed(DevCtx& c, DistComm& m, cq_node* q, cqgpu_table* const* tables, int ntables, cq_table** res) {
    const int N = m.world;
    if (ntables != 2 || N > 16) return false;
    TypedJoin tj;
    std::string why;
    if (!typed_join_plan(q, tables[0], tables[1], tj, why)) return false;   // (the plan: the same everywhere)
    struct Drop {
        cqgpu_table* const* t;
        ~Drop() { t[0]->tsend.reset(); t[1]->tsend.reset(); }
    } drop_{tables};
    std::string err;
    bool bad = false;
    auto gather_words = [&](const std::vector<uint64_t>& mine, std::vector<uint64_t>& all) {
        const size_t W = mine.size();
        all.assign(W * (size_t)N, 0);
        DevBuf dc(W * 8 * ((size_t)N + 1));
        HIPCHECK(hipMemcpyAsync(dc.as<uint8_t>() + W * 8 * N, mine.data(), W * 8, hipMemcpyHostToDevice, c.stream));
        m.be->all_gather(dc.as<uint8_t>() + W * 8 * N, dc.p, W, CD_U64, c.stream);
        HIPCHECK(hipMemcpyAsync(all.data(), dc.p, W * 8 * N, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
    };
    // the first qbase: the ranks' sampled build keys' minimum / N
    std::vector<uint64_t> g;
    gather_words({tables[0]->n > tables[0]->data_begin ? typed_sample_kmin(tables[0], tj.kl) : ~0ull}, g);
    uint64_t smin = ~0ull;
    for (int r = 0; r < N; r++) smin = std::min(smin, g[r]);
    uint64_t qbase = smin == ~0ull ? 0 : smin / (uint64_t)N;
    // count passes: per rank [counts_u[N], counts_o[N], flags, kmin, kmax, records, bad]
    const size_t W = 2 * (size_t)N + 5;
    for (int attempt = 0;; attempt++) {
        std::vector<uint64_t> mine(W, 0);
        try {
            if (getenv("CQGPU_TEST_TYPED_FAIL"))                 // test knob: this rank's send fails
                throw HipError{"dist_join: injected typed-exchange failure (CQGPU_TEST_TYPED_FAIL)"};
            const TypedSend& su = typed_count_pass(c, tables[0], true, tj.kl, N, qbase);
            const TypedSend& so = typed_count_pass(c, tables[1], false, tj.kr, N, qbase, tj.vcol);
            for (int d = 0; d < N; d++) { mine[d] = su.counts[d]; mine[N + d] = so.counts[d]; }
            mine[2 * N] = su.flags | so.flags;
            mine[2 * N + 1] = su.krange[0];
            mine[2 * N + 2] = su.krange[1];
            mine[2 * N + 3] = su.nrec;
        } catch (HipError& e) { bad = true; err = e.msg; } catch (Ineligible& e) { bad = true; err = e.why; }
        (void)hipGetLastError();
        mine[2 * N + 4] = bad ? 1 : 0;
        gather_words(mine, g);
        uint64_t flags = 0, kmin = ~0ull;
        for (int r = 0; r < N; r++) {
            const uint64_t* x = g.data() + W * r;
            if (x[2 * N + 4]) throw PeerFail{bad ? err : std::string("a peer rank failed")};
            flags |= x[2 * N];
            kmin = std::min(kmin, x[2 * N + 1]);
        }
        if ((flags & (1u | 8u)) || ((flags & 16u) && attempt >= 1)) return false;   // every rank to the CSV exchange
        if (flags & 16u) {                                        // again with the build keys' own minimum
            qbase = kmin / (uint64_t)N;
            continue;
        }
        break;
    }
    uint64_t kmin = ~0ull, kmax = 0, gbase = 0, total = 0;
    std::vector<uint64_t> recv_u(N, 0), recv_o(N, 0);
    for (int r = 0; r < N; r++) {
        const uint64_t* x = g.data() + W * r;
        kmin = std::min(kmin, x[2 * N + 1]);
        kmax = std::max(kmax, x[2 * N + 2]);
        if (r < m.rank) gbase += x[2 * N + 3];
        total += x[2 * N + 3];
        for (int d = 0; d < N; d++) { recv_u[d] += x[d]; recv_o[d] += x[N + d]; }
    }
    if (total >= (1ull << 32)) return false;
    if (kmin > kmax) kmin = kmax = qbase * (uint64_t)N;            // no build keys anywhere
    const uint64_t qoff = kmin / (uint64_t)N - qbase, range = kmax / (uint64_t)N - kmin / (uint64_t)N + 1;
    if (range > 4 * *std::min_element(recv_u.begin(), recv_u.end()) + 1024 || range >= (1ull << 31))
        return false;                                             // not a dense key range on every rank
    // emit passes, then one agreement on their flags (a GROUP BY value or a payload the
    // entries cannot carry: every rank to the CSV exchange) and on failures
    uint32_t ef = 0;
    DevBuf ru, ro;
    try {
        ef |= typed_emit_pass(c, tables[0], true, tj.kl, tj.gcol, gbase);
        ef |= typed_emit_pass(c, tables[1], false, tj.kr, tj.vcol, 0);
        DevBuf a(std::max<uint64_t>(recv_u[m.rank], 1) * 16), b(std::max<uint64_t>(recv_o[m.rank], 1) * 8);
        std::swap(ru.p, a.p);
        std::swap(ro.p, b.p);
    } catch (HipError& e) { bad = true; err = e.msg; }
    (void)hipGetLastError();
    {
        DistBufs& b = dist_bufs();
        b.hword[0] = bad ? 1u : 0u;
        b.hword[1] = ef ? 1u : 0u;
        uint32_t* dw = b.word.as<uint32_t>() + 8;
        HIPCHECK(hipMemcpyAsync(dw, b.hword, 8, hipMemcpyHostToDevice, c.stream));
        m.be->all_reduce(dw, 2, CD_U32, CR_MAX, c.stream);
        HIPCHECK(hipMemcpyAsync(b.hword + 4, dw, 8, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        if (b.hword[4]) throw PeerFail{bad ? err : std::string("a peer rank failed")};
        if (b.hword[5]) return false;
    }
    // the entries: region d of every rank to rank d, in one grouped send / recv per side
    for (int side = 0; side < 2; side++) {
        const TypedSend& ts = *tables[side]->tsend;
        uint8_t* rb = side == 0 ? ru.as<uint8_t>() : ro.as<uint8_t>();
        m.be->group_start();
        uint64_t at = 0;
        for (int d = 0; d < N; d++) {
            const uint64_t ns = ts.counts[d];
            if (ns) m.be->send(ts.ent.as<uint8_t>() + ts.rstart[d] * ts.esize, ns * ts.esize, CD_U8, d, c.stream);
            const uint64_t nr = g[W * d + (size_t)side * N + m.rank];          // from source d
            if (nr) m.be->recv(rb + at * ts.esize, nr * ts.esize, CD_U8, d, c.stream);
            at += nr;
        }
        m.be->group_end(c.stream);
    }
    tables[0]->tsend.reset();
    tables[1]->tsend.reset();
    // this rank's STAR join over its entries; a rank whose entries do not fit (a repeated
    // build key, more than JX_G groups) sends every rank back to the CSV exchange
    JoinPartial jp;
    uint32_t fl = 0;
    try {
        fl = typed_receive(c, tj, ru.p, recv_u[m.rank], ro.p, recv_o[m.rank], qoff, range, jp);
    } catch (HipError& e) { bad = true; err = e.msg; }
    (void)hipGetLastError();
    {
        DistBufs& b = dist_bufs();
        b.hword[0] = bad ? 1u : 0u;
        b.hword[1] = fl ? 1u : 0u;
        uint32_t* dw = b.word.as<uint32_t>() + 8;
        HIPCHECK(hipMemcpyAsync(dw, b.hword, 8, hipMemcpyHostToDevice, c.stream));
        m.be->all_reduce(dw, 2, CD_U32, CR_MAX, c.stream);
        HIPCHECK(hipMemcpyAsync(b.hword + 4, dw, 8, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
        if (b.hword[4]) throw PeerFail{bad ? err : std::string("a peer rank failed")};
        if (b.hword[5]) return false;
    }
    void* blob = nullptr;
    size_t n = 0;
    try {
        Blob bb;
        join_blob(jp, bb);
        blob = malloc(std::max<size_t>(bb.d.size(), 1));
        if (!blob) throw HipError{"out of host memory"};
        memcpy(blob, bb.d.data(), bb.d.size());
        n = bb.d.size();
    } catch (HipError& e) { err = e.msg; n = 0; }
    g_join_typed = true;
    dist_blob_send(c, m, q, blob, n, err, res);
    return true;
}

void dist_join(DevCtx& c, DistComm& m, cq_node* q, cqgpu_table* const* tables, int ntables, cq_table** res) {
    if (!getenv("CQGPU_NO_TYPED_JOIN") && dist_join_typed(c, m, q, tables, ntables, res)) return;
    const int N = m.world;
    std::string err;
    bool bad = false;
    struct TabFree { void operator()(cqgpu_table* t) const { if (t) cqgpu_table_free(t); } };
    std::vector<std::unique_ptr<cqgpu_table, TabFree>> routed;
    auto plan_failed = [&]() {
        bad = true;
        err = g_err.empty() ? g_inel : g_err;
        if (!g_inel.empty()) err = "query outside the GPU executor's subset: " + g_inel;
    };
    // the routing mode, agreed before either side moves (cqgpu_route_plan2): a JOIN
    // without ON keeps side 0 and sends side 1 to every rank; keys of several value
    // classes (value_compare's cross-class "equal", csv_reader.c:126-129) route the
    // majority class by key and replicate the others.  Both sides' mode-0 plans give
    // the class counts; they are kept when the mode stays 0.
    cq_node* j0 = q && q->kind == CQ_N_QUERY && q->u.q.join_count > 0 ? q->u.q.joins[0] : nullptr;
    const bool cross = j0 && j0->kind == CQ_N_JOIN && j0->u.join.on == nullptr;
    uint32_t mode = 0;
    std::unique_ptr<RouteState> pre[2];
    std::vector<uint64_t> pre_nb[2], pre_nr[2];
    if (!cross) {
        uint64_t cc[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
        for (int side = 0; side < 2 && !bad; side++) {
            pre_nb[side].assign(N, 0);
            pre_nr[side].assign(N, 0);
            if (cqgpu_route_plan2(q, tables, ntables, side, N, m.rank, 0, pre_nb[side].data(), pre_nr[side].data(),
                                  cc[side]) < 0)
                plan_failed();
            else
                pre[side] = std::move(tables[side]->route);    // (tables[0] may be tables[1]: a self-join)
        }
        std::vector<uint64_t> mine(9, 0), all(9 * (size_t)N, 0);
        for (int k = 0; k < 4; k++) { mine[k] = cc[0][k]; mine[4 + k] = cc[1][k]; }
        mine[8] = bad ? 1 : 0;
        {
            DevBuf dc(9 * 8 * (N + 1));
            uint64_t* dp = dc.as<uint64_t>();
            HIPCHECK(hipMemcpyAsync(dp + 9 * N, mine.data(), 9 * 8, hipMemcpyHostToDevice, c.stream));
            m.be->all_gather(dp + 9 * N, dp, 9, CD_U64, c.stream);
            HIPCHECK(hipMemcpyAsync(all.data(), dp, 9 * N * 8, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
        }
        uint64_t lc[4] = {0, 0, 0, 0}, rc[4] = {0, 0, 0, 0};
        for (int r = 0; r < N; r++) {
            if (all[(size_t)r * 9 + 8]) throw PeerFail{bad ? err : std::string("a peer rank failed")};
            for (int k = 0; k < 4; k++) { lc[k] += all[(size_t)r * 9 + k]; rc[k] += all[(size_t)r * 9 + 4 + k]; }
        }
        mode = cqgpu_route_major(lc, rc);
        if (mode) pre[0].reset(), pre[1].reset();     // re-planned with the mode below
    }
    for (int side = 0; side < 2; side++) {
        std::vector<uint64_t> nb(N, 0), nr(N, 0);
        uint64_t nown = 0;                         // this rank's records of the side (global id span)
        if (!bad && pre[side]) {
            nb = pre_nb[side];
            nr = pre_nr[side];
            nown = pre[side]->n;
            tables[side]->route = std::move(pre[side]);
        } else if (!bad) {
            const int64_t n = cqgpu_route_plan2(q, tables, ntables, side, N, m.rank, mode, nb.data(), nr.data(),
                                                nullptr);
            if (n < 0) plan_failed();
            else nown = (uint64_t)n;
        }
        // all ranks' counts: [nb(N), nr(N), bad, own records] per rank
        const size_t W = 2 * (size_t)N + 2;
        std::vector<uint64_t> mine(W, 0), all(W * N, 0);
        for (int d = 0; d < N; d++) { mine[d] = bad ? 0 : nb[d]; mine[N + d] = bad ? 0 : nr[d]; }
        mine[2 * N] = bad ? 1 : 0;
        mine[2 * N + 1] = bad ? 0 : nown;
        {
            DevBuf dc(W * 8 * (N + 1));
            uint64_t* dp = dc.as<uint64_t>();
            HIPCHECK(hipMemcpyAsync(dp + W * N, mine.data(), W * 8, hipMemcpyHostToDevice, c.stream));
            m.be->all_gather(dp + W * N, dp, W, CD_U64, c.stream);
            HIPCHECK(hipMemcpyAsync(all.data(), dp, W * N * 8, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
        }
        for (int r = 0; r < N; r++)
            if (all[(size_t)r * W + 2 * N]) {
                if (tables[side]) tables[side]->route.reset();
                throw PeerFail{bad ? err : std::string("a peer rank failed")};
            }
        // global ids: this rank's records follow every lower rank's; the whole input's total
        uint64_t base = 0, total = 0;
        std::vector<uint64_t> sb(N + 1, 0), sr(N + 1, 0), rb(N + 1, 0), rr(N + 1, 0);
        for (int r = 0; r < N; r++) {
            const uint64_t recs = all[(size_t)r * W + 2 * N + 1];
            if (r < m.rank) base += recs;
            total += recs;
        }
        for (int d = 0; d < N; d++) {
            sb[d + 1] = sb[d] + nb[d];
            sr[d + 1] = sr[d] + nr[d];
            rb[d + 1] = rb[d] + all[(size_t)d * W + m.rank];          // from source d, in source order
            rr[d + 1] = rr[d] + all[(size_t)d * W + N + m.rank];
        }
        if (total >= (1ull << 32)) throw PeerFail{"dist_join: 2^32 or more records on a join side"};   // (every rank)
        // every buffer sized by the agreed counts, allocated and filled under one try:
        // a rank that fails here (a receive side sized by key skew can run out of
        // memory) says so in one agreement BEFORE the grouped send / recv, so no rank
        // is left waiting in a transfer its peer never posts
        DevBuf sbytes, sgids, rbytes, rgids, sg32, rg32;
        try {
            if (getenv("CQGPU_TEST_DIST_FAIL_ALLOC"))           // test knob: this rank's allocation fails
                throw HipError{"dist_join: injected exchange allocation failure (CQGPU_TEST_DIST_FAIL_ALLOC)"};
            DevBuf a(std::max<uint64_t>(sb[N], 16)), b(std::max<uint64_t>(sr[N], 2) * 8);
            DevBuf e(std::max<uint64_t>(rb[N], 16)), f(std::max<uint64_t>(rr[N], 2) * 8);
            // the ids travel as 32 bits (total < 2^32 above): 4 bytes a record off the exchange
            DevBuf g(std::max<uint64_t>(sr[N], 2) * 4), h(std::max<uint64_t>(rr[N], 2) * 4);
            std::swap(sbytes.p, a.p);
            std::swap(sgids.p, b.p);
            std::swap(rbytes.p, e.p);
            std::swap(rgids.p, f.p);
            std::swap(sg32.p, g.p);
            std::swap(rg32.p, h.p);
            if (cqgpu_route_fill(tables[side], base, sbytes.p, sgids.as<uint64_t>()) != 0) throw HipError{g_err};
            HIPCHECK(cq_launch_gid_narrow(sgids.as<unsigned long long>(), sr[N], sg32.as<uint32_t>(), c.stream));
        } catch (HipError& e) {
            bad = true;
            err = e.msg;
        } catch (std::exception& e) {
            bad = true;
            err = e.what();
        }
        (void)hipGetLastError();
        if (agree_any(c, m, bad)) {
            if (tables[side]) tables[side]->route.reset();
            throw PeerFail{bad ? err : std::string("a peer rank failed")};
        }
        m.be->group_start();
        for (int d = 0; d < N; d++) {
            if (nb[d]) {
                m.be->send(sbytes.as<uint8_t>() + sb[d], nb[d], CD_U8, d, c.stream);
                m.be->send(sg32.as<uint32_t>() + sr[d], nr[d], CD_U32, d, c.stream);
            }
            if (rb[d + 1] > rb[d]) {
                m.be->recv(rbytes.as<uint8_t>() + rb[d], rb[d + 1] - rb[d], CD_U8, d, c.stream);
                m.be->recv(rg32.as<uint32_t>() + rr[d], rr[d + 1] - rr[d], CD_U32, d, c.stream);
            }
        }
        m.be->group_end(c.stream);
        // a local failure from here on is reported by the next agreement (side 1's count
        // gather, the outer levels' agreement or dist_blob's size gather)
        cqgpu_table* t = nullptr;
        try {
            HIPCHECK(cq_launch_gid_widen(rg32.as<uint32_t>(), rr[N], rgids.as<unsigned long long>(), c.stream));
            const std::string& hdr = tables[side]->header_rec;
            t = cqgpu_table_from_routed(rbytes.p, rb[N], rgids.as<uint64_t>(), rr[N], tables[side]->cfg, hdr.data(),
                                        hdr.size());
            if (!t) throw HipError{g_err};
        } catch (HipError& e) {
            bad = true;
            err = e.msg;
        } catch (std::exception& e) {
            bad = true;
            err = e.what();
        }
        (void)hipGetLastError();
        routed.emplace_back(t);
        if (t) {
            t->gid_total = total;
            t->key_stride = (uint32_t)N;
            t->rep_major = cross ? 0u : mode;
            t->bcast = cross && side == 1;
            t->rep_owner = m.rank == 0;
        }
    }
    std::vector<cqgpu_table*> tabs;
    tabs.push_back(routed[0].get());
    tabs.push_back(routed[1].get());
    for (int i = 2; i < ntables; i++) tabs.push_back(tables[i]);
    // a chain's later RIGHT / FULL levels: every rank's matched flags over the level's
    // whole table, OR-ed by a MAX all-reduce over bytes; rank 0's partial carries the
    // records no rank matched (cqgpu_join_outer_* in include/cqgpu.h)
    g_outer_sets.clear();
    struct ClearSets { ~ClearSets() { g_outer_sets.clear(); } } clear_sets_;
    const int nj = q && q->kind == CQ_N_QUERY ? q->u.q.join_count : 0;
    // every rank runs every level up to the plan's join count -- the plan is the same on
    // every rank, its table list may not be: a missing table is this rank's failure,
    // never a skipped collective
    for (int j = 1; j < nj; j++) {
        cq_node* jn = q->u.q.joins[j];
        if (!jn || jn->kind != CQ_N_JOIN || (jn->u.join.kind != CQ_JOIN_RIGHT && jn->u.join.kind != CQ_JOIN_FULL))
            continue;
        cqgpu_table* T = 1 + j < ntables ? tables[1 + j] : nullptr;   // whole on every rank: the same record count
        if (getenv("CQGPU_TEST_DIST_CHAIN_MISSING")) T = nullptr;     // test knob: this rank lacks the table
        uint64_t nrec = 0;
        if (!T) {
            bad = true;                           // (still in every collective below)
            err = "dist_join: a chain table is missing";
        } else {
            try {
                if (!T->rec_starts) {
                    std::unique_ptr<DevBuf> b(new DevBuf());
                    T->nrec_starts = all_records(c, T, *b);
                    T->rec_starts = std::move(b);
                }
                nrec = T->nrec_starts;
            } catch (HipError& e) {
                bad = true;
                err = e.msg;
            }
            (void)hipGetLastError();
        }
        {                                         // every rank sizes the flags alike
            DevBuf dn(16);
            uint64_t hv[2] = {nrec, ~nrec};       // MAX of n and of ~n: max and min at once
            HIPCHECK(hipMemcpyAsync(dn.p, hv, 16, hipMemcpyHostToDevice, c.stream));
            m.be->all_reduce(dn.p, 2, CD_U64, CR_MAX, c.stream);
            HIPCHECK(hipMemcpyAsync(hv, dn.p, 16, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
            if ((hv[0] != ~hv[1] || hv[0] != nrec) && !bad) {
                bad = true;
                err = "dist_join: a chain table's record count differs between ranks";
            }
            nrec = hv[0];
        }
        std::vector<uint8_t> flags;
        DevBuf dm;
        try {
            flags.assign(nrec, 0);
            if (nrec) {
                DevBuf x(nrec);
                std::swap(dm.p, x.p);
            }
        } catch (HipError& e) {
            bad = true;
            err = e.msg;
        } catch (std::exception& e) {
            bad = true;
            err = e.what();
        }
        if (agree_any(c, m, bad)) throw PeerFail{bad ? err : std::string("a peer rank failed")};
        {
            const uint8_t* fl = nullptr;
            uint64_t n = 0;
            const int r = cqgpu_join_outer_matched(q, tabs.data(), (int)tabs.size(), j, &fl, &n);
            if (r < 0 || (r == 1 && n != nrec)) {
                bad = true;
                err = r < 0 ? g_err : std::string("join_outer_matched: record count differs");
            } else if (r == 1 && n) {
                memcpy(flags.data(), fl, n);
            }
        }
        if (nrec) {
            HIPCHECK(hipMemcpyAsync(dm.p, flags.data(), nrec, hipMemcpyHostToDevice, c.stream));
            m.be->all_reduce(dm.p, nrec, CD_U8, CR_MAX, c.stream);
            HIPCHECK(hipMemcpyAsync(flags.data(), dm.p, nrec, hipMemcpyDeviceToHost, c.stream));
            HIPCHECK(hipStreamSynchronize(c.stream));
        }
        OuterSet& o = g_outer_sets[j];
        o.matched.swap(flags);
        o.emit = m.rank == 0;
    }
    dist_blob(c, m, q, tabs.data(), (int)tabs.size(), res, bad, err);
}

// the merge the plan takes, decided from the AST and the header alone (no device
// work: a table copy without its sample), so every rank decides the same
int dist_path(cq_node* q, const cqgpu_table* t, Compiled& D) {
    cqgpu_table shadow;
    shadow.names = t->names;
    shadow.cfg = t->cfg;
    check_plan_shape(q, &shadow);
    if (is_row_query(q)) return DP_BLOB;
    compile_aggregate(&shadow, q, D);
    if (gm_eligible(D)) return DP_GM;
    return dense_eligible(D) ? DP_DENSE : DP_BLOB;
}

}  // namespace

extern "C" {

int cqgpu_comm_unique_id(void* id_out) {
    g_err.clear();
    if (!id_out) return -1;
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        set_err("cq_amd: ncclGetUniqueId: %s", ncclGetErrorString(r));
        return -1;
    }
    static_assert(sizeof(ncclUniqueId) == CQGPU_COMM_ID_BYTES, "RCCL unique id size");
    memcpy(id_out, &id, sizeof id);
    return 0;
}

int cqgpu_comm_init(const void* id, int rank, int world) {
    g_err.clear();
    try {
        if (!id || world < 1 || rank < 0 || rank >= world) throw HipError{"comm_init: bad arguments"};
        int dev = 0;
        HIPCHECK(hipGetDevice(&dev));
        DistComm& m = g_comm[dev & 63];
        m.be.reset();
        ncclUniqueId uid;
        memcpy(&uid, id, sizeof uid);
        (void)ctx();                                   // the device context (stream) first
        std::unique_ptr<RcclColl> r(new RcclColl);
        NCCLCHECK(ncclCommInitRank(&r->comm, world, uid, rank));
        m.be = std::move(r);
        m.rank = rank;
        m.world = world;
        return 0;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return -1;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return -1;
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
        return -1;
    }
}

int cqgpu_comm_init_host(int rank, int world, cqgpu_coll_fn fn, void* user) {
    g_err.clear();
    try {
        if (!fn || world < 1 || rank < 0 || rank >= world) throw HipError{"comm_init_host: bad arguments"};
        int dev = 0;
        HIPCHECK(hipGetDevice(&dev));
        DistComm& m = g_comm[dev & 63];
        m.be.reset();
        (void)ctx();
        std::unique_ptr<HostColl> h(new HostColl);
        h->fn = fn;
        h->user = user;
        h->world = world;
        m.be = std::move(h);
        m.rank = rank;
        m.world = world;
        return 0;
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
        return -1;
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
        return -1;
    }
}

void cqgpu_comm_destroy(void) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    DistComm& m = g_comm[dev & 63];
    m.be.reset();
    m.rank = 0;
    m.world = 1;
}

cq_table* cqgpu_dist_query(cq_node* q, cqgpu_table* t, int* status, int* path) {
    g_err.clear();
    g_inel.clear();
    memset(&g_stats, 0, sizeof g_stats);
    if (status) *status = 0;
    if (path) *path = 0;
    cq_table* res = nullptr;
    try {
        if (!t) throw HipError{"dist_query: no table"};
        DevCtx& c = ctx();
        DistComm& m = dist_comm();
        bump_reset(c);
        const double t0 = now_ms();
        Compiled D;
        int dp = dist_path(q, t, D);                     // Ineligible: the same on every rank
        if (dp == DP_GM && dist_gm(c, m, q, t, D, &res) == GM_DECLINE) dp = DP_DENSE;
        if (dp == DP_DENSE && dist_dense(c, m, q, t, &res) != 0) dp = DP_BLOB;
        if (dp == DP_BLOB) dist_blob(c, m, q, &t, 1, &res);
        if (path) *path = dp;
        g_stats.total_ms = now_ms() - t0;
        if (m.rank == 0) g_stats.path = 1;
        return res;
    } catch (PeerFail& e) {
        set_err("cq_amd: %s", e.msg.c_str());
    } catch (Ineligible& e) {
        g_inel = e.why;
        set_err("cq_amd: query outside the GPU executor's subset: %s", e.why.c_str());
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
    }
    if (res) cqgpu_result_free(res);
    if (status) *status = -1;
    return nullptr;
}

cq_table* cqgpu_dist_join(cq_node* q, cqgpu_table* const* tables, int ntables, int* status) {
    g_err.clear();
    g_inel.clear();
    memset(&g_stats, 0, sizeof g_stats);
    if (status) *status = 0;
    cq_table* res = nullptr;
    try {
        if (ntables < 2 || !tables || !tables[0] || !tables[1]) throw HipError{"dist_join: two join sides needed"};
        DevCtx& c = ctx();
        DistComm& m = dist_comm();
        const double t0 = now_ms();
        g_join_typed = false;
        dist_join(c, m, q, tables, ntables, &res);
        g_stats.total_ms = now_ms() - t0;
        if (g_join_typed) g_stats.scan_kernel = 5;      // (the typed exchange's STAR join)
        if (m.rank == 0) g_stats.path = 1;
        return res;
    } catch (PeerFail& e) {
        set_err("cq_amd: %s", e.msg.c_str());
    } catch (Ineligible& e) {
        g_inel = e.why;
        set_err("cq_amd: query outside the GPU executor's subset: %s", e.why.c_str());
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
    }
    if (res) cqgpu_result_free(res);
    if (status) *status = -1;
    return nullptr;
}

// simulated ranks in one process: every shard's pack, then the root's merge
cq_table* cqgpu_gm_local(cq_node* q, cqgpu_table* const* shards, int n) {
    g_err.clear();
    g_inel.clear();
    memset(&g_stats, 0, sizeof g_stats);
    try {
        if (n < 1 || !shards) throw HipError{"gm_local: no shards"};
        DevCtx& c = ctx();
        bump_reset(c);
        Compiled D;
        if (dist_path(q, shards[0], D) != DP_GM) throw Ineligible{"gather-merge: plan outside it"};
        Compiled C;
        compile_aggregate(shards[0], q, C);
        const uint64_t B = gm_rank_bytes(C);
        DevBuf recv(B * (uint64_t)n);
        for (int r = 0; r < n; r++) {
            Compiled Cr;
            compile_aggregate(shards[r], q, Cr);
            std::string err;
            if (gm_local_part(c, shards[r], Cr, recv.as<uint8_t>() + (uint64_t)r * B, err) != GM_OK)
                throw HipError{"gm_local: shard " + std::to_string(r) + ": " + err};
        }
        GmRoot g = gm_merge_launch(c, C, recv.as<uint8_t>(), B, (uint32_t)n);
        HIPCHECK(hipStreamSynchronize(c.stream));
        uint32_t st = 0;
        memcpy(&st, g.mail + sizeof(ScanStats) + 4, 4);
        if (st == GM_DECLINE) throw Ineligible{"gather-merge: declined by the data"};
        if (st != GM_OK) throw HipError{"gm_local: merge failed"};
        return gm_finish_root(c, q, C, g.mail);
    } catch (Ineligible& e) {
        g_inel = e.why;
        set_err("cq_amd: %s", e.why.c_str());
    } catch (HipError& e) {
        set_err("cq_amd: %s", e.msg.c_str());
    } catch (std::exception& e) {
        set_err("cq_amd: %s", e.what());
    } catch (...) {
        set_err("cq_amd: %s", "unexpected C++ exception");
    }
    return nullptr;
}

}  // extern "C"
