/*
 * cqgpu.h -- C ABI of libcqgpu, the MI355X executor for cq's SELECT path.
 *
 * Drop-in boundary: the unchanged cq CLI and parser call
 *     ResultSet* evaluate_query(ASTNode* query_ast);     reference include/evaluator.h:32
 * and read/write the global CSV configuration
 *     extern CsvConfig global_csv_config;                reference include/evaluator.h:29,
 *                                                        defined evaluator.c:23
 * libcqgpu exports both symbols with the reference's exact binary layout
 * (include/cq_abi.h), so `main.c` plus the reference front-end objects link
 * against libcqgpu.so instead of the reference evaluator.
 *
 * Below the drop-in entry point the library exposes the pieces the benchmark
 * and the multi-GPU driver use: tables resident in HBM (the second boundary,
 * replacing csv_load, reference csv_reader.h:76, on the GPU path only) and
 * queries over resident tables.
 *
 * Error convention (reference evaluator.c:28, evaluator_joins.c:221): NULL
 * result plus a message on stderr; cqgpu_last_error() returns the message.
 * Calls are synchronous and not reentrant, like the reference's.
 */
#ifndef CQGPU_H
#define CQGPU_H

#include <stddef.h>
#include <stdint.h>
#include "cq_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- drop-in (reference evaluator.h) ------------------------------------- */
/* replaces evaluate_query (reference evaluator.c:290-348); returns a heap
 * result table the caller frees with the reference's csv_free (csv_reader.c:467)
 * or cqgpu_result_free. */
cq_table* evaluate_query(cq_node* query_ast);
/* replaces the reference global (evaluator.c:23), written by main.c:99-101 */
extern cq_csv_config global_csv_config;

/* ---- device-resident table cache of evaluate_query ------------------------
 * evaluate_query keeps each file's uploaded bytes in HBM between calls (the
 * reference re-reads the file per query), keyed by path + device/inode/size/
 * mtime + CSV config, so a changed file is re-read; LRU within a byte budget
 * (env CQGPU_TABLE_CACHE_BYTES, default 32 GiB; 0 disables). */
void cqgpu_cache_clear(void);
/* new budget in bytes (0 disables and empties); returns the previous budget */
long long cqgpu_set_cache_limit(long long bytes);
int cqgpu_cache_info(uint64_t* entries, uint64_t* bytes, uint64_t* hits);

/* ---- resident tables (replace csv_load on the GPU path) ------------------- */
typedef struct cqgpu_table cqgpu_table;
/* mmap + upload to the current HIP device (reference mmap.c:78-108 + csv_load) */
cqgpu_table* cqgpu_table_open(const char* path, cq_csv_config cfg);
/* upload a caller buffer; `base_offset` is the position of data[0] in the whole
 * file (0 unless this is a shard) and `header` the file's header record bytes
 * when the shard does not start at the file start (NULL otherwise). */
cqgpu_table* cqgpu_table_from_bytes(const void* data, size_t n, cq_csv_config cfg,
                                    uint64_t base_offset, const char* header, size_t header_len);
/* ---- range partition of one file over nranks GPUs ---
 * The data region (after the header record) is cut into nranks equal byte
 * ranges; every cut is snapped to the byte after the next run of '\n' / '\r'
 * (records split on any terminator, quote-blind, reference csv_reader.c:404-408),
 * so each record lies in exactly one range.  Rank 0's range starts at byte 0
 * (leading blank lines and the header included).  range_bounds is pure host
 * code (no device); it writes rank `rank`'s [*lo, *hi) and the header record
 * [*hdr_lo, *hdr_hi) (empty when cfg.has_header is false and the file has no
 * records).  Returns 0, or -1 on bad arguments. */
int cqgpu_range_bounds(const void* data, size_t n, cq_csv_config cfg, int rank, int nranks,
                       uint64_t* lo, uint64_t* hi, uint64_t* hdr_lo, uint64_t* hdr_hi);
/* mmap `path` and upload rank `rank`'s range of it (with its whole-file base
 * offset and the header record) to the current HIP device: the shard each rank
 * scans with cqgpu_query_partial before cqgpu_merge_partials. */
cqgpu_table* cqgpu_table_open_range(const char* path, cq_csv_config cfg, int rank, int nranks);
/* whole-file byte offset of a table's first byte (0 unless it is a shard) */
uint64_t cqgpu_table_base_offset(const cqgpu_table* t);

void cqgpu_table_free(cqgpu_table* t);
size_t cqgpu_table_bytes(const cqgpu_table* t);
int cqgpu_table_ncols(const cqgpu_table* t);

/* ---- queries over resident tables ---------------------------------------- */
/* FROM binds tables[0]; the j-th JOIN binds tables[1 + j]; paths in the plan
 * are ignored.  Same result contract as evaluate_query. */
cq_table* cqgpu_query(cq_node* query_ast, cqgpu_table* const* tables, int ntables);
void cqgpu_result_free(cq_table* r);

/* ---- partial aggregation for range-partitioned multi-GPU queries --------- */
/* Run the aggregate part of `query_ast` on this rank's shard and serialize the
 * per-group partial state (canonical keys, counts, sums, extremes, first-row
 * positions in whole-file byte offsets, representative cells) into a malloc'd
 * blob.  Returns blob size (0 on error); *blob_out is freed with free(). */
size_t cqgpu_query_partial(cq_node* query_ast, cqgpu_table* const* tables, int ntables,
                           void** blob_out);
/* A chain's later RIGHT / FULL JOIN across partials (perform_join's unmatched right
 * rows, evaluator_joins.c:143-171, chained through process_joins :268-270).  The
 * level's table is whole on every rank; its unmatched records are the ones no rank's
 * joined rows matched.  For each such level j, in order, before cqgpu_query_partial:
 *   every rank: cqgpu_join_outer_matched(q, tables, n, j, &flags, &nrec) -- this rank's
 *     matched flags over the level's records (one byte each, library memory valid
 *     until the next call), the earlier levels' sets applied; returns 1, or 0 when
 *     level j needs no set (level 0, INNER / LEFT), -1 on error;
 *   the ranks OR the flags (an all-reduce MAX over bytes);
 *   every rank: cqgpu_join_outer_set(j, global_flags, nrec, emit) with emit = 1 on
 *     exactly one rank: that rank's partial carries the unmatched records.
 * The sets stay until cqgpu_join_outer_clear. */
int cqgpu_join_outer_matched(cq_node* query_ast, cqgpu_table* const* tables, int ntables, int level,
                             const uint8_t** flags, uint64_t* nrec);
int cqgpu_join_outer_set(int level, const uint8_t* matched, uint64_t nrec, int emit);
void cqgpu_join_outer_clear(void);
/* Merge the partial blobs of all ranks (any order) into the final result, with
 * HAVING / ORDER BY / DISTINCT / LIMIT applied as evaluate_query would. */
cq_table* cqgpu_merge_partials(cq_node* query_ast, const void* const* blobs, const size_t* sizes,
                               int nblobs);

/* ---- device-side merge of range-partitioned GROUP BY partials --------------
 * ("RCCL reduce for the final aggregate merge").  The
 * library keeps this rank's partial groups on the device and asks the caller
 * for one collective at a time; the sequence depends on the plan only, so every
 * rank asks for the same ones:
 *   p = cqgpu_partial_new(q, tables, 1)          this rank's scan (NULL + cqgpu_last_ineligible:
 *                                                plan outside the dense path -> blobs above)
 *   result = NULL, sizes = NULL
 *   loop:
 *     cqgpu_partial_next(p, result, sizes, rank, world, &c)   takes the last result, returns the next
 *     c.op == CQGPU_COLL_DONE: stop;  CQGPU_COLL_DECLINE: too many keys, take the blob path
 *     buf = device buffer of c.count elements (bytes for ALLGATHER, 8-byte words otherwise)
 *     cqgpu_partial_put(p, buf)                   this rank's payload into buf
 *     run c.op on buf (ALLGATHER: result = the ranks' payloads concatenated in rank
 *     order, sizes = their byte counts; the reduces in place: result = buf)
 *   rank 0: r = cqgpu_partial_result(p, q); every rank: cqgpu_partial_free(p)
 * All buffers are device memory; the library copies what it keeps, so the caller
 * may free `result` once next returns.  Returns 0 / -1 (cqgpu_last_error). */
typedef struct cqgpu_partial cqgpu_partial;
enum {
    CQGPU_COLL_DONE = 0,
    CQGPU_COLL_ALLGATHER = 1,          /* uint8, variable size per rank */
    CQGPU_COLL_ALLREDUCE_MIN_I64 = 2,  /* int64 (signed) */
    CQGPU_COLL_ALLREDUCE_SUM_F64 = 3,  /* double */
    CQGPU_COLL_REDUCE_SUM_I64 = 4,     /* int64, to rank 0 */
    CQGPU_COLL_REDUCE_SUM_F64 = 5,     /* double, to rank 0 */
    CQGPU_COLL_DECLINE = 6
};
typedef struct {
    int32_t op;
    int32_t pad;
    uint64_t count;
} cqgpu_coll;
cqgpu_partial* cqgpu_partial_new(cq_node* query_ast, cqgpu_table* const* tables, int ntables);
int cqgpu_partial_next(cqgpu_partial* p, const void* result, const uint64_t* result_sizes, int rank, int world,
                       cqgpu_coll* next);
int cqgpu_partial_put(cqgpu_partial* p, void* dev_dst);
cq_table* cqgpu_partial_result(cqgpu_partial* p, cq_node* query_ast);
void cqgpu_partial_free(cqgpu_partial* p);

/* ---- the whole N > 1 step inside the library, over RCCL ---
 * One process per GPU.  The launcher creates the communicator once: rank 0 calls
 * cqgpu_comm_unique_id, broadcasts the CQGPU_COMM_ID_BYTES bytes to the other ranks
 * by any means (bench.py / cq_amd.dist: torch.distributed), then every rank calls
 * cqgpu_comm_init on its current HIP device.  Replaces the caller-driven
 * cqgpu_partial_next / put loop (kept above for the CPU choreography tests):
 * every collective runs on the library's own stream, a rank-local failure travels
 * as a status word inside the payloads, and the host synchronises only where a
 * size is data-dependent.
 *
 * cqgpu_dist_query: this rank's range shard (cqgpu_table_open_range) of the FROM
 * table.  Every rank calls it with the same query.  Plans whose items are COUNT /
 * SUM / AVG / group columns / constants over a one-column (or no) GROUP BY take the
 * gather-merge: each rank packs its groups (first-appearance order, no table
 * addresses) and sends them to rank 0, whose device merges them (dictionary of
 * first occurrences = the global first-appearance order, sums in rank order,
 * representative cells of the first occurrence) -- one collective plus the final
 * status broadcast.  Other aggregates run the dense merge above over RCCL
 * (all_gather of keys, MIN / SUM all-reduces, SUM reduces to rank 0); MEDIAN and
 * row-returning SELECTs the partial blobs (one all_gather).  Rank 0 returns the
 * result (evaluate_query's contract), the other ranks NULL.  *status: 0, or -1 on
 * EVERY rank when any rank failed (cqgpu_last_error: this rank's message or "a
 * peer rank failed"). *path (optional): 1 gather-merge, 2 dense, 3 blobs. */
#define CQGPU_COMM_ID_BYTES 128
int cqgpu_comm_unique_id(void* id_out);
int cqgpu_comm_init(const void* id, int rank, int world);
void cqgpu_comm_destroy(void);
/* Test backend of the same step: instead of RCCL, every collective stages its device
 * buffers through host memory and calls fn(user, op, dtype, redop, peer, send, recv,
 * count) -- count elements of dtype (0 u8, 1 u32, 2 u64, 3 i64, 4 f64), redop 0 SUM,
 * 1 MIN, 2 MAX, peer the root / peer rank or -1.  ALLREDUCE / REDUCE / BROADCAST work
 * in place on `send` (== recv); ALLGATHER fills recv with world * count elements;
 * SEND / RECV post a transfer whose host buffer stays valid until GROUP_END, which
 * must complete every posted transfer.  fn returns 0, anything else fails the step.
 * cq_amd.dist.init_host_comm binds it to torch.distributed gloo, so the library's
 * own N > 1 protocol (cqgpu_dist_query / cqgpu_dist_join) runs at world size 2 and 3
 * with the ranks sharing one GPU.  Not for production: RCCL is the product path. */
enum { CQGPU_HC_ALLREDUCE = 1, CQGPU_HC_ALLGATHER = 2, CQGPU_HC_REDUCE = 3, CQGPU_HC_BROADCAST = 4,
       CQGPU_HC_SEND = 5, CQGPU_HC_RECV = 6, CQGPU_HC_GROUP_END = 7 };
typedef int (*cqgpu_coll_fn)(void* user, int op, int dtype, int redop, int peer, const void* send, void* recv,
                             uint64_t count);
int cqgpu_comm_init_host(int rank, int world, cqgpu_coll_fn fn, void* user);
cq_table* cqgpu_dist_query(cq_node* query_ast, cqgpu_table* shard, int* status, int* path);
/* cqgpu_dist_join: the repartitioned JOIN step (perform_join / process_joins,
 * evaluator_joins.c:63-181, 237-274, over inputs spread across the ranks) inside the
 * library.  tables = [this rank's shard of the FROM table, this rank's shard of the
 * first JOIN's table, a chain's later tables whole].  Both sides are routed by the
 * first ON key (cqgpu_route_plan's rule: whole number keys by key mod N), the
 * records and their global ids exchanged in one grouped ncclSend / ncclRecv per
 * side, rebuilt as this rank's sides (key stride N: a dense build key range stays
 * on the STAR join), joined locally, and the join partials merged on rank 0
 * (cqgpu_merge_partials' nested-loop order).  Rank 0 returns the result; *status:
 * 0, or -1 on EVERY rank when any rank failed (refusals included). */
cq_table* cqgpu_dist_join(cq_node* query_ast, cqgpu_table* const* tables, int ntables, int* status);
/* ---- the typed exchange of the repartitioned JOIN (SURVEY.md section 8e's
 * (key, row id, payload) entries; cqgpu_dist_join takes it whenever the plan and the
 * data allow, falling back to the CSV-record exchange below together on every rank).
 * Plan: one INNER JOIN `l.k = r.k` without WHERE, COUNT / SUM / AVG of one right
 * column, GROUP BY one left column (its value the only other item) or none.  Every
 * record of the FROM table (side 0, the build side) becomes a 16-byte entry
 * {key / N - qbase, global record id, GROUP BY bytes}, every record of the JOIN table
 * (side 1) an 8-byte entry {key / N - qbase, SUM argument in 10^-3 units or
 * 0x80000000 for NULL}, in the region of rank key mod N (perform_join's keys as
 * canonical INTEGERs, evaluator_joins.c:40-60; a NULL probe key and a probe key
 * outside the build keys' window match nothing and are not sent).  The receiver
 * joins the entries with the STAR join (one residue class of a dense key range) and
 * writes the same "CQJ1" partial cqgpu_query_partial would.
 *   cqgpu_typed_plan     1 when the plan takes the typed exchange (0: *_ineligible says why)
 *   cqgpu_typed_sample_kmin  the build side's sampled key minimum (first qbase = min / N)
 *   cqgpu_typed_count    the count pass over side `side` (kept by the table): counts[N]
 *                        the entries per destination, krange the build side's keys'
 *                        min and max, flags 1 not typable (quote, key shape), 8 a NULL
 *                        build key, 16 a build key / N - qbase outside 32 bits (retry
 *                        with qbase = kmin / N); returns the side's records (build; the
 *                        caller sums the lower ranks' into gid_base) or entries (probe)
 *   cqgpu_typed_send     the emit pass after the count: the entries, destination d's
 *                        contiguous (no atomics, no holes); flags 1 (a GROUP BY value or
 *                        numeral the entries cannot carry), 512 (a payload over 31 bits)
 *   cqgpu_typed_region   region `dest` of a table's entries (device pointer)
 *   cqgpu_typed_reset    drop a table's counts and entries
 *   cqgpu_typed_gather   regions `dest` of several tables, concatenated into dev_out (one
 *                        GPU standing in for the exchange: tests and the benchmark)
 *   cqgpu_typed_partial  the receiving rank's STAR join over its entries: slot = q32 - qoff,
 *                        range slots (qoff = kmin / N - qbase, range = kmax / N - kmin / N + 1
 *                        over the global build keys); the blob as cqgpu_query_partial's,
 *                        0 + *_ineligible when the entries do not fit the STAR join */
int cqgpu_typed_plan(cq_node* query_ast, cqgpu_table* const* tables, int ntables);
uint64_t cqgpu_typed_sample_kmin(cq_node* query_ast, cqgpu_table* const* tables, int ntables);
int64_t cqgpu_typed_count(cq_node* query_ast, cqgpu_table* const* tables, int ntables, int side, int nranks,
                          uint64_t qbase, uint64_t* counts, uint64_t* krange, uint32_t* flags);
int cqgpu_typed_send(cq_node* query_ast, cqgpu_table* const* tables, int ntables, int side, uint64_t gid_base,
                     uint32_t* flags);
const void* cqgpu_typed_region(const cqgpu_table* t, int dest, uint64_t* entries, uint64_t* entry_bytes);
void cqgpu_typed_reset(cqgpu_table* t);
int64_t cqgpu_typed_gather(cqgpu_table* const* senders, int nsenders, int dest, void* dev_out, uint64_t cap_entries);
size_t cqgpu_typed_partial(cq_node* query_ast, cqgpu_table* const* tables, int ntables, const void* dev_build,
                           uint64_t nbuild, const void* dev_probe, uint64_t nprobe, uint64_t qoff, uint64_t range,
                           void** blob_out);

/* test entry: the gather-merge of `n` shards held by this one process (simulated
 * ranks, no RCCL): every shard's pack, then rank 0's merge kernels; NULL +
 * cqgpu_last_ineligible when the plan or the data leaves the gather-merge */
cq_table* cqgpu_gm_local(cq_node* query_ast, cqgpu_table* const* shards, int n);

/* ---- join-key repartition for the multi-GPU JOIN ---
 * One INNER / LEFT / RIGHT / FULL JOIN with an `ident = ident` ON (reference
 * evaluator_joins.c:40-60, :63-181) over range-partitioned inputs: every rank routes each record of its
 * shard of side `side` (0 = FROM table, 1 = JOIN table) to rank
 * hash(key value class, key code) mod nranks, exchanges the records with an
 * all-to-all (RCCL over xGMI), rebuilds each side from what it received
 * (concatenated in source-rank order) and runs cqgpu_query_partial on the pair;
 * cqgpu_merge_partials gives the whole-input result -- groups in first-appearance
 * order of the (l, r) nested loop, as perform_join + create_groups would.
 * Keys of several value classes (which value_compare calls "equal" across classes)
 * and a JOIN without ON take cqgpu_route_plan2's replicated routing below; with plain
 * cqgpu_route_plan such inputs are refused by the merge.
 *
 * route_plan: computes the routing of tables[side] (tables = {FROM shard, JOIN
 * shard}, needed to bind the ON operands) and writes per destination rank the
 * byte count and record count of the send buffer.  Returns 0, or -1 with
 * cqgpu_last_error() / cqgpu_last_ineligible() set. */
int cqgpu_route_plan(cq_node* query_ast, cqgpu_table* const* tables, int ntables, int side, int nranks,
                     uint64_t* bytes_per_rank, uint64_t* recs_per_rank);
/* route_plan2: route_plan for the caller's `rank` with a routing mode, which lifts
 * two refusals of route_plan:
 *  - keys of different value classes (value_compare calls any two non-NULL keys of
 *    different classes equal, csv_reader.c:126-129, used by the join at
 *    evaluator_joins.c:53-55): mode = cqgpu_route_major(every rank's class counts of
 *    both sides); keys of class `mode` and NULL keys route by key as before, every
 *    other record goes to EVERY rank (in each destination's region, file order kept);
 *  - a JOIN without ON (every pair matches, evaluator_joins.c:41): side 0's records
 *    stay on `rank`, side 1's go to every rank (mode ignored).
 * class_counts (optional, 4 entries): this side's ON keys per value class (NULL,
 * number, string, date) -- mode 0's plan returns them for the agreement.  The
 * receiver marks both rebuilt sides with cqgpu_table_set_replicated.  N <= 64.
 * Returns this side's record count on this rank (the span of its global ids: a
 * replicated record counts once, though it is in every destination's count), or -1. */
int64_t cqgpu_route_plan2(cq_node* query_ast, cqgpu_table* const* tables, int ntables, int side, int nranks,
                          int rank, uint32_t mode, uint64_t* bytes_per_rank, uint64_t* recs_per_rank,
                          uint64_t* class_counts);
/* the routing mode for every rank's summed class counts of the two sides: 0 when no
 * pair of keys of different non-NULL classes can occur, else the class (1-3) most
 * keys hold (it routes by key; the others are replicated) */
uint32_t cqgpu_route_major(const uint64_t* left_class_counts, const uint64_t* right_class_counts);
/* a routed side's replication, for cqgpu_query_partial: mode 0 none, 1-3 the
 * route_plan2 mode (a pair of two replicated records is found on every rank and kept
 * only where owner != 0; outer joins are refused in this mode), 4 every record of
 * this side is on every rank (a JOIN without ON's side 1; owner != 0: this rank
 * emits a RIGHT / FULL join's unmatched rows).  Exactly one rank passes owner = 1. */
int cqgpu_table_set_replicated(cqgpu_table* t, uint32_t mode, int owner);
/* route_fill: writes the planned send buffer into device memory: records grouped
 * by destination rank (file order within a rank, each '\n'-terminated) into
 * dev_bytes, and their global record ids (gid_base + local record index) into
 * dev_gids.  gid_base = records of this side on lower ranks.  Each record carries
 * only the fields the plan reads from this side (ON keys, WHERE, SELECT, GROUP BY,
 * aggregates, HAVING / ORDER BY, a chain's later levels): every other field is
 * empty with its delimiter kept, the record ends after its last needed field, and a
 * record whose needed fields are all empty is a lone delimiter (environment
 * CQGPU_NO_ROUTE_PROJECT=1: whole records). */
int cqgpu_route_fill(cqgpu_table* t, uint64_t gid_base, void* dev_bytes, uint64_t* dev_gids);
/* table over received records (device memory, copied) with their global ids and
 * the side's header record */
cqgpu_table* cqgpu_table_from_routed(const void* dev_bytes, size_t n, const uint64_t* dev_gids, size_t nrec,
                                     cq_csv_config cfg, const char* header, size_t header_len);
/* the record count of the whole input a routed table came from (the sum of every
 * rank's route_plan records): a chain of JOINs across partials orders its rows by
 * mixed-radix keys over it (route.hip chain_key_kernel).  -1 if below the table's
 * own record count.  A chain's later tables are passed whole to query_partial. */
int cqgpu_table_set_record_total(cqgpu_table* t, uint64_t total);
/* A routed table's key stride: cqgpu_route_plan sends whole-number keys to rank
 * (key mod N), so each rank holds one residue class of them; with stride N the
 * STAR join indexes a dense key range by (key - kmin) / N instead of declining it
 * as sparse (the reference's perform_join, evaluator_joins.c:63-181, is unaffected:
 * the stride only sizes the key-indexed arrays).  -1 for stride 0. */
int cqgpu_table_set_key_stride(cqgpu_table* t, uint32_t stride);

/* ---- output ----------------------------------------------------------------
 * replaces write_csv_file (reference utils.c:220-289, called by main.c:133 for
 * `-o FILE`): the same bytes for any result table -- header by the host, every
 * row formatted on the GPU (%lld, %.2f, %04d-%02d-%02d, strings quoted when they
 * hold the delimiter, a quote or a line break).  Returns 0, or -1 with a message
 * on stderr. */
int cqgpu_write_csv(const char* filename, const cq_table* result, char delimiter);

/* ---- introspection -------------------------------------------------------- */
typedef struct {
    double scan_ms;              /* device time of the last fused scan kernel (HIP events) */
    double total_ms;             /* wall time of the last query inside the library */
    uint64_t scan_bytes;         /* table bytes the scan covered */
    uint64_t records;            /* data records scanned */
    uint64_t groups;             /* result groups before HAVING/LIMIT */
    uint64_t lds_spills;         /* records aggregated directly in HBM (LDS table full) */
    int grid;                    /* scan blocks launched */
    int path;                    /* 1 = GPU executor, 2 = fallback evaluator */
    int retries;                 /* global group table regrowths */
    uint64_t slow_records;       /* records the fast field path handed to the general parser */
    uint64_t passed;             /* records that passed WHERE */
    int scan_kernel;             /* 2 = fast_kernel, 1 = lean_kernel (both wave-autonomous), 0 = general scan_kernel */
    int wide;                    /* 1 = a plan over more than 8 distinct columns (cells path, scan.hip PairView) */
} cqgpu_stats;
int cqgpu_last_stats(cqgpu_stats* out);
const char* cqgpu_last_error(void);
/* why the last plan was not GPU-eligible ("" when it was) */
const char* cqgpu_last_ineligible(void);

/* Tokenizer / typing checks: record start offsets of all data records (file
 * order; returns the total count, writes at most `cap`), and the typed cells
 * of columns `cols` at given records (a result table, freed like any other). */
size_t cqgpu_debug_records(cqgpu_table* t, unsigned long long* out, size_t cap);
cq_table* cqgpu_debug_cells(cqgpu_table* t, const int* cols, int ncols,
                            const unsigned long long* recs, size_t nrec);
/* every data record's start offset in file order, as the join and the key
 * routing see them: method 0 = the two-pass record-start kernels (route.hip),
 * 1 = through the general scan path; returns the count ((size_t)-1 on error) */
size_t cqgpu_debug_all_records(cqgpu_table* t, int method, unsigned long long* out, size_t cap);
/* the fused scan kernel's own parse of ascending columns `cols` for every
 * record (rows in arbitrary order, their record offsets in recs_out) */
cq_table* cqgpu_debug_scan_cells(cqgpu_table* t, const int* cols, int ncols,
                                 unsigned long long* recs_out, size_t cap);
/* Planner check without a device: compile `query_ast` against a header line and
 * describe the plan (or why it is not GPU-eligible) into `out`. */
int cqgpu_explain(cq_node* query_ast, const char* header, cq_csv_config cfg, char* out, size_t cap);
/* profiling builds (-DCQ_CLOCKS): shader cycles per scan phase of the last scan,
 * summed over waves (all zero in the normal build) */
int cqgpu_debug_clocks(unsigned long long* out8);

/* Scan kernel choice: 0 = automatic (fast_kernel, else lean_kernel, else the
 * general scan_kernel, by the plan shapes each covers), 1 = always scan_kernel,
 * 2 = never fast_kernel.  Returns the previous mode.  All produce identical
 * results; the knob exists for A/B measurements and parity tests of every kernel. */
int cqgpu_set_scan_kernel(int mode);

/* Optional fallback for plans outside the GPU subset: the reference evaluator
 * compiled with evaluate_query renamed.  Without one, such
 * plans return NULL with a message. */
typedef cq_table* (*cqgpu_fallback_fn)(cq_node*);
void cqgpu_set_fallback(cqgpu_fallback_fn fn);

#ifdef __cplusplus
}
#endif
#endif /* CQGPU_H */
