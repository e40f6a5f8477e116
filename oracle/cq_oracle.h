/*
 * oracle/cq_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference cq SELECT path, used as the parity checker
 * for the HIP executor (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 * Never linked into, loaded by, or called from the product (cq_amd/).
 *
 * Pinned against the reference: the tests/golden JSON vectors were produced by running
 * the unmodified reference (oracle/ref.mk + oracle/ref_probe.c) and
 * tests/test_oracle_golden.py checks this restatement against every vector.
 */
#ifndef CQ_ORACLE_H
#define CQ_ORACLE_H
#include "../include/cq_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* parse_date (reference date_utils.c:88-100 / :26-86 / :19-24) */
int orc_parse_date(const char* s, cq_date* out);
/* parse_value + infer_type (reference csv_reader.c:133-240) */
cq_value orc_parse_cell(const char* s, size_t len);
/* value_compare (reference csv_reader.c:98-130) */
int orc_compare(const cq_value* a, const cq_value* b);
/* csv_load (reference csv_reader.c:278-465) over an in-memory byte buffer */
cq_table* orc_load(const char* bytes, size_t n, cq_csv_config cfg);
cq_table* orc_load_file(const char* path, cq_csv_config cfg);
/* evaluate_query SELECT subset (reference evaluator.c:26-287); NULL + stderr on error.
 * *unsupported is set to 1 when the plan uses a feature the restatement lacks. */
cq_table* orc_evaluate(cq_node* query, cq_csv_config cfg, int* unsupported);
void orc_free(cq_table* t);

#ifdef __cplusplus
}
#endif
#endif
