/*
 * cq_abi.h -- binary-layout contract with the reference cq front end.
 *
 * libcqgpu replaces the reference evaluator behind `evaluate_query`
 * (reference include/evaluator.h:32).  Its input is the plan the UNCHANGED
 * reference parser builds (reference include/parser.h:55-201) and its output is
 * the reference's result table (reference include/csv_reader.h:8-70, typedef
 * ResultSet evaluator.h:26), which the unchanged CLI prints and frees with
 * csv_free (csv_reader.c:467).  This header restates ONLY the memory layout of
 * those types (x86-64 LP64), under our own names, so that our C++ executor can
 * read the plan and build the result without including reference sources.
 *
 * The layout is pinned by tests/golden/abi_layout.json, produced by
 * oracle/ref_probe.c compiled against the reference headers, and checked by
 * tests/test_abi.py (sizeof/offsetof of every field we touch).
 */
#ifndef CQ_ABI_H
#define CQ_ABI_H

#include <stddef.h>
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- plan node kinds: order matches reference parser.h:11-36 ---------------- */
enum cq_node_kind {
    CQ_N_QUERY = 0, CQ_N_SELECT, CQ_N_FROM, CQ_N_JOIN, CQ_N_WHERE, CQ_N_GROUP_BY,
    CQ_N_ORDER_BY, CQ_N_FUNCTION, CQ_N_CONDITION, CQ_N_LITERAL, CQ_N_IDENTIFIER,
    CQ_N_ALIAS, CQ_N_LIST, CQ_N_SUBQUERY, CQ_N_BINARY_OP, CQ_N_SET_OP, CQ_N_INSERT,
    CQ_N_UPDATE, CQ_N_DELETE, CQ_N_ASSIGNMENT, CQ_N_CREATE_TABLE, CQ_N_ALTER_TABLE,
    CQ_N_CASE, CQ_N_WINDOW_FUNCTION
};

/* join kinds: parser.h:38-43 */
enum cq_join_kind { CQ_JOIN_INNER = 0, CQ_JOIN_LEFT, CQ_JOIN_RIGHT, CQ_JOIN_FULL };

typedef struct cq_node cq_node;

/* One plan node (reference `ASTNode`, 80 bytes).  Only the variants the SELECT
 * executor reads are spelled out; the rest of the union is opaque padding. */
struct cq_node {
    int refcount;
    int kind;                                  /* enum cq_node_kind */
    union {
        struct {                               /* CQ_N_QUERY */
            cq_node* select;
            cq_node* from;
            cq_node** joins;
            int join_count;
            cq_node* where;
            cq_node* group_by;
            cq_node* having;
            cq_node* order_by;
            int limit;                         /* -1 = none */
            int offset;                        /* -1 = none */
        } q;
        struct {                               /* CQ_N_SELECT */
            char** texts;                      /* column strings, " AS alias" appended */
            cq_node** exprs;                   /* may be NULL entries ('*') */
            int count;
            bool distinct;
        } sel;
        struct {                               /* CQ_N_CONDITION and CQ_N_BINARY_OP */
            cq_node* lhs;
            cq_node* rhs;
            char* op;
        } bin;
        struct {                               /* CQ_N_FUNCTION */
            char* name;
            cq_node** args;
            int nargs;
        } fn;
        struct {                               /* CQ_N_LIST */
            cq_node** items;
            int nitems;
        } list;
        struct {                               /* CQ_N_ORDER_BY */
            char* key;
            bool desc;
        } ord;
        struct {                               /* CQ_N_GROUP_BY */
            char** keys;
            int nkeys;
        } grp;
        struct {                               /* CQ_N_FROM */
            char* path;
            cq_node* subquery;
            char* alias;
        } from;
        struct {                               /* CQ_N_JOIN */
            int kind;                          /* enum cq_join_kind */
            char* path;
            char* alias;
            cq_node* on;
        } join;
        struct {                               /* CQ_N_SUBQUERY */
            cq_node* query;
        } sub;
        char* text;                            /* CQ_N_LITERAL / CQ_N_IDENTIFIER */
        unsigned char _opaque[72];
    } u;
};

/* ---- cell values: csv_reader.h:8-32 ---------------------------------------- */
enum cq_value_kind { CQ_V_NULL = 0, CQ_V_INT, CQ_V_DOUBLE, CQ_V_STRING, CQ_V_DATE };

typedef struct { int y, m, d; } cq_date;

typedef struct {
    int kind;                                  /* enum cq_value_kind */
    union {
        long long i;
        double f;
        char* s;                               /* malloc'd, NUL-terminated */
        cq_date date;
    } u;
} cq_value;                                    /* 24 bytes */

typedef struct { cq_value* values; int ncols; } cq_row;           /* 16 bytes */
typedef struct { char* name; int inferred_kind; } cq_column;     /* 16 bytes */

/* the reference's `CsvTable` == `ResultSet` (72 bytes) */
typedef struct {
    char* filename;
    char* data;                                /* mmap base; NULL for results */
    size_t file_size;
    int fd;                                    /* -1 for results */
    cq_column* columns;
    int ncols;
    bool has_header;
    cq_row* rows;
    int nrows;
    int row_capacity;
    char delimiter;
    char quote;
} cq_table;

/* the reference's `CsvConfig` (csv_reader.h:66-70) */
typedef struct { char delimiter; char quote; bool has_header; } cq_csv_config;

#ifdef __cplusplus
}
#endif
#endif /* CQ_ABI_H */
