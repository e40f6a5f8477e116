/*
 * oracle/ref_probe.c -- TEST INFRASTRUCTURE ONLY (golden-vector generator).
 *
 * A dump driver of our own, compiled against the reference headers where they
 * lie (/root/reference/include) and linked with oracle/_ref/libcqref.so, the
 * unmodified reference built by oracle/ref.mk.  It prints what the reference
 * computes, as JSON, so tests/golden/ can pin our CPU restatement (oracle/) and
 * our HIP executor (cq_amd/) to the reference's own behaviour.
 *
 *   ref_probe layout                      sizeof/offsetof of the ABI types
 *   ref_probe cells FILE [DELIM] [HDR]    csv_load (csv_reader.c:375) typed cells
 *   ref_probe query SQL [DELIM]           parse + evaluate_query (evaluator.c:290)
 *   ref_probe time SQL [DELIM]            wall time of parse + evaluate_query
 *
 * Value encoding: {"t":"N"} | {"t":"I","v":<int>} | {"t":"D","v":"%.17g"} |
 * {"t":"S","v":"latin-1 escaped"} | {"t":"T","v":[y,m,d]}.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stddef.h>
#include <time.h>
#include "parser.h"
#include "evaluator.h"
#include "csv_reader.h"

static void put_str(const char* s) {
    putchar('"');
    for (const unsigned char* p = (const unsigned char*)s; p && *p; p++) {
        if (*p == '"' || *p == '\\') printf("\\%c", *p);
        else if (*p < 0x20 || *p >= 0x7f) printf("\\u%04x", *p);
        else putchar(*p);
    }
    putchar('"');
}

static void put_value(const Value* v) {
    switch (v->type) {
        case VALUE_TYPE_NULL: printf("{\"t\":\"N\"}"); break;
        case VALUE_TYPE_INTEGER: printf("{\"t\":\"I\",\"v\":%lld}", v->int_value); break;
        case VALUE_TYPE_DOUBLE: printf("{\"t\":\"D\",\"v\":\"%.17g\"}", v->double_value); break;
        case VALUE_TYPE_STRING: printf("{\"t\":\"S\",\"v\":"); put_str(v->string_value); putchar('}'); break;
        case VALUE_TYPE_DATE:
            printf("{\"t\":\"T\",\"v\":[%d,%d,%d]}", v->date_value.year, v->date_value.month, v->date_value.day);
            break;
        default: printf("{\"t\":\"?\"}");
    }
}

static void put_table(const CsvTable* t) {
    printf("{\"columns\":[");
    for (int i = 0; i < t->column_count; i++) {
        if (i) putchar(',');
        put_str(t->columns[i].name);
    }
    printf("],\"rows\":[");
    for (int r = 0; r < t->row_count; r++) {
        if (r) putchar(',');
        putchar('[');
        for (int c = 0; c < t->rows[r].column_count; c++) {
            if (c) putchar(',');
            put_value(&t->rows[r].values[c]);
        }
        putchar(']');
    }
    printf("]}\n");
}

#define OFF(T, f) printf("\"%s.%s\":%zu,", #T, #f, offsetof(T, f))
static int cmd_layout(void) {
    printf("{");
    printf("\"sizeof.ASTNode\":%zu,\"sizeof.Value\":%zu,\"sizeof.Row\":%zu,\"sizeof.Column\":%zu,"
           "\"sizeof.CsvTable\":%zu,\"sizeof.CsvConfig\":%zu,\"sizeof.DateValue\":%zu,",
           sizeof(ASTNode), sizeof(Value), sizeof(Row), sizeof(Column), sizeof(CsvTable),
           sizeof(CsvConfig), sizeof(DateValue));
    OFF(ASTNode, refcount); OFF(ASTNode, type);
    OFF(ASTNode, query.select); OFF(ASTNode, query.from); OFF(ASTNode, query.joins);
    OFF(ASTNode, query.join_count); OFF(ASTNode, query.where); OFF(ASTNode, query.group_by);
    OFF(ASTNode, query.having); OFF(ASTNode, query.order_by); OFF(ASTNode, query.limit);
    OFF(ASTNode, query.offset);
    OFF(ASTNode, select.columns); OFF(ASTNode, select.column_nodes);
    OFF(ASTNode, select.column_count); OFF(ASTNode, select.distinct);
    OFF(ASTNode, condition.left); OFF(ASTNode, condition.right); OFF(ASTNode, condition.operator);
    OFF(ASTNode, function.name); OFF(ASTNode, function.args); OFF(ASTNode, function.arg_count);
    OFF(ASTNode, list.nodes); OFF(ASTNode, list.node_count);
    OFF(ASTNode, order_by.column); OFF(ASTNode, order_by.descending);
    OFF(ASTNode, group_by.columns); OFF(ASTNode, group_by.column_count);
    OFF(ASTNode, from.table); OFF(ASTNode, from.subquery); OFF(ASTNode, from.alias);
    OFF(ASTNode, join.join_type); OFF(ASTNode, join.table); OFF(ASTNode, join.alias);
    OFF(ASTNode, join.condition);
    OFF(ASTNode, subquery.query);
    OFF(ASTNode, binary_op.left); OFF(ASTNode, binary_op.right); OFF(ASTNode, binary_op.operator);
    OFF(ASTNode, set_op.op_type); OFF(ASTNode, literal); OFF(ASTNode, identifier);
    OFF(Value, type); OFF(Value, int_value); OFF(Value, double_value); OFF(Value, string_value);
    OFF(Value, date_value);
    OFF(Row, values); OFF(Row, column_count);
    OFF(Column, name); OFF(Column, inferred_type);
    OFF(CsvTable, filename); OFF(CsvTable, data); OFF(CsvTable, file_size); OFF(CsvTable, fd);
    OFF(CsvTable, columns); OFF(CsvTable, column_count); OFF(CsvTable, has_header);
    OFF(CsvTable, rows); OFF(CsvTable, row_count); OFF(CsvTable, row_capacity);
    OFF(CsvTable, delimiter); OFF(CsvTable, quote);
    OFF(CsvConfig, delimiter); OFF(CsvConfig, quote); OFF(CsvConfig, has_header);
    printf("\"enum.NODE_TYPE_QUERY\":%d,\"enum.NODE_TYPE_CONDITION\":%d,\"enum.NODE_TYPE_BINARY_OP\":%d,"
           "\"enum.NODE_TYPE_WINDOW_FUNCTION\":%d,\"enum.VALUE_TYPE_DATE\":%d}\n",
           NODE_TYPE_QUERY, NODE_TYPE_CONDITION, NODE_TYPE_BINARY_OP, NODE_TYPE_WINDOW_FUNCTION,
           VALUE_TYPE_DATE);
    return 0;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: ref_probe layout|cells|query|time ...\n"); return 2; }
    const char* cmd = argv[1];
    if (!strcmp(cmd, "layout")) return cmd_layout();
    if (!strcmp(cmd, "cells") && argc >= 3) {
        CsvConfig cfg = csv_config_default();
        if (argc >= 4) cfg.delimiter = argv[3][0];
        if (argc >= 5) cfg.has_header = atoi(argv[4]) != 0;
        CsvTable* t = csv_load(argv[2], cfg);
        if (!t) { printf("{\"error\":true}\n"); return 0; }
        put_table(t);
        csv_free(t);
        return 0;
    }
    if ((!strcmp(cmd, "query") || !strcmp(cmd, "time")) && argc >= 3) {
        if (argc >= 4) global_csv_config.delimiter = argv[3][0];
        double t0 = now_s();
        ASTNode* ast = parse(argv[2]);
        if (!ast) { printf("{\"error\":true,\"stage\":\"parse\"}\n"); return 0; }
        ResultSet* r = evaluate_query(ast);
        double t1 = now_s();
        if (!r) { printf("{\"error\":true,\"stage\":\"evaluate\"}\n"); releaseNode(ast); return 0; }
        if (!strcmp(cmd, "time")) {
            printf("{\"seconds\":%.6f,\"result_rows\":%d}\n", t1 - t0, r->row_count);
        } else {
            put_table(r);
        }
        /* the reference result has fd=0 (calloc); csv_free would close stdin: mask it */
        r->fd = -1;
        csv_free(r);
        releaseNode(ast);
        return 0;
    }
    fprintf(stderr, "bad command\n");
    return 2;
}
