/*
 * oracle/cq_oracle.c -- TEST INFRASTRUCTURE ONLY: the parity checker.
 *
 * A plain-C restatement of the reference cq SELECT path (krow89/cq snapshot at
 * /root/reference), written from its behaviour, not copied.  Each function cites
 * the reference file:line it follows.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load this (as liboracle.so); the product never does.
 *
 * Arithmetic deliberately uses the same libc primitives the reference uses
 * (sscanf for dates, strtoll/strtod for numbers, snprintf for group keys), so
 * the restatement is bit-exact by construction; it is pinned against the
 * reference's own outputs by tests/golden/ (see tests/test_oracle_golden.py).
 *
 * Scope: FROM file [alias], JOIN (INNER/LEFT/RIGHT/FULL, nested loop), WHERE
 * (NOT/AND/OR, = != <> < > <= >=, IN/NOT IN list, LIKE/ILIKE, arithmetic),
 * GROUP BY (single, composite, SELECT-alias), COUNT/SUM/AVG/MIN/MAX/STDDEV/
 * MEDIAN, projection, HAVING, ORDER BY, DISTINCT, LIMIT/OFFSET.  Subqueries,
 * CASE, scalar and window functions set *unsupported.
 */
#define _GNU_SOURCE
#include "cq_oracle.h"
#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

static char* xstrndup(const char* s, size_t n) {
    char* r = malloc(n + 1);
    memcpy(r, s, n);
    r[n] = 0;
    return r;
}

/* ------------------------------------------------------------------ dates */
/* is_valid_date / days_in_month: date_utils.c:8-24 */
static int leap(int y) { return (y % 4 == 0 && y % 100 != 0) || (y % 400 == 0); }
static int valid_ymd(int y, int m, int d) {
    static const int dm[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    if (y < 1000 || y > 9999 || m < 1 || m > 12 || d < 1) return 0;
    int lim = (m == 2 && leap(y)) ? 29 : dm[m - 1];
    return d <= lim;
}

/* parse_date: ISO, US, EU, COMPACT in that order (date_utils.c:88-100, :26-86) */
int orc_parse_date(const char* s, cq_date* out) {
    int y = 0, m = 0, d = 0;
    if (sscanf(s, "%d-%d-%d", &y, &m, &d) == 3 && valid_ymd(y, m, d)) goto ok;
    y = m = d = 0;
    if (sscanf(s, "%d/%d/%d", &m, &d, &y) == 3 && valid_ymd(y, m, d)) goto ok;
    y = m = d = 0;
    if (sscanf(s, "%d/%d/%d", &d, &m, &y) == 3 && valid_ymd(y, m, d)) goto ok;
    y = 0;
    if (sscanf(s, "%8d", &y) == 1) {
        d = y % 100; y /= 100; m = y % 100; y /= 100;
        if (valid_ymd(y, m, d)) goto ok;
    }
    return 0;
ok:
    out->y = y; out->m = m; out->d = d;
    return 1;
}

/* ------------------------------------------------------------------ cells */
/* copy [s, s+len) trimmed of isspace on both ends into buf (csv_reader.c:143-149) */
static void trimmed_copy(const char* s, size_t len, char* buf) {
    memcpy(buf, s, len);
    buf[len] = 0;
    char* t = buf;
    while (*t && isspace((unsigned char)*t)) t++;
    size_t tl = strlen(t);
    while (tl > 0 && isspace((unsigned char)t[tl - 1])) t[--tl] = 0;
    memmove(buf, t, tl + 1);
}

/* parse_value + infer_type (csv_reader.c:133-240) */
cq_value orc_parse_cell(const char* s, size_t len) {
    cq_value v;
    memset(&v, 0, sizeof v);
    v.kind = CQ_V_NULL;
    if (len == 0) return v;
    if (len >= 8 && len <= 10) {                     /* :137-156 */
        char buf[32];
        trimmed_copy(s, len, buf);
        cq_date dt;
        if (orc_parse_date(buf, &dt)) { v.kind = CQ_V_DATE; v.u.date = dt; return v; }
    }
    size_t i = 0;                                    /* :159-192 */
    int has_dot = 0, has_digit = 0, is_num = 1;
    while (i < len && isspace((unsigned char)s[i])) i++;
    if (i < len && (s[i] == '+' || s[i] == '-')) i++;
    if (i < len) {
        while (i < len && !isspace((unsigned char)s[i])) {
            if (isdigit((unsigned char)s[i])) has_digit = 1;
            else if (s[i] == '.' && !has_dot) has_dot = 1;
            else { is_num = 0; break; }
            i++;
        }
        while (i < len && isspace((unsigned char)s[i])) i++;
        if (is_num && has_digit && i == len) {
            /* like the reference (csv_reader.c:207-210) strtoll/strtod run on the raw
             * buffer, not on a len-bounded copy: they stop at the delimiter, quote or
             * line end that follows the field -- or, for an unclosed quoted field whose
             * len counts only its "" pairs (:299-314), further inside the record.
             * orc_load keeps the buffer NUL-terminated so this never runs off the end. */
            if (has_dot) { v.kind = CQ_V_DOUBLE; v.u.f = strtod(s, NULL); }
            else { v.kind = CQ_V_INT; v.u.i = strtoll(s, NULL, 10); }
            return v;
        }
    }
    v.kind = CQ_V_STRING;                            /* :233-235 */
    char* str = xstrndup(s, len);
    char* t = str;
    while (*t && isspace((unsigned char)*t)) t++;
    size_t tl = strlen(t);
    while (tl > 0 && isspace((unsigned char)t[tl - 1])) t[--tl] = 0;
    memmove(str, t, tl + 1);
    v.u.s = str;
    return v;
}

static void vfree(cq_value* v) {
    if (v->kind == CQ_V_STRING) { free(v->u.s); v->u.s = NULL; }
}
static cq_value vcopy(const cq_value* v) {
    cq_value r = *v;
    if (v->kind == CQ_V_STRING) r.u.s = v->u.s ? strdup(v->u.s) : NULL;
    return r;
}

/* value_compare (csv_reader.c:98-130) */
int orc_compare(const cq_value* a, const cq_value* b) {
    if (a->kind == CQ_V_NULL && b->kind == CQ_V_NULL) return 0;
    if (a->kind == CQ_V_NULL) return -1;
    if (b->kind == CQ_V_NULL) return 1;
    if (a->kind == CQ_V_DATE && b->kind == CQ_V_DATE) {     /* compare_dates date_utils.c:195 */
        if (a->u.date.y != b->u.date.y) return a->u.date.y - b->u.date.y;
        if (a->u.date.m != b->u.date.m) return a->u.date.m - b->u.date.m;
        return a->u.date.d - b->u.date.d;
    }
    int an = a->kind == CQ_V_INT || a->kind == CQ_V_DOUBLE;
    int bn = b->kind == CQ_V_INT || b->kind == CQ_V_DOUBLE;
    if (an && bn) {
        double x = a->kind == CQ_V_INT ? (double)a->u.i : a->u.f;
        double y = b->kind == CQ_V_INT ? (double)b->u.i : b->u.f;
        return x < y ? -1 : (x > y ? 1 : 0);
    }
    if (a->kind == CQ_V_STRING && b->kind == CQ_V_STRING) return strcmp(a->u.s, b->u.s);
    return 0;
}

/* ------------------------------------------------------------------ tables */
static cq_table* table_new(const char* name) {
    cq_table* t = calloc(1, sizeof *t);
    t->filename = strdup(name);
    t->fd = -1;
    t->has_header = true;
    t->delimiter = ',';
    t->quote = '"';
    return t;
}

static void table_add_row(cq_table* t, cq_row r) {
    if (t->nrows >= t->row_capacity) {
        t->row_capacity = t->row_capacity ? t->row_capacity * 2 : 64;
        t->rows = realloc(t->rows, sizeof(cq_row) * (size_t)t->row_capacity);
    }
    t->rows[t->nrows++] = r;
}

void orc_free(cq_table* t) {
    if (!t) return;
    for (int i = 0; i < t->nrows; i++) {
        for (int j = 0; j < t->rows[i].ncols; j++) vfree(&t->rows[i].values[j]);
        free(t->rows[i].values);
    }
    free(t->rows);
    for (int i = 0; i < t->ncols; i++) free(t->columns[i].name);
    free(t->columns);
    free(t->filename);
    free(t);
}

/* parse_line (csv_reader.c:278-373): quote-aware field split inside one record */
static void split_record(cq_table* t, const char* p, const char* end, int header, char quote,
                         char delim) {
    size_t cap = 16, nf = 0;
    const char** fs = malloc(cap * sizeof *fs);
    size_t* fl = malloc(cap * sizeof *fl);
    while (p < end) {
        while (p < end && isspace((unsigned char)*p) && *p != '\n' && *p != '\r') p++;
        if (p >= end) break;                       /* trailing empty field dropped */
        const char* fstart = p;
        size_t flen = 0;
        if (*p == quote) {
            p++;
            fstart = p;
            while (p < end) {
                if (*p == quote) {
                    if (p + 1 < end && p[1] == quote) { p += 2; flen += 2; }
                    else { flen = (size_t)(p - fstart); p++; break; }
                } else p++;
            }
            while (p < end && *p != delim && *p != '\n' && *p != '\r') p++;
        } else {
            while (p < end && *p != delim && *p != '\n' && *p != '\r') p++;
            flen = (size_t)(p - fstart);
        }
        if (nf == cap) { cap *= 2; fs = realloc(fs, cap * sizeof *fs); fl = realloc(fl, cap * sizeof *fl); }
        fs[nf] = fstart; fl[nf] = flen; nf++;
        if (p < end && *p == delim) p++;
    }
    if (header) {
        t->ncols = (int)nf;
        t->columns = malloc(sizeof(cq_column) * (nf ? nf : 1));
        for (size_t i = 0; i < nf; i++) {
            if (t->has_header && fl[i] > 0) {
                char* nm = xstrndup(fs[i], fl[i]);
                char* s = nm;
                while (*s && isspace((unsigned char)*s)) s++;
                size_t sl = strlen(s);
                while (sl > 0 && isspace((unsigned char)s[sl - 1])) s[--sl] = 0;
                memmove(nm, s, sl + 1);
                t->columns[i].name = nm;
            } else {
                char b[32];
                snprintf(b, sizeof b, "$%zu", i);
                t->columns[i].name = strdup(b);
            }
            t->columns[i].inferred_kind = CQ_V_STRING;
        }
    } else {
        cq_row r;
        r.ncols = (int)nf;
        r.values = malloc(sizeof(cq_value) * (nf ? nf : 1));
        for (size_t i = 0; i < nf; i++) r.values[i] = orc_parse_cell(fs[i], fl[i]);
        table_add_row(t, r);
    }
    free(fs);
    free(fl);
}

/* csv_load (csv_reader.c:375-427): records end at any \n or \r, empty lines skipped */
cq_table* orc_load(const char* bytes, size_t n, cq_csv_config cfg) {
    char* data = malloc(n + 1);                  /* NUL-terminated private copy */
    memcpy(data, bytes, n);
    data[n] = 0;
    cq_table* t = table_new("memory");
    t->has_header = cfg.has_header;
    t->delimiter = cfg.delimiter;
    t->quote = cfg.quote;
    const char* p = data;
    const char* end = data + n;
    int first = 1;
    while (p < end) {
        const char* ls = p;
        while (p < end && *p != '\n' && *p != '\r') p++;
        if (p > ls) {
            if (first) {
                split_record(t, ls, p, 1, cfg.quote, cfg.delimiter);
                first = 0;
                if (!cfg.has_header) split_record(t, ls, p, 0, cfg.quote, cfg.delimiter);
            } else {
                split_record(t, ls, p, 0, cfg.quote, cfg.delimiter);
            }
        }
        while (p < end && (*p == '\n' || *p == '\r')) p++;
    }
    free(data);
    return t;
}

cq_table* orc_load_file(const char* path, cq_csv_config cfg) {
    int fd = open(path, O_RDONLY);
    if (fd < 0) return NULL;
    struct stat sb;
    if (fstat(fd, &sb) < 0 || sb.st_size == 0) { close(fd); return NULL; }   /* mmap.c:80-95 */
    char* d = mmap(NULL, (size_t)sb.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (d == MAP_FAILED) return NULL;
    cq_table* t = orc_load(d, (size_t)sb.st_size, cfg);
    munmap(d, (size_t)sb.st_size);
    free(t->filename);
    t->filename = strdup(path);
    return t;
}

/* ------------------------------------------------------------------ context */
typedef struct {
    const char* alias[2];
    cq_table* table[2];
    int ntables;
    cq_node* query;
    int* unsupported;
} octx;

static int col_index(const cq_table* t, const char* name) {     /* csv_reader.c:500-509 */
    if (!t || !name) return -1;
    for (int i = 0; i < t->ncols; i++)
        if (strcasecmp(t->columns[i].name, name) == 0) return i;
    return -1;
}

static int col_index_fallback(const cq_table* t, const char* name) {  /* evaluator_aggregates.c:20-36 */
    int c = col_index(t, name);
    if (c < 0) {
        const char* dot = strchr(name, '.');
        if (dot) c = col_index(t, dot + 1);
    }
    return c;
}

static cq_value eval_expr(octx* c, cq_node* e, cq_row* row, int ti);

static cq_value vnull(void) { cq_value v; memset(&v, 0, sizeof v); return v; }

static cq_value cell_or_null(cq_row* row, int idx) {
    /* reference reads values[idx] unchecked (UB when the row is short); we read NULL */
    if (idx < 0 || idx >= row->ncols) return vnull();
    return vcopy(&row->values[idx]);
}

/* resolve_column (evaluator_core.c:70-167), without outer rows */
static cq_value resolve(octx* c, const char* name, cq_row* row, int ti) {
    if (!name || !row || ti < 0 || ti >= c->ntables) return vnull();
    cq_table* t = c->table[ti];
    const char* dot = strchr(name, '.');
    if (dot) {
        int idx = col_index(t, name);
        if (idx >= 0) return cell_or_null(row, idx);
        char* al = xstrndup(name, (size_t)(dot - name));
        int k = -1;
        for (int i = 0; i < c->ntables; i++)
            if (strcasecmp(c->alias[i], al) == 0) { k = i; break; }
        free(al);
        if (k < 0) return vnull();
        idx = col_index(c->table[k], dot + 1);
        if (idx < 0) return vnull();
        return cell_or_null(row, idx);                 /* index bound from alias table, value from row */
    }
    int idx = col_index(t, name);
    if (idx >= 0) return cell_or_null(row, idx);
    /* SELECT-alias extension (:132-160) */
    cq_node* sel = c->query ? c->query->u.q.select : NULL;
    if (sel && sel->kind == CQ_N_SELECT && sel->u.sel.exprs) {
        for (int i = 0; i < sel->u.sel.count; i++) {
            const char* cs = sel->u.sel.texts[i];
            if (!cs) continue;
            const char* as = strcasestr(cs, " AS ");
            if (!as) continue;
            const char* a = as + 4;
            while (*a && isspace((unsigned char)*a)) a++;
            if (strcasecmp(a, name) == 0) return eval_expr(c, sel->u.sel.exprs[i], row, ti);
        }
    }
    return vnull();
}

/* evaluate_expression (evaluator_expressions.c:23-263) */
static cq_value eval_expr(octx* c, cq_node* e, cq_row* row, int ti) {
    if (!e) return vnull();
    switch (e->kind) {
        case CQ_N_LITERAL: return orc_parse_cell(e->u.text, strlen(e->u.text));
        case CQ_N_IDENTIFIER: return resolve(c, e->u.text, row, ti);
        case CQ_N_BINARY_OP: {
            const char* op = e->u.bin.op;
            if (!e->u.bin.lhs || !e->u.bin.rhs) {
                cq_node* only = e->u.bin.lhs ? e->u.bin.lhs : e->u.bin.rhs;
                if (!only) return vnull();
                cq_value x = eval_expr(c, only, row, ti);
                if (strcmp(op, "-") == 0) {
                    if (x.kind == CQ_V_INT) { x.u.i = (long long)(0ULL - (unsigned long long)x.u.i); return x; }
                    if (x.kind == CQ_V_DOUBLE) { x.u.f = -x.u.f; return x; }
                } else if (strcmp(op, "+") == 0) {
                    return x;
                }
                vfree(&x);
                return vnull();
            }
            cq_value l = eval_expr(c, e->u.bin.lhs, row, ti);
            cq_value r = eval_expr(c, e->u.bin.rhs, row, ti);
            int li = l.kind == CQ_V_INT, ri = r.kind == CQ_V_INT;
            int ln = li || l.kind == CQ_V_DOUBLE, rn = ri || r.kind == CQ_V_DOUBLE;
            if (!ln || !rn) { vfree(&l); vfree(&r); return vnull(); }
            double lv = li ? (double)l.u.i : l.u.f, rv = ri ? (double)r.u.i : r.u.f;
            double res = 0;
            long long resi = 0;
            int is_int = 0;
            if (!strcmp(op, "+")) res = lv + rv;
            else if (!strcmp(op, "-")) res = lv - rv;
            else if (!strcmp(op, "*")) res = lv * rv;
            else if (!strcmp(op, "/")) { if (rv == 0) return vnull(); res = lv / rv; }
            else if (!strcmp(op, "%")) {
                if (li && ri) { if (r.u.i == 0) return vnull(); resi = l.u.i % r.u.i; is_int = 1; }
                else { if (rv == 0) return vnull(); res = fmod(lv, rv); }
            } else if (!strcmp(op, "&") || !strcmp(op, "|") || !strcmp(op, "^")) {
                if (!(li && ri)) return vnull();
                resi = op[0] == '&' ? (l.u.i & r.u.i) : op[0] == '|' ? (l.u.i | r.u.i) : (l.u.i ^ r.u.i);
                is_int = 1;
            }
            cq_value o = vnull();
            if (is_int) { o.kind = CQ_V_INT; o.u.i = resi; }
            else if (li && ri && res >= -9223372036854775808.0 && res < 9223372036854775808.0 &&
                     res == (double)(long long)res) {
                /* (long long)res on x86-64 yields INT64_MIN out of range, which never
                 * compares equal except at -2^63 itself: the range test restates that */
                o.kind = CQ_V_INT; o.u.i = (long long)res;
            } else { o.kind = CQ_V_DOUBLE; o.u.f = res; }
            return o;
        }
        case CQ_N_FUNCTION:
        case CQ_N_CASE:
        case CQ_N_SUBQUERY:
            *c->unsupported = 1;
            return vnull();
        default:
            return vnull();
    }
}

/* match_pattern (evaluator_conditions.c:16-59) */
static int like_match(const char* s, const char* p, int cs) {
    const char *star = NULL, *ss = NULL;
    while (*s) {
        if (*p == '%') { star = p++; ss = s; }
        else if (*p == '_') { s++; p++; }
        else {
            int m = cs ? (*s == *p) : (tolower((unsigned char)*s) == tolower((unsigned char)*p));
            if (m) { s++; p++; }
            else if (star) { p = star + 1; s = ++ss; }
            else return 0;
        }
    }
    while (*p == '%') p++;
    return *p == 0;
}

/* evaluate_condition (evaluator_conditions.c:62-164) */
static int eval_cond(octx* c, cq_node* n, cq_row* row, int ti) {
    if (!n) return 1;
    if (n->kind != CQ_N_CONDITION) return 0;
    const char* op = n->u.bin.op;
    if (!strcasecmp(op, "NOT")) return !eval_cond(c, n->u.bin.lhs, row, ti);
    if (!strcasecmp(op, "AND")) {
        int a = eval_cond(c, n->u.bin.lhs, row, ti);
        int b = eval_cond(c, n->u.bin.rhs, row, ti);
        return a && b;
    }
    if (!strcasecmp(op, "OR")) {
        int a = eval_cond(c, n->u.bin.lhs, row, ti);
        int b = eval_cond(c, n->u.bin.rhs, row, ti);
        return a || b;
    }
    cq_value l = eval_expr(c, n->u.bin.lhs, row, ti);
    cq_value r = eval_expr(c, n->u.bin.rhs, row, ti);
    int cmp = orc_compare(&l, &r), res = 0;
    if (!strcmp(op, "=")) res = cmp == 0;
    else if (!strcmp(op, "!=") || !strcmp(op, "<>")) res = cmp != 0;
    else if (!strcmp(op, ">")) res = cmp > 0;
    else if (!strcmp(op, "<")) res = cmp < 0;
    else if (!strcmp(op, ">=")) res = cmp >= 0;
    else if (!strcmp(op, "<=")) res = cmp <= 0;
    else if (!strcasecmp(op, "IN") || !strcasecmp(op, "NOT IN")) {
        int neg = !strcasecmp(op, "NOT IN");
        cq_node* rn = n->u.bin.rhs;
        if (rn && rn->kind == CQ_N_SUBQUERY) { *c->unsupported = 1; res = 0; }
        else if (rn && rn->kind == CQ_N_LIST) {
            int found = 0;
            for (int i = 0; i < rn->u.list.nitems && !found; i++) {
                cq_value x = eval_expr(c, rn->u.list.items[i], row, ti);
                if (orc_compare(&l, &x) == 0) found = 1;
                vfree(&x);
            }
            res = neg ? !found : found;
        } else res = neg;
    } else if (!strcasecmp(op, "LIKE") || !strcasecmp(op, "ILIKE")) {
        int cs = !strcasecmp(op, "LIKE");
        res = (l.kind == CQ_V_STRING && r.kind == CQ_V_STRING) ? like_match(l.u.s, r.u.s, cs) : 0;
    }
    vfree(&l);
    vfree(&r);
    return res;
}

/* ------------------------------------------------------------------ joins */
/* perform_join (evaluator_joins.c:63-181) */
static int join_match(octx* c, cq_node* on, cq_row* lr, cq_row* rr) {   /* :40-60 */
    if (!on) return 1;
    if (on->kind == CQ_N_CONDITION && !strcmp(on->u.bin.op, "=") && on->u.bin.lhs &&
        on->u.bin.rhs && on->u.bin.lhs->kind == CQ_N_IDENTIFIER &&
        on->u.bin.rhs->kind == CQ_N_IDENTIFIER) {
        /* resolve_column returns NULL (no match) when the name is unknown */
        cq_table* save_q = NULL;
        (void)save_q;
        int lk = 0, rk = 0;
        cq_value a = vnull(), b = vnull();
        /* we need "found" vs "NULL value": re-implement the lookup to know */
        const char* names[2] = {on->u.bin.lhs->u.text, on->u.bin.rhs->u.text};
        cq_row* rows[2] = {lr, rr};
        cq_value* outs[2] = {&a, &b};
        int* oks[2] = {&lk, &rk};
        for (int s = 0; s < 2; s++) {
            const char* nm = names[s];
            cq_table* t = c->table[s];
            const char* dot = strchr(nm, '.');
            int idx = col_index(t, nm);
            if (idx < 0 && dot) {
                char* al = xstrndup(nm, (size_t)(dot - nm));
                int k = -1;
                for (int i = 0; i < c->ntables; i++)
                    if (strcasecmp(c->alias[i], al) == 0) { k = i; break; }
                free(al);
                if (k >= 0) idx = col_index(c->table[k], dot + 1);
            }
            if (idx < 0 && !dot) {
                /* SELECT-alias extension would evaluate an expression here; treated as no match */
                *oks[s] = 0;
                continue;
            }
            if (idx < 0) { *oks[s] = 0; continue; }
            *oks[s] = 1;
            *outs[s] = cell_or_null(rows[s], idx);
        }
        int m = lk && rk && orc_compare(&a, &b) == 0;
        vfree(&a);
        vfree(&b);
        return m;
    }
    return 0;
}

static cq_table* do_join(octx* c, cq_table* L, const char* la, cq_table* R, const char* ra,
                         cq_node* on, int kind) {
    cq_table* out = table_new("joined_result");
    out->ncols = L->ncols + R->ncols;
    out->columns = malloc(sizeof(cq_column) * (size_t)(out->ncols ? out->ncols : 1));
    char nb[256];
    for (int i = 0; i < L->ncols; i++) {
        snprintf(nb, sizeof nb, "%s.%s", la, L->columns[i].name);
        out->columns[i].name = strdup(nb);
        out->columns[i].inferred_kind = L->columns[i].inferred_kind;
    }
    for (int i = 0; i < R->ncols; i++) {
        snprintf(nb, sizeof nb, "%s.%s", ra, R->columns[i].name);
        out->columns[L->ncols + i].name = strdup(nb);
        out->columns[L->ncols + i].inferred_kind = R->columns[i].inferred_kind;
    }
    octx jc = *c;
    jc.ntables = 2;
    jc.alias[0] = la; jc.table[0] = L;
    jc.alias[1] = ra; jc.table[1] = R;
    for (int l = 0; l < L->nrows; l++) {
        int found = 0;
        for (int r = 0; r < R->nrows; r++) {
            int m = join_match(&jc, on, &L->rows[l], &R->rows[r]);
            if (m || (kind == CQ_JOIN_INNER && on == NULL)) {
                found = 1;
                cq_row nr;
                nr.ncols = out->ncols;
                nr.values = malloc(sizeof(cq_value) * (size_t)(out->ncols ? out->ncols : 1));
                for (int i = 0; i < L->ncols; i++) nr.values[i] = cell_or_null(&L->rows[l], i);
                for (int i = 0; i < R->ncols; i++) nr.values[L->ncols + i] = cell_or_null(&R->rows[r], i);
                table_add_row(out, nr);
            }
        }
        if (!found && (kind == CQ_JOIN_LEFT || kind == CQ_JOIN_FULL)) {
            cq_row nr;
            nr.ncols = out->ncols;
            nr.values = calloc((size_t)(out->ncols ? out->ncols : 1), sizeof(cq_value));
            for (int i = 0; i < L->ncols; i++) nr.values[i] = cell_or_null(&L->rows[l], i);
            table_add_row(out, nr);
        }
    }
    if (kind == CQ_JOIN_RIGHT || kind == CQ_JOIN_FULL) {
        for (int r = 0; r < R->nrows; r++) {
            int found = 0;
            for (int l = 0; l < L->nrows && !found; l++)
                if (join_match(&jc, on, &L->rows[l], &R->rows[r])) found = 1;
            if (!found) {
                cq_row nr;
                nr.ncols = out->ncols;
                nr.values = calloc((size_t)(out->ncols ? out->ncols : 1), sizeof(cq_value));
                for (int i = 0; i < R->ncols; i++) nr.values[L->ncols + i] = cell_or_null(&R->rows[r], i);
                table_add_row(out, nr);
            }
        }
    }
    return out;
}

/* load_table (evaluator_joins.c:184-234 uses the path verbatim) */
static cq_table* load_path(const char* path, cq_csv_config cfg) {
    cq_table* t = orc_load_file(path, cfg);
    if (!t) fprintf(stderr, "oracle: failed to load table from '%s'\n", path);
    return t;
}

/* ------------------------------------------------------------------ grouping */
typedef struct {
    char* key;
    int* rows;
    int nrows, cap;
} ogroup;

typedef struct {
    ogroup* g;
    int n, cap;
    /* open-addressing index over keys (first-appearance order kept in g[]) */
    int* slots;
    size_t nslots;
} ogroups;

static unsigned long long fnv(const char* s) {
    unsigned long long h = 1469598103934665603ULL;
    while (*s) { h ^= (unsigned char)*s++; h *= 1099511628211ULL; }
    return h;
}

static int groups_find_or_add(ogroups* gs, const char* key) {
    if (gs->n * 2 >= (int)gs->nslots) {
        size_t ns = gs->nslots ? gs->nslots * 2 : 1024;
        int* sl = malloc(ns * sizeof(int));
        for (size_t i = 0; i < ns; i++) sl[i] = -1;
        for (int i = 0; i < gs->n; i++) {
            size_t h = fnv(gs->g[i].key) & (ns - 1);
            while (sl[h] >= 0) h = (h + 1) & (ns - 1);
            sl[h] = i;
        }
        free(gs->slots);
        gs->slots = sl;
        gs->nslots = ns;
    }
    size_t h = fnv(key) & (gs->nslots - 1);
    while (gs->slots[h] >= 0) {
        if (!strcmp(gs->g[gs->slots[h]].key, key)) return gs->slots[h];
        h = (h + 1) & (gs->nslots - 1);
    }
    if (gs->n == gs->cap) {
        gs->cap = gs->cap ? gs->cap * 2 : 16;
        gs->g = realloc(gs->g, sizeof(ogroup) * (size_t)gs->cap);
    }
    ogroup* g = &gs->g[gs->n];
    g->key = strdup(key);
    g->cap = 16;
    g->nrows = 0;
    g->rows = malloc(sizeof(int) * 16);
    gs->slots[h] = gs->n;
    return gs->n++;
}

static void group_add(ogroup* g, int r) {
    if (g->nrows == g->cap) { g->cap *= 2; g->rows = realloc(g->rows, sizeof(int) * (size_t)g->cap); }
    g->rows[g->nrows++] = r;
}

/* key text for one value (evaluator_aggregates.c:122-141) */
static void key_text(const cq_value* v, char* buf /* 256 */) {
    switch (v->kind) {
        case CQ_V_NULL: strcpy(buf, "NULL"); break;
        case CQ_V_INT: snprintf(buf, 256, "%lld", v->u.i); break;
        case CQ_V_DOUBLE: snprintf(buf, 256, "%.6f", v->u.f); break;
        case CQ_V_DATE: snprintf(buf, 256, "%04d-%02d-%02d", v->u.date.y, v->u.date.m, v->u.date.d); break;
        case CQ_V_STRING: strncpy(buf, v->u.s, 255); buf[255] = 0; break;
        default: strcpy(buf, "");
    }
}

static void groups_free(ogroups* gs) {
    for (int i = 0; i < gs->n; i++) { free(gs->g[i].key); free(gs->g[i].rows); }
    free(gs->g);
    free(gs->slots);
}

/* ------------------------------------------------------------------ aggregates */
static int is_agg_name(const char* f) {              /* evaluator_aggregates.c:43-52 */
    return !strcasecmp(f, "COUNT") || !strcasecmp(f, "SUM") || !strcasecmp(f, "AVG") ||
           !strcasecmp(f, "MIN") || !strcasecmp(f, "MAX") || !strcasecmp(f, "STDDEV") ||
           !strcasecmp(f, "STDDEV_POP") || !strcasecmp(f, "MEDIAN");
}

static int has_aggregates(cq_node* sel) {           /* :55-106 (column_nodes branch) */
    if (!sel || sel->kind != CQ_N_SELECT) return 0;
    if (sel->u.sel.exprs) {
        for (int i = 0; i < sel->u.sel.count; i++) {
            cq_node* n = sel->u.sel.exprs[i];
            if (!n || n->kind != CQ_N_FUNCTION) continue;
            const char* f = n->u.fn.name;
            if (!strcasecmp(f, "COUNT") || !strcasecmp(f, "SUM") || !strcasecmp(f, "AVG") ||
                !strcasecmp(f, "MIN") || !strcasecmp(f, "MAX") || !strcasecmp(f, "STDDEV") ||
                !strcasecmp(f, "MEDIAN"))
                return 1;
        }
        return 0;
    }
    for (int i = 0; i < sel->u.sel.count; i++) {
        const char* cs = sel->u.sel.texts[i];
        if ((strstr(cs, "COUNT(") || strstr(cs, "SUM(") || strstr(cs, "AVG(") || strstr(cs, "MIN(") ||
             strstr(cs, "MAX(") || strstr(cs, "STDDEV(") || strstr(cs, "MEDIAN(")) &&
            !strcasestr(cs, "OVER"))
            return 1;
    }
    return 0;
}

static int cmp_dbl(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}

/* evaluate_aggregate (evaluator_aggregates.c:263-414) */
static cq_value aggregate(const char* fn, cq_table* t, const int* rows, int n, const char* col) {
    cq_value res = vnull();
    if (!strcasecmp(fn, "COUNT") && !strcmp(col, "*")) { res.kind = CQ_V_INT; res.u.i = n; return res; }
    int ci = col_index_fallback(t, col);
    if (ci < 0) return res;
    if (!strcasecmp(fn, "COUNT")) { res.kind = CQ_V_INT; res.u.i = n; return res; }
#define CELL(k) ((ci < t->rows[rows[k]].ncols) ? &t->rows[rows[k]].values[ci] : &nullv)
    cq_value nullv = vnull();
    if (!strcasecmp(fn, "AVG") || !strcasecmp(fn, "SUM")) {
        double s = 0;
        int cnt = 0;
        for (int k = 0; k < n; k++) {
            const cq_value* v = CELL(k);
            if (v->kind == CQ_V_INT) { s += v->u.i; cnt++; }
            else if (v->kind == CQ_V_DOUBLE) { s += v->u.f; cnt++; }
        }
        res.kind = CQ_V_DOUBLE;
        res.u.f = !strcasecmp(fn, "SUM") ? s : (cnt > 0 ? s / cnt : 0);
        return res;
    }
    if (!strcasecmp(fn, "MIN") || !strcasecmp(fn, "MAX")) {
        const cq_value* ex = NULL;
        int mn = !strcasecmp(fn, "MIN");
        for (int k = 0; k < n; k++) {
            const cq_value* v = CELL(k);
            if (v->kind == CQ_V_NULL) continue;
            if (!ex || (mn && orc_compare(v, ex) < 0) || (!mn && orc_compare(v, ex) > 0)) ex = v;
        }
        if (ex) return vcopy(ex);
    }
    if (!strcasecmp(fn, "STDDEV") || !strcasecmp(fn, "STDDEV_POP")) {
        double s = 0;
        int cnt = 0;
        for (int k = 0; k < n; k++) {
            const cq_value* v = CELL(k);
            if (v->kind == CQ_V_INT) { s += v->u.i; cnt++; }
            else if (v->kind == CQ_V_DOUBLE) { s += v->u.f; cnt++; }
        }
        if (cnt == 0) return res;
        double mean = s / cnt, vs = 0;
        for (int k = 0; k < n; k++) {
            const cq_value* v = CELL(k);
            double x;
            if (v->kind == CQ_V_INT) x = v->u.i;
            else if (v->kind == CQ_V_DOUBLE) x = v->u.f;
            else continue;
            double d = x - mean;
            vs += d * d;
        }
        res.kind = CQ_V_DOUBLE;
        res.u.f = sqrt(vs / cnt);
        return res;
    }
    if (!strcasecmp(fn, "MEDIAN")) {
        double* xs = malloc(sizeof(double) * (size_t)(n ? n : 1));
        int cnt = 0;
        for (int k = 0; k < n; k++) {
            const cq_value* v = CELL(k);
            if (v->kind == CQ_V_INT) xs[cnt++] = (double)v->u.i;
            else if (v->kind == CQ_V_DOUBLE) xs[cnt++] = v->u.f;
        }
        if (cnt) {
            /* the reference's exchange sort is O(n^2); any correct sort yields the
             * same order statistics for non-NaN doubles */
            qsort(xs, (size_t)cnt, sizeof(double), cmp_dbl);
            res.kind = CQ_V_DOUBLE;
            res.u.f = (cnt % 2) ? xs[cnt / 2] : (xs[cnt / 2 - 1] + xs[cnt / 2]) / 2.0;
        }
        free(xs);
        return res;
    }
#undef CELL
    return res;
}

static void rtrim(char* s) {
    size_t l = strlen(s);
    while (l > 0 && isspace((unsigned char)s[l - 1])) s[--l] = 0;
}

/* build_aggregated_result (evaluator_aggregates.c:533-696) */
static cq_table* build_agg(octx* c, ogroups* gs, cq_node* sel) {
    cq_table* out = table_new("query_result");
    cq_table* t = c->table[0];
    if (!sel) return out;
    out->ncols = sel->u.sel.count;
    out->columns = malloc(sizeof(cq_column) * (size_t)(out->ncols ? out->ncols : 1));
    for (int i = 0; i < out->ncols; i++) {
        const char* cs = sel->u.sel.texts[i];
        const char* as = strcasestr(cs, " AS ");
        if (as) out->columns[i].name = strdup(as + 4);
        else {
            const char* par = strchr(cs, '(');
            if (par) {
                char fb[256], ab[128], dn[600];
                const char* pc = strchr(par, ')');
                int fl = (int)(par - cs);
                memcpy(fb, cs, (size_t)fl); fb[fl] = 0;
                int al = pc ? (int)(pc - par - 1) : (int)strlen(par + 1);
                if (al > 127) al = 127;
                memcpy(ab, par + 1, (size_t)al); ab[al] = 0;
                const char* dot = strchr(ab, '.');
                snprintf(dn, sizeof dn, "%s(%s)", fb, dot ? dot + 1 : ab);
                dn[255] = 0;
                out->columns[i].name = strdup(dn);
            } else {
                const char* dot = strchr(cs, '.');
                out->columns[i].name = strdup(dot ? dot + 1 : cs);
            }
        }
        out->columns[i].inferred_kind = CQ_V_STRING;
    }
    out->nrows = out->row_capacity = gs->n;
    out->rows = malloc(sizeof(cq_row) * (size_t)(gs->n ? gs->n : 1));
    for (int g = 0; g < gs->n; g++) {
        ogroup* gr = &gs->g[g];
        cq_row* r = &out->rows[g];
        r->ncols = out->ncols;
        r->values = calloc((size_t)(out->ncols ? out->ncols : 1), sizeof(cq_value));
        for (int ci = 0; ci < out->ncols; ci++) {
            const char* cs = sel->u.sel.texts[ci];
            char cn[512];
            const char* as = strcasestr(cs, " AS ");
            if (as) { size_t l = (size_t)(as - cs); memcpy(cn, cs, l); cn[l] = 0; }
            else snprintf(cn, sizeof cn, "%s", cs);
            rtrim(cn);
            char* par = strchr(cn, '(');
            if (par) {
                char fn[64];
                size_t fl = (size_t)(par - cn);
                if (fl > 63) fl = 63;
                memcpy(fn, cn, fl); fn[fl] = 0;
                if (is_agg_name(fn)) {
                    char* pc = strchr(par + 1, ')');
                    char arg[512];
                    if (pc) { size_t al = (size_t)(pc - par - 1); memcpy(arg, par + 1, al); arg[al] = 0; }
                    else snprintf(arg, sizeof arg, "%s", cn);
                    r->values[ci] = aggregate(fn, t, gr->rows, gr->nrows, arg);
                } else {
                    *c->unsupported = 1;                 /* scalar function over group */
                }
            } else {
                cq_node* cn_node = sel->u.sel.exprs ? sel->u.sel.exprs[ci] : NULL;
                if (cn_node && cn_node->kind != CQ_N_IDENTIFIER) {
                    if (gr->nrows > 0) r->values[ci] = eval_expr(c, cn_node, &t->rows[gr->rows[0]], 0);
                } else {
                    int idx = col_index_fallback(t, cn);
                    if (idx >= 0 && gr->nrows > 0) r->values[ci] = cell_or_null(&t->rows[gr->rows[0]], idx);
                }
            }
        }
    }
    return out;
}

/* ------------------------------------------------------------------ projection */
/* build_result (evaluator_utils.c:249-549), expression columns only */
static cq_table* build_rows(octx* c, const int* rows, int n) {
    cq_table* out = table_new("query_result");
    cq_node* sel = c->query->u.q.select;
    cq_table* t = c->table[0];
    if (!sel) return out;
    int star = 0;
    for (int i = 0; i < sel->u.sel.count; i++)
        if (!strcmp(sel->u.sel.texts[i], "*")) star = 1;
    int total = star ? sel->u.sel.count - 1 + t->ncols : sel->u.sel.count;
    int* src = malloc(sizeof(int) * (size_t)(total ? total : 1));     /* table col for '*', else -1 */
    int* orig = malloc(sizeof(int) * (size_t)(total ? total : 1));    /* select index or -1 */
    out->ncols = total;
    out->columns = malloc(sizeof(cq_column) * (size_t)(total ? total : 1));
    int k = 0;
    for (int i = 0; i < sel->u.sel.count; i++) {
        const char* cs = sel->u.sel.texts[i];
        if (star && !strcmp(cs, "*")) {
            for (int j = 0; j < t->ncols; j++) {
                out->columns[k].name = strdup(t->columns[j].name);
                out->columns[k].inferred_kind = CQ_V_STRING;
                src[k] = j; orig[k] = -1; k++;
            }
            continue;
        }
        const char* as = strcasestr(cs, " AS ");
        char cn[512];
        if (as) {
            out->columns[k].name = strdup(as + 4);
            size_t l = (size_t)(as - cs); memcpy(cn, cs, l); cn[l] = 0;
        } else {
            snprintf(cn, sizeof cn, "%s", cs);
            if (strchr(cn, '(')) out->columns[k].name = strdup(cn);
            else { const char* dot = strchr(cn, '.'); out->columns[k].name = strdup(dot ? dot + 1 : cn); }
        }
        out->columns[k].inferred_kind = CQ_V_STRING;
        src[k] = strchr(cn, '(') ? -1 : col_index_fallback(t, cn);
        orig[k] = i;
        k++;
    }
    out->nrows = out->row_capacity = n;
    out->rows = malloc(sizeof(cq_row) * (size_t)(n ? n : 1));
    for (int i = 0; i < n; i++) {
        cq_row* row = &t->rows[rows[i]];
        cq_row* r = &out->rows[i];
        r->ncols = total;
        r->values = calloc((size_t)(total ? total : 1), sizeof(cq_value));
        for (int j = 0; j < total; j++) {
            cq_node* cn = (orig[j] >= 0 && sel->u.sel.exprs) ? sel->u.sel.exprs[orig[j]] : NULL;
            if (cn) {
                if (cn->kind == CQ_N_SUBQUERY || cn->kind == CQ_N_WINDOW_FUNCTION) *c->unsupported = 1;
                else r->values[j] = eval_expr(c, cn, row, 0);
            } else if (orig[j] >= 0 && strchr(sel->u.sel.texts[orig[j]], '(')) {
                *c->unsupported = 1;
            } else if (src[j] >= 0 && src[j] < row->ncols) {
                r->values[j] = vcopy(&row->values[src[j]]);
            }
        }
    }
    free(src);
    free(orig);
    return out;
}

/* ------------------------------------------------------------------ post-ops */
static int g_sort_col, g_sort_desc;
static int cmp_rows(const void* a, const void* b) {      /* evaluator_utils.c:560-576 */
    const cq_row* x = a;
    const cq_row* y = b;
    if (g_sort_col < 0 || g_sort_col >= x->ncols) return 0;
    int c = orc_compare(&x->values[g_sort_col], &y->values[g_sort_col]);
    return g_sort_desc ? -c : c;
}

/* stable merge sort: glibc qsort is a merge sort for these sizes */
static void msort_rows(cq_row* a, int n) {
    if (n < 2) return;
    cq_row* tmp = malloc(sizeof(cq_row) * (size_t)n);
    for (int w = 1; w < n; w *= 2) {
        for (int lo = 0; lo < n; lo += 2 * w) {
            int mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
            int i = lo, j = mid, k = lo;
            while (i < mid && j < hi) tmp[k++] = cmp_rows(&a[j], &a[i]) < 0 ? a[j++] : a[i++];
            while (i < mid) tmp[k++] = a[i++];
            while (j < hi) tmp[k++] = a[j++];
        }
        memcpy(a, tmp, sizeof(cq_row) * (size_t)n);
    }
    free(tmp);
}

static void norm_func(const char* spec, char* out /*256*/) {
    const char* par = strchr(spec, '(');
    if (par) {
        char fn[64], ab[128];
        size_t fl = (size_t)(par - spec);
        if (fl > 63) fl = 63;
        memcpy(fn, spec, fl); fn[fl] = 0;
        const char* pc = strchr(par + 1, ')');
        if (!pc) { out[0] = 0; return; }
        size_t al = (size_t)(pc - par - 1);
        if (al > 127) al = 127;
        memcpy(ab, par + 1, al); ab[al] = 0;
        const char* dot = strchr(ab, '.');
        snprintf(out, 256, "%s(%s)", fn, dot ? dot + 1 : ab);
    } else {
        const char* dot = strchr(spec, '.');
        snprintf(out, 256, "%s", dot ? dot + 1 : spec);
    }
}

/* sort_result (evaluator_utils.c:579-700) */
static void sort_result(cq_table* r, cq_node* sel, const char* spec, int desc) {
    if (!r || r->nrows == 0) return;
    char look[256];
    norm_func(spec, look);
    int ci = -1;
    for (int i = 0; i < r->ncols; i++)
        if (!strcasecmp(r->columns[i].name, look)) { ci = i; break; }
    if (ci < 0 && sel) {
        for (int i = 0; i < sel->u.sel.count; i++) {
            const char* cs = sel->u.sel.texts[i];
            char eb[256];
            const char* as = strcasestr(cs, " AS ");
            if (as) { size_t l = (size_t)(as - cs); if (l > 255) l = 255; memcpy(eb, cs, l); eb[l] = 0; }
            else { strncpy(eb, cs, 255); eb[255] = 0; }
            rtrim(eb);
            char ne[256];
            norm_func(eb, ne);
            if (!strcasecmp(ne, look)) { ci = i; break; }
        }
    }
    if (ci < 0) return;
    g_sort_col = ci;
    g_sort_desc = desc;
    msort_rows(r->rows, r->nrows);
}

static void free_rows(cq_row* rows, int a, int b) {
    for (int i = a; i < b; i++) {
        for (int j = 0; j < rows[i].ncols; j++) vfree(&rows[i].values[j]);
        free(rows[i].values);
    }
}

/* apply_limit_offset (evaluator_utils.c:703-733) */
static void limit_offset(cq_table* r, int limit, int offset) {
    if (limit < 0 && offset < 0) return;
    int off = offset >= 0 ? offset : 0;
    int lim = limit >= 0 ? limit : r->nrows;
    if (off >= r->nrows) { free_rows(r->rows, 0, r->nrows); r->nrows = 0; return; }
    int cnt = lim;
    if (off + cnt > r->nrows) cnt = r->nrows - off;
    free_rows(r->rows, 0, off);
    free_rows(r->rows, off + cnt, r->nrows);
    if (off > 0 && cnt > 0) memmove(r->rows, r->rows + off, sizeof(cq_row) * (size_t)cnt);
    r->nrows = cnt;
}

/* apply_distinct (evaluator_utils.c:868-932) */
static void distinct(cq_table* r) {
    if (r->nrows <= 1) return;
    char* keep = calloc((size_t)r->nrows, 1);
    int w = 0;
    for (int i = 0; i < r->nrows; i++) {
        int dup = 0;
        for (int j = 0; j < i && !dup; j++) {
            if (!keep[j]) continue;
            int eq = 1;
            for (int c = 0; c < r->ncols && eq; c++)
                if (orc_compare(&r->rows[i].values[c], &r->rows[j].values[c]) != 0) eq = 0;
            if (eq) dup = 1;
        }
        if (!dup) keep[i] = 1;
    }
    for (int i = 0; i < r->nrows; i++) {
        if (keep[i]) r->rows[w++] = r->rows[i];
        else free_rows(r->rows, i, i + 1);
    }
    r->nrows = w;
    free(keep);
}

/* HAVING (evaluator_aggregates.c:417-530) */
static cq_value having_expr(cq_node* e, cq_table* r, int ri, cq_node* sel) {
    cq_value v = vnull();
    if (!e) return v;
    if (e->kind == CQ_N_LITERAL) return orc_parse_cell(e->u.text, strlen(e->u.text));
    if (e->kind == CQ_N_FUNCTION) {
        char fs[256];
        snprintf(fs, sizeof fs, "%s(", e->u.fn.name);
        for (int i = 0; i < e->u.fn.nargs; i++) {
            if (i > 0) strncat(fs, ", ", sizeof fs - strlen(fs) - 1);
            cq_node* a = e->u.fn.args[i];
            if (a && (a->kind == CQ_N_IDENTIFIER || a->kind == CQ_N_LITERAL))
                strncat(fs, a->u.text, sizeof fs - strlen(fs) - 1);
        }
        strncat(fs, ")", sizeof fs - strlen(fs) - 1);
        for (int c = 0; c < r->ncols; c++) {
            if (!strcasecmp(r->columns[c].name, fs) ||
                (sel && c < sel->u.sel.count && !strncasecmp(sel->u.sel.texts[c], fs, strlen(fs))))
                return vcopy(&r->rows[ri].values[c]);
        }
    }
    if (e->kind == CQ_N_IDENTIFIER) {
        for (int c = 0; c < r->ncols; c++)
            if (!strcasecmp(r->columns[c].name, e->u.text)) return vcopy(&r->rows[ri].values[c]);
    }
    return v;
}

static int having_cond(cq_node* n, cq_table* r, int ri, cq_node* sel) {
    if (!n) return 1;
    if (n->kind != CQ_N_CONDITION) return 0;
    const char* op = n->u.bin.op;
    if (!strcasecmp(op, "AND")) return having_cond(n->u.bin.lhs, r, ri, sel) && having_cond(n->u.bin.rhs, r, ri, sel);
    if (!strcasecmp(op, "OR")) return having_cond(n->u.bin.lhs, r, ri, sel) || having_cond(n->u.bin.rhs, r, ri, sel);
    cq_value a = having_expr(n->u.bin.lhs, r, ri, sel), b = having_expr(n->u.bin.rhs, r, ri, sel);
    int c = orc_compare(&a, &b), res = 0;
    if (!strcmp(op, "=")) res = c == 0;
    else if (!strcmp(op, "!=") || !strcmp(op, "<>")) res = c != 0;
    else if (!strcmp(op, ">")) res = c > 0;
    else if (!strcmp(op, "<")) res = c < 0;
    else if (!strcmp(op, ">=")) res = c >= 0;
    else if (!strcmp(op, "<=")) res = c <= 0;
    vfree(&a);
    vfree(&b);
    return res;
}

static void apply_having(cq_table* r, cq_node* h, cq_node* sel) {
    if (!h || r->nrows == 0) return;
    int w = 0;
    for (int i = 0; i < r->nrows; i++) {
        if (having_cond(h, r, i, sel)) r->rows[w++] = r->rows[i];
        else free_rows(r->rows, i, i + 1);
    }
    r->nrows = w;
}

/* ------------------------------------------------------------------ query */
/* evaluate_query_internal (evaluator.c:26-287) */
cq_table* orc_evaluate(cq_node* q, cq_csv_config cfg, int* unsupported) {
    int dummy = 0;
    if (!unsupported) unsupported = &dummy;
    *unsupported = 0;
    if (!q || q->kind != CQ_N_QUERY) { *unsupported = 1; return NULL; }
    cq_node* from = q->u.q.from;
    if (!from || from->kind != CQ_N_FROM) return NULL;
    if (from->u.from.subquery || !from->u.from.path) { *unsupported = 1; return NULL; }
    cq_table* base = load_path(from->u.from.path, cfg);
    if (!base) return NULL;
    octx c;
    memset(&c, 0, sizeof c);
    c.query = q;
    c.unsupported = unsupported;
    c.ntables = 1;
    c.alias[0] = from->u.from.alias ? from->u.from.alias : "main";
    c.table[0] = base;
    /* process_joins (evaluator_joins.c:237-274) */
    cq_table* work = base;
    const char* walias = c.alias[0];
    int joined = 0;
    for (int j = 0; j < q->u.q.join_count; j++) {
        cq_node* jn = q->u.q.joins[j];
        if (!jn || jn->kind != CQ_N_JOIN) continue;
        cq_table* R = load_path(jn->u.join.path, cfg);
        if (!R) continue;
        const char* ra = jn->u.join.alias ? jn->u.join.alias : "right";
        cq_table* J = do_join(&c, work, walias, R, ra, jn->u.join.on, jn->u.join.kind);
        if (joined) orc_free(work);
        orc_free(R);
        work = J;
        walias = "joined";
        joined = 1;
    }
    if (joined) { orc_free(base); c.table[0] = work; }
    cq_table* t = c.table[0];
    /* filter_rows (evaluator_utils.c:986-1006) */
    int* keep = malloc(sizeof(int) * (size_t)(t->nrows ? t->nrows : 1));
    int nk = 0;
    for (int i = 0; i < t->nrows; i++)
        if (!q->u.q.where || eval_cond(&c, q->u.q.where, &t->rows[i], 0)) keep[nk++] = i;
    cq_node* sel = q->u.q.select;
    cq_node* gb = q->u.q.group_by;
    cq_table* res = NULL;
    cq_node* ob = q->u.q.order_by;
    if (gb && gb->kind == CQ_N_GROUP_BY && gb->u.grp.keys && gb->u.grp.nkeys > 0) {
        int nk2 = gb->u.grp.nkeys;
        cq_node** gexpr = calloc((size_t)nk2, sizeof(cq_node*));
        for (int g = 0; g < nk2; g++) {                    /* alias check evaluator.c:78-103 */
            if (!sel || sel->kind != CQ_N_SELECT || !sel->u.sel.exprs) continue;
            for (int i = 0; i < sel->u.sel.count; i++) {
                const char* cs = sel->u.sel.texts[i];
                if (!cs) continue;
                const char* as = strcasestr(cs, " AS ");
                if (!as) continue;
                const char* a = as + 4;
                while (*a && isspace((unsigned char)*a)) a++;
                if (!strcasecmp(a, gb->u.grp.keys[g])) { gexpr[g] = sel->u.sel.exprs[i]; break; }
            }
        }
        ogroups gs;
        memset(&gs, 0, sizeof gs);
        if (nk2 == 1 && !gexpr[0]) {                       /* create_groups :108-176 */
            int gi = col_index_fallback(t, gb->u.grp.keys[0]);
            if (gi >= 0) {
                for (int k = 0; k < nk; k++) {
                    cq_value v = cell_or_null(&t->rows[keep[k]], gi);
                    char kb[256];
                    key_text(&v, kb);
                    vfree(&v);
                    int gix = groups_find_or_add(&gs, kb);
                    group_add(&gs.g[gix], keep[k]);
                }
            }
        } else {
            for (int k = 0; k < nk; k++) {                 /* composite :113-212 and by-expression */
                char ck[1024] = "";
                for (int g = 0; g < nk2; g++) {
                    if (g > 0) strcat(ck, "\t");
                    char kp[256];
                    cq_value v;
                    if (gexpr[g]) v = eval_expr(&c, gexpr[g], &t->rows[keep[k]], 0);
                    else {
                        /* the composite path does NOT strip the table prefix (evaluator.c:152);
                         * the single-column by-expression path (create_groups_by_expression) is
                         * the same key text */
                        int gi = col_index(t, gb->u.grp.keys[g]);
                        v = gi >= 0 ? cell_or_null(&t->rows[keep[k]], gi) : vnull();
                    }
                    key_text(&v, kp);
                    vfree(&v);
                    strncat(ck, kp, sizeof ck - strlen(ck) - 1);
                }
                int gix = groups_find_or_add(&gs, ck);
                group_add(&gs.g[gix], keep[k]);
            }
        }
        free(gexpr);
        res = build_agg(&c, &gs, sel);
        groups_free(&gs);
        if (q->u.q.having) apply_having(res, q->u.q.having, sel);
        if (ob && ob->kind == CQ_N_ORDER_BY && ob->u.ord.key) sort_result(res, sel, ob->u.ord.key, ob->u.ord.desc);
    } else if (has_aggregates(sel)) {                      /* evaluator.c:232-258 */
        ogroups gs;
        memset(&gs, 0, sizeof gs);
        gs.n = gs.cap = 1;
        gs.g = calloc(1, sizeof(ogroup));
        gs.g[0].key = strdup("_all_");
        gs.g[0].rows = keep;
        gs.g[0].nrows = nk;
        res = build_agg(&c, &gs, sel);
        free(gs.g[0].key);
        free(gs.g);
        keep = NULL;
        if (q->u.q.having) apply_having(res, q->u.q.having, sel);
        if (ob && ob->kind == CQ_N_ORDER_BY && ob->u.ord.key) sort_result(res, sel, ob->u.ord.key, ob->u.ord.desc);
    } else {
        res = build_rows(&c, keep, nk);
        if (ob && ob->kind == CQ_N_ORDER_BY && ob->u.ord.key) sort_result(res, sel, ob->u.ord.key, ob->u.ord.desc);
    }
    free(keep);
    orc_free(c.table[0]);
    if (sel && sel->u.sel.distinct) distinct(res);
    limit_offset(res, q->u.q.limit, q->u.q.offset);
    return res;
}
