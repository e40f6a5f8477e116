/* Every SQL line of a file through the reference parser and the oracle
 * (oracle/cq_oracle.c), both built with AddressSanitizer (scripts/asan_parse.sh
 * oracle): finds heap corruption in the test-side C code without a GPU. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "parser.h"
#include "csv_reader.h"
#include "../oracle/cq_oracle.h"

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "r");
    if (!f) return 2;
    CsvConfig rc = csv_config_default();
    cq_csv_config cfg;
    memcpy(&cfg, &rc, sizeof cfg < sizeof rc ? sizeof cfg : sizeof rc);
    static char line[1 << 16];
    int n = 0;
    while (fgets(line, sizeof line, f)) {
        size_t k = strlen(line);
        while (k && (line[k - 1] == '\n' || line[k - 1] == '\r')) line[--k] = 0;
        if (!k) continue;
        fprintf(stderr, "[%d] %s\n", n++, line);
        ASTNode* a = parse(line);
        if (!a) continue;
        int unsup = 0;
        cq_table* t = orc_evaluate((cq_node*)a, cfg, &unsup);
        if (t) orc_free(t);
        releaseNode(a);
    }
    fclose(f);
    return 0;
}
