/* Parse-and-release every SQL line of a file through the reference parser built
 * with AddressSanitizer (scripts/asan_parse.sh): finds the statements whose parse
 * corrupts the heap of the process that hosts the parser (the tests' front end). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "parser.h"

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "r");
    if (!f) return 2;
    static char line[1 << 16];
    int n = 0;
    while (fgets(line, sizeof line, f)) {
        size_t k = strlen(line);
        while (k && (line[k - 1] == '\n' || line[k - 1] == '\r')) line[--k] = 0;
        if (!k) continue;
        fprintf(stderr, "[%d] %s\n", n++, line);
        ASTNode* a = parse(line);
        if (a) releaseNode(a);
    }
    fclose(f);
    return 0;
}
