// Host-side AddressSanitizer driver for the dense merge (cqgpu_partial_*): the
// reference parser builds the plan, every "rank" is a range table of one file in
// this process, and the collectives are done by hand (an all-gather is a
// concatenation, the reductions run on the host).  Built by scripts/asan_dense.sh
// with -fsanitize=address on the host side only.
//   asan_dense FILE NRANKS "SQL" ["SQL" ...]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "cqgpu.h"

extern "C" void* parse(const char* sql);
extern "C" void releaseNode(void* node);

#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "hip error line %d\n", __LINE__); exit(3); } } while (0)

static int run(const char* path, int n, const char* sql) {
    void* ast = parse(sql);
    if (!ast) { fprintf(stderr, "parse failed\n"); return 1; }
    cq_csv_config cfg{',', '"', true};
    std::vector<cqgpu_table*> tabs(n);
    std::vector<cqgpu_partial*> parts(n);
    for (int r = 0; r < n; r++) tabs[r] = cqgpu_table_open_range(path, cfg, r, n);
    for (int r = 0; r < n; r++) {
        parts[r] = cqgpu_partial_new((cq_node*)ast, &tabs[r], 1);
        if (!parts[r]) { fprintf(stderr, "partial_new: %s\n", cqgpu_last_error()); return 1; }
    }
    std::vector<void*> results(n, nullptr);
    std::vector<uint64_t> sizes(n, 0);
    bool have_sizes = false;
    std::vector<void*> owned;
    int rc = 0;
    while (true) {
        std::vector<cqgpu_coll> co(n);
        for (int r = 0; r < n; r++)
            if (cqgpu_partial_next(parts[r], results[r], have_sizes ? sizes.data() : nullptr, r, n, &co[r]) != 0) {
                fprintf(stderr, "next: %s\n", cqgpu_last_error());
                return 1;
            }
        const int op = co[0].op;
        if (op == CQGPU_COLL_DONE) {
            cq_table* t = cqgpu_partial_result(parts[0], (cq_node*)ast);
            if (!t) { fprintf(stderr, "result: %s\n", cqgpu_last_error()); rc = 1; }
            else { printf("rows %d\n", t->nrows); cqgpu_result_free(t); }
            break;
        }
        if (op == CQGPU_COLL_DECLINE) { printf("declined\n"); break; }
        const size_t esz = op == CQGPU_COLL_ALLGATHER ? 1 : 8;
        std::vector<void*> bufs(n);
        for (int r = 0; r < n; r++) {
            CK(hipMalloc(&bufs[r], co[r].count * esz + 16));
            owned.push_back(bufs[r]);
            if (cqgpu_partial_put(parts[r], co[r].count ? bufs[r] : nullptr) != 0) {
                fprintf(stderr, "put: %s\n", cqgpu_last_error());
                return 1;
            }
        }
        CK(hipDeviceSynchronize());
        have_sizes = false;
        if (op == CQGPU_COLL_ALLGATHER) {
            uint64_t tot = 0;
            for (int r = 0; r < n; r++) { sizes[r] = co[r].count; tot += co[r].count; }
            void* cat;
            CK(hipMalloc(&cat, tot + 16));
            owned.push_back(cat);
            uint64_t at = 0;
            for (int r = 0; r < n; r++) {
                if (co[r].count) CK(hipMemcpy((char*)cat + at, bufs[r], co[r].count, hipMemcpyDeviceToDevice));
                at += co[r].count;
            }
            for (int r = 0; r < n; r++) results[r] = cat;
            have_sizes = true;
        } else {
            const uint64_t cnt = co[0].count;
            std::vector<std::vector<uint64_t>> h(n, std::vector<uint64_t>(cnt + 1));
            for (int r = 0; r < n; r++)
                if (cnt) CK(hipMemcpy(h[r].data(), bufs[r], cnt * 8, hipMemcpyDeviceToHost));
            std::vector<uint64_t> red(h[0]);
            for (int r = 1; r < n; r++)
                for (uint64_t i = 0; i < cnt; i++) {
                    if (op == CQGPU_COLL_ALLREDUCE_MIN_I64) {
                        if ((long long)h[r][i] < (long long)red[i]) red[i] = h[r][i];
                    } else if (op == CQGPU_COLL_REDUCE_SUM_I64) {
                        red[i] += h[r][i];
                    } else {
                        double a, b;
                        memcpy(&a, &red[i], 8);
                        memcpy(&b, &h[r][i], 8);
                        a += b;
                        memcpy(&red[i], &a, 8);
                    }
                }
            void* rb;
            CK(hipMalloc(&rb, cnt * 8 + 16));
            owned.push_back(rb);
            if (cnt) CK(hipMemcpy(rb, red.data(), cnt * 8, hipMemcpyHostToDevice));
            const bool to_all = op == CQGPU_COLL_ALLREDUCE_MIN_I64 || op == CQGPU_COLL_ALLREDUCE_SUM_F64;
            for (int r = 0; r < n; r++) results[r] = (r == 0 || to_all) ? rb : bufs[r];
        }
    }
    for (int r = 0; r < n; r++) cqgpu_partial_free(parts[r]);
    for (int r = 0; r < n; r++) cqgpu_table_free(tabs[r]);
    for (void* p : owned) CK(hipFree(p));
    releaseNode(ast);
    return rc;
}

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    int rc = 0;
    for (int i = 3; i < argc; i++) {
        fprintf(stderr, "[%d] %s\n", i - 3, argv[i]);
        rc |= run(argv[1], atoi(argv[2]), argv[i]);
    }
    printf("done rc=%d\n", rc);
    return rc;
}
