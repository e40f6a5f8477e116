// Ingest A/B (host file bytes -> HBM) for the table upload (executor.hip upload()).
// Modes, each over the same page-cached file:
//   memcpy   mmap + P host threads memcpy into pinned 32 MiB chunks, async H2D (current)
//   pread    P host threads pread() into pinned 32 MiB chunks, async H2D
//   register hipHostRegister of the mmap'd file in chunks, H2D straight from them
// Build: hipcc -O2 -std=c++17 ingest.cpp -o ingest -lpthread ; run: ./ingest FILE [mode]
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const char* path = argv[1];
    std::string mode = argc > 2 ? argv[2] : "all";
    const size_t P = argc > 3 ? (size_t)atoi(argv[3]) : 8;
    const size_t CH = (argc > 4 ? (size_t)atoi(argv[4]) : 32) << 20;
    int fd = open(path, O_RDONLY);
    struct stat sb;
    fstat(fd, &sb);
    const size_t n = (size_t)sb.st_size;
    uint8_t* dev = nullptr;
    CK(hipMalloc(&dev, n + 4096));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    uint8_t* pin = nullptr;
    CK(hipHostMalloc((void**)&pin, 2 * P * CH, hipHostMallocDefault));
    hipEvent_t ev[2];
    CK(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
    const size_t nch = (n + CH - 1) / CH;
    auto run_staged = [&](bool use_pread) {
        const uint8_t* host = nullptr;
        void* m = nullptr;
        if (!use_pread) {
            m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
            madvise(m, n, MADV_SEQUENTIAL);
            host = (const uint8_t*)m;
        }
        for (size_t g0 = 0, grp = 0; g0 < nch; g0 += P, grp++) {
            uint8_t* base = pin + (grp & 1) * P * CH;
            if (grp >= 2) CK(hipEventSynchronize(ev[grp & 1]));
            const size_t gn = std::min(P, nch - g0);
            auto part = [&](size_t k) {
                const size_t off = (g0 + k) * CH, len = std::min(CH, n - off);
                if (use_pread) {
                    size_t got = 0;
                    while (got < len) {
                        ssize_t r = pread(fd, base + k * CH + got, len - got, (off_t)(off + got));
                        if (r <= 0) { perror("pread"); exit(1); }
                        got += (size_t)r;
                    }
                } else {
                    memcpy(base + k * CH, host + off, len);
                }
            };
            std::vector<std::thread> th;
            for (size_t k = 1; k < gn; k++) th.emplace_back(part, k);
            part(0);
            for (auto& x : th) x.join();
            for (size_t k = 0; k < gn; k++) {
                const size_t off = (g0 + k) * CH;
                CK(hipMemcpyAsync(dev + off, base + k * CH, std::min(CH, n - off), hipMemcpyHostToDevice, s));
            }
            CK(hipEventRecord(ev[grp & 1], s));
        }
        CK(hipStreamSynchronize(s));
        if (m) munmap(m, n);
    };
    auto run_register = [&](size_t RC) {
        void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        const uint8_t* host = (const uint8_t*)m;
        const size_t nr = (n + RC - 1) / RC;
        std::vector<void*> regd(nr, nullptr);
        // register chunk k+1 while chunk k copies
        auto reg = [&](size_t k) {
            const size_t off = k * RC, len = std::min(RC, n - off);
            hipError_t e = hipHostRegister((void*)(host + off), len, hipHostRegisterReadOnly);
            if (e != hipSuccess) { fprintf(stderr, "register: %s\n", hipGetErrorString(e)); exit(1); }
            regd[k] = (void*)(host + off);
        };
        reg(0);
        for (size_t k = 0; k < nr; k++) {
            const size_t off = k * RC, len = std::min(RC, n - off);
            CK(hipMemcpyAsync(dev + off, host + off, len, hipMemcpyHostToDevice, s));
            if (k + 1 < nr) reg(k + 1);
            CK(hipStreamSynchronize(s));
            CK(hipHostUnregister(regd[k]));
        }
        munmap(m, n);
    };
    // warm the page cache
    {
        std::vector<uint8_t> b(64 << 20);
        for (size_t off = 0; off < n; off += b.size()) (void)!pread(fd, b.data(), b.size(), (off_t)off);
    }
    for (int rep = 0; rep < 3; rep++) {
        if (mode == "all" || mode == "memcpy") {
            double t0 = now(); run_staged(false); double t = now() - t0;
            printf("memcpy   P=%zu CH=%zuMiB  %.3f s  %.1f GB/s\n", P, CH >> 20, t, n / t / 1e9);
        }
        if (mode == "all" || mode == "pread") {
            double t0 = now(); run_staged(true); double t = now() - t0;
            printf("pread    P=%zu CH=%zuMiB  %.3f s  %.1f GB/s\n", P, CH >> 20, t, n / t / 1e9);
        }
        if (mode == "all" || mode == "register") {
            for (size_t rc : {64ull << 20, 256ull << 20}) {
                double t0 = now(); run_register(rc); double t = now() - t0;
                printf("register RC=%zuMiB  %.3f s  %.1f GB/s\n", rc >> 20, t, n / t / 1e9);
            }
        }
        fflush(stdout);
    }
    return 0;
}
