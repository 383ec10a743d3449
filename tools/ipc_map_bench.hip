// How long hipIpcOpenMemHandle takes for a window of a given size and kind
// (uncached device memory, as gg_dist_ipc_export allocates, or plain hipMalloc),
// between two processes on one GPU. Usage:
//   ipc_map_bench export <GiB> <uncached 0|1>   -> prints the handle (hex), waits for a line on stdin
//   ipc_map_bench import <hex>                  -> opens it, prints the time, writes+reads a word
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    if (!std::strcmp(argv[1], "exports")) {  // exports <uncached> <GiB>...: one window after another
        const bool uc = std::atoi(argv[2]);
        for (int k = 3; k < argc; ++k) {
            const size_t bytes = (size_t)(std::atof(argv[k]) * (1ull << 30));
            void* p = nullptr;
            if (uc) CK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
            else CK(hipMalloc(&p, bytes));
            CK(hipMemset(p, 0, bytes));
            CK(hipDeviceSynchronize());
            hipIpcMemHandle_t h;
            CK(hipIpcGetMemHandle(&h, p));
            for (size_t i = 0; i < sizeof(h); ++i) std::printf("%02x", ((unsigned char*)&h)[i]);
            std::printf("\n");
            std::fflush(stdout);
            char line[64];
            if (!std::fgets(line, sizeof line, stdin)) return 0;
            CK(hipFree(p));
            std::fprintf(stderr, "exporter: freed window %d (%.2f GiB)\n", k - 2, bytes / double(1ull << 30));
        }
        return 0;
    }
    if (!std::strcmp(argv[1], "imports")) {  // imports <n>: n handles from stdin, each opened, touched, closed
        CK(hipSetDevice(0));
        CK(hipFree(nullptr));
        for (int k = 0; k < std::atoi(argv[2]); ++k) {
            char hex[256];
            if (!std::fgets(hex, sizeof hex, stdin)) return 3;
            hipIpcMemHandle_t h;
            for (size_t i = 0; i < sizeof(h); ++i) {
                unsigned v = 0;
                std::sscanf(hex + 2 * i, "%2x", &v);
                ((unsigned char*)&h)[i] = (unsigned char)v;
            }
            void* q = nullptr;
            auto t0 = std::chrono::steady_clock::now();
            CK(hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess));
            auto t1 = std::chrono::steady_clock::now();
            unsigned long long v = 0x1234;
            CK(hipMemcpy(q, &v, 8, hipMemcpyHostToDevice));
            CK(hipIpcCloseMemHandle(q));
            std::printf("import %d: open %.3f s\n", k, std::chrono::duration<double>(t1 - t0).count());
            std::fflush(stdout);
            std::fprintf(stderr, "next\n");
        }
        return 0;
    }
    if (!std::strcmp(argv[1], "export")) {
        const size_t bytes = (size_t)(std::atof(argv[2]) * (1ull << 30));
        const bool uc = argc > 3 && std::atoi(argv[3]);
        void* p = nullptr;
        auto t0 = std::chrono::steady_clock::now();
        if (uc) CK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
        else CK(hipMalloc(&p, bytes));
        CK(hipMemset(p, 0, bytes));
        CK(hipDeviceSynchronize());
        auto t1 = std::chrono::steady_clock::now();
        hipIpcMemHandle_t h;
        CK(hipIpcGetMemHandle(&h, p));
        std::string hex;
        for (size_t i = 0; i < sizeof(h); ++i) {
            char b[3];
            std::snprintf(b, 3, "%02x", ((unsigned char*)&h)[i]);
            hex += b;
        }
        std::printf("%s\n", hex.c_str());
        std::fflush(stdout);
        std::fprintf(stderr, "export: %.2f GiB %s, alloc+memset %.3f s\n", bytes / double(1ull << 30),
                     uc ? "uncached" : "hipMalloc", std::chrono::duration<double>(t1 - t0).count());
        char line[64];
        if (!std::fgets(line, sizeof line, stdin)) return 0;
        CK(hipFree(p));
        return 0;
    }
    hipIpcMemHandle_t h;
    const char* hex = argv[2];
    for (size_t i = 0; i < sizeof(h); ++i) {
        unsigned v = 0;
        std::sscanf(hex + 2 * i, "%2x", &v);
        ((unsigned char*)&h)[i] = (unsigned char)v;
    }
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    void* q = nullptr;
    auto t0 = std::chrono::steady_clock::now();
    CK(hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess));
    auto t1 = std::chrono::steady_clock::now();
    unsigned long long v = 0x1234;
    CK(hipMemcpy(q, &v, 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(&v, q, 8, hipMemcpyDeviceToHost));
    auto t2 = std::chrono::steady_clock::now();
    CK(hipIpcCloseMemHandle(q));
    auto t3 = std::chrono::steady_clock::now();
    std::printf("import: open %.3f s, first access %.3f s, close %.3f s (%llx)\n",
                std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count(),
                std::chrono::duration<double>(t3 - t2).count(), v);
    return 0;
}
