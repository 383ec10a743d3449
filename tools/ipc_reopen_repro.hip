// ipc_reopen_repro.hip — which hipIpcOpenMemHandle sequences return, between
// two processes on one GPU? (tools only; the root cause behind the 8-rank
// stall of round 5: DESIGN.md §5.4.) The parent forks before any HIP call; the
// child exports windows, the parent imports them; handles travel over pipes.
// Every step of the parent runs under a watchdog: a step that does not return
// within 20 s is reported and the process exits (the wait is on the host, in
// the runtime; the GPU runs nothing here).
//   1  open a handle, close it, open the same handle again
//   2  the exporter frees the window and allocates a new one of the same size
//      (same address: the allocator reuses it) after the importer closed its
//      mapping; open the new handle
//   3  as 2, but the exporter frees while the importer still maps the old
//      window (no barrier), then the importer closes and opens the new handle
//   4  as 3 with a window of another size (another address)
//   5-7 both processes export and map each other's windows, twice (both() below)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ipc_reopen_repro tools/ipc_reopen_repro.hip
//   tools/ipc_reopen_repro SCENARIO   (exit 1: an open hung)
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            _exit(2);                                                            \
        }                                                                        \
    } while (0)

static int c2p[2], p2c[2];  // child -> parent: handles + addresses; parent -> child: step acks

static void send_all(int fd, const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    while (n) {
        ssize_t k = write(fd, c, n);
        if (k <= 0) _exit(3);
        c += k;
        n -= (size_t)k;
    }
}
static void recv_all(int fd, void* p, size_t n) {
    char* c = static_cast<char*>(p);
    while (n) {
        ssize_t k = read(fd, c, n);
        if (k <= 0) _exit(3);
        c += k;
        n -= (size_t)k;
    }
}

struct Msg {
    hipIpcMemHandle_t h;
    unsigned long long addr;
};

static int g_scn = 1;

// scenario 13: kernels store into the peer's mapped window (and read their own)
// before the second window is exported and mapped
__global__ void touch(unsigned long long* peer, const unsigned long long* own, size_t n, unsigned long long v) {
    unsigned long long acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        peer[i] = v + i;
        acc += own[i];
    }
    __threadfence_system();
    if (acc == 0x5a5a5a5a5a5a5a5aull) peer[0] = acc;  // (keeps the loads)
}
static std::atomic<int> g_step{0};

static void watchdog(int who) {
    std::thread([who] {  // a step that does not return in 20 s
        int last = -1;
        auto t = std::chrono::steady_clock::now();
        for (;;) {
            std::this_thread::sleep_for(std::chrono::milliseconds(200));
            const int s = g_step.load();
            if (s < 0) return;
            if (s == 0) continue;  // (runtime start-up is not timed)
            if (s != last) {
                last = s;
                t = std::chrono::steady_clock::now();
            } else if (std::chrono::steady_clock::now() - t > std::chrono::seconds(20)) {
                printf("[%d] scenario %d step %d: did not return within 20 s (HANG)\n", who, g_scn, s);
                fflush(stdout);
                _exit(1);
            }
        }
    }).detach();
}

// Scenarios 1-4: the child exports, the parent imports (one direction).
static void child() {
    CK(hipSetDevice(0));
    const size_t a = 64ull << 20, b = 96ull << 20;
    void* w = nullptr;
    Msg m{};
    char ack;
    auto export_new = [&](size_t bytes) {
        CK(hipExtMallocWithFlags(&w, bytes, hipDeviceMallocUncached));
        CK(hipMemset(w, 0, bytes));
        CK(hipIpcGetMemHandle(&m.h, w));
        m.addr = (unsigned long long)w;
        send_all(c2p[1], &m, sizeof m);
    };
    export_new(a);
    recv_all(p2c[0], &ack, 1);  // the parent opened it (1: and closed, and opened again)
    if (g_scn >= 2) {
        CK(hipFree(w));         // 2: after the importer closed; 3, 4: while it still maps it
        export_new(g_scn == 4 ? b : a);
        recv_all(p2c[0], &ack, 1);
    }
    CK(hipFree(w));
}

static void parent() {
    watchdog(0);
    CK(hipSetDevice(0));
    Msg m{};
    void* p = nullptr;
    const char ack = 1;
    auto open_ = [&](int step, const char* what) {
        g_step = step;
        printf("scenario %d step %d: %s (exporter window at %#llx) ...\n", g_scn, step, what, m.addr);
        fflush(stdout);
        CK(hipIpcOpenMemHandle(&p, m.h, hipIpcMemLazyEnablePeerAccess));
        printf("scenario %d step %d: opened at %p\n", g_scn, step, p);
        fflush(stdout);
    };
    recv_all(c2p[0], &m, sizeof m);
    open_(1, "open");
    if (g_scn == 1) {
        CK(hipIpcCloseMemHandle(p));
        open_(2, "open the same handle again after closing it");
    } else if (g_scn == 2) {
        CK(hipIpcCloseMemHandle(p));
        send_all(p2c[1], &ack, 1);
        recv_all(c2p[0], &m, sizeof m);
        open_(2, "open the new window the exporter allocated after our close");
    } else {
        void* old = p;
        send_all(p2c[1], &ack, 1);
        recv_all(c2p[0], &m, sizeof m);
        open_(2, g_scn == 3 ? "open the new window (same size) while the freed old one is still mapped here"
                            : "open the new window (another size) while the freed old one is still mapped here");
        CK(hipIpcCloseMemHandle(old));
    }
    CK(hipIpcCloseMemHandle(p));
    send_all(p2c[1], &ack, 1);
    g_step = -1;
    printf("scenario %d: every open returned\n", g_scn);
}

// Scenarios 5-7: both processes export a window and map the other's (the
// engines' exchange), twice:
//   5  unmap, barrier, free, allocate a new window, export, map again (the
//      collective teardown, then the next bench leg)
//   6  unmap and free with no barrier in between, then as 5 (round 5's bench)
//   7  unmap, barrier, export the SAME window again (hipIpcGetMemHandle once
//      more) and map again (an engine re-importing after gg_dist_ipc_close)
//   8  a second, larger window beside the first (nothing unmapped or freed):
//      export, map (a window pool that only grows)
//   9  export the same window again while the peer still maps it; the peer maps
//      the new handle too
//   10 a second window of REPRO_GB GiB (default 8) beside the first: export, both map at once
//   11 as 10, the two processes mapping in turn (process 0, then 1)
//   12 one window of REPRO_GB GiB (or REPRO_BYTES bytes), nothing before it: export, both map at once
//   13 kernels store into the first mapped window (50 launches), then as 10
//   14 REPRO_FILL_GB (default 80) of other device allocations first, then as 12
//   15 REPRO_TEMP_GB (default 24) of temporaries allocated, written and freed first, then as 12
// REPRO_CACHED=1: windows from hipMalloc instead of hipExtMallocWithFlags(uncached).
static void both(int who) {
    const int tx = who ? c2p[1] : p2c[1], rx = who ? p2c[0] : c2p[0];
    watchdog(who);
    CK(hipSetDevice(0));
    const size_t a = 64ull << 20;
    void* w = nullptr;
    void* peer = nullptr;
    Msg mine{}, theirs{};
    const char ack = 1;
    char got;
    auto barrier = [&]() {
        send_all(tx, &ack, 1);
        recv_all(rx, &got, 1);
    };
    auto exchange_and_open = [&](int step) {
        CK(hipIpcGetMemHandle(&mine.h, w));
        mine.addr = (unsigned long long)w;
        send_all(tx, &mine, sizeof mine);
        recv_all(rx, &theirs, sizeof theirs);
        g_step = step;
        printf("[%d] scenario %d step %d: open the peer's window %#llx ...\n", who, g_scn, step, theirs.addr);
        fflush(stdout);
        CK(hipIpcOpenMemHandle(&peer, theirs.h, hipIpcMemLazyEnablePeerAccess));
        printf("[%d] scenario %d step %d: opened at %p\n", who, g_scn, step, peer);
        fflush(stdout);
    };
    const bool uncached = !(getenv("REPRO_CACHED") && *getenv("REPRO_CACHED"));  // REPRO_CACHED=1: plain hipMalloc windows
    auto alloc = [&](void** q, size_t n) {
        if (uncached) CK(hipExtMallocWithFlags(q, n, hipDeviceMallocUncached));
        else CK(hipMalloc(q, n));
        CK(hipMemset(*q, 0, n));
    };
    if (g_scn == 15) {  // REPRO_TEMP_GB of temporaries allocated, written, freed first (then as 12)
        const double tg = getenv("REPRO_TEMP_GB") ? atof(getenv("REPRO_TEMP_GB")) : 24.0;
        std::vector<void*> tmp;
        for (double got = 0; got < tg; got += 4.0) {
            void* x = nullptr;
            CK(hipMalloc(&x, 4ull << 30));
            CK(hipMemset(x, 7, 4ull << 30));
            tmp.push_back(x);
        }
        CK(hipDeviceSynchronize());
        for (void* x : tmp) CK(hipFree(x));
        printf("[%d] scenario 15: %.0f GiB of temporaries allocated and freed\n", who, tg);
        fflush(stdout);
        g_scn = 12;
    }
    if (g_scn == 14) {  // REPRO_FILL_GB of other allocations (2 GiB chunks) first, then as 12
        const double fill = getenv("REPRO_FILL_GB") ? atof(getenv("REPRO_FILL_GB")) : 80.0;
        const double chunk = getenv("REPRO_CHUNK_MB") ? atof(getenv("REPRO_CHUNK_MB")) : 2048.0;
        const size_t cb = (size_t)(chunk * (1 << 20));
        for (double got = 0; got < fill; got += chunk / 1024.0) {
            void* x = nullptr;
            CK(hipMalloc(&x, cb));
            CK(hipMemset(x, 1, cb));
        }
        printf("[%d] scenario 14: %.0f GiB allocated\n", who, fill);
        fflush(stdout);
        g_scn = 12;
    }
    if (g_scn == 12) {
        size_t big = (size_t)((getenv("REPRO_GB") ? atof(getenv("REPRO_GB")) : 8.0) * (1ull << 30));
        if (getenv("REPRO_BYTES")) big = strtoull(getenv("REPRO_BYTES"), nullptr, 10);  // an exact size
        printf("[%d] scenario 12: window of %zu bytes\n", who, big);
        alloc(&w, big);
        const auto t0 = std::chrono::steady_clock::now();
        exchange_and_open(1);
        printf("[%d] scenario 12: %.3f s\n", who,
               std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        barrier();
        CK(hipIpcCloseMemHandle(peer));
        barrier();
        CK(hipFree(w));
        g_step = -1;
        printf("[%d] scenario %d: every open returned\n", who, g_scn);
        return;
    }
    alloc(&w, a);
    exchange_and_open(1);
    barrier();
    if (g_scn == 13) {  // kernels use the first mapping, then a second window (REPRO_GB GiB)
        for (int k = 0; k < 50; ++k)
            hipLaunchKernelGGL(touch, dim3(256), dim3(256), 0, 0, (unsigned long long*)peer,
                               (const unsigned long long*)w, a / 8, (unsigned long long)k);
        CK(hipDeviceSynchronize());
        barrier();
        g_scn = 10;  // then as scenario 10
    }
    if (g_scn == 10 || g_scn == 11) {  // a second window of REPRO_GB GiB beside the first (11: opens in turn)
        const size_t big = (size_t)(getenv("REPRO_GB") ? atof(getenv("REPRO_GB")) : 8.0) * (1ull << 30);
        void* w1 = w;
        void* p1 = peer;
        alloc(&w, big);
        CK(hipIpcGetMemHandle(&mine.h, w));
        mine.addr = (unsigned long long)w;
        send_all(tx, &mine, sizeof mine);
        recv_all(rx, &theirs, sizeof theirs);
        for (int turn = 0; turn < 2; ++turn) {
            if (g_scn == 11 && turn != who) {
                barrier();
                continue;
            }
            if (g_scn == 10 && turn == 1) break;
            g_step = 2;
            printf("[%d] scenario %d step 2: open the peer's %.1f GiB window %#llx ...\n", who, g_scn,
                   big / 1073741824.0, theirs.addr);
            fflush(stdout);
            const auto t0 = std::chrono::steady_clock::now();
            CK(hipIpcOpenMemHandle(&peer, theirs.h, hipIpcMemLazyEnablePeerAccess));
            printf("[%d] scenario %d step 2: opened at %p in %.3f s\n", who, g_scn, peer,
                   std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
            fflush(stdout);
            if (g_scn == 11) barrier();
        }
        barrier();
        CK(hipIpcCloseMemHandle(peer));
        CK(hipIpcCloseMemHandle(p1));
        barrier();
        CK(hipFree(w));
        CK(hipFree(w1));
        g_step = -1;
        printf("[%d] scenario %d: every open returned\n", who, g_scn);
        return;
    }
    if (g_scn == 8) {  // a second window beside the first (nothing unmapped or freed): export, map
        void* w1 = w;
        void* p1 = peer;
        alloc(&w, 2 * a);
        exchange_and_open(2);
        barrier();
        CK(hipIpcCloseMemHandle(peer));
        CK(hipIpcCloseMemHandle(p1));
        barrier();
        CK(hipFree(w));
        CK(hipFree(w1));
        g_step = -1;
        printf("[%d] scenario %d: every open returned\n", who, g_scn);
        return;
    }
    if (g_scn == 9) {  // export the same window again while the peer still maps it; the peer maps it again
        void* p1 = peer;
        exchange_and_open(2);
        barrier();
        CK(hipIpcCloseMemHandle(peer));
        CK(hipIpcCloseMemHandle(p1));
        barrier();
        CK(hipFree(w));
        g_step = -1;
        printf("[%d] scenario %d: every open returned\n", who, g_scn);
        return;
    }
    if (g_scn == 5) {
        CK(hipIpcCloseMemHandle(peer));
        barrier();
        CK(hipFree(w));
        alloc(&w, a);
    } else if (g_scn == 6) {
        CK(hipIpcCloseMemHandle(peer));
        CK(hipFree(w));
        alloc(&w, a);
    } else {
        CK(hipIpcCloseMemHandle(peer));
        barrier();
    }
    exchange_and_open(2);
    barrier();
    CK(hipIpcCloseMemHandle(peer));
    barrier();
    CK(hipFree(w));
    g_step = -1;
    printf("[%d] scenario %d: every open returned\n", who, g_scn);
}

int main(int argc, char** argv) {
    g_scn = argc > 1 ? atoi(argv[1]) : 1;
    if (pipe(c2p) || pipe(p2c)) return 2;
    const pid_t pid = fork();  // before any HIP call in either process
    if (pid < 0) return 2;
    if (pid == 0) {
        if (g_scn >= 5) both(1);
        else child();
        _exit(0);
    }
    if (g_scn >= 5) both(0);
    else parent();
    int st = 0;
    waitpid(pid, &st, 0);
    return 0;
}
