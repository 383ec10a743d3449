// graph_memset_repro.hip — does a hipMemsetAsync captured into a hipGraph clear
// its target on every replay? (tools only; ADVICE r5: the root cause behind
// the engine's zero_words kernel, DESIGN.md §4.2 "No memset nodes in captured
// batches".)
//
// Mirrors the engine's dist batches: a graph = [memset of the batch's counter
// rows] + [a kernel that atomically adds into those rows], instantiated once and
// replayed; between replays the host poisons the rows with pointer-like words
// and runs other runtime work outside the graph (memsets and copies of other
// buffers, as the engine's resets and injection uploads do). After each replay
// every row must hold exactly the kernel's sums. Variants: the memset node (HIP's
// own fill) or our zero kernel in its place. Run two instances at once to mimic
// the 2-rank rehearsal (two processes on one GPU).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/graph_memset_repro tools/graph_memset_repro.hip
//   tools/graph_memset_repro [replays] [memset|kernel]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            exit(2);                                                             \
        }                                                                        \
    } while (0)

constexpr int kSlots = 64, kCounters = 32;  // the engine's counter row shape
constexpr size_t kRow = (size_t)kSlots * kCounters;

__global__ void add_counts(unsigned long long* c, int rounds) {
    // every block adds 1 to counter (blockIdx % 32) of slot (blockIdx % 64) of every round
    for (int r = 0; r < rounds; ++r)
        if (threadIdx.x == 0) atomicAdd(&c[r * kRow + (blockIdx.x % kSlots) * kCounters + blockIdx.x % kCounters], 1ull);
}

__global__ void zero_words(unsigned long long* p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = 0;
}

int main(int argc, char** argv) {
    const int replays = argc > 1 ? atoi(argv[1]) : 200;
    const bool use_memset = !(argc > 2 && std::string(argv[2]) == "kernel");
    const int rounds = 23, blocks = 4096, k0 = 5;  // a batch of 23 rounds at ring offset 5
    const size_t ring = 256 * kRow;
    unsigned long long *ctr, *other;
    CK(hipMalloc(&ctr, ring * 8));
    CK(hipMalloc(&other, 64 << 20));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned long long* rows = ctr + k0 * kRow;
    const size_t bytes = rounds * kRow * 8;
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    if (use_memset) {
        CK(hipMemsetAsync(rows, 0, bytes, s));
    } else {
        hipLaunchKernelGGL(zero_words, dim3(64), dim3(256), 0, s, rows, rounds * kRow);
    }
    hipLaunchKernelGGL(add_counts, dim3(blocks), dim3(64), 0, s, rows, rounds);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    std::vector<unsigned long long> want(rounds * kRow, 0), got(rounds * kRow);
    for (int b = 0; b < blocks; ++b)
        for (int r = 0; r < rounds; ++r) want[r * kRow + (b % kSlots) * kCounters + b % kCounters]++;
    std::vector<unsigned long long> poison(rounds * kRow);
    int bad_replays = 0;
    size_t bad_words = 0;
    for (int k = 0; k < replays; ++k) {
        for (size_t i = 0; i < poison.size(); ++i) poison[i] = 0x00007f0000000000ull + ((uint64_t)k << 20) + i * 8;
        CK(hipMemcpy(rows, poison.data(), bytes, hipMemcpyHostToDevice));
        // other runtime work outside the graph: fills and copies of another buffer
        CK(hipMemsetAsync(other, k & 0xff, (size_t)(1 + k % 7) << 20, s));
        CK(hipMemcpyAsync(other + (8 << 20) / 8, other, 1 << 20, hipMemcpyDeviceToDevice, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(got.data(), rows, bytes, hipMemcpyDeviceToHost));
        size_t bw = 0;
        for (size_t i = 0; i < got.size(); ++i) bw += got[i] != want[i];
        if (bw) {
            if (bad_replays < 5) {
                size_t i = 0;
                while (got[i] == want[i]) ++i;
                printf("replay %d: %zu words wrong, first at word %zu: got %#llx want %llu\n", k, bw, i, got[i], want[i]);
            }
            ++bad_replays;
            bad_words += bw;
        }
    }
    printf("%s node: %d of %d replays wrong (%zu words)\n", use_memset ? "hipMemsetAsync" : "zero kernel", bad_replays,
           replays, bad_words);
    return bad_replays ? 1 : 0;
}
