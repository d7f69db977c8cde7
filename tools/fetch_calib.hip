// fetch_calib.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE counters on gfx950 for the access
// classes of the pull kernel k_bu (VERDICT r2 "pin the traffic figure").  Every kernel below touches an
// EXACTLY known set of 64-B lines, far more than the Infinity Cache holds, so the counter's report per
// kernel divided by the known bytes is the correction factor for that class:
//   k_stream8    coalesced 8-B loads, lane-consecutive (k_finalize's / the visited words' pattern)
//   k_rand4      scattered 4-B loads, one per distinct line (top1 of sparse candidates, frontier probes)
//   k_rand8      scattered 8-B loads, one per distinct line (state words)
//   k_rand16     scattered 16-B loads, one per distinct line (rest[v])
//   k_rand4x2    scattered 4-B loads, two per line (the two words of one line from two lanes)
//   k_store8     scattered 8-B stores, one per distinct line (the state stores of found vertices)
//   k_wstream8   coalesced 8-B stores
// Lines are chosen by a bijection (odd multiplier mod 2^k) of the access index, so no line is touched
// twice.  Build: hipcc -O3 --offload-arch=gfx950 -o tools/fetch_calib tools/fetch_calib.hip
// Run: rocprofv3 --pmc FETCH_SIZE -- tools/fetch_calib  (and WRITE_SIZE in a pass of its own); the
// program prints the known bytes per kernel; tools/fetch_calib_summary.py joins them with the counters.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                            \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) {                                                                          \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));            \
            exit(1);                                                                                     \
        }                                                                                                \
    } while (0)

using u64 = unsigned long long;
constexpr u64 kMul = 0x9E3779B97F4A7C15ull | 1ull; // odd: i -> i * kMul mod 2^k is a bijection

__device__ inline u64 line_of(u64 i, u64 lines_mask) { return (i * kMul) & lines_mask; }

__global__ void k_stream8(const u64 *__restrict__ a, u64 n, u64 *__restrict__ sink) {
    u64 acc = 0;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) acc ^= a[i];
    if (acc == 0x1234567ull) sink[0] = acc;
}
__global__ void k_rand4(const unsigned *__restrict__ a, u64 r, u64 lines_mask, u64 *__restrict__ sink) {
    unsigned acc = 0;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < r; i += (u64)gridDim.x * blockDim.x)
        acc ^= a[line_of(i, lines_mask) * 16 + (i & 15)];
    if (acc == 0x1234567u) sink[0] = acc;
}
__global__ void k_rand4x2(const unsigned *__restrict__ a, u64 r, u64 lines_mask, u64 *__restrict__ sink) {
    unsigned acc = 0;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < r; i += (u64)gridDim.x * blockDim.x)
        acc ^= a[line_of(i >> 1, lines_mask) * 16 + (i & 1) * 8]; // lanes 2k, 2k+1 share a line
    if (acc == 0x1234567u) sink[0] = acc;
}
__global__ void k_rand8(const u64 *__restrict__ a, u64 r, u64 lines_mask, u64 *__restrict__ sink) {
    u64 acc = 0;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < r; i += (u64)gridDim.x * blockDim.x)
        acc ^= a[line_of(i, lines_mask) * 8 + (i & 7)];
    if (acc == 0x1234567ull) sink[0] = acc;
}
__global__ void k_rand16(const uint4 *__restrict__ a, u64 r, u64 lines_mask, u64 *__restrict__ sink) {
    unsigned acc = 0;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < r; i += (u64)gridDim.x * blockDim.x) {
        const uint4 x = a[line_of(i, lines_mask) * 4 + (i & 3)];
        acc ^= x.x ^ x.y ^ x.z ^ x.w;
    }
    if (acc == 0x1234567u) sink[0] = acc;
}
__global__ void k_store8(u64 *__restrict__ a, u64 r, u64 lines_mask) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < r; i += (u64)gridDim.x * blockDim.x)
        a[line_of(i, lines_mask) * 8 + (i & 7)] = i;
}
__global__ void k_wstream8(u64 *__restrict__ a, u64 n) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) a[i] = i;
}

int main(int argc, char **argv) {
    const int lines_log = argc > 1 ? atoi(argv[1]) : 27; // 2^27 lines of 64 B = 8 GiB, 32x the Infinity Cache
    const u64 lines = 1ull << lines_log, mask = lines - 1;
    const u64 bytes = lines * 64;
    const u64 r = lines / 8;         // scattered accesses per kernel: distinct lines, 1/8 of the array's
    const u64 stream = 1ull << 28;   // coalesced words (2 GiB)
    void *buf = nullptr;
    u64 *sink = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 1, bytes));
    CK(hipDeviceSynchronize());
    const dim3 grid(8192), block(256);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("{\"lines_log\": %d, \"array_bytes\": %llu, \"kernels\": {\n", lines_log, bytes);
    auto run = [&](const char *name, u64 known_read, u64 known_write, auto launch, bool last = false) {
        launch(); // warm (page tables), then the measured launch
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("  \"%s\": {\"launches\": 2, \"known_read_bytes_per_launch\": %llu, \"known_write_bytes_per_launch\": %llu, "
               "\"ms\": %.4f}%s\n", name, known_read, known_write, ms, last ? "" : ",");
    };
    run("k_stream8", stream * 8, 0, [&] { hipLaunchKernelGGL(k_stream8, grid, block, 0, 0, (const u64 *)buf, stream, sink); });
    run("k_rand4", r * 64, 0, [&] { hipLaunchKernelGGL(k_rand4, grid, block, 0, 0, (const unsigned *)buf, r, mask, sink); });
    run("k_rand4x2", r * 64, 0,
        [&] { hipLaunchKernelGGL(k_rand4x2, grid, block, 0, 0, (const unsigned *)buf, 2 * r, mask, sink); });
    run("k_rand8", r * 64, 0, [&] { hipLaunchKernelGGL(k_rand8, grid, block, 0, 0, (const u64 *)buf, r, mask, sink); });
    run("k_rand16", r * 64, 0, [&] { hipLaunchKernelGGL(k_rand16, grid, block, 0, 0, (const uint4 *)buf, r, mask, sink); });
    run("k_store8", 0, r * 64, [&] { hipLaunchKernelGGL(k_store8, grid, block, 0, 0, (u64 *)buf, r, mask); });
    run("k_wstream8", 0, stream * 8, [&] { hipLaunchKernelGGL(k_wstream8, grid, block, 0, 0, (u64 *)buf, stream); },
        true);
    printf("}}\n");
    CK(hipGetLastError());
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
