// Standalone check of rocprim::segmented_radix_sort_keys with very many tiny segments (the tail chunk of a
// relabelled CSR build: hundreds of millions of rows of degree 1..7).  Per segment: sorted, and the key sum
// and xor preserved.   hipcc -O2 --offload-arch=gfx950 -std=c++17 tools/segsortcheck.hip -o tools/segsortcheck
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>

__device__ inline uint64_t mix(uint64_t x) {
    x *= 0x9E3779B97F4A7C15ull;
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    return x ^ (x >> 32);
}
__global__ void k_len(int64_t *len, int64_t rows) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r <= rows; r += (int64_t)gridDim.x * blockDim.x)
        len[r] = r < rows ? 1 + (int64_t)(mix(r) % 7) : 0;
}
__global__ void k_fill(const int64_t *off, int64_t rows, uint32_t *k, unsigned long long *sums) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
        for (int64_t j = off[r]; j < off[r + 1]; j++) {
            k[j] = (uint32_t)(mix(j + 12345) & 0x3FFFFFFF);
            atomicAdd(sums, (unsigned long long)k[j] * (unsigned long long)(r % 1000 + 1));
        }
    }
}
__global__ void k_verify(const int64_t *off, int64_t rows, const uint32_t *k, unsigned long long *sums) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
        for (int64_t j = off[r]; j < off[r + 1]; j++) {
            atomicAdd(sums + 1, (unsigned long long)k[j] * (unsigned long long)(r % 1000 + 1));
            if (j > off[r] && k[j - 1] > k[j]) atomicAdd(sums + 2, 1ull);
        }
    }
}

struct Sub {
    int64_t b;
    __host__ __device__ int64_t operator()(int64_t x) const { return x - b; }
};

int main(int argc, char **argv) {
    const int64_t rows = argc > 1 ? atoll(argv[1]) : (int64_t)1 << 28;
    int64_t *len, *off;
    hipMalloc(&len, (rows + 1) * 8);
    hipMalloc(&off, (rows + 1) * 8);
    k_len<<<8192, 256>>>(len, rows);
    size_t tb = 0;
    rocprim::exclusive_scan(nullptr, tb, len, off, (int64_t)0, (size_t)(rows + 1), rocprim::plus<int64_t>());
    void *tmp;
    hipMalloc(&tmp, tb);
    rocprim::exclusive_scan(tmp, tb, len, off, (int64_t)0, (size_t)(rows + 1), rocprim::plus<int64_t>());
    hipFree(tmp);
    int64_t n = 0;
    hipMemcpy(&n, off + rows, 8, hipMemcpyDeviceToHost);
    uint32_t *k, *k2;
    unsigned long long *s;
    hipMalloc(&k, n * 4);
    hipMalloc(&k2, n * 4);
    hipMalloc(&s, 24);
    hipMemset(s, 0, 24);
    k_fill<<<8192, 256>>>(off, rows, k, s);
    tb = 0;
    hipError_t e = rocprim::segmented_radix_sort_keys(nullptr, tb, k, k2, (unsigned)n, (unsigned)rows, off, off + 1, 0, 30);
    hipMalloc(&tmp, tb);
    e = rocprim::segmented_radix_sort_keys(tmp, tb, k, k2, (unsigned)n, (unsigned)rows, off, off + 1, 0, 30);
    k_verify<<<8192, 256>>>(off, rows, k2, s);
    unsigned long long h[3];
    hipMemcpy(h, s, 24, hipMemcpyDeviceToHost);
    printf("rows=%lld n=%lld err=%d sum_in=%llu sum_out=%llu unsorted=%llu -> %s\n", (long long)rows, (long long)n,
           (int)e, h[0], h[1], h[2], (h[0] == h[1] && !h[2]) ? "OK" : "BAD");
    return (h[0] == h[1] && !h[2]) ? 0 : 1;
}
