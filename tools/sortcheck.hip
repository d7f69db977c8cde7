// Standalone check of rocprim::radix_sort_pairs at n = 2^30 (u32 keys ~deg-like, u32 ids): is the output
// a permutation of the ids, sorted by key, ties by id?  Default config vs a power-of-two block config.
//   hipcc -O2 --offload-arch=gfx950 -std=c++17 tools/sortcheck.hip -o tools/sortcheck && ./tools/sortcheck 30
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>

__global__ void k_keys(uint32_t *k, uint32_t *id, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t x = i * 0x9E3779B97F4A7C15ull;
        x ^= x >> 29;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 32;
        k[i] = ~(uint32_t)(__builtin_ctzll(x | (1ull << 40)) * 3 + (x & 3)); // few distinct keys, many ties
        id[i] = (uint32_t)i;
    }
}
__global__ void k_check(const uint32_t *k, const uint32_t *id, size_t n, unsigned long long *bad, uint32_t *seen) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        if (id[i] >= n) { atomicAdd(bad, 1ull); continue; }
        atomicAdd(&seen[id[i]], 1u);
        if (i > 0 && (k[i - 1] > k[i] || (k[i - 1] == k[i] && id[i - 1] >= id[i]))) atomicAdd(bad + 1, 1ull);
    }
}
__global__ void k_seen(const uint32_t *seen, size_t n, unsigned long long *bad) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (seen[i] != 1u) atomicAdd(bad + 2, 1ull);
}

using Pow2Cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                           rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>,
                                                                               rocprim::kernel_config<1024, 8>, 8, rocprim::block_radix_rank_algorithm::match>>;

template <class Cfg>
int run(size_t n, const char *name) {
    uint32_t *k, *id, *k2, *id2, *seen;
    unsigned long long *bad;
    hipMalloc(&k, n * 4); hipMalloc(&id, n * 4); hipMalloc(&k2, n * 4); hipMalloc(&id2, n * 4);
    hipMalloc(&seen, n * 4); hipMalloc(&bad, 24);
    k_keys<<<8192, 256>>>(k, id, n);
    size_t tb = 0;
    rocprim::radix_sort_pairs<Cfg>(nullptr, tb, k, k2, id, id2, n, 0, 32, 0);
    void *tmp; hipMalloc(&tmp, tb);
    hipError_t e = rocprim::radix_sort_pairs<Cfg>(tmp, tb, k, k2, id, id2, n, 0, 32, 0);
    hipMemset(seen, 0, n * 4); hipMemset(bad, 0, 24);
    k_check<<<8192, 256>>>(k2, id2, n, bad, seen);
    k_seen<<<8192, 256>>>(seen, n, bad);
    unsigned long long h[3];
    hipMemcpy(h, bad, 24, hipMemcpyDeviceToHost);
    printf("%s n=%zu err=%d out_of_range=%llu order=%llu not_once=%llu\n", name, n, (int)e, h[0], h[1], h[2]);
    hipFree(k); hipFree(id); hipFree(k2); hipFree(id2); hipFree(seen); hipFree(bad); hipFree(tmp);
    return (h[0] | h[1] | h[2]) ? 1 : 0;
}

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 30;
    int rc = 0;
    for (int s = 26; s <= lg; s += 2) {
        rc |= run<rocprim::default_config>((size_t)1 << s, "default");
        rc |= run<Pow2Cfg>((size_t)1 << s, "pow2   ");
    }
    return rc;
}
