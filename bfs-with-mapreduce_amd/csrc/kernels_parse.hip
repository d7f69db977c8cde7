// kernels_parse.hip -- K0: the algs4 edge-list tokenizer on the GPU (gfx950).
//
// Replaces the per-line parse of GraphFileUtil.convert (GraphFileUtil.java:60-66): every line after the
// two header lines is split on single spaces (String.split(" ")), tokens 0 and 1 are parsed with
// Integer.parseInt rules and must name a vertex in [0, V).  The host parser (bfsx_parse_algs4) reads
// one line at a time; here the file body is copied to the device once and
//   1. line starts are found by a rocPRIM select over "byte i starts a line" (BufferedReader.readLine
//      terminators: "\n", "\r", "\r\n"; no empty line after a final terminator);
//   2. one thread per line parses its two tokens, writing the tuple in place (u[line], v[line]);
//   3. the first bad line in file order (an atomicMin over (line, code)) reproduces the host parser's
//      error -- the same code (E_PARSE before E_RANGE within a line) and the same line number.
// Tokens follow Integer.parseInt, Unicode decimal digits included (java_digits.h).
// The tuples stay on the device for the CSR build: a 7.6 M-edge file is ~100 MB of text but 61 MB of
// tuples that no longer cross PCIe.
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include "bfsx_internal.h"
#include "java_digits.h"

namespace bfsx {

namespace {

constexpr int kBS = 256;

struct LineStart {
    const char *b;
    __host__ __device__ uint8_t operator()(int64_t i) const {
        if (i == 0) return 1;
        const char p = b[i - 1];
        return (p == '\n' || (p == '\r' && b[i] != '\n')) ? 1 : 0;
    }
};

constexpr unsigned long long kErrParse = 1, kErrRange = 2;

__global__ __launch_bounds__(kBS) void k_parse_lines(const char *__restrict__ b, int64_t n,
                                                     const int64_t *__restrict__ starts, int64_t m, int64_t nv,
                                                     uint32_t *__restrict__ u, uint32_t *__restrict__ v,
                                                     unsigned long long *err) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < m; i += (int64_t)gridDim.x * kBS) {
        const int64_t s = starts[i];
        int64_t e = s;
        while (e < n && b[e] != '\n' && b[e] != '\r') e++;
        int64_t sp = s;
        while (sp < e && b[sp] != ' ') sp++;
        unsigned long long code = 0;
        int64_t a = 0, c = 0;
        if (sp == e) {
            code = kErrParse; // one token: index 1 out of bounds
        } else {
            int64_t sp2 = sp + 1;
            while (sp2 < e && b[sp2] != ' ') sp2++;
            const unsigned char *ub = reinterpret_cast<const unsigned char *>(b);
            if (!java_parse_int(ub, s, sp, a) || !java_parse_int(ub, sp + 1, sp2, c)) code = kErrParse;
            else if (a < 0 || a >= nv || c < 0 || c >= nv) code = kErrRange;
        }
        if (code) {
            atomicMin(err, ((unsigned long long)i << 2) | code);
        } else {
            u[i] = (uint32_t)a;
            v[i] = (uint32_t)c;
        }
    }
}

template <class T>
struct DevMem {
    T *p = nullptr;
    ~DevMem() {
        if (p) (void)hipFree(p);
    }
    hipError_t alloc(size_t n) { return hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)); }
    T *release() {
        T *q = p;
        p = nullptr;
        return q;
    }
};

} // namespace

int parse_algs4_device(hipStream_t st, const char *body, size_t n, int64_t nv, int64_t first_lineno, uint32_t **d_u,
                       uint32_t **d_v, int64_t *m_out) {
    DevMem<char> buf;
    DevMem<int64_t> starts, cnt;
    BFSX_HIP_TRY(buf.alloc(n + 1));
    if (n) BFSX_HIP_TRY(hipMemcpyAsync(buf.p, body, n, hipMemcpyHostToDevice, st));
    BFSX_HIP_TRY(starts.alloc(n + 1));
    BFSX_HIP_TRY(cnt.alloc(1));
    int64_t m = 0;
    if (n) {
        rocprim::counting_iterator<int64_t> idx(0);
        auto flags = rocprim::make_transform_iterator(rocprim::counting_iterator<int64_t>(0), LineStart{buf.p});
        size_t tmp_bytes = 0;
        BFSX_HIP_TRY(rocprim::select(nullptr, tmp_bytes, idx, flags, starts.p, cnt.p, n, st));
        DevMem<char> tmp;
        BFSX_HIP_TRY(tmp.alloc(tmp_bytes));
        BFSX_HIP_TRY(rocprim::select(tmp.p, tmp_bytes, idx, flags, starts.p, cnt.p, n, st));
        BFSX_HIP_TRY(hipMemcpyAsync(&m, cnt.p, sizeof(m), hipMemcpyDeviceToHost, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
    }
    DevMem<uint32_t> u, v;
    DevMem<unsigned long long> err;
    BFSX_HIP_TRY(u.alloc(m));
    BFSX_HIP_TRY(v.alloc(m));
    BFSX_HIP_TRY(err.alloc(1));
    BFSX_HIP_TRY(hipMemsetAsync(err.p, 0xFF, sizeof(unsigned long long), st));
    if (m) {
        const int64_t blocks = std::min<int64_t>((m + kBS - 1) / kBS, 16384);
        hipLaunchKernelGGL(k_parse_lines, dim3((unsigned)blocks), dim3(kBS), 0, st, buf.p, (int64_t)n, starts.p, m, nv,
                           u.p, v.p, err.p);
        BFSX_HIP_TRY(hipGetLastError());
    }
    unsigned long long e = 0;
    BFSX_HIP_TRY(hipMemcpyAsync(&e, err.p, sizeof(e), hipMemcpyDeviceToHost, st));
    BFSX_HIP_TRY(hipStreamSynchronize(st));
    if (e != ~0ull) {
        const std::string line = "line " + std::to_string(first_lineno + (int64_t)(e >> 2));
        if ((e & 3) == kErrRange)
            return fail(BFSX_E_RANGE, line + ": vertex id outside [0," + std::to_string(nv) + ")");
        return fail(BFSX_E_PARSE, line + ": expected two int tokens");
    }
    *d_u = u.release();
    *d_v = v.release();
    *m_out = m;
    return BFSX_OK;
}

} // namespace bfsx
