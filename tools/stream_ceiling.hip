// Streaming-bandwidth ceilings of one MI355X for the access shapes of the Gram–Schmidt kernels
// (a measurement tool, not product code): what a plain kernel of the same shape reaches, so the
// product kernels' GB/s can be read against an achievable ceiling as well as the 8 TB/s spec.
//
//   read      : s += x[i]                    (1 stream, read only; the multi-dot's shape at j -> inf)
//   readcols  : s += sum_c Q[c*ld + i]       (C column streams at stride ld, read only; the multi-dot)
//   copy      : y[i] = x[i]                  (1R 1W)
//   triad     : y[i] = d[i] * x[i]           (2R 1W; the diagonal matvec)
//   update    : y[i] = x[i] - sum_c Q[c*ld+i] (C+1 R, 1W; the dual update has C+2 R, 2 W)
//
// Every variant: double2 loads/stores (16 B per lane), U double2 per thread in flight, a grid of G
// 256-thread workgroups sweeping the rows grid-stride; optional non-temporal loads.  Timed with
// HIP events, median of 7 after 2 warm-ups, each on a fresh region so nothing is cache-resident.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_ceiling.hip -o tools/stream_ceiling
// run  : tools/stream_ceiling [GiB per stream, default 0.75] [max columns, default 64]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

constexpr int kT = 256;

template <bool NT>
__device__ __forceinline__ double2 ld(const double* p) {
    if constexpr (NT) {
        double2 v;
        v.x = __builtin_nontemporal_load(p);
        v.y = __builtin_nontemporal_load(p + 1);
        return v;
    } else {
        return *reinterpret_cast<const double2*>(p);
    }
}

__device__ __forceinline__ void st(double* p, double2 v) {
    __builtin_nontemporal_store(v.x, p);
    __builtin_nontemporal_store(v.y, p + 1);
}

// rows per chunk = kT * U * 2 doubles
template <int U, bool NT>
__global__ __launch_bounds__(kT) void k_read(const double* __restrict__ x, int64_t chunks, double* out) {
    double s = 0.0;
    for (int64_t c = blockIdx.x; c < chunks; c += gridDim.x) {
        const double* p = x + c * (kT * U * 2) + 2 * threadIdx.x;
        double2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld<NT>(p + u * 2 * kT);
#pragma unroll
        for (int u = 0; u < U; ++u) s += v[u].x + v[u].y;
    }
    if (s == 12345.678) out[0] = s;   // keep the loads
}

template <int U, bool NT>
__global__ __launch_bounds__(kT) void k_readcols(const double* __restrict__ Q, int64_t ld_, int C, int64_t c_lo,
                                                 int64_t c_hi, double* out) {
    double s = 0.0;
    for (int64_t c = c_lo + blockIdx.x; c < c_hi; c += gridDim.x) {
        const double* p = Q + c * (kT * U * 2) + 2 * threadIdx.x;
        for (int col = 0; col < C; ++col) {
            double2 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = ld<NT>(p + (int64_t)col * ld_ + u * 2 * kT);
#pragma unroll
            for (int u = 0; u < U; ++u) s += v[u].x + v[u].y;
        }
    }
    if (s == 12345.678) out[0] = s;
}

template <int U, bool NT>
__global__ __launch_bounds__(kT) void k_copy(const double* __restrict__ x, double* __restrict__ y, int64_t chunks) {
    for (int64_t c = blockIdx.x; c < chunks; c += gridDim.x) {
        const int64_t o = c * (kT * U * 2) + 2 * threadIdx.x;
        double2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld<NT>(x + o + u * 2 * kT);
#pragma unroll
        for (int u = 0; u < U; ++u) st(y + o + u * 2 * kT, v[u]);
    }
}

template <int U, bool NT>
__global__ __launch_bounds__(kT) void k_triad(const double* __restrict__ d, const double* __restrict__ x,
                                              double* __restrict__ y, int64_t chunks) {
    for (int64_t c = blockIdx.x; c < chunks; c += gridDim.x) {
        const int64_t o = c * (kT * U * 2) + 2 * threadIdx.x;
        double2 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a[u] = ld<NT>(d + o + u * 2 * kT);
            b[u] = ld<NT>(x + o + u * 2 * kT);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) st(y + o + u * 2 * kT, make_double2(a[u].x * b[u].x, a[u].y * b[u].y));
    }
}

template <int U, bool NT>
__global__ __launch_bounds__(kT) void k_update(const double* __restrict__ Q, int64_t ld_, int C,
                                               const double* __restrict__ x, double* __restrict__ y, int64_t c_lo,
                                               int64_t c_hi) {
    for (int64_t c = c_lo + blockIdx.x; c < c_hi; c += gridDim.x) {
        const int64_t o = c * (kT * U * 2) + 2 * threadIdx.x;
        double2 acc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = ld<NT>(x + o + u * 2 * kT);
        for (int col = 0; col < C; ++col) {
            double2 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = ld<NT>(Q + (int64_t)col * ld_ + o + u * 2 * kT);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                acc[u].x -= 0.5 * v[u].x;
                acc[u].y -= 0.5 * v[u].y;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) st(y + o + u * 2 * kT, acc[u]);
    }
}

struct Timer {
    hipEvent_t a, b;
    Timer() {
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
    }
};

template <class F>
double time_ms(F launch, int reps = 7) {
    Timer t;
    std::vector<double> ms;
    for (int r = 0; r < reps + 2; ++r) {
        CK(hipEventRecord(t.a));
        launch(r);
        CK(hipEventRecord(t.b));
        CK(hipEventSynchronize(t.b));
        float f;
        CK(hipEventElapsedTime(&f, t.a, t.b));
        if (r >= 2) ms.push_back(f);
    }
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? std::atof(argv[1]) : 0.75;
    // one stream = n doubles (a multiple of every chunk size); the pool holds 2 x (C + 3) streams so
    // consecutive repetitions alternate between two disjoint regions (nothing stays in the 256 MB MALL)
    const int C = argc > 2 ? std::atoi(argv[2]) : 64;
    const int64_t chunk_max = kT * 16 * 2;
    int64_t n = (int64_t)(gib * (1 << 30) / 8);
    n = n / chunk_max * chunk_max;
    const int64_t ld_ = n + 4096;   // column stride, 32 KiB past the column (as the product pads)
    const int nstreams = C + 3;
    double* pool;
    const size_t bytes = sizeof(double) * (size_t)ld_ * nstreams * 2;
    CK(hipMalloc(&pool, bytes));
    CK(hipMemset(pool, 0, bytes));
    double* out;
    CK(hipMalloc(&out, 64));
    auto region = [&](int r) { return pool + (size_t)(r & 1) * ld_ * nstreams; };
    std::printf("stream = %.3f GB, column stride %lld doubles, %d columns\n", n * 8.0 / 1e9, (long long)ld_, C);

#define SWEEP(NAME, U, NT, BYTES, ...)                                                           \
    for (int G : {256, 512, 768, 1024, 2048}) {                                                     \
        const int64_t chunks = n / (kT * U * 2);                                                    \
        double ms = time_ms([&](int r) {                                                            \
            double* R = region(r);                                                                  \
            (void)R;                                                                                \
            __VA_ARGS__;                                                                            \
        });                                                                                         \
        std::printf("%-9s U=%-2d nt=%d G=%-5d %8.3f ms %8.1f GB/s\n", NAME, U, (int)NT, G, ms,      \
                    (BYTES) / (ms * 1e-3) / 1e9);                                                   \
    }

#define ALLV(NAME, BYTES, ...)                                                              \
    {                                                                                               \
        constexpr int U = 4;                                                                        \
        constexpr bool NT = true;                                                                   \
        SWEEP(NAME, U, NT, BYTES, __VA_ARGS__)                                                      \
    }                                                                                               \
    {                                                                                               \
        constexpr int U = 8;                                                                        \
        constexpr bool NT = true;                                                                   \
        SWEEP(NAME, U, NT, BYTES, __VA_ARGS__)                                                      \
    }                                                                                               \
    {                                                                                               \
        constexpr int U = 16;                                                                       \
        constexpr bool NT = true;                                                                   \
        SWEEP(NAME, U, NT, BYTES, __VA_ARGS__)                                                      \
    }                                                                                               \
    {                                                                                               \
        constexpr int U = 8;                                                                        \
        constexpr bool NT = false;                                                                  \
        SWEEP(NAME, U, NT, BYTES, __VA_ARGS__)                                                      \
    }

    const double sb = 8.0 * n;
    ALLV("read", sb, hipLaunchKernelGGL((k_read<U, NT>), dim3(G), dim3(kT), 0, 0, R, chunks, out))
    ALLV("copy", 2 * sb, hipLaunchKernelGGL((k_copy<U, NT>), dim3(G), dim3(kT), 0, 0, R, R + ld_, chunks))
    ALLV("triad", 3 * sb, hipLaunchKernelGGL((k_triad<U, NT>), dim3(G), dim3(kT), 0, 0, R, R + ld_, R + 2 * ld_, chunks))
    // band = 0: one launch over all chunks; band = 2: one launch per 2 grid-stride rounds (the
    // product's row-band dispatches)
    for (int cols : {8, 32, 64, 128}) {
        if (cols > C) break;
        for (int band : {0, 2}) {
            std::printf("-- %d columns, band %d\n", cols, band);
            ALLV("readcols", cols * sb,
                 for (int64_t lo = 0; lo < chunks; lo += band ? (int64_t)band * G : chunks)
                     hipLaunchKernelGGL((k_readcols<U, NT>), dim3(G), dim3(kT), 0, 0, R + 2 * ld_, ld_, cols, lo,
                                        band ? std::min(chunks, lo + (int64_t)band * G) : chunks, out))
            ALLV("update", (cols + 2) * sb,
                 for (int64_t lo = 0; lo < chunks; lo += band ? (int64_t)band * G : chunks)
                     hipLaunchKernelGGL((k_update<U, NT>), dim3(G), dim3(kT), 0, 0, R + 2 * ld_, ld_, cols, R, R + ld_,
                                        lo, band ? std::min(chunks, lo + (int64_t)band * G) : chunks))
        }
    }
    CK(hipFree(pool));
    return 0;
}
