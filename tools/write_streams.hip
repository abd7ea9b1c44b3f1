// Write-stream probe for the restart rotation (a measurement tool, not product code): the access
// shape of Q[:, :NO] = Q[:, :C] V without its arithmetic — every workgroup reads C column chunks of
// one row tile and writes NO outputs — to separate what the number of written columns costs from
// what the MFMAs cost (the 17–64-kept rotation's ceiling).
//
//   inplace : the NO outputs overwrite columns 0..NO-1 of the tile (the rotation's shape)
//   tilemaj : the NO outputs go to one contiguous tile-major region (ONE write stream, same bytes)
//   bands   : the sweep split into that many dispatches over contiguous row bands (1 = one launch)
//
// Each variant: double2 loads/stores (16 B per lane, non-temporal), U double2 per thread per column
// (a row tile of 512 U rows, 4 U KiB per column), a G-workgroup grid sweeping tiles grid-stride.
// Timed with HIP events, median of 5 after 2 warm-ups.  GB/s = 8 n (C + NO) / time.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/write_streams.hip -o tools/write_streams
// run  : tools/write_streams [rows, default 100014464] [C, default 128] [NO: 1, 6, 16 or 25 only]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

constexpr int kT = 256;
typedef double v2d __attribute__((ext_vector_type(2)));

__device__ __forceinline__ double2 ldnt(const double* p) {
    const v2d v = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(p));
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ void stnt(double* p, double2 v) {
    __builtin_nontemporal_store(v2d{v.x, v.y}, reinterpret_cast<v2d*>(p));
}

template <int U, int NO, bool TM>
__global__ __launch_bounds__(kT) void k_rotshape(double* __restrict__ Q, int64_t ld, int C, double* __restrict__ T,
                                                 int64_t c_lo, int64_t c_hi) {
    constexpr int64_t R = kT * U * 2;
    for (int64_t c = c_lo + blockIdx.x; c < c_hi; c += gridDim.x) {
        const int64_t o = c * R + 2 * threadIdx.x;
        double2 acc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = make_double2(0.0, 0.0);
        for (int col = 0; col < C; col += 2) {
            double2 v[2][U];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int u = 0; u < U; ++u) v[h][u] = ldnt(Q + (int64_t)(col + h) * ld + o + u * 2 * kT);
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    acc[u].x += v[h][u].x;
                    acc[u].y += v[h][u].y;
                }
        }
#pragma unroll
        for (int oo = 0; oo < NO; ++oo) {
            const double s = 1.0 / (oo + 1);   // bounded: repeated runs never overflow
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const double2 val = make_double2(acc[u].x * s * (1.0 / 256), acc[u].y * s * (1.0 / 256));
                double* dst = TM ? T + (c * NO + oo) * R + 2 * threadIdx.x + u * 2 * kT
                                 : Q + (int64_t)oo * ld + o + u * 2 * kT;
                stnt(dst, val);
            }
        }
    }
}

template <class F>
double time_ms(F launch, int reps = 5) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<double> ms;
    for (int r = 0; r < reps + 2; ++r) {
        CK(hipEventRecord(a));
        launch();
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float f;
        CK(hipEventElapsedTime(&f, a, b));
        if (r >= 2) ms.push_back(f);
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
}

template <int U, int NO>
void run(double* Q, int64_t ld, int C, double* T, int64_t n) {
    const int64_t chunks = n / (kT * U * 2);
    for (int G : {512, 768, 1024}) {
        for (int nb : {1, 16, 64}) {   // dispatches, each over one contiguous row band (the product's row bands)
            for (int tm = 0; tm < (NO > 0 && nb == 1 ? 2 : 1); ++tm) {
                const double ms = time_ms([&] {
                    for (int b = 0; b < nb; ++b) {
                        const int64_t lo = chunks * b / nb, hi = chunks * (b + 1) / nb;
                        if (tm)
                            hipLaunchKernelGGL((k_rotshape<U, NO, true>), dim3(G), dim3(kT), 0, 0, Q, ld, C, T, lo, hi);
                        else
                            hipLaunchKernelGGL((k_rotshape<U, NO, false>), dim3(G), dim3(kT), 0, 0, Q, ld, C, T, lo, hi);
                    }
                });
                const double bytes = 8.0 * (double)(chunks * kT * U * 2) * (C + NO);
                std::printf("NO=%-3d %-8s U=%d G=%-5d bands=%-3d %8.3f ms %8.1f GB/s\n", NO, tm ? "tilemaj" : "inplace", U,
                            G, nb, ms, bytes / (ms * 1e-3) / 1e9);
                std::fflush(stdout);
            }
        }
    }
}

template <int NO>
void run_u(double* Q, int64_t ld, int C, double* T, int64_t n) {
    run<2, NO>(Q, ld, C, T, n);
    run<8, NO>(Q, ld, C, T, n);
}

int main(int argc, char** argv) {
    int64_t n = argc > 1 ? std::atoll(argv[1]) : 100014464;
    const int C = argc > 2 ? std::atoi(argv[2]) : 128;
    if (C % 2 || C < 2 || C > 256) {
        std::fprintf(stderr, "C must be even, 2..256\n");
        return 1;
    }
    n = n / 8192 * 8192;                              // whole tiles at every U
    const int64_t ld = (n + 4095) / 4096 * 4096;       // the product's 32 KiB column grid
    double *Q, *T;
    CK(hipMalloc(&Q, sizeof(double) * (size_t)ld * C));
    CK(hipMalloc(&T, sizeof(double) * (size_t)n * 48));
    CK(hipMemset(Q, 0, sizeof(double) * (size_t)ld * C));
    std::printf("rows %lld, column stride %lld doubles, %d columns read\n", (long long)n, (long long)ld, C);
    const int only = argc > 3 ? std::atoi(argv[3]) : -1;   // one NO only (-1: all)
    if (only < 0 || only == 1) run_u<1>(Q, ld, C, T, n);
    if (only < 0 || only == 6) run_u<6>(Q, ld, C, T, n);
    if (only < 0 || only == 16) run_u<16>(Q, ld, C, T, n);
    if (only < 0 || only == 25) run_u<25>(Q, ld, C, T, n);
    CK(hipFree(Q));
    CK(hipFree(T));
    return 0;
}
