// mfma_f64_ceiling.hip — measurement tool (not product code): the f64 matrix-core rate one MI355X
// sustains under load, to price the restart rotation (k_rotate_stream / k_rotate_chunked) against a
// measured ceiling beside the 78.6 TFLOP/s spec.  Every wave issues back-to-back
// v_mfma_f64_16x16x4_f64 on ACC independent accumulators (no memory traffic in the loop); the
// grid covers every CU with WAVES waves per workgroup.  Prints one JSON line per configuration.
//
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_f64_ceiling tools/mfma_f64_ceiling.hip
//   run:   tools/mfma_f64_ceiling
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

#define HK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

template <int ACC>
__global__ void k_mfma_f64(double* out, int iters, double seed) {
    const int lane = threadIdx.x & 63;
    double a = seed + 1e-3 * lane, b = seed - 1e-3 * lane;
    f64x4 acc[ACC];
#pragma unroll
    for (int m = 0; m < ACC; ++m) acc[m] = f64x4{0.0, 0.0, 0.0, 0.0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int m = 0; m < ACC; ++m) acc[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[m], 0, 0, 0);
    }
    double s = 0.0;
#pragma unroll
    for (int m = 0; m < ACC; ++m) s += acc[m][0] + acc[m][1] + acc[m][2] + acc[m][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;   // vector store: keeps the loop live
}

template <int ACC>
static int run(int cus, int waves, int iters) {
    const int threads = 64 * waves, blocks = cus * 4;   // several workgroups per CU
    double* out;
    HK(hipMalloc((void**)&out, (size_t)blocks * threads * sizeof(double)));
    hipEvent_t e0, e1;
    HK(hipEventCreate(&e0));
    HK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_mfma_f64<ACC>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0);   // warm-up
    HK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        HK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k_mfma_f64<ACC>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0);
        HK(hipEventRecord(e1, 0));
        HK(hipEventSynchronize(e1));
        float ms;
        HK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    const double flop = 2.0 * 16 * 16 * 4 * (double)ACC * iters * blocks * waves;
    printf("{\"tool\": \"mfma_f64_ceiling\", \"acc\": %d, \"waves_per_wg\": %d, \"workgroups\": %d, \"ms\": %.3f, "
           "\"tflops\": %.2f, \"frac_of_78.6\": %.4f}\n",
           ACC, waves, blocks, best, flop / (best * 1e-3) / 1e12, flop / (best * 1e-3) / 1e12 / 78.6);
    HK(hipFree(out));
    return 0;
}

int main() {
    int dev = 0;
    hipDeviceProp_t p;
    HK(hipGetDevice(&dev));
    HK(hipGetDeviceProperties(&p, dev));
    const int cus = p.multiProcessorCount;
    const int iters = 20000;
    int rc = 0;
    rc |= run<4>(cus, 4, iters);
    rc |= run<8>(cus, 4, iters);
    rc |= run<8>(cus, 8, iters);
    rc |= run<16>(cus, 4, iters);
    rc |= run<8>(cus, 16, iters / 2);
    return rc;
}
