// core.hip — error state, device info, workspace sizing and the NaN status of the C ABI.
#include "nkv_internal.h"

namespace nkvi {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

// Compute units of the current device (cached per device id; 256 on MI355X).
int device_cus() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int n = 0;
        cus[dev] = (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
                       ? n : 256;
    }
    return cus[dev];
}

int check_layout(const nkv_layout* L) {
    if (!L) return fail(NKV_EINVAL, "layout is NULL");
    if (L->n_wf < 1 || L->n_v < 0 || L->n_p < 0)
        return fail(NKV_EINVAL, "bad layout: n_wf=%d n_v=%lld n_p=%lld", L->n_wf,
                    (long long)L->n_v, (long long)L->n_p);
    if (L->sv < L->n_v || L->sp < L->n_p || L->sv % NKV_TILE || L->sp % NKV_TILE || L->ld % NKV_TILE)
        return fail(NKV_ESHAPE, "layout not padded to NKV_TILE: sv=%lld sp=%lld ld=%lld",
                    (long long)L->sv, (long long)L->sp, (long long)L->ld);
    if (L->ld < rows_of(L) + 1)
        return fail(NKV_ESHAPE, "ld=%lld too small for %lld rows + time", (long long)L->ld,
                    (long long)rows_of(L));
    return NKV_OK;
}

int check_ptr(const void* p, const char* what) {
    if (!p) return fail(NKV_EINVAL, "%s is NULL", what);
    if (reinterpret_cast<uintptr_t>(p) % 16) return fail(NKV_ESHAPE, "%s not 16-byte aligned", what);
    return NKV_OK;
}

}  // namespace nkvi

extern "C" {

int nkv_abi_version(void) { return NKV_ABI_VERSION; }

const char* nkv_last_error(void) { return g_err; }

int nkv_device_info(int* device, int* cu_count, int64_t* hbm_bytes, char* name, int name_len) {
    int dev = 0;
    NKV_HIP(hipGetDevice(&dev));
    hipDeviceProp_t p;
    NKV_HIP(hipGetDeviceProperties(&p, dev));
    if (device) *device = dev;
    if (cu_count) *cu_count = p.multiProcessorCount;
    if (hbm_bytes) *hbm_bytes = (int64_t)p.totalGlobalMem;
    if (name && name_len > 0) {
        snprintf(name, name_len, "%s", p.gcnArchName);
    }
    return NKV_OK;
}

size_t nkv_workspace_bytes(const nkv_layout* L, int max_cols) {
    (void)L;
    if (max_cols < 1) max_cols = 1;
    return kCtrlBytes + (size_t)kMaxBlocks * (size_t)(2 * max_cols + 2) * sizeof(double);  // 2 RHS (DCGS2)
}

int nkv_check_status(void* ws, void* stream) {
    CHECK(check_ptr(ws, "ws"));
    int flag = 0;
    NKV_HIP(hipMemcpyAsync(&flag, nan_flag_of(ws), sizeof(int), hipMemcpyDeviceToHost, S(stream)));
    NKV_HIP(hipStreamSynchronize(S(stream)));
    if (flag) {
        NKV_HIP(hipMemsetAsync(nan_flag_of(ws), 0, sizeof(int), S(stream)));
        return fail(NKV_ENAN, "NaN detected in dot product");  // nek_vectors.f90:108-111
    }
    return NKV_OK;
}

}  // extern "C"
