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

int nkv_layout_init(nkv_layout* L, int ldim, int lx1, int lx2, int64_t nelv, int64_t nelt, int n_scalars,
                    int ifpo, int rank0) {
    if (!L) return fail(NKV_EINVAL, "layout is NULL");
    if ((ldim != 2 && ldim != 3) || lx1 < 2 || (ifpo && lx2 < 1) || nelv < 0 || n_scalars < 0)
        return fail(NKV_EINVAL, "bad layout parameters: ldim=%d lx1=%d lx2=%d nelv=%lld n_scalars=%d", ldim, lx1,
                    lx2, (long long)nelv, n_scalars);
    // k_dot / real_dot weight a scalar over nt = nx1*ny1*nz1*nelt points with bm1s(lx1,ly1,lz1,lelv)
    // (core/krylov_subspace.f90:36-44, nek_vectors.f90:88-99, core/NEKSTAB:86): with nelt != nelv
    // (conjugate heat transfer) the reference reads past its weights, so such a layout is refused
    if (n_scalars > 0 && nelt != nelv)
        return fail(NKV_ESHAPE, "nelt=%lld != nelv=%lld with %d dotted scalar(s): conjugate heat transfer "
                    "layouts are not supported (the reference weights t over nelt elements with the nelv-element "
                    "bm1s, krylov_subspace.f90:36-44, NEKSTAB:86)", (long long)nelt, (long long)nelv, n_scalars);
    int64_t pv = lx1, pp = ifpo ? lx2 : 0;
    for (int d = 1; d < ldim; ++d) {
        pv *= lx1;
        pp *= ifpo ? lx2 : 0;
    }
    auto up = [](int64_t n) { return (n + NKV_TILE - 1) / NKV_TILE * NKV_TILE; };
    L->n_v = pv * nelv;
    L->n_p = pp * nelv;
    L->sv = up(L->n_v);
    L->sp = up(L->n_p);
    L->n_wf = ldim + n_scalars;
    L->ld = up((int64_t)L->n_wf * L->sv + L->sp + 1);
    L->rank0 = rank0 ? 1 : 0;
    return NKV_OK;
}

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
