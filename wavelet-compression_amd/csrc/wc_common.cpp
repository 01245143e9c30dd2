// wc_common.cpp — errors, device buffers, unit validation, the per-device
// context registry and the kernel error word of the C-ABI (wc_ctx.h).  Host
// code over the HIP runtime API only: no kernels (the host-pipeline sanitizer
// test links it against a CPU fake of that API).
#include "wc_ctx.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

namespace wc {

int fail(wc_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

int hip_fail(wc_ctx* c, hipError_t e, const char* what) {
    return fail(c, WC_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

int ensure(wc_ctx* c, DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return WC_OK;
    size_t want = std::max(bytes, b.bytes + b.bytes / 2);
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    hipError_t e = hipMalloc(&b.p, want);
    if (e != hipSuccess) {
        e = hipMalloc(&b.p, bytes);
        want = bytes;
    }
    if (e != hipSuccess) return fail(c, WC_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    b.bytes = want;
    return WC_OK;
}

int validate_units(wc_ctx* c, const wc_unit* units, int n) {
    if (n < 0) return fail(c, WC_ERR_INVALID, "n < 0");
    if (n > 0 && !units) return fail(c, WC_ERR_INVALID, "units is NULL");
    for (int i = 0; i < n; ++i) {
        const wc_unit& u = units[i];
        if (u.nx < 0 || u.ny < 0 || u.nz < 0 || u.reserved != 0)
            return fail(c, WC_ERR_INVALID, "unit " + std::to_string(i) + ": negative dims or reserved != 0");
        const uint64_t cells = (uint64_t)u.nx * u.ny * u.nz;
        // ncoeff is serialized as int32 (src/compressor.cpp:65-67)
        if (cells > 0x7fffffffull)
            return fail(c, WC_ERR_INVALID, "unit " + std::to_string(i) + ": more than 2^31-1 cells");
    }
    return WC_OK;
}

// Device buffers: 16-B aligned (the kernels pick their vector widths from
// element offsets; hipMalloc and torch allocations are 256-B aligned).
int check_aligned(wc_ctx* c, const void* p, const char* what, uintptr_t align) {
    if (((uintptr_t)p & (align - 1)) == 0) return WC_OK;
    return fail(c, WC_ERR_INVALID, std::string(what) + ": device buffer not " + std::to_string(align) + "-byte aligned");
}

hipEvent_t take_event(wc_ctx* c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

int upload(wc_ctx* c, DevBuf& d, const void* h, size_t bytes, const char* what) {
    int rc = ensure(c, d, bytes);
    if (rc) return rc;
    if (!bytes) return WC_OK;
    hipError_t e = hipMemcpyAsync(d.p, h, bytes, hipMemcpyHostToDevice, c->stream);
    return e == hipSuccess ? WC_OK : hip_fail(c, e, what);
}

int set_device(wc_ctx* c) {
    c->staged = false;
    hipError_t e = hipSetDevice(c->device);
    return e == hipSuccess ? WC_OK : hip_fail(c, e, "hipSetDevice");
}

// The launch-order form of the look-backs needs no assumption about dispatch
// order or about other kernels on the device (a wait past its bound derives
// the predecessor itself, wc_device.h spin_wait): it is the form unless the
// caller asks for the tickets.
bool use_ordered(const wc_ctx* c) { return c->opt_ordered && !c->force_tickets; }

// Surface an error bit a kernel raised (malformed payload in the decode) at
// the next synchronisation point, and clear the word.  The reference exits on a malformed payload
// (src/decompressor.cpp:228-231); here it is WC_ERR_FORMAT.
int check_kernel_errors(wc_ctx* c) {
    if (!c->err_check_pending) return WC_OK;
    c->err_check_pending = false;
    uint32_t flag = 0;
    hipError_t e = hipMemcpyAsync(&flag, c->errflag.p, 4, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess && flag) e = hipMemsetAsync(c->errflag.p, 0, 4, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "error flag readback");
    if (flag & (kErrHeader | kErrNegativeRun)) {
        char buf[128];
        std::snprintf(buf, sizeof buf, "malformed payload (flags 0x%x: 1 header, 2 negative run)", flag);
        return fail(c, WC_ERR_FORMAT, buf);
    }
    return WC_OK;
}


uint64_t cells_extent(const wc_unit* units, int n) {
    uint64_t ext = 0;
    for (int i = 0; i < n; ++i)
        ext = std::max(ext, units[i].cell_offset + (uint64_t)units[i].nx * units[i].ny * units[i].nz);
    return ext;
}


}  // namespace wc

extern "C" {

uint64_t wc_payload_bound(const wc_unit* units, int n) {
    uint64_t b = 4;
    for (int i = 0; i < n; ++i) b += 24 + 8 * (uint64_t)units[i].nx * units[i].ny * units[i].nz;
    return b;
}

uint64_t wc_cell_count(const wc_unit* units, int n) {
    uint64_t s = 0;
    for (int i = 0; i < n; ++i) s += (uint64_t)units[i].nx * units[i].ny * units[i].nz;
    return s;
}

uint64_t wc_rowindex_bytes(const wc_unit* units, int n) {
    uint64_t e = 0;
    for (int i = 0; i < n; ++i)  // W*H + 1 entries per unit with cells, none for an empty unit
        if ((uint64_t)units[i].nx * units[i].ny * units[i].nz) e += (uint64_t)units[i].nx * units[i].ny + 1;
    return 8 * e;
}

}  // extern "C"
