// pcie_probe.cpp — what bounds wc_forward_host / wc_inverse_host (C2: 2.15 GB
// of fp64 cells up, 0.65 GB of payloads down; inverse 0.65 GB up, 1.07 GB of
// boxes down)?  Timing-only probe of the copy engines and of the host side of
// a pageable copy; no kernel runs.
//
//   h2d pinned / pageable            hipMemcpyAsync + stream sync
//   d2h pinned / pageable (touched)  the same, destination pages faulted in
//   d2h pageable (fresh)             destination straight from malloc (what a
//                                    caller's new std::vector / np.empty is)
//   h2d + d2h pinned, two streams    both directions at once
//   memcpy pinned -> fresh, T threads  the host half of a pinned bounce buffer
//
// usage: pcie_probe   (one JSON line per case)
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(2);                                                       \
        }                                                                       \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void report(const char* name, size_t bytes, double s) {
    std::printf("{\"case\": \"%s\", \"GB\": %.3f, \"ms\": %.2f, \"GBps\": %.1f}\n", name, bytes / 1e9, s * 1e3,
                bytes / s / 1e9);
    std::fflush(stdout);
}

static double copy_once(void* dst, const void* src, size_t bytes, hipMemcpyKind k, hipStream_t st) {
    CK(hipStreamSynchronize(st));
    const double t0 = now();
    CK(hipMemcpyAsync(dst, src, bytes, k, st));
    CK(hipStreamSynchronize(st));
    return now() - t0;
}

static void par_memcpy(void* dst, const void* src, size_t bytes, int T) {
    std::vector<std::thread> th;
    const size_t per = (bytes / T + 4095) & ~size_t(4095);
    for (int t = 0; t < T; ++t) {
        const size_t lo = std::min(bytes, per * t), hi = std::min(bytes, per * (t + 1));
        th.emplace_back([=] { std::memcpy((char*)dst + lo, (const char*)src + lo, hi - lo); });
    }
    for (auto& x : th) x.join();
}

static char* fresh(size_t bytes, bool huge) {
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) std::exit(3);
    if (huge) madvise(p, bytes, MADV_HUGEPAGE);
    return (char*)p;
}

static void prefault(char* p, size_t bytes, int T) {
    std::vector<std::thread> th;
    const size_t per = (bytes / T + 4095) & ~size_t(4095);
    for (int t = 0; t < T; ++t) {
        const size_t lo = std::min(bytes, per * t), hi = std::min(bytes, per * (t + 1));
        th.emplace_back([=] {
            for (size_t o = lo; o < hi; o += 4096) p[o] = 0;
        });
    }
    for (auto& x : th) x.join();
}

static void thp_settings() {
    for (const char* f : {"/sys/kernel/mm/transparent_hugepage/enabled", "/sys/kernel/mm/transparent_hugepage/defrag"}) {
        char buf[256] = {0};
        FILE* fp = std::fopen(f, "r");
        if (fp) {
            if (!std::fgets(buf, sizeof buf, fp)) buf[0] = 0;
            std::fclose(fp);
        }
        buf[strcspn(buf, "\n")] = 0;
        std::printf("{\"file\": \"%s\", \"value\": \"%s\"}\n", f, buf);
    }
}

int main() {
    thp_settings();
    const size_t up = 2147483648ull, down = 650808168ull, boxes = 1073741824ull;
    hipStream_t a, b;
    CK(hipSetDevice(0));
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    void *dev_up, *dev_down, *pin_up, *pin_down;
    CK(hipMalloc(&dev_up, up));
    CK(hipMalloc(&dev_down, boxes));
    CK(hipHostMalloc(&pin_up, up, hipHostMallocDefault));
    CK(hipHostMalloc(&pin_down, boxes, hipHostMallocDefault));
    std::memset(pin_up, 1, up);
    std::memset(pin_down, 2, boxes);
    char* page_up = (char*)std::malloc(up);
    std::memset(page_up, 3, up);
    CK(hipMemset(dev_down, 4, boxes));
    CK(hipDeviceSynchronize());

    if (std::getenv("PCIE_PROBE_FREE")) {
        // what freeing a destination costs: populated only, after a pageable
        // D2H into it (the runtime pins pageable pages for its DMA), after a
        // D2H into pinned bounce chunks + threaded memcpy into it
        const size_t chunk = size_t(64) << 20;
        char* bounce[2];
        CK(hipHostMalloc((void**)&bounce[0], chunk, hipHostMallocDefault));
        CK(hipHostMalloc((void**)&bounce[1], chunk, hipHostMallocDefault));
        for (int rep = 0; rep < 3; ++rep) {
            for (int mode = 0; mode < 3; ++mode) {
                char* f = fresh(boxes, true);
                prefault(f, boxes, 16);
                double c = 0;
                if (mode == 1) {
                    c = copy_once(f, dev_down, boxes, hipMemcpyDeviceToHost, a);
                } else if (mode == 2) {
                    const double t0 = now();
                    for (size_t o = 0, k = 0; o < boxes; o += chunk, ++k) {
                        const size_t len = std::min(chunk, boxes - o);
                        char* bb = bounce[k & 1];
                        CK(hipMemcpyAsync(bb, (char*)dev_down + o, len, hipMemcpyDeviceToHost, a));
                        CK(hipStreamSynchronize(a));
                        par_memcpy(f + o, bb, len, 16);
                    }
                    c = now() - t0;
                }
                const double t0 = now();
                munmap(f, boxes);
                const double t1 = now();
                const char* names[] = {"munmap 1.07 GB populated only", "munmap 1.07 GB after pageable d2h",
                                       "munmap 1.07 GB after bounce d2h (serial, T=16)"};
                if (mode) report(mode == 1 ? "  pageable d2h" : "  bounce d2h serial", boxes, c);
                report(names[mode], boxes, t1 - t0);
            }
        }
        return 0;
    }
    if (std::getenv("PCIE_PROBE_H2D")) {
        // pageable sources as a caller has them (a new buffer each call, written
        // by the caller), straight vs through pinned bounce chunks filled by T
        // threads while the previous chunk's DMA runs
        const size_t chunk = size_t(64) << 20;
        char* bounce[2];
        CK(hipHostMalloc((void**)&bounce[0], chunk, hipHostMallocDefault));
        CK(hipHostMalloc((void**)&bounce[1], chunk, hipHostMallocDefault));
        hipEvent_t done[2];
        CK(hipEventCreateWithFlags(&done[0], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&done[1], hipEventDisableTiming));
        for (int rep = 0; rep < 3; ++rep) {
            char* src = fresh(up, true);
            prefault(src, up, 16);
            std::memset(src, 5 + rep, up);
            report("h2d pageable new+written 2.15 GB", up, copy_once(dev_up, src, up, hipMemcpyHostToDevice, a));
            report("h2d pageable same again", up, copy_once(dev_up, src, up, hipMemcpyHostToDevice, a));
            munmap(src, up);
            for (int T : {4, 8, 16}) {
                src = fresh(up, true);
                prefault(src, up, 16);
                std::memset(src, 9 + rep, up);
                CK(hipDeviceSynchronize());
                const double t0 = now();
                size_t k = 0;
                for (size_t o = 0; o < up; o += chunk, ++k) {
                    const size_t len = std::min(chunk, up - o);
                    char* bb = bounce[k & 1];
                    if (k >= 2) CK(hipEventSynchronize(done[k & 1]));
                    par_memcpy(bb, src + o, len, T);
                    CK(hipMemcpyAsync((char*)dev_up + o, bb, len, hipMemcpyHostToDevice, a));
                    CK(hipEventRecord(done[k & 1], a));
                }
                CK(hipStreamSynchronize(a));
                char name[96];
                std::snprintf(name, sizeof name, "h2d via 2 x 64 MiB pinned bounce, T=%d memcpy", T);
                report(name, up, now() - t0);
                munmap(src, up);
            }
        }
        return 0;
    }
    for (int rep = 0; rep < 2; ++rep) {
        for (bool huge : {false, true}) {
            for (size_t sz : {down, boxes}) {
                char* f = fresh(sz, huge);
                char name[96];
                std::snprintf(name, sizeof name, "d2h mmap fresh %s %.2f GB", huge ? "MADV_HUGEPAGE" : "4K", sz / 1e9);
                report(name, sz, copy_once(f, dev_down, sz, hipMemcpyDeviceToHost, a));
                munmap(f, sz);
            }
            for (int T : {1, 8, 16}) {
                char* f = fresh(boxes, huge);
                const double t0 = now();
                prefault(f, boxes, T);
                const double t1 = now();
                const double c = copy_once(f, dev_down, boxes, hipMemcpyDeviceToHost, a);
                char name[96];
                std::snprintf(name, sizeof name, "prefault %s T=%d 1.07 GB", huge ? "MADV_HUGEPAGE" : "4K", T);
                report(name, boxes, t1 - t0);
                report("  d2h after", boxes, c);
                munmap(f, boxes);
            }
        }
        report("h2d pinned 2.15 GB", up, copy_once(dev_up, pin_up, up, hipMemcpyHostToDevice, a));
        report("h2d pageable 2.15 GB", up, copy_once(dev_up, page_up, up, hipMemcpyHostToDevice, a));
        report("h2d pageable 0.65 GB", down, copy_once(dev_up, page_up, down, hipMemcpyHostToDevice, a));
        report("d2h pinned 0.65 GB", down, copy_once(pin_down, dev_down, down, hipMemcpyDeviceToHost, a));
        report("d2h pinned 1.07 GB", boxes, copy_once(pin_down, dev_down, boxes, hipMemcpyDeviceToHost, a));
        {
            char* f = (char*)std::malloc(down);
            report("d2h pageable fresh 0.65 GB", down, copy_once(f, dev_down, down, hipMemcpyDeviceToHost, a));
            report("d2h pageable touched 0.65 GB", down, copy_once(f, dev_down, down, hipMemcpyDeviceToHost, a));
            std::free(f);
        }
        {
            char* f = (char*)std::malloc(boxes);
            report("d2h pageable fresh 1.07 GB", boxes, copy_once(f, dev_down, boxes, hipMemcpyDeviceToHost, a));
            report("d2h pageable touched 1.07 GB", boxes, copy_once(f, dev_down, boxes, hipMemcpyDeviceToHost, a));
            std::free(f);
        }
        {
            CK(hipDeviceSynchronize());
            const double t0 = now();
            CK(hipMemcpyAsync(dev_up, pin_up, up, hipMemcpyHostToDevice, a));
            CK(hipMemcpyAsync(pin_down, dev_down, down, hipMemcpyDeviceToHost, b));
            CK(hipStreamSynchronize(b));
            const double tb = now() - t0;
            CK(hipStreamSynchronize(a));
            const double ta = now() - t0;
            report("h2d pinned 2.15 GB || d2h pinned 0.65 GB: both", up + down, ta);
            report("  ... d2h side done", down, tb);
        }
        for (int T : {1, 4, 8, 16}) {
            char* f = (char*)std::malloc(down);
            const double t0 = now();
            par_memcpy(f, pin_down, down, T);
            const double t1 = now();
            par_memcpy(f, pin_down, down, T);
            const double t2 = now();
            char name[64];
            std::snprintf(name, sizeof name, "memcpy pinned->fresh T=%d", T);
            report(name, down, t1 - t0);
            std::snprintf(name, sizeof name, "memcpy pinned->touched T=%d", T);
            report(name, down, t2 - t1);
            std::free(f);
        }
        {
            // register the caller's fresh buffer for the copy instead
            char* f = (char*)std::malloc(down);
            const double t0 = now();
            CK(hipHostRegister(f, down, hipHostRegisterDefault));
            const double t1 = now();
            const double c = copy_once(f, dev_down, down, hipMemcpyDeviceToHost, a);
            const double t2 = now();
            CK(hipHostUnregister(f));
            const double t3 = now();
            report("hipHostRegister fresh 0.65 GB", down, t1 - t0);
            report("  d2h into it", down, c);
            report("  unregister", down, t3 - t2);
            std::free(f);
        }
    }
    return 0;
}
