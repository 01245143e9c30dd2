// wc_hostmem.cpp — see wc_hostmem.h.
#include "wc_hostmem.h"

#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23  // Linux 5.14
#endif

namespace wc {

HostPool::HostPool(int threads) {
    for (int i = 0; i < threads; ++i) workers_.emplace_back([this] { work(); });
}

HostPool::~HostPool() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    wake_.notify_all();
    for (auto& t : workers_) t.join();
}

bool HostPool::take(int& task) {  // mu_ held
    if (!fn_ || next_ >= ntasks_) return false;
    task = next_++;
    return true;
}

void HostPool::work() {
    unsigned long long seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
        wake_.wait(lk, [&] { return stop_ || (gen_ != seen && fn_ && next_ < ntasks_); });
        if (stop_) return;
        seen = gen_;
        int task;
        while (take(task)) {
            const std::function<void(int)>* fn = fn_;
            lk.unlock();
            (*fn)(task);
            lk.lock();
            if (++finished_ == ntasks_) done_.notify_all();
        }
    }
}

void HostPool::run(int ntasks, const std::function<void(int)>& fn) {
    if (ntasks <= 0) return;
    std::unique_lock<std::mutex> lk(mu_);
    fn_ = &fn;
    ntasks_ = ntasks;
    next_ = 0;
    finished_ = 0;
    ++gen_;
    lk.unlock();
    if (ntasks > 1) wake_.notify_all();
    lk.lock();
    int task;
    while (take(task)) {
        lk.unlock();
        fn(task);
        lk.lock();
        ++finished_;
    }
    done_.wait(lk, [&] { return finished_ == ntasks_; });
    fn_ = nullptr;
    ntasks_ = 0;
}

namespace {

std::atomic<bool> g_force_touch{false};

// Does this kernel know MADV_POPULATE_WRITE (Linux 5.14)?  Probed once on a
// private anonymous page, so that EINVAL on a caller's range later means a
// mapping it does not apply to (VM_IO / VM_PFNMAP: left alone), not an old
// kernel.
bool kernel_has_populate() {
    static const bool has = [] {
        const size_t page = (size_t)sysconf(_SC_PAGESIZE);
        void* p = mmap(nullptr, page, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) return false;
        const bool ok = madvise(p, page, MADV_POPULATE_WRITE) == 0;
        munmap(p, page);
        return ok;
    }();
    return has;
}

void populate_range(char* lo, char* hi, size_t page) {
    if (hi <= lo) return;
    if (!g_force_touch.load(std::memory_order_relaxed)) {
        if (kernel_has_populate()) {
            (void)madvise(lo, (size_t)(hi - lo), MADV_POPULATE_WRITE);  // any failure: the copy faults instead
            return;
        }
    }
    for (char* q = lo; q < hi; q += page) {  // kernels before 5.14: a read and a write-back per page
        volatile char* v = q;
        *v = *v;
    }
}

}  // namespace

void populate_force_touch(bool on) { g_force_touch.store(on); }

void populate_for_write(HostPool* pool, void* p, size_t bytes, bool thp) try {
    static const size_t page = (size_t)sysconf(_SC_PAGESIZE);
    constexpr size_t kHuge = size_t(2) << 20;
    const uintptr_t a = (uintptr_t)p, e = a + bytes;
    const uintptr_t lo = (a + page - 1) & ~(uintptr_t)(page - 1), hi = e & ~(uintptr_t)(page - 1);
    if (!p || hi <= lo) return;
    const uintptr_t hlo = (a + kHuge - 1) & ~(uintptr_t)(kHuge - 1), hhi = e & ~(uintptr_t)(kHuge - 1);
    if (thp && hhi > hlo) (void)madvise((void*)hlo, hhi - hlo, MADV_HUGEPAGE);
    // Pieces of whole huge pages (the edges take the rest), a few per thread.
    const int T = pool ? pool->threads() : 1;
    const size_t span = hi - lo;
    size_t piece = std::max(kHuge, (span / (size_t)(4 * T) + kHuge - 1) & ~(kHuge - 1));
    std::vector<std::pair<uintptr_t, uintptr_t>> parts;
    uintptr_t s = lo;
    uintptr_t b = std::min(hi, std::max(lo, hlo));  // first boundary: the first huge-page edge
    if (b > s) {
        parts.emplace_back(s, b);
        s = b;
    }
    while (s < hi) {
        const uintptr_t t = std::min<uintptr_t>(hi, s + piece);
        parts.emplace_back(s, t);
        s = t;
    }
    auto one = [&](int i) { populate_range((char*)parts[i].first, (char*)parts[i].second, page); };
    if (!pool || parts.size() == 1) {
        for (size_t i = 0; i < parts.size(); ++i) one((int)i);
        return;
    }
    pool->run((int)parts.size(), one);
} catch (...) {  // an allocation failure: leave the faults to the copy
}

}  // namespace wc
