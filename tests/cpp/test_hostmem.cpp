// test_hostmem.cpp — the host pool and the destination prefault of the _host
// entry points (wavelet-compression_amd/csrc/wc_hostmem.h), CPU only; built
// plain and under ASan+UBSan / TSan (tests/test_sanitizers.py).
//   * HostPool::run calls every task index exactly once, for pools of 0..15
//     workers and jobs of 0..5000 tasks, many jobs back to back;
//   * RunGate hands runs over in order, never early, and a cancel wakes a waiter;
//   * populate_for_write never changes a byte (data written before it, never
//     touched zeros, unaligned edges, both the MADV_POPULATE_WRITE path and the
//     per-page touch path) and leaves the whole pages of the range resident.
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

#include "wc_hostmem.h"

static int failures = 0, checks = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        ++checks;                                                             \
        if (!(c)) {                                                           \
            ++failures;                                                       \
            std::fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #c); \
        }                                                                     \
    } while (0)

static void pool_tasks() {
    for (int w : {0, 1, 3, 15}) {
        wc::HostPool pool(w);
        CHECK(pool.threads() == w + 1);
        static const int sizes[] = {0, 1, 2, 7, 64, 1000, 5000};
        for (int job = 0; job < 60; ++job) {
            const int n = sizes[job % 7];
            std::vector<std::atomic<int>> hit(n);
            for (auto& h : hit) h.store(0);
            pool.run(n, [&](int i) { hit[i].fetch_add(1); });
            bool once = true;
            for (auto& h : hit) once &= h.load() == 1;
            CHECK(once);
        }
    }
}

static size_t resident_pages(char* lo, char* hi) {
    const size_t page = (size_t)sysconf(_SC_PAGESIZE);
    std::vector<unsigned char> v((hi - lo + page - 1) / page);
    if (mincore(lo, hi - lo, v.data()) != 0) return 0;
    size_t n = 0;
    for (unsigned char b : v) n += b & 1;
    return n;
}

static void populate_keeps_bytes(bool touch, bool thp, wc::HostPool* pool) {
    wc::populate_force_touch(touch);
    const size_t page = (size_t)sysconf(_SC_PAGESIZE);
    const size_t bytes = size_t(40) << 20;
    char* base = (char*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    CHECK(base != MAP_FAILED);
    if (base == MAP_FAILED) return;
    // a written stretch in the middle, the rest never touched
    char* w0 = base + (size_t(9) << 20) + 123;
    const size_t wlen = (size_t(5) << 20) + 77;
    for (size_t i = 0; i < wlen; ++i) w0[i] = (char)(i * 131 + 7);
    // unaligned range over the written stretch and untouched memory
    char* p = base + 3 * page + 517;
    const size_t len = bytes - 7 * page - 1000;
    wc::populate_for_write(pool, p, len, thp);
    bool same = true;
    for (size_t i = 0; i < wlen; ++i) same &= w0[i] == (char)(i * 131 + 7);
    CHECK(same);
    bool zeros = true;
    for (char* q = base; q < w0; q += 97) zeros &= *q == 0;
    for (char* q = w0 + wlen; q < base + bytes; q += 97) zeros &= *q == 0;
    CHECK(zeros);
    // every whole page of [p, p + len) is resident
    char* lo = (char*)(((uintptr_t)p + page - 1) & ~(uintptr_t)(page - 1));
    char* hi = (char*)(((uintptr_t)p + len) & ~(uintptr_t)(page - 1));
    CHECK(resident_pages(lo, hi) == (size_t)(hi - lo) / page);
    munmap(base, bytes);
    wc::populate_force_touch(false);
}

static void populate_edges() {
    char buf[64] = {1, 2, 3};
    wc::populate_for_write(nullptr, nullptr, 1 << 20, true);  // null: nothing
    wc::populate_for_write(nullptr, buf, 0, true);            // empty
    wc::populate_for_write(nullptr, buf, sizeof buf, true);   // no whole page: nothing
    CHECK(buf[0] == 1 && buf[1] == 2 && buf[2] == 3);
    std::vector<float> v(3 << 20, 2.5f);  // heap memory, already written
    wc::HostPool pool(4);
    wc::populate_for_write(&pool, v.data() + 1, (v.size() - 2) * sizeof(float), true);
    bool same = true;
    for (float x : v) same &= x == 2.5f;
    CHECK(same);
}

// RunGate: a publisher thread queues runs one at a time with uneven delays;
// the waiter sees every run exactly in order, never before it is published
// (checked through a value the publisher writes first), and a cancel wakes a
// waiter blocked on a run that never comes.
static void run_gate() {
    for (int rep = 0; rep < 20; ++rep) {
        wc::RunGate gate;
        constexpr int kRuns = 16;
        std::vector<int> payload(kRuns, 0);
        std::thread pub([&] {
            for (int r = 0; r < kRuns; ++r) {
                payload[r] = r + 1;  // written before the run is published
                if ((r + rep) % 3 == 0) std::this_thread::sleep_for(std::chrono::microseconds(50 * (r % 4)));
                gate.publish(r + 1);
            }
        });
        bool ok = true;
        for (int r = 0; r < kRuns; ++r) ok &= gate.wait(r) && payload[r] == r + 1;
        pub.join();
        CHECK(ok);
        wc::RunGate stuck;
        stuck.publish(2);
        std::thread canceller([&] {
            std::this_thread::sleep_for(std::chrono::microseconds(200));
            stuck.cancel();
        });
        CHECK(stuck.wait(1));
        CHECK(!stuck.wait(5));  // returns once cancelled
        canceller.join();
    }
}

int main() {
    pool_tasks();
    run_gate();
    {
        wc::HostPool pool(7);
        for (bool touch : {false, true})
            for (bool thp : {false, true}) {
                populate_keeps_bytes(touch, thp, &pool);
                populate_keeps_bytes(touch, thp, nullptr);
            }
    }
    populate_edges();
    if (failures) {
        std::fprintf(stderr, "%d of %d checks failed\n", failures, checks);
        return 1;
    }
    std::printf("%d checks passed\n", checks);
    return 0;
}
