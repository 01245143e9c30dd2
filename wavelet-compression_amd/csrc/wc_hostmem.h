// wc_hostmem.h — host-memory side of the _host entry points (wc_forward_host,
// wc_inverse_host): the pages of a caller's output range are made resident
// before a device-to-host copy lands in them.
//
// Why (profiles/r04/experiments/gpu_pcie.txt): a copy into pageable memory
// that was never touched (a new std::vector, np.empty) pays the page faults on
// the copy's own thread — 0.65 GB of C2 payloads land at 12–20 GB/s instead of
// the link's 57 GB/s, 1.07 GB of boxes at 14–18 GB/s.  Faulting the same
// range in advance from several threads, with transparent huge pages advised
// on it, takes 4 ms for 1.07 GB at 16 threads, and the copy then runs at the
// link rate.  Plain C++: no HIP, so the pool is tested under ThreadSanitizer
// on the CPU (tests/cpp/test_hostmem.cpp).
#pragma once
#include <condition_variable>
#include <cstddef>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace wc {

// A fixed set of worker threads that run one job at a time: run(n, fn) calls
// fn(0) … fn(n - 1) spread over the workers and the calling thread and
// returns when all have returned.  Not reentrant; one caller at a time (the
// context's host entry points are not called concurrently on one context).
class HostPool {
public:
    explicit HostPool(int threads);  // workers besides the caller (>= 0)
    ~HostPool();
    HostPool(const HostPool&) = delete;
    HostPool& operator=(const HostPool&) = delete;
    void run(int ntasks, const std::function<void(int)>& fn);
    int threads() const { return (int)workers_.size() + 1; }

private:
    void work();
    bool take(int& task);
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable wake_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    int ntasks_ = 0, next_ = 0, finished_ = 0;
    unsigned long long gen_ = 0;
    bool stop_ = false;
};

// Progress of a pipelined _host call's runs, published by one thread and
// awaited by another: a copy from or to pageable host memory returns only
// when it is done, so the uploads (the call's thread) and the downloads (a
// helper thread) of different runs overlap only from different threads.
class RunGate {
public:
    void publish(int runs) {  // runs [0, runs) are queued
        {
            std::lock_guard<std::mutex> lk(mu_);
            done_ = runs;
        }
        cv_.notify_all();
    }
    void cancel() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            cancelled_ = true;
        }
        cv_.notify_all();
    }
    bool wait(int r) {  // false: cancelled before run r was published
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return done_ > r || cancelled_; });
        return done_ > r;
    }

private:
    std::mutex mu_;
    std::condition_variable cv_;
    int done_ = 0;
    bool cancelled_ = false;
};

// Make every whole page of [p, p + bytes) resident and writable without
// changing a byte (MADV_POPULATE_WRITE; on kernels without it, a read and a
// write-back of one byte per page, so the range must not be written
// concurrently).  thp: advise transparent huge pages on the 2-MiB-aligned
// interior first.  pool may be null (the calling thread does it all).  Every
// failure is ignored: this only moves the faults off the copy's thread.
void populate_for_write(HostPool* pool, void* p, size_t bytes, bool thp);

// Tests only: take the pre-5.14 path (read + write-back per page) always.
void populate_force_touch(bool on);

}  // namespace wc
