// write_behind.cpp — opt-in write-behind of compress()'s .xz files.
//
// The reference's compress() (src/compressor.cpp:250-291) encodes and writes
// each component's file before it returns, and its -c loop calls it once per
// box (src/modes.cpp:100-103): only the box's few components can encode at
// once, so the drop-in -c is bound by one xz stream per component per box.
// With write-behind on ($WCAMD_WRITE_BEHIND=1 or set_write_behind(true)),
// compress() hands each component's serialized payload to this process-wide
// queue and returns; host_threads() workers encode and write the files while
// the caller's loop moves on to the next boxes.  Every file is complete, with
// the bytes compress() would have written, by the time
//   * flush_writes() returns (explicit),
//   * decompress() reads it (it waits for that file's pending writes only:
//     -estimate reads what -c wrote), or
//   * the process exits normally (an atexit handler drains the queue; the
//     queue itself is never destroyed, so a thread still blocked in submit()
//     at exit never waits on a destroyed condition variable).
// A file that cannot be opened is skipped, as in compress(); an encoder
// failure (compress() would log and exit) is logged and exits the process from
// the next flush, or at exit, once every other queued file is written (a
// worker never exits the process itself: exit would wait on the queue it
// holds).  The queued bytes are bounded ($WCAMD_WRITE_BEHIND_MB, default 2048): submit() waits while the
// queue holds more.
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <fstream>
#include <filesystem>
#include <mutex>
#include <thread>
#include <unordered_map>

#include "host_ctx.h"
#include "wavelet_amd/xz_pool.h"

namespace wavelet_amd {

namespace {

std::atomic<int> g_on{-1};  // -1: not chosen yet ($WCAMD_WRITE_BEHIND)

struct Job {
    std::string payload;
    std::string path;
    std::string key;  // path_key(path)
};

// A queued file's key: its absolute, lexically normal path (compress() joins
// std::filesystem paths, the -d loop concatenates strings).
std::string path_key(const std::string& p) {
    std::error_code ec;
    std::filesystem::path a = std::filesystem::absolute(p, ec);
    return (ec ? std::filesystem::path(p) : a).lexically_normal().string();
}

class Writer {
public:
    Writer() {
        const char* mb = std::getenv("WCAMD_WRITE_BEHIND_MB");
        const long v = mb ? std::atol(mb) : 0;
        limit_ = (uint64_t)(v > 0 ? v : 2048) << 20;
        const int n = std::max(1, host_threads());
        // detached: the Writer lives until the process ends (writer())
        for (int i = 0; i < n; ++i) std::thread([this] { run(); }).detach();
    }
    // At exit (atexit handler): every queued file written; an encoder failure
    // reported, failing the process as compress() would have.
    void at_exit() {
        drain();
        std::lock_guard<std::mutex> lk(mu_);
        if (!error_.empty()) {
            std::fprintf(stderr, "[error] %s\n", error_.c_str());
            std::_Exit(EXIT_FAILURE);
        }
    }
    void submit(std::string payload, std::string path) {
        std::unique_lock<std::mutex> lk(mu_);
        const uint64_t b = payload.size();
        // one job larger than the bound still goes in once the queue is empty
        room_.wait(lk, [&] { return queued_ == 0 || queued_ + b <= limit_; });
        queued_ += b;
        ++pending_;
        std::string key = path_key(path);
        ++paths_[key];
        q_.push_back(Job{std::move(payload), std::move(path), std::move(key)});
        lk.unlock();
        work_.notify_one();
    }
    // Every queued file (path empty), or only `path`'s pending writes.
    void flush(const std::string* path = nullptr) {
        std::string e;
        {
            std::unique_lock<std::mutex> lk(mu_);
            ++waiters_;
            if (path) {
                const std::string key = path_key(*path);
                done_.wait(lk, [&] { return paths_.find(key) == paths_.end(); });
                // a file queued under another spelling (e.g. relative to a working
                // directory that has changed since) is not found by its key: if the
                // file is not there yet, drain everything
                std::error_code ec;
                if (pending_ != 0 && !std::filesystem::exists(*path, ec))
                    done_.wait(lk, [&] { return pending_ == 0; });
            } else {
                done_.wait(lk, [&] { return pending_ == 0; });
            }
            --waiters_;
            e = error_;
        }
        if (!e.empty()) fatal(e);
    }

private:
    void drain() {
        std::unique_lock<std::mutex> lk(mu_);
        ++waiters_;
        done_.wait(lk, [&] { return pending_ == 0; });
        --waiters_;
    }
    void run() {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> lk(mu_);
                work_.wait(lk, [&] { return !q_.empty(); });
                j = std::move(q_.front());
                q_.pop_front();
            }
            const char* err = nullptr;
            {
                std::ofstream f(j.path, std::ios::binary);
                std::string xz;
                if (f.is_open()) {  // the reference skips a file it cannot open (src/compressor.cpp:256-257)
                    if (xz_encode_try(reinterpret_cast<const uint8_t*>(j.payload.data()), j.payload.size(), xz, err))
                        f.write(xz.data(), (std::streamsize)xz.size());
                }
            }
            bool wake;
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (err && error_.empty()) error_ = std::string(err) + ": " + j.path;
                queued_ -= j.payload.size();
                --pending_;
                auto it = paths_.find(j.key);
                if (it != paths_.end() && --it->second == 0) paths_.erase(it);
                wake = waiters_ != 0;
            }
            if (wake) done_.notify_all();  // a full flush or a one-file wait may be done
            room_.notify_all();
        }
    }

    std::mutex mu_;
    std::condition_variable work_, room_, done_;
    std::deque<Job> q_;
    uint64_t queued_ = 0, limit_ = 0;
    size_t pending_ = 0;  // queued + being written
    std::unordered_map<std::string, size_t> paths_;  // path_key -> its queued + in-progress writes
    size_t waiters_ = 0;  // threads in flush() / drain()
    std::string error_;   // the first encoder failure
};

Writer& writer() {
    // never destroyed (its workers and condition variables outlive every
    // caller); drained by an atexit handler registered after it is built, so
    // it runs before the destructors of statics built earlier
    static Writer* w = [] {
        Writer* p = new Writer();
        std::atexit([] { writer().at_exit(); });
        return p;
    }();
    return *w;
}

}  // namespace

bool write_behind() {
    int v = g_on.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* e = std::getenv("WCAMD_WRITE_BEHIND");
        v = e && *e && std::string(e) != "0" ? 1 : 0;
        int expect = -1;
        g_on.compare_exchange_strong(expect, v);
        v = g_on.load(std::memory_order_relaxed);
    }
    return v == 1;
}

void set_write_behind(bool on) {
    if (!on) flush_writes();
    g_on.store(on ? 1 : 0, std::memory_order_relaxed);
}

void write_behind_submit(std::string payload, std::string path) { writer().submit(std::move(payload), std::move(path)); }

static std::atomic<bool> g_used{false};

void flush_writes() {
    if (g_used.load(std::memory_order_acquire)) writer().flush();
}

void flush_writes(const std::string& path) {
    if (g_used.load(std::memory_order_acquire)) writer().flush(&path);
}

void note_write_behind_used() { g_used.store(true, std::memory_order_release); }

}  // namespace wavelet_amd
