// host_pool.h -- a few parked host threads for the per-call O(n) scans over the caller's
// arrays (read lengths, amplicon indices).  One thread reads ~13 GB/s from host memory:
// the length scan of a 1M-read call took 0.6 ms of its 2.9 ms on one core.
//
// One job at a time per process; a caller that finds the pool busy (another context's
// call on another host thread), or a forked child (the threads stayed in the parent),
// runs the parts itself.
#pragma once

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <unistd.h>

namespace nw_host {

class Pool {
public:
    // The process-wide pool: CRISPR_NW_HOST_THREADS (default min(16, cores): a GPU box gives a
    // process 16 CPUs; the FASTQ ingest parses and inflates on all of them) threads in
    // all, the caller included.  Never destroyed: parked threads end with the process.
    static Pool& get() {
        static Pool* p = [] {
            int nt = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
            if (const char* e = std::getenv("CRISPR_NW_HOST_THREADS")) nt = std::max(1, std::min(64, std::atoi(e)));
            return new Pool(nt);
        }();
        return *p;
    }

    int threads() const { return nt_; }

    // f(part) for part in [0, parts), parts <= threads(); the caller runs part 0.
    void run(int parts, const std::function<void(int)>& f) {
        parts = std::max(1, std::min(parts, nt_));
        std::unique_lock<std::mutex> busy(call_m_, std::try_to_lock);
        if (parts == 1 || !busy.owns_lock() || getpid() != pid_) {
            for (int q = 0; q < parts; ++q) f(q);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &f;
            parts_ = parts;
            remaining_ = nt_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [&] { return remaining_ == 0; });
        job_ = nullptr;
    }

    // [lo, hi) of part q of n items split in `parts`
    static void range(int64_t n, int parts, int q, int64_t* lo, int64_t* hi) {
        *lo = n * q / parts;
        *hi = n * (q + 1) / parts;
    }

private:
    explicit Pool(int nt) : nt_(nt), pid_(getpid()) {
        for (int i = 1; i < nt_; ++i) std::thread([this, i] { worker(i); }).detach();
    }

    void worker(int id) {
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(m_);
            cv_.wait(lk, [&] { return gen_ != seen; });
            seen = gen_;
            const std::function<void(int)>* f = job_;
            const int parts = parts_;
            lk.unlock();
            if (id < parts) (*f)(id);
            lk.lock();
            if (--remaining_ == 0) done_.notify_one();
        }
    }

    int nt_;
    pid_t pid_;
    std::mutex call_m_, m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    int parts_ = 0, remaining_ = 0;
    uint64_t gen_ = 0;
};

}  // namespace nw_host
