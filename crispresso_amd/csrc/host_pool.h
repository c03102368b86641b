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
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <sched.h>
#include <unistd.h>

namespace nw_host {

// The host threads this process may use: CRISPR_NW_HOST_THREADS when set (the rank binder,
// crispresso_amd/placement.py, sets it to the size of the rank's CPU slice), else the CPUs of
// the process's affinity mask capped by the cgroup CPU quota (a GPU box shows the whole
// machine -- 256 CPUs -- to sched_getaffinity and hardware_concurrency but gives a job 16 of
// them), divided among the node's ranks (LOCAL_WORLD_SIZE: 8 processes of one node must not
// each start a pool sized for all of it), at most 64.
inline int default_threads() {
    if (const char* e = std::getenv("CRISPR_NW_HOST_THREADS")) return std::max(1, std::min(64, std::atoi(e)));
    int cpus = 0;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = CPU_COUNT(&set);
    if (cpus <= 0) cpus = (int)std::max(1u, std::thread::hardware_concurrency());
    double quota = 0;
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {   // cgroup v2: "<quota|max> <period>"
        char q[32] = {0};
        long per = 0;
        if (std::fscanf(f, "%31s %ld", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0)
            quota = std::atof(q) / (double)per;
        std::fclose(f);
    } else if (FILE* g = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {   // cgroup v1
        long q = -1, per = 0;
        if (std::fscanf(g, "%ld", &q) != 1) q = -1;
        std::fclose(g);
        if (FILE* h = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
            if (std::fscanf(h, "%ld", &per) != 1) per = 0;
            std::fclose(h);
        }
        if (q > 0 && per > 0) quota = (double)q / (double)per;
    }
    if (quota >= 1.0) cpus = std::min(cpus, (int)quota);
    int ranks = 1;
    if (const char* e = std::getenv("LOCAL_WORLD_SIZE")) ranks = std::max(1, std::atoi(e));
    return std::max(1, std::min(64, cpus / ranks));
}

class Pool {
public:
    // The process-wide pool: default_threads() threads in all, the caller included (the FASTQ
    // ingest parses and inflates on all of them).  Never destroyed: parked threads end with
    // the process.
    static Pool& get() {
        static Pool* p = new Pool(default_threads());
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
