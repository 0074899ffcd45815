// sv_pool.h — a small process-wide host thread pool for the host-buffer entry points
// (staging copies into pinned memory and the table expansion of the outputs).
//
// parallel_for(n, fn) runs fn(i) for i in [0, n) on the pool and on the calling thread,
// and returns when all have finished; calls from several threads (one per context) share
// the pool.  Worker count: SV_HOST_THREADS, else min(8, the CPUs this process may use).
#pragma once

#include <sched.h>

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace sv {

class HostPool {
public:
    static HostPool& get() {
        static HostPool* p = new HostPool();   // never destroyed: workers may outlive main's statics
        return *p;
    }

    int threads() const { return (int)workers_.size() + 1; }

    // fn(i) for i in [0, n); the caller participates.  Exceptions must not escape fn.
    void parallel_for(int n, const std::function<void(int)>& fn) {
        if (n <= 0) return;
        if (n == 1 || workers_.empty()) {
            for (int i = 0; i < n; ++i) fn(i);
            return;
        }
        Job job;
        job.fn = &fn;
        job.n = n;
        {
            std::lock_guard<std::mutex> lk(mu_);
            jobs_.push_back(&job);
        }
        cv_.notify_all();
        run(job);
        std::unique_lock<std::mutex> lk(mu_);
        // every index finished and no worker still holds the job (it lives on this stack)
        done_cv_.wait(lk, [&] { return job.finished.load() == job.n && job.active == 0; });
        for (auto it = jobs_.begin(); it != jobs_.end(); ++it)
            if (*it == &job) {
                jobs_.erase(it);
                break;
            }
    }

private:
    struct Job {
        const std::function<void(int)>* fn = nullptr;
        int n = 0;
        std::atomic<int> next{0};
        std::atomic<int> finished{0};
        int active = 0;   // workers inside run(), guarded by mu_
    };

    HostPool() {
        int nt = 0;
        if (const char* e = std::getenv("SV_HOST_THREADS")) nt = std::atoi(e);
        if (nt <= 0) {
            cpu_set_t set;
            int cpus = 0;
            if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = CPU_COUNT(&set);
            if (cpus <= 0) cpus = (int)std::thread::hardware_concurrency();
            nt = cpus < 8 ? cpus : 8;
        }
        if (nt < 1) nt = 1;
        try {
            for (int i = 0; i + 1 < nt; ++i) workers_.emplace_back([this] { loop(); });
        } catch (...) {   // fewer workers: parallel_for still completes on the caller
        }
        for (auto& t : workers_) t.detach();
    }

    // Claim and run indices of `job` until none is left.
    void run(Job& job) {
        for (;;) {
            const int i = job.next.fetch_add(1);
            if (i >= job.n) return;
            (*job.fn)(i);
            if (job.finished.fetch_add(1) + 1 == job.n) {
                std::lock_guard<std::mutex> lk(mu_);
                done_cv_.notify_all();
            }
        }
    }

    void loop() {
        for (;;) {
            Job* job = nullptr;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] {
                    for (Job* j : jobs_)
                        if (j->next.load() < j->n) return true;
                    return false;
                });
                for (Job* j : jobs_)
                    if (j->next.load() < j->n) {
                        job = j;
                        ++job->active;
                        break;
                    }
            }
            if (!job) continue;
            run(*job);
            std::lock_guard<std::mutex> lk(mu_);
            --job->active;
            done_cv_.notify_all();
        }
    }

    std::vector<std::thread> workers_;
    std::deque<Job*> jobs_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
};

}  // namespace sv
