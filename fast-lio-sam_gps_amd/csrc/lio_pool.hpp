// lio_pool.hpp — a small persistent host worker pool for the host halves of the uploads (sweep packing,
// ICP cloud staging): a copy split over a few threads without creating threads per call.  Workers sleep
// on a condition variable between jobs; the caller runs a share of every job itself.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace lio {

class HostPool {
  public:
    static HostPool& get() {
        // + the calling thread: 4 share a job by default; LIO_HOST_THREADS (1..16) sets the total (A/B)
        static HostPool pool([] {
            const char* e = std::getenv("LIO_HOST_THREADS");
            const int t = e ? std::atoi(e) : 4;
            return (t >= 1 && t <= 16 ? t : 4) - 1;
        }());
        return pool;
    }
    int threads() const { return (int)workers_.size() + 1; }
    // fn(i) for i in [0, n), spread over the workers and the caller; returns when every index has run and
    // no worker holds the job any more.  Calls from several threads at once run one job at a time.
    void parallel_for(int n, const std::function<void(int)>& fn) {
        if (n <= 0) return;
        if (n == 1 || workers_.empty()) {
            for (int i = 0; i < n; ++i) fn(i);
            return;
        }
        std::lock_guard<std::mutex> one_job(job_mu_);
        Job job;
        job.fn = &fn;
        job.n = n;
        job.left = n;
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &job;
            ++gen_;
        }
        cv_.notify_all();
        run(job);
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return job.left == 0 && job.users == 0; });
        job_ = nullptr;
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread& t : workers_) t.join();
    }

  private:
    struct Job {
        const std::function<void(int)>* fn = nullptr;
        int n = 0;
        std::atomic<int> next{0};
        int left = 0;   // indices not finished (under mu_)
        int users = 0;  // workers holding the job (under mu_)
    };
    explicit HostPool(int nw) {
        for (int w = 0; w < nw; ++w) workers_.emplace_back([this] { loop(); });
    }
    void run(Job& j) {
        for (;;) {
            const int i = j.next.fetch_add(1, std::memory_order_relaxed);
            if (i >= j.n) return;
            (*j.fn)(i);
            std::lock_guard<std::mutex> lk(mu_);
            if (--j.left == 0) done_cv_.notify_all();
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            Job* j;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || (job_ && gen_ != seen); });
                if (stop_) return;
                seen = gen_;
                j = job_;
                ++j->users;
            }
            run(*j);
            std::lock_guard<std::mutex> lk(mu_);
            if (--j->users == 0 && j->left == 0) done_cv_.notify_all();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex job_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    Job* job_ = nullptr;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace lio
