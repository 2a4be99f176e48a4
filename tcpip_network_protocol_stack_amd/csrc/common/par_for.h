// par_for.h — not installed.  Split [0, n) into `threads` contiguous ranges and
// run fn(i0, i1) on each, the first range on the calling thread.  Exception
// safe: every worker thread that started is joined on every path, and an
// exception thrown inside fn is carried out and rethrown on the calling thread
// after the join, instead of terminating the process.  A range whose thread
// fails to start (EAGAIN) runs on the calling thread instead — the work is
// done, so that is not an error.
#pragma once

#include <algorithm>
#include <condition_variable>
#include <cstddef>
#include <exception>
#include <functional>
#include <mutex>
#include <system_error>
#include <thread>
#include <vector>

namespace icsum::detail {

template <typename Fn>
void parallel_ranges(size_t n, size_t threads, Fn&& fn)
{
    if (threads <= 1 || n < 2) {
        fn(size_t(0), n);
        return;
    }
    std::exception_ptr err{};
    std::mutex mu{};
    auto guarded = [&](size_t i0, size_t i1) {
        try {
            fn(i0, i1);
        } catch (...) {
            std::lock_guard<std::mutex> lock(mu);
            if (!err) err = std::current_exception();
        }
    };
    std::vector<std::thread> pool{};
    pool.reserve(threads - 1);
    try {
        for (size_t t = 1; t < threads; ++t) pool.emplace_back(guarded, n * t / threads, n * (t + 1) / threads);
    } catch (const std::system_error&) {  // a thread failed to start: the caller runs what is left
    }
    // ranges whose thread did not start run here
    for (size_t t = pool.size() + 1; t < threads; ++t) guarded(n * t / threads, n * (t + 1) / threads);
    guarded(0, n / threads);
    for (auto& th : pool) th.join();
    if (err) std::rethrow_exception(err);
}

// A fixed set of worker threads for repeated parallel_ranges-style jobs (the
// host pipeline's staging copies run one per 32 MiB chunk: starting and
// joining threads for each would cost a good part of a chunk's copy time).
// run() splits [0, n) into `parts` contiguous ranges, the first on the calling
// thread, waits for all of them and rethrows the first exception a range
// threw.  Workers that fail to start leave a smaller pool; one caller at a
// time (the owner serialises its calls).
class WorkerPool {
public:
    explicit WorkerPool(size_t workers)
    {
        try {
            for (size_t i = 0; i < workers; ++i) threads_.emplace_back([this] { loop(); });
        } catch (const std::system_error&) {  // fewer workers; run() adapts
        }
    }
    ~WorkerPool()
    {
        {
            std::lock_guard<std::mutex> lock(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : threads_) t.join();
    }
    WorkerPool(const WorkerPool&) = delete;
    WorkerPool& operator=(const WorkerPool&) = delete;

    size_t workers() const { return threads_.size(); }

    template <typename Fn>
    void run(size_t n, size_t parts, Fn&& fn)
    {
        parts = std::min(parts, threads_.size() + 1);
        if (parts <= 1 || n < 2) {
            fn(size_t(0), n);
            return;
        }
        std::function<void(size_t, size_t)> job(std::ref(fn));
        {
            std::lock_guard<std::mutex> lock(mu_);
            job_ = &job;
            n_ = n;
            parts_ = parts;
            next_ = 1;
            pending_ = parts - 1;
            err_ = nullptr;
        }
        cv_.notify_all();
        std::exception_ptr mine{};
        try {
            fn(size_t(0), n / parts);
        } catch (...) {
            mine = std::current_exception();
        }
        std::unique_lock<std::mutex> lock(mu_);
        done_.wait(lock, [this] { return pending_ == 0; });
        job_ = nullptr;
        if (mine) std::rethrow_exception(mine);
        if (err_) std::rethrow_exception(err_);
    }

private:
    void loop()
    {
        std::unique_lock<std::mutex> lock(mu_);
        for (;;) {
            cv_.wait(lock, [this] { return stop_ || next_ < parts_; });
            if (stop_) return;
            const size_t r = next_++;
            const size_t i0 = n_ * r / parts_, i1 = n_ * (r + 1) / parts_;
            auto* job = job_;
            lock.unlock();
            try {
                (*job)(i0, i1);
            } catch (...) {
                std::lock_guard<std::mutex> g(mu_);
                if (!err_) err_ = std::current_exception();
            }
            lock.lock();
            if (--pending_ == 0) done_.notify_all();
        }
    }

    std::vector<std::thread> threads_{};
    std::mutex mu_{};
    std::condition_variable cv_{}, done_{};
    std::function<void(size_t, size_t)>* job_ = nullptr;
    size_t n_ = 0, parts_ = 0, next_ = 0, pending_ = 0;
    std::exception_ptr err_{};
    bool stop_ = false;
};

}  // namespace icsum::detail
