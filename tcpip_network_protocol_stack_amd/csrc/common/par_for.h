// par_for.h — not installed.  Split [0, n) into `threads` contiguous ranges and
// run fn(i0, i1) on each, the first range on the calling thread.  Exception
// safe: every worker thread that started is joined on every path, and an
// exception thrown inside fn is carried out and rethrown on the calling thread
// after the join, instead of terminating the process.  A range whose thread
// fails to start (EAGAIN) runs on the calling thread instead — the work is
// done, so that is not an error.
#pragma once

#include <cstddef>
#include <exception>
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

}  // namespace icsum::detail
