// gather_pool.h — the host context's gather workers (csum_ctx.cpp).
//
// Header-only so that tests/sanitize/pool_san.cpp can run it under TSan and
// ASan on the CPU, without the HIP runtime.
#pragma once

#include <pthread.h>
#include <stdint.h>

#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace lvlip {

// The context's gather workers, started on first use and kept until the
// context is destroyed, so that a piece of a few hundred KB can be gathered
// by several threads (a std::thread start costs more than copying 1 MB).
// Only the context's owning thread submits work.
class GatherPool {
   public:
    ~GatherPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_job_.notify_all();
        for (auto& t : th_) t.join();
    }
    // fn(0 .. parts-1), part 0 on the calling thread; returns when all are done.
    // Workers that cannot be started (std::thread throws std::system_error
    // under a thread limit) are not an error: their parts run on the calling
    // thread after part 0, so the call still completes (never std::terminate
    // through the C ABI).
    void run(int parts, const std::function<void(int)>& fn) {
        if (parts <= 1) {
            fn(0);
            return;
        }
        while ((int)th_.size() < parts - 1) {
            // a new worker waits for the generation after the current one (this
            // thread is gen_'s only writer, so it may read it unlocked)
            const int id = (int)th_.size() + 1;
            const uint64_t g0 = gen_;
            try {
                th_.emplace_back([this, id, g0] { worker(id, g0); });
            } catch (const std::exception&) {
                break;
            }
        }
        const int w = (int)th_.size() < parts - 1 ? (int)th_.size() : parts - 1;  // parts 1..w
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &fn;
            parts_ = w + 1;
            pending_ = w;
            ++gen_;
        }
        cv_job_.notify_all();
        fn(0);
        for (int p = w + 1; p < parts; ++p) fn(p);
        std::unique_lock<std::mutex> g(m_);
        cv_done_.wait(g, [this] { return pending_ == 0; });
        job_ = nullptr;
    }

   private:
    void worker(int id, uint64_t seen) {
        // named, so per-thread CPU accounting (/proc/<pid>/task/*/comm) can
        // tell the gather workers from the caller and the HIP runtime's threads
        pthread_setname_np(pthread_self(), "lvlip-gather");
        std::unique_lock<std::mutex> g(m_);
        for (;;) {
            cv_job_.wait(g, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            if (id >= parts_) continue;
            const std::function<void(int)>* job = job_;
            g.unlock();
            (*job)(id);
            g.lock();
            if (--pending_ == 0) cv_done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_job_, cv_done_;
    const std::function<void(int)>* job_ = nullptr;
    uint64_t gen_ = 0;
    int parts_ = 0, pending_ = 0;
    bool stop_ = false;
};

}  // namespace lvlip
