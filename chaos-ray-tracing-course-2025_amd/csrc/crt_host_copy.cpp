/*
 * crt_host_copy.cpp — the host half of crt_hip_render's image copy
 * (crt_api.hip image_to_host).
 *
 * render_image returns a host fp32 image (crt_image.h:11-27; the CLI times the
 * whole call, main.cpp:37-43).  A 1920x1080 frame is 24.9 MB; over PCIe that
 * is ~0.46 ms, eight times the render.  Most of a course frame is background
 * (the miss colour, crt_renderer.cpp:142-144), so only each row's span of
 * non-background pixels crosses PCIe and the host writes the background
 * itself, on a few persistent threads, while the GPU renders.
 */
#include <emmintrin.h>
#include <xmmintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "crt_host.h"

namespace crt_amd {

/* Plain (cached) stores: a caller that renders frame after frame into one
 * buffer finds it in the host's L3 (the GPU box's EPYC: 32 MB per CCD), where
 * plain stores run at 100 GB/s a thread and streaming ones at 50
 * (scripts/host_fill_bw.cpp, gpurun_out r06/fill_bw.txt). */
void fill_background(float *dst, int64_t n, const float bg[3]) {
    if (n <= 0) return;
    int64_t nf = 3 * n;
    const float pat[12] = {bg[0], bg[1], bg[2], bg[0], bg[1], bg[2], bg[0], bg[1], bg[2], bg[0], bg[1], bg[2]};
    const __m128 a = _mm_loadu_ps(pat), b = _mm_loadu_ps(pat + 4), c = _mm_loadu_ps(pat + 8);
    /* 48 B (four pixels) per round */
    while (nf >= 12) {
        _mm_storeu_ps(dst, a);
        _mm_storeu_ps(dst + 4, b);
        _mm_storeu_ps(dst + 8, c);
        dst += 12;
        nf -= 12;
    }
    for (int64_t i = 0; i < nf; ++i) dst[i] = pat[i];
}

void store_fence() { _mm_sfence(); }

/* ---- HostPool ---- */

struct HostPool::Impl {
    struct Worker {
        std::atomic<uint64_t> go{0}, done{0};
        std::thread th;
    };
    std::vector<Worker> workers;
    std::mutex run_mu;                 /* one job at a time */
    std::mutex sleep_mu;
    std::condition_variable sleep_cv;
    std::atomic<bool> stop{false};
    uint64_t gen = 0;
    void (*fn)(void *, int) = nullptr;
    void *arg = nullptr;
    int n = 0;

    explicit Impl(int nw) : workers((size_t)nw) {}

    void loop(int slot) {
        Worker &w = workers[(size_t)slot - 1];
        uint64_t seen = 0;
        const int T = (int)workers.size() + 1;
        for (;;) {
            /* spin ~0.5 ms for the next job, then sleep */
            const auto t0 = std::chrono::steady_clock::now();
            int polls = 0;
            while (w.go.load(std::memory_order_acquire) == seen) {
                if (stop.load(std::memory_order_relaxed)) return;
                _mm_pause();
                if (++polls == 256) {
                    polls = 0;
                    if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(500)) {
                        std::unique_lock<std::mutex> l(sleep_mu);
                        sleep_cv.wait(l, [&]() { return stop.load() || w.go.load(std::memory_order_acquire) != seen; });
                    }
                }
            }
            if (stop.load()) return;
            seen = w.go.load(std::memory_order_acquire);
            for (int i = slot; i < n; i += T) fn(arg, i);
            w.done.store(seen, std::memory_order_release);
        }
    }
};

HostPool::HostPool(int nw) : impl_(new Impl(std::max(0, nw))) {
    for (size_t i = 0; i < impl_->workers.size(); ++i)
        impl_->workers[i].th = std::thread([this, i]() { impl_->loop((int)i + 1); });
}

HostPool::~HostPool() {
    impl_->stop = true;
    {
        std::lock_guard<std::mutex> g(impl_->sleep_mu);
    }
    impl_->sleep_cv.notify_all();
    for (auto &w : impl_->workers) w.th.join();
    delete impl_;
}

HostPool &HostPool::get() {
    /* seven workers + the caller: a frame's copy needs a few host threads'
     * store bandwidth, not a machine's (the box grants 16 CPUs) */
    static HostPool pool((int)std::min(7u, std::max(1u, std::thread::hardware_concurrency()) - 1));
    return pool;
}

int HostPool::threads() const { return (int)impl_->workers.size() + 1; }

void HostPool::run(int n, void (*fn)(void *, int), void *arg) {
    std::lock_guard<std::mutex> one(impl_->run_mu);
    Impl &I = *impl_;
    const int T = (int)I.workers.size() + 1;
    I.fn = fn;
    I.arg = arg;
    I.n = n;
    const uint64_t g = ++I.gen;
    const int used = std::min(T, n) - 1;   /* workers with a task */
    for (int k = 0; k < used; ++k) I.workers[(size_t)k].go.store(g, std::memory_order_release);
    if (used > 0) {
        std::lock_guard<std::mutex> l(I.sleep_mu);
    }
    if (used > 0) I.sleep_cv.notify_all();
    for (int i = 0; i < n; i += T) fn(arg, i);
    for (int k = 0; k < used; ++k)
        while (I.workers[(size_t)k].done.load(std::memory_order_acquire) != g) _mm_pause();
}

}  // namespace crt_amd
