// host_fill_bw.cpp — A/B tool: host write bandwidth of a background fill into
// page-locked memory (the host half of a compact image copy), persistent
// threads, NT vs plain stores, unpinned / spread / packed thread placement.
//   g++ -O3 -mavx2 -o /tmp/host_fill_bw scripts/host_fill_bw.cpp -lpthread
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static void fill_nt(float *p, size_t nfl, const float *pat) {
    const __m256 a = _mm256_loadu_ps(pat), b = _mm256_loadu_ps(pat + 8), c = _mm256_loadu_ps(pat + 16);
    for (size_t i = 0; i + 24 <= nfl; i += 24) {
        _mm256_stream_ps(p + i, a);
        _mm256_stream_ps(p + i + 8, b);
        _mm256_stream_ps(p + i + 16, c);
    }
    _mm_sfence();
}
static void fill_plain(float *p, size_t nfl, const float *pat) {
    for (size_t i = 0; i + 24 <= nfl; i += 24) std::memcpy(p + i, pat, 96);
}

int main(int argc, char **argv) {
    const size_t bytes = 21u << 20;
    const int maxT = argc > 1 ? atoi(argv[1]) : 16;
    float *p = (float *)aligned_alloc(4096, bytes);
    memset(p, 1, bytes);
    mlock(p, bytes);
    float pat[24];
    for (int i = 0; i < 24; ++i) pat[i] = (i % 3 == 1) ? 0.5f : 0.0f;
    const size_t nfl = bytes / 4 / 24 * 24;
    cpu_set_t all;
    sched_getaffinity(0, sizeof all, &all);
    std::vector<int> cpus;
    for (int c = 0; c < CPU_SETSIZE; ++c)
        if (CPU_ISSET(c, &all)) cpus.push_back(c);
    printf("affinity cpus %zu, hw %u\n", cpus.size(), std::thread::hardware_concurrency());
    for (int place = 0; place < 3; ++place)
        for (int mode = 0; mode < 2; ++mode)
            for (int T = 1; T <= maxT; T *= 2) {
                std::atomic<int> go{0}, done{0};
                std::atomic<bool> stop{false};
                std::vector<std::thread> th;
                const size_t per = nfl / T / 24 * 24;
                for (int k = 0; k < T; ++k)
                    th.emplace_back([&, k]() {
                        if (place > 0) {
                            cpu_set_t s;
                            CPU_ZERO(&s);
                            const size_t idx = place == 1 ? (size_t)k * cpus.size() / T : (size_t)k;
                            CPU_SET(cpus[idx % cpus.size()], &s);
                            sched_setaffinity(0, sizeof s, &s);
                        }
                        int seen = 0;
                        while (!stop.load()) {
                            const int g = go.load(std::memory_order_acquire);
                            if (g == seen) { _mm_pause(); continue; }
                            seen = g;
                            const size_t n = k == T - 1 ? nfl - per * k : per;
                            if (mode == 0) fill_nt(p + per * k, n, pat); else fill_plain(p + per * k, n, pat);
                            done.fetch_add(1, std::memory_order_acq_rel);
                        }
                    });
                double best = 1e9, sum = 0;
                const int reps = 30;
                for (int r = 0; r < reps; ++r) {
                    done.store(0);
                    const auto t0 = std::chrono::steady_clock::now();
                    go.fetch_add(1, std::memory_order_acq_rel);
                    while (done.load(std::memory_order_acquire) < T) _mm_pause();
                    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                    best = s < best ? s : best;
                    sum += s;
                }
                stop = true;
                for (auto &x : th) x.join();
                printf("%-7s %-5s T=%2d best %7.1f us (%6.1f GB/s)  mean %7.1f us\n",
                       place == 0 ? "free" : place == 1 ? "spread" : "packed", mode ? "plain" : "nt", T, best * 1e6,
                       bytes / best / 1e9, sum / reps * 1e6);
            }
    return 0;
}
