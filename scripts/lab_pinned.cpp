// Lab: host-side access costs of the context's pinned buffers (hipHostMalloc)
// against malloc'd memory, one thread: big memcpy in, sequential reads, and the
// frame gather's pattern (40K ~800-B copies into 16-B slots, slot offsets read
// from a descriptor array in pinned or in malloc'd memory).
//   hipcc -O2 -std=c++17 -o scripts/lab_pinned scripts/lab_pinned.cpp   (git-ignored)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <thread>
#include <vector>

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Desc { uint64_t off; uint32_t len, pad; };

int main() {
    const size_t B = 64u << 20, half = 32u << 20;
    uint8_t* src = (uint8_t*)malloc(B);
    uint8_t* heap = (uint8_t*)malloc(B);
    memset(src, 1, B);
    memset(heap, 2, B);
    uint8_t* pin = nullptr;
    uint8_t* pin_wc = nullptr;
    if (hipHostMalloc((void**)&pin, B, hipHostMallocDefault) != hipSuccess) return 2;
    if (hipHostMalloc((void**)&pin_wc, B, hipHostMallocWriteCombined) != hipSuccess) return 2;
    memset(pin, 3, B);
    memset(pin_wc, 3, B);
    const uint32_t n = 40000;
    std::vector<Desc> d(n);
    uint64_t o = 0, so = 0;
    std::vector<uint64_t> soff(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t len = 48 + (uint32_t)((i * 2654435761u) % 1440u);
        d[i] = {o, len, 0};
        soff[i] = so;
        o = (o + len + 15) & ~15ull;
        so += len;
    }
    Desc* dpin = nullptr;
    hipHostMalloc((void**)&dpin, n * sizeof(Desc), hipHostMallocDefault);
    memcpy(dpin, d.data(), n * sizeof(Desc));
    struct T { const char* name; uint8_t* dst; };
    for (int rep = 0; rep < 3; ++rep) {
        for (T t : {T{"heap", heap}, T{"pinned", pin}, T{"pinned_wc", pin_wc}}) {
            double t0 = now_ms();
            memcpy(t.dst, src, half);
            const double cp = now_ms() - t0;
            t0 = now_ms();
            uint64_t acc = 0;
            const uint64_t* p = (const uint64_t*)t.dst;
            for (size_t k = 0; k < half / 8; ++k) acc += p[k];
            const double rd = now_ms() - t0;
            t0 = now_ms();
            for (uint32_t i = 0; i < n; ++i) memcpy(t.dst + d[i].off, src + soff[i], d[i].len);
            const double g1 = now_ms() - t0;
            t0 = now_ms();
            for (uint32_t i = 0; i < n; ++i) memcpy(t.dst + dpin[i].off, src + soff[i], dpin[i].len);
            const double g2 = now_ms() - t0;
            printf("%-9s memcpy 32MB %6.2f GB/s  read %6.2f GB/s  gather(desc heap) %6.2f GB/s  "
                   "gather(desc pinned) %6.2f GB/s  (acc %llu)\n",
                   t.name, half / cp / 1e6, half / rd / 1e6, so / g1 / 1e6, so / g2 / 1e6,
                   (unsigned long long)(acc & 1));
        }
    }
    // threads: the gather split into T contiguous frame ranges, and the bulk
    // memcpy split into T spans, into the pinned buffer (8x the frames: 320K)
    const uint32_t n8 = 8 * n;
    std::vector<Desc> d8(n8);
    std::vector<uint64_t> s8(n8);
    uint64_t o8 = 0, so8 = 0;
    for (uint32_t i = 0; i < n8; ++i) {
        const uint32_t len = 48 + (uint32_t)((i * 2654435761u) % 1440u);
        d8[i] = {o8, len, 0};
        s8[i] = so8;
        o8 = (o8 + len + 15) & ~15ull;
        so8 += len;
    }
    uint8_t* big_src = (uint8_t*)malloc(so8 + 64);
    uint8_t* big_pin = nullptr;
    hipHostMalloc((void**)&big_pin, o8 + 64, hipHostMallocDefault);
    uint8_t* big_heap = (uint8_t*)malloc(o8 + 64);
    memset(big_src, 5, so8 + 64);
    memset(big_pin, 5, o8 + 64);
    memset(big_heap, 5, o8 + 64);
    for (int rep = 0; rep < 2; ++rep)
        for (int T : {1, 2, 4, 8, 12, 16}) {
            for (int which = 0; which < 2; ++which) {
                uint8_t* dst = which ? big_heap : big_pin;
                double t0 = now_ms();
                std::vector<std::thread> th;
                for (int t = 0; t < T; ++t)
                    th.emplace_back([&, t] {
                        const uint32_t lo = (uint64_t)n8 * t / T, hi = (uint64_t)n8 * (t + 1) / T;
                        for (uint32_t i = lo; i < hi; ++i) memcpy(dst + d8[i].off, big_src + s8[i], d8[i].len);
                    });
                for (auto& x : th) x.join();
                const double g = now_ms() - t0;
                th.clear();
                t0 = now_ms();
                for (int t = 0; t < T; ++t)
                    th.emplace_back([&, t] {
                        const uint64_t lo = so8 * t / T, hi = so8 * (t + 1) / T;
                        memcpy(dst + lo, big_src + lo, hi - lo);
                    });
                for (auto& x : th) x.join();
                const double b = now_ms() - t0;
                printf("threads %2d %-6s gather %6.2f GB/s  bulk %6.2f GB/s\n", T, which ? "heap" : "pinned",
                       so8 / g / 1e6, so8 / b / 1e6);
            }
        }
    return 0;
}
