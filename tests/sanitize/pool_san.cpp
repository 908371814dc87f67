// pool_san.cpp — the host context's gather pool (level-ip_amd/csrc/gather_pool.h)
// alone, on the CPU, under TSan or ASan (tests/test_sanitize_host.py).
//
// Jobs of 1..24 parts, back to back, with the pool growing as parts grow: every
// part of every job runs exactly once and run() returns only after all of
// them; then pools made and destroyed with and without work, and a pool whose
// workers were started by one job and left idle across many 1-part jobs.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <vector>

#include "gather_pool.h"

#define CHECK(c, ...)                                   \
    do {                                                \
        if (!(c)) {                                     \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);               \
            fprintf(stderr, "\n");                      \
            exit(1);                                    \
        }                                               \
    } while (0)

int main() {
    {
        lvlip::GatherPool pool;
        std::vector<int> hits(64, 0);  // written by the parts, read after run()
        for (int job = 0; job < 3000; ++job) {
            const int parts = 1 + (job * 7) % 24;
            for (int k = 0; k < parts; ++k) hits[k] = 0;
            std::atomic<int> calls{0};
            pool.run(parts, [&](int k) {
                hits[k] += 1 + job;  // a plain write per part: TSan sees any overlap
                calls.fetch_add(1, std::memory_order_relaxed);
            });
            CHECK(calls.load() == parts, "job %d: %d calls for %d parts", job, calls.load(), parts);
            for (int k = 0; k < parts; ++k)
                CHECK(hits[k] == 1 + job, "job %d part %d ran %d times", job, k, hits[k] / (1 + job));
        }
    }
    for (int i = 0; i < 50; ++i) {  // create/destroy, with and without work
        lvlip::GatherPool p;
        if (i % 2) {
            uint64_t sum[8] = {0};
            p.run(8, [&](int k) { sum[k] = (uint64_t)k * 3u; });
            for (int k = 0; k < 8; ++k) CHECK(sum[k] == (uint64_t)k * 3u, "sum %d", k);
        }
    }
    {
        lvlip::GatherPool p;
        int x[16] = {0};
        p.run(16, [&](int k) { x[k] = k; });
        for (int j = 0; j < 1000; ++j) p.run(1, [&](int) { x[0] += 1; });  // workers stay idle
        CHECK(x[0] == 1000, "inline parts %d", x[0]);
        p.run(16, [&](int k) { x[k] += 1; });
        for (int k = 1; k < 16; ++k) CHECK(x[k] == k + 1, "part %d", k);
    }
    printf("all checks passed\n");
    return 0;
}
