/* scripts/dropin_bench.c — per-call cost of the drop-in checksum() on a
 * cache-hot buffer, by length (round 6 A/B of the short-buffer path).
 * Usage: dropin_bench REPS LEN... ; prints one JSON object. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

uint16_t checksum(void *addr, int count, int start_sum);

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 1000000;
    uint8_t *b = aligned_alloc(64, 65536);
    for (int i = 0; i < 65536; i++) b[i] = (uint8_t)(i * 7 + 3);
    volatile uint32_t acc = 0;
    printf("{");
    for (int a = 2; a < argc; a++) {
        const int len = atoi(argv[a]);
        double best = 1e9;
        for (int k = 0; k < 5; k++) {
            const double t0 = now();
            for (int r = 0; r < reps; r++) acc += checksum(b + 34 + (r & 7) * 2, len, r);
            const double t = (now() - t0) / reps * 1e9;
            if (t < best) best = t;
        }
        printf("%s\"%d\": %.2f", a > 2 ? ", " : "", len, best);
    }
    printf("}\n");
    return (int)(acc & 0);
}
