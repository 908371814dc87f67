/*
 * multi_gpu.c — INTEGRATION.md §4a as a plain C program against the C ABI only
 * (include/lvlip_csum.h): one checksum batch over several GPU contexts, one
 * host thread per context, the way a multi-threaded level-ip process
 * (src/main.c:83-89) would shard a batch over the node's GPUs.
 *
 * The batch is ragged (a 20-B IPv4 header and a 64-1460-B TCP or ICMP payload
 * per frame, the skb layout of include/ip.h:47-50 and include/tcp.h:224-227,
 * TCP seeds from lvlip_pseudo_sum) in one host buffer.  With K contexts
 * (context k on device k % lvlip_device_count(), so K > 1 also runs on one
 * GPU) the program
 *   1. runs lvlip_csum_batch_host_flat_multi (the library's own thread per
 *      context), and
 *   2. does the same by hand: lvlip_partition_bytes, then one pthread per
 *      context calling lvlip_csum_batch_host_flat on its part,
 *   3. shards it device-resident, the way the headline metric shards
 *      (BASELINE configs[4], bench.py --gpus N): part k's span copied once
 *      into device k % lvlip_device_count()'s HBM (HIP runtime C API), then
 *      one lvlip_csum_batch_dev per part on its own device, the parts'
 *      threads running at once, no exchange between them,
 * and checks every result of all three against the per-call drop-in
 * checksum() (src/utils.c:40-55 semantics).  Prints "multi_gpu ok ..." and
 * exits 0.
 *
 *   make -C examples && examples/build/multi_gpu [frames] [contexts]
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "lvlip_csum.h"

#define MAX_CTX 16

static uint64_t rng_state = 0x5EED5EEDull;
static uint64_t rnd(void) /* splitmix64 */
{
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct part {
    lvlip_csum_ctx *ctx;
    const uint8_t *base;
    size_t base_bytes;
    const lvlip_csum_desc *d;
    uint32_t n;
    uint16_t *out;
    int rc;
};

static void *run_part(void *arg)
{
    struct part *p = (struct part *)arg;
    p->rc = p->n ? lvlip_csum_batch_host_flat(p->ctx, p->base, p->base_bytes, p->d, p->n, p->out) : 0;
    return NULL;
}

/* 3.: one shard in HBM.  The part's descriptors keep their offsets from the
 * span's first byte rounded down to 16 (lvlip_csum_batch_dev wants a 16-B
 * aligned base, and every packet keeps its address mod 16). */
struct dev_part {
    int device;
    const uint8_t *base;
    const lvlip_csum_desc *d;
    uint32_t n;
    uint16_t *out;
    int rc;
    char err[160];
};

static void *run_dev_part(void *arg)
{
    struct dev_part *p = (struct dev_part *)arg;
    p->rc = 0;
    if (!p->n)
        return NULL;
    uint64_t lo = UINT64_MAX, hi = 0;
    for (uint32_t i = 0; i < p->n; i++) {
        const uint64_t e = p->d[i].offset + (uint64_t)(p->d[i].len > 0 ? p->d[i].len : 0);
        lo = p->d[i].offset < lo ? p->d[i].offset : lo;
        hi = e > hi ? e : hi;
    }
    lo &= ~15ull;
    const size_t span = (size_t)((hi - lo + 15u) & ~15ull);
    lvlip_csum_desc *dd = malloc((size_t)p->n * sizeof *dd);
    void *dbase = NULL, *ddesc = NULL, *dout = NULL;
    hipError_t e = hipSetDevice(p->device);
    if (e == hipSuccess) e = hipMalloc(&dbase, span ? span : 16);
    if (e == hipSuccess) e = hipMalloc(&ddesc, (size_t)p->n * sizeof *dd);
    if (e == hipSuccess) e = hipMalloc(&dout, (size_t)p->n * sizeof(uint16_t));
    if (e == hipSuccess && dd) {
        for (uint32_t i = 0; i < p->n; i++) {
            dd[i] = p->d[i];
            dd[i].offset -= lo;
        }
        /* the span's tail past hi is read as whole 16-B chunks: copy the
         * bytes that exist, the rest of the last chunk stays unset */
        e = hipMemcpy(dbase, p->base + lo, (size_t)(hi - lo), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(ddesc, dd, (size_t)p->n * sizeof *dd, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess || !dd) {
        snprintf(p->err, sizeof p->err, "device %d: %s", p->device, dd ? hipGetErrorString(e) : "out of memory");
        p->rc = -1;
    } else if ((p->rc = lvlip_csum_batch_dev(dbase, ddesc, p->n, dout, NULL)) != 0) {
        snprintf(p->err, sizeof p->err, "lvlip_csum_batch_dev: %s", lvlip_strerror(p->rc));
    } else if ((e = hipDeviceSynchronize()) != hipSuccess ||
               (e = hipMemcpy(p->out, dout, (size_t)p->n * sizeof(uint16_t), hipMemcpyDeviceToHost)) != hipSuccess) {
        snprintf(p->err, sizeof p->err, "device %d: %s", p->device, hipGetErrorString(e));
        p->rc = -1;
    }
    (void)hipFree(dbase);
    (void)hipFree(ddesc);
    (void)hipFree(dout);
    free(dd);
    return NULL;
}

int main(int argc, char **argv)
{
    const uint32_t frames = argc > 1 ? (uint32_t)strtoul(argv[1], NULL, 0) : 65536u;
    uint32_t k = argc > 2 ? (uint32_t)strtoul(argv[2], NULL, 0) : 0u;
    const int ndev = lvlip_device_count();
    if (ndev <= 0) {
        fprintf(stderr, "multi_gpu: no HIP device\n");
        return 1;
    }
    if (k == 0)
        k = (uint32_t)ndev;
    if (k > MAX_CTX)
        k = MAX_CTX;

    /* the ragged batch: frame = 14 + 20 + payload, 16-B aligned frame starts */
    const uint32_t n = 2u * frames;
    lvlip_csum_desc *d = calloc(n, sizeof *d);
    uint64_t off = 0;
    for (uint32_t f = 0; f < frames; f++) {
        const uint32_t plen = 64u + (uint32_t)(rnd() % 1397u);
        d[2 * f].offset = off + 14;
        d[2 * f].len = 20;
        d[2 * f].start_sum = 0;
        d[2 * f + 1].offset = off + 34;
        d[2 * f + 1].len = (int32_t)plen;
        d[2 * f + 1].start_sum = (rnd() & 1) ? lvlip_pseudo_sum((uint32_t)rnd(), (uint32_t)rnd(), 6,
                                                               (uint16_t)plen)
                                             : 0u;
        off += (34u + plen + 15u) & ~15ull;
    }
    const size_t base_bytes = (size_t)off;
    uint8_t *base = malloc(base_bytes);
    for (size_t i = 0; i < base_bytes; i++)
        base[i] = (uint8_t)rnd();
    uint16_t *want = malloc(n * sizeof *want), *got1 = malloc(n * sizeof *got1), *got2 = malloc(n * sizeof *got2);
    for (uint32_t i = 0; i < n; i++)
        want[i] = checksum(base + d[i].offset, d[i].len, (int)d[i].start_sum);

    lvlip_csum_ctx *ctx[MAX_CTX];
    for (uint32_t c = 0; c < k; c++) {
        const int rc = lvlip_csum_ctx_create(&ctx[c], (int)(c % (uint32_t)ndev), 16u << 20);
        if (rc) {
            fprintf(stderr, "multi_gpu: ctx_create: %s\n", lvlip_strerror(rc));
            return 1;
        }
    }

    /* 1. the library's thread per context */
    int rc = lvlip_csum_batch_host_flat_multi(ctx, k, base, base_bytes, d, n, got1);
    if (rc) {
        fprintf(stderr, "multi_gpu: batch_host_flat_multi: %s (%s)\n", lvlip_strerror(rc), lvlip_last_hip_error());
        return 1;
    }

    /* 2. by hand: the partition, then one pthread per context */
    uint32_t cuts[MAX_CTX + 1];
    if ((rc = lvlip_partition_bytes(d, n, k, cuts)) != 0) {
        fprintf(stderr, "multi_gpu: partition: %s\n", lvlip_strerror(rc));
        return 1;
    }
    struct part parts[MAX_CTX];
    pthread_t th[MAX_CTX];
    for (uint32_t c = 0; c < k; c++) {
        parts[c] = (struct part){ctx[c], base, base_bytes, d + cuts[c], cuts[c + 1] - cuts[c], got2 + cuts[c], 0};
        if (pthread_create(&th[c], NULL, run_part, &parts[c]) != 0) {
            fprintf(stderr, "multi_gpu: pthread_create failed for part %u\n", c);
            return 1;
        }
    }
    for (uint32_t c = 0; c < k; c++) {
        pthread_join(th[c], NULL);
        if (parts[c].rc) {
            fprintf(stderr, "multi_gpu: part %u: %s\n", c, lvlip_strerror(parts[c].rc));
            return 1;
        }
    }
    /* 3. device-resident shards: one lvlip_csum_batch_dev per device */
    uint16_t *got3 = malloc(n * sizeof *got3);
    struct dev_part dparts[MAX_CTX];
    for (uint32_t c = 0; c < k; c++) {
        dparts[c] = (struct dev_part){(int)(c % (uint32_t)ndev), base, d + cuts[c], cuts[c + 1] - cuts[c],
                                      got3 + cuts[c], 0, ""};
        if (pthread_create(&th[c], NULL, run_dev_part, &dparts[c]) != 0) {
            fprintf(stderr, "multi_gpu: pthread_create failed for device part %u\n", c);
            return 1;
        }
    }
    for (uint32_t c = 0; c < k; c++) {
        pthread_join(th[c], NULL);
        if (dparts[c].rc) {
            fprintf(stderr, "multi_gpu: device part %u: %s\n", c, dparts[c].err);
            return 1;
        }
    }
    uint32_t bad1 = 0, bad2 = 0, bad3 = 0;
    for (uint32_t i = 0; i < n; i++) {
        bad1 += got1[i] != want[i];
        bad2 += got2[i] != want[i];
        bad3 += got3[i] != want[i];
    }
    for (uint32_t c = 0; c < k; c++)
        lvlip_csum_ctx_destroy(ctx[c]);
    if (bad1 || bad2 || bad3) {
        fprintf(stderr, "multi_gpu: %u / %u / %u of %u checksums differ from checksum()\n", bad1, bad2, bad3, n);
        return 1;
    }
    printf("multi_gpu ok: %u descriptors over %u contexts on %d device(s) (host-resident and "
           "device-resident shards), parts", n, k, ndev);
    for (uint32_t c = 0; c < k; c++)
        printf(" %u", cuts[c + 1] - cuts[c]);
    printf("\n");
    free(d);
    free(base);
    free(want);
    free(got1);
    free(got2);
    free(got3);
    return 0;
}
