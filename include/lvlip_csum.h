/*
 * lvlip_csum.h — C-ABI of the MI355X Internet-checksum offload for level-ip.
 *
 * This is the drop-in boundary between level-ip's C stack and the gfx950 HIP
 * kernels in level-ip_amd/csrc/.  Every entry point is plain C: pointers,
 * sizes and integers, no HIP or torch types.  Citations are to the reference
 * tree (saminiir/level-ip v1) as path:line.
 *
 *  Group 1 — per-call drop-in (CPU, reentrant, no shared state).
 *    Same names, signatures and results as include/utils.h:13-14
 *    (src/utils.c:22-55).  The stack keeps calling these from
 *    src/ip_input.c:38, src/ip_output.c:10, src/icmpv4.c:47, src/tcp.c:97.
 *
 *  Group 2 — batched checksum over packet descriptors on the GPU.
 *    out[i] == checksum(base + d[i].offset, d[i].len, (int)d[i].start_sum)
 *    bit for bit, including the reference's u32 wrap-around of the seed
 *    (src/utils.c:46-48, src/tcp.c:92-97).
 *
 *  Group 3 — host-resident batches through a per-thread context (pinned
 *    staging arena + HIP stream): gathers skb bytes, H2D, kernel, D2H.
 *
 *  Group 4 — one batch over several GPUs: a byte-balanced contiguous
 *    partition, and a host batch run by one thread per device context.
 *
 * Error convention: 0 = success, negative LVLIP_E* on failure.  A batch call
 * that fails writes nothing meaningful to out[] and never substitutes a CPU
 * result: the caller decides what to do.
 */
#ifndef LVLIP_CSUM_H
#define LVLIP_CSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
/* The library is built with -fvisibility=hidden: exactly the entry points
 * declared in this header are exported. */
#pragma GCC visibility push(default)

/* 2 (round 4): what changed from 1 for a caller of lvlip_csum_batch_dev_ex:
 * FLAT's unroll takes only 2, 4 or 8 (the group-order bits << 8 and the
 * 512-descriptor tile bit 1 << 10, A/B shapes, are now LVLIP_EINVAL here and
 * live in liblvlip_lab.so); the kernel ids the A/B library retired in round 4
 * (2, 4, 5, 11, 12, 14, 15) are LVLIP_EINVAL in both libraries (the product
 * already refused every id but 0, 3, 8 and 10 in ABI 1).  Added: Group 4
 * (lvlip_partition_bytes, lvlip_csum_batch_host_flat_multi) and
 * lvlip_icmp_echo_reply_dev_ex (include/lvlip_skb.h).  INTEGRATION.md §5.
 * Round 5 changed no entry point: the host frame calls' implementation moved
 * to the device (include/lvlip_skb.h), with the same results.  Round 6 added
 * entry points only (the size-based dispatch and its counters below, the
 * context-free CPU frame calls of include/lvlip_skb.h); a context's host calls
 * of at most LVLIP_CPU_MAX_DEFAULT packets / frames now run on the CPU by
 * default, with identical results. */
#define LVLIP_CSUM_ABI_VERSION 2

/* ---- error codes ------------------------------------------------------- */
#define LVLIP_OK              0
#define LVLIP_EINVAL         -1  /* bad argument (NULL, n too large, ...)   */
#define LVLIP_ENODEV         -2  /* no HIP device / device index invalid     */
#define LVLIP_EHIP           -3  /* a HIP runtime call failed                */
#define LVLIP_ENOMEM         -4  /* device or pinned allocation failed       */
#define LVLIP_ERANGE         -5  /* batch does not fit the context's arena   */

/* ======================================================================= */
/* Group 1: per-call drop-in, replaces src/utils.c:22-55                    */
/* ======================================================================= */

/* Replaces sum_every_16bits, src/utils.c:22-38 (decl include/utils.h:13).
 * Sum of count/2 native little-endian u16 words, modulo 2^32, plus the odd
 * trailing byte zero-extended; count <= 0 gives 0. */
uint32_t sum_every_16bits(void *addr, int count);

/* Replaces checksum, src/utils.c:40-55 (decl include/utils.h:14).
 * T = (uint32_t)start_sum + sum_every_16bits(addr, count) (mod 2^32), folded
 * with while (T >> 16) T = (T & 0xffff) + (T >> 16), returned as (uint16_t)~T.
 * The result is stored raw (no htons) by every caller. */
uint16_t checksum(void *addr, int count, int start_sum);

/* Seed arithmetic of tcp_udp_checksum, src/tcp.c:87-96: saddr + daddr +
 * htons(proto) + htons(len), all as u32 with plain wrap-around (the carry out
 * of bit 31 is lost, exactly as the reference loses it).  saddr/daddr are
 * network-order words as passed at src/tcp_output.c:126. */
uint32_t lvlip_pseudo_sum(uint32_t saddr, uint32_t daddr, uint8_t proto,
                          uint16_t len);

/* The reference's own wrappers around checksum(), kept with their signatures
 * so a build that links this library in place of src/utils.c + these
 * functions sees the same symbols. */
struct sk_buff;
struct iphdr;

/* src/tcp.c:87-98: checksum(data, len, lvlip_pseudo_sum(saddr, daddr, proto, len)). */
int tcp_udp_checksum(uint32_t saddr, uint32_t daddr, uint8_t proto, uint8_t *data,
                     uint16_t len);

/* src/tcp.c:100-103: tcp_udp_checksum(saddr, daddr, 6, skb->data, skb->len).
 * Reads skb->len and skb->data at the offsets struct sk_buff has in
 * include/skbuff.h:9-23 on LP64 (40 and 72). */
int tcp_v4_checksum(struct sk_buff *skb, uint32_t saddr, uint32_t daddr);

/* src/ip_output.c:8-12: ihdr->csum = checksum(ihdr, ihdr->ihl * 4, 0), stored
 * raw; like the reference it does not zero the field first (its callers do,
 * src/ip_output.c:42,50). */
void ip_send_check(struct iphdr *ihdr);

/* ======================================================================= */
/* Group 2: device-resident batches                                         */
/* ======================================================================= */

/* One packet (or header) to checksum.  16 bytes, naturally aligned.
 *   offset    byte offset of the first byte from the batch base pointer
 *   len       byte count (the reference's `int count`); <= 0 means empty
 *   start_sum the `int start_sum` seed, as its u32 bit pattern:
 *             0 for IPv4 headers (src/ip_input.c:38, src/ip_output.c:10)
 *             and ICMP (src/icmpv4.c:47); lvlip_pseudo_sum(...) for TCP
 *             (src/tcp.c:97). */
typedef struct lvlip_csum_desc {
    uint64_t offset;
    int32_t  len;
    uint32_t start_sum;
} lvlip_csum_desc;

/* Largest batch one call accepts (packet indices are 32-bit on the GPU). */
#define LVLIP_MAX_BATCH 0xFFFFFFF0u

/* Checksums n descriptors whose bytes, descriptors and outputs are all in
 * device memory of the current HIP device.  Asynchronous on `stream` (a
 * hipStream_t passed as void*, NULL = the null stream).
 *
 * Contract on base: 16-byte aligned, and readable from base up to
 * round_up(max(offset + len), 16): the kernel reads whole 16-byte chunks and
 * masks the bytes outside each packet.  Any byte alignment of offset is
 * accepted (odd offsets included).  out[i] is a raw u16 (no byte swap). */
int lvlip_csum_batch_dev(const void *base, const lvlip_csum_desc *descs,
                         uint32_t n, uint16_t *out, void *stream);

/* Kernel selection for lvlip_csum_batch_dev_ex.  AUTO picks by len_hint:
 * >= 896 B -> WINDOW (shape by the hint); 1-32 B -> LANE; otherwise or
 * unknown -> FLAT (measured: DESIGN.md §4-5).  lvlip_auto_kernel() tells
 * which kernel and shape AUTO runs.  Ids 1, 9 and 13 are A/B variants
 * measured against these (liblvlip_lab.so, not this library), and 2, 4-7,
 * 11, 12, 14 and 15 are retired: here all of them return
 * LVLIP_EINVAL. */
#define LVLIP_KERNEL_AUTO        0  /* the default                                 */
#define LVLIP_KERNEL_FLAT        3  /* chunk-balanced tile sweep (ragged batches)  */
#define LVLIP_KERNEL_WINDOW      8  /* one wavefront per packet, persistent, packets
                                       dealt in small groups round robin over the
                                       grid (one narrow window of the batch in
                                       flight)                                 */
#define LVLIP_KERNEL_LANE       10  /* a few lanes per packet, chunks summed in
                                       registers (batches of small packets)   */

typedef struct lvlip_launch_cfg {
    int32_t  kernel;        /* LVLIP_KERNEL_*                               */
    int32_t  unroll;        /* 0 = default.  WINDOW: 2-KiB pieces in flight
                               per wave (2, 3, 4) | packets per group << 8
                               (1, 2, 3, 4 or 8; 0 = by len_hint);
                               FLAT: 64-chunk loads per round (2, 4, 8);
                               LANE: packets per lane group | 16-B chunks
                               per lane << 8 | lanes per packet << 16 (1, 2,
                               4, 8) | unconditional loads << 24; longer
                               packets go to a whole-wave loop (0 = 4 | 2 << 8
                               | 2 << 16)                                   */
    int32_t  waves_per_cu;  /* WINDOW: resident waves per CU (0 = 8)        */
    int32_t  len_hint;      /* average packet length in bytes if the caller
                               knows it (AUTO uses it), 0 = unknown         */
} lvlip_launch_cfg;

int lvlip_csum_batch_dev_ex(const void *base, const lvlip_csum_desc *descs,
                            uint32_t n, uint16_t *out, void *stream,
                            const lvlip_launch_cfg *cfg);

/* The kernel and launch shape LVLIP_KERNEL_AUTO runs for n descriptors of
 * average length len_hint on the current HIP device: returns the kernel id
 * and, when resolved != NULL, fills it with that id, its unroll and
 * waves_per_cu words and len_hint. */
int lvlip_auto_kernel(int32_t len_hint, uint32_t n, lvlip_launch_cfg *resolved);

/* How many kernel launches lvlip_csum_batch_dev_ex issues, back to back on
 * its stream, for a batch of n descriptors with cfg (NULL = AUTO, resolved as
 * the call resolves it) on the current HIP device: a WINDOW batch of more than
 * ~120 packet groups per wave goes out in launches of ~80, any
 * batch beyond 2^30 descriptors in launches of 2^30.  0 when n is 0 or above
 * LVLIP_MAX_BATCH.  For profilers: per-launch figures are the batch's / this. */
uint32_t lvlip_batch_launches(uint32_t n, const lvlip_launch_cfg *cfg);

/* ======================================================================= */
/* Group 3: host-resident batches (per-thread context)                      */
/* ======================================================================= */

/* One host packet: the bytes a reference call site would pass to
 * checksum(ptr, len, start_sum).  ptr may be any address (skb->head + 14 /
 * + 34 are 2 mod 4, include/ip.h:47-50, include/tcp.h:224-227). */
typedef struct lvlip_csum_iov {
    const void *ptr;
    int32_t     len;
    uint32_t    start_sum;
} lvlip_csum_iov;

typedef struct lvlip_csum_ctx lvlip_csum_ctx;

/* Creates a context on HIP device `device` with a pinned host arena and a
 * device arena of `arena_bytes` each (0 = 64 MiB), and its own stream.
 * A context is owned by one thread at a time (src/main.c:83-89 runs the
 * checksum from several threads: give each its own context).  Creation also
 * starts the copy engine (1 MiB each way per slot, LVLIP_WARM_BYTES) and
 * loads the kernels' code object, so the first call pays neither start-up
 * (~7 ms and ~2 ms measured).  Returns 0,
 * LVLIP_ENODEV, LVLIP_ENOMEM (an arena allocation failed) or LVLIP_EHIP. */
int lvlip_csum_ctx_create(lvlip_csum_ctx **out, int device,
                          size_t arena_bytes);
int lvlip_csum_ctx_destroy(lvlip_csum_ctx *ctx);

/* Gathers the n host packets into the pinned arena (each at a 16-B aligned
 * slot), copies to the device, runs the kernel, copies the n results back
 * and waits.  Batches larger than the arena are processed in arena-sized
 * pieces, double-buffered so the copy of one piece overlaps the kernel of
 * the previous one.  out is host memory. */
int lvlip_csum_batch_host(lvlip_csum_ctx *ctx, const lvlip_csum_iov *pkts,
                          uint32_t n, uint16_t *out);

/* Same, for packets already laid out in one host buffer (descriptor
 * offsets relative to `base`, which must hold round_up(max end,16) bytes).
 * Descriptors that cover their span densely and in order (see "densely"
 * below) move as spans; others are gathered packet by packet. */
int lvlip_csum_batch_host_flat(lvlip_csum_ctx *ctx, const void *base,
                               size_t base_bytes, const lvlip_csum_desc *d,
                               uint32_t n, uint16_t *out);

/* f3: zero-copy host staging.  Registers host memory that
 * holds packets (an skb slab, a frame pool, a receive ring) with the context
 * (hipHostRegister, whole pages pinned in place).  Batches whose bytes lie in
 * one registered region skip the gather into the pinned arena:
 *   LVLIP_REG_DMA       batch_host_flat copies each piece's span straight
 *                       from the region with the copy engine (no CPU memcpy);
 *                       so does batch_host when its packets cover their span
 *                       densely (else it gathers them)
 *   LVLIP_REG_ZEROCOPY  the kernel reads the packets in place over PCIe: only
 *                       descriptors go down and results come back, for
 *                       batch_host, batch_host_flat and the frame calls of
 *                       lvlip_skb.h when their packets / frames lie thinly
 *                       over the region; when they cover their span densely
 *                       the span moves with the copy engine, as for
 *                       LVLIP_REG_DMA (faster: 2-5 % for packet batches,
 *                       ~20 % for the frame calls, whose per-frame parse reads
 *                       over PCIe).  Exception: the header-only
 *                       lvlip_rx_verify (flags 0) needs 74 B of each frame
 *                       and always reads a zero-copy region in place
 * "Densely" means the packets' byte span is at most twice their bytes plus
 * 1 MiB (the factor is LVLIP_SPAN_RATIO, 1-64) AND they come in address order: the sum of the jumps between
 * consecutive start addresses is at most twice the span plus 1 MiB (a
 * shuffled batch over a large slab would cut into pieces of one or two
 * packets, each moving a whole span).  A DMA region's batch that is not dense
 * is gathered packet by packet into the pinned arena.
 * Regions must not overlap; the memory must stay valid until unregistered
 * (lvlip_csum_ctx_destroy unregisters what is left).  Results are identical
 * on every path. */
#define LVLIP_REG_DMA      0u
#define LVLIP_REG_ZEROCOPY 1u
int lvlip_csum_register(lvlip_csum_ctx *ctx, void *ptr, size_t bytes, uint32_t flags);
int lvlip_csum_unregister(lvlip_csum_ctx *ctx, void *ptr);

/* Size-based dispatch of the host calls (SURVEY.md §5 "Config/flags", §7
 * step 5).  A host call over at most cpu_max packets (lvlip_csum_batch_host,
 * lvlip_csum_batch_host_flat) or frames (lvlip_rx_verify, lvlip_tx_checksum
 * and their _skb_list forms, include/lvlip_skb.h) runs on the CALLING THREAD
 * with the library's own CPU code (Group 1's checksum(); lvlip_rx_verify_cpu /
 * lvlip_tx_checksum_cpu), never touching the GPU: a GPU round trip costs a
 * host call ~20 us before the first byte is summed, more than one core needs
 * for level-ip's usual flushes of 1-30 frames (DESIGN.md §9 measures the
 * crossover).  This is a performance choice only: results, return codes and
 * the untouched-on-error rule are identical on both sides of the threshold
 * (the GPU tests check both).  It is distinct from the error rule above: a
 * call that goes to the GPU and fails still returns LVLIP_E* with no CPU
 * substitute.  0 = every call goes to the GPU.  The default is the env var
 * LVLIP_CPU_MAX when set when the context is created, else
 * LVLIP_CPU_MAX_DEFAULT.  Device-resident calls (Groups 2 and the _dev frame
 * calls) are never dispatched to the CPU. */
#define LVLIP_CPU_MAX_DEFAULT 16384u
int lvlip_csum_ctx_set_cpu_max(lvlip_csum_ctx *ctx, uint32_t cpu_max);
/* The context's current threshold (0 for a NULL context). */
uint32_t lvlip_csum_ctx_cpu_max(const lvlip_csum_ctx *ctx);

/* Counters of a context since it was created (for tests, benches and a
 * maintainer's own monitoring). */
typedef struct lvlip_ctx_stats {
    uint64_t gpu_calls;  /* host calls that ran on the GPU                  */
    uint64_t cpu_calls;  /* host calls run on the calling thread (cpu_max)  */
    uint64_t pieces;     /* device pieces launched by the GPU calls         */
    uint64_t h2d_bytes;  /* bytes the pieces moved host->device: each piece's
                            gathered arena bytes or copied span, whether the
                            copy engine or (small pieces, zero-copy) the
                            kernel moved them; descriptors not counted     */
} lvlip_ctx_stats;
int lvlip_csum_ctx_stats(const lvlip_csum_ctx *ctx, lvlip_ctx_stats *out);

/* ======================================================================= */
/* Group 4: one batch over several GPUs                     */
/* ======================================================================= */

/* Packets are independent, so a batch shards by contiguous descriptor ranges
 * with no exchange on the data path.  Fills cuts[0 .. parts] (parts + 1
 * entries): part p is descriptors [cuts[p], cuts[p + 1]), cuts[0] = 0,
 * cuts[parts] = n, non-decreasing.  Balanced by bytes: part p takes the
 * descriptors whose byte prefix (sum of max(len, 0) before them) lies in
 * [p T / parts, (p + 1) T / parts), T the total, so a ragged batch gives
 * every GPU about the same HBM traffic; an all-empty batch splits by count.
 * The same cuts as level-ip_amd/shard.py partition().  Host only (no GPU).
 * Returns 0, or LVLIP_EINVAL (parts == 0, NULL with n > 0). */
int lvlip_partition_bytes(const lvlip_csum_desc *d, uint32_t n, uint32_t parts,
                          uint32_t *cuts);

/* lvlip_csum_batch_host_flat over nctx contexts at once (one per GPU, each
 * created with lvlip_csum_ctx_create on its own device): the batch is cut
 * with lvlip_partition_bytes into nctx parts, and context k checksums part k
 * on a host thread of its own (its gather, copies and kernel overlap with the
 * other devices').  Waits for all parts; out[] is in descriptor order.  The
 * contexts are used by this call's threads only while it runs (the caller
 * must not use them concurrently), and must be distinct (a context is owned
 * by one thread at a time: the same pointer twice is LVLIP_EINVAL).  Returns
 * 0 or the first part's LVLIP_E* in part order (results of failed parts are
 * not meaningful); lvlip_last_hip_error() on the calling thread then holds
 * that part's HIP message.  A part whose thread cannot be started runs on the
 * calling thread. */
int lvlip_csum_batch_host_flat_multi(lvlip_csum_ctx *const *ctxs, uint32_t nctx,
                                     const void *base, size_t base_bytes,
                                     const lvlip_csum_desc *d, uint32_t n,
                                     uint16_t *out);

/* ======================================================================= */
/* Misc                                                                     */
/* ======================================================================= */
const char *lvlip_strerror(int err);
int lvlip_abi_version(void);
/* Number of visible HIP devices (0 when none). */
int lvlip_device_count(void);
/* Last HIP error string recorded by this library in the calling thread. */
const char *lvlip_last_hip_error(void);
/* Hash of the sources this library was built from (the files listed in
 * level-ip_amd/BUILD_SOURCES, SHA-256, first 16 hex digits): the tests and
 * the bench refuse a library whose hash differs from the tree's. */
const char *lvlip_build_id(void);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif /* LVLIP_CSUM_H */
