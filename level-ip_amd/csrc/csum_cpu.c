/*
 * csum_cpu.c — Group 1 of include/lvlip_csum.h: the per-call drop-in for
 * level-ip's src/utils.c:22-55, plus the pseudo-header seed of src/tcp.c:87-96.
 *
 * These stay on the CPU by design: every reference call site (src/ip_input.c:38,
 * src/ip_output.c:10, src/icmpv4.c:47, src/tcp.c:97) checksums one 20-1500 B
 * buffer synchronously, far below what a PCIe round trip costs.  The GPU path
 * is the batched API (csum_kernels.hip).  Reentrant, no shared state
 * (called concurrently from the core, IPC and timer threads).
 *
 * Bit-exactness: the reference adds u16 words into a uint32_t with plain
 * wrap-around.  Accumulating the same words in 64 bits and truncating once is
 * the same value mod 2^32, so the result is identical for every count.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "lvlip_csum.h"

/* src/utils.c:22-38 */
uint32_t sum_every_16bits(void *addr, int count)
{
    const uint8_t *p = (const uint8_t *)addr;
    uint64_t s0 = 0, s1 = 0;

    /* 16 bytes per step: eight native-endian u16 words into two accumulators
     * of two 32-bit fields each.  A field gains <= 2 * 0xffff per step, so
     * 16384 steps stay below 2^31 and no field carries into its neighbour. */
    while (count >= 16) {
        int steps = count >> 4;
        if (steps > 16384)
            steps = 16384;
        uint64_t a = 0, b = 0;
        for (int i = 0; i < steps; i++) {
            uint64_t x, y;
            memcpy(&x, p, 8);
            memcpy(&y, p + 8, 8);
            a += (x & 0x0000ffff0000ffffull) + (y & 0x0000ffff0000ffffull);
            b += ((x >> 16) & 0x0000ffff0000ffffull) + ((y >> 16) & 0x0000ffff0000ffffull);
            p += 16;
        }
        count -= steps << 4;
        s0 += (a & 0xffffffffull) + (a >> 32);
        s1 += (b & 0xffffffffull) + (b >> 32);
    }
    while (count > 1) {
        uint16_t w;
        memcpy(&w, p, 2);
        s0 += w;
        p += 2;
        count -= 2;
    }
    if (count > 0) /* utils.c:34-35: left-over byte, zero-extended */
        s0 += *p;
    return (uint32_t)(s0 + s1);
}

/* src/utils.c:40-55 */
uint16_t checksum(void *addr, int count, int start_sum)
{
    uint32_t sum = (uint32_t)start_sum;
    sum += sum_every_16bits(addr, count);
    sum = (sum & 0xffff) + (sum >> 16); /* <= 0x1fffe */
    sum = (sum & 0xffff) + (sum >> 16); /* <= 0xffff: same as the while loop */
    return (uint16_t)~sum;
}

/* src/tcp.c:87-96 (htons on a little-endian host is a byte swap) */
uint32_t lvlip_pseudo_sum(uint32_t saddr, uint32_t daddr, uint8_t proto, uint16_t len)
{
    uint32_t sum = 0;
    sum += saddr;
    sum += daddr;
    sum += (uint32_t)(uint16_t)((uint16_t)proto << 8);
    sum += (uint32_t)(uint16_t)((len << 8) | (len >> 8));
    return sum;
}

/* src/tcp.c:87-98 */
int tcp_udp_checksum(uint32_t saddr, uint32_t daddr, uint8_t proto, uint8_t *data, uint16_t len)
{
    return checksum(data, len, (int)lvlip_pseudo_sum(saddr, daddr, proto, len));
}

/* The leading fields of struct sk_buff, include/skbuff.h:9-23, as laid out on
 * LP64: only len and data are read. */
struct lvlip_sk_buff_abi {
    void *list_next, *list_prev; /* struct list_head */
    void *rt;
    void *dev;
    int refcnt;
    uint16_t protocol;
    uint32_t len;
    uint32_t dlen;
    uint32_t seq;
    uint32_t end_seq;
    uint8_t *end;
    uint8_t *head;
    uint8_t *data;
    uint8_t *payload;
};
_Static_assert(offsetof(struct lvlip_sk_buff_abi, len) == 40, "sk_buff.len offset");
_Static_assert(offsetof(struct lvlip_sk_buff_abi, data) == 72, "sk_buff.data offset");

/* src/tcp.c:100-103 */
int tcp_v4_checksum(struct sk_buff *skb, uint32_t saddr, uint32_t daddr)
{
    const struct lvlip_sk_buff_abi *s = (const struct lvlip_sk_buff_abi *)(const void *)skb;
    return tcp_udp_checksum(saddr, daddr, 6, s->data, (uint16_t)s->len);
}

/* src/ip_output.c:8-12; ihl is the low nibble of byte 0 (include/ip.h:33-34) */
void ip_send_check(struct iphdr *ihdr)
{
    uint8_t *h = (uint8_t *)(void *)ihdr;
    const uint16_t c = checksum(h, (h[0] & 0x0f) * 4, 0);
    memcpy(h + 10, &c, 2);
}
