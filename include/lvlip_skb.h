/*
 * lvlip_skb.h — batch-and-dispatch over level-ip frames.
 *
 * level-ip handles one frame at a time: netdev_rx_loop reads one frame per
 * read(2) (src/netdev.c:86-101) and every checksum is a synchronous per-packet
 * call.  These entry points take N frames at once and run all their checksums
 * as ONE GPU batch through a context (include/lvlip_csum.h, Group 3).
 *
 * A frame is what an sk_buff holds (include/skbuff.h:9-23): `head` points at the
 * Ethernet header, the IPv4 header is at head + 14 (ip_hdr(), include/ip.h:47-50)
 * and the TCP/ICMP header right after it (tcp_hdr(), include/tcp.h:224-227).
 *
 * The device parses every frame (the same kernels as the _dev calls below):
 * the host moves whole frames to the GPU (a gather into a pinned arena, or,
 * for frames inside a registered region, DMA of its spans or in-place reads),
 * and gets back one verdict (RX) or one record of the two fields (TX) per
 * frame.  The plan and apply steps below are the same decisions as plain host
 * logic (no GPU): the CPU tests and the sanitizer harness exercise them.
 * (Round 4's host frame path batched the planned pieces through
 * lvlip_csum_batch_host; round 5 retired it, slower from every source.)
 */
#ifndef LVLIP_SKB_H
#define LVLIP_SKB_H

#include <stdint.h>

#include "lvlip_csum.h"

#ifdef __cplusplus
extern "C" {
#endif
#pragma GCC visibility push(default)

typedef struct lvlip_frame {
    uint8_t *head;  /* Ethernet header (skb->head) */
    uint32_t len;   /* bytes valid from head */
} lvlip_frame;

/* ---- f1: RX ------------------------------------------------------------ */

/* Verdicts, in the order ip_rcv (src/ip_input.c:17-43) takes its decisions. */
#define LVLIP_RX_OK          1  /* ip_rcv hands the packet to icmpv4_incoming/tcp_in */
#define LVLIP_RX_NOT_IP      2  /* ethertype != 0x0800 (netdev_receive, src/netdev.c:67-80) */
#define LVLIP_RX_SHORT       3  /* frame shorter than 14 + 20, 14 + ihl*4, or (with
                                   VERIFY_L4) 14 + the IP total length; the
                                   reference has no such check (it would read past
                                   the frame) */
#define LVLIP_RX_BAD_VERSION 4  /* src/ip_input.c:22-25                          */
#define LVLIP_RX_BAD_IHL     5  /* src/ip_input.c:27-30                          */
#define LVLIP_RX_TTL0        6  /* src/ip_input.c:32-36                          */
#define LVLIP_RX_BAD_CSUM    7  /* checksum(ih, ihl*4, 0) != 0, src/ip_input.c:38-43 */
#define LVLIP_RX_BAD_L4      8  /* only with LVLIP_RX_VERIFY_L4                  */
#define LVLIP_RX_UNKNOWN_PROTO 9 /* not ICMP/TCP, src/ip_input.c:51-60         */

/* Also verify TCP (pseudo header, RFC arithmetic: the seed's carries are folded
 * back in) and ICMP checksums.  The reference never verifies them on RX
 * (src/tcp.c:79-81 is commented out, src/icmpv4.c:11 is a TODO), so this is off
 * by default. */
#define LVLIP_RX_VERIFY_L4   0x1u

/* Verdict per frame; frames are not modified.  Must run before ip_init_pkt's
 * in-place byte swaps (src/ip_input.c:47).  n <= LVLIP_MAX_BATCH / 2 (up to two
 * checksums per frame).  Returns 0 or LVLIP_E* (LVLIP_ERANGE: with
 * LVLIP_RX_VERIFY_L4, a frame longer than the context's arena).  A call of at
 * most the context's cpu_max frames runs on the calling thread
 * (lvlip_csum_ctx_set_cpu_max, include/lvlip_csum.h), with the same results. */
int lvlip_rx_verify(lvlip_csum_ctx *ctx, const lvlip_frame *frames, uint32_t n,
                    uint32_t flags, uint8_t *verdict);

/* Plan: verdict[] gets the header-field decisions, or 0 / 0x80|X = pending on
 * the checksums (X is the verdict if the header checksum passes);
 * iov[]/tag[] (capacity 2n) get the checksums to run, tag = frame << 1 | is_l4.
 * Returns the number of iov entries. */
uint32_t lvlip_rx_plan(const lvlip_frame *frames, uint32_t n, uint32_t flags,
                       uint8_t *verdict, lvlip_csum_iov *iov, uint32_t *tag);
/* Apply: BAD_CSUM if the header checksum fails, else BAD_L4 if an L4 one does,
 * else the deferred verdict (OK for 0). */
void lvlip_rx_apply(uint32_t n, uint8_t *verdict, uint32_t m, const uint32_t *tag,
                    const uint16_t *csum);

/* ---- f2: TX ------------------------------------------------------------ */

/* Frames fully built by tcp_transmit_skb / ip_output / icmpv4_reply except their
 * checksums.  Fills, stored raw as the reference stores them, the values the
 * reference computes with each field zeroed first (whatever the field holds):
 *   TCP  : checksum(tcp, ip.len - ihl*4, pseudo(saddr, daddr, 6, len))
 *          src/tcp_output.c:110,126 -> src/tcp.c:87-98 (u32 seed, carry lost);
 *          saddr/daddr are the header's network-order words, as
 *          tcp_transmit_skb passes htonl(sk->saddr), htonl(sk->daddr)
 *   ICMP : checksum(icmp, ip.len - ihl*4, 0), src/icmpv4.c:46-47
 *   IPv4 : checksum(ih, ihl*4, 0), src/ip_output.c:42,53 (ip_send_check)
 * The IPv4 header checksum does not cover the L4 bytes, so all 2n checksums
 * are one batch; n <= LVLIP_MAX_BATCH / 2.  Returns 0 or LVLIP_E* (frames
 * untouched on error): LVLIP_EINVAL for a malformed frame (not IPv4, ihl < 5,
 * shorter than 14 + its IP length), LVLIP_ERANGE for a frame longer than the
 * context's arena.  A call of at most the context's cpu_max frames runs on the
 * calling thread, with the same results and codes. */
int lvlip_tx_checksum(lvlip_csum_ctx *ctx, lvlip_frame *frames, uint32_t n);

/* Plan: fills iov[]/field[] (capacity 2n; field = where each result goes),
 * frames unmodified (each seed is compensated for its field's current value).
 * Returns the number of iov entries, or 0xFFFFFFFF if a frame is malformed. */
uint32_t lvlip_tx_plan(lvlip_frame *frames, uint32_t n, lvlip_csum_iov *iov,
                       uint8_t **field);
void lvlip_tx_apply(uint32_t m, uint8_t *const *field, const uint16_t *csum);

/* ---- f4: RFC 1624 incremental update for the echo reply ----------------- */

/* icmpv4_reply (src/icmpv4.c:44-47) turns an echo request into the reply by
 * setting type 8 -> 0 and recomputing the ICMP checksum over the whole
 * message.  Given the request's stored checksum field (raw u16, as loaded
 * from the frame) of a request whose ICMP checksum VERIFIED (checksum over
 * the message == 0, e.g. LVLIP_RX_OK from lvlip_rx_verify with
 * LVLIP_RX_VERIFY_L4), returns the reply's checksum field, bit-identical to
 * the reference's full recomputation, without reading the message; or
 * LVLIP_CSUM_RECOMPUTE in the one case the field cannot decide (the reply's
 * one's-complement sum is 0xffff, which is also what an all-zero reply
 * gives), where the caller recomputes with checksum(). */
#define LVLIP_CSUM_RECOMPUTE 0xFFFFFFFFu
uint32_t lvlip_icmp_echo_reply_csum(uint16_t req_csum);

/* In place over n verified echo-request frames: ICMP type 8 -> 0 and the
 * checksum field updated as above (recomputed with checksum() in the
 * undecidable case).  Returns the number of frames that needed the
 * recomputation, or 0xFFFFFFFF (frames untouched) if one is not an ICMP echo
 * request. */
uint32_t lvlip_icmp_echo_reply_fill(lvlip_frame *frames, uint32_t n);

/* ---- f1/f2 over level-ip's own skb queues -------------------------------- */

/* The same calls over an sk_buff_head (include/skbuff.h:25-29) as level-ip
 * fills it, walked in list order through the intrusive list_head at the start
 * of every sk_buff (include/list.h; LP64 offsets of include/skbuff.h:9-23:
 * len 40, end 56, head 64, data 72).  The queue is only read.
 *
 * RX: skbs as netdev_rx_loop allocates and fills them (src/netdev.c:86-101,
 * alloc_skb src/skbuff.c:5-20): the frame is skb->data .. skb->end (tun_read
 * writes it at skb->data; the rest of the BUFLEN buffer is zero).  verdict[k]
 * is the k-th skb's; cap is verdict's capacity.  Returns the number of skbs,
 * LVLIP_ERANGE if more than cap, or LVLIP_E*. */
struct sk_buff_head;
int lvlip_rx_verify_skb_list(lvlip_csum_ctx *ctx, struct sk_buff_head *q, uint32_t flags,
                             uint8_t *verdict, uint32_t cap);

/* TX: skbs as ip_output leaves them before dst_neigh_output
 * (src/ip_output.c:14-56): skb->data at the IPv4 header, skb->len covering it
 * and the TCP/ICMP segment, the Ethernet header's 14 bytes reserved in front
 * (the frame is skb->data - 14 .. skb->data + skb->len).  Fills the TCP/ICMP
 * and IPv4 checksums as lvlip_tx_checksum, i.e. what tcp_transmit_skb
 * (src/tcp_output.c:126), icmpv4_reply (src/icmpv4.c:47) and ip_send_check
 * (src/ip_output.c:53) would have stored.  Returns the number of skbs or
 * LVLIP_E* (skbs untouched on error). */
int lvlip_tx_checksum_skb_list(lvlip_csum_ctx *ctx, struct sk_buff_head *q);

/* ---- f1/f2 on the calling thread (no context, no GPU) --------------------- */

/* The same calls computed by the library's CPU code on the calling thread,
 * with the same results and return codes (LVLIP_EINVAL on a malformed frame,
 * frames untouched; no arena, so LVLIP_ERANGE only for an RX queue longer than
 * cap).  A context's calls of at
 * most its cpu_max frames run these (lvlip_csum_ctx_set_cpu_max,
 * include/lvlip_csum.h).  A caller that deferred its TX checksums also calls
 * them when the GPU call fails (LVLIP_ENODEV, LVLIP_EHIP, LVLIP_ENOMEM,
 * LVLIP_ERANGE; or no context could be made), so that no frame leaves with a
 * deferred, still-zero field (src/ip_output.c:53-55 sends
 * whatever the fields hold).  Reentrant; one checksum() per field, as the
 * reference's call sites. */
int lvlip_rx_verify_cpu(const lvlip_frame *frames, uint32_t n, uint32_t flags,
                        uint8_t *verdict);
int lvlip_tx_checksum_cpu(lvlip_frame *frames, uint32_t n);
int lvlip_rx_verify_skb_list_cpu(struct sk_buff_head *q, uint32_t flags,
                                 uint8_t *verdict, uint32_t cap);
int lvlip_tx_checksum_skb_list_cpu(struct sk_buff_head *q);

/* ---- f1/f2/f4 on device-resident frames ---------------------------------- */

/* Frames already in HBM (a receive ring filled by a GPU-direct NIC, or frames
 * built on the GPU): one frame = `len` bytes at base + offset, Ethernet header
 * first.  Parse, checksum and apply run as one kernel on the caller's stream;
 * nothing returns to the host.  Pointers are device pointers; `base` is 16-B
 * aligned and readable up to the last frame's end rounded up to 16 B.
 * `workspace` is reserved and may be NULL: lvlip_frames_workspace_bytes()
 * returns 0 (ABI 1 kept the argument from the earlier three-kernel form). */
typedef struct lvlip_frame_desc {
    uint64_t offset;
    uint32_t len;
    uint32_t reserved;  /* 0 */
} lvlip_frame_desc;

size_t lvlip_frames_workspace_bytes(uint32_t n);

/* verdict[i] as lvlip_rx_verify (same decisions, same flags). */
int lvlip_rx_verify_dev(const void *base, const lvlip_frame_desc *frames, uint32_t n,
                        uint32_t flags, uint8_t *verdict, void *workspace, void *stream);

/* Fills the TCP/ICMP and IPv4 checksums in place, as lvlip_tx_checksum.  A
 * malformed frame (not IPv4, short) is left untouched and gets status 0 (1 =
 * filled); status may be NULL. */
int lvlip_tx_checksum_dev(void *base, const lvlip_frame_desc *frames, uint32_t n,
                          uint8_t *status, void *workspace, void *stream);

/* f4 on frames in HBM: lvlip_icmp_echo_reply_fill in one launch, one lane per
 * frame.  Every frame that is an IPv4 ICMP echo request (type 8, code 0, the
 * message inside the frame) becomes the reply's ICMP part: type 0 and the
 * RFC 1624 checksum field derived from the request's field alone; in the one
 * undecidable case (LVLIP_CSUM_RECOMPUTE) the lane sums the message itself.
 * status[i] (may be NULL): 1 updated from the field, 2 recomputed, 0 not an
 * echo request (frame untouched).  Nothing else of the message is read.
 *
 * PRECONDITION: the request's ICMP checksum verified (e.g. the frame got
 * LVLIP_RX_OK from lvlip_rx_verify_dev with LVLIP_RX_VERIFY_L4).  Only then
 * is the field bit-identical to icmpv4_reply's full recomputation
 * (src/icmpv4.c:44-47).  The call does NOT check it: status 1 does not mean
 * the request verified, and for a request whose checksum is wrong the field
 * written differs from the reference's (which answers such requests with a
 * correct checksum, src/icmpv4.c:11 never verifies).  For frames nobody
 * verified, use lvlip_icmp_echo_reply_dev_ex with LVLIP_ECHO_FULL. */
int lvlip_icmp_echo_reply_dev(void *base, const lvlip_frame_desc *frames, uint32_t n,
                              uint8_t *status, void *stream);

/* flags of lvlip_icmp_echo_reply_dev_ex */
#define LVLIP_ECHO_FULL 0x1u /* sum every request's message (one lane per frame)
                                and write icmpv4_reply's field exactly: for
                                any request, verified or not; status 2.  Costs
                                a full read of each message by its one lane
                                (serial 16-B loads), where flags 0 reads one
                                64-B sector per frame (DESIGN.md §9 times
                                both) */

/* lvlip_icmp_echo_reply_dev with flags: 0 is lvlip_icmp_echo_reply_dev (the
 * precondition above holds); LVLIP_ECHO_FULL computes the reply's field as
 * icmpv4_reply does, from the whole message with type and field zeroed
 * (src/icmpv4.c:45-47), bit-identical for every echo request.  Other flag bits
 * are LVLIP_EINVAL. */
int lvlip_icmp_echo_reply_dev_ex(void *base, const lvlip_frame_desc *frames, uint32_t n,
                                 uint32_t flags, uint8_t *status, void *stream);

/* RFC 1071 pseudo-header seed with the carries folded back (for RX verify of
 * checksums produced by RFC-correct peers). */
uint32_t lvlip_pseudo_sum_rfc(uint32_t saddr, uint32_t daddr, uint8_t proto,
                              uint16_t len);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif /* LVLIP_SKB_H */
