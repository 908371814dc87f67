/*
 * oracle/ref_clock.c — a fixed clock for level-ip's initial send sequence
 * number.  TEST INFRASTRUCTURE ONLY.
 *
 * generate_iss() (src/tcp.c:150-154) returns time(NULL) * rand(): two runs of
 * the stack started in different seconds send different sequence numbers, so
 * their frames (and checksums) differ.  oracle/Makefile redirects tcp.o's
 * `time` call to this function in both builds the TX composition test
 * compares (_ref/libref_fixclock.so, the reference as it is, and
 * _ref/libref_txq.so, the batch-and-dispatch build), objcopy on our own copy
 * of the object, so both send the same bytes.  rand() is unseeded (the same
 * sequence in every fresh process) and the timer thread is not started, so
 * generate_port() (src/tcp.c:138-148) is deterministic too.
 */
#include <time.h>

time_t lvlip_ref_fixed_time(time_t *t)
{
    const time_t now = 1700000000;
    if (t) *t = now;
    return now;
}
