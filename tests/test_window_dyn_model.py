"""CPU model of the lab kernel k_window_dyn's claim / window / count logic
(level-ip_amd/csrc/lab_kernels.hip): one workgroup of WPB waves with random
speeds, its LDS claim ring starting as garbage.  Every packet of the
workgroup's pool must be issued exactly once, and no invalid index may reach
a descriptor fetch or a result store.  (A first version initialised only 64 of
the 128 static slots for G = 1 and counted valid packets by popcount instead of
as a prefix: this model reproduces the resulting out-of-range descriptor fetch,
which faulted the GPU once in round 3.)"""
import random

import pytest

import heapq
BAD = 0xffffffff
def run(n, G, WPB, grid, bx, seed):
    rnd = random.Random(seed)
    GPW = 64 // G
    nw = grid * WPB
    ng = (n + G - 1) // G
    def item_pkt(it, p):
        if it == BAD: return BAD
        g = (it // WPB) * nw + bx * WPB + (it % WPB)
        k = g * G + p
        return k if (g < ng and k < n) else BAD
    ctr = [2 * GPW * WPB]
    written = {}
    waves = []
    for w in range(WPB):
        claim = [[rnd.randrange(0, 1 << 32) for _ in range(GPW)] for _ in range(4)]  # garbage LDS
        for q in range(2 * GPW):
            claim[q // GPW][q % GPW] = q * WPB + w
        waves.append(dict(w=w, claim=claim, cnt=0, open=True, ip=0, claiming=True, speed=rnd.uniform(0.7, 1.3)))
    def wave_pkt(W, k):
        return item_pkt(W['claim'][(k >> 6) & 3][(k & 63) // G], k % G)
    def extend(W, v):
        if not W['open']: return
        c = 0
        while c < 64 and wave_pkt(W, v * 64 + c) != BAD: c += 1
        W['cnt'] = v * 64 + c
        W['open'] = c == 64
    def fetch(W, v):
        for l in range(64):
            k = v * 64 + l
            k = k if k < W['cnt'] else (W['cnt'] - 1 if W['cnt'] else 0)
            pk = wave_pkt(W, k) if W['cnt'] else 0
            assert pk != BAD, ('fetch BAD', W['w'], v, l)
    def do_claim(W):
        it = BAD
        if W['claiming']:
            it = ctr[0]; ctr[0] += 1
        ip = W['ip']
        W['claim'][((ip >> 6) + 2) & 3][(ip & 63) // G] = it
        if item_pkt(it, 0) == BAD: W['claiming'] = False
    for W in waves:
        extend(W, 0); extend(W, 1)
    events = []
    for W in waves:
        if W['cnt'] == 0: continue
        fetch(W, 0); fetch(W, 1)
        do_claim(W)
        heapq.heappush(events, (W['speed'] * rnd.random(), W['w']))
    while events:
        t, wi = heapq.heappop(events)
        W = waves[wi]
        ip = W['ip']
        assert ip < W['cnt']
        pk = wave_pkt(W, ip)
        assert pk != BAD, ('issue BAD', wi, ip)
        assert pk not in written, ('dup', pk)
        written[pk] = wi
        W['ip'] = ip = ip + 1
        if ip < W['cnt']:
            if ip & 63 == 0:
                extend(W, (ip >> 6) + 1)
                fetch(W, (ip >> 6) + 1)
            if ip % G == 0: do_claim(W)
            heapq.heappush(events, (t + W['speed'] * rnd.uniform(0.5, 1.5), wi))
    # pool of this workgroup
    pool = set()
    for r in range(WPB):
        j = 0
        while True:
            g = j * nw + bx * WPB + r
            if g >= ng: break
            for p in range(G):
                if g * G + p < n: pool.add(g * G + p)
            j += 1
    assert set(written) == pool, (len(written), len(pool))
    return len(pool), max(W['ip'] for W in waves), min(W['ip'] for W in waves if W['ip']) if any(W['ip'] for W in waves) else 0


@pytest.mark.parametrize("seed", range(24))
def test_window_dyn_claims_cover_the_pool_once(seed):
    rnd = random.Random(1000 + seed)
    G = rnd.choice([1, 2, 4])
    WPB = rnd.choice([8, 12])
    grid = rnd.choice([8, 16, 256])
    n = rnd.choice([1, 5, 100, 3000, 50000, 200000]) + rnd.randrange(0, 7)
    ng = (n + G - 1) // G
    while grid > 8 and grid * WPB > ng:
        grid //= 2
    bx = rnd.randrange(grid)
    run(n, G, WPB, grid, bx, seed)
