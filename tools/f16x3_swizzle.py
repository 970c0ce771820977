"""Search the 16-B-chunk XOR swizzles of the f16x3 conv LDS images (128-B rows:
xh 32 ch | xl 32 ch of a 32-channel chunk) for conflict-free ds_read_b128
fragment reads.  Halo image: physical chunk = k ^ SH[(y & 3) * 4 + (x & 3)]
(halo coords y, x); weight image: physical chunk = k ^ SW[co & 15].
python tools/f16x3_swizzle.py"""
import itertools
import random

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]


def halo_cost(SH):
    worst = 0
    total = 0
    for pyy, pxx in itertools.product(range(2), range(2)):
        for kd, kh, kw in itertools.product(range(3), range(3), range(3)):
            for p in range(2):
                for g in GROUPS:
                    cnt = {}
                    for l in g:
                        vq, cq = l & 15, l >> 4
                        y = pyy * 4 + (vq >> 2) + kh
                        x = pxx * 4 + (vq & 3) + kw
                        k = 4 * p + cq
                        q = 8 * (x & 1) + (k ^ SH[(y & 3) * 4 + (x & 3)])
                        cnt[q] = cnt.get(q, 0) + 1
                    m = max(cnt.values())
                    worst = max(worst, m)
                    total += m - 1
    return worst, total


def weight_cost(SW):
    worst = total = 0
    for p in range(2):
        for g in GROUPS:
            cnt = {}
            for l in g:
                vq, cq = l & 15, l >> 4
                q = 8 * (vq & 1) + ((4 * p + cq) ^ SW[vq])
                cnt[q] = cnt.get(q, 0) + 1
            m = max(cnt.values())
            worst = max(worst, m)
            total += m - 1
    return worst, total


def search(cost, n, iters=200000, seed=0):
    rng = random.Random(seed)
    best = [0] * n
    bc = cost(best)
    cur, cc = best[:], bc
    for it in range(iters):
        cand = cur[:]
        cand[rng.randrange(n)] = rng.randrange(8)
        c = cost(cand)
        if c <= cc or rng.random() < 0.01:
            cur, cc = cand, c
            if c < bc:
                best, bc = cand[:], c
                if bc[1] == 0:
                    break
    return best, bc


if __name__ == "__main__":
    print("no swizzle: halo", halo_cost([0] * 16), "weights", weight_cost([0] * 16))
    sw, c = search(weight_cost, 16, 20000)
    print("SW", sw, c)
    sh, c = search(halo_cost, 16, 20000)
    print("SH", sh, c)


def halo_constraints():
    """every (instruction, lane group) as a list of (slot, key) with key = 8 (x & 1) + k:
    lanes of one group need distinct 8 (x & 1) + (k ^ S[slot])."""
    cons = []
    for pyy, pxx in itertools.product(range(2), range(2)):
        for kd, kh, kw in itertools.product(range(1), range(3), range(3)):
            for p in range(2):
                for g in GROUPS:
                    items = []
                    for l in g:
                        vq, cq = l & 15, l >> 4
                        y = pyy * 4 + (vq >> 2) + kh
                        x = pxx * 4 + (vq & 3) + kw
                        items.append(((y & 3) * 4 + (x & 3), x & 1, 4 * p + cq))
                    cons.append(items)
    return cons


def exact(cons, n=16):
    S = [None] * n

    def ok():
        for items in cons:
            seen = set()
            for slot, par, k in items:
                if S[slot] is None:
                    continue
                q = 8 * par + (k ^ S[slot])
                if q in seen:
                    return False
                seen.add(q)
        return True

    def rec(i):
        if i == n:
            return True
        for v in range(8):
            S[i] = v
            if ok() and rec(i + 1):
                return True
        S[i] = None
        return False

    return S if rec(0) else None


if __name__ == "__main__":
    sh = exact(halo_constraints())
    print("SH exact", sh, halo_cost(sh) if sh else None)
    wc = [[(vq, vq & 1, 4 * p + cq) for l in g for vq, cq in [(l & 15, l >> 4)]] for p in range(2) for g in GROUPS]
    sw = exact(wc)
    print("SW exact", sw, weight_cost(sw) if sw else None)
