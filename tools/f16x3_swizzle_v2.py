"""Exact search of the 16-B-chunk XOR swizzles of the f16x3 v2 conv's LDS images
(64-B rows: xh 16 ch | xl 16 ch of a 16-channel chunk; 4 chunks per row) for
conflict-free ds_read_b128 fragment reads.  Halo rows (ht, hy, hx) of a 6 x 6 x 10
halo, physical chunk = k ^ SH[(hy & 3) * 4 + (hx & 3)] (2-bit); weight rows co
(2 taps x 160), physical chunk = k ^ SW[co & 15].  A fragment read: lane (vq,
cq) of wave (pxx, th) reads voxel (t = 2 th + i, y = vq >> 2, x = 4 pxx + (vq & 3))
shifted by tap a (cq < 2) or tap b (cq >= 2), chunk (cq & 1) + 2 p.
python tools/f16x3_swizzle_v2.py"""
import itertools

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]
TAPS = [(kd, kh, kw) for kd in range(3) for kh in range(3) for kw in range(3)]
PAIRS = [(TAPS[2 * q], TAPS[2 * q + 1] if 2 * q + 1 < 27 else TAPS[2 * q]) for q in range(14)]


def halo_cons():
    cons = []
    for pxx, th, i in itertools.product(range(2), range(2), range(2)):
        for ta, tb in PAIRS:
            for p in range(2):
                for g in GROUPS:
                    items = []
                    for l in g:
                        vq, cq = l & 15, l >> 4
                        kd, kh, kw = ta if cq < 2 else tb
                        t, y, x = 2 * th + i + kd, (vq >> 2) + kh, 4 * pxx + (vq & 3) + kw
                        row = (t * 6 + y) * 10 + x
                        items.append(((y & 3) * 4 + (x & 3), row & 3, (cq & 1) + 2 * p))
                    cons.append(items)
    return cons


def weight_cons():
    cons = []
    for p in range(2):
        for g in GROUPS:
            items = []
            for l in g:
                vq, cq = l & 15, l >> 4
                tsel = 0 if cq < 2 else 1
                co = vq                                  # co & 15 = vq
                row = tsel * 160 + co
                items.append((co & 15, row & 3, (cq & 1) + 2 * p))
            cons.append(items)
    return cons


def exact(cons, n=16, vals=4):
    S = [None] * n

    def ok():
        for items in cons:
            seen = set()
            for slot, rq, k in items:
                if S[slot] is None:
                    continue
                q = 4 * rq + (k ^ S[slot])
                if q in seen:
                    return False
                seen.add(q)
        return True

    def rec(i):
        if i == n:
            return True
        for v in range(vals):
            S[i] = v
            if ok() and rec(i + 1):
                return True
        S[i] = None
        return False

    return S if rec(0) else None


if __name__ == "__main__":
    print("SH", exact(halo_cons()))
    print("SW", exact(weight_cons()))
