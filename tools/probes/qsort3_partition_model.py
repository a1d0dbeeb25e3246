#!/usr/bin/env python3
"""Dev model (not product code): one partition step of bzip2's fallbackQSort3
(bz:blocksort.c:93-180) computed in closed form -- prefix counts, the
crossing point, and the two rotating queues resolved by pointer chasing -- and
checked against the serial step on random inputs.  This is the arithmetic a
workgroup-parallel exact replay uses (periodic blocks).

    python tools/probes/qsort3_partition_model.py
"""
import random


def main():
    r = random.Random(5)
    for t in range(20000):
        n = r.randint(1, 60)
        keys = [r.randrange(r.randint(1, 5)) for _ in range(n)]
        lo, hi = 0, n - 1
        med = keys[r.choice([lo, (lo + hi) // 2, hi])]
        perm_s, rng_s = serial_step_idx(keys, lo, hi, med)
        perm_c, rng_c = closed_form_idx(keys, lo, hi, med)
        assert perm_s == perm_c and rng_s == rng_c, (t, keys, med, perm_s, perm_c, rng_s, rng_c)
    print("closed form == serial fallbackQSort3 partition on 20000 random ranges")


def serial_step_idx(keys, lo, hi, med):
    """serial_step on (key, original index) pairs -> final index order."""
    a = list(range(len(keys)))
    unLo = ltLo = lo
    unHi = gtHi = hi
    while True:
        while unLo <= unHi:
            n = keys[a[unLo]] - med
            if n == 0:
                a[unLo], a[ltLo] = a[ltLo], a[unLo]
                ltLo += 1
                unLo += 1
                continue
            if n > 0:
                break
            unLo += 1
        while unLo <= unHi:
            n = keys[a[unHi]] - med
            if n == 0:
                a[unHi], a[gtHi] = a[gtHi], a[unHi]
                gtHi -= 1
                unHi -= 1
                continue
            if n < 0:
                break
            unHi -= 1
        if unLo > unHi:
            break
        a[unLo], a[unHi] = a[unHi], a[unLo]
        unLo += 1
        unHi -= 1
    if gtHi < ltLo:
        return a, None
    n = min(ltLo - lo, unLo - ltLo)
    for i in range(n):
        a[lo + i], a[unLo - n + i] = a[unLo - n + i], a[lo + i]
    m = min(hi - gtHi, gtHi - unHi)
    for i in range(m):
        a[unLo + i], a[hi - m + 1 + i] = a[hi - m + 1 + i], a[unLo + i]
    return a, (lo + unLo - ltLo - 1, hi - (gtHi - unHi) + 1)


def closed_form_idx(keys, lo, hi, med):
    """The same permutation from counts: '>' from the left pair with '<' from
    the right while they have not crossed (k swaps, crossing point X); on each
    side the '=' keys go to the outer end in scan order, and the queue of '<'
    (mirrored: '>') keys rotates once per '=' -- the element at step q is its
    own arrival, or (when step q met an '=') the one that stood at the queue
    front, lo + #'=' before q: a pointer chase, log depth by pointer jumping."""
    a = list(range(len(keys)))
    cls = {i: (keys[i] > med) - (keys[i] < med) for i in range(lo, hi + 1)}
    g = [i for i in range(lo, hi + 1) if cls[i] > 0]
    l = [i for i in range(hi, lo - 1, -1) if cls[i] < 0]
    k = 0
    while k < min(len(g), len(l)) and g[k] < l[k]:
        k += 1
    lk = l[k - 1] if k else hi + 1
    X = min(g[k] if k < len(g) else hi + 1, lk)
    sin = {g[j]: l[j] for j in range(k)}
    sout = {l[j]: g[j] for j in range(k)}
    src = {q: (sin.get(q, q) if q < X else sout.get(q, q)) for q in range(lo, hi + 1)}
    out = list(a)
    eqb, e = {}, 0
    for q in range(lo, X):
        eqb[q] = e
        e += cls[src[q]] == 0
    ltLo = lo + e
    eqL = [q for q in range(lo, X) if cls[src[q]] == 0]
    for i, q in enumerate(eqL):
        out[lo + i] = src[q]
    for q in range(ltLo, X):
        p = q
        while cls[src[p]] == 0:
            p = lo + eqb[p]
        out[q] = src[p]
    eqa, e = {}, 0
    for q in range(hi, X - 1, -1):
        eqa[q] = e
        e += cls[src[q]] == 0
    gtHi = hi - e
    eqR = [q for q in range(hi, X - 1, -1) if cls[src[q]] == 0]
    for i, q in enumerate(eqR):
        out[hi - i] = src[q]
    for q in range(X, gtHi + 1):
        p = q
        while cls[src[p]] == 0:
            p = hi - eqa[p]
        out[q] = src[p]
    unLo, unHi = X, X - 1
    if gtHi < ltLo:
        return out, None
    n = min(ltLo - lo, unLo - ltLo)
    for i in range(n):
        out[lo + i], out[unLo - n + i] = out[unLo - n + i], out[lo + i]
    m = min(hi - gtHi, gtHi - unHi)
    for i in range(m):
        out[unLo + i], out[hi - m + 1 + i] = out[hi - m + 1 + i], out[unLo + i]
    return out, (lo + unLo - ltLo - 1, hi - (gtHi - unHi) + 1)


if __name__ == "__main__":
    main()
