"""CPU model of the block sort's work split for one 900 KB block (dev tool).

Prints the packed-key geometry and how the rotations of the first block of a
synthetic chromosome fall into the size classes the GPU sort uses
(W <= 64, S <= 256, M1 <= 1024, M2 <= 2048, M3 <= 4096, L > 4096), at the top
level and after one 8-bit partition of the L buckets.

    python tools/bwt_class_sim.py [kind]      # kind: starch_gen_bed kind (0 = BED3)
"""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import starch_amd  # noqa: E402
from tests import oracle_lib  # noqa: E402


def classify(sizes):
    out, el = collections.Counter(), collections.Counter()
    for m in sizes:
        if m < 2:
            continue
        k = ("W" if m <= 64 else "S" if m <= 256 else "M1" if m <= 1024 else "M2" if m <= 2048
             else "M3" if m <= 4096 else "L")
        out[k] += 1
        el[k] += int(m)
    return out, el


def main():
    kind = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    bed = starch_amd.gen_bed(kind, int(os.environ.get("TOTAL", "100000000")), chroms=[0])
    _, segs = oracle_lib.transform(bytes(bed))
    blk = np.frombuffer(segs[0][2][:899981], dtype=np.uint8)
    n = len(blk)
    used = np.unique(blk)
    B = int(np.ceil(np.log2(len(used))))
    D = 64 // B
    KB = D * B
    m = np.zeros(256, np.uint64)
    m[used] = np.arange(len(used))
    sym = m[blk]
    ext = np.concatenate([sym, sym[:64]])
    key = np.zeros(n, np.uint64)
    for k in range(D):
        key = (key << np.uint64(B)) | ext[k:k + n]
    print("nInUse", len(used), "B", B, "D", D)
    _, cnt = np.unique(key, return_counts=True)
    print("distinct keys", len(cnt), "tied elems", int(cnt[cnt > 1].sum()), "max group", int(cnt.max()))
    top = (key >> np.uint64(KB - 12)).astype(np.int64)
    sizes = np.bincount(top, minlength=4096)
    c0, e0 = classify(sizes)
    print("level0 items", dict(c0))
    print("level0 elems", dict(e0))
    tot, tel = collections.Counter(), collections.Counter()
    for b in np.nonzero(sizes > 4096)[0]:
        sub = key[top == b]
        d = ((sub >> np.uint64(KB - 20)) & np.uint64(255)).astype(np.int64)
        c2, e2 = classify(np.bincount(d, minlength=256))
        tot += c2
        tel += e2
    print("level1 (from L) items", dict(tot))
    print("level1 (from L) elems", dict(tel))


if __name__ == "__main__":
    main()


def lsd_model(key, KB, groups_sel=None):
    """For each leaf group (top-12-bit bucket or its 8-bit L partition), the
    k3_sort_lds path it takes: MSD digit + compare, or LSD fallback."""
    top = (key >> np.uint64(KB - 12))
    order = np.argsort(key, kind="stable")
    sk = key[order]
    res = collections.defaultdict(lambda: [0, 0, 0, 0])   # class -> [groups, lsd groups, lsd passes, sum z^2]
    ratios = collections.defaultdict(list)
    def leaf(sub):
        m = len(sub)
        if m < 2 or m <= 64:
            return
        cls = "S" if m <= 256 else "M1" if m <= 1024 else "M2" if m <= 2048 else "M3"
        E = {"S": 4, "M1": 4, "M2": 8, "M3": 16}[cls]
        CAP = {"S": 256, "M1": 1024, "M2": 2048, "M3": 4096}[cls]
        IDXB = 8 if CAP <= 256 else 12
        KEYB = 64 - IDXB
        DB = 8 if CAP <= 256 else (10 if CAP <= 1024 else 11)
        km = sub & np.uint64((1 << KEYB) - 1)
        diff = np.bitwise_or.reduce(km ^ km[0])
        r = res[cls]
        r[0] += 1
        if diff == 0:
            return
        hb = int(diff).bit_length() - 1
        lo = max(hb + 1 - DB, 0)
        dg = ((km >> np.uint64(lo)) & np.uint64((1 << DB) - 1)).astype(np.int64)
        z = np.bincount(dg)
        r[3] += int((z.astype(np.int64) ** 2).sum())
        ratios[cls].append(float((z.astype(np.int64) ** 2).sum()) / m)
        if z.max() > 256 // E:
            r[1] += 1
            r[2] += sum(1 for d in range(0, KEYB, 8) if (int(diff) >> d) & 0xFF)
    tops = (sk >> np.uint64(KB - 12)).astype(np.int64)
    bounds = np.flatnonzero(np.diff(tops)) + 1
    for g in np.split(sk, bounds):
        if len(g) > 4096:
            d = ((g >> np.uint64(KB - 20)) & np.uint64(255)).astype(np.int64)
            for h in np.split(g, np.flatnonzero(np.diff(d)) + 1):
                leaf(h)
        else:
            leaf(g)
    for k, v in sorted(res.items()):
        print("%-3s groups %6d  lsd %6d  lsd passes %6d  sum z^2" % (k, v[0], v[1], v[2]), v[3])
        rr = np.array(ratios[k])
        print("    sum z^2 / m quantiles 50/75/90/95/99/max:",
              np.percentile(rr, [50, 75, 90, 95, 99, 100]).round(1) if len(rr) else "-")


if __name__ == "__main__" and os.environ.get("LSD_MODEL"):
    kind = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    bed = starch_amd.gen_bed(kind, int(os.environ.get("TOTAL", "100000000")), chroms=[0])
    _, segs = oracle_lib.transform(bytes(bed))
    blk = np.frombuffer(segs[0][2][:899981], dtype=np.uint8)
    used = np.unique(blk)
    B = int(np.ceil(np.log2(len(used))))
    D = 64 // B
    m = np.zeros(256, np.uint64)
    m[used] = np.arange(len(used))
    sym = m[blk]
    ext = np.concatenate([sym, sym[:64]])
    key = np.zeros(len(blk), np.uint64)
    for k in range(D):
        key = (key << np.uint64(B)) | ext[k:k + len(blk)]
    lsd_model(key, D * B)


def rank_cost_model(key, KB):
    """Comparison-rank cost of k3_sort_grp in digit order: for each wave, sum
    over its rows of the largest sub-bucket a row touches (loop trip count),
    for several MSD digit widths."""
    order = np.argsort(key, kind="stable")
    sk = key[order]
    tops = (sk >> np.uint64(KB - 12)).astype(np.int64)
    leaves = []
    for g in np.split(sk, np.flatnonzero(np.diff(tops)) + 1):
        if len(g) > 4096:
            d = ((g >> np.uint64(KB - 20)) & np.uint64(255)).astype(np.int64)
            leaves += [h for h in np.split(g, np.flatnonzero(np.diff(d)) + 1) if len(h) > 64]
        elif len(g) > 64:
            leaves.append(g)
    for cls, lo_m, hi_m, NW, E, dbs in (("S", 65, 256, 1, 4, (8, 9, 10, 11)),
                                         ("M1", 257, 1024, 4, 4, (10, 11, 12, 13)),
                                         ("M2", 1025, 2048, 4, 8, (11, 12, 13, 14))):
        gs = [g for g in leaves if lo_m <= len(g) <= hi_m]
        if not gs:
            continue
        IDXB = 8 if NW * 64 * E <= 256 else 12
        KEYB = 64 - IDXB
        out = []
        for DB in dbs:
            tot = 0
            for g in gs:
                km = g & np.uint64((1 << KEYB) - 1)
                diff = int(np.bitwise_or.reduce(km ^ km[0]))
                if diff == 0:
                    continue
                hb = diff.bit_length() - 1
                lo = max(hb + 1 - DB, 0)
                dg = ((km >> np.uint64(lo)) & np.uint64((1 << DB) - 1)).astype(np.int64)
                z = np.bincount(dg, minlength=1 << DB)
                zs = np.repeat(z[z > 0], z[z > 0])      # sub-bucket size at each digit-order position
                m = len(g)
                wc = []
                for w in range(NW):
                    c = 0
                    for e in range(E):
                        a = w * 64 * E + e * 64
                        if a < m:
                            c += int(zs[a:min(a + 64, m)].max())
                    wc.append(c)
                tot += max(wc)
            out.append((DB, round(tot / len(gs), 1)))
        print("%-3s %5d groups, avg elems %6.1f, per-group wave loop trips by digit bits:" %
              (cls, len(gs), np.mean([len(g) for g in gs])), out)


if __name__ == "__main__" and os.environ.get("RANK_MODEL"):
    kind = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    bed = starch_amd.gen_bed(kind, int(os.environ.get("TOTAL", "100000000")), chroms=[0])
    _, segs = oracle_lib.transform(bytes(bed))
    blk = np.frombuffer(segs[0][2][:899981], dtype=np.uint8)
    used = np.unique(blk)
    B = int(np.ceil(np.log2(len(used))))
    D = 64 // B
    mp = np.zeros(256, np.uint64)
    mp[used] = np.arange(len(used))
    sym = mp[blk]
    ext = np.concatenate([sym, sym[:64]])
    key = np.zeros(len(blk), np.uint64)
    for k in range(D):
        key = (key << np.uint64(B)) | ext[k:k + len(blk)]
    rank_cost_model(key, D * B)


def two_level_model(key, KB, lim=32, db2s=(4, 5, 6, 8)):
    """M groups: sum z^2 / m after the first MSD digit, and after a second digit
    of db2 bits (the bits right below the first) on sub-buckets larger than lim."""
    order = np.argsort(key, kind="stable")
    sk = key[order]
    tops = (sk >> np.uint64(KB - 12)).astype(np.int64)
    leaves = []
    for g in np.split(sk, np.flatnonzero(np.diff(tops)) + 1):
        if len(g) > 4096:
            d = ((g >> np.uint64(KB - 20)) & np.uint64(255)).astype(np.int64)
            leaves += [h for h in np.split(g, np.flatnonzero(np.diff(d)) + 1) if len(h) > 256]
        elif len(g) > 256:
            leaves.append(g)
    for DB2 in db2s:
        r1, r2, mx2 = [], [], []
        for g in leaves:
            m = len(g)
            DB = 10 if m <= 1024 else (11 if m <= 2048 else 11)
            km = g & np.uint64((1 << 52) - 1)
            diff = int(np.bitwise_or.reduce(km ^ km[0]))
            if diff == 0:
                continue
            hb = diff.bit_length() - 1
            lo = max(hb + 1 - DB, 0)
            d1 = ((km >> np.uint64(lo)) & np.uint64((1 << DB) - 1)).astype(np.int64)
            z1 = np.bincount(d1)
            r1.append((z1.astype(np.int64) ** 2).sum() / m)
            lo2 = max(lo - DB2, 0)
            d2 = ((km >> np.uint64(lo2)) & np.uint64((1 << (lo - lo2)) - 1)).astype(np.int64) if lo > 0 else np.zeros(m, np.int64)
            big = z1[d1] > lim
            comp = np.where(big, (d1 << 16) | d2, d1 << 16)
            _, z2 = np.unique(comp, return_counts=True)
            r2.append((z2.astype(np.int64) ** 2).sum() / m)
            mx2.append(z2.max())
        print("DB2 %d: groups %d  ratio1 median %.1f mean %.1f | ratio2 median %.1f mean %.1f p95 %.1f | max z2 p50 %d p95 %d" %
              (DB2, len(r1), np.median(r1), np.mean(r1), np.median(r2), np.mean(r2), np.percentile(r2, 95),
               np.median(mx2), np.percentile(mx2, 95)))


if __name__ == "__main__" and os.environ.get("TWO_LEVEL"):
    kind = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    bed = starch_amd.gen_bed(kind, int(os.environ.get("TOTAL", "100000000")), chroms=[0])
    _, segs = oracle_lib.transform(bytes(bed))
    blk = np.frombuffer(segs[0][2][:899981], dtype=np.uint8)
    used = np.unique(blk)
    B = int(np.ceil(np.log2(len(used))))
    D = 64 // B
    mp = np.zeros(256, np.uint64)
    mp[used] = np.arange(len(used))
    sym = mp[blk]
    ext = np.concatenate([sym, sym[:64]])
    key = np.zeros(len(blk), np.uint64)
    for k in range(D):
        key = (key << np.uint64(B)) | ext[k:k + len(blk)]
    two_level_model(key, D * B)
