"""Seeded test corpora shared by tests/ and tools/make_goldens.py.

Everything here is deterministic (python ``random.Random`` with fixed seeds)
so fixtures can be regenerated and large cases can be pinned by sha256
instead of being committed.
"""
import random

HG38 = [  # (name, length) in BEDOPS sort-bed (lexicographic) order
    ("chr1", 248956422), ("chr10", 133797422), ("chr11", 135086622), ("chr12", 133275309),
    ("chr13", 114364328), ("chr14", 107043718), ("chr15", 101991189), ("chr16", 90338345),
    ("chr17", 83257441), ("chr18", 80373285), ("chr19", 58617616), ("chr2", 242193529),
    ("chr20", 64444167), ("chr21", 46709983), ("chr22", 50818468), ("chr3", 198295559),
    ("chr4", 190214555), ("chr5", 181538259), ("chr6", 170805979), ("chr7", 159345973),
    ("chr8", 145138636), ("chr9", 138394717), ("chrX", 156040895), ("chrY", 57227415),
]


def edge_cases():
    """SURVEY Appendix A edge table (+ a few more), as (name, bytes)."""
    T = "\t"
    c = [
        ("basic_mixed", "chr1\t10\t20\nchr1\t25\t35\nchr1\t40\t60\tid1\t0\t+\nchr2\t5\t10\n"),
        ("overlap", "chr1\t10\t100\nchr1\t20\t30\n"),
        ("stop_lt_start", "chr1\t50\t40\nchr1\t60\t70\n"),
        ("two_fields", "chr1\t10\nchr1\t20\t30\n"),
        ("zero_len_at_0", "chr1\t0\t0\nchr1\t5\t9\n"),
        ("zero_zero_then", "chr1\t0\t0\nchr1\t0\t0\nchr1\t3\t5\n"),
        ("start0", "chr1\t0\t10\nchr1\t10\t20\n"),
        ("dups3", "chr1\t10\t20\nchr1\t10\t20\nchr1\t10\t20\n"),
        ("crlf_bed3", "chr1\t10\t20\r\nchr1\t30\t40\r\n"),
        ("crlf_bed6", "chr1\t10\t20\ta\t0\t+\r\nchr1\t30\t45\tb\t0\t-\r\n"),
        ("trailing_tab", "chr1\t10\t20\t\n"),
        ("rem_with_tabs", "chr1\t10\t20\ta\t\tb\t\n"),
        ("double_tab", "chr1\t\t10\t20\n"),
        ("unsorted_chr", "chr1\t10\t20\nchr2\t10\t20\nchr1\t30\t40\n"),
        ("track_header", "track name=x\nchr1\t10\t20\n"),
        ("big_coords", "chr1\t9000000000\t9000000010\n"),
        ("no_trailing_nl", "chr1\t10\t20\nchr1\t30\t40"),
        ("leading_ws_sign", "chr1\t  +7\t -3\nchr1\t+10\t0012\n"),
        ("garbage_numbers", "chr1\tabc\t20\nchr1\t10\txyz\nchr1\t-\t5\n"),
        ("empty_line", "chr1\t10\t20\n\nchr1\t30\t40\n"),
        ("only_chr", "chr1\nchr1\n"),
        ("neg_deltas", "chr1\t100\t200\nchr1\t50\t60\nchr1\t55\t400\n"),
        ("stop_zero_abs", "chr1\t5\t0\nchr1\t7\t9\nchr1\t9\t9\n"),
        ("triple_tab", "a\t\t\tb\t1\n"),
        ("tab_then_nl", "chr1\t\nchr1\t5\t6\n"),
        ("rem_long", "chr1\t1\t2\t" + "x" * 300 + "\n"),
        ("nul_in_rem", "chr1\t1\t2\tab\x00cd\n"),
        ("nul_in_chr", "chr\x001\t1\t2\nchr\x002\t3\t4\n"),
        ("ff_truncates", "chr1\t1\t2\nchr1\t3\t4\xffchr1\t5\t6\n"),
        ("huge_number", "chr1\t99999999999999999999\t5\nchr1\t1\t-99999999999999999999\n"),
        ("int64_edges", "chr1\t-9223372036854775807\t9223372036854775807\n"),
        ("spaces_fields", "chr 1\t1\t2\nchr 1\t3\t4\n"),
        ("many_segments", "".join("c%d\t%d\t%d\n" % (i % 3, i, i + 1) for i in range(30))),
    ]
    return [(n, s.encode("latin-1")) for n, s in c]


def cfg1_bed(n=10000, seed=1):
    """cfg1: single-chrom sorted BED3: pos += U{0..200}, len U{1..500}."""
    r = random.Random(seed)
    pos, out = 0, []
    for _ in range(n):
        pos += r.randint(0, 200)
        out.append("chr1\t%d\t%d\n" % (pos, pos + r.randint(1, 500)))
    return "".join(out).encode()


def multi_chrom_bed(nchr, nlines, seed, kind="bed3"):
    r = random.Random(seed)
    out = []
    for ci in range(nchr):
        name, L = HG38[ci % len(HG38)]
        starts = sorted(r.randrange(0, 1000000) for _ in range(nlines))
        for i, s in enumerate(starts):
            ln = r.randint(1, 1500)
            if kind == "bed3":
                out.append("%s\t%d\t%d\n" % (name, s, s + ln))
            elif kind == "bed6":
                out.append("%s\t%d\t%d\tid%d\t%d\t%s\n" % (name, s, s + ln, i, r.randint(0, 1000), r.choice("+-.")))
            else:  # narrowPeak BED6+4
                out.append("%s\t%d\t%d\tpeak%d\t%d\t.\t%.5f\t%.5f\t%.5f\t%d\n" % (
                    name, s, s + ln, i, r.randint(0, 1000), r.uniform(0, 100), r.uniform(0, 50),
                    r.uniform(0, 20), r.randrange(0, ln)))
    return "".join(out).encode()


def fuzz_bed(seed, nlines=60):
    """Adversarial-but-safe lines (no 0xFF/NUL, lines < 300 B) for parse quirks."""
    r = random.Random(seed)
    chrs = ["chr1", "chr2", "chrX", "", " chr1", "chr1 "]
    nums = ["0", "1", "10", "-5", "+7", " 12", "007", "", "x", "-", "3.5", "1e3", "\t9",
            "9223372036854775807", "-9223372036854775808", "123456789012", "\r", "42\r"]
    rems = ["", "a", "id\t0\t+", "\t", "a b", "x\ty\tz", "+\r", "9\t9"]
    out = []
    for _ in range(nlines):
        k = r.random()
        ch = r.choice(chrs) if r.random() < 0.3 else "chr1"
        if k < 0.1:
            line = ch
        elif k < 0.2:
            line = ch + "\t" + r.choice(nums)
        elif k < 0.7:
            line = "%s\t%s\t%s" % (ch, r.choice(nums), r.choice(nums))
        else:
            line = "%s\t%s\t%s\t%s" % (ch, r.choice(nums), r.choice(nums), r.choice(rems))
        if r.random() < 0.05:
            line = line.replace("\t", "\t\t", 1)
        out.append(line + "\n")
    return "".join(out).encode("latin-1")


def parseable_fuzz_bed(seed, nlines=3000):
    """Lines whose start and stop always parse (no stale values), in mixed
    shapes: plain digits, signs and blanks, CRLF, 19-20 digit values, NUL bytes
    in the chromosome or remainder, tab quirks, and runs of long lines so that
    whole 256-line groups exceed the transform's LDS staging sizes."""
    r = random.Random(seed)
    chrs = ["chr1", "chr2", "chr10", "chrX", "c\x00hr", "chr1 "]
    out, ci, pos = [], 0, 0
    long_phase = 0
    for i in range(nlines):
        if i % 256 == 0 and r.random() < 0.3:
            long_phase = r.choice([0, 90, 130, 400])
        if r.random() < 0.01 or (i % 256 == 0 and r.random() < 0.2):
            ci = r.randrange(len(chrs))
            pos = 0
        pos += r.randint(0, 300)
        a, b = str(pos), str(pos + r.randint(0, 900))
        k = r.random()
        if k < 0.03:
            a = r.choice([" ", "+", "  +", "0"]) + a
        elif k < 0.05:
            b = r.choice(["99999999999999999999", "9223372036854775807", "1234567890123456789",
                          "123456789012345678"])
        elif k < 0.06:
            a = "-" + a
        line = "%s\t%s\t%s" % (chrs[ci], a, b)
        k = r.random()
        if long_phase:
            line += "\t" + "".join(r.choice("ACGT.") for _ in range(r.randint(long_phase // 2, long_phase)))
        elif k < 0.2:
            line += "\t" + r.choice(["id%d\t0\t+" % i, "a\x00b", "", "\t", "x\ty"])
        if r.random() < 0.03:
            line += "\r"
        if r.random() < 0.02:
            line = line.replace("\t", "\t\t", 1) if r.random() < 0.5 else line + "\t\t"
        out.append(line + "\n")
    return "".join(out).encode("latin-1")


TRANSFORM_GENERATORS = {
    "cfg1_t10k": lambda: cfg1_bed(10000),
    "multi24_bed3": lambda: multi_chrom_bed(24, 400, seed=7, kind="bed3"),
    "multi24_bed6": lambda: multi_chrom_bed(24, 300, seed=8, kind="bed6"),
    "multi8_narrowpeak": lambda: multi_chrom_bed(8, 500, seed=9, kind="narrowpeak"),
}


# ---------------------------------------------------------------------------
# bzip2 corpora
# ---------------------------------------------------------------------------
def _periodic(r, p, k):
    unit = bytes(r.randrange(0, 8) + 97 for _ in range(p))
    return unit * k


def bz2_small_cases():
    r = random.Random(42)
    cases = [
        ("empty", b"", 9), ("one", b"a", 9), ("aaa", b"aaa", 9), ("aaaa", b"aaaa", 9),
        ("aaaaa", b"aaaaa", 9), ("run255", b"z" * 255, 9), ("run256", b"z" * 256, 9),
        ("run1000", b"q" * 1000, 9), ("run4_mix", b"aaaabbbbbcccccccc" * 3, 9),
        ("allbytes", bytes(range(256)), 9), ("allbytes_rev", bytes(range(255, -1, -1)) * 3, 9),
        ("rand100", bytes(r.randrange(256) for _ in range(100)), 9),
        ("rand3000", bytes(r.randrange(256) for _ in range(3000)), 9),
        ("text", b"the quick brown fox jumps over the lazy dog\n" * 20, 9),
        ("ab", b"ab", 9), ("aab", b"aab", 9), ("abab", b"abab", 9), ("p2_even", b"0\n" * 500, 9),
        ("p2_odd", b"0\n" * 500 + b"0", 9), ("n0_even", b"\n0" * 300, 9),
        ("runs_of_count_bytes", b"\x04\x04\x04\x04\x04\x00" * 50, 9),
        ("bs1_text", b"12\n-3\np45\n" * 200, 1),
    ]
    for i in range(25):   # periodic blocks: origPtr follows fallbackSort tie order
        p = r.randint(1, 40)
        k = r.randint(2, 60)
        cases.append(("periodic_%d_p%d_k%d" % (i, p, k), _periodic(r, p, k), 9))
    for i in range(10):   # small alphabet, near-periodic
        n = r.randint(20, 3000)
        cases.append(("smallalpha_%d" % i, bytes(r.choice(b"01\n") for _ in range(n)), 9))
    for i in range(8):    # runs of random length incl. > 255
        out = bytearray()
        while len(out) < 4000:
            out += bytes([r.randrange(4) + 48]) * r.choice([1, 2, 3, 4, 5, 6, 250, 255, 256, 259, 600])
        cases.append(("runs_%d" % i, bytes(out), 9))
    return cases


def _runs_bytes(seed, total):
    r = random.Random(seed)
    out = bytearray()
    while len(out) < total:
        out += bytes([r.randrange(5) + 48]) * r.choice([1, 1, 2, 3, 4, 7, 100, 255, 256, 511, 600])
    return bytes(out[:total])


def _textish(seed, total):
    r = random.Random(seed)
    out = []
    n = 0
    while n < total:
        s = ("p%d\n" % r.randint(20, 999)) if r.random() < 0.7 else ""
        s += "%d\n" % r.randint(-990, 60)
        out.append(s)
        n += len(s)
    return "".join(out).encode()[:total]


def _perpos(chrom_len, start=0):
    # per-position transform text: first line "p1\n<start>\n", then "0\n" 
    return b"p1\n" + str(start).encode() + b"\n" + b"0\n" * (chrom_len - 1)


def bz2_large_cases():
    """(name, generator, blockSize100k) -- pinned by sha256 in bz2_cases.json."""
    r = random.Random(5)
    big_periodic = _periodic(r, 997, 30)
    return [
        ("multiblock_text_bs1", lambda: _textish(11, 350000), 1),
        ("runs_cross_cut_bs1", lambda: _runs_bytes(12, 320000), 1),
        ("periodic_p2_even_bs9", lambda: b"0\n" * 300000, 9),
        ("periodic_p997_k30_bs9", lambda: big_periodic, 9),
        ("perpos_bs1", lambda: _perpos(260000, 1234), 1),
        ("perpos_bs9", lambda: _perpos(470000, 5), 9),
        ("cfg1_transform_text", lambda: _textish(13, 92000), 9),
        ("textish_bs9_2blocks", lambda: _textish(14, 1300000), 9),
        ("exact_max_bs1", lambda: _textish(15, 99981), 1),
        ("max_plus_one_bs1", lambda: _textish(16, 99982), 1),
    ]


LARGE_GENERATORS = {name: (gen, bs) for name, gen, bs in bz2_large_cases()}
