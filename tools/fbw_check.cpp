// Host model check of the wave-parallel fallbackQSort3 partition
// (fbw_partition in starch_amd/csrc/bz2_bwt.hip) against the serial step
// (fbp_partition, bz:blocksort.c:93-180): the same passes written as plain
// loops over 64-lane rows, on random ranges with few distinct keys.
//   g++ -O2 -std=c++17 -o /tmp/fbw_check tools/fbw_check.cpp && /tmp/fbw_check
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <random>
#include <vector>

static void swp(uint32_t* key, uint32_t* fm, int a, int b)
{
    std::swap(key[a], key[b]);
    std::swap(fm[a], fm[b]);
}

static bool serial(uint32_t* key, uint32_t* fm, int lo, int hi, uint32_t med, int& alo, int& ahi, int& blo, int& bhi)
{
    int unLo = lo, ltLo = lo, unHi = hi, gtHi = hi;
    for (;;) {
        while (unLo <= unHi) {
            const uint32_t k = key[unLo];
            if (k == med) { swp(key, fm, unLo, ltLo); ++ltLo; ++unLo; continue; }
            if (k > med) break;
            ++unLo;
        }
        while (unLo <= unHi) {
            const uint32_t k = key[unHi];
            if (k == med) { swp(key, fm, unHi, gtHi); --gtHi; --unHi; continue; }
            if (k < med) break;
            --unHi;
        }
        if (unLo > unHi) break;
        swp(key, fm, unLo, unHi);
        ++unLo;
        --unHi;
    }
    if (gtHi < ltLo) return false;
    int n = std::min(ltLo - lo, unLo - ltLo);
    for (int a = lo, b = unLo - n; n > 0; --n, ++a, ++b) swp(key, fm, a, b);
    int m = std::min(hi - gtHi, gtHi - unHi);
    for (int a = unLo, b = hi - m + 1; m > 0; --m, ++a, ++b) swp(key, fm, a, b);
    const int nn = lo + unLo - ltLo - 1, mm = hi - (gtHi - unHi) + 1;
    if (nn - lo > hi - mm) { alo = lo; ahi = nn; blo = mm; bhi = hi; }
    else { alo = mm; ahi = hi; blo = lo; bhi = nn; }
    return true;
}

static const uint32_t RES = 0x80000000u;

static bool wave(uint32_t* key, uint32_t* fm, int lo, int hi, uint32_t med, int& alo, int& ahi, int& blo, int& bhi)
{
    const uint32_t m = (uint32_t)(hi - lo + 1);
    uint32_t* kk = key + lo;
    uint32_t* ff = fm + lo;
    std::vector<uint32_t> A(m), B(m);
    uint32_t nL = 0, nG = 0;
    for (uint32_t j = 0; j < m; ++j) { nL += kk[j] < med; nG += kk[j] > med; }
    const uint32_t nE = m - nL - nG;
    if (nL + nG == 0) return false;
    uint32_t rL = 0, rG = 0, p = m, lbp = nL, gbp = nG;
    for (uint32_t j = 0; j < m; ++j) {
        const bool isL = kk[j] < med, isG = kk[j] > med;
        if (isL) A[rL] = j;
        if (isG) A[nL + rG] = j;
        if (p == m && (isL || isG) && rL + rG >= nL) { p = j; lbp = rL; gbp = rG; }
        rL += isL;
        rG += isG;
    }
    const uint32_t nEL = p - lbp - gbp, nER = nE - nEL;
    rL = rG = 0;
    uint32_t rE = 0;
    for (uint32_t j = 0; j < m; ++j) {
        const uint32_t k = kk[j];
        const bool isL = k < med, isG = k > med, isE = k == med;
        uint32_t v;
        if (j < p) {
            if (isE) v = rE == j ? RES : rE;
            else if (isL) v = RES | j;
            else v = RES | A[nL - 1 - rG];
        } else {
            const uint32_t ea = nE - rE - 1;
            if (isE) v = ea == m - 1 - j ? RES : m - 1 - ea;
            else if (isG) v = RES | j;
            else v = RES | A[2 * nL - rL - 1];
        }
        B[j] = v;
        rL += isL;
        rG += isG;
        rE += isE;
    }
    for (int pass = 0;; ++pass) {
        bool un = false;
        for (uint32_t j = 0; j < m; ++j) {
            const uint32_t v = B[j];
            if (!(v & RES)) {
                if (j < p ? v >= j : (v <= j || v < p)) { printf("bad pointer %u -> %u\n", j, v); return false; }
                const uint32_t w = B[v];
                B[j] = w;
                un |= !(w & RES);
            }
        }
        if (!un) break;
    }
    const uint32_t n1 = std::min(nEL, p - nEL);
    const uint32_t ul = m - p, m1 = std::min(nER, ul - nER);
    auto phi = [&](uint32_t q) -> uint32_t {
        if (q < n1) return q + (p - n1);
        if (q < p && q >= p - n1) return q - (p - n1);
        if (q >= p && q < p + m1) return q + (m - m1 - p);
        if (q >= m - m1) return q - (m - m1 - p);
        return q;
    };
    std::vector<uint32_t> seen(m, 0);
    rE = 0;
    for (uint32_t j = 0; j < m; ++j) {
        const bool isE = kk[j] == med;
        auto put = [&](uint32_t t, uint32_t src) { A[t] = src; ++seen[t]; };
        if (j < p) {
            if (isE) put(phi(rE), j);
            if (j >= nEL) put(phi(j), B[j] & ~RES);
        } else {
            if (isE) put(phi(m - 1 - (nE - rE - 1)), j);
            if (m - 1 - j >= nER) put(phi(j), B[j] & ~RES);
        }
        rE += isE;
    }
    for (uint32_t j = 0; j < m; ++j)
        if (seen[j] != 1) { printf("target %u written %u times\n", j, seen[j]); return false; }
    for (uint32_t j = 0; j < m; ++j) B[j] = kk[A[j]];
    for (uint32_t j = 0; j < m; ++j) kk[j] = B[j];
    for (uint32_t j = 0; j < m; ++j) B[j] = ff[A[j]];
    for (uint32_t j = 0; j < m; ++j) ff[j] = B[j];
    const int nn = lo + (int)nL - 1, mm = hi - (int)nG + 1;
    if (nn - lo > hi - mm) { alo = lo; ahi = nn; blo = mm; bhi = hi; }
    else { alo = mm; ahi = hi; blo = lo; bhi = nn; }
    return true;
}

int main()
{
    std::mt19937 rng(7);
    int bad = 0;
    for (int t = 0; t < 200000 && bad < 5; ++t) {
        const int m = 1 + (int)(rng() % (t < 1000 ? 4000 : 300));
        const int nk = 1 + (int)(rng() % 5);
        const int pad = (int)(rng() % 7);
        std::vector<uint32_t> k1(m + 2 * pad), f1(m + 2 * pad);
        for (size_t i = 0; i < k1.size(); ++i) { k1[i] = 10 + rng() % nk; f1[i] = (uint32_t)i; }
        std::vector<uint32_t> k2 = k1, f2 = f1;
        const int lo = pad, hi = pad + m - 1;
        const uint32_t med = k1[lo + (int)(rng() % m)];
        int a1 = 0, b1 = 0, c1 = 0, d1 = 0, a2 = 0, b2 = 0, c2 = 0, d2 = 0;
        const bool r1 = serial(k1.data(), f1.data(), lo, hi, med, a1, b1, c1, d1);
        const bool r2 = wave(k2.data(), f2.data(), lo, hi, med, a2, b2, c2, d2);
        if (r1 != r2 || k1 != k2 || f1 != f2 || (r1 && (a1 != a2 || b1 != b2 || c1 != c2 || d1 != d2))) {
            printf("mismatch t=%d m=%d nk=%d r=%d/%d\n", t, m, nk, r1, r2);
            ++bad;
        }
    }
    printf(bad ? "FAILED\n" : "ok\n");
    return bad ? 1 : 0;
}
