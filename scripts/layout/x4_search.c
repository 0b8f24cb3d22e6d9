// Search br512x4 spectrum slot tables sidx(q) = SF[4 q0 + q2] + SG1[q1] + SG3[q3] that are bank-conflict
// free for every access pattern (scripts/layout/x4_banks.py states the model) including the pass-B
// transpose read (lane (u, r) reads q = 16 u + c + 4 r), with all 256 slots distinct and a small range.
// cc -O2 x4_search.c -o x4_search && ./x4_search [seed]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int RDG[4][16], WRG[8][8];
static unsigned rs = 1;
static int rnd(int n) { rs = rs * 1103515245u + 12345u; return (int)((rs >> 8) % (unsigned)n); }
static int SF[16], G1[4], G3[4];
static int sidx(int q) { return SF[4 * (q & 3) + ((q >> 4) & 3)] + G1[(q >> 2) & 3] + G3[q >> 6]; }
// pattern p, fixed index f, lane l -> q
static int pat_q(int p, int f, int l) {
    int u = l & 15, r = l >> 4;
    switch (p) {
    case 0: return u + 16 * (r + 4 * f);      // pass A / A^-1 / MAC (same residues)
    case 1: return 16 * u + r + 4 * f;        // pass B / B^-1
    case 2: return 16 * u + f + 4 * r;        // pass B transpose read
    default: return 64 * f + l;               // MAC position
    }
}
static int cost(int with_t) {
    int c = 0;
    for (int p = 0; p < 4; p++) {
        if (p == 2 && !with_t) continue;
        for (int f = 0; f < 4; f++) {
            // reads (all patterns are read somewhere)
            for (int g = 0; g < 4; g++) {
                int cnt[16] = {0}, mx = 0;
                for (int k = 0; k < 16; k++) {
                    int b = ((sidx(pat_q(p, f, RDG[g][k])) % 16) + 16) % 16;
                    if (++cnt[b] > mx) mx = cnt[b];
                }
                c += mx - 1;
            }
            if (p == 2) continue;  // the transpose pattern is only read
            for (int g = 0; g < 8; g++) {
                int cnt[8] = {0}, mx = 0;
                for (int k = 0; k < 8; k++) {
                    int b = ((sidx(pat_q(p, f, WRG[g][k])) % 8) + 8) % 8;
                    if (++cnt[b] > mx) mx = cnt[b];
                }
                c += mx - 1;
            }
        }
    }
    return c;
}
int main(int argc, char **argv) {
    rs = argc > 1 ? (unsigned)atoi(argv[1]) : 1u;
    int with_t = argc > 2 ? atoi(argv[2]) : 1;
    int gA[16] = {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27};
    int gB[16] = {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31};
    for (int k = 0; k < 16; k++) { RDG[0][k] = gA[k]; RDG[1][k] = gB[k]; RDG[2][k] = gA[k] + 32; RDG[3][k] = gB[k] + 32; }
    for (int g = 0; g < 8; g++) for (int k = 0; k < 8; k++) WRG[g][k] = 8 * g + k;
    int best_range = 1 << 30;
    for (int restart = 0; restart < 4000; restart++) {
        for (int i = 0; i < 16; i++) SF[i] = rnd(16);
        for (int i = 0; i < 4; i++) { G1[i] = rnd(16); G3[i] = rnd(16); }
        int c = cost(with_t);
        for (int it = 0; it < 2000 && c; it++) {
            int k = rnd(24), *a = k < 16 ? &SF[k] : (k < 20 ? &G1[k - 16] : &G3[k - 20]);
            int old = *a;
            *a = rnd(16);
            int c2 = cost(with_t);
            if (c2 <= c) c = c2; else *a = old;
        }
        if (restart < 5 || (restart % 500) == 0) { fprintf(stderr, "restart %d cost %d\n", restart, c); }
        if (c) continue;
        // lift residues: add multiples of 16, keep slots distinct, minimise the range
        int rf[16], r1[4], r3[4];
        memcpy(rf, SF, sizeof rf); memcpy(r1, G1, sizeof r1); memcpy(r3, G3, sizeof r3);
        for (int t = 0; t < 200000; t++) {
            for (int i = 0; i < 16; i++) SF[i] = rf[i] + 16 * rnd(6);
            for (int i = 0; i < 4; i++) { G1[i] = r1[i] + 16 * rnd(6); G3[i] = r3[i] + 16 * rnd(18); }
            static unsigned char seen[2048];
            memset(seen, 0, sizeof seen);
            int lo = 1 << 30, hi = -(1 << 30), ok = 1;
            for (int q = 0; q < 256 && ok; q++) {
                int s = sidx(q);
                if (seen[s]) ok = 0;
                seen[s] = 1;
                if (s < lo) lo = s;
                if (s > hi) hi = s;
            }
            if (!ok) continue;
            if (hi - lo + 1 < best_range) {
                best_range = hi - lo + 1;
                printf("range %d: SF", best_range);
                for (int i = 0; i < 16; i++) printf(" %d", SF[i] - lo);
                printf(" | SG1");
                for (int i = 0; i < 4; i++) printf(" %d", G1[i]);
                printf(" | SG3");
                for (int i = 0; i < 4; i++) printf(" %d", G3[i]);
                printf("  (cost %d)\n", cost(with_t));
                fflush(stdout);
            }
        }
        memcpy(SF, rf, sizeof rf);
    }
    return 0;
}
