// CPU check of mcs_orb_core.h's FAST helpers (built and run by tests/test_orb_core_cpu.py):
// orb_fast_score against the direct 16 x 9 arc scan of its specification, and orb_fast_test(t)
// against score > t, on random and adversarial (few-level, arc-shaped) circles.
#include <cmath>
#include <cstdio>
#include <initializer_list>
#include <cstdlib>
#include "mcs_orb_core.h"

static int direct_score(const uint8_t *p, int step)
{
    int d[16];
    const int c = p[0];
    for (int i = 0; i < 16; i++)
        d[i] = (int)p[mcs::kFastCircle[i][1] * step + mcs::kFastCircle[i][0]] - c;
    int best = -255;
    for (int s = 0; s < 16; s++) {
        int lo = 255, hi = 255;
        for (int k = 0; k < 9; k++) {
            const int v = d[(s + k) & 15];
            lo = v < lo ? v : lo;
            hi = -v < hi ? -v : hi;
        }
        best = (lo > hi ? lo : hi) > best ? (lo > hi ? lo : hi) : best;
    }
    return best;
}

int main(int argc, char **argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 2000000;
    uint8_t img[7 * 7];
    uint32_t r = 12345u;
    auto rnd = [&] { r = r * 1664525u + 1013904223u; return r >> 8; };
    long bad = 0, corners = 0;
    for (int it = 0; it < n; it++) {
        const int mode = it % 4;
        const int c = rnd() & 255;
        for (int i = 0; i < 49; i++) {
            int v;
            if (mode == 0) v = rnd() & 255;                      // uniform
            else if (mode == 1) v = c + (int)(rnd() % 81) - 40;  // near the centre
            else v = (rnd() & 1) ? c + 30 : c - 30;              // two levels
            img[i] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
        }
        img[24] = (uint8_t)c;
        if (mode == 3) {                                          // an arc of random length
            const int s0 = rnd() & 15, len = 7 + (rnd() % 4), up = rnd() & 1;
            for (int k = 0; k < len; k++) {
                const int q = (s0 + k) & 15;
                const int v = up ? c + 21 + (int)(rnd() % 5) : c - 21 - (int)(rnd() % 5);
                img[(3 + mcs::kFastCircle[q][1]) * 7 + 3 + mcs::kFastCircle[q][0]] =
                    (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
            }
        }
        const uint8_t *p = img + 3 * 7 + 3;
        const int s = mcs::orb_fast_score(p, 7), ref = direct_score(p, 7);
        if (s != ref) bad++;
        for (int t : {0, 1, 10, 20, 21, 22, 40, 254}) {
            const bool a = mcs::orb_fast_test(p, 7, t);
            if (a != (ref > t)) bad++;
            corners += a;
        }
    }
    printf("%d %ld %ld\n", n, corners, bad);
    return bad ? 1 : 0;
}
