/*
 * orc_match.c -- TEST INFRASTRUCTURE ONLY (the parity checker), never the product path.
 *
 * CPU restatement of brute-force k=2 matching of 256-bit binary descriptors under the Hamming
 * distance: cv2.BFMatcher(cv2.NORM_HAMMING).knnMatch(query, train, k=2), the binary-descriptor
 * form of the reference's matcher (PostScripts/Stitcher/StitcherClass.py:405-448, which uses
 * the float-L2 BFMatcher on SIFT).  OpenCV is third-party (not vendored, version unpinned);
 * restated from OpenCV 3.4 modules/core/src/batch_distance.cpp (batchDistance with K > 0):
 * train descriptors are visited in index order and one enters the sorted top-K list only when
 * its distance is strictly smaller than the current K-th, shifting entries whose distance is
 * strictly larger -- so among equal distances the lower train index ranks first.
 * Parity against a real cv2 is unpinned (none in this image).
 */
#include <math.h>
#include <stdint.h>

static inline int popcount32(uint32_t v) { return __builtin_popcount(v); }

void orc_hamming_knn2(const uint8_t *query, int nq, const uint8_t *train, int nt, int32_t *idx2,
                      int32_t *dist2)
{
#pragma omp parallel for schedule(static)
    for (int q = 0; q < nq; q++) {
        const uint32_t *a = (const uint32_t *)(query + (long)q * 32);
        int best_d[2] = {0x7fffffff, 0x7fffffff}, best_i[2] = {-1, -1};
        for (int j = 0; j < nt; j++) {
            const uint32_t *b = (const uint32_t *)(train + (long)j * 32);
            int d = 0;
            for (int w = 0; w < 8; w++) d += popcount32(a[w] ^ b[w]);
            if (d < best_d[1]) {
                int k = 1;
                for (; k > 0 && best_d[k - 1] > d; k--) {
                    best_d[k] = best_d[k - 1];
                    best_i[k] = best_i[k - 1];
                }
                best_d[k] = d;
                best_i[k] = j;
            }
        }
        for (int k = 0; k < 2; k++) {
            idx2[2 * q + k] = best_i[k];
            dist2[2 * q + k] = best_i[k] < 0 ? -1 : best_d[k];
        }
    }
}

/* BFMatcher(NORM_L2).knnMatch(query, train, k=2) for float descriptors (StitcherClass.py:423-424,
 * SURVEY.md 8f-3).  OpenCV computes sqrt(sum (a - b)^2) in float; for descriptors that are
 * integers in [0, 255] (SIFT's output) every partial sum is an integer below 2^24, so its result
 * is exactly float(sqrt(d2)) of the integer d2 whatever its summation order -- restated here
 * with int64 sums.  Other data: sum in double, distance float(sqrt) (a reference for tolerance
 * checks, not OpenCV's rounding).  Order: distance, then train index (batchDistance insertion).
 * Returns 1 when the exact integer form applied. */
int orc_l2_knn2(const float *query, int nq, const float *train, int nt, int dim, int32_t *idx2,
                float *dist2)
{
    int exact = 1;
    for (long i = 0; i < (long)(nq + 0) * dim && exact; i++) {
        const float v = query[i];
        exact = v >= 0.f && v <= 255.f && v == (float)(int)v;
    }
    for (long i = 0; i < (long)nt * dim && exact; i++) {
        const float v = train[i];
        exact = v >= 0.f && v <= 255.f && v == (float)(int)v;
    }
#pragma omp parallel for schedule(static)
    for (int q = 0; q < nq; q++) {
        float bd[2] = {0, 0};
        int bi[2] = {-1, -1};
        for (int t = 0; t < nt; t++) {
            double d2;
            if (exact) {
                int64_t s = 0;
                for (int k = 0; k < dim; k++) {
                    const int64_t d = (int64_t)query[(long)q * dim + k] -
                                      (int64_t)train[(long)t * dim + k];
                    s += d * d;
                }
                d2 = (double)s;
            } else {
                d2 = 0.0;
                for (int k = 0; k < dim; k++) {
                    const double d = (double)query[(long)q * dim + k] -
                                     (double)train[(long)t * dim + k];
                    d2 += d * d;
                }
            }
            const float f = (float)sqrt(d2);
            if (bi[0] < 0 || f < bd[0]) {
                bd[1] = bd[0], bi[1] = bi[0];
                bd[0] = f, bi[0] = t;
            } else if (bi[1] < 0 || f < bd[1]) {
                bd[1] = f, bi[1] = t;
            }
        }
        for (int m = 0; m < 2; m++) {
            idx2[2 * q + m] = bi[m];
            dist2[2 * q + m] = bi[m] < 0 ? -1.f : bd[m];
        }
    }
    return exact;
}
