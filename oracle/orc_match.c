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
