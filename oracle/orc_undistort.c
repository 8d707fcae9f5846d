/*
 * orc_undistort.c -- TEST INFRASTRUCTURE ONLY (the parity checker), never the product path.
 *
 * cv::undistort(src, dst, cameraMatrix, distCoeffs) of OpenCV 3.4 (imgproc/src/undistort.cpp),
 * restated (the reference calls it per frame at
 * video_mapping_node.py:157-158 and MediaPlayer/view.py:380-381).  OpenCV is third-party and
 * absent here (version unpinned, the reference needs 2.4 or 3.x): this follows 3.4's source
 * semantics, which agree with 2.4's for the k1..k3, p1, p2 model.
 *
 *   undistort:  stripe_size0 = min(max(1, 4096 / cols), rows); map1 CV_16SC2, map2 CV_16UC1;
 *               newCameraMatrix = A; for each stripe starting at row y: Ar = A with
 *               Ar(1,2) = A(1,2) - y; initUndistortRectifyMap(A, dist, I, Ar, (cols, stripe))
 *               then remap(src, dst rows [y, y+stripe), INTER_LINEAR, BORDER_CONSTANT 0);
 *   init...Map: iR = (Ar * I).inv(DECOMP_LU) (3x3 closed form, orc_invert3x3); per map row i:
 *               _x = i*ir1 + ir2, _y = i*ir4 + ir5, _w = i*ir7 + ir8, then per column j (adding
 *               ir0, ir3, ir6 after each column): w = 1/_w, x = _x w, y = _y w,
 *               kr = (1 + ((k3 r2 + k2) r2 + k1) r2) / (1 + ((k6 r2 + k5) r2 + k4) r2),
 *               xd = x kr + p1 2xy + p2 (r2 + 2 x^2) + s1 r2 + s2 r2 r2, yd likewise,
 *               (tilt identity) u = fx xd + u0, v = fy yd + v0,
 *               iu = cvRound(u * 32), iv = cvRound(v * 32), map1 = ((short)(iu >> 5),
 *               (short)(iv >> 5)), map2 = (iv & 31) * 32 + (iu & 31).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int orc_invert3x3(const double *m, double *out);
void orc__remap_bilinear_px(const uint8_t *src, int sw, int sh, long sstep, int cn, int sx, int sy,
                            int alpha, uint8_t *d);

int orc_undistort(const uint8_t *src, int w, int h, int cn, const double *A, const double *dist,
                  int n_dist, uint8_t *dst)
{
    double k[14];
    memset(k, 0, sizeof(k));
    if (!(n_dist == 0 || n_dist == 4 || n_dist == 5 || n_dist == 8 || n_dist == 12 ||
          n_dist == 14))
        return -1;
    for (int i = 0; i < n_dist; i++) k[i] = dist[i];
    if (k[12] != 0.0 || k[13] != 0.0) return -1;
    const long step = (long)w * cn;
    int stripe0 = 4096 / (w > 1 ? w : 1);
    if (stripe0 < 1) stripe0 = 1;
    if (stripe0 > h) stripe0 = h;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < h; y += stripe0) {
        const int n = h - y < stripe0 ? h - y : stripe0;
        double Ar[9], ir[9];
        memcpy(Ar, A, sizeof(Ar));
        Ar[5] = A[5] - y;
        orc_invert3x3(Ar, ir);
        for (int i = 0; i < n; i++) {
            double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
            uint8_t *D = dst + (long)(y + i) * step;
            for (int j = 0; j < w; j++) {
                const double ww = 1. / _w, x = _x * ww, yy = _y * ww;
                const double x2 = x * x, y2 = yy * yy, r2 = x2 + y2, xy2 = 2 * x * yy;
                const double kr = (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2) /
                                  (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2);
                const double xd = x * kr + k[2] * xy2 + k[3] * (r2 + 2 * x2) + k[8] * r2 +
                                  k[9] * r2 * r2;
                const double yd = yy * kr + k[2] * (r2 + 2 * y2) + k[3] * xy2 + k[10] * r2 +
                                  k[11] * r2 * r2;
                const double u = A[0] * xd + A[2], v = A[4] * yd + A[5];
                const int iu = (int)lrint(u * 32), iv = (int)lrint(v * 32);
                orc__remap_bilinear_px(src, w, h, step, cn, (short)(iu >> 5), (short)(iv >> 5),
                                       (iv & 31) * 32 + (iu & 31), D + (long)j * cn);
                _x += ir[0];
                _y += ir[3];
                _w += ir[6];
            }
        }
    }
    return 0;
}
