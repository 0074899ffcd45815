/* A C consumer of the drop-in boundary (include/stereovision_amd.h): no Python, no PyTorch.
 *
 * Builds a synthetic rectified pair in host memory (random texture, the right image shifted
 * left by a known disparity), runs the app-1 drop-in (`sv_depth_map`, the replacement of
 * depth_map.py:837-946's disparity + median + depth post) and checks the disparity map
 * recovers the shift in the interior.  Then times repeated calls.
 *
 *   gcc -std=c99 -O2 -Iinclude examples/depth_map_c.c -Lstereovision_amd/lib -lsvhip \
 *       -Wl,-rpath,'$ORIGIN/../stereovision_amd/lib' -o examples/depth_map_c
 *   ./examples/depth_map_c [H W num_disp win calls]
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "stereovision_amd.h"

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

int main(int argc, char** argv) {
    const int H = argc > 1 ? atoi(argv[1]) : 1080;
    const int W = argc > 2 ? atoi(argv[2]) : 1920;
    const int D = argc > 3 ? atoi(argv[3]) : 128;
    const int win = argc > 4 ? atoi(argv[4]) : 9;
    const int calls = argc > 5 ? atoi(argv[5]) : 50;
    const int shift = D / 3;
    if (H < 16 || W <= D + 2 * win || D < 4 || (win & 1) == 0 || calls < 1) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    int ndev = 0;
    if (sv_device_count(&ndev) != 0 || ndev < 1) {
        fprintf(stderr, "no HIP device: %s\n", sv_last_error());
        return 3;
    }
    sv_ctx* ctx = NULL;
    if (sv_create(0, &ctx) != 0) {
        fprintf(stderr, "sv_create: %s\n", sv_last_error());
        return 1;
    }
    const size_t n = (size_t)H * W;
    uint8_t* L = malloc(n);
    uint8_t* R = malloc(n);
    float* depth = malloc(n * sizeof(float));
    float* disp = malloc(n * sizeof(float));
    uint8_t* norm = malloc(n);
    if (!L || !R || !depth || !disp || !norm) return 1;
    uint32_t s = 12345u;
    for (size_t i = 0; i < n; ++i) {
        s = s * 1664525u + 1013904223u;
        L[i] = (uint8_t)(s >> 24);
    }
    for (int y = 0; y < H; ++y)   /* right view: scene content moved left by `shift` */
        for (int x = 0; x < W; ++x) R[(size_t)y * W + x] = L[(size_t)y * W + (x + shift < W ? x + shift : W - 1)];

    /* depth_map.py defaults: min_depth 0.3, max_depth 2.0, MIN_DISP 0 */
    const float min_depth = 0.3f, max_depth = 2.0f, range = (float)(2.0 - 0.3);
    int rc = sv_depth_map(ctx, L, R, H, W, 1, W, 0, D, win, SV_COST_SAD, min_depth, max_depth, range, 0.0f,
                          depth, disp, norm);
    if (rc != 0) {
        fprintf(stderr, "sv_depth_map: %d %s\n", rc, sv_last_error());
        return 1;
    }
    /* interior pixels (away from the matched band's edges and the replicated right border)
     * must recover the shift exactly */
    long bad = 0, checked = 0;
    for (int y = win; y < H - win; ++y)
        for (int x = D + win; x < W - shift - win; ++x, ++checked)
            if (disp[(size_t)y * W + x] != (float)shift) ++bad;
    const double t0 = now_s();
    for (int i = 0; i < calls && rc == 0; ++i)
        rc = sv_depth_map(ctx, L, R, H, W, 1, W, 0, D, win, SV_COST_SAD, min_depth, max_depth, range, 0.0f,
                          depth, disp, norm);
    const double dt = now_s() - t0;
    printf("{\"H\": %d, \"W\": %d, \"num_disp\": %d, \"win\": %d, \"shift\": %d, \"checked\": %ld, "
           "\"mismatched\": %ld, \"calls\": %d, \"ms_per_call\": %.3f, \"rc\": %d}\n",
           H, W, D, win, shift, checked, bad, calls, 1e3 * dt / calls, rc);
    sv_destroy(ctx);
    free(L);
    free(R);
    free(depth);
    free(disp);
    free(norm);
    return (bad == 0 && rc == 0) ? 0 : 1;
}
