/*
 * sv_oracle.c — independent C restatement of the stereo-disparity hot path.
 *
 * TEST INFRASTRUCTURE ONLY: linked/loaded exclusively by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg (as the checker / CPU baseline), never by the product
 * library.  Semantics are identical to oracle/sv_oracle.py (see its header for the
 * reference file:line each stage follows and for the parity status: parity is UNPINNED
 * against the reference's OpenCV SGBM, which is absent from this image).
 *
 * Algorithm: per disparity, per row band, horizontal running box sums of the per-pixel
 * cost followed by vertical running sums (O(1) per cost cell), first-min argmin.
 * Threads: OpenMP over row bands (nthreads <= 0 means "OpenMP default").
 * Build: see oracle/Makefile (gcc -O3 -fopenmp -ffp-contract=off).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { SVO_SAD = 0, SVO_SSD = 1, SVO_HOG = 2 };

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline int refl101(int i, int n) {
    if (n == 1) return 0;
    if (i < 0) i = -i;
    if (i >= n) i = 2 * (n - 1) - i;
    return i;
}

int svo_valid_columns(int W, int min_disp, int num_disp, int* x0, int* x1) {
    int maxd = min_disp + num_disp;
    int a = maxd > 0 ? maxd : 0;
    int b = W + (min_disp < 0 ? min_disp : 0);
    if (b > W) b = W;
    if (b < a) b = a;
    *x0 = a; *x1 = b;
    return 0;
}

/* cvtColor BGR2GRAY, 14-bit fixed point (depth_map.py:871-880 call site). */
void svo_gray(const uint8_t* bgr, int H, int W, int pitch, uint8_t* out) {
    for (int y = 0; y < H; ++y) {
        const uint8_t* s = bgr + (size_t)y * pitch;
        for (int x = 0; x < W; ++x) {
            int v = s[3 * x] * 1868 + s[3 * x + 1] * 9617 + s[3 * x + 2] * 4899 + (1 << 13);
            out[(size_t)y * W + x] = (uint8_t)(v >> 14);
        }
    }
}

static void sobel_at(const uint8_t* g, int H, int W, int pitch, int x, int y, int* gx, int* gy) {
    int xm = refl101(x - 1, W), xp = refl101(x + 1, W);
    int ym = refl101(y - 1, H), yp = refl101(y + 1, H);
    const uint8_t* rm = g + (size_t)ym * pitch;
    const uint8_t* r0 = g + (size_t)y * pitch;
    const uint8_t* rp = g + (size_t)yp * pitch;
    *gx = (rm[xp] + 2 * r0[xp] + rp[xp]) - (rm[xm] + 2 * r0[xm] + rp[xm]);
    *gy = (rp[xm] + 2 * rp[x] + rp[xp]) - (rm[xm] + 2 * rm[x] + rm[xp]);
}

/* Harris response, cornerHarris(blockSize=3, ksize=3, k=0.04) convention. */
void svo_harris(const uint8_t* g, int H, int W, int pitch, float* out) {
    int* gxx = (int*)malloc(sizeof(int) * (size_t)H * W * 3);
    int* gxy = gxx + (size_t)H * W;
    int* gyy = gxy + (size_t)H * W;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int gx, gy;
            sobel_at(g, H, W, pitch, x, y, &gx, &gy);
            size_t i = (size_t)y * W + x;
            gxx[i] = gx * gx; gxy[i] = gx * gy; gyy[i] = gy * gy;
        }
    const float s2 = (float)((1.0 / (4.0 * 3.0 * 255.0)) * (1.0 / (4.0 * 3.0 * 255.0)));
    const float k = 0.04f;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int sxx = 0, sxy = 0, syy = 0;
            for (int j = -1; j <= 1; ++j)
                for (int i = -1; i <= 1; ++i) {
                    size_t q = (size_t)refl101(y + j, H) * W + refl101(x + i, W);
                    sxx += gxx[q]; sxy += gxy[q]; syy += gyy[q];
                }
            float a = (float)sxx * s2, b = (float)sxy * s2, c = (float)syy * s2;
            float t1 = a * c, t2 = b * b, t3 = a + c, t4 = t3 * t3;
            float r = t1 - t2;
            float kt = k * t4;
            out[(size_t)y * W + x] = r - kt;
        }
    free(gxx);
}

/* Per-pixel HOG (bin, magnitude); window histograms [9][H][W] u16 (replicate clamp). */
static const int64_t HOG_C[8] = {15396, 12551, 8192, 2845, -2845, -8192, -12551, -15396};
static const int64_t HOG_S[8] = {5604, 10531, 14189, 16135, 16135, 14189, 10531, 5604};

void svo_hog_hist(const uint8_t* g, int H, int W, int pitch, int win, uint16_t* hist) {
    int r = win / 2;
    uint8_t* bin = (uint8_t*)malloc((size_t)H * W);
    uint8_t* mag = (uint8_t*)malloc((size_t)H * W);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int gx, gy;
            sobel_at(g, H, W, pitch, x, y, &gx, &gy);
            int m = (abs(gx) + abs(gy)) >> 3;
            if (gy < 0 || (gy == 0 && gx < 0)) { gx = -gx; gy = -gy; }
            int b = 0;
            for (int k = 0; k < 8; ++k) b += (HOG_C[k] * gy - HOG_S[k] * gx >= 0);
            bin[(size_t)y * W + x] = (uint8_t)b;
            mag[(size_t)y * W + x] = (uint8_t)m;
        }
    /* per bin: horizontal then vertical running sums with clamped coordinates */
    uint32_t* hs = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)H * W);
    for (int b = 0; b < 9; ++b) {
        for (int y = 0; y < H; ++y) {
            const uint8_t* br = bin + (size_t)y * W;
            const uint8_t* mr = mag + (size_t)y * W;
            for (int x = 0; x < W; ++x) {
                uint32_t s = 0;
                for (int i = -r; i <= r; ++i) {
                    int c = clampi(x + i, 0, W - 1);
                    s += br[c] == b ? mr[c] : 0;
                }
                hs[(size_t)y * W + x] = s;
            }
        }
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                uint32_t s = 0;
                for (int j = -r; j <= r; ++j) s += hs[(size_t)clampi(y + j, 0, H - 1) * W + x];
                hist[((size_t)b * H + y) * W + x] = (uint16_t)s;
            }
    }
    free(hs); free(bin); free(mag);
}

/* One band of output rows [y0, y1) for SAD/SSD. */
static void band_box(const uint8_t* L, const uint8_t* R, int H, int W, int pitch, int minD,
                     int D, int r, int cost, int X0, int X1, int y0, int y1, int16_t* out,
                     int opitch) {
    const int nx = X1 - X0, nrows = (y1 - y0) + 2 * r, na = nx + 2 * r;
    uint32_t* hs = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)nrows * nx);
    uint32_t* ad = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)na);
    uint32_t* vs = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)nx);
    uint32_t* bc = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(y1 - y0) * nx);
    int* bd = (int*)malloc(sizeof(int) * (size_t)(y1 - y0) * nx);
    int* cl = (int*)malloc(sizeof(int) * (size_t)na);
    for (int i = 0; i < na; ++i) cl[i] = clampi(X0 - r + i, 0, W - 1);
    for (size_t i = 0; i < (size_t)(y1 - y0) * nx; ++i) { bc[i] = UINT32_MAX; bd[i] = minD; }
    for (int d = minD; d < minD + D; ++d) {
        for (int q = 0; q < nrows; ++q) {
            int yy = clampi(y0 - r + q, 0, H - 1);
            const uint8_t* lr = L + (size_t)yy * pitch;
            const uint8_t* rr = R + (size_t)yy * pitch;
            for (int i = 0; i < na; ++i) {
                int lv = lr[cl[i]];
                int rv = rr[clampi(X0 - r + i - d, 0, W - 1)];
                int df = lv - rv;
                ad[i] = cost == SVO_SAD ? (uint32_t)abs(df) : (uint32_t)(df * df);
            }
            uint32_t s = 0;
            for (int i = 0; i <= 2 * r; ++i) s += ad[i];
            uint32_t* h = hs + (size_t)q * nx;
            h[0] = s;
            for (int x = 1; x < nx; ++x) { s += ad[x + 2 * r] - ad[x - 1]; h[x] = s; }
        }
        for (int x = 0; x < nx; ++x) {
            uint32_t s = 0;
            for (int q = 0; q <= 2 * r; ++q) s += hs[(size_t)q * nx + x];
            vs[x] = s;
        }
        for (int y = 0; y < y1 - y0; ++y) {
            if (y > 0) {
                const uint32_t* add = hs + (size_t)(y + 2 * r) * nx;
                const uint32_t* sub = hs + (size_t)(y - 1) * nx;
                for (int x = 0; x < nx; ++x) vs[x] += add[x] - sub[x];
            }
            uint32_t* bcr = bc + (size_t)y * nx;
            int* bdr = bd + (size_t)y * nx;
            for (int x = 0; x < nx; ++x)
                if (vs[x] < bcr[x]) { bcr[x] = vs[x]; bdr[x] = d; }
        }
    }
    for (int y = y0; y < y1; ++y)
        for (int x = 0; x < nx; ++x) out[(size_t)y * opitch + X0 + x] = (int16_t)(bd[(size_t)(y - y0) * nx + x] * 16);
    free(hs); free(ad); free(vs); free(bc); free(bd); free(cl);
}

static void band_hog(const uint16_t* hl, const uint16_t* hr, int H, int W, int minD, int D,
                     int X0, int X1, int y0, int y1, int16_t* out, int opitch) {
    for (int y = y0; y < y1; ++y)
        for (int x = X0; x < X1; ++x) {
            uint32_t best = UINT32_MAX;
            int bdv = minD;
            for (int d = minD; d < minD + D; ++d) {
                int xr = clampi(x - d, 0, W - 1);
                uint32_t c = 0;
                for (int b = 0; b < 9; ++b) {
                    int a = hl[((size_t)b * H + y) * W + x];
                    int e = hr[((size_t)b * H + y) * W + xr];
                    c += (uint32_t)abs(a - e);
                }
                if (c < best) { best = c; bdv = d; }
            }
            out[(size_t)y * opitch + x] = (int16_t)(bdv * 16);
        }
}

/*
 * Disparity (x16, int16) for output rows [row0, row1); every other output element is
 * set to the invalid value (minD-1)*16.  Returns 0 or a negative error.
 */
int svo_disparity16(const uint8_t* L, const uint8_t* R, int H, int W, int pitch, int min_disp,
                    int num_disp, int win, int cost, int row0, int row1, int16_t* out,
                    int out_pitch, int nthreads) {
    if (!L || !R || !out || H <= 0 || W <= 0 || num_disp <= 0 || win < 1 || (win & 1) == 0)
        return -22;
    if (row0 < 0) row0 = 0;
    if (row1 > H) row1 = H;
    const int16_t inv = (int16_t)((min_disp - 1) * 16);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) out[(size_t)y * out_pitch + x] = inv;
    int X0, X1;
    svo_valid_columns(W, min_disp, num_disp, &X0, &X1);
    if (X1 <= X0 || row1 <= row0) return 0;
    const int r = win / 2;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    if (cost == SVO_HOG) {
        uint16_t* hl = (uint16_t*)malloc(sizeof(uint16_t) * 9 * (size_t)H * W);
        uint16_t* hr = (uint16_t*)malloc(sizeof(uint16_t) * 9 * (size_t)H * W);
        svo_hog_hist(L, H, W, pitch, win, hl);
        svo_hog_hist(R, H, W, pitch, win, hr);
        const int BAND = 8;
        int nb = (row1 - row0 + BAND - 1) / BAND;
#pragma omp parallel for schedule(dynamic, 1)
        for (int b = 0; b < nb; ++b) {
            int y0 = row0 + b * BAND, y1 = y0 + BAND > row1 ? row1 : y0 + BAND;
            band_hog(hl, hr, H, W, min_disp, num_disp, X0, X1, y0, y1, out, out_pitch);
        }
        free(hl); free(hr);
        return 0;
    }
    if (cost != SVO_SAD && cost != SVO_SSD) return -22;
    const int BAND = 32;
    int nb = (row1 - row0 + BAND - 1) / BAND;
#pragma omp parallel for schedule(dynamic, 1)
    for (int b = 0; b < nb; ++b) {
        int y0 = row0 + b * BAND, y1 = y0 + BAND > row1 ? row1 : y0 + BAND;
        band_box(L, R, H, W, pitch, min_disp, num_disp, r, cost, X0, X1, y0, y1, out, out_pitch);
    }
    return 0;
}

/* medianBlur(., 5) with replicate border, then /16 (depth_map.py:909-912). */
void svo_median5_f32(const int16_t* in, int H, int W, float* out) {
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y) {
        int v[25];
        for (int x = 0; x < W; ++x) {
            int n = 0;
            for (int j = -2; j <= 2; ++j)
                for (int i = -2; i <= 2; ++i)
                    v[n++] = in[(size_t)clampi(y + j, 0, H - 1) * W + clampi(x + i, 0, W - 1)];
            for (int a = 0; a <= 12; ++a) {            /* partial selection sort */
                int m = a;
                for (int b = a + 1; b < 25; ++b) if (v[b] < v[m]) m = b;
                int t = v[a]; v[a] = v[m]; v[m] = t;
            }
            out[(size_t)y * W + x] = (float)v[12] / 16.0f;
        }
    }
}

/* depth_map.py:915-937.  minf/maxf/rangef are f32(min_depth), f32(max_depth),
 * f32(max_depth - min_depth computed in double), as NumPy-2 casts them. */
void svo_depth_post(const float* disp, int n, float minf, float maxf, float rangef,
                    float min_disp_global, float* depth_final, uint8_t* norm) {
    const float fxb = (float)(700 * 0.08);
    const float eps = (float)1e-6;
    for (int i = 0; i < n; ++i) {
        float d = disp[i];
        float den = d + eps;
        float depth = fxb / den;
        float dc = depth < minf ? minf : depth;  /* np.clip = minimum(maximum(a, lo), hi) */
        dc = dc > maxf ? maxf : dc;
        int valid = (d > min_disp_global) && (dc >= minf) && (dc <= maxf);
        depth_final[i] = valid ? dc : 0.0f;
        float t = dc - minf;
        t = t / rangef;
        t = t * 255.0f;
        norm[i] = (uint8_t)(int)t;
    }
}

/* fused_depth_map.py:1010-1029. */
void svo_scaled_post(const float* disp, int n, int min_disp, int num_disp, float* dnorm,
                     uint8_t* dnorm_u8, float* conf) {
    const float lo = (float)min_disp, hi = (float)(min_disp + num_disp - 1);
    for (int i = 0; i < n; ++i) {
        float d = disp[i];
        float c = d < lo ? lo : d;
        c = c > hi ? hi : c;
        float t = c - lo;
        t = t / (float)num_disp;
        t = t * 255.0f;
        uint8_t u = (uint8_t)(int)t;
        dnorm_u8[i] = u;
        dnorm[i] = (float)u;
        conf[i] = (d > (float)(min_disp + 1) && d < (float)(min_disp + num_disp - 1)) ? 1.0f : 0.0f;
    }
}

/* Whole app-1 path for one gray pair: disparity16 -> median/16 -> depth post. */
int svo_depth_map(const uint8_t* L, const uint8_t* R, int H, int W, int min_disp, int num_disp,
                  int win, int cost, float minf, float maxf, float rangef, float* depth_final,
                  float* disparity, uint8_t* norm, int nthreads) {
    int16_t* d16 = (int16_t*)malloc(sizeof(int16_t) * (size_t)H * W);
    int rc = svo_disparity16(L, R, H, W, W, min_disp, num_disp, win, cost, 0, H, d16, W, nthreads);
    if (rc == 0) {
        svo_median5_f32(d16, H, W, disparity);
        svo_depth_post(disparity, H * W, minf, maxf, rangef, (float)min_disp, depth_final, norm);
    }
    free(d16);
    return rc;
}

int svo_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
