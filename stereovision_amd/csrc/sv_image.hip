// sv_image.hip — the stencil kernels around the disparity engine (gfx950).
//
//  * k_gray        cv2.cvtColor(BGR2GRAY), 14-bit fixed point   (depth_map.py:871-880)
//  * k_harris_lds  Harris response, cornerHarris(3, 3, 0.04) convention (north_star)
//  * k_hog_hist_cr per-pixel 9-bin gradient orientation + window histograms (north_star),
//                  4 columns per lane (k_hog_hist: the 64x16 tile form for > 2 GB records)
//  * k_median_i16  medianBlur(disparity, 5) on the int16 x16 map, fused with the
//                  reference's post-processing (depth_map.py:909-937 or
//                  fused_depth_map.py:1004-1029) so the filtered map never round-trips HBM
//  * k_median_f32  medianBlur(f32, 5) for arbitrary float input (the public sv_median5_f32)
//  * k_post        the post-processing alone on an f32 disparity
// All are HBM-bound stencils: LDS tiles with halos, one read and one write per pixel.
// Built with -ffp-contract=off so every f32 operation rounds exactly like NumPy's.
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include "sv_internal.h"
#include "sv_median_net.h"

namespace sv {
namespace {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }
__device__ __forceinline__ int refl101(int i, int n) {
    if (n == 1) return 0;
    i = i < 0 ? -i : i;
    return i >= n ? 2 * (n - 1) - i : i;
}

// ---------------------------------------------------------------------------------------
__global__ void k_gray(const uint8_t* __restrict__ bgr, int H, int W, int pitch,
                       uint8_t* __restrict__ gray) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= W) return;
    const uint8_t* p = bgr + (size_t)y * pitch + 3 * x;
    const int v = p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13);
    gray[(size_t)y * W + x] = (uint8_t)(v >> 14);
}

__device__ __forceinline__ void sobel(const uint8_t* g, int H, int W, int pitch, int x, int y,
                                      int& gx, int& gy) {
    const int xm = refl101(x - 1, W), xp = refl101(x + 1, W);
    const uint8_t* rm = g + (size_t)refl101(y - 1, H) * pitch;
    const uint8_t* r0 = g + (size_t)y * pitch;
    const uint8_t* rp = g + (size_t)refl101(y + 1, H) * pitch;
    gx = (rm[xp] + 2 * r0[xp] + rp[xp]) - (rm[xm] + 2 * r0[xm] + rp[xm]);
    gy = (rp[xm] + 2 * rp[x] + rp[xp]) - (rm[xm] + 2 * rm[x] + rm[xp]);
}

// ---------------------------------------------------------------------------------------
// Harris as one LDS stencil pass (north_star: Sobel + structure tensor fused): a block
// stages the (64+4) x (16+4) image bytes of its 64 x 16 output tile once, forms the
// gradient products of the (64+2) x (16+2) in-image positions around it from LDS, and box-
// sums them per output (4 rows per thread).  Reflect-101 borders index the staged rows/cols
// directly (every reflected index used lies inside the staged window), so the response is
// identical to cv2.cornerHarris's convention.  grid.z = frame of a batch.
constexpr int HX2 = 64, HY2 = 16;
__global__ __launch_bounds__(256) void k_harris_lds(const uint8_t* __restrict__ g, int H, int W, int pitch,
                                                    float* __restrict__ out, long long fs_in, long long fs_out) {
    __shared__ uint8_t img[HY2 + 4][HX2 + 4];
    __shared__ int pxx[HY2 + 2][HX2 + 2], pxy[HY2 + 2][HX2 + 2], pyy[HY2 + 2][HX2 + 2];
    g += blockIdx.z * fs_in;
    out += blockIdx.z * fs_out;
    const int x0 = blockIdx.x * HX2, y0 = blockIdx.y * HY2;
    for (int i = threadIdx.x; i < (HY2 + 4) * (HX2 + 4); i += 256) {
        const int r = i / (HX2 + 4), c = i - r * (HX2 + 4);
        img[r][c] = g[(size_t)clampi(y0 - 2 + r, 0, H - 1) * pitch + clampi(x0 - 2 + c, 0, W - 1)];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < (HY2 + 2) * (HX2 + 2); i += 256) {
        const int r = i / (HX2 + 2), c = i - r * (HX2 + 2);
        const int y = y0 - 1 + r, x = x0 - 1 + c;
        if (y < 0 || y >= H || x < 0 || x >= W) continue;   // never read (box sums reflect)
        const int ym = refl101(y - 1, H) - (y0 - 2), yp = refl101(y + 1, H) - (y0 - 2), yc = y - (y0 - 2);
        const int xm = refl101(x - 1, W) - (x0 - 2), xp = refl101(x + 1, W) - (x0 - 2), xc = x - (x0 - 2);
        const int gx = (img[ym][xp] + 2 * img[yc][xp] + img[yp][xp]) - (img[ym][xm] + 2 * img[yc][xm] + img[yp][xm]);
        const int gy = (img[yp][xm] + 2 * img[yp][xc] + img[yp][xp]) - (img[ym][xm] + 2 * img[ym][xc] + img[ym][xp]);
        pxx[r][c] = gx * gx;
        pxy[r][c] = gx * gy;
        pyy[r][c] = gy * gy;
    }
    __syncthreads();
    const int tx = threadIdx.x % HX2, tq = 4 * (threadIdx.x / HX2);
    const int x = x0 + tx;
    if (x >= W) return;
    const int cm = refl101(x - 1, W) - (x0 - 1), cc = x - (x0 - 1), cp = refl101(x + 1, W) - (x0 - 1);
    const float s2 = (float)((1.0 / (4.0 * 3.0 * 255.0)) * (1.0 / (4.0 * 3.0 * 255.0)));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int y = y0 + tq + q;
        if (y >= H) break;
        const int rows[3] = {refl101(y - 1, H) - (y0 - 1), y - (y0 - 1), refl101(y + 1, H) - (y0 - 1)};
        int sxx = 0, sxy = 0, syy = 0;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int rr = rows[j];
            sxx += pxx[rr][cm] + pxx[rr][cc] + pxx[rr][cp];
            sxy += pxy[rr][cm] + pxy[rr][cc] + pxy[rr][cp];
            syy += pyy[rr][cm] + pyy[rr][cc] + pyy[rr][cp];
        }
        const float a = (float)sxx * s2, b = (float)sxy * s2, c = (float)syy * s2;
        const float t1 = a * c, t2 = b * b, t3 = a + c, t4 = t3 * t3;
        const float rr = t1 - t2;
        const float kt = 0.04f * t4;
        out[(size_t)y * W + x] = rr - kt;
    }
}

// ---------------------------------------------------------------------------------------
// Harris, register/DPP form (the default for W, H >= 8): one wave = 64 consecutive columns
// (lane j <-> column x0 - 2 + j, 60 outputs for lanes 2..61) walking down a band of HB output
// rows (PF image rows prefetched); no LDS, no barriers.  Per product row a lane loads ONE image byte (its column of the
// next row, reflect-101), its left/right neighbours come by wave_shr/wave_shl DPP: the Sobel
// column sums and row smooths, the 3 gradient products, their vertical 3-row sums from a
// register ring and the horizontal 3-sums by DPP again; coalesced f32 stores.  Reflect-101
// of the PRODUCT images (cv2.cornerHarris box-filters the products with reflect-101) falls
// out of computing every product from reflect-101 pixels, except the cross product's sign:
// outside the image gx (row) or gy (column) flips, so gxy is negated once per dimension in
// which the position lies outside (gxx, gyy are even).  Sums are exact integers; the float
// epilogue is the LDS kernel's, so outputs are identical.
// One wave's band: output columns x0 .. x0+59, rows y0 .. y0+HB-1 of one frame.
template <int HB, int PF>
__device__ __forceinline__ void harris_wave(const uint8_t* __restrict__ g, int H, int W, int pitch,
                                            float* __restrict__ out, int x0, int y0, int lane) {
    const int c = x0 - 2 + lane;
    const int cc = refl101(clampi(c, -2, W + 1), W);              // loaded column
    const int csign = (c < 0 || c >= W) ? -1 : 1;                  // gxy sign outside the image
    const bool emit = lane >= 2 && lane < 62 && c < W;
    auto ldrow = [&](int r) -> int {   // image row r (reflect-101), this lane's column
        return (int)g[(size_t)refl101(clampi(r, -2, H + 1), H) * pitch + cc];
    };
    // lane j-1 / j+1 through a plain v_mov_b32_dpp wave_shr/shl:1 kept unfolded: folded into
    // an ALU op (v_subrev_u32_dpp ... wave_shr:1 bound_ctrl:1, what the compiler emits for
    // old = 0) the wave shifts read 0 on every lane on gfx950 (tools/microbench/dpp_check)
    auto shr1 = [](int v) {
        int t = __builtin_amdgcn_update_dpp(v, v, 0x138, 0xF, 0xF, false);
        asm volatile("" : "+v"(t));
        return t;
    };
    auto shl1 = [](int v) {
        int t = __builtin_amdgcn_update_dpp(v, v, 0x130, 0xF, 0xF, false);
        asm volatile("" : "+v"(t));
        return t;
    };
    auto rowsm = [&](int v) { return shr1(v) + 2 * v + shl1(v); };
    const float s2 = (float)((1.0 / (4.0 * 3.0 * 255.0)) * (1.0 / (4.0 * 3.0 * 255.0)));
    // product rows y0-1 .. y0+HB; image rows y0-2 .. y0+HB+1
    // PF image rows in flight ahead of the one being used (the loads are one byte per lane:
    // latency, not bandwidth, is what they cost)
    int im = ldrow(y0 - 2), ic = ldrow(y0 - 1);
    int pre[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) pre[k] = ldrow(y0 + k);
    int rsm = rowsm(im), rsc = rowsm(ic);
    int pxx[3] = {0, 0, 0}, pxy[3] = {0, 0, 0}, pyy[3] = {0, 0, 0};
    const int rend = min(y0 + HB, H);                               // last output row + 1
    for (int r = y0 - 1; r <= rend; ++r) {
        const int ip = pre[0];
#pragma unroll
        for (int k = 0; k + 1 < PF; ++k) pre[k] = pre[k + 1];
        pre[PF - 1] = ldrow(r + 1 + PF);
        const int rsp = rowsm(ip);
        const int col = im + 2 * ic + ip;
        const int gx = shl1(col) - shr1(col);
        const int gy = rsp - rsm;
        const int rsign = (r < 0 || r >= H) ? -csign : csign;
        pxx[0] = pxx[1]; pxx[1] = pxx[2]; pxx[2] = __mul24(gx, gx);
        pyy[0] = pyy[1]; pyy[1] = pyy[2]; pyy[2] = __mul24(gy, gy);
        pxy[0] = pxy[1]; pxy[1] = pxy[2]; pxy[2] = rsign * __mul24(gx, gy);
        im = ic;
        ic = ip;
        rsm = rsc;
        rsc = rsp;
        if (r >= y0 + 1) {   // output row r - 1 from product rows r-2 .. r
            const int vxx = pxx[0] + pxx[1] + pxx[2], vxy = pxy[0] + pxy[1] + pxy[2], vyy = pyy[0] + pyy[1] + pyy[2];
            const int sxx = shr1(vxx) + vxx + shl1(vxx);
            const int sxy = shr1(vxy) + vxy + shl1(vxy);
            const int syy = shr1(vyy) + vyy + shl1(vyy);
            const float a = (float)sxx * s2, b = (float)sxy * s2, cf = (float)syy * s2;
            const float t1 = a * cf, t2 = b * b, t3 = a + cf, t4 = t3 * t3;
            const float rr = t1 - t2;
            const float kt = 0.04f * t4;
            if (emit) out[(size_t)(r - 1) * W + c] = rr - kt;
        }
    }
}

template <int HB, int PF>
__global__ __launch_bounds__(64) void k_harris_dpp(const uint8_t* __restrict__ g, int H, int W, int pitch,
                                                   float* __restrict__ out, long long fs_in, long long fs_out) {
    harris_wave<HB, PF>(g + blockIdx.z * fs_in, H, W, pitch, out + blockIdx.z * fs_out, blockIdx.x * 60,
                        blockIdx.y * HB, threadIdx.x);
}

// Harris, 4 columns per lane (the default for W >= 1024; any W >= 256 works): lane j holds columns x0-4+4j ..
// x0-1+4j as one dword per image row (interior waves: one aligned dword load per lane-row;
// waves touching an image border or unaligned rows assemble it from 4 reflect-101 byte
// loads), the lane's first/last neighbours come by wave_shr/shl:1 DPP; 248 output columns
// per wave (lanes 1..62), f32x4 stores.  Same arithmetic, same reflect-101 product rule and
// the same float epilogue as k_harris_dpp: bit-identical outputs.
__device__ __forceinline__ int dpp_shr1_keep(int v) {   // lane j-1 (lane 0 keeps its own)
    int t = __builtin_amdgcn_update_dpp(v, v, 0x138, 0xF, 0xF, false);
    asm volatile("" : "+v"(t));
    return t;
}
__device__ __forceinline__ int dpp_shl1_keep(int v) {   // lane j+1 (lane 63 keeps its own)
    int t = __builtin_amdgcn_update_dpp(v, v, 0x130, 0xF, 0xF, false);
    asm volatile("" : "+v"(t));
    return t;
}

// One wave's band: output columns x0 .. x0+247, rows y0 .. y0+HB-1 of one frame.
template <int HB, int PF>
__device__ __forceinline__ void harris_wave4(const uint8_t* __restrict__ g, int H, int W, int pitch,
                                             float* __restrict__ out, int x0, int y0, int lane) {
    const int c0 = x0 - 4 + 4 * lane;                               // first column of the lane
    // interior: every lane's 4 columns inside the image and dword-aligned rows (uniform)
    const bool fast = x0 >= 4 && x0 + 252 <= W && ((pitch & 3) == 0) && ((((uintptr_t)g) & 3) == 0);
    int cc[4], csg[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = c0 + i;
        cc[i] = refl101(clampi(c, -2, W + 1), W);
        csg[i] = (c < 0 || c >= W) ? -1 : 1;
    }
    auto ldrow = [&](int r) -> uint32_t {   // image row r (reflect-101), the lane's 4 columns
        const uint8_t* row = g + (size_t)refl101(clampi(r, -2, H + 1), H) * pitch;
        if (fast) return *reinterpret_cast<const uint32_t*>(row + c0);
        return (uint32_t)row[cc[0]] | ((uint32_t)row[cc[1]] << 8) | ((uint32_t)row[cc[2]] << 16) |
               ((uint32_t)row[cc[3]] << 24);
    };
    auto unpack = [](uint32_t w, int (&p)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) p[i] = (int)((w >> (8 * i)) & 0xffu);
    };
    // row smooth p[i-1] + 2 p[i] + p[i+1] of the lane's 4 columns (neighbour bytes by DPP)
    auto rowsm4 = [&](uint32_t w, int (&o)[4]) {
        int p[4];
        unpack(w, p);
        const int lft = (int)(((uint32_t)dpp_shr1_keep((int)w)) >> 24);
        const int rgt = (int)(((uint32_t)dpp_shl1_keep((int)w)) & 0xffu);
        o[0] = lft + 2 * p[0] + p[1];
        o[1] = p[0] + 2 * p[1] + p[2];
        o[2] = p[1] + 2 * p[2] + p[3];
        o[3] = p[2] + 2 * p[3] + rgt;
    };
    const float s2 = (float)((1.0 / (4.0 * 3.0 * 255.0)) * (1.0 / (4.0 * 3.0 * 255.0)));
    int im[4], ic[4], rsm[4], rsc[4];
    {
        const uint32_t wm = ldrow(y0 - 2), wc = ldrow(y0 - 1);
        unpack(wm, im);
        unpack(wc, ic);
        rowsm4(wm, rsm);
        rowsm4(wc, rsc);
    }
    uint32_t pre[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) pre[k] = ldrow(y0 + k);
    int pxx[3][4] = {}, pxy[3][4] = {}, pyy[3][4] = {};
    const int rend = min(y0 + HB, H);
    const bool emit_lane = lane >= 1 && lane < 63;
    for (int r = y0 - 1; r <= rend; ++r) {
        const uint32_t wp = pre[0];
#pragma unroll
        for (int k = 0; k + 1 < PF; ++k) pre[k] = pre[k + 1];
        pre[PF - 1] = ldrow(r + 1 + PF);
        int ip[4], rsp[4], col[4];
        unpack(wp, ip);
        rowsm4(wp, rsp);
#pragma unroll
        for (int i = 0; i < 4; ++i) col[i] = im[i] + 2 * ic[i] + ip[i];
        const int cl = dpp_shr1_keep(col[3]), cr = dpp_shl1_keep(col[0]);
        const bool rout = r < 0 || r >= H;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int gx = (i < 3 ? col[i + 1] : cr) - (i > 0 ? col[i - 1] : cl);
            const int gy = rsp[i] - rsm[i];
            const int sg = rout ? -csg[i] : csg[i];
            pxx[0][i] = pxx[1][i]; pxx[1][i] = pxx[2][i]; pxx[2][i] = __mul24(gx, gx);
            pyy[0][i] = pyy[1][i]; pyy[1][i] = pyy[2][i]; pyy[2][i] = __mul24(gy, gy);
            pxy[0][i] = pxy[1][i]; pxy[1][i] = pxy[2][i]; pxy[2][i] = sg * __mul24(gx, gy);
            im[i] = ic[i];
            ic[i] = ip[i];
            rsm[i] = rsc[i];
            rsc[i] = rsp[i];
        }
        if (r >= y0 + 1) {   // output row r - 1
            int vxx[4], vxy[4], vyy[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                vxx[i] = pxx[0][i] + pxx[1][i] + pxx[2][i];
                vxy[i] = pxy[0][i] + pxy[1][i] + pxy[2][i];
                vyy[i] = pyy[0][i] + pyy[1][i] + pyy[2][i];
            }
            const int lxx = dpp_shr1_keep(vxx[3]), rxx = dpp_shl1_keep(vxx[0]);
            const int lxy = dpp_shr1_keep(vxy[3]), rxy = dpp_shl1_keep(vxy[0]);
            const int lyy = dpp_shr1_keep(vyy[3]), ryy = dpp_shl1_keep(vyy[0]);
            float o[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int sxx = (i > 0 ? vxx[i - 1] : lxx) + vxx[i] + (i < 3 ? vxx[i + 1] : rxx);
                const int sxy = (i > 0 ? vxy[i - 1] : lxy) + vxy[i] + (i < 3 ? vxy[i + 1] : rxy);
                const int syy = (i > 0 ? vyy[i - 1] : lyy) + vyy[i] + (i < 3 ? vyy[i + 1] : ryy);
                const float a = (float)sxx * s2, b = (float)sxy * s2, cf = (float)syy * s2;
                const float t1 = a * cf, t2 = b * b, t3 = a + cf, t4 = t3 * t3;
                const float rr = t1 - t2;
                const float kt = 0.04f * t4;
                o[i] = rr - kt;
            }
            if (emit_lane) {
                float* orow = out + (size_t)(r - 1) * W;
                if (c0 + 3 < W && ((W & 3) == 0) && ((((uintptr_t)out) & 15) == 0)) {
                    *reinterpret_cast<float4*>(orow + c0) = make_float4(o[0], o[1], o[2], o[3]);
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (c0 + i >= 0 && c0 + i < W) orow[c0 + i] = o[i];
                }
            }
        }
    }
}

template <int HB, int PF>
__global__ __launch_bounds__(64) void k_harris_dpp4(const uint8_t* __restrict__ g, int H, int W, int pitch,
                                                    float* __restrict__ out, long long fs_in, long long fs_out) {
    harris_wave4<HB, PF>(g + blockIdx.z * fs_in, H, W, pitch, out + blockIdx.z * fs_out, blockIdx.x * 248,
                         blockIdx.y * HB, threadIdx.x);
}

// ---------------------------------------------------------------------------------------
// HOG window histograms: 64x16 output tile, window radius r <= 7.
constexpr int GT_W = 64, GT_H = 16, GR_MAX = 7;
constexpr int GX_MAX = GT_W + 2 * GR_MAX, GY_MAX = GT_H + 2 * GR_MAX;
// bin boundaries at 20°·(k+1): round(16384·cos), round(16384·sin); cos[7-k] = -cos[k] and
// sin[7-k] = sin[k], so the 8 tests need only 4 products pairs: boundary k is
// cos·gy >= sin·gx, boundary 7-k is -cos·gy >= sin·gx.
constexpr int kHogCos[4] = {15396, 12551, 8192, 2845};
constexpr int kHogSin[4] = {5604, 10531, 14189, 16135};

template <int r>   // window radius: compile-time, so the tile loops index by constants
__global__ __launch_bounds__(256) void k_hog_hist(const uint8_t* __restrict__ g, int H, int W,
                                                  int pitch, int row0, int row1,
                                                  uint16_t* __restrict__ hist) {
    __shared__ uint8_t simg[GY_MAX + 2][GX_MAX + 2];
    __shared__ uint16_t sbm[GY_MAX][GX_MAX];             // (bin << 8) | magnitude
    // window-sum records: bins 2k, 2k+1 as the u16 halves of dword k (dword 4's high half
    // is the zero pad bin 9).  Sums stay below 2^16 (<= 15*15*255), so packed adds and
    // subtracts never carry or borrow between halves.
    __shared__ uint32_t vrec[GT_H][GX_MAX][5];
    const int x0 = blockIdx.x * GT_W, y0 = row0 + blockIdx.y * GT_H;
    constexpr int nx = GT_W + 2 * r, ny = GT_H + 2 * r;
    // stage the image bytes once (all loads independent): rows y0-r-1 .. y0+GT_H+r and
    // columns x0-r-1 .. x0+GT_W+r, clamped; every pixel the gradients below read (the
    // replicate-clamped window positions and their reflect-101 neighbours) lies inside
    const int sy0 = y0 - r - 1, sx0 = x0 - r - 1;
    // rows below row1 + r feed only outputs at or past row1 (never stored): clamp the staging
    // there too, so a band-only input buffer (rows [row0 - r - 1, row1 + r] + SV_BAND_MARGIN)
    // is never read past its end when row1 - row0 is not a multiple of the tile height
    const int ylast = min(H - 1, row1 + r);
    for (int i = threadIdx.x; i < (ny + 2) * (nx + 2); i += 256) {
        const int ty = i / (nx + 2), tx = i - ty * (nx + 2);
        simg[ty][tx] = g[(size_t)clampi(sy0 + ty, 0, ylast) * pitch + clampi(sx0 + tx, 0, W - 1)];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nx * ny; i += 256) {
        const int ty = i / nx, tx = i % nx;
        const int yy = clampi(y0 - r + ty, 0, H - 1);
        const int xx = clampi(x0 - r + tx, 0, W - 1);
        const int ym = refl101(yy - 1, H) - sy0, yc = yy - sy0, yp = refl101(yy + 1, H) - sy0;
        const int xm = refl101(xx - 1, W) - sx0, xc = xx - sx0, xp = refl101(xx + 1, W) - sx0;
        int gx = (simg[ym][xp] + 2 * simg[yc][xp] + simg[yp][xp]) - (simg[ym][xm] + 2 * simg[yc][xm] + simg[yp][xm]);
        int gy = (simg[yp][xm] + 2 * simg[yp][xc] + simg[yp][xp]) - (simg[ym][xm] + 2 * simg[ym][xc] + simg[ym][xp]);
        const int m = (abs(gx) + abs(gy)) >> 3;
        if (gy < 0 || (gy == 0 && gx < 0)) { gx = -gx; gy = -gy; }
        int b = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int cy = kHogCos[k] * gy, sx = kHogSin[k] * gx;   // |products| < 2^24
            b += (cy >= sx) + (-cy >= sx);
        }
        sbm[ty][tx] = (uint16_t)((b << 8) | m);
    }
    __syncthreads();
    // vertical window sums: task = (column, half of the tile's rows), one packed record
    auto acc = [](uint32_t (&v)[5], uint32_t code, bool add) {
        const int k = (int)(code >> 9);                                  // bin / 2
        const uint32_t val = (code & 0xFFu) << ((code & 0x100u) ? 16 : 0);
#pragma unroll
        for (int kk = 0; kk < 5; ++kk) {
            const uint32_t t = kk == k ? val : 0u;
            v[kk] = add ? v[kk] + t : v[kk] - t;
        }
    };
    for (int task = threadIdx.x; task < nx * 2; task += 256) {
        const int tx = task >> 1, oy0 = (task & 1) * (GT_H / 2);
        uint32_t v[5] = {0u, 0u, 0u, 0u, 0u};
        for (int j = 0; j <= 2 * r; ++j) acc(v, sbm[oy0 + j][tx], true);
#pragma unroll
        for (int kk = 0; kk < 5; ++kk) vrec[oy0][tx][kk] = v[kk];
        for (int oy = oy0 + 1; oy < oy0 + GT_H / 2; ++oy) {
            acc(v, sbm[oy + 2 * r][tx], true);
            acc(v, sbm[oy - 1][tx], false);
#pragma unroll
            for (int kk = 0; kk < 5; ++kk) vrec[oy][tx][kk] = v[kk];
        }
    }
    __syncthreads();
    // horizontal window sums: task = (row, run of 4 columns): 256 running sums of 4 steps,
    // each thread storing its 4 records (80 contiguous bytes) straight to HBM
    {
        const int oy = threadIdx.x >> 4, c0 = (threadIdx.x & 15) * 4;
        const int y = y0 + oy, x = x0 + c0;
        uint32_t o[4][5];
        uint32_t v[5] = {0u, 0u, 0u, 0u, 0u};
        for (int i = 0; i <= 2 * r; ++i)
#pragma unroll
            for (int kk = 0; kk < 5; ++kk) v[kk] += vrec[oy][c0 + i][kk];
#pragma unroll
        for (int kk = 0; kk < 5; ++kk) o[0][kk] = v[kk];
#pragma unroll
        for (int q = 1; q < 4; ++q) {
#pragma unroll
            for (int kk = 0; kk < 5; ++kk) {
                v[kk] += vrec[oy][c0 + q + 2 * r][kk] - vrec[oy][c0 + q - 1][kk];
                o[q][kk] = v[kk];
            }
        }
        if (y < row1 && x < W) {
            uint32_t* dst = reinterpret_cast<uint32_t*>(hist + ((size_t)y * W + x) * 10);
            if (x + 3 < W && ((uintptr_t)dst & 15) == 0) {
                const uint32_t* f = &o[0][0];
                uint4* d4 = reinterpret_cast<uint4*>(dst);
#pragma unroll
                for (int k = 0; k < 5; ++k) d4[k] = make_uint4(f[4 * k], f[4 * k + 1], f[4 * k + 2], f[4 * k + 3]);
            } else {
                for (int q = 0; q < 4 && x + q < W; ++q)
#pragma unroll
                    for (int kk = 0; kk < 5; ++kk) dst[q * 5 + kk] = o[q][kk];
            }
        }
    }
}

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------
// HOG window histograms, column-run form (round 5): lane L owns K = 4 CONSECUTIVE columns,
// so the horizontal window sum is a running sum inside the lane over the vertical sums of its
// K columns and of the r columns either side, which belong to the HL = ceil(r / K) neighbour
// lanes on each side (read from LDS) — instead of a 64-lane prefix scan per row; lanes
// HL .. 63-HL emit, the HL lanes at each end are the halo.  Per step (one image row) a lane
// loads the K + 2 bytes of the one new Sobel row, forms the K Sobel pairs as packed u16
// (S = a0 + 2a1 + a2, D = a2 - a0), the magnitudes packed, and each bin with 4 v_dot2 on the
// sign-normalised (gx, gy) pair (the 8 boundary tests of k_hog_hist folded into 4: below).
// Vertical window sums: 5 packed dwords per column in LDS, one ds_add / ds_sub per code; the
// last 2r+1 codes per column in a register ring of packed u16 (slot = step mod 2r+1 through
// s_set_gpr_idx, so the body is not unrolled 2r+1 times).  Records are staged in LDS and
// leave as coalesced 16-byte stores.  118 VGPRs and 9.9 KB of LDS at r = 7 (4 waves per
// SIMD); 4K r = 7, 4 images per launch: 205 us (round 4's 64-lane strips: 249).
// Bins: with (gx', gy') sign-normalised (gy' > 0, or gy' = 0 and gx' >= 0) and F_k =
// cos_k gy' - sin_k |gx'|, k_hog_hist's b = sum_k [cos_k gy' >= sin_k gx'] + [-cos_k gy' >=
// sin_k gx'] is 4 - #{F_k < 0} for gx' >= 0 and 8 - #{F_k > 0} for gx' < 0 (cos_k, sin_k > 0:
// one of each pair of tests is decided by the sign of gx'), i.e. base - #{G_k < 0} with G_k =
// dot2((gx', gx' < 0 ? -gy' : gy'), (-sin_k, cos_k)) — except for gx' = gy' = 0, where the
// magnitude is 0 and the bin never matters.
constexpr int HC_K = 4, HC_ROWS = 24;
template <int r, int K>
struct HogCr {
    static constexpr int HL = (r + K - 1) / K;        // halo lanes per side (a window reaches HL lanes)
    static constexpr int NOUT = (64 - 2 * HL) * K;     // columns a wave emits
    static constexpr int NP = K / 2 + 1;               // packed byte pairs per image row and lane
    static constexpr int NCH = (NOUT * 20 / 16 + 63) / 64;   // 16-byte chunks per lane and row
};

typedef short v2i16 __attribute__((ext_vector_type(2)));
typedef unsigned short v2u16 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2u16 as_u2(uint32_t v) { return __builtin_bit_cast(v2u16, v); }
__device__ __forceinline__ v2i16 as_i2(uint32_t v) { return __builtin_bit_cast(v2i16, v); }
__device__ __forceinline__ uint32_t u2_as(v2u16 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t i2_as(v2i16 v) { return __builtin_bit_cast(uint32_t, v); }

template <int r, int K>
__global__ __launch_bounds__(64) void k_hog_hist_cr(const uint8_t* __restrict__ g, int H, int W, int pitch,
                                                     int row0, int row1, uint16_t* __restrict__ hist, int hs_rows,
                                                     const uint8_t* __restrict__ g1, uint16_t* __restrict__ hist1,
                                                     long long fs_in, long long fs_hist) {
    using C = HogCr<r, K>;
    constexpr int HL = C::HL, NOUT = C::NOUT, NP = C::NP;
    if (blockIdx.z) {   // image pairs: z = 2 * frame + (0 left, 1 right)
        const int f = blockIdx.z >> 1;
        if (blockIdx.z & 1) {
            g = g1;
            hist = hist1;
        }
        g += f * fs_in;
        hist += f * fs_hist;
    }
    constexpr int W2 = 2 * r + 1;
    const int lane = threadIdx.x;
    const int x0 = blockIdx.x * NOUT;
    const int xs = x0 + (lane - HL) * K;   // this lane's first column (< 0 or >= W: halo / past the edge)
    const int ys = row0 + blockIdx.y * hs_rows;
    const int ye = min(ys + hs_rows, row1);
    const int nsteps = ye - ys + 2 * r;
    const auto gsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(g), 0, 0x7FFFFFFF, 0x00020000);
    const auto hdst = __builtin_amdgcn_make_buffer_rsrc(hist, 0, 0x7FFFFFFF, 0x00020000);

    // the K + 2 byte columns xs-1 .. xs+K: reflect-101 (the neighbours of columns 0 and W-1),
    // then clamped (columns past the edge read something valid; their codes are replaced below)
    int bcol[K + 2];
#pragma unroll
    for (int i = 0; i < K + 2; ++i) bcol[i] = clampi(refl101(xs - 1 + i, W), 0, W - 1);
    auto load_row = [&](int row, int (&b)[K + 2]) {
#pragma unroll
        for (int i = 0; i < K + 2; ++i) b[i] = (int)__builtin_amdgcn_raw_buffer_load_b8(gsrc, bcol[i], row * pitch, 0);
    };
    auto pack_row = [&](const int (&b)[K + 2], uint32_t (&p)[NP]) {
#pragma unroll
        for (int m = 0; m < NP; ++m) p[m] = (uint32_t)b[2 * m] | ((uint32_t)b[2 * m + 1] << 16);
    };
    auto crow = [&](int t) { return clampi(ys - r + t, 0, H - 1); };

    // vertical window sums, [bin pair][column j][lane] (conflict-free: lane-consecutive)
    __shared__ uint32_t vs[5 * K * 64];
#pragma unroll
    for (int i = 0; i < 5 * K; ++i) vs[i * 64 + lane] = 0u;

    uint32_t R0[NP], R1[NP], R2[NP];
    int nb[K + 2];
    {
        const int c = crow(0);
        load_row(refl101(c - 1, H), nb);
        pack_row(nb, R0);
        load_row(c, nb);
        pack_row(nb, R1);
        load_row(refl101(c + 1, H), nb);
        pack_row(nb, R2);
    }

    // the code ring: K/2 packed dwords (K u16 codes) per slot, slot = step mod 2r+1 (uniform:
    // s_set_gpr_idx-relative moves, no per-slot copy of the loop body)
    typedef uint32_t v16u __attribute__((ext_vector_type(16)));
    v16u ring[K / 2];
#pragma unroll
    for (int q = 0; q < K / 2; ++q) ring[q] = (v16u)(0u);   // code 0: adds nothing

    // a row's records (NOUT of them, contiguous in HBM) are staged in LDS and leave as 16-byte
    // chunks over all 64 lanes: the same NCH + 3 stores per row on every path (a chunk past the
    // row's end rewrites the last whole chunk's bytes, a tail dword past it the last dword's,
    // both with the same values), so the next step's wait for its prefetched row counts them
    // and never waits on them.  (Dropping such stores by an offset past num_records did not
    // work: the stores landed 2 GB past the buffer.)
    __shared__ __attribute__((aligned(16))) uint32_t stage[NOUT * 5];
    const int nbytes = 20 * min(NOUT, W - x0);   // >= 20
    const int last16 = (nbytes & ~15) - 16, tb = nbytes & ~15, owner = (tb >> 4) & 63;

    const bool first_wave = x0 == 0;
    const bool last_wave = x0 + (64 - HL) * K > W;   // some column of this wave is >= W
    const int jw = (W - 1 - x0) % K, lw = (W - 1 - x0) / K + HL;   // column W-1: lane lw, j jw
    uint32_t code[K];
    int cprev = -1;
    int slot = 0;
    uint32_t Rn[NP];   // the packed row the next advancing step brings in
    // one row of codes: Sobel, bins, the edge columns, the ring and the vertical sums
    auto step = [&](int t) {
        const int c = crow(t);
        if (c != cprev) {   // uniform: a new Sobel centre row (clamped rows repeat the codes)
            if (cprev >= 0) {
#pragma unroll
                for (int m = 0; m < NP; ++m) {
                    R0[m] = R1[m];
                    R1[m] = R2[m];
                    R2[m] = Rn[m];
                }
            }
            cprev = c;
            uint32_t S[NP], D[NP];
#pragma unroll
            for (int m = 0; m < NP; ++m) {
                S[m] = u2_as(as_u2(R0[m]) + (as_u2(R1[m]) << (unsigned short)1) + as_u2(R2[m]));
                D[m] = u2_as(as_u2(R2[m]) - as_u2(R0[m]));
            }
#pragma unroll
            for (int q = 0; q < K / 2; ++q) {
                const v2i16 gx = as_i2(u2_as(as_u2(S[q + 1]) - as_u2(S[q])));
                const uint32_t dmid = __builtin_amdgcn_alignbyte(D[q + 1], D[q], 2);   // (D[2q+1], D[2q+2])
                const v2i16 gy = as_i2(u2_as(as_u2(D[q]) + (as_u2(dmid) << (unsigned short)1) + as_u2(D[q + 1])));
                const v2i16 ax = __builtin_elementwise_max(gx, -gx), ay = __builtin_elementwise_max(gy, -gy);
                const uint32_t mm = u2_as((as_u2(i2_as(ax)) + as_u2(i2_as(ay))) >> (unsigned short)3);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    // p = (gy << 16) | gx, then sign-normalised: flip iff (gy, gx) < (0, 0)
                    const uint32_t p = __builtin_amdgcn_perm(i2_as(gy), i2_as(gx), h ? 0x07060302u : 0x05040100u);
                    const int vkey = (int)p - (int)((p & 0x8000u) << 1);   // gy * 65536 + gx
                    const uint32_t fm = (uint32_t)(vkey >> 31);
                    const uint32_t pn = u2_as(as_u2(p ^ fm) - as_u2(fm));
                    const uint32_t gm = (uint32_t)((int)(pn << 16) >> 31);    // gx' < 0
                    const uint32_t hm = gm & 0xFFFF0000u;
                    const v2i16 qv = as_i2(u2_as(as_u2(pn ^ hm) - as_u2(hm)));
                    uint32_t nneg = 0;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const v2i16 w = {(short)-kHogSin[k], (short)kHogCos[k]};
                        nneg += (uint32_t)__builtin_amdgcn_sdot2(qv, w, 0, false) >> 31;
                    }
                    const uint32_t b = 4u + (gm & 4u) - nneg;
                    const uint32_t m = h ? mm >> 16 : mm & 0xFFFFu;
                    code[2 * q + h] = (b << 8) | m;
                }
            }
            // columns past the image edge take the edge column's code (clamped positions)
            if (first_wave) {
                const uint32_t c0 = __builtin_amdgcn_readlane(code[0], HL);
                if (lane < HL)
#pragma unroll
                    for (int j = 0; j < K; ++j) code[j] = c0;
            }
            if (last_wave) {
                uint32_t cw = code[0];
#pragma unroll
                for (int j = 1; j < K; ++j) cw = jw == j ? code[j] : cw;
                const uint32_t cwb = __builtin_amdgcn_readlane(cw, lw);
#pragma unroll
                for (int j = 0; j < K; ++j) code[j] = xs + j >= W ? cwb : code[j];
            }
        }
#pragma unroll
        for (int q = 0; q < K / 2; ++q) {
            const uint32_t nc = code[2 * q] | (code[2 * q + 1] << 16), oc = ring[q][slot];
            ring[q][slot] = nc;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int j = 2 * q + h;
                const uint32_t cn = code[j], co = h ? oc >> 16 : oc & 0xFFFFu;
                __hip_atomic_fetch_add(&vs[((cn >> 9) * K + j) * 64 + lane], (cn & 0xFFu) << ((cn >> 4) & 16u),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                __hip_atomic_fetch_sub(&vs[((co >> 9) * K + j) * 64 + lane], (co & 0xFFu) << ((co >> 4) & 16u),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            }
        }
        slot = slot + 1 == W2 ? 0 : slot + 1;
    };
    // each iteration loads the row step t + 1 brings in if it advances (unconditionally, at its
    // top) and packs it at its end, after the stores: no loaded register lives across the
    // back edge (a copy there would wait for the load), and the wait counts the stores
    auto prefetch = [&](int t) { load_row(refl101(crow(min(t + 1, nsteps - 1)) + 1, H), nb); };
    for (int t = 0; t < 2 * r && t < nsteps; ++t) {   // warm-up: the vertical window only
        prefetch(t);
        step(t);
        pack_row(nb, Rn);
    }
    const bool own = lane >= HL && lane < 64 - HL;
    uint32_t* srec = &stage[(own ? lane - HL : 0) * 5 * K];
    for (int t = 2 * r; t < nsteps; ++t) {
        prefetch(t);
        step(t);
        // the neighbour lanes' vertical sums of this step, just updated by their wavefront-scope
        // atomics, are read below: an acquire-release fence at wavefront scope orders the two
        // for the compiler (no instruction on gfx950: a wave's LDS ops complete in order); the
        // next step's atomics come after the barriers below
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        // horizontal window: a running sum over columns -r .. K-1+r, the outer ones the
        // neighbour lanes' vertical sums (read from LDS; LDS ops of a wave complete in order);
        // each plane's K sums go straight to the row's staging area
#pragma unroll
        for (int p = 0; p < 5; ++p) {
            uint32_t v[K + 2 * r];
#pragma unroll
            for (int i = 0; i < K + 2 * r; ++i) {
                const int col = i - r;
                const int dl = col >= 0 ? col / K : -((K - 1 - col) / K);   // source lane offset
                const int sl = min(max(lane + dl, 0), 63);
                v[i] = vs[(p * K + (col - dl * K)) * 64 + sl];
            }
            uint32_t h = v[0];
#pragma unroll
            for (int i = 1; i <= 2 * r; ++i) h += v[i];
            if (own) srec[p] = h;
#pragma unroll
            for (int j = 1; j < K; ++j) {
                h += v[j + 2 * r] - v[j - 1];
                if (own) srec[5 * j + p] = h;
            }
        }
        __syncthreads();   // (one wave: orders the staging, fences the compiler)
        const int soff = ((ys + t - 2 * r) * W + x0) * 20;
#pragma unroll
        for (int k = 0; k < C::NCH; ++k) {
            int b0 = 16 * (lane + 64 * k);
            b0 = b0 + 16 <= nbytes ? b0 : last16;
            const v4u q = *reinterpret_cast<const v4u*>(&stage[b0 >> 2]);
            __builtin_amdgcn_raw_buffer_store_b128(q, hdst, b0, soff, 0);
        }
#pragma unroll
        for (int d = 0; d < 3; ++d) {   // the tail chunk (nbytes is a multiple of 4, not always of 16)
            int o = tb + 4 * d;
            o = lane == owner && o < nbytes ? o : nbytes - 4;
            __builtin_amdgcn_raw_buffer_store_b32(stage[o >> 2], hdst, o, soff, 0);
        }
        pack_row(nb, Rn);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------
// Post-processing of one f32 disparity value (shared by the median kernels and k_post).
struct PostVals { float a, b; uint8_t u; };

__device__ __forceinline__ PostVals post_vals(const PostParams& pp, float d) {
    PostVals o{0.0f, 0.0f, 0};
    if (pp.mode == POST_DEPTH) {
        // depth_map.py:925-936 — NumPy-2 keeps float32 throughout
        const float fxb = (float)(700 * 0.08);
        const float den = d + (float)1e-6;
        const float depth = fxb / den;
        float dc = depth < pp.minf ? pp.minf : depth;
        dc = dc > pp.maxf ? pp.maxf : dc;
        const bool valid = (d > pp.min_disp_global) && (dc >= pp.minf) && (dc <= pp.maxf);
        o.a = valid ? dc : 0.0f;
        float t = dc - pp.minf;
        t = t / pp.rangef;
        t = t * 255.0f;
        o.u = (uint8_t)(int)t;
    } else if (pp.mode == POST_SCALED) {
        // fused_depth_map.py:1010-1024
        const float lo = (float)pp.min_disp, hi = (float)(pp.min_disp + pp.num_disp - 1);
        float c = d < lo ? lo : d;
        c = c > hi ? hi : c;
        float t = c - lo;
        t = t / (float)pp.num_disp;
        t = t * 255.0f;
        o.u = (uint8_t)(int)t;
        o.a = (float)o.u;
        o.b = (d > (float)(pp.min_disp + 1) && d < hi) ? 1.0f : 0.0f;
    }
    return o;
}

// Post-processing of one f32 disparity value (shared by the median kernels and k_post).
__device__ __forceinline__ void post_one(const PostParams& pp, size_t i, float d) {
    if (pp.mode == POST_NONE) return;
    const PostVals o = post_vals(pp, d);
    pp.out_a[i] = o.a;
    pp.out_u8[i] = o.u;
    if (pp.mode == POST_SCALED) pp.out_b[i] = o.b;
}

// Median-of-25 for the int16 map, 2 columns x 4 rows per lane.
// Two vertically adjacent 5x5 windows (rows y, y+1) share 20 of their 25 values (rows
// y-1..y+2): 5 columns of 4, each read by 5 horizontally adjacent windows, so every column
// is sorted once (5 comparators, in LDS).  Two horizontally adjacent windows (x, x+1) then
// share 4 of those sorted columns: the 13th of 25 has rank 3..12 among the common 16 (9
// values lie outside them), so SEL16H (41 comparators, 76 ops) takes the sorted ranks 3..12
// once per column pair and each window merges its own column in (MRG14: 20 comparators, 32
// ops) to the sorted ranks 4..9 of its 14 — the same 6 candidates C as SEL20S's ranks 7..12
// of 20 (59 comparators, 104 ops per window, the round-3 form).  Each window's unique row is
// sorted with its neighbour's (4 shared values sorted once, 1 inserted each), and the median
// is the 6th smallest of (6 sorted + 5 sorted) = min_i max(C_i, U_{4-i}) (10 ops).  Each
// lane packs two row pairs (rows y,y+1 | y+2,y+3) into short2 halves, so one
// v_pk_min/max_i16 serves both: ~34 network ops per output (46 for the SEL20S form, 113 for
// the plain 25-input network); round 4: 77 -> 68 us per 16 1080p frames.
typedef short s2 __attribute__((ext_vector_type(2)));
constexpr int MT_W = 64, MT_H = 8;        // k_median_f32 tile
constexpr int MQ_W = 128, MQ_H = 16;      // k_median_i16: 128 columns x 16 rows per block

__device__ __forceinline__ s2 as_s2(uint32_t u) { return __builtin_bit_cast(s2, u); }

// Element i of a frame-based array through a 32-bit byte offset from a uniform base, so
// loads and stores take the saddr + 32-bit voffset form (no 64-bit address arithmetic per
// access; launch_median_i16 bounds a frame to < 2^30 elements).
template <typename T>
__device__ __forceinline__ T& at(T* base, uint32_t i) {
    using B = typename std::conditional<std::is_const<T>::value, const char, char>::type;
    return *reinterpret_cast<T*>(reinterpret_cast<B*>(base) + (uint32_t)(i * (uint32_t)sizeof(T)));
}

__device__ __forceinline__ PostVals post_median(const PostParams& pp, int mv) {
    const uint32_t dm = (uint32_t)(mv - pp.lut_m0);
    const uint32_t li = dm >> pp.lut_shift;
    // the whole-disparity table (lut_shift 4) holds multiples of 16 only: any other median (a
    // sub-pixel map passed through these entry points) takes the exact path below
    if (li < (uint32_t)pp.lut_n && (dm & ((1u << pp.lut_shift) - 1u)) == 0) {   // table lookup (exact)
        PostVals o;
        o.a = at(pp.lut_a, li);
        o.u = at(pp.lut_u8, li);
        o.b = pp.mode == POST_SCALED ? at(pp.lut_b, li) : 0.0f;
        return o;
    }
    return post_vals(pp, (float)mv / 16.0f);
}

// Post-processing of an int16 x16 median map (the value OpenCV's fixed-point disparity holds
// after medianBlur, depth_map.py:909-912) into create_depth_map's outputs (depth_map.py:
// 915-936) or the scaled app's (fused_depth_map.py:1010-1024): the median kernel's epilogue
// as a pass of its own, for maps that crossed xGMI as 2 B/px (multi-GPU gathers).  8 pixels
// per thread: one 16-B load, 2 x 16-B f32 stores per output, one 8-B u8 store; table lookup
// as in the median epilogue (bit-identical).  Algorithmic bytes: 2 in + 9 out (DEPTH).
__global__ __launch_bounds__(256) void k_post_m16(const int16_t* __restrict__ in, long long n,
                                                  float* __restrict__ disp, PostParams pp) {
    const long long i0 = ((long long)blockIdx.x * 256 + threadIdx.x) * 8;
    if (i0 >= n) return;
    const bool vec = i0 + 8 <= n && ((((uintptr_t)in) & 15) | (((uintptr_t)disp | (uintptr_t)pp.out_a |
                                                                  (uintptr_t)pp.out_b) & 15) |
                                     ((uintptr_t)pp.out_u8 & 7)) == 0;
    if (vec) {
        const uint4 raw = *reinterpret_cast<const uint4*>(in + i0);
        const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
        int mv[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            mv[2 * q] = (int)(int16_t)(w[q] & 0xFFFFu);
            mv[2 * q + 1] = (int)(int16_t)(w[q] >> 16);
        }
        if (disp) {
            float4* d = reinterpret_cast<float4*>(disp + i0);
            d[0] = make_float4((float)mv[0] / 16.0f, (float)mv[1] / 16.0f, (float)mv[2] / 16.0f, (float)mv[3] / 16.0f);
            d[1] = make_float4((float)mv[4] / 16.0f, (float)mv[5] / 16.0f, (float)mv[6] / 16.0f, (float)mv[7] / 16.0f);
        }
        if (pp.mode == POST_NONE) return;
        PostVals o[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = post_median(pp, mv[q]);
        float4* a = reinterpret_cast<float4*>(pp.out_a + i0);
        a[0] = make_float4(o[0].a, o[1].a, o[2].a, o[3].a);
        a[1] = make_float4(o[4].a, o[5].a, o[6].a, o[7].a);
        uint32_t u[2] = {0u, 0u};
#pragma unroll
        for (int q = 0; q < 8; ++q) u[q >> 2] |= (uint32_t)o[q].u << (8 * (q & 3));
        *reinterpret_cast<uint2*>(pp.out_u8 + i0) = make_uint2(u[0], u[1]);
        if (pp.mode == POST_SCALED) {
            float4* b = reinterpret_cast<float4*>(pp.out_b + i0);
            b[0] = make_float4(o[0].b, o[1].b, o[2].b, o[3].b);
            b[1] = make_float4(o[4].b, o[5].b, o[6].b, o[7].b);
        }
        return;
    }
    for (long long i = i0; i < i0 + 8 && i < n; ++i) {
        const int mv = (int)in[i];
        if (disp) disp[i] = (float)mv / 16.0f;
        if (pp.mode == POST_NONE) continue;
        const PostVals o = post_median(pp, mv);
        pp.out_a[i] = o.a;
        pp.out_u8[i] = o.u;
        if (pp.mode == POST_SCALED) pp.out_b[i] = o.b;
    }
}

// HF: the Harris blocks this instance carries (0 none, 1 60-column waves, 2 248-column waves):
// the 248-column form needs 81 VGPRs, which would cost the plain median (36) its occupancy
template <int HF>
__global__ __launch_bounds__(256) void k_median_i16(const int16_t* __restrict__ in, int H, int W,
                                                    int row0, int row1, float* __restrict__ disp,
                                                    PostParams pp, long long fs_in, long long fs_out,
                                                    HarrisParams hp) {
    // Harris blocks (hp.g != nullptr): blockIdx.x >= hp.mbx; each wave one DPP band of 60
    // columns x 16 rows of the frame's left image (harris_wave, the k_harris_dpp form), so
    // C2's Harris response rides in the median launch instead of a launch of its own
    if (HF != 0 && (int)blockIdx.x >= hp.mbx) {
        const int w = (int)(blockIdx.x - hp.mbx) * 4 + (int)(threadIdx.x >> 6);
        const int y0 = row0 + (int)blockIdx.y * MQ_H;
        if constexpr (HF == 2) {   // 248 columns per wave, one dword per lane-row (W >= 256)
            const int x0 = w * 248;
            if (x0 < W && y0 < row1)
                harris_wave4<MQ_H, 4>(hp.g + blockIdx.z * hp.fs_in, H, W, hp.pitch, hp.out + blockIdx.z * hp.fs_out,
                                      x0, y0, threadIdx.x & 63);
        } else {
            const int x0 = w * 60;
            if (x0 < W && y0 < row1)
                harris_wave<MQ_H, 4>(hp.g + blockIdx.z * hp.fs_in, H, W, hp.pitch, hp.out + blockIdx.z * hp.fs_out,
                                     x0, y0, threadIdx.x & 63);
        }
        return;
    }
    // t2[r][c] = (tile row r, tile row r+2) of column x0-2+c; tile row r = image row y0-2+r
    constexpr int TC = MQ_W + 4, TR = MQ_H + 2;
    __shared__ uint32_t t2[TR][TC];
    // srt[g][i][c]: rank i of column c over the shared pair rows 4g+1..4g+4 of t2
    __shared__ __attribute__((aligned(8))) uint32_t srt[MQ_H / 4][4][TC];
    if (blockIdx.z) {   // frame batch
        in += blockIdx.z * fs_in;
        const long long o = blockIdx.z * fs_out;
        if (disp) disp += o;   // nullable (an int16-only median pass): keep it null
        if (pp.out_a) pp.out_a += o;
        if (pp.out_u8) pp.out_u8 += o;
        if (pp.out_b) pp.out_b += o;
        if (pp.out_bgr) pp.out_bgr += 3 * o;
        if (pp.out_m16) pp.out_m16 += o;
        if (pp.out_d8) pp.out_d8 += o;
    }
    const int x0 = blockIdx.x * MQ_W, y0 = row0 + blockIdx.y * MQ_H;
    {   // thread -> tile column t % 128 (clamped once), rows t / 128, +2, ...; the 4 columns
        // past 128 (72 entries) go to the first 72 threads
        const int c = (int)(threadIdx.x & (MQ_W - 1)), g = (int)(threadIdx.x / MQ_W);
        constexpr int G = 256 / MQ_W;
        static_assert(TR % G == 0, "row groups must tile the pair rows");
        const uint32_t cx = (uint32_t)clampi(x0 - 2 + c, 0, W - 1);
        if (y0 >= 2 && y0 + TR - 1 <= H - 1) {   // interior rows (uniform): no row clamps
            uint32_t off = (uint32_t)(y0 - 2 + g) * W + cx;
            const uint32_t two = 2u * (uint32_t)W, step = (uint32_t)G * W;
#pragma unroll
            for (int k = 0; k < TR / G; ++k) {
                const uint16_t a = (uint16_t)at(in, off);
                const uint16_t b = (uint16_t)at(in, off + two);
                t2[g + G * k][c] = (uint32_t)a | ((uint32_t)b << 16);
                off += step;
            }
        } else {
#pragma unroll
            for (int k = 0; k < TR / G; ++k) {
                const int r = g + G * k;
                const uint16_t a = (uint16_t)at(in, (uint32_t)clampi(y0 - 2 + r, 0, H - 1) * W + cx);
                const uint16_t b = (uint16_t)at(in, (uint32_t)clampi(y0 + r, 0, H - 1) * W + cx);
                t2[r][c] = (uint32_t)a | ((uint32_t)b << 16);
            }
        }
        if (threadIdx.x < 4 * TR) {
            const int r = (int)(threadIdx.x >> 2), ce = MQ_W + (int)(threadIdx.x & 3);
            const uint32_t cxe = (uint32_t)clampi(x0 - 2 + ce, 0, W - 1);
            const uint16_t a = (uint16_t)at(in, (uint32_t)clampi(y0 - 2 + r, 0, H - 1) * W + cxe);
            const uint16_t b = (uint16_t)at(in, (uint32_t)clampi(y0 + r, 0, H - 1) * W + cxe);
            t2[r][ce] = (uint32_t)a | ((uint32_t)b << 16);
        }
    }
    __syncthreads();
    // every thread computes (the tile is clamped, so columns/rows past the edge read valid
    // data); only in-range pixels are written, after the LDS transpose below.  Thread (tb, tx)
    // owns output columns tx, tx+1 (tile columns tx .. tx+5) of rows tb .. tb+3.
    const int tx = 2 * (int)(threadIdx.x & 63), tb = 4 * (int)(threadIdx.x >> 6);
    {   // sort each column of the 4 shared pair rows once (5 comparators); the 5 windows
        // that read a column share the sort.  The 4 columns past 128 of each row group go to
        // the first 16 lanes of wave 0
        auto sort_col = [&](int g4, int c) {
            s2 w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) w[i] = as_s2(t2[g4 + 1 + i][c]);
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const int a = SV_SORT4_NET[k][0], b = SV_SORT4_NET[k][1];
                const s2 lo = __builtin_elementwise_min(w[a], w[b]);
                w[b] = __builtin_elementwise_max(w[a], w[b]);
                w[a] = lo;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) srt[g4 >> 2][i][c] = __builtin_bit_cast(uint32_t, w[i]);
        };
        sort_col(tb, tx);
        sort_col(tb, tx + 1);
        if (threadIdx.x < 16) sort_col(4 * (threadIdx.x >> 2), MQ_W + (threadIdx.x & 3));
    }
    __syncthreads();

    // the two windows share tile columns tx+1 .. tx+4: SEL16H once (their sorted ranks 3..12),
    // then each window merges its own column (MRG14) -> the 6 candidates C of SEL20S
    s2 cm[16], own[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint2 p0 = *reinterpret_cast<const uint2*>(&srt[tb >> 2][i][tx]);
        const uint2 p1 = *reinterpret_cast<const uint2*>(&srt[tb >> 2][i][tx + 2]);
        const uint2 p2 = *reinterpret_cast<const uint2*>(&srt[tb >> 2][i][tx + 4]);
        own[0][i] = as_s2(p0.x);
        cm[0 * 4 + i] = as_s2(p0.y);
        cm[1 * 4 + i] = as_s2(p1.x);
        cm[2 * 4 + i] = as_s2(p1.y);
        cm[3 * 4 + i] = as_s2(p2.x);
        own[1][i] = as_s2(p2.y);
    }
#pragma unroll
    for (int c = 0; c < SV_SEL16H_NCMP; ++c) {
        const int a = SV_SEL16H_NET[c][0], b = SV_SEL16H_NET[c][1], use = SV_SEL16H_NET[c][2];
        const s2 lo = __builtin_elementwise_min(cm[a], cm[b]);
        const s2 hi = __builtin_elementwise_max(cm[a], cm[b]);
        if (use & 1) cm[a] = lo;
        if (use & 2) cm[b] = hi;
    }
    s2 cw[2][6];
#pragma unroll
    for (int w = 0; w < 2; ++w) {
        s2 z[14];
#pragma unroll
        for (int k = 0; k < 10; ++k) z[k] = cm[SV_SEL16H_OUT[k]];
#pragma unroll
        for (int k = 0; k < 4; ++k) z[10 + k] = own[w][k];
#pragma unroll
        for (int c = 0; c < SV_MRG14_NCMP; ++c) {
            const int a = SV_MRG14_NET[c][0], b = SV_MRG14_NET[c][1], use = SV_MRG14_NET[c][2];
            const s2 lo = __builtin_elementwise_min(z[a], z[b]);
            const s2 hi = __builtin_elementwise_max(z[a], z[b]);
            if (use & 1) z[a] = lo;
            if (use & 2) z[b] = hi;
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) cw[w][k] = z[SV_MRG14_OUT[k]];
    }
    // unique rows (tile rows tb, tb+5): the two windows share 4 of their 5 values, sorted once
    // (5 comparators), each inserts its own (4); median = 6th of (C: 6 sorted, U: 5 sorted)
    uint32_t mp[4];   // (column tx | column tx+1) of rows tb, tb+1, tb+2, tb+3
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        s2 q[6];
        {
            const uint2 p0 = *reinterpret_cast<const uint2*>(&t2[tb + 5 * h][tx]);
            const uint2 p1 = *reinterpret_cast<const uint2*>(&t2[tb + 5 * h][tx + 2]);
            const uint2 p2 = *reinterpret_cast<const uint2*>(&t2[tb + 5 * h][tx + 4]);
            q[0] = as_s2(p0.x); q[1] = as_s2(p0.y); q[2] = as_s2(p1.x);
            q[3] = as_s2(p1.y); q[4] = as_s2(p2.x); q[5] = as_s2(p2.y);
        }
        s2 sc[4] = {q[1], q[2], q[3], q[4]};
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const int a = SV_SORT4_NET[k][0], b = SV_SORT4_NET[k][1];
            const s2 lo = __builtin_elementwise_min(sc[a], sc[b]);
            sc[b] = __builtin_elementwise_max(sc[a], sc[b]);
            sc[a] = lo;
        }
        s2 m[2];
#pragma unroll
        for (int w = 0; w < 2; ++w) {
            s2 u[5] = {sc[0], sc[1], sc[2], sc[3], w ? q[5] : q[0]};
#pragma unroll
            for (int k = 3; k >= 0; --k) {   // insertion of u[4]
                const s2 lo = __builtin_elementwise_min(u[k], u[k + 1]);
                u[k + 1] = __builtin_elementwise_max(u[k], u[k + 1]);
                u[k] = lo;
            }
            s2 r = cw[w][5];
#pragma unroll
            for (int i = 0; i < 5; ++i) r = __builtin_elementwise_min(r, __builtin_elementwise_max(cw[w][i], u[4 - i]));
            m[w] = r;
        }
        // h = 0: (row tb, row tb+2), h = 1: (row tb+1, row tb+3); halves x = rows, w = columns
        const uint32_t a0 = __builtin_bit_cast(uint32_t, m[0]), a1 = __builtin_bit_cast(uint32_t, m[1]);
        mp[h] = (a0 & 0xFFFFu) | (a1 << 16);
        mp[h + 2] = (a0 >> 16) | (a1 & 0xFFFF0000u);
    }
    // park the medians in LDS, then re-read them as 4 consecutive columns of one row per
    // thread so the outputs leave as 16-byte (f32) and 4-byte (u8) stores.  med aliases srt
    // (every wave has read its ranks by the barrier): 17.9 KB of LDS, 8 blocks per CU
    static_assert(sizeof(srt) >= MQ_H * (MQ_W / 2) * sizeof(uint32_t), "med must fit in srt");
    auto med = reinterpret_cast<uint32_t (*)[MQ_W / 2]>(&srt[0][0][0]);
    __syncthreads();
    med[tb][tx >> 1] = mp[0];
    med[tb + 1][tx >> 1] = mp[1];
    med[tb + 2][tx >> 1] = mp[2];
    med[tb + 3][tx >> 1] = mp[3];
    __syncthreads();
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        const int r = (int)(threadIdx.x >> 5) + 8 * pass, c4 = (int)(threadIdx.x & 31) * 4;
        const int y = y0 + r, x = x0 + c4;
        if (y >= row1 || x >= W) continue;
        const uint2 raw = *reinterpret_cast<const uint2*>(&med[r][c4 >> 1]);
        const int mv[4] = {(int)(int16_t)(raw.x & 0xFFFF), (int)(int16_t)(raw.x >> 16),
                           (int)(int16_t)(raw.y & 0xFFFF), (int)(int16_t)(raw.y >> 16)};
        const uint32_t i = (uint32_t)y * W + x;
        const bool vec = x + 3 < W && (W & 3) == 0 &&
                         (((uintptr_t)disp | (uintptr_t)pp.out_a | (uintptr_t)pp.out_b) & 15) == 0 &&
                         (((uintptr_t)pp.out_u8 | (uintptr_t)pp.out_bgr | (uintptr_t)pp.out_d8) & 3) == 0 &&
                         ((uintptr_t)pp.out_m16 & 7) == 0;
        if (vec) {
            if (disp)
                at(reinterpret_cast<float4*>(disp), i >> 2) =
                    make_float4((float)mv[0] / 16.0f, (float)mv[1] / 16.0f, (float)mv[2] / 16.0f, (float)mv[3] / 16.0f);
            if (pp.out_m16) at(reinterpret_cast<uint2*>(pp.out_m16), i >> 2) = raw;
            if (pp.out_d8)
                at(reinterpret_cast<uint32_t*>(pp.out_d8), i >> 2) =
                    (uint32_t)(uint8_t)((mv[0] >> 4) - pp.d8_base) | ((uint32_t)(uint8_t)((mv[1] >> 4) - pp.d8_base) << 8) |
                    ((uint32_t)(uint8_t)((mv[2] >> 4) - pp.d8_base) << 16) |
                    ((uint32_t)(uint8_t)((mv[3] >> 4) - pp.d8_base) << 24);
            if (pp.mode == POST_NONE) continue;
            PostVals o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = post_median(pp, mv[q]);
            at(reinterpret_cast<float4*>(pp.out_a), i >> 2) = make_float4(o[0].a, o[1].a, o[2].a, o[3].a);
            at(reinterpret_cast<uint32_t*>(pp.out_u8), i >> 2) =
                (uint32_t)o[0].u | ((uint32_t)o[1].u << 8) | ((uint32_t)o[2].u << 16) | ((uint32_t)o[3].u << 24);
            if (pp.mode == POST_SCALED)
                at(reinterpret_cast<float4*>(pp.out_b), i >> 2) = make_float4(o[0].b, o[1].b, o[2].b, o[3].b);
            if (pp.out_bgr) {   // 4 pixels = 12 bytes = 3 dwords (byte offset 3i, i % 4 == 0)
                const uint32_t c0 = pp.cmap[o[0].u], c1 = pp.cmap[o[1].u], c2 = pp.cmap[o[2].u],
                               c3 = pp.cmap[o[3].u];
                uint32_t* d = &at(reinterpret_cast<uint32_t*>(pp.out_bgr), 3 * (i >> 2));
                d[0] = c0 | (c1 << 24);
                d[1] = (c1 >> 8) | (c2 << 16);
                d[2] = (c2 >> 16) | (c3 << 8);
            }
            continue;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (x + q >= W) break;
            if (disp) at(disp, i + q) = (float)mv[q] / 16.0f;
            if (pp.out_m16) at(pp.out_m16, i + q) = (int16_t)mv[q];
            if (pp.out_d8) at(pp.out_d8, i + q) = (uint8_t)((mv[q] >> 4) - pp.d8_base);
            if (pp.mode == POST_NONE) continue;
            const PostVals o = post_median(pp, mv[q]);
            at(pp.out_a, i + q) = o.a;
            at(pp.out_u8, i + q) = o.u;
            if (pp.mode == POST_SCALED) at(pp.out_b, i + q) = o.b;
            if (pp.out_bgr) {
                const uint32_t c = pp.cmap[o.u];
                uint8_t* d = &at(pp.out_bgr, 3 * (i + q));
                d[0] = (uint8_t)c;
                d[1] = (uint8_t)(c >> 8);
                d[2] = (uint8_t)(c >> 16);
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_median_f32(const float* __restrict__ in, int H, int W,
                                                    float* __restrict__ out) {
    __shared__ float tile[MT_H + 4][MT_W + 4];
    const int x0 = blockIdx.x * MT_W, y0 = blockIdx.y * MT_H;
    for (int i = threadIdx.x; i < (MT_H + 4) * (MT_W + 4); i += 256) {
        const int ty = i / (MT_W + 4), tx = i % (MT_W + 4);
        tile[ty][tx] = in[(size_t)clampi(y0 - 2 + ty, 0, H - 1) * W + clampi(x0 - 2 + tx, 0, W - 1)];
    }
    __syncthreads();
    const int tx = threadIdx.x % MT_W, pr = threadIdx.x / MT_W;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        float v[25];
#pragma unroll
        for (int j = 0; j < 5; ++j)
#pragma unroll
            for (int i = 0; i < 5; ++i) v[j * 5 + i] = tile[2 * pr + h + j][tx + i];
#pragma unroll
        for (int c = 0; c < SV_MED25_NCMP; ++c) {
            const int a = SV_MED25_NET[c][0], b = SV_MED25_NET[c][1], use = SV_MED25_NET[c][2];
            const float lo = fminf(v[a], v[b]), hi = fmaxf(v[a], v[b]);
            if (use & 1) v[a] = lo;
            if (use & 2) v[b] = hi;
        }
        const int x = x0 + tx, y = y0 + 2 * pr + h;
        if (x < W && y < H) out[(size_t)y * W + x] = v[SV_MED25_OUT];
    }
}

__global__ void k_post(const float* __restrict__ disp, int n, PostParams pp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) post_one(pp, (size_t)i, disp[i]);
}

__global__ void k_post_lut(PostParams pp, int m0, int n, int step) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) post_one(pp, (size_t)i, (float)(m0 + i * step) / 16.0f);
}

}  // namespace

int launch_gray(const uint8_t* bgr, int H, int W, int pitch, uint8_t* gray, hipStream_t s) {
    hipLaunchKernelGGL(k_gray, dim3((W + 255) / 256, H), dim3(256), 0, s, bgr, H, W, pitch, gray);
    return (int)hipGetLastError();
}

int launch_harris(const uint8_t* g, int H, int W, int pitch, float* out, hipStream_t s, int nf,
                  long long fs_in, long long fs_out) {
    if (nf <= 0) return 0;
    // SV_HARRIS=lds (A/B): the LDS-tile kernel everywhere; it also serves images under 8 px
    static const bool lds = [] {
        const char* e = std::getenv("SV_HARRIS");
        return e && e[0] == 'l';
    }();
    if (!lds && W >= 8 && H >= 8) {
        // 8 output rows per wave: C2 16.8 us per 16 VGA frames (16 rows: 17.7, 32: 21.0; 1080p
        // 99 / 98 / 105 us; the SV_HARRIS_HB A/B switch was removed in round 4)
        // SV_HARRIS=dpp1 (A/B): one column per lane everywhere
        static const bool one = [] {
            const char* e = std::getenv("SV_HARRIS");
            return e && std::strcmp(e, "dpp1") == 0;
        }();
        // 4 columns per lane from 1024 columns (1080p: 91.6 vs 98.6 us per 16 frames); narrower
        // frames keep 1 per lane (VGA: 16.7 vs 21.6 us — a quarter of the waves hides less latency)
        if (!one && W >= 1024) {
            hipLaunchKernelGGL((k_harris_dpp4<8, 4>), dim3((W + 247) / 248, (H + 7) / 8, nf), dim3(64), 0, s, g, H, W,
                               pitch, out, fs_in, fs_out);
            return (int)hipGetLastError();
        }
        hipLaunchKernelGGL((k_harris_dpp<8, 4>), dim3((W + 59) / 60, (H + 7) / 8, nf), dim3(64), 0, s, g, H, W, pitch,
                           out, fs_in, fs_out);
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(k_harris_lds, dim3((W + HX2 - 1) / HX2, (H + HY2 - 1) / HY2, nf), dim3(256), 0, s, g,
                       H, W, pitch, out, fs_in, fs_out);
    return (int)hipGetLastError();
}

// The column-run kernel over nz images (nz = 1: g0 / h0; else z = 2 * frame + side).
// SV_HOG_CR_ROWS: rows per strip wave (A/B; 24 by default: 4K, 4 images per launch, 16 / 24 /
// 32 / 48 rows measured 1,552 / 1,572 / 1,564 / 1,558 C5 HOG frames/s).
static int launch_hog_strips(const uint8_t* g0, const uint8_t* g1, int H, int W, int pitch, int r, int row0,
                             int row1, uint16_t* h0, uint16_t* h1, int nz, long long fs_in, long long fs_hist,
                             hipStream_t s) {
    static const int hc_rows = [] {
        const char* e = std::getenv("SV_HOG_CR_ROWS");
        const int x = e ? std::atoi(e) : 0;
        return x >= 4 && x <= 4096 ? x : HC_ROWS;
    }();
    switch (r) {
#define SV_HOG_C(R)                                                                                              \
    case R: {                                                                                                   \
        constexpr int NOUT = HogCr<R, HC_K>::NOUT;                                                              \
        const dim3 grid((W + NOUT - 1) / NOUT, (row1 - row0 + hc_rows - 1) / hc_rows, nz);                      \
        hipLaunchKernelGGL((k_hog_hist_cr<R, HC_K>), grid, dim3(64), 0, s, g0, H, W, pitch, row0, row1, h0,     \
                           hc_rows, g1, h1, fs_in, fs_hist);                                                    \
    } break;
        SV_HOG_C(0) SV_HOG_C(1) SV_HOG_C(2) SV_HOG_C(3) SV_HOG_C(4) SV_HOG_C(5) SV_HOG_C(6) SV_HOG_C(7)
#undef SV_HOG_C
    }
    return (int)hipGetLastError();
}

int launch_hog_hist(const uint8_t* g, int H, int W, int pitch, int win, int row0, int row1,
                    uint16_t* hist, hipStream_t s) {
    const int r = win / 2;
    if (r > GR_MAX) return (int)hipErrorInvalidValue;
    if (row0 < 0) row0 = 0;
    if (row1 > H) row1 = H;
    if (row1 <= row0) return 0;
    static const int strip = [] {
        const char* e = std::getenv("SV_HOG_STRIP");
        return e ? std::atoi(e) : 1;
    }();
    // (the strip kernels address through 32-bit buffer offsets, stores below 0x7FFFFFF0)
    if (strip && (long long)H * W * 20 < (1LL << 31) - (1LL << 20) && (long long)H * pitch < (1LL << 31)) {
        return launch_hog_strips(g, g, H, W, pitch, r, row0, row1, hist, hist, 1, 0, 0, s);
    }
    const dim3 grid((W + GT_W - 1) / GT_W, (row1 - row0 + GT_H - 1) / GT_H);
    switch (r) {
#define SV_HOG_R(R) case R: hipLaunchKernelGGL(k_hog_hist<R>, grid, dim3(256), 0, s, g, H, W, pitch, row0, row1, hist); break;
        SV_HOG_R(0) SV_HOG_R(1) SV_HOG_R(2) SV_HOG_R(3) SV_HOG_R(4) SV_HOG_R(5) SV_HOG_R(6) SV_HOG_R(7)
#undef SV_HOG_R
    }
    return (int)hipGetLastError();
}

int launch_hog_hist_pairs(const uint8_t* g0, const uint8_t* g1, int H, int W, int pitch, int win, int row0,
                          int row1, uint16_t* h0, uint16_t* h1, int nf, long long fs_in, long long fs_hist,
                          hipStream_t s) {
    const int r = win / 2;
    if (r > GR_MAX || nf <= 0) return (int)hipErrorInvalidValue;
    if (row0 < 0) row0 = 0;
    if (row1 > H) row1 = H;
    if (row1 <= row0) return 0;
    static const int strip = [] {
        const char* e = std::getenv("SV_HOG_STRIP");
        return e ? std::atoi(e) : 1;
    }();
    if (!(strip && (long long)H * W * 20 < (1LL << 31) - (1LL << 20) && (long long)H * pitch < (1LL << 31))) {
        for (int z = 0; z < nf; ++z) {   // the tile kernel: image by image
            int e = launch_hog_hist(g0 + z * fs_in, H, W, pitch, win, row0, row1, h0 + z * fs_hist, s);
            if (!e) e = launch_hog_hist(g1 + z * fs_in, H, W, pitch, win, row0, row1, h1 + z * fs_hist, s);
            if (e) return e;
        }
        return 0;
    }
    return launch_hog_strips(g0, g1, H, W, pitch, r, row0, row1, h0, h1, 2 * nf, fs_in, fs_hist, s);
}

int launch_median_i16(const int16_t* in, int H, int W, int row0, int row1, float* disp,
                      const PostParams& pp, hipStream_t s, int nf, long long fs_in, long long fs_out,
                      const HarrisParams* harris) {
    if (row1 <= row0 || nf <= 0) return 0;
    if ((long long)H * W >= (1LL << 30)) return (int)hipErrorInvalidValue;   // 32-bit offsets
    HarrisParams hp{};
    hp.mbx = (W + MQ_W - 1) / MQ_W;
    int hbx = 0;
    if (harris && harris->g) {   // Harris of rows [row0, row1): 4 waves of 60 (248) columns per block
        hp = *harris;
        hp.mbx = (W + MQ_W - 1) / MQ_W;
        // 248-column waves (k_harris_dpp4's form) from W >= 256: a quarter of the waves and one
        // dword load per lane-row where the band is interior (C2, 640x480 with 3 streams: 238k ->
        // 254-256k frames/s on one box).  SV_HARRIS_MED4=0 (A/B): 60-column waves everywhere
        static const bool med4 = [] {
            const char* e = std::getenv("SV_HARRIS_MED4");
            return !(e && e[0] == '0');
        }();
        hp.form = (med4 && W >= 256) ? 1 : 0;
        hbx = hp.form ? ((W + 247) / 248 + 3) / 4 : ((W + 59) / 60 + 3) / 4;
    }
    void (*fn)(const int16_t*, int, int, int, int, float*, PostParams, long long, long long, HarrisParams) =
        hbx == 0 ? k_median_i16<0> : hp.form ? k_median_i16<2> : k_median_i16<1>;
    hipLaunchKernelGGL(fn, dim3(hp.mbx + hbx, (row1 - row0 + MQ_H - 1) / MQ_H, nf),
                       dim3(256), 0, s, in, H, W, row0, row1, disp, pp, fs_in, fs_out, hp);
    return (int)hipGetLastError();
}

int launch_post_m16(const int16_t* in, long long n, float* disp, const PostParams& pp, hipStream_t s) {
    if (n <= 0) return 0;
    const long long blocks = (n + 8 * 256 - 1) / (8 * 256);
    if (blocks > 0x7FFFFFFFLL) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_post_m16, dim3((unsigned)blocks), dim3(256), 0, s, in, n, disp, pp);
    return (int)hipGetLastError();
}

int launch_median_f32(const float* in, int H, int W, float* out, hipStream_t s) {
    hipLaunchKernelGGL(k_median_f32, dim3((W + MT_W - 1) / MT_W, (H + MT_H - 1) / MT_H), dim3(256),
                       0, s, in, H, W, out);
    return (int)hipGetLastError();
}

int launch_post_lut(const PostParams& pp, int m0, int n, int step, float* lut_a, uint8_t* lut_u8,
                    float* lut_b, hipStream_t s) {
    if (n <= 0 || pp.mode == POST_NONE) return 0;
    PostParams q = pp;
    q.out_a = lut_a;
    q.out_u8 = lut_u8;
    q.out_b = lut_b;
    q.out_bgr = nullptr;
    q.out_m16 = nullptr;
    q.lut_n = 0;
    hipLaunchKernelGGL(k_post_lut, dim3((n + 255) / 256), dim3(256), 0, s, q, m0, n, step);
    return (int)hipGetLastError();
}

int launch_post(const float* disp, int n, const PostParams& pp, hipStream_t s) {
    if (n <= 0 || pp.mode == POST_NONE) return 0;
    hipLaunchKernelGGL(k_post, dim3((n + 255) / 256), dim3(256), 0, s, disp, n, pp);
    return (int)hipGetLastError();
}

}  // namespace sv
