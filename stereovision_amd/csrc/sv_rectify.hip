// sv_rectify.hip — the rectification stage in front of the disparity path (gfx950).
//
//  * k_undistort_map  cv2.initUndistortRectifyMap(K, dist, R, P, size, CV_16SC2)
//                     (depth_map.py:636-641, fused_depth_map.py:402-407): per output pixel,
//                     f64 ray through inv(P[:, :3] R), Brown-Conrady distortion, 1/32-pixel
//                     fixed point.  One-time setup; computed in f64 exactly as the oracle
//                     (oracle/sv_rectify_oracle.py) with -ffp-contract=off.
//  * k_remap          cv2.remap(img, map1, map2, INTER_LINEAR) with BORDER_CONSTANT 0
//                     (depth_map.py:815-826, fused_depth_map.py:480-491), u8 gray or BGR,
//                     optionally fused with cvtColor(BGR2GRAY) so the rectified gray image
//                     the matcher reads is written directly (rectify -> gray in one pass).
//
// k_remap is HBM-bound: per output pixel it reads the 6-byte map entry once, 4 source taps
// (mostly L2 hits: neighbouring output pixels read neighbouring source pixels) and writes
// 1 (gray) or 3 (BGR) bytes.  Each lane owns 4 consecutive output pixels of a row so the
// map and output accesses are 16/8/4-byte vectors; the 2x2 taps of one source row come
// from dword loads + v_alignbyte (the unaligned 2- or 6-byte span) instead of byte loads.
#include "sv_internal.h"
#include "sv_xcd.h"

#include <cstdlib>

namespace sv {
namespace {

__device__ __forceinline__ int cv_round_i32(double v) {
    // saturate_cast<int>(double) on x86: round half to even; NaN / out of range -> INT_MIN
    if (!(v > -2147483648.5 && v < 2147483647.5)) return (int)0x80000000u;
    return (int)__builtin_rint(v);
}

__global__ void k_undistort_map(UndistortParams p, short2* __restrict__ map1,
                                uint16_t* __restrict__ map2) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    if (j >= p.W) return;
    const double* ir = p.ir;
    const double di = (double)i, dj = (double)j;
    const double _x = (di * ir[1] + ir[2]) + dj * ir[0];
    const double _y = (di * ir[4] + ir[5]) + dj * ir[3];
    const double _w = (di * ir[7] + ir[8]) + dj * ir[6];
    const double w = 1.0 / _w, x = _x * w, y = _y * w;
    const double x2 = x * x, y2 = y * y;
    const double r2 = x2 + y2, _2xy = 2 * x * y;
    const double* k = p.k;   // k1 k2 p1 p2 k3 k4 k5 k6 s1 s2 s3 s4
    const double kr = (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2) / (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2);
    const double xd = x * kr + k[2] * _2xy + k[3] * (r2 + 2 * x2) + k[8] * r2 + k[9] * r2 * r2;
    const double yd = y * kr + k[2] * (r2 + 2 * y2) + k[3] * _2xy + k[10] * r2 + k[11] * r2 * r2;
    const double u = p.fx * xd + p.u0;
    const double v = p.fy * yd + p.v0;
    const int iu = cv_round_i32(u * 32.0);
    const int iv = cv_round_i32(v * 32.0);
    const size_t o = (size_t)i * p.W + j;
    map1[o] = make_short2((short)(iu >> 5), (short)(iv >> 5));
    map2[o] = (uint16_t)((iv & 31) * 32 + (iu & 31));
}

struct RemapArgs {
    const uint8_t* src;
    int sH, sW, spitch;
    const short2* map1;
    const uint16_t* map2;     // may be null: integer maps (fraction 0)
    int H, W;                 // output (= map) size; maps are dense H x W
    uint8_t* dst;
    int dpitch;
    long long sfs, dfs;       // frame strides (bytes) for grid.z batches
    size_t src_bytes;         // bytes of one source frame: (sH-1)*spitch + sW*CN
    bool aligned;             // source frames start on a dword: dword-span fast path allowed
    bool vec;                 // W % 4 == 0 and 16/8-byte aligned maps: vector map loads
    bool xcd_map;             // XCD-aware row order (sv_xcd.h); off (see launch_remap)
};

// Bytes [p, p+n) of a row as a little-endian 64-bit value, from dword loads (n <= 6 needs
// 3 dwords when p & 3 == 3).  Caller guarantees the aligned span is inside the frame.
template <int CN>
__device__ __forceinline__ uint64_t load_span(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p & ~(uintptr_t)3;
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a);
    const uint32_t w0 = q[0], w1 = q[1];
    const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
    if (CN == 1) return lo;
    const uint32_t hi = __builtin_amdgcn_alignbyte(q[2], w1, sh);
    return ((uint64_t)hi << 32) | lo;
}

template <int CN, bool GRAY>
__global__ __launch_bounds__(256) void k_remap(RemapArgs a) {
    // XCD-aware row order (sv_xcd.h): the bilinear taps of rows y and y+1 share source rows
    int bx, by, bz;
    xcd_tile(a.xcd_map != 0, bx, by, bz);
    const int x0 = (bx * blockDim.x + threadIdx.x) * 4;
    const int y = by;
    if (x0 >= a.W) return;
    const int z = bz;
    const uint8_t* src = a.src + z * a.sfs;
    uint8_t* drow = a.dst + z * a.dfs + (size_t)y * a.dpitch;
    const size_t mrow = (size_t)y * a.W;
    const int n = min(4, a.W - x0);

    short2 m1[4];
    uint16_t m2[4] = {0, 0, 0, 0};
    if (n == 4 && a.vec) {
        const int4 v = *reinterpret_cast<const int4*>(a.map1 + mrow + x0);
        m1[0] = *reinterpret_cast<const short2*>(&v.x);
        m1[1] = *reinterpret_cast<const short2*>(&v.y);
        m1[2] = *reinterpret_cast<const short2*>(&v.z);
        m1[3] = *reinterpret_cast<const short2*>(&v.w);
        if (a.map2) {
            const uint2 f = *reinterpret_cast<const uint2*>(a.map2 + mrow + x0);
            m2[0] = (uint16_t)(f.x & 0xffff);
            m2[1] = (uint16_t)(f.x >> 16);
            m2[2] = (uint16_t)(f.y & 0xffff);
            m2[3] = (uint16_t)(f.y >> 16);
        }
    } else {
        for (int k = 0; k < 4; ++k) {
            m1[k] = k < n ? a.map1[mrow + x0 + k] : make_short2(0, 0);
            if (a.map2 && k < n) m2[k] = a.map2[mrow + x0 + k];
        }
    }

    uint32_t outv[CN == 3 && !GRAY ? 3 : 1] = {};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int sx = m1[k].x, sy = m1[k].y;
        const int f = m2[k] & 1023;
        const int fx = f & 31, fy = f >> 5;
        const int w00 = (32 - fy) * (32 - fx), w01 = (32 - fy) * fx, w10 = fy * (32 - fx), w11 = fy * fx;
        int acc[CN];
        const bool inner = (unsigned)sx < (unsigned)(a.sW - 1) && (unsigned)sy < (unsigned)(a.sH - 1);
        const size_t off0 = (size_t)sy * a.spitch + (size_t)sx * CN;
        const size_t off1 = off0 + a.spitch;
        // the aligned span of the second row must stay inside the frame
        const bool fast = a.aligned && inner && (((off1 & ~(size_t)3) + (CN == 1 ? 8 : 12)) <= a.src_bytes);
        if (fast) {
            const uint64_t r0 = load_span<CN>(src + off0);
            const uint64_t r1 = load_span<CN>(src + off1);
#pragma unroll
            for (int c = 0; c < CN; ++c) {
                const int v00 = (int)((r0 >> (8 * c)) & 0xff), v01 = (int)((r0 >> (8 * (c + CN))) & 0xff);
                const int v10 = (int)((r1 >> (8 * c)) & 0xff), v11 = (int)((r1 >> (8 * (c + CN))) & 0xff);
                acc[c] = v00 * w00 + v01 * w01 + v10 * w10 + v11 * w11;
            }
        } else {
            const bool okx0 = (unsigned)sx < (unsigned)a.sW, okx1 = (unsigned)(sx + 1) < (unsigned)a.sW;
            const bool oky0 = (unsigned)sy < (unsigned)a.sH, oky1 = (unsigned)(sy + 1) < (unsigned)a.sH;
            const uint8_t* p0 = src + (size_t)sy * a.spitch + (size_t)sx * CN;
            const uint8_t* p1 = p0 + a.spitch;
#pragma unroll
            for (int c = 0; c < CN; ++c) {
                const int v00 = (okx0 && oky0) ? p0[c] : 0, v01 = (okx1 && oky0) ? p0[c + CN] : 0;
                const int v10 = (okx0 && oky1) ? p1[c] : 0, v11 = (okx1 && oky1) ? p1[c + CN] : 0;
                acc[c] = v00 * w00 + v01 * w01 + v10 * w10 + v11 * w11;
            }
        }
        if (k >= n) continue;
        if (CN == 1) {
            outv[0] |= (uint32_t)((acc[0] + 512) >> 10) << (8 * k);
        } else if (GRAY) {
            const int b = (acc[0] + 512) >> 10, g = (acc[1] + 512) >> 10, r = (acc[2] + 512) >> 10;
            const int gy = (b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14;
            outv[0] |= (uint32_t)gy << (8 * k);
        } else {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int byte = 3 * k + c;
                outv[byte >> 2] |= (uint32_t)((acc[c] + 512) >> 10) << (8 * (byte & 3));
            }
        }
    }
    constexpr int OB = (CN == 3 && !GRAY) ? 3 : 1;   // output bytes per pixel
    uint8_t* d = drow + (size_t)x0 * OB;
    if (n == 4 && (((uintptr_t)d & 3) == 0)) {
        uint32_t* d32 = reinterpret_cast<uint32_t*>(d);
#pragma unroll
        for (int q = 0; q < OB; ++q) d32[q] = outv[q];
    } else {
        for (int b = 0; b < n * OB; ++b) d[b] = (uint8_t)(outv[b >> 2] >> (8 * (b & 3)));
    }
}


// cv2.resize(src, (dW, dH), interpolation=INTER_LINEAR) for u8 (fused_depth_map.py:474-476,
// :2498-2507, depth_map.py:757-776, ensure_same_size): OpenCV's fixed-point two-pass
// bilinear (INTER_RESIZE_COEF_BITS = 11), coordinates from the f32 source position
// (dx + 0.5) * scale - 0.5, x clamped with a zero fraction at the borders, rows clamped
// to the image; the vertical pass rounds as the scalar FixedPtCast<int, uchar, 22>.
// An exact 2x downscale takes OpenCV's INTER_AREA fast path (2x2 mean, +2 >> 2).
struct ResizeArgs {
    const void* src;
    int sH, sW, spitch, cn;   // pitches in bytes
    void* dst;
    int dH, dW, dpitch;
    double scale_x, scale_y;
    long long sfs, dfs;       // frame strides in bytes
    int area2;
};

__device__ __forceinline__ void resize_coord(int d, double scale, int n, bool clamp_frac, int& s0,
                                             int& s1, float& f) {
    f = (float)((d + 0.5) * scale - 0.5);
    int s = (int)floorf(f);
    f -= (float)s;
    if (clamp_frac) {   // x: OpenCV clamps the column and zeroes the fraction
        if (s < 0) f = 0.f, s = 0;
        if (s >= n - 1) f = 0.f, s = n - 1;
    }
    s0 = min(max(s, 0), n - 1);
    s1 = min(max(s + 1, 0), n - 1);
}

// T = uint8_t: fixed point (2^11 coefficients, (h0 b0 + h1 b1 + 2^21) >> 22);
// T = float: OpenCV's float path, S0*b0 + S1*b1 in f32 without contraction.
template <typename T>
__global__ __launch_bounds__(256) void k_resize_linear(ResizeArgs a) {
    const int dx = blockIdx.x * blockDim.x + threadIdx.x;
    const int dy = blockIdx.y;
    if (dx >= a.dW) return;
    const uint8_t* src = static_cast<const uint8_t*>(a.src) + blockIdx.z * a.sfs;
    T* d = reinterpret_cast<T*>(static_cast<uint8_t*>(a.dst) + blockIdx.z * a.dfs + (size_t)dy * a.dpitch) +
           (size_t)dx * a.cn;
    if (a.area2) {
        const T* p = reinterpret_cast<const T*>(src + (size_t)(2 * dy) * a.spitch) + (size_t)(2 * dx) * a.cn;
        const T* p1 = reinterpret_cast<const T*>(reinterpret_cast<const uint8_t*>(p) + a.spitch);
        for (int c = 0; c < a.cn; ++c) {
            if constexpr (sizeof(T) == 1)
                d[c] = (T)((p[c] + p[c + a.cn] + p1[c] + p1[c + a.cn] + 2) >> 2);
            else
                d[c] = (((p[c] + p[c + a.cn]) + p1[c]) + p1[c + a.cn]) * 0.25f;
        }
        return;
    }
    int x0, x1, y0, y1;
    float fx, fy;
    resize_coord(dx, a.scale_x, a.sW, true, x0, x1, fx);
    resize_coord(dy, a.scale_y, a.sH, false, y0, y1, fy);
    const T* r0 = reinterpret_cast<const T*>(src + (size_t)y0 * a.spitch);
    const T* r1 = reinterpret_cast<const T*>(src + (size_t)y1 * a.spitch);
    if constexpr (sizeof(T) == 1) {
        const int ax0 = (int)__builtin_rintf((1.f - fx) * 2048.f), ax1 = (int)__builtin_rintf(fx * 2048.f);
        const int by0 = (int)__builtin_rintf((1.f - fy) * 2048.f), by1 = (int)__builtin_rintf(fy * 2048.f);
        for (int c = 0; c < a.cn; ++c) {
            const int h0 = r0[x0 * a.cn + c] * ax0 + r0[x1 * a.cn + c] * ax1;
            const int h1 = r1[x0 * a.cn + c] * ax0 + r1[x1 * a.cn + c] * ax1;
            const int v = (h0 * by0 + h1 * by1 + (1 << 21)) >> 22;
            d[c] = (T)min(max(v, 0), 255);
        }
    } else {
        const float ax0 = 1.f - fx, ax1 = fx, by0 = 1.f - fy, by1 = fy;
        for (int c = 0; c < a.cn; ++c) {
            const float h0 = r0[x0 * a.cn + c] * ax0 + r0[x1 * a.cn + c] * ax1;
            const float h1 = r1[x0 * a.cn + c] * ax0 + r1[x1 * a.cn + c] * ax1;
            d[c] = h0 * by0 + h1 * by1;
        }
    }
}

}  // namespace

int launch_resize_linear(const void* src, int sH, int sW, int cn, int spitch, long long sfs, void* dst,
                         int dH, int dW, int dpitch, long long dfs, int nf, bool f32, hipStream_t s) {
    if (dH <= 0 || dW <= 0 || nf <= 0) return 0;
    ResizeArgs a;
    a.src = src;
    a.sH = sH;
    a.sW = sW;
    a.spitch = spitch;
    a.cn = cn;
    a.dst = dst;
    a.dH = dH;
    a.dW = dW;
    a.dpitch = dpitch;
    a.sfs = sfs;
    a.dfs = dfs;
    const double inv_x = (double)dW / sW, inv_y = (double)dH / sH;
    a.scale_x = 1. / inv_x;
    a.scale_y = 1. / inv_y;
    a.area2 = (a.scale_x == 2.0 && a.scale_y == 2.0) ? 1 : 0;
    dim3 grid((dW + 255) / 256, dH, nf);
    if (f32)
        hipLaunchKernelGGL(k_resize_linear<float>, grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_resize_linear<uint8_t>, grid, dim3(256), 0, s, a);
    return (int)hipGetLastError();
}

int launch_undistort_map(const UndistortParams& p, short2* map1, uint16_t* map2, hipStream_t s) {
    if (p.H <= 0 || p.W <= 0) return 0;
    dim3 grid((p.W + 255) / 256, p.H);
    hipLaunchKernelGGL(k_undistort_map, grid, dim3(256), 0, s, p, map1, map2);
    return (int)hipGetLastError();
}

int launch_remap(const uint8_t* src, int sH, int sW, int channels, int spitch, long long sfs,
                 const short2* map1, const uint16_t* map2, int H, int W, bool gray_out, uint8_t* dst,
                 int dpitch, long long dfs, int nf, hipStream_t s) {
    if (H <= 0 || W <= 0 || nf <= 0) return 0;
    RemapArgs a;
    a.src = src;
    a.sH = sH;
    a.sW = sW;
    a.spitch = spitch;
    a.map1 = map1;
    a.map2 = map2;
    a.H = H;
    a.W = W;
    a.dst = dst;
    a.dpitch = dpitch;
    a.sfs = sfs;
    a.dfs = dfs;
    a.src_bytes = (size_t)(sH - 1) * spitch + (size_t)sW * channels;
    a.aligned = (((uintptr_t)src | (uintptr_t)sfs) & 3) == 0;
    a.vec = (W & 3) == 0 && ((uintptr_t)map1 & 15) == 0 && ((uintptr_t)map2 & 7) == 0;
    // plain dispatch order: an XCD-aware row order measured 82-83 vs 85 us per 16-frame
    // BGR->gray batch alone but 51.4 vs 49.0 us per 8-frame batch inside the two-camera
    // pipeline (round 3, gpurun_out/remap1), so it was dropped
    a.xcd_map = false;
    dim3 grid((W + 4 * 256 - 1) / (4 * 256), H, nf);
    if (channels == 1)
        hipLaunchKernelGGL((k_remap<1, false>), grid, dim3(256), 0, s, a);
    else if (gray_out)
        hipLaunchKernelGGL((k_remap<3, true>), grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((k_remap<3, false>), grid, dim3(256), 0, s, a);
    return (int)hipGetLastError();
}

}  // namespace sv
