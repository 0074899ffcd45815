// sv_stats.hip — reductions on either side of the disparity path.
//
//  * k_frame_stats   the image statistics behind detect_camera_occlusion
//                    (fused_depth_map.py:131-301, run every OCCLUSION_CHECK_INTERVAL frames on
//                    the rectified pair, :2515-2522): per 48x48 block the exact integer
//                    moments (sum, sum of squares) that np.std(block) is built from, and the
//                    256-bin histogram (cv2.calcHist) whose moments also give the global
//                    np.mean / np.std.  BGR input is converted to gray on the fly (cvtColor).
//  * k_select_hist   one pass of a radix select over float32 keys: the order statistics
//                    np.percentile interpolates between (calibrate_midas_to_stereo
//                    fused_depth_map.py:1169-1257, normalize_to_stereo_range :1503-1554),
//                    with the reference's boolean masks (x > 0, confidence > 0.7) applied
//                    as predicates, so the masked array is never materialised.
//  * k_affine_f32    the elementwise epilogues of those functions, in NumPy's precision
//                    (float32 ops in order, or float64 scale/offset then astype(float32)).
// All HBM-bound: one read of the image / map per pass.
#include "sv_internal.h"

namespace sv {
namespace {

constexpr int kTile = 48;   // compute_block_homogeneity block_size (fused_depth_map.py:185)

// Wave64 sum of a 32-bit value (xor butterfly through DPP/permute).
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// LDS histogram increment with wave aggregation: up to GROUPS distinct bins of the wave
// (flat image regions; the few high digits of a radix pass) are added by a leader lane
// with the bin's population, since same-address LDS atomics from many lanes serialise;
// the remaining lanes add 1 each.
template <int GROUPS>
__device__ __forceinline__ void hist_add(uint32_t* h, uint32_t bin) {
    unsigned long long rem = __ballot(1);
#pragma unroll
    for (int it = 0; it < GROUPS; ++it) {
        const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)bin, (int)__builtin_ctzll(rem));
        const unsigned long long grp = __ballot(bin == b0) & rem;
        if (__lane_id() == (unsigned)__builtin_ctzll(grp)) atomicAdd(&h[b0], (uint32_t)__builtin_popcountll(grp));
        if (bin == b0) return;
        rem &= ~grp;
    }
    atomicAdd(&h[bin], 1u);
}

// One wave per 48x48 tile, four tiles side by side per workgroup (grid.z = image).  The
// tile is 48 rows x 12 dword groups = 576 slots, 9 per lane, all loaded before any is
// used (one memory latency per tile); the tile moments are a wave reduction.  One LDS
// histogram copy per wave, merged into the image's global histogram at the end.
constexpr int kSlots = (kTile * kTile / 4 + 63) / 64;   // 9

__device__ __forceinline__ uint32_t gray_at(const uint8_t* p, int cn) {
    return cn == 3 ? (uint32_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13)) >> 14) : (uint32_t)p[0];
}

template <int AGG>
__global__ __launch_bounds__(256) void k_frame_stats(FrameStatsArgs a) {
    __shared__ uint32_t hist[4][256];
    const int z = blockIdx.z;
    const int f = a.per == 2 ? z >> 1 : z;
    const uint8_t* img = (a.per == 2 && (z & 1) ? a.img1 : a.img0) + f * a.fs;
    const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
    for (int i = t; i < 4 * 256; i += 256) (&hist[0][0])[i] = 0;
    __syncthreads();
    const int tx = blockIdx.x * 4 + wv, ty = blockIdx.y;
    const int x0 = tx * kTile, y0 = ty * kTile;
    if (x0 < a.W) {
        const int w = min(kTile, a.W - x0), h = min(kTile, a.H - y0);
        const int groups = (w + 3) >> 2;
        const bool fast = a.cn == 1 && w == kTile && ((a.pitch & 3) == 0) && ((((uintptr_t)img) & 3) == 0);
        uint32_t s = 0, q = 0;
        if (fast) {
            uint32_t d[kSlots];
#pragma unroll
            for (int k = 0; k < kSlots; ++k) {
                const int i = lane + 64 * k;
                const int r = i / 12, g = i - r * 12;
                d[k] = (i < 576 && r < h) ? *reinterpret_cast<const uint32_t*>(img + (size_t)(y0 + r) * a.pitch + x0 + 4 * g)
                                          : 0u;
            }
#pragma unroll
            for (int k = 0; k < kSlots; ++k) {
                const int i = lane + 64 * k;
                if (i < 576 && i / 12 < h) {
                    if (AGG == 2) {
                        // slot-level aggregation: a dword of 4 equal bytes adds 4 at once, and
                        // when every active lane holds the same such dword one lane adds the
                        // wave's total (flat regions: same-address LDS atomics serialise);
                        // other dwords add byte by byte
                        const uint32_t dk = d[k];
                        const bool same4 = ((dk ^ (dk >> 8)) & 0xFFFFFFu) == 0u;
                        const uint32_t b0 = dk & 0xffu;
                        if (same4) {
                            s += 4 * b0;
                            q += 4 * b0 * b0;
                            const unsigned long long act = __ballot(1);
                            const uint32_t lead = (uint32_t)__builtin_amdgcn_readfirstlane((int)dk);
                            const unsigned long long uni = __ballot(dk == lead) & act;
                            if (uni == act) {
                                if (__lane_id() == (unsigned)__builtin_ctzll(act))
                                    atomicAdd(&hist[wv][b0], 4u * (uint32_t)__builtin_popcountll(act));
                            } else {
                                atomicAdd(&hist[wv][b0], 4u);
                            }
                        } else {
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                const uint32_t v = (dk >> (8 * j)) & 0xff;
                                s += v;
                                q += v * v;
                                atomicAdd(&hist[wv][v], 1u);
                            }
                        }
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const uint32_t v = (d[k] >> (8 * j)) & 0xff;
                            s += v;
                            q += v * v;
                            hist_add<AGG>(hist[wv], v);
                        }
                    }
                }
            }
        } else {
            for (int i = lane; i < h * groups; i += 64) {
                const int r = i / groups, g = i - r * groups;
                const int n = min(4, w - 4 * g);
                const uint8_t* p = img + (size_t)(y0 + r) * a.pitch + (size_t)(x0 + 4 * g) * a.cn;
                for (int j = 0; j < n; ++j) {
                    const uint32_t v = gray_at(p + j * a.cn, a.cn);
                    s += v;
                    q += v * v;
                    hist_add<AGG == 2 ? 1 : AGG>(hist[wv], v);
                }
            }
        }
        s = wave_sum(s);
        q = wave_sum(q);
        if (lane == 0 && tx < a.bw && ty < a.bh) {   // a block of compute_block_homogeneity
            const int b = z * a.bh * a.bw + ty * a.bw + tx;
            a.block_sum[b] = s;
            a.block_sq[b] = q;
        }
    }
    __syncthreads();
    const uint32_t c = hist[0][t] + hist[1][t] + hist[2][t] + hist[3][t];
    const int copy = (blockIdx.y * gridDim.x + blockIdx.x) % kHistCopies;
    if (c) atomicAdd(&a.hist_copies[((size_t)copy * gridDim.z + z) * 256 + t], c);
}

// dst[i] = sum over copies of acc[c * stride + i]; the accumulators are left zeroed for
// the next call (no memset launch).
__global__ __launch_bounds__(256) void k_fold_u32(uint32_t* acc, int copies, size_t stride, int n, uint32_t* dst) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t v = 0;
    for (int k = 0; k < copies; ++k) {
        v += acc[(size_t)k * stride + i];
        acc[(size_t)k * stride + i] = 0;
    }
    dst[i] = v;
}

// Order-preserving map of float32 bits to uint32 (-0.0 folded onto +0.0, NaN excluded by
// the caller's predicate and counted separately).
__device__ __forceinline__ uint32_t f32_key(float f) {
    uint32_t u = __float_as_uint(f);
    if (u == 0x80000000u) u = 0;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Pass `shift` of the select: histogram of digit (key >> shift) & (nbins-1) over the
// selected elements whose key agrees with prefix[r] above the digit, for each rank r.
// Pass 0 (shift = 21, all prefixes empty) also counts selected elements and NaNs.
constexpr int kSelVec = 4;   // float4 loads per thread per iteration (16 elements)

// The pass's scalars, copied out of the kernel arguments once (the kernels never modify or
// take the address of their SelectArgs: a by-value argument indexed by blockIdx.y, or
// written to, is copied to scratch memory and every use becomes a scratch load).
struct SelPass {
    int mode, shift, bits, nranks, nb;
    float thr;
    uint32_t pre[kMaxRanks];
};

__device__ __forceinline__ void select_one(const SelPass& q, uint32_t* h, float v, float m, uint32_t& cnt,
                                           uint32_t& nan) {
    if (q.mode == SEL_MASK_GT && !(m > q.thr)) return;   // confidence > 0.7
    if (v != v) {                                         // NaN in the selection -> nan
        nan += q.mode != SEL_POSITIVE;
        return;
    }
    if (q.mode == SEL_POSITIVE && !(v > 0.f)) return;    // disparity > 0
    ++cnt;
    const uint32_t k = f32_key(v);
    const uint32_t d = (k >> q.shift) & (uint32_t)(q.nb - 1);
    const uint32_t hi = q.shift + q.bits >= 32 ? 0u : (k >> (q.shift + q.bits));
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)
        if (r < q.nranks && hi == q.pre[r]) hist_add<4>(h + r * q.nb, d);
}

// Pass `shift` of the select: histogram of digit (key >> shift) & (nbins-1) over the
// selected elements whose key agrees with prefix[r] above the digit, for each rank r.
// Pass 0 (shift = 21, all prefixes empty) also counts selected elements and NaNs.
// Each thread loads kSelVec float4s (and mask float4s) before using any of them.
__global__ __launch_bounds__(256) void k_select_hist(const SelectArgs a) {
    extern __shared__ uint32_t h[];   // [nranks][1 << bits]: sized per pass (occupancy)
    const int y = blockIdx.y;                   // array of a batch
    SelPass q;
    q.mode = a.mask_mode;
    q.shift = a.shift;
    q.bits = a.bits;
    q.nranks = a.nranks;
    q.nb = 1 << a.bits;
    q.thr = a.thr;
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r) q.pre[r] = a.prefix[y][r];
    const float* x = a.x + y * a.xstride;
    const float* mk = a.mask ? a.mask + y * a.mstride : nullptr;
    uint32_t* ghist = a.ghist + (size_t)y * kHistCopies * kMaxRanks * 2048;
    unsigned long long* counts = a.counts + (size_t)y * kCountSlots * 16;
    const size_t n = a.n;
    for (int i = threadIdx.x; i < q.nranks * q.nb; i += 256) h[i] = 0;
    __syncthreads();
    uint32_t cnt = 0, nan = 0;
    const bool use_mask = q.mode == SEL_MASK_GT;
    const bool vec = ((((uintptr_t)x) & 15) == 0) && (!use_mask || ((((uintptr_t)mk) & 15) == 0));
    const size_t n4 = vec ? n / 4 : 0;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const float4* m4 = reinterpret_cast<const float4*>(mk);
    const size_t step = (size_t)gridDim.x * 256 * kSelVec;
    for (size_t base = (size_t)blockIdx.x * 256 * kSelVec + threadIdx.x; base < n4; base += step) {
        float4 v[kSelVec], m[kSelVec];
#pragma unroll
        for (int k = 0; k < kSelVec; ++k) {
            const size_t j = base + (size_t)k * 256;
            const size_t jj = j < n4 ? j : n4 - 1;
            v[k] = x4[jj];
            m[k] = use_mask ? m4[jj] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < kSelVec; ++k) {
            if (base + (size_t)k * 256 < n4) {
                select_one(q, h, v[k].x, m[k].x, cnt, nan);
                select_one(q, h, v[k].y, m[k].y, cnt, nan);
                select_one(q, h, v[k].z, m[k].z, cnt, nan);
                select_one(q, h, v[k].w, m[k].w, cnt, nan);
            }
        }
    }
    // scalar elements: the tail after the float4s, or everything when unaligned
    for (size_t i = 4 * n4 + (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        select_one(q, h, x[i], use_mask ? mk[i] : 0.f, cnt, nan);
    __syncthreads();
    for (int r = 0; r < q.nranks; ++r)
        for (int i = threadIdx.x; i < q.nb; i += 256)
            if (h[r * q.nb + i]) atomicAdd(&ghist[((blockIdx.x % kHistCopies) * kMaxRanks + r) * 2048 + i], h[r * q.nb + i]);
    {   // one add per block, striped over slots (same-address atomics serialise at L2)
        __shared__ uint32_t part[2][4];
        cnt = wave_sum(cnt);
        nan = wave_sum(nan);
        if ((threadIdx.x & 63) == 0) {
            part[0][threadIdx.x >> 6] = cnt;
            part[1][threadIdx.x >> 6] = nan;
        }
        __syncthreads();
        if (threadIdx.x < 2) {
            const uint32_t* p = part[threadIdx.x];
            atomicAdd(&counts[(blockIdx.x % kCountSlots) * 16 + threadIdx.x],
                      (unsigned long long)p[0] + p[1] + p[2] + p[3]);
        }
    }
}

// hist_out = sum of the accumulator copies (nranks x 2048 bins, 8 blocks per rank), counts_out
// = sum of the count slots; every accumulator read is zeroed for the next pass.
__global__ __launch_bounds__(256) void k_select_fold(const SelectArgs a) {
    const int y = blockIdx.y;
    uint32_t* ghist = a.ghist + (size_t)y * kHistCopies * kMaxRanks * 2048;
    unsigned long long* counts = a.counts + (size_t)y * kCountSlots * 16;
    uint32_t* hist_out = a.hist_out + (size_t)y * kMaxRanks * 2048;
    unsigned long long* counts_out = a.counts_out + (size_t)y * 2;
    const int i = blockIdx.x * 256 + threadIdx.x;   // < nranks * 2048
    uint32_t v = 0;
    for (int k = 0; k < kHistCopies; ++k) {
        uint32_t* p = ghist + (size_t)k * kMaxRanks * 2048 + i;
        v += *p;
        *p = 0;
    }
    hist_out[i] = v;
    if (blockIdx.x == 0 && threadIdx.x < 2) {
        unsigned long long c = 0;
        for (int k = 0; k < kCountSlots; ++k) {
            c += counts[k * 16 + threadIdx.x];
            counts[k * 16 + threadIdx.x] = 0;
        }
        counts_out[threadIdx.x] = c;
    }
}

__global__ __launch_bounds__(256) void k_affine_f32(AffineArgs a) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += stride) {
        const float x = a.x[i];
        float y;
        if (a.mode == AFF_F32) {          // c + ((x - a) / b) * d, float32, in this order
            const float nrm = (x - a.fa) / a.fb;
            y = a.fc + nrm * a.fd;
        } else if (a.mode == AFF_F64) {   // astype(float32) of (float64(x) * s + o)
            y = (float)((double)x * a.ds + a.doff);
        } else {                          // np.full_like(x, c)
            y = a.fc;
        }
        a.out[i] = y;
    }
}

}  // namespace

int launch_frame_stats(const FrameStatsArgs& a, int nimg, hipStream_t s) {
    if (a.H <= 0 || a.W <= 0 || nimg <= 0) return 0;
    const int tiles_x = (a.W + kTile - 1) / kTile;
    dim3 grid((tiles_x + 3) / 4, (a.H + kTile - 1) / kTile, nimg);
    const size_t nh = (size_t)nimg * 256;
    // SV_STATS_AGG (A/B): 0 plain LDS atomics per byte, 1 a wave-aggregated add per byte,
    // 2 (default) slot-level aggregation of flat dwords / flat waves
    static const int agg = [] {
        const char* e = std::getenv("SV_STATS_AGG");
        const int v = e ? std::atoi(e) : 2;
        return v >= 0 && v <= 2 ? v : 2;
    }();
    if (agg == 2) hipLaunchKernelGGL(k_frame_stats<2>, grid, dim3(256), 0, s, a);
    else if (agg == 1) hipLaunchKernelGGL(k_frame_stats<1>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_frame_stats<0>, grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_fold_u32, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, s, a.hist_copies,
                       kHistCopies, nh, (int)nh, a.hist);
    return (int)hipGetLastError();
}

int launch_select_hist(const SelectArgs& a, hipStream_t s) {
    // 16 elements per thread: each block zeroes and merges a 2048-bin histogram per rank
    int blocks = (int)((a.n + 256 * 4 * kSelVec - 1) / (256 * 4 * kSelVec));
    if (blocks > 1024) blocks = 1024;
    const int narr = a.narr > 0 ? a.narr : 1;
    const size_t lds = (size_t)(a.nranks > 0 ? a.nranks : 1) * ((size_t)1 << a.bits) * sizeof(uint32_t);
    if (a.n > 0) hipLaunchKernelGGL(k_select_hist, dim3(blocks, narr), dim3(256), lds, s, a);
    // the fold runs for n = 0 too: it writes the (empty) result
    hipLaunchKernelGGL(k_select_fold, dim3(a.nranks * 8, narr), dim3(256), 0, s, a);
    return (int)hipGetLastError();
}

int launch_affine_f32(const AffineArgs& a, hipStream_t s) {
    if (a.n == 0) return 0;
    int blocks = (int)((a.n + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_affine_f32, dim3(blocks), dim3(256), 0, s, a);
    return (int)hipGetLastError();
}

}  // namespace sv
