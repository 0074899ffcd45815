// sv_capi_dev.cpp — the single-device entry points of the C ABI (include/stereovision_amd.h):
// device-memory entry points (frames resident in HBM), host-buffer entry points (the
// drop-ins' path: NumPy frames in and out), rectification, reductions and SGBM-3WAY.
#include "sv_ctx.h"

extern "C" {

// ---------------------------------------------------------------- device entry points
int sv_gray_dev(sv_ctx* c, const uint8_t* d_bgr, int H, int W, int pitch, uint8_t* d_gray, void* stream) {
    SV_ENTER(c);
    if (check_image(d_bgr, H, W) || !d_gray) return fail(SV_EINVAL, "bad gray arguments");
    hipStream_t s = pick(c, stream);
    SV_LAUNCH(c, SV_K_GRAY, s, sv::launch_gray(d_bgr, H, W, pitch, d_gray, s));
    return 0;
}

int sv_disparity_dev(sv_ctx* c, const uint8_t* d_left, const uint8_t* d_right, int H, int W, int pitch,
                     int min_disp, int num_disp, int win, int cost, int row0, int row1, int16_t* d_disp16,
                     int out_pitch, void* stream) {
    SV_ENTER(c);
    if (check_image(d_left, H, W) || check_image(d_right, H, W) || !d_disp16)
        return fail(SV_EINVAL, "bad disparity arguments");
    if (pitch < W || out_pitch < W) return fail(SV_EINVAL, "pitch smaller than width");
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    return enqueue_disparity(c, d_left, d_right, H, W, pitch, min_disp, num_disp, win, cost, row0, row1,
                             d_disp16, out_pitch, s);
}

int sv_median_rows_dev(sv_ctx* c, const int16_t* d_disp16, int H, int W, int row0, int row1, int min_disp,
                       int num_disp, int cost, const sv_map_out* out, void* stream) {
    SV_ENTER(c);
    if (check_image(d_disp16, H, W)) return fail(SV_EINVAL, "bad median arguments");
    if ((long long)H * W >= (1LL << 30)) return fail(SV_EINVAL, "frame too large for the median kernel");
    if (row0 < 0) row0 = 0;
    if (row1 > H) row1 = H;
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    sv::PostParams pp;
    float* disp = nullptr;
    int rc = map_out_post(c, out, min_disp, num_disp, cost, false, s, &pp, &disp);
    if (rc) return rc;
    SV_LAUNCH(c, SV_K_MEDIAN, s, sv::launch_median_i16(d_disp16, H, W, row0, row1, disp, pp, s));
    return 0;
}

int sv_post_m16_dev(sv_ctx* c, const int16_t* d_med16, int64_t n, int mode, float min_depth, float max_depth,
                    float depth_range, float min_disp_global, int min_disp, int num_disp, float* d_disparity,
                    float* d_out_a, uint8_t* d_out_u8, float* d_out_b, void* stream) {
    SV_ENTER(c);
    if (n < 0 || (n > 0 && !d_med16)) return fail(SV_EINVAL, "bad median map");
    if (mode != SV_POST_NONE && mode != SV_POST_DEPTH && mode != SV_POST_SCALED) return fail(SV_EINVAL, "bad mode");
    if (mode == SV_POST_NONE && !d_disparity) return fail(SV_EINVAL, "no outputs");
    if (mode == SV_POST_DEPTH && (!d_out_a || !d_out_u8)) return fail(SV_EINVAL, "depth post outputs missing");
    if (mode == SV_POST_SCALED && (!d_out_a || !d_out_u8 || !d_out_b || num_disp <= 0))
        return fail(SV_EINVAL, "scaled post outputs missing");
    if (n == 0) return 0;
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    sv::PostParams pp = make_post(mode, min_depth, max_depth, depth_range, min_disp_global, min_disp, num_disp,
                                  d_out_a, d_out_u8, d_out_b);
    int rc = attach_lut(c, pp, s);
    if (rc) return rc;
    SV_LAUNCH(c, SV_K_POST, s, sv::launch_post_m16(d_med16, (long long)n, d_disparity, pp, s));
    return 0;
}

int sv_disparity_batch_dev(sv_ctx* c, const uint8_t* d_left, const uint8_t* d_right, int n_frames, int H,
                           int W, int pitch, int64_t frame_stride, int min_disp, int num_disp, int win,
                           int cost, int16_t* d_disp16, int out_pitch, int64_t out_frame_stride,
                           void* stream) {
    SV_ENTER(c);
    if (check_image(d_left, H, W) || check_image(d_right, H, W) || !d_disp16 || n_frames < 0)
        return fail(SV_EINVAL, "bad disparity arguments");
    if (pitch < W || out_pitch < W) return fail(SV_EINVAL, "pitch smaller than width");
    if (n_frames > 1 && (frame_stride < (int64_t)pitch * H || out_frame_stride < (int64_t)out_pitch * H))
        return fail(SV_EINVAL, "frame stride smaller than a frame");
    if (n_frames == 0) return 0;
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    return enqueue_disparity(c, d_left, d_right, H, W, pitch, min_disp, num_disp, win, cost, 0, H, d_disp16,
                             out_pitch, s, n_frames, frame_stride, out_frame_stride);
}

int sv_depth_map_batch_dev(sv_ctx* c, const uint8_t* d_left, const uint8_t* d_right, int n_frames, int H, int W,
                           int pitch, int64_t frame_stride, int min_disp, int num_disp, int win, int cost, int stages,
                           int16_t* d_disp16, const sv_map_out* out, void* stream) {
    SV_ENTER(c);
    if (stages != SV_STAGE_ALL && stages != SV_STAGE_MATCH && stages != SV_STAGE_MEDIAN)
        return fail(SV_EINVAL, "stages must be SV_STAGE_MATCH, SV_STAGE_MEDIAN or SV_STAGE_ALL");
    const bool match = stages & SV_STAGE_MATCH, median = stages & SV_STAGE_MEDIAN;
    if (n_frames < 0 || H <= 0 || W <= 0) return fail(SV_EINVAL, "bad depth-map arguments");
    if (match && (check_image(d_left, H, W) || check_image(d_right, H, W)))
        return fail(SV_EINVAL, "bad depth-map arguments");
    if (!d_disp16 && stages != SV_STAGE_ALL)
        return fail(SV_EINVAL, "the stages run apart exchange the int16 maps through d_disp16");
    if (median && !out) return fail(SV_EINVAL, "null outputs");
    if (median && out->harris && check_image(d_left, H, W)) return fail(SV_EINVAL, "Harris needs the left frames");
    if (pitch < W) return fail(SV_EINVAL, "pitch smaller than width");
    if (n_frames > 1 && frame_stride < (int64_t)pitch * H) return fail(SV_EINVAL, "frame stride smaller than a frame");
    if ((long long)H * W >= (1LL << 30)) return fail(SV_EINVAL, "frame too large for the median kernel");
    if (n_frames == 0) return 0;
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    const long long fs = (long long)H * W;
    int16_t* d16 = d_disp16;
    if (!d16) {
        SV_HIP(c->d16.ensure((size_t)n_frames * fs * sizeof(int16_t)));
        d16 = c->d16.as<int16_t>();
    }
    if (match) {
        const int rc = enqueue_disparity(c, d_left, d_right, H, W, pitch, min_disp, num_disp, win, cost, 0, H, d16, W,
                                         s, n_frames, frame_stride, fs);
        if (rc) return rc;
    }
    if (!median) return 0;
    sv::PostParams pp;
    float* disp = nullptr;
    int rc = map_out_post(c, out, min_disp, num_disp, cost, true, s, &pp, &disp);
    if (rc) return rc;
    const long long fin = n_frames > 1 ? frame_stride : 0;
    if (out->harris && (W < 8 || H < 8)) {   // the DPP form needs 8 px a side: a launch of its own
        SV_LAUNCH(c, SV_K_MEDIAN, s, sv::launch_median_i16(d16, H, W, 0, H, disp, pp, s, n_frames, fs, fs));
        SV_LAUNCH(c, SV_K_HARRIS, s, sv::launch_harris(d_left, H, W, pitch, out->harris, s, n_frames, fin, fs));
        return 0;
    }
    // the Harris response rides in the median launch (extra blocks)
    sv::HarrisParams hp{d_left, pitch, fin, out->harris, fs, 0, 0};
    SV_LAUNCH(c, SV_K_MEDIAN, s,
              sv::launch_median_i16(d16, H, W, 0, H, disp, pp, s, n_frames, fs, fs, out->harris ? &hp : nullptr));
    return 0;
}

int sv_harris_dev(sv_ctx* c, const uint8_t* d_gray, int H, int W, int pitch, float* d_out, void* stream) {
    SV_ENTER(c);
    if (check_image(d_gray, H, W) || !d_out) return fail(SV_EINVAL, "bad harris arguments");
    hipStream_t s = pick(c, stream);
    SV_LAUNCH(c, SV_K_HARRIS, s, sv::launch_harris(d_gray, H, W, pitch, d_out, s));
    return 0;
}

int sv_harris_batch_dev(sv_ctx* c, const uint8_t* d_gray, int n_frames, int H, int W, int pitch,
                        int64_t frame_stride, float* d_out, void* stream) {
    SV_ENTER(c);
    if (check_image(d_gray, H, W) || !d_out || n_frames < 0) return fail(SV_EINVAL, "bad harris arguments");
    if (pitch < W) return fail(SV_EINVAL, "pitch smaller than width");
    if (n_frames > 1 && frame_stride < (int64_t)pitch * H) return fail(SV_EINVAL, "frame stride smaller than a frame");
    if (n_frames == 0) return 0;
    hipStream_t s = pick(c, stream);
    SV_LAUNCH(c, SV_K_HARRIS, s,
              sv::launch_harris(d_gray, H, W, pitch, d_out, s, n_frames, (long long)frame_stride,
                                (long long)H * W));
    return 0;
}

int sv_hog_hist_dev(sv_ctx* c, const uint8_t* d_gray, int H, int W, int pitch, int win, int row0, int row1,
                    uint16_t* d_out, void* stream) {
    SV_ENTER(c);
    if (check_image(d_gray, H, W) || !d_out) return fail(SV_EINVAL, "bad hog arguments");
    if (win < 1 || win > 15 || (win & 1) == 0) return fail(SV_EINVAL, "win must be odd in [1, 15]");
    hipStream_t s = pick(c, stream);
    SV_LAUNCH(c, SV_K_HOG, s, sv::launch_hog_hist(d_gray, H, W, pitch, win, row0, row1, d_out, s));
    return 0;
}

// ---------------------------------------------------------------- host entry points
int sv_gray(sv_ctx* c, const uint8_t* bgr, int H, int W, int stride, uint8_t* gray) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (check_image(bgr, H, W) || !gray) return fail(SV_EINVAL, "bad gray arguments");
    const size_t row = (size_t)W * 3, n = row * H;
    if (stride < (int)row) return fail(SV_EINVAL, "stride smaller than a row");
    SV_HIP(c->hin.ensure(n));
    for (int y = 0; y < H; ++y) std::memcpy(c->hin.as<uint8_t>() + y * row, bgr + (size_t)y * stride, row);
    SV_HIP(c->img[0].ensure(n));
    SV_HIP(c->gray[0].ensure((size_t)H * W));
    SV_HIP(hipMemcpyAsync(c->img[0].p, c->hin.p, n, hipMemcpyHostToDevice, c->stream));
    SV_LAUNCH(c, SV_K_GRAY, c->stream,
              sv::launch_gray(c->img[0].as<uint8_t>(), H, W, (int)row, c->gray[0].as<uint8_t>(), c->stream));
    Out o[] = {{gray, c->gray[0].p, (size_t)H * W}};
    return collect(c, o, 1);
}

int sv_disparity(sv_ctx* c, const uint8_t* left, const uint8_t* right, int H, int W, int channels, int stride,
                 int min_disp, int num_disp, int win, int cost, int16_t* disp16, float* harris) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!disp16) return fail(SV_EINVAL, "null disparity output");
    sv::MatchPlan plan;
    int rc = check_match(H, W, min_disp, num_disp, win, cost, &plan);
    if (rc) return rc;
    rc = stage_pair(c, left, right, H, W, channels, stride);
    if (rc) return rc;
    SV_HIP(c->d16.ensure((size_t)H * W * sizeof(int16_t)));
    rc = enqueue_disparity(c, c->gray[0].as<uint8_t>(), c->gray[1].as<uint8_t>(), H, W, W, min_disp, num_disp,
                           win, cost, 0, H, c->d16.as<int16_t>(), W, c->stream);
    if (rc) return rc;
    if (harris) {
        SV_HIP(c->harris.ensure((size_t)H * W * sizeof(float)));
        SV_LAUNCH(c, SV_K_HARRIS, c->stream,
                  sv::launch_harris(c->gray[0].as<uint8_t>(), H, W, W, c->harris.as<float>(), c->stream));
    }
    Out o[] = {{disp16, c->d16.p, (size_t)H * W * sizeof(int16_t)},
               {harris, c->harris.p, (size_t)H * W * sizeof(float)}};
    return collect(c, o, 2);
}

int sv_disparity_rows(sv_ctx* c, const uint8_t* left, const uint8_t* right, int H, int W, int channels,
                      int stride, int min_disp, int num_disp, int win, int cost, int row0, int row1,
                      int16_t* disp16) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!disp16) return fail(SV_EINVAL, "null disparity output");
    if (row0 < 0) row0 = 0;
    if (row1 > H) row1 = H;
    if (row1 <= row0) return 0;
    sv::MatchPlan plan;
    int rc = check_match(H, W, min_disp, num_disp, win, cost, &plan);
    if (rc) return rc;
    rc = stage_pair(c, left, right, H, W, channels, stride);
    if (rc) return rc;
    SV_HIP(c->d16.ensure((size_t)H * W * sizeof(int16_t)));
    rc = enqueue_disparity(c, c->gray[0].as<uint8_t>(), c->gray[1].as<uint8_t>(), H, W, W, min_disp, num_disp,
                           win, cost, row0, row1, c->d16.as<int16_t>(), W, c->stream);
    if (rc) return rc;
    const size_t off = (size_t)row0 * W;
    Out o[] = {{disp16 + off, c->d16.as<int16_t>() + off, (size_t)(row1 - row0) * W * sizeof(int16_t)}};
    return collect(c, o, 1);
}


int sv_median5_f32(sv_ctx* c, const float* in, int H, int W, float* out) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (check_image(in, H, W) || !out) return fail(SV_EINVAL, "bad median arguments");
    const size_t n = (size_t)H * W * sizeof(float);
    SV_HIP(c->hin.ensure(n));
    SV_HIP(c->fin.ensure(n));
    SV_HIP(c->fa.ensure(n));
    std::memcpy(c->hin.p, in, n);
    SV_HIP(hipMemcpyAsync(c->fin.p, c->hin.p, n, hipMemcpyHostToDevice, c->stream));
    SV_LAUNCH(c, SV_K_MEDIAN, c->stream, sv::launch_median_f32(c->fin.as<float>(), H, W, c->fa.as<float>(), c->stream));
    Out o[] = {{out, c->fa.p, n}};
    return collect(c, o, 1);
}

static int post_common(sv_ctx* c, const float* disparity, int n, const sv::PostParams& tmpl, float* a,
                       uint8_t* u8, float* b) {
    if (!disparity || n <= 0) return fail(SV_EINVAL, "bad post arguments");
    const size_t nb = (size_t)n * sizeof(float);
    SV_HIP(c->hin.ensure(nb));
    SV_HIP(c->fin.ensure(nb));
    SV_HIP(c->fa.ensure(nb));
    SV_HIP(c->fb.ensure(nb));
    SV_HIP(c->u8.ensure((size_t)n));
    std::memcpy(c->hin.p, disparity, nb);
    SV_HIP(hipMemcpyAsync(c->fin.p, c->hin.p, nb, hipMemcpyHostToDevice, c->stream));
    sv::PostParams pp = tmpl;
    pp.out_a = c->fa.as<float>();
    pp.out_u8 = c->u8.as<uint8_t>();
    pp.out_b = c->fb.as<float>();
    SV_LAUNCH(c, SV_K_POST, c->stream, sv::launch_post(c->fin.as<float>(), n, pp, c->stream));
    Out o[] = {{a, c->fa.p, nb}, {u8, c->u8.p, (size_t)n}, {b, c->fb.p, nb}};
    return collect(c, o, 3);
}

int sv_depth_post(sv_ctx* c, const float* disparity, int n, float min_depth, float max_depth, float depth_range,
                  float min_disp_global, float* depth_final, uint8_t* depth_normalized) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!depth_final || !depth_normalized) return fail(SV_EINVAL, "null outputs");
    sv::PostParams pp = make_post(SV_POST_DEPTH, min_depth, max_depth, depth_range, min_disp_global, 0, 0,
                                  nullptr, nullptr, nullptr);
    return post_common(c, disparity, n, pp, depth_final, depth_normalized, nullptr);
}

int sv_scaled_post(sv_ctx* c, const float* disparity, int n, int min_disp, int num_disp,
                   float* disparity_normalized, uint8_t* normalized_u8, float* confidence) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!disparity_normalized || !normalized_u8 || !confidence || num_disp <= 0)
        return fail(SV_EINVAL, "bad scaled post arguments");
    sv::PostParams pp = make_post(SV_POST_SCALED, 0.f, 0.f, 0.f, 0.f, min_disp, num_disp, nullptr, nullptr,
                                  nullptr);
    return post_common(c, disparity, n, pp, disparity_normalized, normalized_u8, confidence);
}

}  // extern "C"

namespace {

// Host ranges registered through sv_host_register (page-locked and device-visible): the
// host-buffer frame path DMAs its outputs straight into them instead of expanding the int16
// medians on the host.
std::mutex g_reg_mu;
std::map<uintptr_t, size_t> g_reg;   // start -> bytes

bool host_registered(const void* p, size_t bytes) {
    if (!p) return false;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.upper_bound(a);
    if (it == g_reg.begin()) return false;
    --it;
    return a >= it->first && a + bytes <= it->first + it->second;
}

// Host memory -> pinned staging -> device, in chunks: the DMA of one chunk runs while the
// host threads copy the next (one call per frame, as the reference calls the path).
// Rows [y0, y1) of a host image -> the pinned staging buffer (host pool threads) -> the
// device image (one async H2D per sub-chunk on the compute stream, so a sub-chunk's DMA
// overlaps the next one's copy).
int stage_rows(sv_ctx* c, const uint8_t* src, int y0, int y1, size_t row, int stride, uint8_t* stage, uint8_t* dev,
               int nsub) {
    // contiguous rows go to the device straight from the caller's pageable memory (the HIP
    // runtime's own pinned staging, pipelined with its DMA): measured faster than copying
    // into our pinned buffer on the pool threads (1080p create_depth_map 1.03-1.11k vs
    // 0.79-0.89k frames/s per call, 1.49-1.57k vs 0.72-1.18k with 4 in flight,
    // gpurun_out/host3; round 4 the same rates either way, profiles/r04_misc/
    // host_stage_ab_r04h.txt); strided rows take the pinned copy.
    if ((size_t)stride == row) {
        SV_HIP(hipMemcpyAsync(dev + (size_t)y0 * row, src + (size_t)y0 * row, (size_t)(y1 - y0) * row,
                              hipMemcpyHostToDevice, c->stream));
        return 0;
    }
    sv::HostPool& pool = sv::HostPool::get();
    for (int k = 0; k < nsub; ++k) {
        const int a0 = y0 + (int)((long long)(y1 - y0) * k / nsub), a1 = y0 + (int)((long long)(y1 - y0) * (k + 1) / nsub);
        if (a1 <= a0) continue;
        const int parts = pool.threads();
        pool.parallel_for(parts, [&](int p) {
            const int a = a0 + (int)((long long)(a1 - a0) * p / parts), b = a0 + (int)((long long)(a1 - a0) * (p + 1) / parts);
            if (b <= a) return;
            if ((size_t)stride == row)
                std::memcpy(stage + (size_t)a * row, src + (size_t)a * row, (size_t)(b - a) * row);
            else
                for (int y = a; y < b; ++y) std::memcpy(stage + (size_t)y * row, src + (size_t)y * stride, row);
        });
        SV_HIP(hipMemcpyAsync(dev + (size_t)a0 * row, stage + (size_t)a0 * row, (size_t)(a1 - a0) * row,
                              hipMemcpyHostToDevice, c->stream));
    }
    return 0;
}

// Host copy of the context's post-processing table (the one attach_lut attached).
int host_lut(sv_ctx* c, const sv::PostParams& pp) {
    if (c->hl_valid && c->hl_key == c->lut_key) return 0;
    const size_t n = (size_t)pp.lut_n;
    try {
        c->hl_a.resize(n);
        c->hl_b.resize(n);
        c->hl_u8.resize(n);
    } catch (...) {
        return fail(SV_ENOMEM, "host table allocation failed");
    }
    SV_HIP(hipMemcpyAsync(c->hl_a.data(), pp.lut_a, n * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    SV_HIP(hipMemcpyAsync(c->hl_b.data(), pp.lut_b, n * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    SV_HIP(hipMemcpyAsync(c->hl_u8.data(), pp.lut_u8, n, hipMemcpyDeviceToHost, c->stream));
    SV_HIP(hipStreamSynchronize(c->stream));
    c->hl_key = c->lut_key;
    c->hl_valid = true;
    return 0;
}

struct FrameOut {
    float* a;        // DEPTH: depth_final; SCALED: disparity_normalized
    float* disp;     // disparity (f32 = median / 16)
    uint8_t* u8;     // DEPTH: depth_normalized; SCALED: its u8 image (nullable)
    float* b;        // SCALED: confidence
    uint8_t* bgr;    // colormap of u8 through `table` (nullable)
};

// create_depth_map / create_depth_map_stereo_scaled on host buffers (depth_map.py:868-937,
// fused_depth_map.py:976-1024): the frames go up in chunks, gray + disparity + median run on
// the device, and only the int16 x16 median map comes back (2 B/px).  The host expands it
// with the table the device built (bit-identical to the median kernel's epilogue, which
// reads the same table): disparity = m / 16, the post-processing outputs = table[m - m0],
// the colormap = table_bgr[u8].  Chunks of rows come back behind events, so the expansion
// of one chunk runs while the next is in flight.
// Pixels [a, b) of the host expansion: disparity = m / 16 (a power of two: exact), the f32
// output and u8 / BGR from the packed table entry.  The BGR triple goes out as one 4-byte
// store whose 4th byte the next pixel overwrites (same thread); the last pixel of the range
// stores 3 bytes, so ranges of different threads never overlap.  Returns the number of
// medians outside the table (left unwritten).
template <bool U8, bool SCALED, bool BGR>
int expand_rows(const int16_t* med, size_t a, size_t b, int m0, int nl, const HostEnt* ent, const float* lb,
                const FrameOut& o) {
    for (size_t i = a; i < b; ++i) o.disp[i] = (float)med[i] * 0.0625f;
    int nbad = 0;
    for (size_t i = a; i < b; ++i) {
        const uint32_t li = (uint32_t)(med[i] - m0);
        if (__builtin_expect(li >= (uint32_t)nl, 0)) {
            ++nbad;
            continue;
        }
        const HostEnt e = ent[li];
        o.a[i] = e.a;
        if (U8) o.u8[i] = (uint8_t)e.ubgr;
        if (SCALED) o.b[i] = lb[li];
        if (BGR) {
            const uint32_t v = e.ubgr >> 8;
            uint8_t* d = o.bgr + 3 * i;
            if (i + 1 < b) std::memcpy(d, &v, 4);
            else std::memcpy(d, &v, 3);
        }
    }
    return nbad;
}

// Host-side stage timings of the host-buffer path (sv_host_profile_enable / _read; the
// device side — uploads, kernels, downloads — is the context's own event profile,
// SV_K_H2D / SV_K_GRAY / SV_K_MATCH / SV_K_MEDIAN / SV_K_D2H).  SV_HOST_PROFILE=1 also prints
// the averages on stderr every 200 calls.
struct HostProf {
    std::atomic<bool> on{std::getenv("SV_HOST_PROFILE") != nullptr};
    bool print = std::getenv("SV_HOST_PROFILE") != nullptr;
    std::mutex mu;
    double t[6] = {0, 0, 0, 0, 0, 0};     // since the last print (stderr)
    double acc[6] = {0, 0, 0, 0, 0, 0};   // since the last reset (sv_host_profile_read)
    long n = 0, nacc = 0;
    void add(const double* d) {
        std::lock_guard<std::mutex> lk(mu);
        for (int i = 0; i < 6; ++i) {
            t[i] += d[i];
            acc[i] += d[i];
        }
        ++nacc;
        if (print && ++n % 200 == 0) {
            std::fprintf(stderr, "[sv host] per call (ms): prepare %.3f  stage+issue %.3f  wait-first %.3f  expand %.3f  "
                         "wait-rest %.3f  total %.3f\n", t[0] / n, t[1] / n, t[2] / n, t[3] / n, t[4] / n, t[5] / n);
            for (double& v : t) v = 0;
            n = 0;
        }
    }
};
HostProf& host_prof() {
    static HostProf* p = new HostProf();
    return *p;
}
int env_int(const char* name, int dflt, int lo, int hi) {
    const char* e = std::getenv(name);
    if (!e) return dflt;
    const int v = std::atoi(e);
    return v < lo ? lo : v > hi ? hi : v;
}
double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int host_frame_path(sv_ctx* c, const uint8_t* left, const uint8_t* right, int H, int W, int channels, int stride,
                    int min_disp, int num_disp, int win, int cost, sv::PostParams pp, const uint8_t* table,
                    FrameOut o) {
    const bool prof = host_prof().on;
    double tm[6] = {0, 0, 0, 0, 0, 0}, t0 = prof ? now_ms() : 0, tp = t0;
    sv::MatchPlan plan;
    int rc = check_match(H, W, min_disp, num_disp, win, cost, &plan);
    if (rc) return rc;
    if ((long long)H * W >= (1LL << 30)) return fail(SV_EINVAL, "frame too large");
    if (check_image(left, H, W) || check_image(right, H, W)) return SV_EINVAL;
    if (channels != 1 && channels != 3) return fail(SV_EINVAL, "channels must be 1 or 3");
    const size_t row = (size_t)W * channels;
    if (stride < (int)row) return fail(SV_EINVAL, "stride smaller than a row");
    const size_t n = (size_t)H * W;
    SV_HIP(c->hin.ensure(2 * row * H));
    SV_HIP(c->gray[0].ensure(n));
    SV_HIP(c->gray[1].ensure(n));
    if (channels == 3) {
        SV_HIP(c->img[0].ensure(row * H));
        SV_HIP(c->img[1].ensure(row * H));
    }
    SV_HIP(c->d16.ensure(n * sizeof(int16_t)));
    SV_HIP(c->m16.ensure(n * sizeof(int16_t)));
    SV_HIP(c->hout.ensure(n * sizeof(int16_t)));
    rc = attach_lut(c, pp, c->stream);
    if (rc) return rc;
    if (pp.lut_n <= 0) return fail(SV_EINVAL, "no post-processing table for these parameters");
    const bool scaled = pp.mode == SV_POST_SCALED;
    // registered outputs: the median kernel's epilogue writes every output on the device and
    // they come back by DMA; otherwise only the int16 medians come back and the host expands
    // them with the table the device built
    const bool reg = host_registered(o.a, n * 4) && host_registered(o.disp, n * 4) &&
                     (!o.u8 || host_registered(o.u8, n)) && (!scaled || host_registered(o.b, n * 4)) &&
                     (!o.bgr || host_registered(o.bgr, 3 * n));
    sv::PostParams mp = pp;
    int m0 = 0, nl = 0;
    const HostEnt* ent = nullptr;
    const float* lb = nullptr;
    if (reg) {
        SV_HIP(c->fa.ensure(n * 4));
        SV_HIP(c->fb.ensure(n * 4));
        SV_HIP(c->u8.ensure(n));
        if (scaled) SV_HIP(c->fc.ensure(n * 4));
        if (o.bgr) SV_HIP(c->bgr.ensure(3 * n));
        mp.out_a = c->fa.as<float>();
        mp.out_u8 = c->u8.as<uint8_t>();
        mp.out_b = scaled ? c->fc.as<float>() : nullptr;
        rc = attach_cmap(c, mp, table, o.bgr ? c->bgr.as<uint8_t>() : nullptr, c->stream);
        if (rc) return rc;
    } else {
        rc = host_lut(c, pp);
        if (rc) return rc;
        mp.mode = SV_POST_NONE;      // the median kernel writes only the int16 medians
        mp.out_m16 = c->m16.as<int16_t>();
        m0 = pp.lut_m0;
        nl = pp.lut_n;
        // one 8-byte entry per table index: the f32 output and (u8, B, G, R) packed, so a
        // pixel costs one L1 load instead of the dependent u8 -> colormap lookups
        try {
            c->hl_ent.resize((size_t)nl);
        } catch (...) {
            return fail(SV_ENOMEM, "host table allocation failed");
        }
        for (int i = 0; i < nl; ++i) {
            const uint8_t u = c->hl_u8[i];
            const uint32_t bgr = table ? (uint32_t)table[3 * u] | (uint32_t)table[3 * u + 1] << 8 |
                                         (uint32_t)table[3 * u + 2] << 16 : 0u;
            c->hl_ent[i] = HostEnt{c->hl_a[i], u | bgr << 8};
        }
        ent = c->hl_ent.data();
        lb = c->hl_b.data();
    }
    if (prof) { const double t = now_ms(); tm[0] = t - tp; tp = t; }

    // One pass over the whole frame (round 3 also built pipelined row bands, band k's outputs
    // returning on a download stream while band k+1 uploaded: bit-exact but no faster in
    // rounds 3 and 4, so it was removed): stage + upload, gray, disparity, median, then the
    // outputs return in 8 pieces on the compute stream, each behind its own event so the host
    // expansion of one piece runs while the next is in flight.
    // D2H pieces: every hipMemcpyAsync costs ~15-90 us of copy-engine setup on these boxes
    // (tools/microbench/pcie_rate: 4.1 MB pinned in 1 piece 0.08-0.33 ms, 8 pieces 0.2-1.0 ms),
    // so the DMA path (nothing to overlap on the host) downloads each output in one piece and
    // the expansion path in two, the second's transfer under the first's host expansion
    // (round 5 A/B, profiles/r05b/host_ab.txt: 2 pieces 1.47-1.51k frames/s per call, 4
    // pieces 1.41-1.45k, 8 pieces 1.23-1.35k).
    // SV_HOST_PIECES / SV_HOST_PIECES_DMA override (A/B measurements).
    static const int pieces_exp = env_int("SV_HOST_PIECES", 2, 1, 8);
    static const int pieces_dma = env_int("SV_HOST_PIECES_DMA", 1, 1, 8);
    constexpr int kmaxp = 8;
    const int npiece = reg ? pieces_dma : pieces_exp;
    hipStream_t ds = c->stream;
    int bands[kmaxp][2] = {};   // output rows of each D2H piece
    std::atomic<int> bad{0};
    sv::HostPool& pool = sv::HostPool::get();
    auto expand = [&](int k) -> int {   // host expansion of piece k's medians
        const int y0 = bands[k][0], y1 = bands[k][1];
        if (y1 <= y0) return 0;
        SV_HIP(hipEventSynchronize(c->dev_done[k]));
        if (prof) { const double t = now_ms(); tm[k ? 4 : 2] += t - tp; tp = t; }
        const size_t i0 = (size_t)y0 * W, i1 = (size_t)y1 * W;
        const int16_t* med = c->hout.as<int16_t>();
        const int parts = pool.threads();
        pool.parallel_for(parts, [&](int p) {
            const size_t a = i0 + (i1 - i0) * p / parts, b = i0 + (i1 - i0) * (p + 1) / parts;
            const int sel = (o.u8 ? 1 : 0) | (scaled ? 2 : 0) | (o.bgr ? 4 : 0);
            int nb = 0;
            switch (sel) {   // the output set picks the instantiation (no per-pixel branches)
                case 0: nb = expand_rows<false, false, false>(med, a, b, m0, nl, ent, lb, o); break;
                case 1: nb = expand_rows<true, false, false>(med, a, b, m0, nl, ent, lb, o); break;
                case 2: nb = expand_rows<false, true, false>(med, a, b, m0, nl, ent, lb, o); break;
                case 3: nb = expand_rows<true, true, false>(med, a, b, m0, nl, ent, lb, o); break;
                case 4: nb = expand_rows<false, false, true>(med, a, b, m0, nl, ent, lb, o); break;
                case 5: nb = expand_rows<true, false, true>(med, a, b, m0, nl, ent, lb, o); break;
                case 6: nb = expand_rows<false, true, true>(med, a, b, m0, nl, ent, lb, o); break;
                default: nb = expand_rows<true, true, true>(med, a, b, m0, nl, ent, lb, o); break;
            }
            if (nb) bad.fetch_add(nb);
        });
        if (prof) { const double t = now_ms(); tm[3] += t - tp; tp = t; }
        return 0;
    };
    const uint8_t* src[2] = {left, right};
    for (int i = 0; i < 2; ++i) {
        uint8_t* stage = c->hin.as<uint8_t>() + (size_t)i * row * H;
        uint8_t* dst = channels == 1 ? c->gray[i].as<uint8_t>() : c->img[i].as<uint8_t>();
        {   // (profile on: device events around each upload; closed on every exit path)
            ProfScope ph(c, SV_K_H2D, c->stream);
            rc = stage_rows(c, src[i], 0, H, row, stride, stage, dst, 6);
            if (rc) return rc;
            ph.done();
        }
        if (channels == 3)
            SV_LAUNCH(c, SV_K_GRAY, c->stream,
                      sv::launch_gray(c->img[i].as<uint8_t>(), H, W, (int)row, c->gray[i].as<uint8_t>(), c->stream));
    }
    rc = enqueue_disparity(c, c->gray[0].as<uint8_t>(), c->gray[1].as<uint8_t>(), H, W, W, min_disp, num_disp, win,
                           cost, 0, H, c->d16.as<int16_t>(), W, c->stream);
    if (rc) return rc;
    SV_LAUNCH(c, SV_K_MEDIAN, c->stream,
              sv::launch_median_i16(c->d16.as<int16_t>(), H, W, 0, H, reg ? c->fb.as<float>() : nullptr, mp,
                                    c->stream));
    {
        ProfScope pd(c, SV_K_D2H, ds);   // an SV_HIP failure below returns through prof_abort
        for (int q = 0; q < npiece; ++q) {
            const int p0 = (int)((long long)H * q / npiece), p1 = (int)((long long)H * (q + 1) / npiece);
            bands[q][0] = p0;
            bands[q][1] = p1;
            if (p1 <= p0) continue;
            const size_t i0 = (size_t)p0 * W, m = (size_t)(p1 - p0) * W;
            if (reg) {
                SV_HIP(hipMemcpyAsync(o.disp + i0, c->fb.as<float>() + i0, m * 4, hipMemcpyDeviceToHost, ds));
                SV_HIP(hipMemcpyAsync(o.a + i0, c->fa.as<float>() + i0, m * 4, hipMemcpyDeviceToHost, ds));
                if (o.u8) SV_HIP(hipMemcpyAsync(o.u8 + i0, c->u8.as<uint8_t>() + i0, m, hipMemcpyDeviceToHost, ds));
                if (scaled) SV_HIP(hipMemcpyAsync(o.b + i0, c->fc.as<float>() + i0, m * 4, hipMemcpyDeviceToHost, ds));
                if (o.bgr)
                    SV_HIP(hipMemcpyAsync(o.bgr + 3 * i0, c->bgr.as<uint8_t>() + 3 * i0, 3 * m, hipMemcpyDeviceToHost, ds));
            } else {
                SV_HIP(hipMemcpyAsync(c->hout.as<int16_t>() + i0, c->m16.as<int16_t>() + i0, m * 2, hipMemcpyDeviceToHost,
                                      ds));
                if (!c->dev_done[q]) SV_HIP(hipEventCreateWithFlags(&c->dev_done[q], hipEventDisableTiming));
                SV_HIP(hipEventRecord(c->dev_done[q], ds));
            }
        }
        pd.done();
    }
    if (prof) { const double t = now_ms(); tm[1] = t - tp; tp = t; }
    if (!reg) {
        for (int q = 0; q < npiece; ++q) {
            rc = expand(q);
            if (rc) return rc;
        }
    }
    SV_HIP(hipStreamSynchronize(ds));
    if (prof) {
        const double t = now_ms();
        tm[4] += t - tp;
        tm[5] = t - t0;
        host_prof().add(tm);
    }
    if (bad.load()) return fail(SV_EHIP, "median value outside the post-processing table");
    return 0;
}

}  // namespace

extern "C" {

int sv_host_profile_enable(int enable) {
    host_prof().on = enable != 0;
    return 0;
}

int sv_host_profile_read(double* ms6, long long* calls, int reset) {
    HostProf& hp = host_prof();
    std::lock_guard<std::mutex> lk(hp.mu);
    if (ms6)
        for (int i = 0; i < 6; ++i) ms6[i] = hp.acc[i];
    if (calls) *calls = hp.nacc;
    if (reset) {
        for (double& v : hp.acc) v = 0;
        hp.nacc = 0;
    }
    return 0;
}

int sv_host_register(void* ptr, uint64_t bytes) {
    if (!ptr || bytes == 0) return fail(SV_EINVAL, "null or empty host range");
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        if (g_reg.count(reinterpret_cast<uintptr_t>(ptr))) return fail(SV_EINVAL, "host range already registered");
    }
    SV_HIP(hipHostRegister(ptr, (size_t)bytes, hipHostRegisterPortable));
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg[reinterpret_cast<uintptr_t>(ptr)] = (size_t)bytes;
    return 0;
}

int sv_host_unregister(void* ptr) {
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto it = g_reg.find(reinterpret_cast<uintptr_t>(ptr));
        if (it == g_reg.end()) return fail(SV_EINVAL, "host range not registered");
        g_reg.erase(it);
    }
    SV_HIP(hipHostUnregister(ptr));
    return 0;
}

int sv_depth_map(sv_ctx* c, const uint8_t* left, const uint8_t* right, int H, int W, int channels, int stride,
                 int min_disp, int num_disp, int win, int cost, float min_depth, float max_depth,
                 float depth_range, float min_disp_global, float* depth_final, float* disparity,
                 uint8_t* depth_normalized) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!depth_final || !disparity || !depth_normalized) return fail(SV_EINVAL, "null outputs");
    sv::PostParams pp = make_post(SV_POST_DEPTH, min_depth, max_depth, depth_range, min_disp_global, min_disp,
                                  num_disp, nullptr, nullptr, nullptr);
    return host_frame_path(c, left, right, H, W, channels, stride, min_disp, num_disp, win, cost, pp, nullptr,
                           FrameOut{depth_final, disparity, depth_normalized, nullptr, nullptr});
}

int sv_stereo_scaled(sv_ctx* c, const uint8_t* left, const uint8_t* right, int H, int W, int channels,
                     int stride, int min_disp, int num_disp, int win, int cost, float* disparity_normalized,
                     float* disparity, uint8_t* normalized_u8, float* confidence) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!disparity_normalized || !disparity || !normalized_u8 || !confidence)
        return fail(SV_EINVAL, "null outputs");
    sv::PostParams pp = make_post(SV_POST_SCALED, 0.f, 0.f, 0.f, 0.f, min_disp, num_disp, nullptr, nullptr, nullptr);
    return host_frame_path(c, left, right, H, W, channels, stride, min_disp, num_disp, win, cost, pp, nullptr,
                           FrameOut{disparity_normalized, disparity, normalized_u8, confidence, nullptr});
}

int sv_depth_map_color(sv_ctx* c, const uint8_t* left, const uint8_t* right, int H, int W, int channels,
                       int stride, int min_disp, int num_disp, int win, int cost, float min_depth, float max_depth,
                       float depth_range, float min_disp_global, const uint8_t* cmap_bgr, float* depth_final,
                       float* disparity, uint8_t* depth_normalized, uint8_t* depth_colormap) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!depth_final || !disparity || !depth_colormap || !cmap_bgr) return fail(SV_EINVAL, "null outputs");
    sv::PostParams pp = make_post(SV_POST_DEPTH, min_depth, max_depth, depth_range, min_disp_global, min_disp,
                                  num_disp, nullptr, nullptr, nullptr);
    return host_frame_path(c, left, right, H, W, channels, stride, min_disp, num_disp, win, cost, pp, cmap_bgr,
                           FrameOut{depth_final, disparity, depth_normalized, nullptr, depth_colormap});
}

int sv_stereo_scaled_color(sv_ctx* c, const uint8_t* left, const uint8_t* right, int H, int W, int channels,
                           int stride, int min_disp, int num_disp, int win, int cost, const uint8_t* cmap_bgr,
                           float* disparity_normalized, float* disparity, uint8_t* normalized_u8,
                           float* confidence, uint8_t* depth_colormap) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!disparity_normalized || !disparity || !confidence || !depth_colormap || !cmap_bgr)
        return fail(SV_EINVAL, "null outputs");
    sv::PostParams pp = make_post(SV_POST_SCALED, 0.f, 0.f, 0.f, 0.f, min_disp, num_disp, nullptr, nullptr, nullptr);
    return host_frame_path(c, left, right, H, W, channels, stride, min_disp, num_disp, win, cost, pp, cmap_bgr,
                           FrameOut{disparity_normalized, disparity, normalized_u8, confidence, depth_colormap});
}

int sv_harris(sv_ctx* c, const uint8_t* gray, int H, int W, int stride, float* out) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (check_image(gray, H, W) || !out || stride < W) return fail(SV_EINVAL, "bad harris arguments");
    const size_t n = (size_t)H * W;
    SV_HIP(c->hin.ensure(n));
    for (int y = 0; y < H; ++y) std::memcpy(c->hin.as<uint8_t>() + (size_t)y * W, gray + (size_t)y * stride, W);
    SV_HIP(c->gray[0].ensure(n));
    SV_HIP(c->harris.ensure(n * sizeof(float)));
    SV_HIP(hipMemcpyAsync(c->gray[0].p, c->hin.p, n, hipMemcpyHostToDevice, c->stream));
    SV_LAUNCH(c, SV_K_HARRIS, c->stream,
              sv::launch_harris(c->gray[0].as<uint8_t>(), H, W, W, c->harris.as<float>(), c->stream));
    Out o[] = {{out, c->harris.p, n * sizeof(float)}};
    return collect(c, o, 1);
}

int sv_hog_hist(sv_ctx* c, const uint8_t* gray, int H, int W, int stride, int win, uint16_t* out) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (check_image(gray, H, W) || !out || stride < W) return fail(SV_EINVAL, "bad hog arguments");
    if (win < 1 || win > 15 || (win & 1) == 0) return fail(SV_EINVAL, "win must be odd in [1, 15]");
    const size_t n = (size_t)H * W;
    SV_HIP(c->hin.ensure(n));
    for (int y = 0; y < H; ++y) std::memcpy(c->hin.as<uint8_t>() + (size_t)y * W, gray + (size_t)y * stride, W);
    SV_HIP(c->gray[0].ensure(n));
    SV_HIP(c->hog[0].ensure(n * 10 * sizeof(uint16_t)));
    SV_HIP(hipMemcpyAsync(c->gray[0].p, c->hin.p, n, hipMemcpyHostToDevice, c->stream));
    SV_LAUNCH(c, SV_K_HOG, c->stream,
              sv::launch_hog_hist(c->gray[0].as<uint8_t>(), H, W, W, win, 0, H, c->hog[0].as<uint16_t>(), c->stream));
    Out o[] = {{out, c->hog[0].p, n * 10 * sizeof(uint16_t)}};
    return collect(c, o, 1);
}

// ---------------------------------------------------------------- rectification
int sv_init_undistort_rectify_map_dev(sv_ctx* c, const double* K, const double* dist, int ndist, const double* R,
                                      const double* P, int p_cols, int H, int W, int16_t* d_map1,
                                      uint16_t* d_map2, void* stream) {
    SV_ENTER(c);
    if (!d_map1 || !d_map2) return fail(SV_EINVAL, "null map outputs");
    sv::UndistortParams up;
    int rc = make_undistort(K, dist, ndist, R, P, p_cols, H, W, &up);
    if (rc) return rc;
    hipStream_t s = pick(c, stream);
    SV_LAUNCH(c, SV_K_UNDISTORT, s, sv::launch_undistort_map(up, reinterpret_cast<short2*>(d_map1), d_map2, s));
    return 0;
}

int sv_init_undistort_rectify_map(sv_ctx* c, const double* K, const double* dist, int ndist, const double* R,
                                  const double* P, int p_cols, int H, int W, int16_t* map1, uint16_t* map2) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!map1 || !map2) return fail(SV_EINVAL, "null map outputs");
    sv::UndistortParams up;
    int rc = make_undistort(K, dist, ndist, R, P, p_cols, H, W, &up);
    if (rc) return rc;
    const size_t n = (size_t)H * W;
    SV_HIP(c->rmap1.ensure(n * 4));
    SV_HIP(c->rmap2.ensure(n * 2));
    SV_LAUNCH(c, SV_K_UNDISTORT, c->stream,
              sv::launch_undistort_map(up, c->rmap1.as<short2>(), c->rmap2.as<uint16_t>(), c->stream));
    Out o[] = {{map1, c->rmap1.p, n * 4}, {map2, c->rmap2.p, n * 2}};
    return collect(c, o, 2);
}

int sv_remap_dev(sv_ctx* c, const uint8_t* d_src, int sH, int sW, int channels, int src_pitch,
                 int64_t src_frame_stride, const int16_t* d_map1, const uint16_t* d_map2, int H, int W,
                 int gray_out, uint8_t* d_dst, int dst_pitch, int64_t dst_frame_stride, int n_frames,
                 void* stream) {
    SV_ENTER(c);
    int rc = check_remap(d_src, sH, sW, channels, src_pitch, d_map1, H, W, d_dst);
    if (rc) return rc;
    if (gray_out && channels != 3) return fail(SV_EINVAL, "gray_out needs a 3-channel source");
    const int ob = (channels == 3 && !gray_out) ? 3 : 1;
    if (dst_pitch < W * ob) return fail(SV_EINVAL, "destination pitch smaller than a row");
    if (n_frames < 0) return fail(SV_EINVAL, "negative frame count");
    if (n_frames > 1 && (src_frame_stride < (int64_t)src_pitch * sH || dst_frame_stride < (int64_t)dst_pitch * H))
        return fail(SV_EINVAL, "frame stride smaller than a frame");
    if (n_frames == 0) return 0;
    hipStream_t s = pick(c, stream);
    SV_LAUNCH(c, SV_K_REMAP, s,
              sv::launch_remap(d_src, sH, sW, channels, src_pitch, src_frame_stride,
                               reinterpret_cast<const short2*>(d_map1), d_map2, H, W, gray_out != 0, d_dst,
                               dst_pitch, dst_frame_stride, n_frames, s));
    return 0;
}

// Stage host images (any stride) and host/device maps, remap on the context stream.
static int remap_host_common(sv_ctx* c, const uint8_t* const* srcs, int nimg, int sH, int sW, int channels,
                             int stride, const short2* const* dmap1, const uint16_t* const* dmap2, int H, int W,
                             uint8_t* const* outs) {
    const size_t row = (size_t)sW * channels, n = row * sH;
    SV_HIP(c->hin.ensure(nimg * n));
    for (int k = 0; k < nimg; ++k) {
        SV_HIP(c->img[k].ensure(n));
        uint8_t* dst = c->hin.as<uint8_t>() + k * n;
        if ((size_t)stride == row) {
            std::memcpy(dst, srcs[k], n);
        } else {
            for (int y = 0; y < sH; ++y) std::memcpy(dst + y * row, srcs[k] + (size_t)y * stride, row);
        }
        SV_HIP(hipMemcpyAsync(c->img[k].p, dst, n, hipMemcpyHostToDevice, c->stream));
    }
    const size_t on = (size_t)H * W * channels;
    Out o[2];
    for (int k = 0; k < nimg; ++k) {
        SV_HIP(c->rdst[k].ensure(on));
        SV_LAUNCH(c, SV_K_REMAP, c->stream,
                  sv::launch_remap(c->img[k].as<uint8_t>(), sH, sW, channels, (int)row, 0, dmap1[k], dmap2[k], H, W,
                                   false, c->rdst[k].as<uint8_t>(), W * channels, 0, 1, c->stream));
        o[k] = {outs[k], c->rdst[k].p, on};
    }
    return collect(c, o, nimg);
}

int sv_remap(sv_ctx* c, const uint8_t* src, int sH, int sW, int channels, int stride, const int16_t* map1,
             const uint16_t* map2, int H, int W, uint8_t* dst) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    int rc = check_remap(src, sH, sW, channels, stride, map1, H, W, dst);
    if (rc) return rc;
    const size_t n = (size_t)H * W;
    SV_HIP(c->rmap1.ensure(n * 4));
    SV_HIP(c->rmap2.ensure(n * 2));
    SV_HIP(hipMemcpyAsync(c->rmap1.p, map1, n * 4, hipMemcpyHostToDevice, c->stream));
    if (map2) SV_HIP(hipMemcpyAsync(c->rmap2.p, map2, n * 2, hipMemcpyHostToDevice, c->stream));
    const short2* m1[1] = {c->rmap1.as<short2>()};
    const uint16_t* m2[1] = {map2 ? c->rmap2.as<uint16_t>() : nullptr};
    const uint8_t* srcs[1] = {src};
    uint8_t* outs[1] = {dst};
    return remap_host_common(c, srcs, 1, sH, sW, channels, stride, m1, m2, H, W, outs);
}

int sv_rectify_pair(sv_ctx* c, const int16_t* d_map1_left, const uint16_t* d_map2_left,
                    const int16_t* d_map1_right, const uint16_t* d_map2_right, int H, int W, const uint8_t* left,
                    const uint8_t* right, int sH, int sW, int channels, int stride, uint8_t* out_left,
                    uint8_t* out_right) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    int rc = check_remap(left, sH, sW, channels, stride, d_map1_left, H, W, out_left);
    if (!rc) rc = check_remap(right, sH, sW, channels, stride, d_map1_right, H, W, out_right);
    if (rc) return rc;
    const short2* m1[2] = {reinterpret_cast<const short2*>(d_map1_left), reinterpret_cast<const short2*>(d_map1_right)};
    const uint16_t* m2[2] = {d_map2_left, d_map2_right};
    const uint8_t* srcs[2] = {left, right};
    uint8_t* outs[2] = {out_left, out_right};
    return remap_host_common(c, srcs, 2, sH, sW, channels, stride, m1, m2, H, W, outs);
}

int sv_resize_linear_dev(sv_ctx* c, const uint8_t* d_src, int sH, int sW, int channels, int src_pitch,
                         int64_t src_frame_stride, uint8_t* d_dst, int dH, int dW, int dst_pitch,
                         int64_t dst_frame_stride, int n_frames, void* stream) {
    SV_ENTER(c);
    if (!d_src || !d_dst || sH <= 0 || sW <= 0 || dH <= 0 || dW <= 0 || n_frames < 0)
        return fail(SV_EINVAL, "bad resize arguments");
    if (channels != 1 && channels != 3) return fail(SV_EINVAL, "channels must be 1 or 3");
    if (src_pitch < sW * channels || dst_pitch < dW * channels) return fail(SV_EINVAL, "pitch smaller than a row");
    if (n_frames > 1 && (src_frame_stride < (int64_t)src_pitch * sH || dst_frame_stride < (int64_t)dst_pitch * dH))
        return fail(SV_EINVAL, "frame stride smaller than a frame");
    if (n_frames == 0) return 0;
    hipStream_t s = pick(c, stream);
    SV_LAUNCH(c, SV_K_RESIZE, s,
              sv::launch_resize_linear(d_src, sH, sW, channels, src_pitch, src_frame_stride, d_dst, dH, dW,
                                       dst_pitch, dst_frame_stride, n_frames, false, s));
    return 0;
}

int sv_resize_linear_f32_dev(sv_ctx* c, const float* d_src, int sH, int sW, int src_pitch, float* d_dst, int dH,
                             int dW, int dst_pitch, void* stream) {
    SV_ENTER(c);
    if (!d_src || !d_dst || sH <= 0 || sW <= 0 || dH <= 0 || dW <= 0) return fail(SV_EINVAL, "bad resize arguments");
    if (src_pitch < sW * 4 || dst_pitch < dW * 4) return fail(SV_EINVAL, "pitch smaller than a row");
    hipStream_t s = pick(c, stream);
    SV_LAUNCH(c, SV_K_RESIZE, s,
              sv::launch_resize_linear(d_src, sH, sW, 1, src_pitch, 0, d_dst, dH, dW, dst_pitch, 0, 1, true, s));
    return 0;
}

int sv_resize_linear(sv_ctx* c, const uint8_t* src, int sH, int sW, int channels, int stride, uint8_t* dst,
                     int dH, int dW) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!src || !dst || sH <= 0 || sW <= 0 || dH <= 0 || dW <= 0) return fail(SV_EINVAL, "bad resize arguments");
    if (channels != 1 && channels != 3) return fail(SV_EINVAL, "channels must be 1 or 3");
    const size_t row = (size_t)sW * channels, n = row * sH;
    if (stride < (int)row) return fail(SV_EINVAL, "stride smaller than a row");
    SV_HIP(c->hin.ensure(n));
    for (int y = 0; y < sH; ++y) std::memcpy(c->hin.as<uint8_t>() + y * row, src + (size_t)y * stride, row);
    SV_HIP(c->img[0].ensure(n));
    const size_t on = (size_t)dH * dW * channels;
    SV_HIP(c->rdst[0].ensure(on));
    SV_HIP(hipMemcpyAsync(c->img[0].p, c->hin.p, n, hipMemcpyHostToDevice, c->stream));
    SV_LAUNCH(c, SV_K_RESIZE, c->stream,
              sv::launch_resize_linear(c->img[0].as<uint8_t>(), sH, sW, channels, (int)row, 0,
                                       c->rdst[0].as<uint8_t>(), dH, dW, dW * channels, 0, 1, false, c->stream));
    Out o[] = {{dst, c->rdst[0].p, on}};
    return collect(c, o, 1);
}

// ---------------------------------------------------------------- reductions
static void stats_blocks(int H, int W, int* bh, int* bw) {
    *bh = H / 48 > 0 ? H / 48 : 1;
    *bw = W / 48 > 0 ? W / 48 : 1;
}

int sv_frame_stats_batch_dev(sv_ctx* c, const uint8_t* d_img0, const uint8_t* d_img1, int n_frames,
                             int64_t frame_stride, int H, int W, int channels, int pitch, uint32_t* d_block_sum,
                             uint32_t* d_block_sq, uint32_t* d_hist, void* stream) {
    SV_ENTER(c);
    if (check_image(d_img0, H, W) || !d_block_sum || !d_block_sq || !d_hist || n_frames < 1)
        return fail(SV_EINVAL, "bad frame-stats arguments");
    if (channels != 1 && channels != 3) return fail(SV_EINVAL, "channels must be 1 or 3");
    if (pitch < W * channels) return fail(SV_EINVAL, "pitch smaller than a row");
    if (n_frames > 1 && frame_stride < (int64_t)pitch * H) return fail(SV_EINVAL, "frame stride smaller than a frame");
    const int per = d_img1 ? 2 : 1;
    if ((long long)n_frames * per > 65535) return fail(SV_EINVAL, "too many images in one batch");
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    const int nimg = n_frames * per;
    SV_HIP(c->hist_copies.ensure_zeroed((size_t)sv::kHistCopies * nimg * 256 * sizeof(uint32_t)));
    sv::FrameStatsArgs a{};
    a.hist_copies = c->hist_copies.as<uint32_t>();
    a.img0 = d_img0;
    a.img1 = d_img1;
    a.H = H;
    a.W = W;
    a.pitch = pitch;
    a.cn = channels;
    a.per = per;
    a.fs = n_frames > 1 ? frame_stride : 0;
    stats_blocks(H, W, &a.bh, &a.bw);
    a.block_sum = d_block_sum;
    a.block_sq = d_block_sq;
    a.hist = d_hist;
    SV_LAUNCH(c, SV_K_STATS, s, sv::launch_frame_stats(a, nimg, s));
    return 0;
}

int sv_frame_stats(sv_ctx* c, const uint8_t* img0, const uint8_t* img1, int H, int W, int channels, int stride,
                   uint32_t* block_sum, uint32_t* block_sq, uint32_t* hist) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (check_image(img0, H, W) || !block_sum || !block_sq || !hist) return fail(SV_EINVAL, "bad frame-stats arguments");
    if (channels != 1 && channels != 3) return fail(SV_EINVAL, "channels must be 1 or 3");
    const size_t row = (size_t)W * channels, n = row * H;
    if (stride < (int)row) return fail(SV_EINVAL, "stride smaller than a row");
    const int nimg = img1 ? 2 : 1;
    int bh, bw;
    stats_blocks(H, W, &bh, &bw);
    const size_t nb = (size_t)bh * bw;
    SV_HIP(c->hin.ensure(nimg * n));
    const uint8_t* src[2] = {img0, img1};
    for (int k = 0; k < nimg; ++k) {
        SV_HIP(c->img[k].ensure(n));
        uint8_t* dst = c->hin.as<uint8_t>() + k * n;
        for (int y = 0; y < H; ++y) std::memcpy(dst + y * row, src[k] + (size_t)y * stride, row);
        SV_HIP(hipMemcpyAsync(c->img[k].p, dst, n, hipMemcpyHostToDevice, c->stream));
    }
    SV_HIP(c->stats.ensure(nimg * (2 * nb + 256) * sizeof(uint32_t)));
    uint32_t* d = c->stats.as<uint32_t>();
    SV_HIP(c->hist_copies.ensure_zeroed((size_t)sv::kHistCopies * 2 * 256 * sizeof(uint32_t)));
    sv::FrameStatsArgs a{};
    a.hist_copies = c->hist_copies.as<uint32_t>();
    a.img0 = c->img[0].as<uint8_t>();
    a.img1 = nimg == 2 ? c->img[1].as<uint8_t>() : nullptr;
    a.H = H;
    a.W = W;
    a.pitch = (int)row;
    a.cn = channels;
    a.per = nimg;
    a.fs = 0;
    a.bh = bh;
    a.bw = bw;
    a.block_sum = d;
    a.block_sq = d + nimg * nb;
    a.hist = d + 2 * nimg * nb;
    SV_LAUNCH(c, SV_K_STATS, c->stream, sv::launch_frame_stats(a, nimg, c->stream));
    Out o[] = {{block_sum, a.block_sum, nimg * nb * 4}, {block_sq, a.block_sq, nimg * nb * 4},
               {hist, a.hist, (size_t)nimg * 256 * 4}};
    return collect(c, o, 3);
}

// One select pass over the context stream (a batch of a.narr arrays): hist [narr][kMaxRanks]
// [2048] and counts [narr][2] back on the host.
static int select_pass(sv_ctx* c, sv::SelectArgs& a, uint32_t* hist_host, unsigned long long* counts_host) {
    // device: [kSelBatch][copies][kMaxRanks][2048] accumulators | [kSelBatch] count slots |
    // folded hist [narr][kMaxRanks][2048] | counts [narr][2].  The accumulator regions are
    // laid out for the largest batch whatever narr is: the folds leave them zeroed, and a
    // smaller batch's outputs must never land where a larger batch accumulates
    const size_t na = (size_t)(a.narr > 0 ? a.narr : 1);
    const size_t hb = (size_t)sv::kMaxRanks * 2048 * sizeof(uint32_t);
    const size_t ab = (size_t)sv::kSelBatch * sv::kHistCopies * hb;
    const size_t cb = (size_t)sv::kSelBatch * sv::kCountSlots * 16 * sizeof(unsigned long long);
    const size_t ob = na * hb + na * 16;
    SV_HIP(c->sel.ensure_zeroed(ab + cb + ob));
    uint8_t* base = c->sel.as<uint8_t>();
    a.ghist = reinterpret_cast<uint32_t*>(base);
    a.counts = reinterpret_cast<unsigned long long*>(base + ab);
    a.hist_out = reinterpret_cast<uint32_t*>(base + ab + cb);
    a.counts_out = reinterpret_cast<unsigned long long*>(base + ab + cb + na * hb);
    SV_LAUNCH(c, SV_K_SELECT, c->stream, sv::launch_select_hist(a, c->stream));
    SV_HIP(c->hout.ensure(ob));
    SV_HIP(hipMemcpyAsync(c->hout.p, a.hist_out, ob, hipMemcpyDeviceToHost, c->stream));
    SV_HIP(hipStreamSynchronize(c->stream));
    std::memcpy(hist_host, c->hout.p, na * hb);
    if (counts_host) std::memcpy(counts_host, c->hout.as<uint8_t>() + na * hb, na * 16);
    return 0;
}

// np.percentile's order statistics of a batch of narr arrays (array y at d_x + y * x_stride,
// its mask at d_mask + y * mask_stride): selected / nan counts (nullable) and, with nranks
// > 0, the values of ranks[y][r] (radix select in three passes of 11/11/10 bits, one launch
// + one fold per pass for the whole batch).
static int select_batch(sv_ctx* c, const float* d_x, int64_t n, int64_t x_stride, int narr, int mask_mode,
                        const float* d_mask, int64_t mask_stride, float thr, const int64_t* ranks, int nranks,
                        float* values, int64_t* selected, int64_t* nans) {
    if (!d_x || n < 0) return fail(SV_EINVAL, "bad select arguments");
    if (mask_mode < 0 || mask_mode > 2) return fail(SV_EINVAL, "mask_mode must be 0, 1 or 2");
    if (mask_mode == 2 && !d_mask) return fail(SV_EINVAL, "mask_mode 2 needs a mask array");
    if (narr < 1 || narr > sv::kSelBatch) return fail(SV_EINVAL, "1..16 arrays per batch");
    if (narr > 1 && (x_stride < n || (mask_mode == 2 && mask_stride < n))) return fail(SV_EINVAL, "array stride below n");
    if (nranks < 0 || nranks > sv::kMaxRanks || (nranks > 0 && (!ranks || !values))) return fail(SV_EINVAL, "0..4 ranks");
    sv::SelectArgs a{};
    a.x = d_x;
    a.mask = mask_mode == 2 ? d_mask : nullptr;
    a.thr = thr;
    a.mask_mode = mask_mode;
    a.n = (size_t)n;
    a.narr = narr;
    a.xstride = narr > 1 ? (size_t)x_stride : 0;
    a.mstride = narr > 1 ? (size_t)mask_stride : 0;
    std::vector<uint32_t> h((size_t)narr * sv::kMaxRanks * 2048);
    std::vector<unsigned long long> cnt((size_t)narr * 2, 0ull);
    const size_t hs = (size_t)sv::kMaxRanks * 2048;
    uint32_t prefix[sv::kSelBatch][sv::kMaxRanks] = {};
    int64_t rem[sv::kSelBatch][sv::kMaxRanks];
    for (int y = 0; y < narr; ++y)
        for (int r = 0; r < nranks; ++r) {
            if (ranks[(size_t)y * nranks + r] < 0) return fail(SV_EINVAL, "negative rank");
            rem[y][r] = ranks[(size_t)y * nranks + r];
        }
    const int shifts[3] = {21, 10, 0}, bits[3] = {11, 11, 10};
    const int passes = nranks > 0 ? 3 : 1;
    for (int p = 0; p < passes; ++p) {
        a.shift = shifts[p];
        a.bits = bits[p];
        a.nranks = p == 0 ? 1 : nranks;          // pass 0: one histogram serves every rank
        for (int y = 0; y < narr; ++y)
            for (int r = 0; r < sv::kMaxRanks; ++r) a.prefix[y][r] = p == 0 ? 0u : prefix[y][r];
        if (n > 0) {
            int rc = select_pass(c, a, h.data(), p == 0 ? cnt.data() : nullptr);
            if (rc) return rc;
        }
        if (p == 0) {
            for (int y = 0; y < narr; ++y) {
                if (selected) selected[y] = (int64_t)cnt[2 * y];
                if (nans) nans[y] = (int64_t)cnt[2 * y + 1];
                for (int r = 0; r < nranks; ++r)
                    if ((unsigned long long)rem[y][r] >= cnt[2 * y]) return fail(SV_ERANGE, "rank beyond the selection");
            }
        }
        for (int y = 0; y < narr; ++y)
            for (int r = 0; r < nranks; ++r) {
                const uint32_t* hr = h.data() + (size_t)y * hs + (p == 0 ? 0 : r) * 2048;
                int64_t acc = 0;
                int d = 0;
                for (; d < (1 << bits[p]); ++d) {
                    if (acc + (int64_t)hr[d] > rem[y][r]) break;
                    acc += hr[d];
                }
                if (d == (1 << bits[p])) return fail(SV_EHIP, "select: histogram inconsistent (data changed?)");
                rem[y][r] -= acc;
                prefix[y][r] = (prefix[y][r] << bits[p]) | (uint32_t)d;
            }
    }
    for (int y = 0; y < narr; ++y)
        for (int r = 0; r < nranks; ++r) {
            const uint32_t k = prefix[y][r];
            const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
            std::memcpy(&values[(size_t)y * nranks + r], &u, sizeof(float));
        }
    return 0;
}

int sv_select_count_batch(sv_ctx* c, const float* d_x, int64_t n, int64_t x_stride, int n_arrays, int mask_mode,
                          const float* d_mask, int64_t mask_stride, float thr, int64_t* selected, int64_t* nans) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    return select_batch(c, d_x, n, x_stride, n_arrays, mask_mode, d_mask, mask_stride, thr, nullptr, 0, nullptr,
                        selected, nans);
}

int sv_select_ranks_batch(sv_ctx* c, const float* d_x, int64_t n, int64_t x_stride, int n_arrays, int mask_mode,
                          const float* d_mask, int64_t mask_stride, float thr, const int64_t* ranks, int nranks,
                          float* values) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!ranks || !values || nranks < 1 || nranks > sv::kMaxRanks) return fail(SV_EINVAL, "1..4 ranks");
    return select_batch(c, d_x, n, x_stride, n_arrays, mask_mode, d_mask, mask_stride, thr, ranks, nranks, values,
                        nullptr, nullptr);
}

int sv_affine_f32_dev(sv_ctx* c, const float* d_x, int64_t n, int mode, float fa, float fb, float fc, float fd,
                      double ds, double doff, float* d_out, void* stream) {
    SV_ENTER(c);
    if (!d_x || !d_out || n < 0 || mode < 0 || mode > 2) return fail(SV_EINVAL, "bad affine arguments");
    hipStream_t s = pick(c, stream);
    sv::AffineArgs a{};
    a.x = d_x;
    a.out = d_out;
    a.n = (size_t)n;
    a.mode = mode;
    a.fa = fa;
    a.fb = fb;
    a.fc = fc;
    a.fd = fd;
    a.ds = ds;
    a.doff = doff;
    SV_LAUNCH(c, SV_K_AFFINE, s, sv::launch_affine_f32(a, s));
    return 0;
}

// ---------------------------------------------------------------- SGBM-3WAY mode
int sv_sgbm_dev(sv_ctx* c, const uint8_t* d_left, const uint8_t* d_right, int H, int W, int pitch, int min_disp,
                int num_disp, int block_size, int P1, int P2, int disp12_max_diff, int pre_filter_cap,
                int uniqueness_ratio, int speckle_window_size, int speckle_range, int16_t* d_disp16, int out_pitch,
                void* stream) {
    SV_ENTER(c);
    sv::MatchPlan plan;
    int rc = check_match(H, W, min_disp, num_disp, block_size, SV_COST_SGBM, &plan);
    if (rc) return rc;
    if (check_image(d_left, H, W) || check_image(d_right, H, W) || !d_disp16 || pitch < W || out_pitch < W)
        return fail(SV_EINVAL, "bad SGBM arguments");
    SgbmParams p{P1, P2, disp12_max_diff, pre_filter_cap, uniqueness_ratio, speckle_window_size, speckle_range};
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    return enqueue_sgbm(c, d_left, d_right, H, W, pitch, min_disp, num_disp, block_size, p, d_disp16, out_pitch,
                        s);
}

int sv_sgbm(sv_ctx* c, const uint8_t* left, const uint8_t* right, int H, int W, int channels, int stride,
            int min_disp, int num_disp, int block_size, int P1, int P2, int disp12_max_diff, int pre_filter_cap,
            int uniqueness_ratio, int speckle_window_size, int speckle_range, int16_t* disp16) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!disp16) return fail(SV_EINVAL, "null disparity output");
    sv::MatchPlan plan;
    int rc = check_match(H, W, min_disp, num_disp, block_size, SV_COST_SGBM, &plan);
    if (rc) return rc;
    rc = stage_pair(c, left, right, H, W, channels, stride);
    if (rc) return rc;
    SV_HIP(c->d16.ensure((size_t)H * W * sizeof(int16_t)));
    SgbmParams p{P1, P2, disp12_max_diff, pre_filter_cap, uniqueness_ratio, speckle_window_size, speckle_range};
    rc = enqueue_sgbm(c, c->gray[0].as<uint8_t>(), c->gray[1].as<uint8_t>(), H, W, W, min_disp, num_disp,
                      block_size, p, c->d16.as<int16_t>(), W, c->stream);
    if (rc) return rc;
    Out o[] = {{disp16, c->d16.p, (size_t)H * W * sizeof(int16_t)}};
    return collect(c, o, 1);
}

// cv2.filterSpeckles(img, newVal, maxSpeckleSize, maxDiff) on an int16 map, in place.
int sv_filter_speckles_dev(sv_ctx* c, int16_t* d_img, int H, int W, int pitch, int new_val, int max_speckle_size,
                           int max_diff, void* stream) {
    SV_ENTER(c);
    if (!d_img || H <= 0 || W <= 0 || pitch < W) return fail(SV_EINVAL, "bad speckle-filter arguments");
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    return enqueue_speckles(c, d_img, H, W, pitch, new_val, max_speckle_size, max_diff, s);
}

int sv_filter_speckles(sv_ctx* c, int16_t* img, int H, int W, int new_val, int max_speckle_size, int max_diff) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!img || H <= 0 || W <= 0) return fail(SV_EINVAL, "bad speckle-filter arguments");
    const size_t bytes = (size_t)H * W * sizeof(int16_t);
    SV_HIP(c->d16.ensure(bytes));
    SV_HIP(c->hin.ensure(bytes));
    std::memcpy(c->hin.p, img, bytes);
    SV_HIP(hipMemcpyAsync(c->d16.p, c->hin.p, bytes, hipMemcpyHostToDevice, c->stream));
    const int rc = enqueue_speckles(c, c->d16.as<int16_t>(), H, W, W, new_val, max_speckle_size, max_diff, c->stream);
    if (rc) return rc;
    Out o[] = {{img, c->d16.p, bytes}};
    return collect(c, o, 1);
}


}  // extern "C"
