// sv_capi.cpp — the C ABI (include/stereovision_amd.h) over the gfx950 kernels: errors,
// contexts, device memory, profiling and the enqueue helpers every entry point shares
// (sv_ctx.h).  The entry points themselves: sv_capi_dev.cpp (one device), sv_capi_multi.cpp
// (several devices, RCCL / peer-copy gathers).
//
// A context = one device + one HIP stream + grow-only device buffers + pinned staging.
// Host entry points stage into pinned memory, run the whole chain on the context stream
// and copy results back; device entry points only enqueue.  No exception crosses the ABI.
#include "sv_ctx.h"

namespace {
thread_local std::string g_err;
}  // namespace

namespace svc {

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hipfail(int e, const char* what) {
    return fail(SV_EHIP, std::string(what) + ": " + hipGetErrorString((hipError_t)e));
}

const std::string& last_error_msg() { return g_err; }

int check_image(const void* a, int H, int W) {
    if (!a || H <= 0 || W <= 0) return fail(SV_EINVAL, "null image or non-positive size");
    return 0;
}

int check_match(int H, int W, int min_disp, int num_disp, int win, int cost, sv::MatchPlan* plan) {
    if (H <= 0 || W <= 0) return fail(SV_EINVAL, "non-positive image size");
    if (num_disp <= 0 || num_disp > 512) return fail(SV_EINVAL, "num_disp must be in [1, 512]");
    if (win < 1 || win > 15 || (win & 1) == 0) return fail(SV_EINVAL, "win must be odd in [1, 15]");
    if (min_disp < -4096 || min_disp > 4096) return fail(SV_EINVAL, "min_disp out of range");
    if (cost == SV_COST_SGBM) return 0;   // no lane plan: sv_sgbm.hip sizes itself
    int rc = sv::plan_match(num_disp, win, cost, plan);
    if (rc == -34) return fail(SV_ERANGE, "cost range too large for the argmin key");
    if (rc != 0) return fail(SV_EINVAL, "unsupported (num_disp, win, cost)");
    return 0;
}

SgbmParams sgbm_reference_params(int win) {
    // depth_map.py:894-906 / fused_depth_map.py:988-1000
    return {8 * 3 * win * win, 32 * 3 * win * win, 1, 63, 10, 100, 32};
}

// Enqueue the whole SGBM-3WAY pipeline for one frame (buffers grown in the context).
// cv2.filterSpeckles on an int16 device map (speckle stage of SGBM, sv_filter_speckles).
// nf > 1: a batch of maps, map z at d_img + z*fimg (one launch per stage over grid.z).
int enqueue_speckles(sv_ctx* c, int16_t* d_img, int H, int W, int pitch, int new_val, int max_speckle_size,
                     int max_diff, hipStream_t s, int nf, long long fimg) {
    if (max_speckle_size <= 0) return 0;
    const size_t n = (size_t)H * W * (nf < 1 ? 1 : nf);
    SV_HIP(c->cc_parent.ensure(n * 4));
    SV_HIP(c->cc_size.ensure(n * 4));
    SV_LAUNCH(c, SV_K_SPECKLE, s,
              sv::launch_speckles(d_img, H, W, pitch, new_val, max_speckle_size, max_diff, c->cc_parent.as<int>(),
                                  c->cc_size.as<int>(), s, nf < 1 ? 1 : nf, fimg));
    return 0;
}

// nf > 1: a batch of frames, frame z at L/R + z*fs_in bytes and out + z*fs_out elements.  The
// DP kernels are chains of W (or H) dependent steps, so one frame leaves most SIMDs idle;
// batches run every stage once over grid.z (up to kSgbmChunk frames, or as many as the
// scratch budget allows: ~1.5 GB of volumes per 1080p D=128 frame with int16 paths).
constexpr int kSgbmChunk = 32;
// Scratch budget of a batch's volumes: SV_SGBM_BUDGET_GB (GiB) if set, else a quarter of the
// device's free memory at the call (capped at 48 GiB), so several contexts on one device do
// not each pin tens of GB; sv_release_scratch returns them after a large batch
size_t sgbm_budget(int device) {
    static const long long env_gb = [] {
        const char* e = std::getenv("SV_SGBM_BUDGET_GB");
        return e ? std::atoll(e) : 0LL;
    }();
    if (env_gb > 0) return (size_t)env_gb << 30;
    size_t fr = 0, tot = 0;
    (void)device;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr == 0) return (size_t)8 << 30;
    return std::min<size_t>(fr / 4, (size_t)48 << 30);
}

int enqueue_sgbm(sv_ctx* c, const uint8_t* L, const uint8_t* R, int H, int W, int pitch, int min_disp,
                 int num_disp, int win, SgbmParams p, int16_t* out, int opitch, hipStream_t s, int nf,
                 long long fs_in, long long fs_out) {
    if (nf < 1) nf = 1;
    if (sv::sgbm_dp(num_disp) < 0) return fail(SV_EINVAL, "num_disp must be in [1, 512]");
    if (W > 16384) return fail(SV_EINVAL, "SGBM: width beyond 16384");
    if (p.P1 < 0 || p.P2 < 0) return fail(SV_EINVAL, "negative P1/P2");
    if (p.P2 <= p.P1) p.P2 = p.P1 + 1;                       // OpenCV: P2 = max(P2, P1 + 1)
    if (p.P2 >= 349525) return fail(SV_ERANGE, "SGBM: P2 too large for the 32-bit argmin key");
    p.cap = (p.cap > 15 ? p.cap : 15) | 1;                   // OpenCV's ftzero
    if (p.cap > 127) return fail(SV_EINVAL, "preFilterCap must be <= 127");
    sv::SgbmArgs a{};
    a.L = L;
    a.R = R;
    a.H = H;
    a.W = W;
    a.pitch = pitch;
    a.minD = min_disp;
    a.D = num_disp;
    a.r = win / 2;
    const int maxd = min_disp + num_disp;
    a.X0 = maxd > 0 ? maxd : 0;
    int X1 = W + (min_disp < 0 ? min_disp : 0);
    if (X1 > W) X1 = W;
    a.Wb = X1 > a.X0 ? X1 - a.X0 : 0;
    a.cap = p.cap;
    a.P1 = p.P1;
    a.P2 = p.P2;
    a.uniq = p.uniq < 0 ? 10 : p.uniq;
    a.disp12 = p.disp12;
    const long long cmax = (long long)(2 * p.cap + 63) * win * win;   // max window cost
    if (cmax > 65535) return fail(SV_EINVAL, "SGBM: window cost beyond 16 bits (lower preFilterCap/blockSize)");
    a.l32 = (cmax > 32767 || p.P2 > 32768) ? 1 : 0;
    a.Dp = sv::sgbm_dp(num_disp);
    const size_t vol = (size_t)H * a.Wb * a.Dp;
    // hsum + C (u16), L_lr (int16: in the hsum volume), L_rl (unfused only), L_tb, band
    const size_t lsz = a.l32 ? 4 : 2;
    const bool cost1 = sv::sgbm_cost_fused(num_disp, a.r);   // k_sgbm_cost: per-pixel record planes
    const size_t rec_frame = cost1 ? (size_t)2 * H * W * 16 : 0;
    const size_t per_frame = vol * (4 + lsz * 3) + (size_t)H * a.Wb * 8 + rec_frame;   // unfused (the larger)
    // volumes already held count towards the budget (they are reused, not added to)
    const size_t held = c->sg_hsum.cap + c->sg_c.cap + c->sg_l.cap + c->sg_lt.cap + c->sg_band.cap + c->sg_rec.cap;
    const size_t kSgbmBudget = std::max(sgbm_budget(c->device) + held, per_frame);
    int chunk = (int)std::max<size_t>(1, std::min<size_t>({(size_t)nf, (size_t)kSgbmChunk,
                                                            kSgbmBudget / std::max<size_t>(per_frame, 1)}));
    const bool fused = sv::sgbm_fused(chunk, num_disp);
    if (fused)   // no L_rl volume: a third more frames fit the budget
        chunk = (int)std::max<size_t>(1, std::min<size_t>({(size_t)nf, (size_t)kSgbmChunk,
                                                            kSgbmBudget / (per_frame - vol * lsz)}));
    a.fused = fused ? 1 : 0;
    SV_HIP(c->sg_hsum.ensure(vol * 2 * chunk + 256));
    SV_HIP(c->sg_c.ensure(vol * 2 * chunk + 256));
    const int nl = (a.l32 ? 1 : 0) + (fused ? 0 : 1);   // volumes in sg_l: L_lr (int32), L_rl
    SV_HIP(c->sg_l.ensure(vol * lsz * nl * chunk + 256));
    SV_HIP(c->sg_lt.ensure(vol * (a.l32 ? 4 : 2) * chunk + 256));
    if (!c->sg_aux) {
        SV_HIP(hipStreamCreateWithFlags(&c->sg_aux, hipStreamNonBlocking));
        SV_HIP(hipEventCreateWithFlags(&c->sg_ev[0], hipEventDisableTiming));
        SV_HIP(hipEventCreateWithFlags(&c->sg_ev[1], hipEventDisableTiming));
    }
    const size_t band_bytes = (size_t)H * a.Wb * 8 * chunk;
    SV_HIP(c->sg_band.ensure(band_bytes + 256 + 64 * 128));
    a.hsum = c->sg_hsum.as<uint16_t>();
    a.C = c->sg_c.as<uint16_t>();
    // int16 paths: L_lr reuses the hsum volume (dead after the window-row sums); every volume
    // holds `chunk` frames at a stride of vol elements of its type (SgbmArgs::select_frame)
    a.Llr = a.l32 ? c->sg_l.p : c->sg_hsum.p;
    a.Lrl = fused ? nullptr : a.l32 ? (void*)(c->sg_l.as<int32_t>() + vol * chunk) : c->sg_l.p;
    a.Ltb = c->sg_lt.p;
    a.band = c->sg_band.p;
    a.recs = nullptr;
    if (cost1) {
        SV_HIP(c->sg_rec.ensure(rec_frame * chunk + 256));
        a.recs = c->sg_rec.as<uint4>();
    }
    a.dummy = c->sg_band.as<uint8_t>() + (band_bytes + 255) / 256 * 256;
    a.opitch = opitch;
    a.fs_in = fs_in;
    a.fs_out = fs_out;
    for (int z0 = 0; z0 < nf; z0 += chunk) {
        const int n = std::min(chunk, nf - z0);
        a.L = L + z0 * fs_in;
        a.R = R + z0 * fs_in;
        a.out = out + z0 * fs_out;
        SV_LAUNCH(c, SV_K_SGBM, s, sv::launch_sgbm(a, n, s, c->sg_aux, c->sg_ev[0], c->sg_ev[1]));
        const int rc = enqueue_speckles(c, a.out, H, W, opitch, (min_disp - 1) * 16, p.speckle_win,
                                        16 * p.speckle_range, s, n, fs_out);
        if (rc) return rc;
    }
    return 0;
}

// Enqueue disparity for rows [row0,row1) of gray device images.
// nf > 1: a batch of frames, frame z at L/R + z*fs_in bytes and out + z*fs_out elements
// (one launch over grid.z; HOG: one histogram launch over both images of every frame, then
// one match launch reading frame z's histograms at z * H*W*10).
int enqueue_disparity(sv_ctx* c, const uint8_t* L, const uint8_t* R, int H, int W, int pitch,
                      int min_disp, int num_disp, int win, int cost, int row0, int row1,
                      int16_t* out, int opitch, hipStream_t s, int nf, long long fs_in,
                      long long fs_out) {
    sv::MatchPlan plan;
    int rc = check_match(H, W, min_disp, num_disp, win, cost, &plan);
    if (rc) return rc;
    if (row0 < 0) row0 = 0;
    if (row1 > H) row1 = H;
    if (row1 <= row0) return 0;
    if (cost == SV_COST_SGBM) {   // the top-down path crosses rows: whole frames only
        if (row0 != 0 || row1 != H) return fail(SV_EINVAL, "SGBM cannot compute a row band (use frames)");
        return enqueue_sgbm(c, L, R, H, W, pitch, min_disp, num_disp, win, sgbm_reference_params(win), out, opitch,
                            s, nf, fs_in, fs_out);
    }
    sv::MatchParams a{};
    a.L = L;
    a.R = R;
    a.H = H;
    a.W = W;
    a.pitch = pitch;
    a.minD = min_disp;
    a.D = num_disp;
    a.win = win;
    a.r = cost == SV_COST_HOG ? 0 : win / 2;
    int maxd = min_disp + num_disp;
    a.X0 = maxd > 0 ? maxd : 0;
    a.X1 = W + (min_disp < 0 ? min_disp : 0);
    if (a.X1 > W) a.X1 = W;
    if (a.X1 < a.X0) a.X1 = a.X0;
    a.row0 = row0;
    a.row1 = row1;
    a.lpg = plan.lpg;
    a.lpg_log2 = plan.lpg == 16 ? 4 : plan.lpg == 32 ? 5 : 6;
    a.dbits = plan.dbits;
    a.pad_key = (uint32_t)((sv::max_cost(win, cost) + 1) << plan.dbits);
    a.out = out;
    a.opitch = opitch;
    SV_HIP(c->wctr.ensure_zeroed(256));
    a.work_ctr = c->wctr.as<unsigned>();
    a.nf = nf < 1 ? 1 : nf;
    a.fs_in = fs_in;
    a.fs_out = fs_out;
    a.fs_hist = 0;
    if (cost == SV_COST_HOG && a.X1 > a.X0) {
        const long long fh = (long long)H * W * 10;   // elements per frame's histograms
        const size_t hb = (size_t)fh * sizeof(uint16_t) * a.nf;
        SV_HIP(c->hog[0].ensure(hb));
        SV_HIP(c->hog[1].ensure(hb));
        SV_LAUNCH(c, SV_K_HOG, s,
                  sv::launch_hog_hist_pairs(L, R, H, W, pitch, win, row0, row1, c->hog[0].as<uint16_t>(),
                                            c->hog[1].as<uint16_t>(), a.nf, a.nf > 1 ? fs_in : 0, fh, s));
        a.HL = c->hog[0].as<uint16_t>();
        a.HR = c->hog[1].as<uint16_t>();
        a.fs_hist = a.nf > 1 ? fh : 0;
    }
    if (sv::ring_split(cost, win, num_disp) && a.X1 > a.X0) {
        const long long ke = sv::ring_split_elems(a.nf, fs_out, row1, opitch);
        SV_HIP(c->keys.ensure((size_t)(2 * ke) * sizeof(uint32_t)));
        a.keys = c->keys.as<uint32_t>();
        a.keys_stride = ke;
    }
    SV_LAUNCH(c, SV_K_MATCH, s, sv::launch_match(a, plan, cost, s));
    return 0;
}

// Attach the cached post-processing table for the median kernel (built on first use of a
// parameter set; covers every int16 x16 value a map with this (min_disp, num_disp) holds).
// whole: the median map holds whole disparities only (medians of an integer-cost matcher's
// int16 x16 output: multiples of 16), so the table can hold one entry per disparity
int attach_lut(sv_ctx* c, sv::PostParams& pp, hipStream_t s, bool whole) {
    pp.lut_n = 0;
    pp.lut_shift = 0;
    if (pp.mode == SV_POST_NONE || pp.num_disp <= 0 || pp.num_disp > 512) return 0;
    sv_ctx::LutKey k;
    k.mode = pp.mode;
    k.min_disp = pp.min_disp;
    k.num_disp = pp.num_disp;
    k.m0 = (pp.min_disp - 1) * 16;
    k.n = whole ? pp.num_disp + 1 : (pp.num_disp + 1) * 16;
    k.minf = pp.minf;
    k.maxf = pp.maxf;
    k.rangef = pp.rangef;
    k.mdg = pp.min_disp_global;
    DevBuf& buf = whole ? c->lutw : c->lut;
    sv_ctx::LutKey& key = whole ? c->lutw_key : c->lut_key;
    hipEvent_t& ev = whole ? c->lutw_ev : c->lut_ev;
    hipStream_t& bs = whole ? c->lutw_stream : c->lut_stream;
    const size_t n = (size_t)k.n;
    float* la = buf.as<float>();
    if (!(k == key) || !ev) {
        SV_HIP(buf.ensure(n * (2 * sizeof(float) + 1)));
        la = buf.as<float>();
        if (!ev) SV_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        int e = sv::launch_post_lut(pp, k.m0, k.n, whole ? 16 : 1, la, reinterpret_cast<uint8_t*>(la + 2 * n), la + n,
                                    s);
        if (e) return hipfail(e, "launch_post_lut");
        SV_HIP(hipEventRecord(ev, s));
        key = k;
        bs = s;
    } else if (s != bs) {
        SV_HIP(hipStreamWaitEvent(s, ev, 0));   // built earlier on another stream
    }
    pp.lut_a = la;
    pp.lut_b = la + n;
    pp.lut_u8 = reinterpret_cast<const uint8_t*>(la + 2 * n);
    pp.lut_m0 = k.m0;
    pp.lut_n = k.n;
    pp.lut_shift = whole ? 4 : 0;
    return 0;
}

// Device copy of a 256-entry BGR colormap table (re-uploaded only when it changes).
int attach_cmap(sv_ctx* c, sv::PostParams& pp, const uint8_t* table, uint8_t* d_bgr, hipStream_t s) {
    pp.out_bgr = nullptr;
    pp.cmap = nullptr;
    if (!d_bgr) return 0;
    if (!table) return fail(SV_EINVAL, "colormap output without a table");
    SV_HIP(c->cmap.ensure(256 * sizeof(uint32_t)));
    if (!c->cmap_valid || std::memcmp(c->cmap_host, table, 768) != 0) {
        uint32_t packed[256];
        for (int i = 0; i < 256; ++i)
            packed[i] = (uint32_t)table[3 * i] | ((uint32_t)table[3 * i + 1] << 8) | ((uint32_t)table[3 * i + 2] << 16);
        SV_HIP(hipMemcpyAsync(c->cmap.p, packed, sizeof(packed), hipMemcpyHostToDevice, s));
        SV_HIP(hipStreamSynchronize(s));   // `packed` lives on this stack frame
        std::memcpy(c->cmap_host, table, 768);
        c->cmap_valid = true;
    }
    pp.out_bgr = d_bgr;
    pp.cmap = c->cmap.as<uint32_t>();
    return 0;
}

sv::PostParams make_post(int mode, float minf, float maxf, float rangef, float mdg, int min_disp,
                         int num_disp, float* a, uint8_t* u8, float* b) {
    sv::PostParams pp{};
    pp.mode = mode;
    pp.minf = minf;
    pp.maxf = maxf;
    pp.rangef = rangef;
    pp.min_disp_global = mdg;
    pp.min_disp = min_disp;
    pp.num_disp = num_disp;
    pp.out_a = a;
    pp.out_u8 = u8;
    pp.out_b = b;
    return pp;
}

int map_out_post(sv_ctx* c, const sv_map_out* out, int min_disp, int num_disp, int cost, bool allow_harris,
                 hipStream_t s, sv::PostParams* pp, float** disp) {
    if (!out) return fail(SV_EINVAL, "null outputs");
    const int mode = out->mode;
    if (mode != SV_POST_NONE && mode != SV_POST_DEPTH && mode != SV_POST_SCALED) return fail(SV_EINVAL, "bad post mode");
    if (mode == SV_POST_DEPTH && (!out->out_a || !out->out_u8)) return fail(SV_EINVAL, "depth post outputs missing");
    if (mode == SV_POST_SCALED && (!out->out_a || !out->out_u8 || !out->out_b || num_disp <= 0))
        return fail(SV_EINVAL, "scaled post outputs missing");
    if (mode == SV_POST_NONE && (out->out_a || out->out_u8 || out->out_b))
        return fail(SV_EINVAL, "post outputs without a post mode");
    if (out->bgr && (mode == SV_POST_NONE || !out->cmap_bgr))
        return fail(SV_EINVAL, "a colormap output needs a post mode and a table");
    if (out->harris && !allow_harris) return fail(SV_EINVAL, "the Harris output belongs to sv_depth_map_batch_dev");
    if (out->d8 && (cost == SV_COST_SGBM || num_disp < 1 || num_disp > 255))
        return fail(SV_EINVAL, "u8 disparity indices need an integer-disparity cost and num_disp <= 255");
    if (!out->disparity && !out->med16 && !out->d8 && mode == SV_POST_NONE && !out->harris)
        return fail(SV_EINVAL, "no outputs");
    *pp = make_post(mode, out->min_depth, out->max_depth, out->depth_range, out->min_disp_global, min_disp, num_disp,
                    out->out_a, out->out_u8, out->out_b);
    // integer-disparity maps: every median is a multiple of 16 (the whole-disparity table)
    int rc = attach_lut(c, *pp, s, cost != SV_COST_SGBM);
    if (!rc) rc = attach_cmap(c, *pp, out->cmap_bgr, out->bgr, s);
    if (rc) return rc;
    pp->out_m16 = out->med16;
    pp->out_d8 = out->d8;
    pp->d8_base = min_disp - 1;
    *disp = out->disparity;
    return 0;
}

int check_map(int fmt, const void* map, int cost, int num_disp) {
    if (fmt != SV_MAP_M16 && fmt != SV_MAP_D8) return fail(SV_EINVAL, "map format must be SV_MAP_M16 or SV_MAP_D8");
    if (!map) return fail(SV_EINVAL, "null map");
    if (fmt == SV_MAP_D8 && (cost == SV_COST_SGBM || num_disp < 1 || num_disp > 255))
        return fail(SV_EINVAL, "u8 disparity indices need an integer-disparity cost and num_disp <= 255");
    return 0;
}

// Median epilogue of a context that only produces a map: int16 x16 or u8 indices into `dst`
// (full-frame element offsets), no post-processing outputs.
sv::PostParams map_post(int fmt, void* dst, int d8_base) {
    sv::PostParams pp = make_post(SV_POST_NONE, 0.f, 0.f, 0.f, 0.f, 0, 0, nullptr, nullptr, nullptr);
    if (fmt == SV_MAP_D8) {
        pp.out_d8 = static_cast<uint8_t*>(dst);
        pp.d8_base = d8_base;
    } else {
        pp.out_m16 = static_cast<int16_t*>(dst);
    }
    return pp;
}


// Stage two host images (HxW or HxWx3, any stride) into the context's device gray buffers.
int stage_pair(sv_ctx* c, const uint8_t* left, const uint8_t* right, int H, int W, int channels,
               int stride) {
    if (check_image(left, H, W) || check_image(right, H, W)) return SV_EINVAL;
    if (channels != 1 && channels != 3) return fail(SV_EINVAL, "channels must be 1 or 3");
    const size_t row = (size_t)W * channels;
    if (stride < (int)row) return fail(SV_EINVAL, "stride smaller than a row");
    const size_t n = row * H;
    SV_HIP(c->hin.ensure(2 * n));
    SV_HIP(c->gray[0].ensure((size_t)H * W));
    SV_HIP(c->gray[1].ensure((size_t)H * W));
    const uint8_t* src[2] = {left, right};
    for (int k = 0; k < 2; ++k) {
        uint8_t* dst = c->hin.as<uint8_t>() + k * n;
        if ((size_t)stride == row) {
            std::memcpy(dst, src[k], n);
        } else {
            for (int y = 0; y < H; ++y) std::memcpy(dst + y * row, src[k] + (size_t)y * stride, row);
        }
    }
    if (channels == 1) {
        SV_HIP(hipMemcpyAsync(c->gray[0].p, c->hin.p, n, hipMemcpyHostToDevice, c->stream));
        SV_HIP(hipMemcpyAsync(c->gray[1].p, c->hin.as<uint8_t>() + n, n, hipMemcpyHostToDevice, c->stream));
    } else {
        SV_HIP(c->img[0].ensure(n));
        SV_HIP(c->img[1].ensure(n));
        for (int k = 0; k < 2; ++k) {
            SV_HIP(hipMemcpyAsync(c->img[k].p, c->hin.as<uint8_t>() + k * n, n, hipMemcpyHostToDevice, c->stream));
            SV_LAUNCH(c, SV_K_GRAY, c->stream,
                      sv::launch_gray(c->img[k].as<uint8_t>(), H, W, (int)row, c->gray[k].as<uint8_t>(), c->stream));
        }
    }
    return 0;
}

// Copy device results to caller buffers through the pinned output staging, then wait.
int collect(sv_ctx* c, const Out* outs, int n) {
    size_t total = 0;
    for (int i = 0; i < n; ++i)
        if (outs[i].host) total += (outs[i].bytes + 255) & ~(size_t)255;
    SV_HIP(c->hout.ensure(total ? total : 256));
    size_t off = 0;
    for (int i = 0; i < n; ++i) {
        if (!outs[i].host) continue;
        SV_HIP(hipMemcpyAsync(c->hout.as<uint8_t>() + off, outs[i].dev, outs[i].bytes, hipMemcpyDeviceToHost, c->stream));
        off += (outs[i].bytes + 255) & ~(size_t)255;
    }
    SV_HIP(hipStreamSynchronize(c->stream));
    off = 0;
    for (int i = 0; i < n; ++i) {
        if (!outs[i].host) continue;
        std::memcpy(outs[i].host, c->hout.as<uint8_t>() + off, outs[i].bytes);
        off += (outs[i].bytes + 255) & ~(size_t)255;
    }
    return 0;
}

// initUndistortRectifyMap's setup: ir = inv(P[:, :3] * R) with OpenCV's Matx33d product and
// cofactor inverse (the same operation order as oracle/sv_rectify_oracle.py).
int make_undistort(const double* K, const double* dist, int ndist, const double* R, const double* P,
                   int p_cols, int H, int W, sv::UndistortParams* out) {
    if (!K || H <= 0 || W <= 0) return fail(SV_EINVAL, "bad map arguments");
    if (H > 32767 || W > 32767) return fail(SV_EINVAL, "map size beyond the int16 coordinate range");
    if (!(ndist == 0 || ndist == 4 || ndist == 5 || ndist == 8 || ndist == 12 || ndist == 14) ||
        (ndist > 0 && !dist))
        return fail(SV_EINVAL, "distCoeffs must have 0, 4, 5, 8, 12 or 14 elements");
    if (ndist == 14 && (dist[12] != 0.0 || dist[13] != 0.0))
        return fail(SV_EINVAL, "tilted sensor model (tauX, tauY != 0) is not supported");
    if (P && p_cols != 3 && p_cols != 4) return fail(SV_EINVAL, "P must be 3x3 or 3x4");
    double A[9], Rm[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, M[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) A[i * 3 + j] = P ? P[i * p_cols + j] : K[i * 3 + j];
    if (R) std::memcpy(Rm, R, sizeof(Rm));
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            M[i * 3 + j] = (A[i * 3 + 0] * Rm[0 * 3 + j] + A[i * 3 + 1] * Rm[1 * 3 + j]) + A[i * 3 + 2] * Rm[2 * 3 + j];
    auto a = [&](int i, int j) { return M[i * 3 + j]; };
    const double det = a(0, 0) * (a(1, 1) * a(2, 2) - a(2, 1) * a(1, 2)) -
                       a(0, 1) * (a(1, 0) * a(2, 2) - a(2, 0) * a(1, 2)) +
                       a(0, 2) * (a(1, 0) * a(2, 1) - a(2, 0) * a(1, 1));
    if (det == 0.0) return fail(SV_EINVAL, "singular newCameraMatrix * R");
    const double d = 1.0 / det;
    double* b = out->ir;
    b[0] = (a(1, 1) * a(2, 2) - a(1, 2) * a(2, 1)) * d;
    b[1] = (a(0, 2) * a(2, 1) - a(0, 1) * a(2, 2)) * d;
    b[2] = (a(0, 1) * a(1, 2) - a(0, 2) * a(1, 1)) * d;
    b[3] = (a(1, 2) * a(2, 0) - a(1, 0) * a(2, 2)) * d;
    b[4] = (a(0, 0) * a(2, 2) - a(0, 2) * a(2, 0)) * d;
    b[5] = (a(0, 2) * a(1, 0) - a(0, 0) * a(1, 2)) * d;
    b[6] = (a(1, 0) * a(2, 1) - a(1, 1) * a(2, 0)) * d;
    b[7] = (a(0, 1) * a(2, 0) - a(0, 0) * a(2, 1)) * d;
    b[8] = (a(0, 0) * a(1, 1) - a(0, 1) * a(1, 0)) * d;
    out->fx = K[0];
    out->fy = K[4];
    out->u0 = K[2];
    out->v0 = K[5];
    for (int i = 0; i < 12; ++i) out->k[i] = i < ndist ? dist[i] : 0.0;
    out->H = H;
    out->W = W;
    return 0;
}

int check_remap(const void* src, int sH, int sW, int channels, int pitch, const void* map1, int H, int W,
                const void* dst) {
    if (!src || !map1 || !dst || sH <= 0 || sW <= 0 || H <= 0 || W <= 0)
        return fail(SV_EINVAL, "bad remap arguments");
    if (channels != 1 && channels != 3) return fail(SV_EINVAL, "channels must be 1 or 3");
    if (pitch < sW * channels) return fail(SV_EINVAL, "source pitch smaller than a row");
    return 0;
}

}  // namespace svc

int sv::set_error(int code, const std::string& msg) { return fail(code, msg); }

extern "C" {

int sv_version(void) { return SV_API_VERSION; }

const char* sv_last_error(void) { return g_err.c_str(); }

int sv_device_count(int* n) {
    if (!n) return fail(SV_EINVAL, "null output");
    int k = 0;
    hipError_t e = hipGetDeviceCount(&k);
    if (e != hipSuccess) {
        *n = 0;
        return hipfail((int)e, "hipGetDeviceCount");
    }
    *n = k;
    return 0;
}

int sv_create(int device, sv_ctx** out) {
    if (!out) return fail(SV_EINVAL, "null output");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(SV_ENODEV, "no HIP device visible");
    if (device < 0 || device >= n) return fail(SV_ENODEV, "device index out of range");
    sv_ctx* c = new (std::nothrow) sv_ctx();
    if (!c) return fail(SV_ENOMEM, "context allocation failed");
    c->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return hipfail((int)e, "sv_create");
    }
    *out = c;
    return 0;
}

void sv_destroy(sv_ctx* c) {
    if (!c) return;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
        c->prof_drain();
        for (auto e : c->pool) (void)hipEventDestroy(e);
        DevBuf* bufs[] = {&c->wctr, &c->img[0], &c->img[1], &c->gray[0], &c->gray[1], &c->d16, &c->fa, &c->fb,
                          &c->fc, &c->u8, &c->harris, &c->hog[0], &c->hog[1], &c->fin, &c->lut,
                          &c->rmap1, &c->rmap2, &c->rdst[0], &c->rdst[1], &c->stats, &c->sel,
                          &c->sg_hsum, &c->sg_c, &c->sg_l, &c->sg_lt, &c->sg_band, &c->cc_parent,
                          &c->hist_copies, &c->cmap, &c->bgr, &c->m16,
                          &c->cc_size, &c->sg_rec, &c->gm16, &c->keys, &c->lutw};
        if (c->lut_ev) (void)hipEventDestroy(c->lut_ev);
        if (c->lutw_ev) (void)hipEventDestroy(c->lutw_ev);
        if (c->scr_ev) (void)hipEventDestroy(c->scr_ev);
        if (c->xev) (void)hipEventDestroy(c->xev);
        if (c->sev) (void)hipEventDestroy(c->sev);
        if (c->gev) (void)hipEventDestroy(c->gev);
        for (auto e : c->wev)
            if (e) (void)hipEventDestroy(e);
        if (c->region_open) {
            (void)hipEventDestroy(c->region.a);
            (void)hipEventDestroy(c->region.b);
        }
        for (auto e : c->dev_done)
            if (e) (void)hipEventDestroy(e);
        for (auto e : c->tmr)
            if (e) (void)hipEventDestroy(e);
        if (c->sg_aux) {
            (void)hipStreamSynchronize(c->sg_aux);
            (void)hipStreamDestroy(c->sg_aux);
        }
        for (auto e : c->sg_ev)
            if (e) (void)hipEventDestroy(e);
        for (auto* b : bufs) b->release();
        c->hin.release();
        c->hout.release();
        (void)hipStreamDestroy(c->stream);
    }
    delete c;
}

int sv_event_record(sv_ctx* c, int slot, void* stream) {
    SV_ENTER(c);
    if (slot < 0 || slot >= 16) return fail(SV_EINVAL, "event slot must be in [0, 16)");
    hipEvent_t& e = c->wev[slot];
    if (!e) SV_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    SV_HIP(hipEventRecord(e, pick(c, stream)));
    return 0;
}

int sv_stream_wait_event(sv_ctx* c, int slot, void* stream) {
    SV_ENTER(c);
    if (slot < 0 || slot >= 16 || !c->wev[slot]) return fail(SV_EINVAL, "event slot never recorded");
    SV_HIP(hipStreamWaitEvent(pick(c, stream), c->wev[slot], 0));
    return 0;
}

int sv_release_scratch(sv_ctx* c) {
    SV_ENTER(c);
    SV_HIP(hipStreamSynchronize(c->stream));
    if (c->sg_aux) SV_HIP(hipStreamSynchronize(c->sg_aux));
    // the grow-only work buffers (not the post table, colormap or staging): the next call
    // allocates what it needs again
    DevBuf* bufs[] = {&c->img[0], &c->img[1], &c->gray[0], &c->gray[1], &c->d16, &c->fa, &c->fb, &c->fc,
                      &c->u8, &c->harris, &c->hog[0], &c->hog[1], &c->fin, &c->sg_hsum, &c->sg_c,
                      &c->sg_l, &c->sg_lt, &c->sg_band, &c->sg_rec, &c->cc_parent, &c->cc_size, &c->m16,
                      &c->gm16, &c->keys};
    for (auto* b : bufs) b->release();
    return 0;
}

int sv_synchronize(sv_ctx* c) {
    SV_ENTER(c);
    SV_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

void* sv_stream(sv_ctx* c) { return c ? static_cast<void*>(c->stream) : nullptr; }

int sv_plan(int num_disp, int win, int cost, int* dpl, int* lpg, int* lds_bytes) {
    sv::MatchPlan p;
    int rc = sv::plan_match(num_disp, win, cost, &p);
    if (rc == -34) return fail(SV_ERANGE, "cost range too large for the argmin key");
    if (rc) return fail(SV_EINVAL, "unsupported (num_disp, win, cost)");
    if (dpl) *dpl = p.dpl;
    if (lpg) *lpg = p.lpg;
    if (lds_bytes) *lds_bytes = (int)sv::match_lds_bytes(p, cost == SV_COST_HOG ? 0 : win / 2, cost);
    return 0;
}

// ---------------------------------------------------------------- device memory
int sv_dev_alloc(sv_ctx* c, uint64_t bytes, void** out) {
    SV_ENTER(c);
    if (!out || bytes == 0) return fail(SV_EINVAL, "bad allocation request");
    *out = nullptr;
    SV_HIP(hipMalloc(out, (size_t)bytes));
    return 0;
}

int sv_dev_free(sv_ctx* c, void* p) {
    SV_ENTER(c);
    if (p) SV_HIP(hipFree(p));
    return 0;
}

int sv_copy_to_device(sv_ctx* c, void* dst, const void* src, uint64_t bytes, void* stream) {
    SV_ENTER(c);
    if (!dst || !src) return fail(SV_EINVAL, "null pointer");
    if (!bytes) return 0;
    if (stream) {   // enqueued: the caller keeps src alive (and pinned, for overlap)
        SV_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, static_cast<hipStream_t>(stream)));
        return 0;
    }
    SV_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, c->stream));
    SV_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

int sv_copy_to_host(sv_ctx* c, void* dst, const void* src, uint64_t bytes, void* stream) {
    SV_ENTER(c);
    if (!dst || !src) return fail(SV_EINVAL, "null pointer");
    if (!bytes) return 0;
    if (stream) {
        SV_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, static_cast<hipStream_t>(stream)));
        return 0;
    }
    SV_HIP(hipStreamSynchronize(c->stream));   // results of enqueued device work
    SV_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, c->stream));
    SV_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

// ---------------------------------------------------------------- profiling
int sv_profile_enable(sv_ctx* c, int on) {
    SV_ENTER(c);
    c->prof = on != 0;
    // create the events up front: hipEventCreate inside a timed loop costs host time
    while (c->prof && c->pool.size() + 2 * c->pending.size() < 1024) {
        hipEvent_t e = nullptr;
        if (hipEventCreate(&e) != hipSuccess) break;
        c->pool.push_back(e);
    }
    return 0;
}

int sv_profile_read(sv_ctx* c, int kernel, double* total_ms, long long* count) {
    SV_ENTER(c);
    if (kernel < 0 || kernel >= SV_NKERNELS) return fail(SV_EINVAL, "kernel id out of range");
    c->prof_drain();
    if (total_ms) *total_ms = c->acc_ms[kernel];
    if (count) *count = c->cnt[kernel];
    return 0;
}

int sv_timer_begin(sv_ctx* c, void* stream) {
    SV_ENTER(c);
    for (auto& e : c->tmr)
        if (!e) SV_HIP(hipEventCreate(&e));
    SV_HIP(hipEventRecord(c->tmr[0], pick(c, stream)));
    return 0;
}

int sv_timer_end(sv_ctx* c, void* stream, double* ms) {
    SV_ENTER(c);
    if (!c->tmr[0] || !ms) return fail(SV_EINVAL, "sv_timer_end without sv_timer_begin");
    SV_HIP(hipEventRecord(c->tmr[1], pick(c, stream)));
    SV_HIP(hipEventSynchronize(c->tmr[1]));
    float f = 0.f;
    SV_HIP(hipEventElapsedTime(&f, c->tmr[0], c->tmr[1]));
    *ms = f;
    return 0;
}

int sv_profile_region_begin(sv_ctx* c, int kernel, void* stream) {
    SV_ENTER(c);
    if (kernel < 0 || kernel >= SV_NKERNELS) return fail(SV_EINVAL, "kernel id out of range");
    if (c->region_open) return fail(SV_EINVAL, "profiling regions do not nest");
    if (!c->prof) return 0;
    c->region.a = c->get_event();
    c->region.b = c->get_event();
    c->region.kid = kernel;
    SV_HIP(hipEventRecord(c->region.a, pick(c, stream)));
    c->region_open = true;
    return 0;
}

int sv_profile_region_end(sv_ctx* c, void* stream) {
    SV_ENTER(c);
    if (!c->region_open) return 0;   // profiling was off at the matching begin
    c->region_open = false;
    SV_HIP(hipEventRecord(c->region.b, pick(c, stream)));
    c->pending.push_back(c->region);
    return 0;
}

int sv_profile_reset(sv_ctx* c) {
    SV_ENTER(c);
    c->prof_drain();
    for (int k = 0; k < SV_NKERNELS; ++k) {
        c->acc_ms[k] = 0.0;
        c->cnt[k] = 0;
    }
    return 0;
}

}  // extern "C"
