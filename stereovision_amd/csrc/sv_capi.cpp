// sv_capi.cpp — the C ABI (include/stereovision_amd.h) over the gfx950 kernels.
//
// A context = one device + one HIP stream + grow-only device buffers + pinned staging.
// Host entry points stage into pinned memory, run the whole chain on the context stream
// and copy results back; device entry points only enqueue.  No exception crosses the ABI.
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <new>
#include <string>
#include <vector>

#include "sv_internal.h"
#include "sv_pool.h"
#include "../../include/stereovision_amd.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

}  // namespace

int sv::set_error(int code, const std::string& msg) { return fail(code, msg); }

namespace {

int hipfail(int e, const char* what) {
    return fail(SV_EHIP, std::string(what) + ": " + hipGetErrorString((hipError_t)e));
}

#define SV_HIP(call)                                               \
    do {                                                           \
        hipError_t e_ = (call);                                    \
        if (e_ != hipSuccess) return hipfail((int)e_, #call);      \
    } while (0)

#define SV_LAUNCH(ctx, kid, stream, call)                          \
    do {                                                           \
        (ctx)->prof_begin((kid), (stream));                        \
        int e_ = (call);                                           \
        if (e_ != 0) return hipfail(e_, #call);                    \
        (ctx)->prof_end((stream));                                 \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) cap = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    // for self-cleaning accumulators (the kernels that read them zero them again)
    hipError_t ensure_zeroed(size_t n) {
        if (n <= cap) return hipSuccess;
        hipError_t e = ensure(n);
        if (e == hipSuccess) e = hipMemset(p, 0, cap);
        if (e == hipSuccess) e = hipDeviceSynchronize();
        return e;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipHostMalloc(&p, n, hipHostMallocDefault);
        if (e == hipSuccess) cap = n;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

struct EvPair {
    hipEvent_t a, b;
    int kid;
};

}  // namespace

// one entry of the host copy of the post-processing table (host-buffer frame path)
struct HostEnt {
    float a;          // depth_final / disparity_normalized
    uint32_t ubgr;    // u8 | B << 8 | G << 16 | R << 24
};

struct sv_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    DevBuf wctr;   // persistent matcher's work counters (zeroed once; the kernel resets them)
    DevBuf img[2], gray[2], d16, fa, fb, fc, u8, harris, hog[2], fin, lut, rmap1, rmap2, rdst[2], stats, sel,
        sg_hsum, sg_c, sg_l, sg_lt, sg_band, sg_rec, cc_parent, cc_size, hist_copies, cmap, bgr;
    uint8_t cmap_host[768] = {};   // BGR table currently in `cmap`
    bool cmap_valid = false;
    // host-buffer frame path: int16 medians come back over PCIe and are expanded on the
    // host with a host copy of the post-processing table (hl_*, valid for hl_key)
    DevBuf m16;
    // multi-device entry points: int16 x16 medians a context sends to the root (peers) or
    // receives from the peers (root), 2 B/px over xGMI
    DevBuf gm16;
    DevBuf keys;       // split ring kind (SAD, D > 256): two argmin-key planes
    std::vector<float> hl_a, hl_b;
    std::vector<uint8_t> hl_u8;
    std::vector<HostEnt> hl_ent;
    bool hl_valid = false;
    // host-buffer frame path: `dev_done[k]` marks the arrival of output piece k
    hipEvent_t dev_done[8] = {};
    hipEvent_t tmr[2] = {nullptr, nullptr};   // sv_timer_begin / sv_timer_end
    // SGBM: second stream + fork/join events for the vertical path beside the horizontal ones
    hipStream_t sg_aux = nullptr;
    hipEvent_t sg_ev[2] = {nullptr, nullptr};
    // cached post-processing table: key = (mode, params, range); `lut_ev` marks its build
    struct LutKey {
        int mode = -1, min_disp = 0, num_disp = 0, m0 = 0, n = 0;
        float minf = 0, maxf = 0, rangef = 0, mdg = 0;
        bool operator==(const LutKey& o) const {
            return mode == o.mode && min_disp == o.min_disp && num_disp == o.num_disp && m0 == o.m0 &&
                   n == o.n && std::memcmp(&minf, &o.minf, sizeof(float)) == 0 &&
                   std::memcmp(&maxf, &o.maxf, sizeof(float)) == 0 &&
                   std::memcmp(&rangef, &o.rangef, sizeof(float)) == 0 &&
                   std::memcmp(&mdg, &o.mdg, sizeof(float)) == 0;
        }
    } lut_key, hl_key;
    hipEvent_t lut_ev = nullptr;
    hipStream_t lut_stream = nullptr;   // stream the table was built on
    // the whole-disparity table (lut_shift 4: integer-cost depth-map batches), cached apart
    DevBuf lutw;
    LutKey lutw_key;
    hipEvent_t lutw_ev = nullptr;
    hipStream_t lutw_stream = nullptr;
    HostBuf hin, hout;
    // Cross-stream ordering of the context's scratch (d16, the post table, HOG histograms,
    // SGBM volumes, reduction accumulators): `*_dev` calls may pass any stream, so a call on
    // stream s first waits for the event recorded after the previous scratch user when that
    // ran on another stream, and records a new one after enqueueing (ScratchUse below).
    hipStream_t scr_stream = nullptr;
    hipEvent_t scr_ev = nullptr;
    hipEvent_t xev = nullptr;   // multi-device entry points: this context's part is enqueued
    hipEvent_t sev = nullptr;   // sv_depth_map_rows_scatter: the root's inputs are ready
    // multi-device entry points (root): recorded on the root stream once the root's previous
    // users of its receive buffer (gm16) are ordered before it; peer copies into gm16 wait
    // for it (RCCL receives run on the root stream and need no event)
    hipEvent_t gev = nullptr;
    hipEvent_t wev[16] = {};    // sv_event_record / sv_stream_wait_event slots
    bool prof = false;
    std::vector<EvPair> pending;
    std::vector<hipEvent_t> pool;
    double acc_ms[SV_NKERNELS] = {};
    long long cnt[SV_NKERNELS] = {};
    EvPair cur{};
    EvPair region{};            // sv_profile_region_begin/end (separate from `cur`: kernels
    bool region_open = false;   // launched inside a region keep their own pairs)

    hipEvent_t get_event() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
    void prof_begin(int kid, hipStream_t s) {
        if (!prof) return;
        cur.a = get_event();
        cur.b = get_event();
        cur.kid = kid;
        (void)hipEventRecord(cur.a, s);
    }
    void prof_end(hipStream_t s) {
        if (!prof) return;
        (void)hipEventRecord(cur.b, s);
        pending.push_back(cur);
    }
    void prof_drain() {
        for (auto& p : pending) {
            (void)hipEventSynchronize(p.b);
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
                acc_ms[p.kid] += ms;
                cnt[p.kid] += 1;
            }
            pool.push_back(p.a);
            pool.push_back(p.b);
        }
        pending.clear();
    }
};

namespace {

inline hipStream_t pick(sv_ctx* c, void* s) { return s ? static_cast<hipStream_t>(s) : c->stream; }

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


struct SgbmParams {
    int P1, P2, disp12, cap, uniq, speckle_win, speckle_range;
};

SgbmParams sgbm_reference_params(int win) {
    // depth_map.py:894-906 / fused_depth_map.py:988-1000
    return {8 * 3 * win * win, 32 * 3 * win * win, 1, 63, 10, 100, 32};
}

// Enqueue the whole SGBM-3WAY pipeline for one frame (buffers grown in the context).
// cv2.filterSpeckles on an int16 device map (speckle stage of SGBM, sv_filter_speckles).
// nf > 1: a batch of maps, map z at d_img + z*fimg (one launch per stage over grid.z).
int enqueue_speckles(sv_ctx* c, int16_t* d_img, int H, int W, int pitch, int new_val, int max_speckle_size,
                     int max_diff, hipStream_t s, int nf = 1, long long fimg = 0) {
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
                 int num_disp, int win, SgbmParams p, int16_t* out, int opitch, hipStream_t s, int nf = 1,
                 long long fs_in = 0, long long fs_out = 0) {
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
                      int16_t* out, int opitch, hipStream_t s, int nf = 1, long long fs_in = 0,
                      long long fs_out = 0) {
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
int attach_lut(sv_ctx* c, sv::PostParams& pp, hipStream_t s, bool whole = false) {
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

// Gather-only outputs of the multi-device entry points: instead of create_depth_map's outputs
// (the root expands the peers' int16 x16 medians with k_post_m16), the full median map lands
// on the root as int16 x16 (SV_MAP_M16) or u8 disparity indices (SV_MAP_D8: median / 16 −
// (min_disp − 1), 1 B/px) and nothing is expanded (sv_post_m16_dev turns it into the outputs).
struct MapOut {
    int fmt = 0;           // 0: create_depth_map outputs on the root
    void* map = nullptr;   // fmt != 0: the root's full map (frames dense, or one frame)
    int d8_base = 0;
    size_t el() const { return fmt == SV_MAP_D8 ? 1 : 2; }
};

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

struct Out {
    void* host;
    const void* dev;
    size_t bytes;
};

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

// RAII: wait for the previous user of the context scratch if it ran on another stream;
// on scope exit (after this call's enqueues) record the event the next user waits for.
struct ScratchUse {
    sv_ctx* c;
    hipStream_t s;
    int rc = 0;
    ScratchUse(sv_ctx* ctx, hipStream_t stream) : c(ctx), s(stream) {
        if (c->scr_stream && c->scr_stream != s && c->scr_ev) {
            hipError_t e = hipStreamWaitEvent(s, c->scr_ev, 0);
            if (e != hipSuccess) rc = hipfail((int)e, "hipStreamWaitEvent (context scratch)");
        }
    }
    ~ScratchUse() {
        if (!c->scr_ev && hipEventCreateWithFlags(&c->scr_ev, hipEventDisableTiming) != hipSuccess) {
            c->scr_ev = nullptr;
            return;
        }
        if (hipEventRecord(c->scr_ev, s) == hipSuccess) c->scr_stream = s;
    }
};

#define SV_SCRATCH(ctx, stream)                                             \
    ScratchUse scratch_(ctx, stream);                                       \
    if (scratch_.rc) return scratch_.rc

struct Guard {
    sv_ctx* c;
    std::unique_lock<std::mutex> lk;
    int rc = 0;
    explicit Guard(sv_ctx* ctx) : c(ctx), lk(ctx->mu) {
        hipError_t e = hipSetDevice(ctx->device);
        if (e != hipSuccess) rc = hipfail((int)e, "hipSetDevice");
    }
};

#define SV_ENTER(ctx)                                                       \
    if (!(ctx)) return fail(SV_EINVAL, "null context");                     \
    Guard guard_(ctx);                                                      \
    if (guard_.rc) return guard_.rc


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

}  // namespace

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

int sv_median_post_dev(sv_ctx* c, const int16_t* d_disp16, int H, int W, int row0, int row1, int mode,
                       float min_depth, float max_depth, float depth_range, float min_disp_global,
                       int min_disp, int num_disp, float* d_disparity, float* d_out_a, uint8_t* d_out_u8,
                       float* d_out_b, void* stream) {
    SV_ENTER(c);
    if (check_image(d_disp16, H, W) || !d_disparity) return fail(SV_EINVAL, "bad median arguments");
    if (mode == SV_POST_DEPTH && (!d_out_a || !d_out_u8)) return fail(SV_EINVAL, "depth post outputs missing");
    if (mode == SV_POST_SCALED && (!d_out_a || !d_out_u8 || !d_out_b || num_disp <= 0))
        return fail(SV_EINVAL, "scaled post outputs missing");
    if (row0 < 0) row0 = 0;
    if (row1 > H) row1 = H;
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    sv::PostParams pp = make_post(mode, min_depth, max_depth, depth_range, min_disp_global, min_disp, num_disp,
                                  d_out_a, d_out_u8, d_out_b);
    int lrc = attach_lut(c, pp, s);
    if (lrc) return lrc;
    SV_LAUNCH(c, SV_K_MEDIAN, s, sv::launch_median_i16(d_disp16, H, W, row0, row1, d_disparity, pp, s));
    return 0;
}

int sv_median_post_m16_dev(sv_ctx* c, const int16_t* d_disp16, int H, int W, int row0, int row1, int mode,
                           float min_depth, float max_depth, float depth_range, float min_disp_global,
                           int min_disp, int num_disp, float* d_disparity, float* d_out_a, uint8_t* d_out_u8,
                           float* d_out_b, int16_t* d_med16, void* stream) {
    SV_ENTER(c);
    if (check_image(d_disp16, H, W) || (!d_disparity && !d_med16)) return fail(SV_EINVAL, "bad median arguments");
    if (mode != SV_POST_NONE && mode != SV_POST_DEPTH && mode != SV_POST_SCALED) return fail(SV_EINVAL, "bad mode");
    if (mode == SV_POST_DEPTH && (!d_out_a || !d_out_u8)) return fail(SV_EINVAL, "depth post outputs missing");
    if (mode == SV_POST_SCALED && (!d_out_a || !d_out_u8 || !d_out_b || num_disp <= 0))
        return fail(SV_EINVAL, "scaled post outputs missing");
    if ((long long)H * W >= (1LL << 30)) return fail(SV_EINVAL, "frame too large for the median kernel");
    if (row0 < 0) row0 = 0;
    if (row1 > H) row1 = H;
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    sv::PostParams pp = make_post(mode, min_depth, max_depth, depth_range, min_disp_global, min_disp, num_disp,
                                  d_out_a, d_out_u8, d_out_b);
    int lrc = attach_lut(c, pp, s);
    if (lrc) return lrc;
    pp.out_m16 = d_med16;
    SV_LAUNCH(c, SV_K_MEDIAN, s, sv::launch_median_i16(d_disp16, H, W, row0, row1, d_disparity, pp, s));
    return 0;
}

int sv_median_map_dev(sv_ctx* c, const int16_t* d_disp16, int H, int W, int row0, int row1, int map_format,
                      int min_disp, int num_disp, void* d_map, void* stream) {
    SV_ENTER(c);
    if (check_image(d_disp16, H, W)) return fail(SV_EINVAL, "bad median arguments");
    int rc = check_map(map_format, d_map, SV_COST_SAD, num_disp);
    if (rc) return rc;
    if ((long long)H * W >= (1LL << 30)) return fail(SV_EINVAL, "frame too large for the median kernel");
    if (row0 < 0) row0 = 0;
    if (row1 > H) row1 = H;
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    sv::PostParams pp = map_post(map_format, d_map, min_disp - 1);
    SV_LAUNCH(c, SV_K_MEDIAN, s, sv::launch_median_i16(d_disp16, H, W, row0, row1, nullptr, pp, s));
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

int sv_median_post_color_dev(sv_ctx* c, const int16_t* d_disp16, int H, int W, int row0, int row1, int mode,
                             float min_depth, float max_depth, float depth_range, float min_disp_global,
                             int min_disp, int num_disp, const uint8_t* cmap_bgr, float* d_disparity,
                             float* d_out_a, uint8_t* d_out_u8, float* d_out_b, uint8_t* d_bgr, void* stream) {
    SV_ENTER(c);
    if (check_image(d_disp16, H, W) || !d_out_a || !d_out_u8 || !d_bgr || !cmap_bgr)
        return fail(SV_EINVAL, "bad median arguments");
    if (mode != SV_POST_DEPTH && mode != SV_POST_SCALED) return fail(SV_EINVAL, "mode must be DEPTH or SCALED");
    if (mode == SV_POST_SCALED && (!d_out_b || num_disp <= 0)) return fail(SV_EINVAL, "scaled post outputs missing");
    if (row0 < 0) row0 = 0;
    if (row1 > H) row1 = H;
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    sv::PostParams pp = make_post(mode, min_depth, max_depth, depth_range, min_disp_global, min_disp, num_disp,
                                  d_out_a, d_out_u8, d_out_b);
    int rc = attach_lut(c, pp, s);
    if (!rc) rc = attach_cmap(c, pp, cmap_bgr, d_bgr, s);
    if (rc) return rc;
    SV_LAUNCH(c, SV_K_MEDIAN, s, sv::launch_median_i16(d_disp16, H, W, row0, row1, d_disparity, pp, s));
    return 0;
}

int sv_depth_map_dev(sv_ctx* c, const uint8_t* d_left, const uint8_t* d_right, int H, int W, int pitch,
                     int min_disp, int num_disp, int win, int cost, float min_depth, float max_depth,
                     float depth_range, float min_disp_global, float* d_depth, float* d_disparity,
                     uint8_t* d_norm, void* stream) {
    SV_ENTER(c);
    if (check_image(d_left, H, W) || check_image(d_right, H, W) || !d_depth || !d_disparity || !d_norm)
        return fail(SV_EINVAL, "bad depth-map arguments");
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    SV_HIP(c->d16.ensure((size_t)H * W * sizeof(int16_t)));
    int rc = enqueue_disparity(c, d_left, d_right, H, W, pitch, min_disp, num_disp, win, cost, 0, H,
                               c->d16.as<int16_t>(), W, s);
    if (rc) return rc;
    sv::PostParams pp = make_post(SV_POST_DEPTH, min_depth, max_depth, depth_range, min_disp_global, min_disp,
                                  num_disp, d_depth, d_norm, nullptr);
    rc = attach_lut(c, pp, s);
    if (rc) return rc;
    SV_LAUNCH(c, SV_K_MEDIAN, s, sv::launch_median_i16(c->d16.as<int16_t>(), H, W, 0, H, d_disparity, pp, s));
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

int sv_median_post_batch_dev(sv_ctx* c, const int16_t* d_disp16, int n_frames, int H, int W, int mode,
                             float min_depth, float max_depth, float depth_range, float min_disp_global,
                             int min_disp, int num_disp, float* d_disparity, float* d_out_a,
                             uint8_t* d_out_u8, float* d_out_b, void* stream) {
    SV_ENTER(c);
    if (check_image(d_disp16, H, W) || !d_disparity || n_frames < 0) return fail(SV_EINVAL, "bad median arguments");
    if (mode == SV_POST_DEPTH && (!d_out_a || !d_out_u8)) return fail(SV_EINVAL, "depth post outputs missing");
    if (mode == SV_POST_SCALED && (!d_out_a || !d_out_u8 || !d_out_b || num_disp <= 0))
        return fail(SV_EINVAL, "scaled post outputs missing");
    if (n_frames == 0) return 0;
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    sv::PostParams pp = make_post(mode, min_depth, max_depth, depth_range, min_disp_global, min_disp, num_disp,
                                  d_out_a, d_out_u8, d_out_b);
    int rc = attach_lut(c, pp, s);
    if (rc) return rc;
    const long long fs = (long long)H * W;
    SV_LAUNCH(c, SV_K_MEDIAN, s, sv::launch_median_i16(d_disp16, H, W, 0, H, d_disparity, pp, s, n_frames, fs, fs));
    return 0;
}

int sv_depth_map_batch_dev(sv_ctx* c, const uint8_t* d_left, const uint8_t* d_right, int n_frames, int H, int W,
                           int pitch, int64_t frame_stride, int min_disp, int num_disp, int win, int cost,
                           float min_depth, float max_depth, float depth_range, float min_disp_global,
                           float* d_depth, float* d_disparity, uint8_t* d_norm, void* stream) {
    return sv_depth_map_batch_m16_dev(c, d_left, d_right, n_frames, H, W, pitch, frame_stride, min_disp, num_disp,
                                      win, cost, min_depth, max_depth, depth_range, min_disp_global, d_depth,
                                      d_disparity, d_norm, nullptr, stream);
}

int sv_depth_map_batch_m16_dev(sv_ctx* c, const uint8_t* d_left, const uint8_t* d_right, int n_frames, int H,
                               int W, int pitch, int64_t frame_stride, int min_disp, int num_disp, int win,
                               int cost, float min_depth, float max_depth, float depth_range,
                               float min_disp_global, float* d_depth, float* d_disparity, uint8_t* d_norm,
                               int16_t* d_med16, void* stream) {
    SV_ENTER(c);
    if (check_image(d_left, H, W) || check_image(d_right, H, W) || !d_depth || !d_disparity || !d_norm ||
        n_frames < 0)
        return fail(SV_EINVAL, "bad depth-map arguments");
    if (pitch < W) return fail(SV_EINVAL, "pitch smaller than width");
    if (n_frames > 1 && frame_stride < (int64_t)pitch * H) return fail(SV_EINVAL, "frame stride smaller than a frame");
    if (n_frames == 0) return 0;
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    const long long fs = (long long)H * W;
    SV_HIP(c->d16.ensure((size_t)n_frames * fs * sizeof(int16_t)));
    int rc = enqueue_disparity(c, d_left, d_right, H, W, pitch, min_disp, num_disp, win, cost, 0, H,
                               c->d16.as<int16_t>(), W, s, n_frames, frame_stride, fs);
    if (rc) return rc;
    sv::PostParams pp = make_post(SV_POST_DEPTH, min_depth, max_depth, depth_range, min_disp_global, min_disp,
                                  num_disp, d_depth, d_norm, nullptr);
    rc = attach_lut(c, pp, s, cost != SV_COST_SGBM);
    if (rc) return rc;
    pp.out_m16 = d_med16;   // nullable: the int16 x16 medians beside the f32 disparity
    SV_LAUNCH(c, SV_K_MEDIAN, s,
              sv::launch_median_i16(c->d16.as<int16_t>(), H, W, 0, H, d_disparity, pp, s, n_frames, fs, fs));
    return 0;
}

int sv_depth_map_batch_d8_dev(sv_ctx* c, const uint8_t* d_left, const uint8_t* d_right, int n_frames, int H, int W,
                              int pitch, int64_t frame_stride, int min_disp, int num_disp, int win, int cost,
                              float min_depth, float max_depth, float depth_range, float min_disp_global,
                              float* d_depth, float* d_disparity, uint8_t* d_norm, uint8_t* d_d8, void* stream) {
    SV_ENTER(c);
    if (check_image(d_left, H, W) || check_image(d_right, H, W) || !d_depth || !d_disparity || !d_norm || !d_d8 ||
        n_frames < 0)
        return fail(SV_EINVAL, "bad depth-map arguments");
    if (cost == SV_COST_SGBM || num_disp < 1 || num_disp > 255)
        return fail(SV_EINVAL, "u8 disparity indices need an integer-disparity cost and num_disp <= 255");
    if (pitch < W) return fail(SV_EINVAL, "pitch smaller than width");
    if (n_frames > 1 && frame_stride < (int64_t)pitch * H) return fail(SV_EINVAL, "frame stride smaller than a frame");
    if (n_frames == 0) return 0;
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    const long long fs = (long long)H * W;
    SV_HIP(c->d16.ensure((size_t)n_frames * fs * sizeof(int16_t)));
    int rc = enqueue_disparity(c, d_left, d_right, H, W, pitch, min_disp, num_disp, win, cost, 0, H,
                               c->d16.as<int16_t>(), W, s, n_frames, frame_stride, fs);
    if (rc) return rc;
    sv::PostParams pp = make_post(SV_POST_DEPTH, min_depth, max_depth, depth_range, min_disp_global, min_disp,
                                  num_disp, d_depth, d_norm, nullptr);
    rc = attach_lut(c, pp, s, cost != SV_COST_SGBM);
    if (rc) return rc;
    pp.out_d8 = d_d8;   // median / 16 - (min_disp - 1): 0 = invalid, 1 + d - min_disp otherwise
    pp.d8_base = min_disp - 1;
    SV_LAUNCH(c, SV_K_MEDIAN, s,
              sv::launch_median_i16(c->d16.as<int16_t>(), H, W, 0, H, d_disparity, pp, s, n_frames, fs, fs));
    return 0;
}

int sv_depth_map_harris_batch_dev(sv_ctx* c, const uint8_t* d_left, const uint8_t* d_right, int n_frames, int H,
                                  int W, int pitch, int64_t frame_stride, int min_disp, int num_disp, int win,
                                  int cost, float min_depth, float max_depth, float depth_range,
                                  float min_disp_global, float* d_depth, float* d_disparity, uint8_t* d_norm,
                                  float* d_harris, void* stream) {
    SV_ENTER(c);
    if (check_image(d_left, H, W) || check_image(d_right, H, W) || !d_depth || !d_disparity || !d_norm ||
        !d_harris || n_frames < 0)
        return fail(SV_EINVAL, "bad depth-map arguments");
    if (pitch < W) return fail(SV_EINVAL, "pitch smaller than width");
    if (n_frames > 1 && frame_stride < (int64_t)pitch * H) return fail(SV_EINVAL, "frame stride smaller than a frame");
    if (n_frames == 0) return 0;
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    const long long fs = (long long)H * W;
    SV_HIP(c->d16.ensure((size_t)n_frames * fs * sizeof(int16_t)));
    int rc = enqueue_disparity(c, d_left, d_right, H, W, pitch, min_disp, num_disp, win, cost, 0, H,
                               c->d16.as<int16_t>(), W, s, n_frames, frame_stride, fs);
    if (rc) return rc;
    sv::PostParams pp = make_post(SV_POST_DEPTH, min_depth, max_depth, depth_range, min_disp_global, min_disp,
                                  num_disp, d_depth, d_norm, nullptr);
    rc = attach_lut(c, pp, s, cost != SV_COST_SGBM);
    if (rc) return rc;
    const long long fin = n_frames > 1 ? frame_stride : 0;
    if (W >= 8 && H >= 8) {   // the Harris response rides in the median launch (extra blocks)
        sv::HarrisParams hp{d_left, pitch, fin, d_harris, fs, 0};
        SV_LAUNCH(c, SV_K_MEDIAN, s,
                  sv::launch_median_i16(c->d16.as<int16_t>(), H, W, 0, H, d_disparity, pp, s, n_frames, fs, fs, &hp));
        return 0;
    }
    SV_LAUNCH(c, SV_K_MEDIAN, s,
              sv::launch_median_i16(c->d16.as<int16_t>(), H, W, 0, H, d_disparity, pp, s, n_frames, fs, fs));
    SV_LAUNCH(c, SV_K_HARRIS, s, sv::launch_harris(d_left, H, W, pitch, d_harris, s, n_frames, fin, fs));
    return 0;
}

// One shard of sv_multi_gpu_batch: frames [f0, f1) on context c (host buffers in and out).
namespace {
int check_contexts(sv_ctx* const* ctxs, int ndev) {
    if (!ctxs || ndev < 1) return fail(SV_EINVAL, "no contexts");
    for (int k = 0; k < ndev; ++k) {
        if (!ctxs[k]) return fail(SV_EINVAL, "null context");
        for (int j = 0; j < k; ++j)
            if (ctxs[j] == ctxs[k]) return fail(SV_EINVAL, "a context appears twice");
    }
    return 0;
}

int depth_map_shard(sv_ctx* c, const uint8_t* left, const uint8_t* right, int f0, int f1, int H, int W,
                    int channels, int min_disp, int num_disp, int win, int cost, float min_depth,
                    float max_depth, float depth_range, float min_disp_global, float* depth_final,
                    float* disparity, uint8_t* depth_normalized) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    const int nf = f1 - f0;
    if (nf <= 0) return 0;
    const size_t n = (size_t)H * W, fin = n * channels;
    // host frames -> pinned staging -> device (one copy per camera for the whole shard)
    SV_HIP(c->hin.ensure(2 * nf * fin));
    SV_HIP(c->gray[0].ensure(nf * n));
    SV_HIP(c->gray[1].ensure(nf * n));
    const uint8_t* src[2] = {left, right};
    for (int k = 0; k < 2; ++k) {
        uint8_t* stage = c->hin.as<uint8_t>() + k * nf * fin;
        std::memcpy(stage, src[k] + (size_t)f0 * fin, nf * fin);
        if (channels == 1) {
            SV_HIP(hipMemcpyAsync(c->gray[k].p, stage, nf * fin, hipMemcpyHostToDevice, c->stream));
        } else {
            SV_HIP(c->img[k].ensure(nf * fin));
            SV_HIP(hipMemcpyAsync(c->img[k].p, stage, nf * fin, hipMemcpyHostToDevice, c->stream));
            // contiguous frames: the shard's BGR stack is one (nf*H) x W image, one launch
            SV_LAUNCH(c, SV_K_GRAY, c->stream,
                      sv::launch_gray(c->img[k].as<uint8_t>(), nf * H, W, W * channels, c->gray[k].as<uint8_t>(),
                                      c->stream));
        }
    }
    SV_HIP(c->d16.ensure(nf * n * sizeof(int16_t)));
    SV_HIP(c->fa.ensure(nf * n * sizeof(float)));
    SV_HIP(c->fb.ensure(nf * n * sizeof(float)));
    SV_HIP(c->u8.ensure(nf * n));
    int rc = enqueue_disparity(c, c->gray[0].as<uint8_t>(), c->gray[1].as<uint8_t>(), H, W, W, min_disp, num_disp,
                               win, cost, 0, H, c->d16.as<int16_t>(), W, c->stream, nf, (long long)n, (long long)n);
    if (rc) return rc;
    sv::PostParams pp = make_post(SV_POST_DEPTH, min_depth, max_depth, depth_range, min_disp_global, min_disp,
                                  num_disp, c->fb.as<float>(), c->u8.as<uint8_t>(), nullptr);
    rc = attach_lut(c, pp, c->stream);
    if (rc) return rc;
    SV_LAUNCH(c, SV_K_MEDIAN, c->stream,
              sv::launch_median_i16(c->d16.as<int16_t>(), H, W, 0, H, c->fa.as<float>(), pp, c->stream, nf,
                                    (long long)n, (long long)n));
    Out o[] = {{depth_final + (size_t)f0 * n, c->fb.p, nf * n * sizeof(float)},
               {disparity + (size_t)f0 * n, c->fa.p, nf * n * sizeof(float)},
               {depth_normalized + (size_t)f0 * n, c->u8.p, nf * n}};
    return collect(c, o, 3);
}
}  // namespace

int sv_multi_gpu_batch(sv_ctx* const* ctxs, int ndev, const uint8_t* left, const uint8_t* right, int n_frames,
                       int H, int W, int channels, int min_disp, int num_disp, int win, int cost, float min_depth,
                       float max_depth, float depth_range, float min_disp_global, float* depth_final,
                       float* disparity, uint8_t* depth_normalized) {
    int rc = check_contexts(ctxs, ndev);
    if (rc) return rc;
    if (n_frames < 0) return fail(SV_EINVAL, "negative frame count");
    if (n_frames == 0) return 0;
    if (!left || !right || !depth_final || !disparity || !depth_normalized) return fail(SV_EINVAL, "null buffers");
    if (channels != 1 && channels != 3) return fail(SV_EINVAL, "channels must be 1 or 3");
    sv::MatchPlan plan;
    rc = check_match(H, W, min_disp, num_disp, win, cost, &plan);
    if (rc) return rc;
    // contiguous shards, one host thread per context: each stages, computes and collects
    // its frames on its own device/stream concurrently with the others (every device
    // returns its shard over its own PCIe link).  No C++ exception may cross the ABI: any
    // allocation or thread-start failure becomes SV_ENOMEM.
    int spawn_rc = 0;
    std::vector<int> rcs;
    std::vector<std::string> errs;
    std::vector<std::thread> th;
    try {
        rcs.assign(ndev, 0);
        errs.resize(ndev);
        th.reserve(ndev);
        for (int k = 0; k < ndev; ++k) {
            const int f0 = (int)((long long)n_frames * k / ndev), f1 = (int)((long long)n_frames * (k + 1) / ndev);
            th.emplace_back([&, k, f0, f1]() noexcept {
                try {
                    rcs[k] = depth_map_shard(ctxs[k], left, right, f0, f1, H, W, channels, min_disp, num_disp, win,
                                             cost, min_depth, max_depth, depth_range, min_disp_global, depth_final,
                                             disparity, depth_normalized);
                    if (rcs[k]) errs[k] = g_err;
                } catch (...) {
                    rcs[k] = SV_ENOMEM;
                }
            });
        }
    } catch (...) {
        spawn_rc = SV_ENOMEM;
    }
    for (auto& t : th) t.join();
    if (spawn_rc) return fail(spawn_rc, "could not start the per-device host threads");
    for (int k = 0; k < ndev; ++k)
        if (rcs[k]) return fail(rcs[k], "device shard " + std::to_string(k) + ": " + errs[k]);
    return 0;
}

namespace {

// Locks every context of a multi-device call (in address order: no lock-order inversion
// between concurrent calls over overlapping context sets).
struct MultiLock {
    std::vector<std::unique_lock<std::mutex>> locks;
    bool ok = true;
    MultiLock(sv_ctx* const* ctxs, int n) {
        try {
            std::vector<sv_ctx*> v(ctxs, ctxs + n);
            std::sort(v.begin(), v.end());
            for (sv_ctx* c : v) locks.emplace_back(c->mu);
        } catch (...) {
            ok = false;
        }
    }
};

// Row bands of a row-tiled frame: output rows [r0, r1) of `rank`,
// disparity rows [h0, h1) (+ the 5x5 median's 2-row halo) and the input rows [in0, in1) the
// kernels read for them: the matching window's r rows, the four-row waves' 3 extra rows below
// a band's last row and the HOG histograms' Sobel row (r + 4 each side, clamped).
struct SvRows {
    int r0 = 0, r1 = 0, h0 = 0, h1 = 0, in0 = 0, in1 = 0;
};
void band_rows_of(int H, int rank, int world, int win, SvRows& b) {
    b.r0 = (int)((long long)H * rank / world);
    b.r1 = (int)((long long)H * (rank + 1) / world);
    b.h0 = b.r0 - 2 > 0 ? b.r0 - 2 : 0;
    b.h1 = b.r1 + 2 < H ? b.r1 + 2 : H;
    const int halo = win / 2 + 4;
    b.in0 = b.h0 - halo > 0 ? b.h0 - halo : 0;
    b.in1 = b.h1 + halo < H ? b.h1 + halo : H;
}

// Scratch hazard (ScratchUse) for an explicit device/stream, and the join event.
int scratch_wait(sv_ctx* c, hipStream_t s) {
    if (c->scr_stream && c->scr_stream != s && c->scr_ev) SV_HIP(hipStreamWaitEvent(s, c->scr_ev, 0));
    return 0;
}
int scratch_mark(sv_ctx* c, hipStream_t s) {
    if (!c->scr_ev) SV_HIP(hipEventCreateWithFlags(&c->scr_ev, hipEventDisableTiming));
    SV_HIP(hipEventRecord(c->scr_ev, s));
    c->scr_stream = s;
    return 0;
}
// The root's receive buffers are free once its stream reaches this point (every earlier
// reader of gm16 / the caller's map is on the root stream, ordered by scratch_wait): peer
// copies of the gather wait for it.
int recv_ready(sv_ctx* root) {
    if (!root->gev) SV_HIP(hipEventCreateWithFlags(&root->gev, hipEventDisableTiming));
    SV_HIP(hipEventRecord(root->gev, root->stream));
    return 0;
}
int join_event(sv_ctx* c, hipStream_t s) {
    if (!c->xev) SV_HIP(hipEventCreateWithFlags(&c->xev, hipEventDisableTiming));
    SV_HIP(hipEventRecord(c->xev, s));
    return 0;
}

int check_comms(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev) {
    if (!comms) return 0;
    for (int k = 0; k < ndev; ++k) {
        if (!comms[k]) return fail(SV_EINVAL, "comms[k] is null");
        if (sv::comm_device(comms[k]) != ctxs[k]->device || sv::comm_rank(comms[k]) != k ||
            sv::comm_size(comms[k]) != ndev)
            return fail(SV_EINVAL, "comms[k] must be rank k of an ndev-rank communicator on ctxs[k]'s device");
    }
    return 0;
}

// One block (device bytes) of context k -> the root's buffer, by peer copy on k's stream.
int peer_copy(sv_ctx* root, sv_ctx* c, void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (!bytes) return 0;
    if (c->device == root->device) {
        SV_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
    } else {
        SV_HIP(hipMemcpyPeerAsync(dst, root->device, src, c->device, bytes, s));
    }
    return 0;
}

int enable_peer(int from, int to) {
    if (from == to) return 0;
    int can = 0;
    SV_HIP(hipDeviceCanAccessPeer(&can, from, to));
    if (!can) return 0;   // hipMemcpyPeerAsync still works (staged by the runtime)
    SV_HIP(hipSetDevice(from));
    hipError_t e = hipDeviceEnablePeerAccess(to, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return hipfail((int)e, "hipDeviceEnablePeerAccess");
    (void)hipGetLastError();   // clear the sticky "already enabled"
    return 0;
}

struct Block {
    void* dst;        // on the root device
    const void* src;  // on context k's device
    size_t bytes;
};

// Gather the blocks of contexts 1..ndev-1 into the root's buffers: RCCL send/recv in one
// group (comms) or peer copies; the root stream then waits for every part.
int gather_blocks_impl(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev,
                       const std::vector<std::vector<Block>>& blocks);

// ... timed on the root stream as SV_K_GATHER (from the point where the root's own work is
// enqueued to the last part's arrival: includes waiting for the slowest context), and every
// context's scratch-ready event recorded AFTER its sends / peer copies were enqueued, so a
// later call on another stream cannot overwrite fa/fb/u8 while the gather still reads them.
int gather_blocks(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev, const std::vector<std::vector<Block>>& blocks,
                  const std::vector<int>& active) {
    sv_ctx* root = ctxs[0];
    SV_HIP(hipSetDevice(root->device));
    const bool timed = ndev > 1 && root->prof && !root->region_open;
    if (timed) root->prof_begin(SV_K_GATHER, root->stream);
    int rc = gather_blocks_impl(ctxs, comms, ndev, blocks);
    if (rc) return rc;
    SV_HIP(hipSetDevice(root->device));
    if (timed) root->prof_end(root->stream);
    for (int k : active) {
        SV_HIP(hipSetDevice(ctxs[k]->device));
        rc = scratch_mark(ctxs[k], ctxs[k]->stream);
        if (rc) return rc;
    }
    SV_HIP(hipSetDevice(root->device));
    return 0;
}

int gather_blocks_impl(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev,
                       const std::vector<std::vector<Block>>& blocks) {
    sv_ctx* root = ctxs[0];
    if (comms && ndev > 1) {
        int rc = sv::comm_group_start();
        if (rc) return rc;
        int erc = 0;
        for (int k = 1; k < ndev && !erc; ++k)
            for (const Block& b : blocks[k]) {
                if (!b.bytes) continue;
                erc = sv::comm_send(comms[k], b.src, b.bytes, 0, ctxs[k]->stream);
                if (!erc) erc = sv::comm_recv(comms[0], b.dst, b.bytes, k, root->stream);
                if (erc) break;
            }
        rc = sv::comm_group_end();
        if (erc) return erc;
        if (rc) return rc;
        return 0;
    }
    for (int k = 1; k < ndev; ++k) {
        sv_ctx* c = ctxs[k];
        SV_HIP(hipSetDevice(c->device));
        // the root's receive buffer may still be read by an earlier call's work on the root
        // stream (the expansion of the previous gather): copy only after it (recv_ready)
        if (root->gev) SV_HIP(hipStreamWaitEvent(c->stream, root->gev, 0));
        for (const Block& b : blocks[k]) {
            int rc = peer_copy(root, c, b.dst, b.src, b.bytes, c->stream);
            if (rc) return rc;
        }
        int rc = join_event(c, c->stream);
        if (rc) return rc;
    }
    SV_HIP(hipSetDevice(root->device));
    for (int k = 1; k < ndev; ++k) SV_HIP(hipStreamWaitEvent(root->stream, ctxs[k]->xev, 0));
    return 0;
}

// The root's expansion of the peers' gathered int16 x16 medians (n pixels at root->gm16 +
// in_off) into the create_depth_map outputs at element offset `off` (k_post_m16 on the root
// stream, after the gather), timed as SV_K_POST.
int expand_on_root(sv_ctx* root, size_t n, size_t in_off, size_t off, float min_depth, float max_depth, float depth_range,
                   float min_disp_global, int min_disp, int num_disp, float* d_depth, float* d_disparity,
                   uint8_t* d_norm) {
    if (!n) return 0;
    SV_HIP(hipSetDevice(root->device));
    sv::PostParams pp = make_post(SV_POST_DEPTH, min_depth, max_depth, depth_range, min_disp_global, min_disp,
                                  num_disp, d_depth + off, d_norm + off, nullptr);
    int rc = attach_lut(root, pp, root->stream);
    if (rc) return rc;
    SV_LAUNCH(root, SV_K_POST, root->stream,
              sv::launch_post_m16(root->gm16.as<int16_t>() + in_off, (long long)n, d_disparity + off, pp,
                                  root->stream));
    return scratch_mark(root, root->stream);
}

// Median (+ post) of output rows [r0, r1) of context k's disparity band: the root writes the
// create_depth_map outputs in place (or, gather-only, its rows of the map), a peer only its
// int16 x16 medians / u8 indices (c->gm16, full-frame layout) for the gather.
int band_median(sv_ctx* c, int k, int H, int W, int r0, int r1, float min_depth, float max_depth, float depth_range,
                float min_disp_global, int min_disp, int num_disp, float* d_depth, float* d_disparity,
                uint8_t* d_norm, const MapOut& mo, hipStream_t s) {
    sv::PostParams pp;
    float* o_disp = nullptr;
    if (k > 0) {
        SV_HIP(c->gm16.ensure((size_t)H * W * sizeof(int16_t)));
        pp = map_post(mo.fmt ? mo.fmt : SV_MAP_M16, c->gm16.p, mo.d8_base);
    } else if (mo.fmt) {
        pp = map_post(mo.fmt, mo.map, mo.d8_base);
    } else {
        pp = make_post(SV_POST_DEPTH, min_depth, max_depth, depth_range, min_disp_global, min_disp, num_disp,
                       d_depth, d_norm, nullptr);
        o_disp = d_disparity;
        int rc = attach_lut(c, pp, s);
        if (rc) return rc;
    }
    SV_LAUNCH(c, SV_K_MEDIAN, s, sv::launch_median_i16(c->d16.as<int16_t>(), H, W, r0, r1, o_disp, pp, s));
    return 0;
}

int multi_prologue(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev) {
    int rc = check_contexts(ctxs, ndev);
    if (rc) return rc;
    rc = check_comms(ctxs, comms, ndev);
    if (rc) return rc;
    if (!comms)
        for (int k = 1; k < ndev; ++k) {
            rc = enable_peer(ctxs[k]->device, ctxs[0]->device);
            if (rc) return rc;
        }
    return 0;
}

}  // namespace

namespace {
// C4 over ndev contexts.  mo.fmt == 0: create_depth_map outputs on the root (its own frames
// written by its median epilogue, the peers' from their gathered int16 x16 medians); else only
// the map of every frame (int16 x16 or u8 indices), gathered into mo.map.
int multi_frames(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev, const uint8_t* const* d_left,
                 const uint8_t* const* d_right, const int* n_frames, int H, int W, int pitch, int64_t frame_stride,
                 int min_disp, int num_disp, int win, int cost, float min_depth, float max_depth, float depth_range,
                 float min_disp_global, float* d_depth, float* d_disparity, uint8_t* d_norm, const MapOut& mo) {
    int rc = multi_prologue(ctxs, comms, ndev);
    if (rc) return rc;
    sv::MatchPlan plan;
    rc = check_match(H, W, min_disp, num_disp, win, cost, &plan);
    if (rc) return rc;
    if (pitch < W) return fail(SV_EINVAL, "pitch smaller than width");
    for (int k = 0; k < ndev; ++k) {
        if (n_frames[k] < 0) return fail(SV_EINVAL, "negative frame count");
        if (n_frames[k] > 0 && (check_image(d_left[k], H, W) || check_image(d_right[k], H, W)))
            return fail(SV_EINVAL, "null frames");
        if (n_frames[k] > 1 && frame_stride < (int64_t)pitch * H) return fail(SV_EINVAL, "frame stride smaller than a frame");
    }
    MultiLock lock(ctxs, ndev);
    if (!lock.ok) return fail(SV_ENOMEM, "lock allocation failed");
    const size_t n = (size_t)H * W;
    std::vector<std::vector<Block>> blocks;
    std::vector<int> active;
    try {
        blocks.resize(ndev);
        active.reserve(ndev);
    } catch (...) {
        return fail(SV_ENOMEM, "allocation failed");
    }
    sv_ctx* root = ctxs[0];
    size_t total = 0;
    for (int k = 0; k < ndev; ++k) total += (size_t)n_frames[k];
    const size_t n0 = (size_t)n_frames[0];   // the root's own frames come first
    const size_t el = mo.fmt ? mo.el() : sizeof(int16_t);
    // the peers' maps land in mo.map (gather-only) or the root's gm16 (frames n0 .. total-1, dense)
    SV_HIP(hipSetDevice(root->device));
    rc = scratch_wait(root, root->stream);
    if (!rc) rc = recv_ready(root);
    if (rc) return rc;
    if (total > n0 && !mo.fmt) SV_HIP(root->gm16.ensure((total - n0) * n * sizeof(int16_t)));
    uint8_t* recv = mo.fmt ? static_cast<uint8_t*>(mo.map) + n0 * n * el : root->gm16.as<uint8_t>();
    size_t f_off = 0;
    for (int k = 0; k < ndev; ++k) {
        sv_ctx* c = ctxs[k];
        const int nf = n_frames[k];
        const size_t off = f_off;
        f_off += (size_t)nf;
        if (nf == 0) continue;
        SV_HIP(hipSetDevice(c->device));
        hipStream_t s = c->stream;
        rc = scratch_wait(c, s);
        if (rc) return rc;
        SV_HIP(c->d16.ensure((size_t)nf * n * sizeof(int16_t)));
        rc = enqueue_disparity(c, d_left[k], d_right[k], H, W, pitch, min_disp, num_disp, win, cost, 0, H,
                               c->d16.as<int16_t>(), W, s, nf, frame_stride, (long long)n);
        if (rc) return rc;
        sv::PostParams pp;
        float* o_disp = nullptr;
        if (k > 0) {   // peers: only the map (2 or 1 B/px), sent to the root
            SV_HIP(c->gm16.ensure((size_t)nf * n * sizeof(int16_t)));
            pp = map_post(mo.fmt ? mo.fmt : SV_MAP_M16, c->gm16.p, mo.d8_base);
        } else if (mo.fmt) {
            pp = map_post(mo.fmt, mo.map, mo.d8_base);
        } else {       // the root's own frames: create_depth_map's outputs in place
            pp = make_post(SV_POST_DEPTH, min_depth, max_depth, depth_range, min_disp_global, min_disp, num_disp,
                           d_depth + off * n, d_norm + off * n, nullptr);
            o_disp = d_disparity + off * n;
            rc = attach_lut(c, pp, s);
            if (rc) return rc;
        }
        SV_LAUNCH(c, SV_K_MEDIAN, s,
                  sv::launch_median_i16(c->d16.as<int16_t>(), H, W, 0, H, o_disp, pp, s, nf, (long long)n,
                                        (long long)n));
        active.push_back(k);
        if (k > 0) blocks[k] = {{recv + (off - n0) * n * el, c->gm16.p, (size_t)nf * n * el}};
    }
    rc = gather_blocks(ctxs, comms, ndev, blocks, active);
    if (rc || mo.fmt) return rc;
    return expand_on_root(root, (total - n0) * n, 0, n0 * n, min_depth, max_depth, depth_range, min_disp_global,
                          min_disp, num_disp, d_depth, d_disparity, d_norm);
}

// C5: one frame row-tiled over ndev contexts.  scatter: the frame is on the root only
// (d_left[0] / d_right[0]) and context k > 0 first receives its band's input rows into its
// scratch; else every context holds the full frame.  Outputs: create_depth_map's (mo.fmt 0,
// the peers' bands expanded on the root) or the gathered map only.
int rows_impl(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev, const uint8_t* const* d_left,
              const uint8_t* const* d_right, bool scatter, int H, int W, int pitch, int min_disp, int num_disp,
              int win, int cost, float min_depth, float max_depth, float depth_range, float min_disp_global,
              float* d_depth, float* d_disparity, uint8_t* d_norm, const MapOut& mo) {
    int rc = multi_prologue(ctxs, comms, ndev);
    if (rc) return rc;
    sv::MatchPlan plan;
    rc = check_match(H, W, min_disp, num_disp, win, cost, &plan);
    if (rc) return rc;
    if (cost == SV_COST_SGBM && ndev > 1) return fail(SV_EINVAL, "SGBM cannot be row-tiled (top-down path)");
    if (pitch < W) return fail(SV_EINVAL, "pitch smaller than width");
    for (int k = 0; k < (scatter ? 1 : ndev); ++k)
        if (check_image(d_left[k], H, W) || check_image(d_right[k], H, W)) return fail(SV_EINVAL, "null frames");
    MultiLock lock(ctxs, ndev);
    if (!lock.ok) return fail(SV_ENOMEM, "lock allocation failed");
    const size_t n = (size_t)H * W;
    std::vector<std::vector<Block>> blocks;
    std::vector<int> active;
    std::vector<SvRows> rows;
    try {
        blocks.resize(ndev);
        active.reserve(ndev);
        rows.resize(ndev);
    } catch (...) {
        return fail(SV_ENOMEM, "allocation failed");
    }
    sv_ctx* root = ctxs[0];
    for (int k = 0; k < ndev; ++k) band_rows_of(H, k, ndev, win, rows[k]);
    SV_HIP(hipSetDevice(root->device));
    rc = scratch_wait(root, root->stream);
    if (!rc) rc = recv_ready(root);
    if (rc) return rc;
    const size_t el = mo.fmt ? mo.el() : sizeof(int16_t);
    if (!mo.fmt) SV_HIP(root->gm16.ensure(n * sizeof(int16_t)));
    uint8_t* recv = mo.fmt ? static_cast<uint8_t*>(mo.map) : root->gm16.as<uint8_t>();
    if (scatter) {
        // 1. context k > 0 receives input rows [in0, in1) of both images into its scratch
        //    (img[0], img[1]: SV_BAND_MARGIN spare rows above and below, never read as data)
        for (int k = 1; k < ndev; ++k) {
            sv_ctx* c = ctxs[k];
            if (rows[k].r1 <= rows[k].r0) continue;
            SV_HIP(hipSetDevice(c->device));
            rc = scratch_wait(c, c->stream);
            if (rc) return rc;
            const size_t bytes = (size_t)(rows[k].in1 - rows[k].in0 + 2 * SV_BAND_MARGIN) * pitch;
            SV_HIP(c->img[0].ensure(bytes));
            SV_HIP(c->img[1].ensure(bytes));
        }
        SV_HIP(hipSetDevice(root->device));
        const bool timed = ndev > 1 && root->prof && !root->region_open;
        if (timed) root->prof_begin(SV_K_SCATTER, root->stream);
        if (comms && ndev > 1) {
            rc = sv::comm_group_start();
            if (rc) return rc;
            int erc = 0;
            for (int k = 1; k < ndev && !erc; ++k) {
                if (rows[k].r1 <= rows[k].r0) continue;
                const size_t off = (size_t)rows[k].in0 * pitch, bytes = (size_t)(rows[k].in1 - rows[k].in0) * pitch;
                for (int i = 0; i < 2 && !erc; ++i) {
                    const uint8_t* src = (i ? d_right[0] : d_left[0]) + off;
                    uint8_t* dst = ctxs[k]->img[i].as<uint8_t>() + (size_t)SV_BAND_MARGIN * pitch;
                    erc = sv::comm_send(comms[0], src, bytes, k, root->stream);
                    if (!erc) erc = sv::comm_recv(comms[k], dst, bytes, 0, ctxs[k]->stream);
                }
            }
            rc = sv::comm_group_end();
            if (erc) return erc;
            if (rc) return rc;
        } else if (ndev > 1) {
            if (!root->sev) SV_HIP(hipEventCreateWithFlags(&root->sev, hipEventDisableTiming));
            SV_HIP(hipEventRecord(root->sev, root->stream));
            for (int k = 1; k < ndev; ++k) {
                sv_ctx* c = ctxs[k];
                if (rows[k].r1 <= rows[k].r0) continue;
                SV_HIP(hipSetDevice(c->device));
                SV_HIP(hipStreamWaitEvent(c->stream, root->sev, 0));
                const size_t off = (size_t)rows[k].in0 * pitch, bytes = (size_t)(rows[k].in1 - rows[k].in0) * pitch;
                for (int i = 0; i < 2; ++i) {
                    rc = peer_copy(c, root, ctxs[k]->img[i].as<uint8_t>() + (size_t)SV_BAND_MARGIN * pitch,
                                   (i ? d_right[0] : d_left[0]) + off, bytes, c->stream);
                    if (rc) return rc;
                }
            }
        }
        SV_HIP(hipSetDevice(root->device));
        if (timed) root->prof_end(root->stream);
    }
    // 2. every context: disparity of its band + median halo, median (+ post) of its band
    for (int k = 0; k < ndev; ++k) {
        sv_ctx* c = ctxs[k];
        const SvRows& b = rows[k];
        if (b.r1 <= b.r0) continue;
        SV_HIP(hipSetDevice(c->device));
        hipStream_t s = c->stream;
        if (k == 0 || !scatter) {
            rc = scratch_wait(c, s);
            if (rc) return rc;
        }
        const uint8_t* L = d_left[scatter ? 0 : k];
        const uint8_t* R = d_right[scatter ? 0 : k];
        if (scatter && k > 0) {
            // band images addressed as full frames: row y of the frame at base + y * pitch for
            // y in [in0, in1) (the kernels clamp rows to [0, H) and read only [in0, in1))
            const ptrdiff_t shift = ((ptrdiff_t)SV_BAND_MARGIN - b.in0) * pitch;
            L = c->img[0].as<uint8_t>() + shift;
            R = c->img[1].as<uint8_t>() + shift;
        }
        SV_HIP(c->d16.ensure(n * sizeof(int16_t)));
        rc = enqueue_disparity(c, L, R, H, W, pitch, min_disp, num_disp, win, cost, b.h0, b.h1,
                               c->d16.as<int16_t>(), W, s);
        if (rc) return rc;
        rc = band_median(c, k, H, W, b.r0, b.r1, min_depth, max_depth, depth_range, min_disp_global, min_disp,
                         num_disp, d_depth, d_disparity, d_norm, mo, s);
        if (rc) return rc;
        active.push_back(k);
        if (k > 0) {
            const size_t o = (size_t)b.r0 * W * el, m = (size_t)(b.r1 - b.r0) * W * el;
            blocks[k] = {{recv + o, c->gm16.as<uint8_t>() + o, m}};
        }
    }
    // 3. the peers' bands of the map -> the root (2 or 1 B/px), expanded there unless gather-only
    rc = gather_blocks(ctxs, comms, ndev, blocks, active);
    if (rc || mo.fmt) return rc;
    const size_t rr1 = (size_t)rows[0].r1 * W;
    return expand_on_root(root, n - rr1, rr1, rr1, min_depth, max_depth, depth_range, min_disp_global, min_disp,
                          num_disp, d_depth, d_disparity, d_norm);
}
}  // namespace

int sv_multi_gpu_depth_map_dev(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev, const uint8_t* const* d_left,
                               const uint8_t* const* d_right, const int* n_frames, int H, int W, int pitch,
                               int64_t frame_stride, int min_disp, int num_disp, int win, int cost, float min_depth,
                               float max_depth, float depth_range, float min_disp_global, float* d_depth,
                               float* d_disparity, uint8_t* d_norm) {
    if (!d_left || !d_right || !n_frames || !d_depth || !d_disparity || !d_norm) return fail(SV_EINVAL, "null arguments");
    return multi_frames(ctxs, comms, ndev, d_left, d_right, n_frames, H, W, pitch, frame_stride, min_disp, num_disp,
                        win, cost, min_depth, max_depth, depth_range, min_disp_global, d_depth, d_disparity, d_norm,
                        MapOut{});
}

int sv_multi_gpu_m16_dev(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev, const uint8_t* const* d_left,
                         const uint8_t* const* d_right, const int* n_frames, int H, int W, int pitch,
                         int64_t frame_stride, int min_disp, int num_disp, int win, int cost, int16_t* d_med16) {
    return sv_multi_gpu_map_dev(ctxs, comms, ndev, d_left, d_right, n_frames, H, W, pitch, frame_stride, min_disp,
                                num_disp, win, cost, SV_MAP_M16, d_med16);
}

int sv_multi_gpu_map_dev(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev, const uint8_t* const* d_left,
                         const uint8_t* const* d_right, const int* n_frames, int H, int W, int pitch,
                         int64_t frame_stride, int min_disp, int num_disp, int win, int cost, int map_format,
                         void* d_map) {
    if (!d_left || !d_right || !n_frames) return fail(SV_EINVAL, "null arguments");
    int rc = check_map(map_format, d_map, cost, num_disp);
    if (rc) return rc;
    MapOut mo{map_format, d_map, min_disp - 1};
    return multi_frames(ctxs, comms, ndev, d_left, d_right, n_frames, H, W, pitch, frame_stride, min_disp, num_disp,
                        win, cost, 0.f, 0.f, 0.f, 0.f, nullptr, nullptr, nullptr, mo);
}

int sv_depth_map_rows_multi(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev, const uint8_t* const* d_left,
                            const uint8_t* const* d_right, int H, int W, int pitch, int min_disp, int num_disp,
                            int win, int cost, float min_depth, float max_depth, float depth_range,
                            float min_disp_global, float* d_depth, float* d_disparity, uint8_t* d_norm) {
    if (!d_left || !d_right || !d_depth || !d_disparity || !d_norm) return fail(SV_EINVAL, "null arguments");
    return rows_impl(ctxs, comms, ndev, d_left, d_right, false, H, W, pitch, min_disp, num_disp, win, cost,
                     min_depth, max_depth, depth_range, min_disp_global, d_depth, d_disparity, d_norm, MapOut{});
}

int sv_depth_map_rows_scatter(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev, const uint8_t* d_left,
                              const uint8_t* d_right, int H, int W, int pitch, int min_disp, int num_disp, int win,
                              int cost, float min_depth, float max_depth, float depth_range, float min_disp_global,
                              float* d_depth, float* d_disparity, uint8_t* d_norm) {
    if (!d_left || !d_right || !d_depth || !d_disparity || !d_norm) return fail(SV_EINVAL, "null arguments");
    return rows_impl(ctxs, comms, ndev, &d_left, &d_right, true, H, W, pitch, min_disp, num_disp, win, cost,
                     min_depth, max_depth, depth_range, min_disp_global, d_depth, d_disparity, d_norm, MapOut{});
}

int sv_depth_map_rows_map(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev, const uint8_t* const* d_left,
                          const uint8_t* const* d_right, int scatter, int H, int W, int pitch, int min_disp,
                          int num_disp, int win, int cost, int map_format, void* d_map) {
    if (!d_left || !d_right) return fail(SV_EINVAL, "null arguments");
    int rc = check_map(map_format, d_map, cost, num_disp);
    if (rc) return rc;
    MapOut mo{map_format, d_map, min_disp - 1};
    return rows_impl(ctxs, comms, ndev, d_left, d_right, scatter != 0, H, W, pitch, min_disp, num_disp, win, cost,
                     0.f, 0.f, 0.f, 0.f, nullptr, nullptr, nullptr, mo);
}

int sv_band_rows_in(int H, int rank, int world, int win, int cost, int* out6) {
    if (!out6 || H <= 0 || world < 1 || rank < 0 || rank >= world || win < 1) return fail(SV_EINVAL, "bad band arguments");
    (void)cost;
    SvRows b;
    band_rows_of(H, rank, world, win, b);
    out6[0] = b.r0;
    out6[1] = b.r1;
    out6[2] = b.h0;
    out6[3] = b.h1;
    out6[4] = b.in0;
    out6[5] = b.in1;
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

int sv_copy_to_device(sv_ctx* c, void* dst, const void* src, uint64_t bytes) {
    SV_ENTER(c);
    if (!dst || !src) return fail(SV_EINVAL, "null pointer");
    SV_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, c->stream));
    SV_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

int sv_copy_to_host(sv_ctx* c, void* dst, const void* src, uint64_t bytes) {
    SV_ENTER(c);
    if (!dst || !src) return fail(SV_EINVAL, "null pointer");
    SV_HIP(hipStreamSynchronize(c->stream));   // results of enqueued device work
    SV_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, c->stream));
    SV_HIP(hipStreamSynchronize(c->stream));
    return 0;
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
        c->prof_begin(SV_K_H2D, c->stream);   // (profile on: device events around each upload)
        rc = stage_rows(c, src[i], 0, H, row, stride, stage, dst, 6);
        c->prof_end(c->stream);
        if (rc) return rc;
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
    c->prof_begin(SV_K_D2H, ds);
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
    c->prof_end(ds);
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

int sv_frame_stats_dev(sv_ctx* c, const uint8_t* d_img0, const uint8_t* d_img1, int H, int W, int channels,
                       int pitch, uint32_t* d_block_sum, uint32_t* d_block_sq, uint32_t* d_hist, void* stream) {
    SV_ENTER(c);
    if (check_image(d_img0, H, W) || !d_block_sum || !d_block_sq || !d_hist)
        return fail(SV_EINVAL, "bad frame-stats arguments");
    if (channels != 1 && channels != 3) return fail(SV_EINVAL, "channels must be 1 or 3");
    if (pitch < W * channels) return fail(SV_EINVAL, "pitch smaller than a row");
    hipStream_t s = pick(c, stream);
    SV_SCRATCH(c, s);
    const int nimg = d_img1 ? 2 : 1;
    SV_HIP(c->hist_copies.ensure_zeroed((size_t)sv::kHistCopies * 2 * 256 * sizeof(uint32_t)));
    sv::FrameStatsArgs a{};
    a.hist_copies = c->hist_copies.as<uint32_t>();
    a.img0 = d_img0;
    a.img1 = d_img1;
    a.H = H;
    a.W = W;
    a.pitch = pitch;
    a.cn = channels;
    a.per = nimg;
    a.fs = 0;
    stats_blocks(H, W, &a.bh, &a.bw);
    a.block_sum = d_block_sum;
    a.block_sq = d_block_sq;
    a.hist = d_hist;
    SV_LAUNCH(c, SV_K_STATS, s, sv::launch_frame_stats(a, nimg, s));
    return 0;
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

int sv_select_count(sv_ctx* c, const float* d_x, int64_t n, int mask_mode, const float* d_mask, float thr,
                    int64_t* selected, int64_t* nans) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (selected) *selected = 0;
    if (nans) *nans = 0;
    return select_batch(c, d_x, n, n, 1, mask_mode, d_mask, n, thr, nullptr, 0, nullptr, selected, nans);
}

int sv_select_ranks(sv_ctx* c, const float* d_x, int64_t n, int mask_mode, const float* d_mask, float thr,
                    const int64_t* ranks, int nranks, float* values) {
    SV_ENTER(c);
    SV_SCRATCH(c, c->stream);
    if (!ranks || !values || nranks < 1 || nranks > sv::kMaxRanks) return fail(SV_EINVAL, "1..4 ranks");
    return select_batch(c, d_x, n, n, 1, mask_mode, d_mask, n, thr, ranks, nranks, values, nullptr, nullptr);
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
