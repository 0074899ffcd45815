// sv_ctx.h — the context (struct sv_ctx) and the helpers shared by the C-ABI translation
// units: sv_capi.cpp (errors, contexts, buffers, profiling, the shared enqueue helpers),
// sv_capi_dev.cpp (single-device entry points) and sv_capi_multi.cpp (multi-device entry
// points).  Internal: nothing here is part of include/stereovision_amd.h.
#pragma once
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

namespace svc {
// Sets the calling thread's sv_last_error() message; returns `code`.
int fail(int code, const std::string& msg);
int hipfail(int e, const char* what);
const std::string& last_error_msg();
}  // namespace svc
using svc::fail;
using svc::hipfail;

#define SV_HIP(call)                                               \
    do {                                                           \
        hipError_t e_ = (call);                                    \
        if (e_ != hipSuccess) return hipfail((int)e_, #call);      \
    } while (0)

// A failing launch still closes its profiling pair (the two events go back to the pool).
#define SV_LAUNCH(ctx, kid, stream, call)                          \
    do {                                                           \
        (ctx)->prof_begin((kid), (stream));                        \
        int e_ = (call);                                           \
        if (e_ != 0) {                                             \
            (ctx)->prof_abort();                                   \
            return hipfail(e_, #call);                             \
        }                                                          \
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
    // the whole-disparity table (lut_shift 4: integer-cost maps), cached apart
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
    hipEvent_t sev = nullptr;   // row tiling with scattered inputs: the root's inputs are ready
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
    bool cur_open = false;
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
        cur_open = true;
        (void)hipEventRecord(cur.a, s);
    }
    void prof_end(hipStream_t s) {
        if (!prof || !cur_open) return;
        (void)hipEventRecord(cur.b, s);
        pending.push_back(cur);
        cur_open = false;
    }
    // a failed call between prof_begin and prof_end: its events go back to the pool
    void prof_abort() {
        if (!cur_open) return;
        pool.push_back(cur.a);
        pool.push_back(cur.b);
        cur_open = false;
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

inline hipStream_t pick(sv_ctx* c, void* s) { return s ? static_cast<hipStream_t>(s) : c->stream; }

// RAII profiling region of a multi-step enqueue (e.g. an output download): closes the pair on
// every exit path, aborting it when the enqueue failed.
struct ProfScope {
    sv_ctx* c;
    hipStream_t s;
    bool ok = false;
    ProfScope(sv_ctx* ctx, int kid, hipStream_t stream) : c(ctx), s(stream) { c->prof_begin(kid, s); }
    void done() { ok = true; }
    ~ProfScope() {
        if (ok) c->prof_end(s);
        else c->prof_abort();
    }
};

namespace svc {

struct SgbmParams {
    int P1, P2, disp12, cap, uniq, speckle_win, speckle_range;
};
SgbmParams sgbm_reference_params(int win);

int check_image(const void* a, int H, int W);
int check_match(int H, int W, int min_disp, int num_disp, int win, int cost, sv::MatchPlan* plan);
// cv2.filterSpeckles on an int16 device map (speckle stage of SGBM, sv_filter_speckles).
// nf > 1: a batch of maps, map z at d_img + z*fimg (one launch per stage over grid.z).
int enqueue_speckles(sv_ctx* c, int16_t* d_img, int H, int W, int pitch, int new_val, int max_speckle_size,
                     int max_diff, hipStream_t s, int nf = 1, long long fimg = 0);
// The whole SGBM-3WAY pipeline for nf frames (buffers grown in the context).
int enqueue_sgbm(sv_ctx* c, const uint8_t* L, const uint8_t* R, int H, int W, int pitch, int min_disp,
                 int num_disp, int win, SgbmParams p, int16_t* out, int opitch, hipStream_t s, int nf = 1,
                 long long fs_in = 0, long long fs_out = 0);
// Disparity for rows [row0,row1) of gray device images; nf > 1: a batch of frames, frame z at
// L/R + z*fs_in bytes and out + z*fs_out elements.
int enqueue_disparity(sv_ctx* c, const uint8_t* L, const uint8_t* R, int H, int W, int pitch,
                      int min_disp, int num_disp, int win, int cost, int row0, int row1,
                      int16_t* out, int opitch, hipStream_t s, int nf = 1, long long fs_in = 0,
                      long long fs_out = 0);
// Attach the cached post-processing table (whole: the map holds whole disparities only).
int attach_lut(sv_ctx* c, sv::PostParams& pp, hipStream_t s, bool whole = false);
// Device copy of a 256-entry BGR colormap table (re-uploaded only when it changes).
int attach_cmap(sv_ctx* c, sv::PostParams& pp, const uint8_t* table, uint8_t* d_bgr, hipStream_t s);
sv::PostParams make_post(int mode, float minf, float maxf, float rangef, float mdg, int min_disp,
                         int num_disp, float* a, uint8_t* u8, float* b);

// Validates an sv_map_out for a median launch over maps of `cost` (whole-pixel maps for every
// cost but SGBM) and fills the kernel's PostParams + the f32 disparity pointer (table and
// colormap attached on stream s).  allow_harris: the batch entry point's extra output.
int map_out_post(sv_ctx* c, const sv_map_out* out, int min_disp, int num_disp, int cost, bool allow_harris,
                 hipStream_t s, sv::PostParams* pp, float** disp);

// Gather-only outputs of the multi-device entry points: the full median map lands on the
// root as int16 x16 (SV_MAP_M16) or u8 disparity indices (SV_MAP_D8) and nothing is expanded.
struct MapOut {
    int fmt = 0;           // 0: create_depth_map outputs on the root
    void* map = nullptr;   // fmt != 0: the root's full map (frames dense, or one frame)
    int d8_base = 0;
    size_t el() const { return fmt == SV_MAP_D8 ? 1 : 2; }
};
int check_map(int fmt, const void* map, int cost, int num_disp);
sv::PostParams map_post(int fmt, void* dst, int d8_base);

// Stage two host images (HxW or HxWx3, any stride) into the context's device gray buffers.
int stage_pair(sv_ctx* c, const uint8_t* left, const uint8_t* right, int H, int W, int channels, int stride);

struct Out {
    void* host;
    const void* dev;
    size_t bytes;
};
// Copy device results to caller buffers through the pinned output staging, then wait.
int collect(sv_ctx* c, const Out* outs, int n);

int make_undistort(const double* K, const double* dist, int ndist, const double* R, const double* P,
                   int p_cols, int H, int W, sv::UndistortParams* out);
int check_remap(const void* src, int sH, int sW, int channels, int pitch, const void* map1, int H, int W,
                const void* dst);

}  // namespace svc
using namespace svc;

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
