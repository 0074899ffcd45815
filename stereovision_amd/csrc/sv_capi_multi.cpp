// sv_capi_multi.cpp — the multi-device entry points of the C ABI: a host-
// frame batch sharded over contexts (sv_multi_gpu_batch), and device-resident frames (C4) or
// the row bands of one frame (C5) over ndev contexts with the finished maps gathered to the
// root over RCCL (xGMI) or peer copies (sv_multi_gpu_dev).
#include "sv_ctx.h"

extern "C" {

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
                    if (rcs[k]) errs[k] = svc::last_error_msg();
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
              const uint8_t* const* d_right, int inputs, int H, int W, int pitch, int min_disp, int num_disp,
              int win, int cost, float min_depth, float max_depth, float depth_range, float min_disp_global,
              float* d_depth, float* d_disparity, uint8_t* d_norm, const MapOut& mo) {
    int rc = multi_prologue(ctxs, comms, ndev);
    if (rc) return rc;
    sv::MatchPlan plan;
    rc = check_match(H, W, min_disp, num_disp, win, cost, &plan);
    if (rc) return rc;
    if (cost == SV_COST_SGBM && ndev > 1) return fail(SV_EINVAL, "SGBM cannot be row-tiled (top-down path)");
    if (pitch < W) return fail(SV_EINVAL, "pitch smaller than width");
    const bool scatter = inputs == SV_INPUTS_SCATTER, host = inputs == SV_INPUTS_HOST;
    for (int k = 0; k < (scatter || host ? 1 : ndev); ++k)
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
    if (host) {
        // 1. every context uploads input rows [in0, in1) of both host images over its own PCIe
        //    link into its scratch (img[0], img[1], SV_BAND_MARGIN spare rows either side): no
        //    xGMI traffic before the compute, and no root link carrying every band
        for (int k = 0; k < ndev; ++k) {
            sv_ctx* c = ctxs[k];
            if (rows[k].r1 <= rows[k].r0) continue;
            SV_HIP(hipSetDevice(c->device));
            rc = scratch_wait(c, c->stream);
            if (rc) return rc;
            const size_t bytes = (size_t)(rows[k].in1 - rows[k].in0 + 2 * SV_BAND_MARGIN) * pitch;
            SV_HIP(c->img[0].ensure(bytes));
            SV_HIP(c->img[1].ensure(bytes));
            ProfScope ps(c, SV_K_H2D, c->stream);
            const size_t off = (size_t)rows[k].in0 * pitch, nb = (size_t)(rows[k].in1 - rows[k].in0) * pitch;
            for (int i = 0; i < 2; ++i)
                SV_HIP(hipMemcpyAsync(c->img[i].as<uint8_t>() + (size_t)SV_BAND_MARGIN * pitch,
                                      (i ? d_right[0] : d_left[0]) + off, nb, hipMemcpyHostToDevice, c->stream));
            ps.done();
        }
        SV_HIP(hipSetDevice(root->device));
    }
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
        if (!host && (k == 0 || !scatter)) {
            rc = scratch_wait(c, s);
            if (rc) return rc;
        }
        const uint8_t* L = d_left[scatter || host ? 0 : k];
        const uint8_t* R = d_right[scatter || host ? 0 : k];
        if ((scatter && k > 0) || host) {
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

int sv_multi_gpu_dev(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev, int shard, int inputs,
                     const uint8_t* const* left, const uint8_t* const* right, const int* n_frames, int H, int W,
                     int pitch, int64_t frame_stride, int min_disp, int num_disp, int win, int cost,
                     const sv_map_out* out) {
    if (!left || !right || !out) return fail(SV_EINVAL, "null arguments");
    if (shard != SV_SHARD_FRAMES && shard != SV_SHARD_ROWS) return fail(SV_EINVAL, "shard must be FRAMES or ROWS");
    if (inputs != SV_INPUTS_RESIDENT && inputs != SV_INPUTS_SCATTER && inputs != SV_INPUTS_HOST)
        return fail(SV_EINVAL, "bad inputs mode");
    if (shard == SV_SHARD_FRAMES && inputs != SV_INPUTS_RESIDENT)
        return fail(SV_EINVAL, "frame sharding takes device-resident frames");
    if (shard == SV_SHARD_FRAMES && !n_frames) return fail(SV_EINVAL, "null frame counts");
    // what the root holds: create_depth_map's outputs (expanded from the peers' int16 maps) or
    // one gathered map
    const bool full = out->mode == SV_POST_DEPTH && out->disparity && out->out_a && out->out_u8;
    const int nmaps = (out->med16 ? 1 : 0) + (out->d8 ? 1 : 0);
    if (full ? (nmaps || out->out_b || out->bgr || out->harris)
             : (nmaps != 1 || out->mode != SV_POST_NONE || out->disparity || out->out_a || out->out_u8 ||
                out->out_b || out->bgr || out->harris))
        return fail(SV_EINVAL, "out must hold create_depth_map's outputs (SV_POST_DEPTH: disparity, out_a, out_u8) "
                               "or exactly one map (med16 or d8)");
    MapOut mo;
    if (!full) {
        const int fmt = out->d8 ? SV_MAP_D8 : SV_MAP_M16;
        void* map = out->d8 ? static_cast<void*>(out->d8) : static_cast<void*>(out->med16);
        const int rc = check_map(fmt, map, cost, num_disp);
        if (rc) return rc;
        mo = MapOut{fmt, map, min_disp - 1};
    }
    const float mind = full ? out->min_depth : 0.f, maxd = full ? out->max_depth : 0.f;
    const float rng = full ? out->depth_range : 0.f, mdg = full ? out->min_disp_global : 0.f;
    if (shard == SV_SHARD_FRAMES)
        return multi_frames(ctxs, comms, ndev, left, right, n_frames, H, W, pitch, frame_stride, min_disp, num_disp,
                            win, cost, mind, maxd, rng, mdg, out->out_a, out->disparity, out->out_u8, mo);
    return rows_impl(ctxs, comms, ndev, left, right, inputs, H, W, pitch, min_disp, num_disp, win, cost, mind, maxd,
                     rng, mdg, out->out_a, out->disparity, out->out_u8, mo);
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

}  // extern "C"
