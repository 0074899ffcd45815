"""Multi-process CPU tests of the multi-GPU layer (stereovision_amd/distributed.py).

* world_size-2/3 gloo: every rank computes its row band (plus the median halo) with the C
  oracle standing in for the GPU kernels, exactly as RowTiledDepthMap does on the device, and
  the bands move through the SAME `gather_rows` / `gather_frames` arithmetic used over RCCL
  (offsets into a full-frame buffer; here the "device pointers" index a NumPy byte buffer and
  the transport is gloo).  Rank 0 checks the reassembled maps bit-for-bit against the
  single-process full-frame result.
* the torch-free rendezvous: FileStore barriers / max-reductions / broadcasts and
  init_process_group(backend="host") over 3 spawned processes (no torch anywhere).
* the product package and bench.py never import torch.
"""
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

import sv_oracle as O
import sv_oracle_c as C
from stereovision_amd import distributed as SD
from stereovision_amd.synthetic import stereo_pair

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class GlooBufferComm:
    """The ProcessGroup.gatherv contract over gloo: "pointers" are byte offsets into this
    rank's NumPy buffer `buf` (so gather_rows' pointer arithmetic runs unchanged)."""

    def __init__(self, dist, buf):
        self.dist, self.buf = dist, buf
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def gatherv(self, d_send, send_bytes, d_recv, offsets, sizes, root=0, stream=0):
        import torch
        mx = max(sizes)
        pad = torch.zeros(mx, dtype=torch.uint8)
        pad[:send_bytes] = torch.from_numpy(self.buf[d_send:d_send + send_bytes].copy())
        out = [torch.zeros(mx, dtype=torch.uint8) for _ in range(self.world)] if self.rank == root else None
        self.dist.gather(pad, out, dst=root)
        if self.rank == root:
            for k in range(self.world):
                self.buf[d_recv + offsets[k]: d_recv + offsets[k] + sizes[k]] = out[k][:sizes[k]].numpy()


def _row_tiled_worker(rank, world, port, H, W, D, win, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L, R, _ = stereo_pair(H, W, D, seed=11)            # every rank holds the full frame
        r0, r1 = SD.band_rows(H, rank, world)
        h0, h1 = SD.median_halo(r0, r1, H)
        d16 = C.disparity16(L, R, 0, D, win, rows=(h0, h1))
        disp_full = np.zeros((H, W), np.float32)
        disp_full[r0:r1] = O.disparity_f32(d16[h0:h1])[r0 - h0:r1 - h0]   # median of the halo'd band
        depth_full = np.zeros((H, W), np.float32)
        depth_full[r0:r1], _ = O.depth_post(disp_full[r0:r1], 0.3, 2.0)
        # both maps in one byte buffer: [disparity | depth], gathered in place band by band
        buf = np.concatenate([disp_full.view(np.uint8).ravel(), depth_full.view(np.uint8).ravel()])
        comm = GlooBufferComm(dist, buf)
        SD.gather_rows(comm, 0, H, 4 * W)
        SD.gather_rows(comm, 4 * H * W, H, 4 * W)
        # gather-only row tiling (--root-outputs m16): the bands' maps only, as u8 disparity
        # indices d - min_disp + 1 (1 B/px) and as int16 x16 medians (2 B/px)
        med16 = np.zeros((H, W), np.int16)
        med16[r0:r1] = O.median5(d16[h0:h1])[r0 - h0:r1 - h0]
        d8 = np.zeros((H, W), np.uint8)
        d8[r0:r1] = (med16[r0:r1] // 16 + 1).astype(np.uint8)       # min_disp 0: index d + 1
        mbuf = np.concatenate([d8.ravel(), med16.view(np.uint8).ravel()])
        mcomm = GlooBufferComm(dist, mbuf)
        SD.gather_rows(mcomm, 0, H, W)
        SD.gather_rows(mcomm, H * W, H, 2 * W)
        # frame gather: rank k contributes k+1 frames of 6 bytes filled with k
        counts = [k + 1 for k in range(world)]
        fbuf = np.full(6 * counts[rank], rank, np.uint8)
        stack = np.zeros(6 * sum(counts), np.uint8)
        fcomm = GlooBufferComm(dist, np.concatenate([fbuf, stack]))
        SD.gather_frames(fcomm, 0, counts[rank], fbuf.size, 6, counts=counts)
        if rank == 0:
            got_disp = buf[:4 * H * W].view(np.float32).reshape(H, W)
            got_depth = buf[4 * H * W:].view(np.float32).reshape(H, W)
            ref_disp = O.disparity_f32(C.disparity16(L, R, 0, D, win))
            ref_depth, _ = O.depth_post(ref_disp, 0.3, 2.0)
            frames = fcomm.buf[fbuf.size:]
            exp_frames = np.concatenate([np.full(6 * counts[k], k, np.uint8) for k in range(world)])
            got_d8 = mbuf[:H * W].reshape(H, W).astype(np.float32) - np.float32(1)
            got_m16 = mbuf[H * W:].view(np.int16).reshape(H, W).astype(np.float32) / np.float32(16)
            q.put(bool(np.array_equal(got_disp, ref_disp) and np.array_equal(got_depth, ref_depth)
                       and np.array_equal(frames, exp_frames) and np.array_equal(got_d8, ref_disp)
                       and np.array_equal(got_m16, ref_disp)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H", [(2, 37), (2, 64), (3, 29)])
def test_row_tiling_reassembles_bit_exactly(world, H):
    import torch.multiprocessing as tmp
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    tmp.start_processes(_row_tiled_worker, args=(world, _free_port(), H, 120, 32, 9, q),
                        nprocs=world, join=True, start_method="spawn")
    assert q.get(timeout=60) is True


def test_band_partition_covers_every_row_once():
    for H in (1, 7, 270, 1080, 2160):
        for world in (1, 2, 3, 4, 8):
            rows = [r for k in range(world) for r in range(*SD.band_rows(H, k, world))]
            assert rows == list(range(H))
            assert SD.max_band(H, world) == -(-H // world) or H < world
            offs, sizes = SD.rows_layout(H, world, 7)
            assert sum(sizes) == 7 * H and offs[0] == 0
            assert all(offs[k] + sizes[k] == offs[k + 1] for k in range(world - 1))
    assert SD.median_halo(0, 10, 100) == (0, 12)
    assert SD.median_halo(50, 60, 61) == (48, 61)
    assert SD.frame_indices(8, 1, 8) == [1]
    assert SD.frame_indices(10, 1, 4) == [1, 5, 9]
    assert SD.frames_layout([2, 1, 3], 10) == ([0, 20, 30], [20, 10, 30])


# ---- torch-free rendezvous ------------------------------------------------------------------
def _store_worker(rank, world, path, q):
    store = SD.FileStore(path, rank, world, timeout=60)
    store.barrier()
    mx = store.allreduce_max(float(rank) * 1.5 - 1.0)
    b = store.broadcast(b"id-%d" % 42 if rank == 0 else None)
    g = store.allgather(bytes([rank]))
    store.barrier()
    # the launch-style entry point, file-store backend (no GPU, no RCCL)
    os.environ.update({"WORLD_SIZE": str(world), "RANK": str(rank), "LOCAL_RANK": str(rank),
                       "SV_RDZV_DIR": path + "_pg"})
    pg = SD.init_process_group(device=0, backend="host", timeout=60)
    t = pg.allreduce_max(10.0 + rank)
    pg.barrier()
    ok = (mx == (world - 1) * 1.5 - 1.0 and b == b"id-42" and g == [bytes([k]) for k in range(world)]
          and pg.backend == "host" and pg.world == world and t == 10.0 + world - 1)
    q.put((rank, ok, "torch" in sys.modules))
    pg.close()
    store.close()


def test_file_store_rendezvous_three_processes():
    world = 3
    path = tempfile.mkdtemp(prefix="sv_store_test_")
    os.rmdir(path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_store_worker, args=(k, world, path, q)) for k in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
    assert not any(t for _, _, t in res), "the rendezvous imported torch"
    assert not os.path.exists(path), "rank 0 removes the store directory"


def test_file_store_times_out_instead_of_hanging(tmp_path):
    store = SD.FileStore(str(tmp_path / "s"), 1, 2, timeout=0.2)
    with pytest.raises(TimeoutError):
        store.barrier()


def test_store_path_is_per_launch(monkeypatch):
    monkeypatch.delenv("SV_RDZV_DIR", raising=False)
    monkeypatch.setenv("MASTER_PORT", "29555")
    p = SD.default_store_path()
    assert "29555" in p and str(os.getppid()) in p


def test_product_and_bench_never_import_torch():
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import stereovision_amd, stereovision_amd.engine, stereovision_amd.distributed\n"
            "import stereovision_amd.depth_map, stereovision_amd.fused_depth_map, stereovision_amd.fusion\n"
            "import stereovision_amd.rectify, stereovision_amd.calib, stereovision_amd.pipeline\n"
            "import bench\n"
            "assert 'torch' not in sys.modules, sorted(m for m in sys.modules if 'torch' in m)\n"
            "print('ok')\n") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       cwd=ROOT)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
    # and no product source imports it
    import re
    pat = re.compile(r"^\s*(import|from)\s+torch\b", re.M)
    files = [os.path.join(ROOT, "stereovision_amd", f) for f in os.listdir(os.path.join(ROOT, "stereovision_amd"))
             if f.endswith(".py")] + [os.path.join(ROOT, "bench.py")]
    for f in files:
        assert not pat.search(open(f).read()), f
