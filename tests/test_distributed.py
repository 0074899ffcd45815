"""world_size-2 gloo tests of the multi-GPU sharding logic on CPU.

Each rank computes its row band (plus the median halo) with the C oracle standing in for
the GPU kernels, exactly as RowTiledDepthMap does on the device, and the bands are
gathered with the same gather_rows used over RCCL.  Rank 0 checks the reassembled maps
against the single-process full-frame result bit-for-bit.
"""
import os
import socket

import numpy as np
import pytest

import sv_oracle as O
import sv_oracle_c as C
from stereovision_amd.synthetic import stereo_pair

# torch (and stereovision_amd.distributed, which imports it) are imported lazily: at module
# level they would load torch's bundled HIP runtime during `pytest -m gpu` collection and
# rebind libsvhip to it ("One HIP runtime per process").


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _row_tiled_worker(rank, world, port, H, W, D, win, q):
    import torch
    import torch.distributed as dist
    from stereovision_amd import distributed as SD
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L, R, _ = stereo_pair(H, W, D, seed=11)            # every rank holds the full frame
        r0, r1 = SD.band_rows(H, rank, world)
        h0, h1 = SD.median_halo(r0, r1, H)
        d16 = C.disparity16(L, R, 0, D, win, rows=(h0, h1))[h0:h1]
        disp_band = O.disparity_f32(d16)[r0 - h0:r1 - h0]   # median of the halo'd band
        depth_band, _ = O.depth_post(disp_band, 0.3, 2.0)
        full_disp = SD.gather_rows(torch.from_numpy(np.ascontiguousarray(disp_band)), H)
        full_depth = SD.gather_rows(torch.from_numpy(np.ascontiguousarray(depth_band)), H)
        frames = SD.gather_frames(torch.full((2, 3), float(rank)))
        if rank == 0:
            ref_disp = O.disparity_f32(C.disparity16(L, R, 0, D, win))
            ref_depth, _ = O.depth_post(ref_disp, 0.3, 2.0)
            ok = (np.array_equal(full_disp.numpy(), ref_disp)
                  and np.array_equal(full_depth.numpy(), ref_depth)
                  and frames.shape == (2 * world, 3)
                  and all((frames[2 * k:2 * k + 2] == k).all() for k in range(world)))
            q.put(bool(ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H", [(2, 37), (2, 64), (3, 29)])
def test_row_tiling_reassembles_bit_exactly(world, H):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_row_tiled_worker, args=(world, _free_port(), H, 120, 32, 9, q),
                       nprocs=world, join=True, start_method="spawn")
    assert q.get(timeout=60) is True


def test_band_partition_covers_every_row_once():
    from stereovision_amd import distributed as SD
    for H in (1, 7, 270, 1080, 2160):
        for world in (1, 2, 3, 4, 8):
            rows = [r for k in range(world) for r in range(*SD.band_rows(H, k, world))]
            assert rows == list(range(H))
            assert SD.max_band(H, world) == -(-H // world) or H < world
    assert SD.median_halo(0, 10, 100) == (0, 12)
    assert SD.median_halo(50, 60, 61) == (48, 61)
    assert SD.frame_indices(8, 1, 8) == [1]
    assert SD.frame_indices(10, 1, 4) == [1, 5, 9]
