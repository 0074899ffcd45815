"""Multi-GPU sharding of the disparity path: one process per GPU, torch.distributed.

The reference has no distributed code; its work sharding is the build's
own:

* **frame sharding** (config C4): independent frames, frame i -> rank i % world.  No
  collective in the data path; the finished maps may be gathered to rank 0 over RCCL/xGMI
  (:func:`gather_frames`) when a consumer on one device needs them.
* **row tiling** (config C5): one large frame, rank k computes output rows
  [H*k/world, H*(k+1)/world).  Every rank holds the full input frame, so the matching
  window's halo rows (and the 5x5 median's 2-row halo, via :func:`median_halo`) are read
  locally: bands reassemble bit-exactly (the border policy is applied only at the true
  image border).  :func:`gather_rows` concatenates the bands on rank 0 with one
  all_gather of equal-sized, padded bands (RCCL over xGMI with the "nccl" backend, or gloo
  on CPU for tests).

torch is imported before the engine library so libsvhip binds to torch's HIP runtime
(one HIP runtime per process).
"""
from __future__ import annotations

import torch  # noqa: F401  (must precede the engine library load)
import torch.distributed as dist

from .engine import POST_DEPTH, POST_SCALED, get_engine


def band_rows(H: int, rank: int, world: int) -> tuple[int, int]:
    """Output rows owned by `rank` in a `world`-way row tiling (balanced, contiguous)."""
    return H * rank // world, H * (rank + 1) // world


def median_halo(r0: int, r1: int, H: int, halo: int = 2) -> tuple[int, int]:
    """Disparity rows a band needs for its 5x5 median (replicate border at the image edge)."""
    return max(0, r0 - halo), min(H, r1 + halo)


def frame_indices(n_frames: int, rank: int, world: int) -> list[int]:
    """Frames processed by `rank` under frame sharding."""
    return list(range(rank, n_frames, world))


def max_band(H: int, world: int) -> int:
    return max(band_rows(H, k, world)[1] - band_rows(H, k, world)[0] for k in range(world))


def gather_rows(band: torch.Tensor, H: int, group=None) -> torch.Tensor | None:
    """Concatenate the row bands of all ranks on rank 0 (None on other ranks).

    `band` is this rank's [r1 - r0, ...] tensor (on the rank's GPU for RCCL, CPU for gloo).
    Bands are padded to the largest band so one all_gather_into_tensor moves them.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    mb = max_band(H, world)
    pad = torch.zeros((mb,) + tuple(band.shape[1:]), dtype=band.dtype, device=band.device)
    pad[: band.shape[0]] = band
    out = torch.empty((world * mb,) + tuple(band.shape[1:]), dtype=band.dtype, device=band.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    if rank != 0:
        return None
    parts = []
    for k in range(world):
        r0, r1 = band_rows(H, k, world)
        parts.append(out[k * mb: k * mb + (r1 - r0)])
    return torch.cat(parts, 0)


def gather_frames(frames: torch.Tensor, group=None) -> torch.Tensor | None:
    """Stack equal-shaped per-rank results [n_local, ...] on rank 0 (rank-major order)."""
    world = dist.get_world_size(group)
    out = torch.empty((world * frames.shape[0],) + tuple(frames.shape[1:]), dtype=frames.dtype,
                      device=frames.device)
    dist.all_gather_into_tensor(out, frames.contiguous(), group=group)
    return out if dist.get_rank(group) == 0 else None


class RowTiledDepthMap:
    """Row-tiled app-1 / app-2 device path for one frame across the ranks of a group.

    Each rank owns full-frame gray inputs in HBM (torch uint8 tensors on its GPU) and
    computes its band: disparity for the band plus the median halo (sv_disparity_dev),
    then median + post for the band (sv_median_post_dev), then the bands are gathered.
    """

    def __init__(self, H: int, W: int, num_disp: int, win: int, min_disp: int = 0,
                 cost: str = "sad", device: int | None = None, group=None,
                 rank: int | None = None, world: int | None = None):
        self.H, self.W = H, W
        self.num_disp, self.win, self.min_disp, self.cost = num_disp, win, min_disp, cost
        self.group = group
        inited = dist.is_available() and dist.is_initialized()
        self.rank = rank if rank is not None else (dist.get_rank(group) if inited else 0)
        self.world = world if world is not None else (dist.get_world_size(group) if inited else 1)
        self.device = torch.cuda.current_device() if device is None else device
        self.engine = get_engine(self.device)
        self.r0, self.r1 = band_rows(H, self.rank, self.world)
        self.h0, self.h1 = median_halo(self.r0, self.r1, H)
        dev = f"cuda:{self.device}"
        n = self.r1 - self.r0
        self.d16 = torch.empty((H, W), dtype=torch.int16, device=dev)
        self.disp = torch.empty((H, W), dtype=torch.float32, device=dev)
        self.out_a = torch.empty((H, W), dtype=torch.float32, device=dev)
        self.out_b = torch.empty((H, W), dtype=torch.float32, device=dev)
        self.out_u8 = torch.empty((H, W), dtype=torch.uint8, device=dev)
        self.rows = n

    def compute(self, d_left: torch.Tensor, d_right: torch.Tensor, mode: int = POST_DEPTH,
                min_depth: float = 0.3, max_depth: float = 2.0, min_disp_global=None):
        """Enqueue this rank's band on the current torch stream; returns band views
        (disparity f32, out_a f32, out_u8, out_b f32)."""
        e, H, W = self.engine, self.H, self.W
        stream = torch.cuda.current_stream(self.device).cuda_stream
        e.disparity_dev(d_left.data_ptr(), d_right.data_ptr(), H, W, W, self.min_disp,
                        self.num_disp, self.win, self.cost, self.h0, self.h1,
                        self.d16.data_ptr(), W, stream=stream)
        mdg = self.min_disp if min_disp_global is None else min_disp_global
        e.median_post_dev(self.d16.data_ptr(), H, W, self.r0, self.r1, mode,
                          self.disp.data_ptr(), self.out_a.data_ptr(), self.out_u8.data_ptr(),
                          self.out_b.data_ptr() if mode == POST_SCALED else 0,
                          min_depth=min_depth, max_depth=max_depth, min_disp_global=mdg,
                          min_disp=self.min_disp, num_disp=self.num_disp, stream=stream)
        sl = slice(self.r0, self.r1)
        return self.disp[sl], self.out_a[sl], self.out_u8[sl], self.out_b[sl]

    def gather(self, band: torch.Tensor) -> torch.Tensor | None:
        if self.world == 1:
            return band
        return gather_rows(band, self.H, self.group)
