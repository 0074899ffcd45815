"""Multi-GPU sharding of the disparity path — no PyTorch.

The reference has no distributed code; its unit of work is one frame pair
per call (depth_map.py:1181-1183; fused_depth_map.py:2591-2598 submits one frame at a time
to a worker pool).  The build's sharding:

* **frame sharding** (config C4): independent frames, frame i -> rank i % world.  No
  collective in the data path; finished maps may be gathered to rank 0 over RCCL/xGMI.
* **row tiling** (config C5): one large frame, rank k computes output rows
  [H*k/world, H*(k+1)/world).  Rank 0 holds the frame; :meth:`RowTiledDepthMap.scatter`
  sends every rank only the input rows its band reads (:func:`band_layout`: the band, the
  5x5 median's 2-row halo and the matching window's halo), so the halo rows are read
  locally and bands reassemble bit-exactly (the border policy applies only at the true
  image border).  :func:`gather_rows` moves every band into rank 0's full-frame buffer with
  one RCCL send/recv group (unequal bands, no padding).  Ranks that already hold the full
  frame skip the scatter (``compute(d_left, d_right)``).

Two ways to run N GPUs:

* one process per GPU (``python -m torch.distributed.run ... bench.py``; only the launcher
  is torch's, the workers never import torch): :func:`init_process_group` reads
  RANK / WORLD_SIZE / LOCAL_RANK, rendezvouses through a directory on the node's local file
  system (:class:`FileStore`; rank 0 publishes the RCCL unique id there) and returns a
  :class:`ProcessGroup` over an RCCL communicator of libsvhip (``sv_comm_*``).  When RCCL
  cannot run (ranks sharing one GPU, library missing) it falls back to the file store for
  barriers and max-reductions and to host staging for gathers.
* one process driving several GPUs: ``engine.multi_gpu_depth_map_dev`` /
  ``engine.depth_map_rows_multi`` (sv_multi_gpu_dev),
  whose gathers run as one RCCL group (``Communicator.init_all``) or peer copies.
"""
from __future__ import annotations

import os
import struct
import sys
import time

import numpy as np

from .engine import BAND_MARGIN, POST_DEPTH, POST_NONE, POST_SCALED, Communicator, get_engine


# ---- partition arithmetic -----------------------------------------------------------------
def band_rows(H: int, rank: int, world: int) -> tuple[int, int]:
    """Output rows owned by `rank` in a `world`-way row tiling (balanced, contiguous)."""
    return H * rank // world, H * (rank + 1) // world


def median_halo(r0: int, r1: int, H: int, halo: int = 2) -> tuple[int, int]:
    """Disparity rows a band needs for its 5x5 median (replicate border at the image edge)."""
    return max(0, r0 - halo), min(H, r1 + halo)


def input_rows(h0: int, h1: int, H: int, win: int) -> tuple[int, int]:
    """Input rows the kernels of disparity rows [h0, h1) read (sv_band_rows_in): the window's
    r rows, the four-row waves' 3 extra rows below the last one and the HOG Sobel row,
    i.e. r + 4 each side, clamped to the frame."""
    halo = win // 2 + 4
    return max(0, h0 - halo), min(H, h1 + halo)


def band_layout(H: int, rank: int, world: int, win: int) -> dict:
    """Output rows r0:r1, disparity rows h0:h1 (median halo) and input rows in0:in1 of a
    rank's band (the same numbers as the C ABI's sv_band_rows_in)."""
    r0, r1 = band_rows(H, rank, world)
    h0, h1 = median_halo(r0, r1, H)
    in0, in1 = input_rows(h0, h1, H, win)
    return {"r0": r0, "r1": r1, "h0": h0, "h1": h1, "in0": in0, "in1": in1}


def scatter_layout(H: int, world: int, win: int, row_nbytes: int) -> tuple[list[int], list[int]]:
    """Byte offsets (into a full frame) and sizes of every rank's input rows."""
    offs, sizes = [], []
    for k in range(world):
        b = band_layout(H, k, world, win)
        offs.append(b["in0"] * row_nbytes)
        sizes.append((b["in1"] - b["in0"]) * row_nbytes)
    return offs, sizes


def frame_indices(n_frames: int, rank: int, world: int) -> list[int]:
    """Frames processed by `rank` under frame sharding."""
    return list(range(rank, n_frames, world))


def max_band(H: int, world: int) -> int:
    return max(band_rows(H, k, world)[1] - band_rows(H, k, world)[0] for k in range(world))


def rows_layout(H: int, world: int, row_nbytes: int) -> tuple[list[int], list[int]]:
    """Byte offsets and sizes of every rank's band inside a full-frame buffer."""
    offs, sizes = [], []
    for k in range(world):
        r0, r1 = band_rows(H, k, world)
        offs.append(r0 * row_nbytes)
        sizes.append((r1 - r0) * row_nbytes)
    return offs, sizes


def frames_layout(counts, frame_nbytes: int) -> tuple[list[int], list[int]]:
    """Byte offsets and sizes of every rank's frames in a rank-major stack."""
    offs, sizes, acc = [], [], 0
    for n in counts:
        offs.append(acc * frame_nbytes)
        sizes.append(n * frame_nbytes)
        acc += n
    return offs, sizes


def gather_rows(comm, d_full: int, H: int, row_nbytes: int, root: int = 0, stream: int = 0):
    """Row-tiled gather in place: every rank's band already sits at its row offset of its own
    full-frame buffer `d_full`; afterwards the root's buffer holds every band."""
    offs, sizes = rows_layout(H, comm.world, row_nbytes)
    me = comm.rank
    comm.gatherv(d_full + offs[me], sizes[me], d_full, offs, sizes, root=root, stream=stream)


def gather_frames(comm, d_send: int, n_local: int, d_recv: int, frame_nbytes: int, counts=None,
                  root: int = 0, stream: int = 0):
    """Frame-sharded gather: rank k's n_local frames land after the frames of ranks < k."""
    counts = [n_local] * comm.world if counts is None else list(counts)
    offs, sizes = frames_layout(counts, frame_nbytes)
    comm.gatherv(d_send, sizes[comm.rank], d_recv, offs, sizes, root=root, stream=stream)


# ---- rendezvous ----------------------------------------------------------------------------
class FileStore:
    """Key/value store in a directory of the node's local file system: the rendezvous of
    the one-process-per-GPU mode (all ranks run on one node).  Values are written to a
    temporary name and renamed, so a reader never sees a partial value."""

    def __init__(self, path: str, rank: int, world: int, timeout: float = 300.0):
        self.path, self.rank, self.world, self.timeout = path, rank, world, timeout
        os.makedirs(path, exist_ok=True)
        self._n = 0

    def set(self, key: str, value: bytes):
        tmp = os.path.join(self.path, f".{key}.{self.rank}.tmp")
        with open(tmp, "wb") as f:
            f.write(value)
        os.replace(tmp, os.path.join(self.path, key))

    def get(self, key: str, timeout: float | None = None) -> bytes:
        p = os.path.join(self.path, key)
        t_end = time.monotonic() + (self.timeout if timeout is None else timeout)
        delay = 0.0005
        while True:
            try:
                with open(p, "rb") as f:
                    return f.read()
            except FileNotFoundError:
                if time.monotonic() > t_end:
                    raise TimeoutError(f"rendezvous: no key {key!r} in {self.path} after "
                                       f"{self.timeout:.0f} s (a rank died or never started?)")
                time.sleep(delay)
                delay = min(delay * 2, 0.01)

    def _tag(self, name: str) -> str:
        self._n += 1
        return f"{name}.{self._n}"

    def barrier(self):
        t = self._tag("barrier")
        self.set(f"{t}.{self.rank}", b"1")
        for k in range(self.world):
            self.get(f"{t}.{k}")

    def allgather(self, value: bytes) -> list[bytes]:
        t = self._tag("allgather")
        self.set(f"{t}.{self.rank}", value)
        return [self.get(f"{t}.{k}") for k in range(self.world)]

    def allreduce_max(self, value: float) -> float:
        vals = self.allgather(struct.pack("<d", float(value)))
        return max(struct.unpack("<d", v)[0] for v in vals)

    def broadcast(self, value: bytes | None, root: int = 0) -> bytes:
        t = self._tag("bcast")
        if self.rank == root:
            self.set(t, value)
            return value
        return self.get(t)

    def close(self):
        """Last barrier; every rank then marks that it has left it, and rank 0 removes the
        directory once all have (a rank still reading the barrier's keys is never cut off)."""
        try:
            self.barrier()
            self.set(f"exit.{self.rank}", b"1")
            if self.rank == 0:
                for k in range(self.world):
                    self.get(f"exit.{k}")
        finally:
            if self.rank == 0:
                for name in os.listdir(self.path):
                    try:
                        os.remove(os.path.join(self.path, name))
                    except OSError:
                        pass
                try:
                    os.rmdir(self.path)
                except OSError:
                    pass


def default_store_path() -> str:
    """Directory shared by the ranks of one launch: MASTER_PORT plus the launcher's pid
    (torch.distributed.run's agent is every local worker's parent, and a new launch has a
    new pid, so a stale directory of an earlier run is never reused)."""
    if os.environ.get("SV_RDZV_DIR"):
        return os.environ["SV_RDZV_DIR"]
    port = os.environ.get("MASTER_PORT", "0")
    run = os.environ.get("TORCHELASTIC_RUN_ID", "")
    restart = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    base = os.environ.get("TMPDIR", "/tmp")
    return os.path.join(base, f"sv_rdzv_{port}_{os.getppid()}_{run}_{restart}")


# ---- process groups --------------------------------------------------------------------------
class ProcessGroup:
    """rank/world of this process plus barrier, max-allreduce and gatherv over device
    buffers: RCCL (`backend == "rccl"`) or the file store with host staging ("host")."""

    def __init__(self, rank: int, world: int, device: int, store: FileStore | None,
                 comm: Communicator | None, engine=None, devices=None, reason: str = ""):
        self.rank, self.world, self.device = rank, world, device
        self.store, self.comm, self.engine = store, comm, engine
        self.backend = "rccl" if comm is not None else ("host" if world > 1 else "local")
        self.devices = list(devices) if devices is not None else [device]
        # why RCCL is not used ("" when it is): ranks sharing a GPU, library missing, "host"
        # requested
        self.reason = reason

    @property
    def rccl_ranks(self) -> int:
        """Ranks of the RCCL communicator (0 when the group runs on the file store)."""
        return self.comm.nranks if self.comm is not None else 0

    def _stream(self, stream: int) -> int:
        """stream 0 = this rank's engine stream (the one compute() enqueues on), never the
        communicator's own stream: the gather must follow the kernels that write the data."""
        if stream:
            return stream
        return (self.engine or get_engine(self.device)).stream

    def barrier(self):
        if self.comm is not None:
            self.comm.barrier()
        elif self.store is not None:
            self.store.barrier()

    def allreduce_max(self, value: float) -> float:
        if self.comm is not None:
            return self.comm.allreduce_max(value)
        if self.store is not None:
            return self.store.allreduce_max(value)
        return float(value)

    def gatherv(self, d_send: int, send_bytes: int, d_recv: int, offsets, sizes, root: int = 0,
                stream: int = 0):
        if self.comm is not None:
            self.comm.gatherv(d_send, send_bytes, d_recv, offsets, sizes, root=root,
                              stream=self._stream(stream))
            return
        eng = self.engine or get_engine(self.device)
        if self.world == 1 or self.store is None:
            if d_send != d_recv + offsets[self.rank] and send_bytes:
                eng.synchronize()
                host = eng.to_host(d_send, (send_bytes,), np.uint8)
                eng.to_device(d_recv + offsets[self.rank], host)
            return
        # host staging through the store (fallback when RCCL cannot run)
        eng.synchronize()
        t = self.store._tag("gatherv")
        if self.rank != root:
            host = eng.to_host(d_send, (send_bytes,), np.uint8) if send_bytes else np.empty(0, np.uint8)
            self.store.set(f"{t}.{self.rank}", host.tobytes())
            self.store.get(f"{t}.done")
            return
        for k in range(self.world):
            if k == root:
                if send_bytes and d_send != d_recv + offsets[k]:
                    eng.to_device(d_recv + offsets[k], eng.to_host(d_send, (send_bytes,), np.uint8))
                continue
            data = np.frombuffer(self.store.get(f"{t}.{k}"), np.uint8)
            if data.size != sizes[k]:
                raise RuntimeError(f"gatherv: rank {k} sent {data.size} bytes, expected {sizes[k]}")
            if data.size:
                eng.to_device(d_recv + offsets[k], data)
        self.store.set(f"{t}.done", b"1")

    def scatterv(self, d_send: int, offsets, sizes, d_recv: int, recv_bytes: int, root: int = 0,
                 stream: int = 0):
        """The root's block k (d_send + offsets[k], sizes[k] bytes) -> rank k's d_recv."""
        if self.comm is not None:
            self.comm.scatterv(d_send, offsets, sizes, d_recv, recv_bytes, root=root,
                               stream=self._stream(stream))
            return
        eng = self.engine or get_engine(self.device)
        if self.world == 1 or self.store is None:
            if recv_bytes and d_recv != d_send + offsets[self.rank]:
                eng.synchronize()
                eng.to_device(d_recv, eng.to_host(d_send + offsets[self.rank], (recv_bytes,), np.uint8))
            return
        # host staging through the store (fallback when RCCL cannot run)
        eng.synchronize()
        t = self.store._tag("scatterv")
        if self.rank == root:
            for k in range(self.world):
                host = eng.to_host(d_send + offsets[k], (sizes[k],), np.uint8) if sizes[k] else np.empty(0, np.uint8)
                if k == root:
                    if sizes[k] and d_recv != d_send + offsets[k]:
                        eng.to_device(d_recv, host)
                else:
                    self.store.set(f"{t}.{k}", host.tobytes())
            return
        data = np.frombuffer(self.store.get(f"{t}.{self.rank}"), np.uint8)
        if data.size != recv_bytes:
            raise RuntimeError(f"scatterv: rank {self.rank} got {data.size} bytes, expected {recv_bytes}")
        if data.size:
            eng.to_device(d_recv, data)

    def dup(self, tag: str = "dup") -> "ProcessGroup":
        """A second group over the same ranks with its own communicator (collective: every rank
        calls it): RCCL — a new ncclCommInitRank, so two streams can run collectives in opposite
        directions at once (e.g. a row tiling's scatter root -> peers beside the previous frame's
        gather peers -> root, each on its own stream and communicator); file store — a
        sub-directory with its own key sequence."""
        store = None
        if self.store is not None:
            store = FileStore(os.path.join(self.store.path, tag), self.rank, self.world, self.store.timeout)
        comm = None
        if self.comm is not None:
            uid = self.store.broadcast(Communicator.unique_id() if self.rank == 0 else None)
            comm = Communicator.init_rank(self.device, self.world, self.rank, uid,
                                          timeout=min(self.store.timeout, 120.0))
        return ProcessGroup(self.rank, self.world, self.device, store, comm, self.engine, self.devices,
                            self.reason)

    def close(self):
        if self.comm is not None:
            self.comm.close()
            self.comm = None
        if self.store is not None:
            self.store.close()
            self.store = None


def _log(msg: str):
    print(f"[stereovision_amd.distributed] {msg}", file=sys.stderr, flush=True)


def init_process_group(device: int | None = None, backend: str = "auto",
                       timeout: float = 300.0, engine=None, strict: bool = False) -> ProcessGroup:
    """Process group of a torch.distributed.run-style launch, from RANK / WORLD_SIZE /
    LOCAL_RANK (world 1 when unset).  backend: "auto" (RCCL unless it cannot run: ranks
    sharing a GPU, library missing), "rccl" (required), "host" (file store only).
    strict: with "auto", ranks on DISTINCT devices must get RCCL (RuntimeError otherwise);
    only ranks sharing a GPU (a 1-GPU rehearsal) may fall back to the file store.  Without
    strict, an ncclCommInitRank failure on any rank makes every rank fall back to the file
    store together (`reason` names it; SV_RCCL_INIT_FAIL=1 forces it, for tests)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device is None:
        from .engine import device_count
        nd = max(1, device_count())
        device = local % nd
    if world == 1:
        return ProcessGroup(0, 1, device, None, None, engine, reason="world size 1")
    store = FileStore(default_store_path(), rank, world, timeout)
    # collective decision (a rank must never be left alone inside ncclCommInitRank)
    ok = backend != "host" and Communicator.available()
    info = store.allgather(struct.pack("<ii", device, int(ok)))
    devs = [struct.unpack("<ii", v)[0] for v in info]
    all_ok = all(struct.unpack("<ii", v)[1] for v in info)
    dup = len(set(devs)) < len(devs)
    use_rccl = all_ok and not dup
    reason = ("file store requested (backend='host')" if backend == "host" else
              f"ranks share a GPU (devices {devs})" if dup else
              "librccl.so.1 not loadable on every rank" if not all_ok else "")
    if backend == "rccl" and not use_rccl:
        raise RuntimeError(f"RCCL backend requested but unusable: {reason}")
    if strict and backend == "auto" and not use_rccl and not dup:
        raise RuntimeError(f"RCCL required on distinct devices {devs} but unusable: {reason}")
    comm = None
    if use_rccl:
        if os.environ.get("MASTER_ADDR", "127.0.0.1") in ("127.0.0.1", "localhost"):
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")   # single-node bootstrap
        uid = store.broadcast(Communicator.unique_id() if rank == 0 else None)
        err = ""
        try:
            if os.environ.get("SV_RCCL_INIT_FAIL", "") not in ("", "0"):
                raise RuntimeError("forced failure (SV_RCCL_INIT_FAIL)")
            # non-blocking with a deadline: if a peer fails inside the initialisation this rank
            # returns (its half-built communicator aborted) instead of blocking forever, so
            # every rank reaches the allgather below
            comm = Communicator.init_rank(device, world, rank, uid, timeout=min(timeout, 120.0))
        except Exception as ex:   # decided collectively below: every rank falls back together
            err = f"ncclCommInitRank failed on rank {rank}: {ex}"
        errs = [e.decode() for e in store.allgather(err.encode()) if e]
        if errs:
            if comm is not None:
                comm.close()
                comm = None
            reason = "; ".join(errs)
            if backend == "rccl" or strict:
                raise RuntimeError(f"RCCL required on devices {devs} but unusable: {reason}")
            use_rccl = False
            if rank == 0:
                _log(f"RCCL init failed ({reason}); barriers/reductions through the file store, "
                     "gathers through host staging")
    elif rank == 0:
        _log(f"RCCL not used ({reason}); barriers/reductions through the file store, "
             "gathers through host staging")
    return ProcessGroup(rank, world, device, store, comm, engine, devices=devs, reason=reason)


class RowTiledDepthMap:
    """Row-tiled app-1 / app-2 device path for one frame across the ranks of a group.

    Inputs either as full frames on every rank (:meth:`compute` with full-frame pointers), or
    band-only (:meth:`scatter` from the root's full frame: rank k receives just the input rows
    [in0, in1) its band reads into :attr:`band_left` / :attr:`band_right`, then
    :meth:`compute` without arguments).  Each rank computes disparity for its band plus the
    median halo (sv_disparity_dev), then the median of the band (sv_median_rows_dev): its
    int16 x16 medians (:attr:`m16`, full-frame row offsets) and, unless ``band_outputs="m16"``,
    the post outputs too.  :meth:`gather` moves the bands' int16 x16 medians into the root's
    :attr:`m16` (2 B/px over xGMI instead of the outputs' 9) and the root expands the other
    ranks' rows into its full-frame outputs (sv_post_m16_dev).  Every operation is enqueued
    on the engine's stream unless a stream is passed, so scatter -> compute -> gather are
    ordered on one stream (the RCCL calls included); two instances on a communication stream
    pipeline consecutive frames (bench.py --mode rowtile).
    """

    def __init__(self, H: int, W: int, num_disp: int, win: int, min_disp: int = 0,
                 cost: str = "sad", device: int = 0, rank: int = 0, world: int = 1, engine=None):
        self.H, self.W = H, W
        self.num_disp, self.win, self.min_disp, self.cost = num_disp, win, min_disp, cost
        self.rank, self.world = rank, world
        self.engine = engine or get_engine(device)
        b = band_layout(H, rank, world, win)
        self.r0, self.r1, self.h0, self.h1 = b["r0"], b["r1"], b["h0"], b["h1"]
        self.in0, self.in1 = b["in0"], b["in1"]
        e, n = self.engine, H * W
        self.d16 = e.dev_alloc(2 * n)
        self.disp = e.dev_alloc(4 * n)
        self.out_a = e.dev_alloc(4 * n)
        self.out_b = e.dev_alloc(4 * n)
        self.out_u8 = e.dev_alloc(n)
        self.m16 = e.dev_alloc(2 * n)
        self.rows = self.r1 - self.r0
        self._post = None   # the post parameters of the last compute (the root's expansion)
        self._band_outputs = None   # what the last compute wrote ("full", "m16" or "d8")
        # band-only inputs: input rows [in0, in1) with BAND_MARGIN spare rows either side
        self.band_bytes = (self.in1 - self.in0) * W
        nb = self.band_bytes + 2 * BAND_MARGIN * W
        self._band = [e.dev_alloc(max(256, nb)), e.dev_alloc(max(256, nb))]
        self.band_left, self.band_right = (p + BAND_MARGIN * W for p in self._band)

    def _stream(self, stream: int) -> int:
        return stream or self.engine.stream

    def scatter(self, pg: "ProcessGroup", d_full_left: int = 0, d_full_right: int = 0,
                root: int = 0, stream: int = 0):
        """Input rows of every rank's band from the root's full-frame gray images (device
        pointers, used on the root only) into each rank's band buffers."""
        offs, sizes = scatter_layout(self.H, pg.world, self.win, self.W)
        s = self._stream(stream)
        for full, band in ((d_full_left, self.band_left), (d_full_right, self.band_right)):
            pg.scatterv(full, offs, sizes, band, self.band_bytes, root=root, stream=s)

    def upload(self, host_left: np.ndarray, host_right: np.ndarray, stream: int = 0):
        """This rank's band input rows [in0, in1) from the full HOST frames (H x W uint8,
        page-locked — sv_host_register — for the copy to overlap device work) into
        :attr:`band_left` / :attr:`band_right` over this GPU's own PCIe link: the band-only
        inputs of :meth:`scatter` without any xGMI traffic (every rank holds the frame in
        host memory, as a camera pipeline's frames arrive).  Enqueued on the engine stream
        unless `stream` is given; the host arrays must stay alive until it has run."""
        for a in (host_left, host_right):
            if a.shape != (self.H, self.W) or a.dtype != np.uint8 or not a.flags["C_CONTIGUOUS"]:
                raise ValueError(f"upload: expected C-contiguous {self.H}x{self.W} uint8 frames")
        s = self._stream(stream)
        for a, band in ((host_left, self.band_left), (host_right, self.band_right)):
            self.engine.to_device(band, a[self.in0:self.in1], stream=s)

    def compute(self, d_left: int = 0, d_right: int = 0, mode: int = POST_DEPTH, min_depth: float = 0.3,
                max_depth: float = 2.0, min_disp_global=None, stream: int = 0, band_outputs: str = "full"):
        """Enqueue this rank's band: its median map at full-frame row offsets of self.m16 —
        int16 x16, or with band_outputs="d8" u8 disparity indices median/16 - (min_disp - 1)
        (1 B/px for the gather; integer costs, num_disp <= 255) — and (band_outputs="full")
        the outputs in self.disp / self.out_a / self.out_u8 (/ self.out_b for POST_SCALED).
        d_left/d_right: full-frame gray images, or 0 for the band buffers filled by
        :meth:`scatter`."""
        if band_outputs not in ("full", "m16", "d8"):
            raise ValueError(f"band_outputs must be 'full', 'm16' or 'd8', got {band_outputs!r}")
        if band_outputs == "d8" and self.cost == "sgbm":   # sub-pixel medians: not whole indices
            raise ValueError("band_outputs='d8' needs an integer-disparity cost (SGBM maps are sub-pixel)")
        e, H, W = self.engine, self.H, self.W
        s = self._stream(stream)
        if not d_left:   # band buffer addressed as a full frame (row y at base + y * W)
            d_left = self.band_left - self.in0 * W
            d_right = self.band_right - self.in0 * W
        e.disparity_dev(d_left, d_right, H, W, W, self.min_disp, self.num_disp, self.win, self.cost,
                        self.h0, self.h1, self.d16, W, stream=s)
        mdg = self.min_disp if min_disp_global is None else min_disp_global
        self._post = dict(min_depth=min_depth, max_depth=max_depth, min_disp_global=mdg,
                          min_disp=self.min_disp, num_disp=self.num_disp)
        self._mode = mode
        self._band_outputs = band_outputs
        if band_outputs == "d8":
            e.median_map_dev(self.d16, H, W, self.r0, self.r1, self.m16, "d8", min_disp=self.min_disp,
                             num_disp=self.num_disp, stream=s, cost=self.cost)
        elif band_outputs == "m16":
            e.median_post_m16_dev(self.d16, H, W, self.r0, self.r1, POST_NONE, d_med16=self.m16, stream=s,
                                  cost=self.cost)
        else:
            e.median_post_m16_dev(self.d16, H, W, self.r0, self.r1, mode, d_disparity=self.disp,
                                  d_out_a=self.out_a, d_out_u8=self.out_u8,
                                  d_out_b=self.out_b if mode == POST_SCALED else 0, d_med16=self.m16,
                                  stream=s, cost=self.cost, **self._post)

    def gather(self, pg: "ProcessGroup", root: int = 0, stream: int = 0, expand: bool = True,
               check: bool = True):
        """Every rank's band of the median map into the root's self.m16 (in place: 2 B/px
        int16 x16, or 1 B/px when the bands were computed with band_outputs="d8"), then
        (expand) the root turns the other ranks' rows into its full-frame outputs; on the engine
        stream unless `stream` is given (never the communicator's own stream: ADVICE r02).
        Gather-only (expand=False) leaves the full map in the root's self.m16.  Expanding needs
        int16 maps and the root's own band computed with band_outputs="full".

        check (every rank must pass the same value): before the collective, the ranks agree on
        the arguments — expand, the gathered element size, the root's own band — with three
        max-reductions, and on a mismatch EVERY rank raises ValueError (a rank raising alone
        would leave the others inside a gather that never completes: ADVICE r05).  A
        pipeline checks its first gather and passes check=False for the identical ones after."""
        s = self._stream(stream)
        el = 1 if self._band_outputs == "d8" else 2
        if check:
            self._agree(pg, root, expand, el)
        gather_rows(pg, self.m16, self.H, self.W * el, root=root, stream=s)
        if not expand or pg.rank != root or self._post is None:
            return
        e, W, mode = self.engine, self.W, self._mode
        mr0, mr1 = band_rows(self.H, root, pg.world)
        # the other ranks' bands are the rows above and below the root's own: <= 2 launches
        for r0, r1 in ((0, mr0), (mr1, self.H)):
            if r1 <= r0:
                continue
            o = r0 * W
            e.post_m16_dev(self.m16 + 2 * o, (r1 - r0) * W, mode, d_disparity=self.disp + 4 * o,
                           d_out_a=self.out_a + 4 * o, d_out_u8=self.out_u8 + o,
                           d_out_b=(self.out_b + 4 * o) if mode == POST_SCALED else 0, stream=s,
                           **self._post)

    def _agree(self, pg: "ProcessGroup", root: int, expand: bool, el: int):
        why = ("compute() was not called" if self._band_outputs is None else
               "expand=True gathers int16 maps, not band_outputs='d8'" if expand and el == 1 else
               "expand=True needs compute(band_outputs='full') on the root (its own rows)"
               if expand and pg.rank == root and self._band_outputs != "full" else "")
        code = 4 * el + (2 if expand else 0)
        bad = pg.allreduce_max(1.0 if why else 0.0)
        hi, lo = pg.allreduce_max(float(code)), -pg.allreduce_max(-float(code))
        if bad or hi != lo:
            raise ValueError("RowTiledDepthMap.gather: the ranks disagree or a rank's arguments are "
                             f"invalid (this rank: {why or 'ok'}; expand={expand}, {el} B/px; codes "
                             f"{lo:.0f}..{hi:.0f}) — every rank raises, no gather is enqueued")

    def close(self):
        for p in (self.d16, self.disp, self.out_a, self.out_b, self.out_u8, self.m16, *self._band):
            if p:
                self.engine.dev_free(p)
        self.d16 = self.disp = self.out_a = self.out_b = self.out_u8 = self.m16 = 0
        self._band = []
