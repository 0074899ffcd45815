"""CPU tests of the multi-GPU bench contract and the band-only row tiling (no GPU).

* bench.py's N > 1 line: the gather is on by default, and the `distributed` object carries
  backend / rccl_ranks / rccl_reason / gather_us_per_step (dist_summary, fed by a file-store
  process group of 2 spawned ranks, the 1-GPU rehearsal of the driver's launch);
* init_process_group(strict=True) refuses a file-store fallback on distinct devices and
  allows it when the ranks share a GPU;
* ProcessGroup / RowTiledDepthMap default to the ENGINE stream for their collectives
  (never the communicator's own stream);
* band-only inputs: the Python layout equals the C ABI's sv_band_rows_in, and a band
  computed by the C oracle from ONLY its input rows (everything else poisoned) equals the
  full-frame result, for every rank of several tilings.
"""
import multiprocessing as mp
import os
import sys
import tempfile

import numpy as np
import pytest

import sv_oracle_c as C
from stereovision_amd import distributed as SD
from stereovision_amd import engine as E
from stereovision_amd.synthetic import stereo_pair

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_gather_is_the_default_for_multi_gpu_frames():
    a = bench.parse_args(["--gpus", "2"])
    assert not a.no_gather and a.mode == "frames"
    assert bench.parse_args(["--gpus", "2", "--no-gather"]).no_gather
    assert not bench.parse_args([]).no_verify


def test_default_batch_and_lanes_at_1080p():
    """One GPU at 1920x1080: 8-frame steps over 2 stream lanes (16 resident frames, one 8-frame
    set per lane); N > 1 (gather beside the compute): 26-frame steps on one
    stream (24.0 rounds of the k_match wave slots); 16 elsewhere and for SGBM / row tiling; an
    explicit batch, stream or frame count wins."""
    a = bench.parse_args([])
    assert (a.batch, a.frames, a.streams, a.schedule) == (8, 16, 2, "lanes")
    assert bench.parse_args(["--win", "11"]).batch == 8
    assert bench.parse_args(["--gpus", "2"]).batch == 26
    assert bench.parse_args(["--streams", "1"]).batch == 26
    assert bench.parse_args(["--height", "480", "--width", "640", "--num-disp", "64"]).batch == 16
    assert bench.parse_args(["--cost", "sgbm"]).batch == 16
    assert bench.parse_args(["--mode", "rowtile"]).batch == 16
    a = bench.parse_args(["--batch", "8", "--streams", "1"])
    assert (a.batch, a.frames) == (8, 8)
    assert bench.parse_args(["--frames", "4"]).frames == 4


def _dist_worker(rank, world, path, q):
    os.environ.update({"WORLD_SIZE": str(world), "RANK": str(rank), "LOCAL_RANK": str(rank),
                       "SV_RDZV_DIR": path})
    # both ranks on "device 0": the 1-GPU rehearsal, where the file store is legitimate
    pg = SD.init_process_group(device=0, backend="auto", timeout=60, strict=True)
    d = bench.dist_summary(2, True, pg, gather=True, gather_ms=1.5, gather_n=3,
                           gather_wall_s=0.002, steps=4, gather_bytes=9 * 1920 * 1080)
    q.put((rank, d, "torch" in sys.modules))
    pg.close()


def _warm_worker(rank, world, path, q):
    os.environ.update({"WORLD_SIZE": str(world), "RANK": str(rank), "LOCAL_RANK": str(rank),
                       "SV_RDZV_DIR": path})
    pg = SD.init_process_group(device=0, backend="auto", timeout=60, strict=True)
    # rank k's steps take (k + 1) ms: alone they would pick different warm-up counts
    n = bench.agreed_extra_warmup(pg, 0.005 * (rank + 1), 5, 1.0)
    q.put((rank, n))
    pg.close()


def test_warmup_count_agreed_across_ranks():
    """Launched runs: every rank runs the same number of warm-up steps (the max over ranks
    of each rank's own estimate), whatever its step rate."""
    path = tempfile.mkdtemp(prefix="sv_bench_warm_")
    os.rmdir(path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_warm_worker, args=(k, 3, path, q)) for k in range(3)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(3))
    for p in ps:
        p.join(timeout=60)
    assert len(set(res.values())) == 1, res
    assert res[0] == int((1.0 - 0.005) / 0.001) + 1     # the fastest rank's (largest) count


def test_dist_fields_under_the_file_store_rehearsal():
    path = tempfile.mkdtemp(prefix="sv_bench_dist_")
    os.rmdir(path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dist_worker, args=(k, 2, path, q)) for k in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (d, t)) for r, d, t in (q.get(timeout=120) for _ in range(2)))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    d, torch_loaded = res[0]
    assert not torch_loaded
    assert d["backend"] == "host" and d["rccl_ranks"] == 0
    assert "share a GPU" in d["rccl_reason"]
    assert d["gather"] is True and d["gather_us_per_step"] == 500.0 and d["gather_events"] == 3
    assert d["gather_bytes_per_step"] == 9 * 1920 * 1080 and d["gather_GBps"] > 0
    assert d["gather_wall_us_per_step"] == 500.0


def test_dist_summary_one_process_modes():
    assert bench.dist_summary(1, False) is None

    class Comm:
        pass
    d = bench.dist_summary(8, False, comms=[Comm()] * 8, gather=True)
    assert d["backend"] == "rccl" and d["rccl_ranks"] == 8 and d["rccl_reason"] is None
    d = bench.dist_summary(4, False, comms=None, rowtile=True, scatter_ms=2.0, scatter_n=4,
                           reason="ncclCommInitAll failed: x")
    assert d["backend"] == "peer" and d["rccl_ranks"] == 0 and "ncclCommInitAll" in d["rccl_reason"]
    assert d["scatter_us_per_step"] == 500.0 and "band-only" in d["inputs"]


def _strict_worker(rank, world, path, q):
    os.environ.update({"WORLD_SIZE": str(world), "RANK": str(rank), "LOCAL_RANK": str(rank),
                       "SV_RDZV_DIR": path})
    E.Communicator.available = staticmethod(lambda: False)    # "librccl.so.1 missing"
    try:
        SD.init_process_group(device=rank, backend="auto", timeout=60, strict=True)
        q.put((rank, "no error"))
    except RuntimeError as e:
        q.put((rank, str(e)))


def test_strict_group_refuses_file_store_on_distinct_devices():
    path = tempfile.mkdtemp(prefix="sv_bench_strict_")
    os.rmdir(path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_strict_worker, args=(k, 2, path, q)) for k in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
    assert all("RCCL required on distinct devices" in msg for _, msg in res), res


def _init_fail_worker(rank, world, path, strict, q):
    """RCCL loads on every rank, but ncclCommInitRank fails on rank 1 only."""
    os.environ.update({"WORLD_SIZE": str(world), "RANK": str(rank), "LOCAL_RANK": str(rank),
                       "SV_RDZV_DIR": path})

    class _Comm:
        nranks = world

        def close(self):
            q.put((rank, "closed"))

    def _init_rank(device, nranks, r, uid, timeout=120.0):
        if r == 1:
            raise RuntimeError("ncclCommInitRank: unhandled system error")
        return _Comm()
    E.Communicator.available = staticmethod(lambda: True)
    E.Communicator.unique_id = staticmethod(lambda: b"\0" * 128)
    E.Communicator.init_rank = staticmethod(_init_rank)
    try:
        pg = SD.init_process_group(device=rank, backend="auto", timeout=60, strict=strict)
        q.put((rank, f"{pg.backend}|{pg.reason}"))
        pg.close()
    except RuntimeError as e:
        q.put((rank, "raised: " + str(e)))


@pytest.mark.parametrize("strict", [False, True])
def test_rccl_init_failure_on_one_rank_falls_back_on_every_rank(strict):
    """VERDICT r04 Next #1: an ncclCommInitRank failure on any rank is decided collectively —
    every rank closes its communicator and uses the file store (backend "host", the failure
    named), or, strict (--require-rccl), every rank raises; no rank is left in a collective."""
    path = tempfile.mkdtemp(prefix="sv_bench_initfail_")
    os.rmdir(path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_init_fail_worker, args=(k, 2, path, strict, q)) for k in range(2)]
    for p in ps:
        p.start()
    res = []
    for _ in range(3):   # one result per rank + rank 0's "closed" (its init succeeded)
        res.append(q.get(timeout=120))
    for p in ps:
        p.join(timeout=60)
    msgs = {r: m for r, m in res if m != "closed"}
    assert (0, "closed") in res and sorted(msgs) == [0, 1], res   # rank 0 gave its communicator back
    if strict:
        assert all(m.startswith("raised:") and "ncclCommInitRank failed on rank 1" in m for m in msgs.values()), res
    else:
        assert all(m.startswith("host|") and "ncclCommInitRank failed on rank 1" in m for m in msgs.values()), res


class _FakeEngine:
    stream = 0xABC


class _FakeComm:
    nranks = 2

    def __init__(self):
        self.streams = []

    def gatherv(self, *a, stream=0, **k):
        self.streams.append(stream)

    def scatterv(self, *a, stream=0, **k):
        self.streams.append(stream)


def test_collectives_default_to_the_engine_stream():
    comm = _FakeComm()
    pg = SD.ProcessGroup(0, 2, 0, None, comm, engine=_FakeEngine())
    assert pg.backend == "rccl" and pg.rccl_ranks == 2
    SD.gather_rows(pg, 0, 10, 4)                 # the documented default-stream call
    SD.gather_frames(pg, 0, 1, 0, 4)
    pg.scatterv(0, [0, 0], [1, 1], 0, 1)
    pg.gatherv(0, 1, 0, [0, 1], [1, 1], stream=77)
    assert comm.streams == [0xABC, 0xABC, 0xABC, 77]


def test_python_band_layout_equals_the_c_abi():
    lib = E.load_library()
    assert lib is not None
    for H in (1, 7, 29, 270, 1080, 2160):
        for world in (1, 2, 3, 8):
            for win in (1, 5, 9, 15):
                for k in range(world):
                    assert SD.band_layout(H, k, world, win) == E.band_rows_in(H, k, world, win), (H, world, win, k)
    offs, sizes = SD.scatter_layout(2160, 8, 15, 3840)
    b = SD.band_layout(2160, 3, 8, 15)
    assert offs[3] == b["in0"] * 3840 and sizes[3] == (b["in1"] - b["in0"]) * 3840


@pytest.mark.parametrize("world,H,win,cost", [(2, 64, 9, 0), (3, 41, 15, 0), (8, 131, 5, 0),
                                               (4, 50, 11, 1), (3, 37, 7, 2)])
def test_band_from_its_input_rows_only_matches_the_full_frame(world, H, win, cost):
    W, D = 160, 48
    L, R, _ = stereo_pair(H, W, D, seed=world * 1000 + H)
    ref = C.disparity16(L, R, 0, D, win, cost)
    ref_med = C.median5_f32(ref)
    for k in range(world):
        b = SD.band_layout(H, k, world, win)
        Lp = np.full_like(L, 0xA5)
        Rp = np.full_like(R, 0x5A)
        Lp[b["in0"]:b["in1"]] = L[b["in0"]:b["in1"]]
        Rp[b["in0"]:b["in1"]] = R[b["in0"]:b["in1"]]
        d16 = C.disparity16(Lp, Rp, 0, D, win, cost, rows=(b["h0"], b["h1"]))
        np.testing.assert_array_equal(d16[b["h0"]:b["h1"]], ref[b["h0"]:b["h1"]])
        med = C.median5_f32(d16[b["h0"]:b["h1"]])[b["r0"] - b["h0"]:b["r1"] - b["h0"]]
        np.testing.assert_array_equal(med, ref_med[b["r0"]:b["r1"]])


def _blocking_init_worker(rank, world, path, q):
    """rank 1's ncclCommInitRank fails while rank 0 is still INSIDE its own
    (collective) initialisation.  The real sv_comm_init_rank is non-blocking with a deadline:
    rank 0's call returns an error once the deadline passes (its half-built communicator
    aborted), so it still reaches the collective decision.  The mock reproduces exactly that:
    rank 0 blocks until rank 1 has failed, then waits out its deadline and fails."""
    os.environ.update({"WORLD_SIZE": str(world), "RANK": str(rank), "LOCAL_RANK": str(rank),
                       "SV_RDZV_DIR": path})
    marker = os.path.join(path + ".marks", "rank1_failed")

    def _init_rank(device, nranks, r, uid, timeout=120.0):
        if r == 1:
            os.makedirs(os.path.dirname(marker), exist_ok=True)
            open(marker, "w").close()
            raise RuntimeError("ncclCommInitRank: unhandled system error")
        import time as _t
        t_end = _t.monotonic() + 60
        while not os.path.exists(marker):     # still "inside" the init when the peer dies
            assert _t.monotonic() < t_end
            _t.sleep(0.01)
        _t.sleep(min(timeout, 0.5))            # the deadline (shortened by the test's timeout)
        raise RuntimeError(f"ncclCommInitRank did not complete within {timeout} s; aborted")
    E.Communicator.available = staticmethod(lambda: True)
    E.Communicator.unique_id = staticmethod(lambda: b"\0" * 128)
    E.Communicator.init_rank = staticmethod(_init_rank)
    try:
        pg = SD.init_process_group(device=rank, backend="auto", timeout=60, strict=False)
        q.put((rank, f"{pg.backend}|{pg.reason}"))
        pg.close()
    except Exception as e:  # noqa: BLE001
        q.put((rank, "raised: " + repr(e)))


def test_rccl_init_failure_while_a_peer_is_still_initialising():
    path = tempfile.mkdtemp(prefix="sv_bench_initblock_")
    os.rmdir(path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_blocking_init_worker, args=(k, 2, path, q)) for k in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    assert sorted(res) == [0, 1], res
    for m in res.values():   # both ranks fell back together, naming both failures
        assert m.startswith("host|") and "failed on rank 1" in m and "failed on rank 0" in m, res


class _MemEngine:
    """Engine stand-in for RowTiledDepthMap's bookkeeping (allocations are fake addresses)."""
    stream = 0x77

    def __init__(self):
        self.n = 0x1000

    def dev_alloc(self, nbytes):
        self.n += max(256, nbytes)
        return self.n

    def dev_free(self, p):
        pass


def _gather_check_worker(rank, world, path, outputs, expand, q):
    os.environ.update({"WORLD_SIZE": str(world), "RANK": str(rank), "LOCAL_RANK": str(rank),
                       "SV_RDZV_DIR": path})
    E.Communicator.available = staticmethod(lambda: False)
    pg = SD.init_process_group(device=0, backend="host", timeout=60)
    tile = SD.RowTiledDepthMap(64, 96, 32, 5, device=0, rank=rank, world=world, engine=_MemEngine())
    tile._band_outputs = outputs[rank]          # what compute() would have recorded
    called = []
    pg.gatherv = lambda *a, **k: called.append(a)   # reached only when every rank agreed
    try:
        tile.gather(pg, root=0, expand=expand)
        q.put((rank, f"gathered {len(called)}"))
    except ValueError as e:
        q.put((rank, "ValueError: " + str(e)))
    finally:
        pg.close()


@pytest.mark.parametrize("outputs,expand,ok", [
    (("m16", "m16"), True, False),     # the root cannot expand without its own band's outputs
    (("full", "d8"), True, False),     # d8 bands cannot be expanded
    (("d8", "m16"), False, False),     # element sizes differ: the gather would corrupt rows
    (("d8", "d8"), False, True),
    (("full", "m16"), True, True),
])
def test_row_tile_gather_arguments_are_agreed_on_every_rank(outputs, expand, ok):
    """a bad gather argument on ANY rank makes EVERY rank raise before the
    collective (a root-only raise left the peers in a gather that never completes)."""
    path = tempfile.mkdtemp(prefix="sv_bench_gchk_")
    os.rmdir(path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_check_worker, args=(k, 2, path, outputs, expand, q)) for k in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    if ok:
        assert all(m.startswith("gathered 1") for m in res.values()), res
    else:
        assert all(m.startswith("ValueError") for m in res.values()), res


def test_row_tile_rejects_d8_for_sgbm():
    """SGBM's sub-pixel medians are not whole-pixel indices."""
    tile = SD.RowTiledDepthMap(64, 96, 32, 5, cost="sgbm", engine=_MemEngine())
    with pytest.raises(ValueError, match="integer-disparity"):
        tile.compute(1, 2, band_outputs="d8")
