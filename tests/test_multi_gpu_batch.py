"""sv_multi_gpu_batch: the per-frame create_depth_map loop (depth_map.py:837-946) frame-
sharded over several device contexts from ONE host process.

On the 1-GPU test box the shards go to several distinct contexts on device 0: the
sharding, the per-shard staging/collection and the concurrent host threads are exercised
exactly as on 8 devices (each context has its own stream and buffers).  Bar: every output
of every frame bit-exact against the oracle's create_depth_map.
"""
import numpy as np
import pytest

import sv_oracle as O
from stereovision_amd.engine import Engine, SVError, multi_gpu_batch
from stereovision_amd.synthetic import stereo_pair, to_bgr


def _stack(F, H, W, D, bgr):
    Ls, Rs = [], []
    for f in range(F):
        L, R, _ = stereo_pair(H, W, D, seed=100 + f)
        Ls.append(to_bgr(L) if bgr else L)
        Rs.append(to_bgr(R) if bgr else R)
    return np.stack(Ls), np.stack(Rs)


@pytest.fixture(scope="module")
def engines(engine):
    extra = [Engine(0) for _ in range(2)]
    yield [engine] + extra
    for e in extra:
        e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("F,ndev,bgr", [(5, 3, True), (4, 2, False), (1, 3, False), (7, 1, True)])
def test_multi_gpu_batch_matches_oracle_per_frame(engines, F, ndev, bgr):
    H, W, D, win = 40, 150, 32, 9
    L, R = _stack(F, H, W, D, bgr)
    depth, disp, norm = multi_gpu_batch(engines[:ndev], L, R, 0, D, win, 0.3, 2.0)
    assert depth.shape == disp.shape == norm.shape == (F, H, W)
    for f in range(F):
        e_depth, e_disp, e_norm = O.create_depth_map(L[f], R[f], 0, D, win, 0.3, 2.0)
        np.testing.assert_array_equal(disp[f], e_disp)
        np.testing.assert_array_equal(depth[f], e_depth)
        np.testing.assert_array_equal(norm[f], e_norm)


@pytest.mark.gpu
def test_multi_gpu_batch_matches_single_context_calls(engines):
    L, R = _stack(6, 64, 200, 64, False)
    depth, disp, norm = multi_gpu_batch(engines, L, R, 0, 64, 11, 0.5, 3.0)
    for f in range(6):
        d1, p1, n1 = engines[0].depth_map(L[f], R[f], 0, 64, 11, 0.5, 3.0)
        np.testing.assert_array_equal(p1, disp[f])
        np.testing.assert_array_equal(d1, depth[f])
        np.testing.assert_array_equal(n1, norm[f])


@pytest.mark.gpu
def test_multi_gpu_batch_errors(engines):
    L, R = _stack(2, 24, 80, 16, False)
    with pytest.raises(SVError):                          # the same context twice
        multi_gpu_batch([engines[0], engines[0]], L, R, 0, 16, 5, 0.3, 2.0)
    with pytest.raises(SVError):                          # even window
        multi_gpu_batch(engines[:2], L, R, 0, 16, 4, 0.3, 2.0)
    with pytest.raises(ValueError):
        multi_gpu_batch(engines[:2], L, R[:1], 0, 16, 5, 0.3, 2.0)
    d, p, n = multi_gpu_batch(engines[:2], L[:0], R[:0], 0, 16, 5, 0.3, 2.0)
    assert d.shape == (0, 24, 80)
