"""N > 1 path on CPU: frame-interleaved sharding + one sum-reduce (pt_amd/shard.py), world_size 2
over gloo.  Each rank renders its frames with the oracle as the CPU stand-in for the GPU render
(which the GPU parity tests pin to the oracle bit for bit).

Tolerance: sharding changes the f32 summation order (per-rank partial sums, then the reduce)
relative to the reference's single sequential accumulator, so the reduced image equals the
single-process accumulation to f32 rounding (rtol 2e-6 of the pixel value); summing the same
partials in rank order on one process reproduces it bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pt_amd.shard import frames_for_rank, reduce_accum

SPP, DEPTH, W, H = 6, 8, 24, 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene():
    import scene_oracle as so
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cam, ps = so.load_scene(os.path.join(root, "scenes", "scene_assets", "CornellBox.xml"),
                            os.path.join(root, "scenes", "scene_assets"))
    st = {"imageWidth": W, "imageHeight": H, "samplesPerPixel": SPP, "pathContinuationProb": 0.9,
          "directLightingOnly": False}
    return ps.triangle_data, ps.bvh_data, so.make_meta(so.screen_dimension(st), cam, st)


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    tri, bvh, meta = _scene()
    f0, n, stride = frames_for_rank(rank, world, SPP)
    acc, _ = oracle.render(tri, bvh, meta, f0, n, stride, DEPTH)
    t = torch.from_numpy(acc.copy())
    reduce_accum(t, dist)
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_frames_for_rank_partition():
    for world in (1, 2, 3, 8):
        for spp in (1, 5, 256, 1024):
            seen = []
            for r in range(world):
                f0, n, s = frames_for_rank(r, world, spp)
                seen += list(range(f0, f0 + n * s, s))
            assert sorted(seen) == list(range(spp))
    with pytest.raises(ValueError):
        frames_for_rank(2, 2, 8)


def test_world2_gloo_reduce(tmp_path):
    import oracle
    out = str(tmp_path / "acc.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    tri, bvh, meta = _scene()
    ref, _ = oracle.render(tri, bvh, meta, 0, SPP, 1, DEPTH)
    assert np.allclose(got, ref, rtol=2e-6, atol=0)
    # exact: rank partials summed in rank order
    parts = [oracle.render(tri, bvh, meta, *frames_for_rank(r, 2, SPP), DEPTH)[0] for r in range(2)]
    assert np.array_equal((parts[0] + parts[1]).view(np.uint32), got.view(np.uint32))
