"""Process-per-GPU path (bench.py's N > 1 mode, pt_amd/shard.py) with the HIP render in every rank:
world size 2 over gloo on the box's one GPU (both ranks render on device 0, their partial
accumulators go through ONE sum-reduce).  With two ranks the reduce is one f32 add per value,
which is commutative, so the result equals the oracle's two shard renders added — bit for bit —
and is within f32 rounding of the single-process render of all frames.  (tests/test_multigpu.py
covers the same plumbing on CPU with the oracle as the stand-in renderer; the RCCL form is the
driver's multi-GPU bench.)"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, SPP, DEPTH = 64, 48, 9, 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tri, bvh, meta, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pt_amd
    from pt_amd.shard import frames_for_rank, reduce_accum
    f0, n, stride = frames_for_rank(rank, world, SPP)
    with pt_amd.Scene(tri, bvh, device=0) as s:
        acc = s.render(meta, f0, n, stride, DEPTH, pt_amd.MODE_AUTO)
    t = torch.from_numpy(acc)
    reduce_accum(t, dist)
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(240, method="thread")
def test_two_ranks_hip_render_gloo_reduce(packed, tmp_path):
    import torch.multiprocessing as mp

    import oracle
    from pt_amd.shard import frames_for_rank
    p = packed["CornellBox"]
    meta = p.meta_for(W, H)
    out = str(tmp_path / "acc.npy")
    mp.spawn(_worker, args=(2, _free_port(), p.triangle_data, p.bvh_data, meta, out), nprocs=2, join=True)
    got = np.load(out)
    parts = [oracle.render(p.triangle_data, p.bvh_data, meta, *frames_for_rank(r, 2, SPP), DEPTH)[0] for r in range(2)]
    assert np.array_equal((parts[0] + parts[1]).view(np.uint32), got.view(np.uint32))
    ref, _ = oracle.render(p.triangle_data, p.bvh_data, meta, 0, SPP, 1, DEPTH)
    assert np.allclose(got, ref, rtol=2e-6, atol=0)
