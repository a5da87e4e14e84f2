"""Multi-GPU sharding of a render.

Every (pixel, frame k) sample is independent (its seed depends only on the pixel index and
t_k, program-raymarch.wgsl:53,76), so frames are dealt round-robin: rank r of N renders
k = r, r+N, r+2N, ... over the whole image into its own f32 accumulator, and ONE sum-reduce
(RCCL over xGMI on GPUs, gloo in the CPU tests) combines the partial accumulators on rank 0.
Interleaving by frame, not by image tile, balances the load: the light, the open box front
and the depth of paths are uneven across tiles but identical in distribution across frames.

Summation order: the reference adds frames into one accumulator in frame order
(program-raymarch.ts:283-285).  Sharded, each rank adds its frames in order and the reduce
then adds the N partial sums, so results match the single-GPU accumulator to f32 rounding,
not bit for bit (tests/test_multigpu.py states the tolerance).
"""
from __future__ import annotations


def frames_for_rank(rank: int, world: int, spp: int, frame0: int = 0):
    """(first frame, count, stride) of rank's share of frames frame0 .. frame0+spp-1."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    count = len(range(rank, spp, world))
    return frame0 + rank, count, world


def reduce_accum(acc, dist, dst: int = 0):
    """Sum-reduce the per-rank accumulators onto `dst` (one collective per render)."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        if acc.is_cuda and dist.get_backend() == "gloo":  # rehearsal backend: through host memory
            h = acc.cpu()
            dist.reduce(h, dst=dst, op=dist.ReduceOp.SUM)
            if dist.get_rank() == dst:
                acc.copy_(h)
        else:
            dist.reduce(acc, dst=dst, op=dist.ReduceOp.SUM)
    return acc
