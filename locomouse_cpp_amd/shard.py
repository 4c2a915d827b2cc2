"""Frame sharding across GPUs: one process per GPU, contiguous frame ranges,
no collective on the data path.

Frames are independent given the geometry except for a one-frame halo: the
pairwise costs of frame f need frame f-1's bottom candidates
(pairwisePotential, LocoMouse_class.cpp:896-919) and the motion check needs
its pixels (checkVelCriterion :1256-1267).  A shard that starts at frame
lo > 0 therefore hands frame lo-1 to its first batch as `prev_frame`; the
context recomputes that frame's candidates in its slot 0.  Inside a shard the
context carries frame state from batch to batch.

`detect(frames, first_frame, prev_frame)` is any callable with the
semantics of runtime.Context.detect (returns a result dict).
"""
from .results import concat_results


def shard_range(n_frames, rank, world):
    """Contiguous [lo, hi) of rank `rank`: ceil(n/world) frames per rank."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("rank must be in [0, world)")
    per = -(-n_frames // world)
    lo = min(n_frames, rank * per)
    return lo, min(n_frames, lo + per)


def detect_range(detect, frames, lo, hi, batch):
    """Frames [lo, hi) of `frames` (indexable by global frame index) in
    batches of at most `batch`; returns the concatenated result dict, or None
    for an empty range."""
    parts = []
    for b0 in range(lo, hi, batch):
        b1 = min(hi, b0 + batch)
        prev = frames[b0 - 1] if (b0 == lo and lo > 0) else None
        parts.append(detect(frames[b0:b1], b0, prev))
    return concat_results(parts) if parts else None


def run_sharded(detect, frames, n_frames, batch, group=None):
    """Every rank detects its shard; rank 0 returns the whole video's results
    in frame order (others return None).  The only exchange is the gather of
    the compact results (host objects over the process group), as the
    reference appends per-frame containers in frame order."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_range(n_frames, rank, world)
    mine = detect_range(detect, frames, lo, hi, batch)
    gathered = [None] * world if rank == 0 else None
    dist.gather_object(mine, gathered, dst=0, group=group)
    if rank != 0:
        return None
    return concat_results([g for g in gathered if g is not None])
