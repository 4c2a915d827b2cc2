"""A runtime.Context-like `detect(frames, first_frame, prev_frame)` backed by
the CPU oracle, so the host-side batching/sharding logic can be exercised
without a GPU.  Test infrastructure only."""
import numpy as np

from locomouse_cpp_amd.results import slice_results


class OracleDetector:
    def __init__(self, cfg):
        self.cfg = cfg
        self.last = None
        self.last_frame = -1

    def __call__(self, frames, first_frame, prev_frame=None):
        from oracle import oracle as O
        frames = np.ascontiguousarray(frames)
        if first_frame == 0:
            run, drop = frames, 0
        else:
            if prev_frame is None:
                if self.last_frame != first_frame - 1:
                    raise ValueError("frame first_frame-1 was not processed: pass prev_frame")
                prev_frame = self.last
            # frame first_frame-1 replayed as the run's frame 0: the halo
            run, drop = np.concatenate([np.asarray(prev_frame)[None], frames]), 1
        res = slice_results(O.OracleRun(self.cfg, run).result, drop)
        res["first_frame"] = first_frame
        self.last = frames[-1].copy()
        self.last_frame = first_frame + len(frames) - 1
        return res
