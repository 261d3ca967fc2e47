"""--trace_steps a:b -> torch.profiler (roctracer on ROCm) Chrome trace per rank; the reference
collected FULL_TRACE RunMetadata every step and never exported it."""
import os

import torch


class StepTracer:
    def __init__(self, spec, outdir, rank=0):
        self.start = self.stop = None
        if spec:
            a, b = spec.split(":")
            self.start, self.stop = int(a), int(b)
        self.outdir, self.rank = outdir, rank
        self.prof = None

    def step(self, i):
        if self.start is None:
            return
        if i == self.start:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self.prof = torch.profiler.profile(activities=acts, record_shapes=False)
            self.prof.__enter__()
        elif i == self.stop and self.prof is not None:
            self.prof.__exit__(None, None, None)
            os.makedirs(self.outdir, exist_ok=True)
            path = os.path.join(self.outdir, "trace_rank%d_steps%d-%d.json" % (self.rank, self.start, self.stop))
            self.prof.export_chrome_trace(path)
            self.prof = None
            return path
        return None
