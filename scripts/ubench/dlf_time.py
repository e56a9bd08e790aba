"""Times svtgpu_dlf_pick + filter on a 4K 10-bit synthetic frame with the library at $SVTGPU_LIB (dev tool)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "svt-av1_pro-anchor-v2.1.0-_amd"))
import torch  # noqa: E402
import svtgpu  # noqa: E402
import synth  # noqa: E402

torch.cuda.init()
W, H, bd = 3840, 2160, 10
ctx = svtgpu.Context(0)
src, rec = synth.frame_pair(W, H, bd, seed=0x5EED0003)
R, S, D = (svtgpu.Frame(ctx, W, H, bd) for _ in range(3))
R.upload(rec)
S.upload(src)
dl = svtgpu.DlfState(ctx, W, H)
dl.set_mode_info(synth.mode_info(W, H, 3))
lf0 = svtgpu.LfParams.make(32, 32, 16, 16)
for _ in range(3):
    lfp = dl.pick(R, S, lf0, 0, 0, 0, 0, 0)
    dl.filter_to(R, D, lfp, 0, 3)
ctx.synchronize() if hasattr(ctx, "synchronize") else None
t0 = time.perf_counter()
for _ in range(10):
    lfp = dl.pick(R, S, lf0, 0, 0, 0, 0, 0)
    dl.filter_to(R, D, lfp, 0, 3)
D.download()
print(os.environ.get("SVTGPU_LIB", "default"), "dlf pick+filter ms", round((time.perf_counter() - t0) * 100, 3),
      lfp.levels())
