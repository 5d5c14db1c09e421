"""cProfile of the engine's host side over 20 training steps at a tiny shape (the GPU
work is negligible there, so the profile is the launch path)."""
import cProfile
import os
import pstats
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
import seg_amd  # noqa: E402
from seg_amd import engine  # noqa: E402

dev = torch.device("cuda", 0)
model = seg_amd.deterministic_init(seg_amd.MobileNetV2UNet(10), seed=0).to(dev).train()
engine.set_conv_math(model, sys.argv[1] if len(sys.argv) > 1 else "f32")
opt = torch.optim.Adam(model.parameters(), lr=1.5e-4)
x, y = seg_amd.synthetic_batch(1, 64, 128, 10, seed=1)
x, y = x.to(dev), y.to(dev)


def step():
    opt.zero_grad(set_to_none=True)
    loss = model.forward_loss(x, y)
    loss.backward()
    opt.step()


# the autograd engine runs our backward on its device thread: profile it there
bprof = cProfile.Profile()
_orig_bwd = engine._SegFunction.backward


def _bwd(ctx, gout):
    return bprof.runcall(_orig_bwd, ctx, gout)


engine._SegFunction.backward = staticmethod(_bwd)
for _ in range(3):
    step()
torch.cuda.synchronize()
bprof = cProfile.Profile()
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(12)
print("==== backward (autograd thread)")
pstats.Stats(bprof).sort_stats("tottime").print_stats(30)
