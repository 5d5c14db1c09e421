"""Which parameter gradients change with SEG_BNOUT (ConvOp._bnout) on vs off -- diagnostic."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "team02-objectdetection_amd"), REPO]
from seg_amd import MobileNetV2UNet, engine  # noqa: E402
from seg_amd.detinit import deterministic_init, synthetic_batch  # noqa: E402

math = sys.argv[1] if len(sys.argv) > 1 else "f32"
x, y = synthetic_batch(4, 64, 128, 10, seed=5)
x, y = x.cuda(), y.cuda()
res = {}
used = {}
orig = engine.ConvOp._bnout


def spy(self, rt, i):
    r = orig(self, rt, i)
    if r is not None:
        used.setdefault(flag, []).append(r[1])
    return r


engine.ConvOp._bnout = spy
for flag in (False, True):
    engine.BNOUT = flag
    model = deterministic_init(MobileNetV2UNet(10), seed=5).cuda()
    engine.set_conv_math(model, math)
    model.train()
    loss = model.forward_loss(x, y)
    loss.backward()
    torch.cuda.synchronize()
    res[flag] = {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}
    names = {id(m): n for n, m in model.named_modules()}
    if flag:
        prog = engine.get_program(model, 4, 64, 128, math)
        for op in used.get(True, []):
            print("bnout for", names.get(id(op.bn)), op.cout, op.y.M)
for k in res[False]:
    a, b = res[True][k].double(), res[False][k].double()
    r = float((a - b).norm() / max(float(b.norm()), 1e-30))
    if r > 1e-6:
        print(f"{r:10.3e}  {k}")
