"""Diagnostic (GPU): bf16-math model vs the fp64 oracle with its dense/pointwise conv
operands rounded to bf16 (emulated bf16 math), and vs the plain fp64 oracle."""
import sys
import torch

sys.path[:0] = ["team02-objectdetection_amd", "."]
from oracle import segref  # noqa: E402
from seg_amd import MobileNetV2UNet, UNet, engine  # noqa: E402
from seg_amd.detinit import deterministic_init, synthetic_batch  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def main(arch="MobileNetV2UNet", N=2, H=64, W=128):
    ctor = (lambda: MobileNetV2UNet(10)) if arch == "MobileNetV2UNet" else (lambda: UNet(10, 64))
    model_cpu = deterministic_init(ctor(), seed=5)
    x, y = synthetic_batch(N, H, W, 10, seed=6)
    p64 = segref.canonical_state(model_cpu.state_dict(), torch.float64)
    l64, z64, g64 = segref.forward_backward(arch, p64, x.double(), y, True)
    with segref.bf16_convs():
        p64 = segref.canonical_state(model_cpu.state_dict(), torch.float64)
        le, ze, ge = segref.forward_backward(arch, p64, x.double(), y, True)
    model = deterministic_init(ctor(), seed=5).cuda().train()
    engine.set_conv_math(model, "bf16")
    z = model(x.cuda())
    model.zero_grad(set_to_none=True)
    loss = model.forward_loss(x.cuda(), y.cuda())
    loss.backward()
    torch.cuda.synchronize()
    print(f"{arch}: emulated-bf16 oracle vs fp64: logits {rel(ze, z64):.3e} loss {rel(le, l64):.3e}")
    print(f"{arch}: GPU bf16 vs emulated: logits {rel(z, ze):.3e} loss {rel(loss, le):.3e}; vs fp64 logits {rel(z, z64):.3e}")
    seen = set()
    worst = []
    for k, p in model.named_parameters():
        if id(p) in seen or p.grad is None or k not in ge:
            continue
        seen.add(id(p))
        worst.append((rel(p.grad, ge[k]), rel(ge[k], g64[k]), k))
    worst.sort(reverse=True)
    for w in worst[:12]:
        print(f"  grad {w[2]}: gpu-vs-emul {w[0]:.3e}  emul-vs-fp64 {w[1]:.3e}")


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["MobileNetV2UNet"]))
    main("UNet", 2, 32, 64)
