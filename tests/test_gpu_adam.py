"""GPU: seg_amd.Adam (one-launch HIP step, csrc/adam.hip) against torch.optim.Adam --
the reference's optimizer (main.py:100) -- on the same parameters and gradients.

Tolerance: the HIP step runs the foreach implementation's fp32 operations in the same
order, so parameters after several steps agree to a few fp32 ulps (rtol 2e-6); the
state (exp_avg, exp_avg_sq, step) matches as well and round-trips through state_dict.
"""
import pytest
import torch

from seg_amd import Adam

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(256, 1344, 3, 3), (10,), (3,), (4097,), (96, 16, 1, 1), (1,), (1000, 1280)]
    return [torch.nn.Parameter(torch.randn(s, generator=g).to(DEV)) for s in shapes]


@pytest.mark.parametrize("lr", [1.5e-4, 1e-2])
def test_adam_matches_torch(lr):
    ref, ours = _params(0), _params(0)
    o_ref = torch.optim.Adam(ref, lr=lr)
    o_ours = Adam(ours, lr=lr)
    g = torch.Generator().manual_seed(1)
    for step in range(5):
        for i, (a, b) in enumerate(zip(ref, ours)):
            if i == len(ref) - 1:  # an unused parameter (the classifier): no gradient, skipped
                a.grad = b.grad = None
                continue
            gr = (torch.randn(a.shape, generator=g) * 10.0 ** (-(i % 4) * 3)).to(DEV)
            if i == 1:
                gr[::2] = 0  # zero gradients: v == 0 -> denominator eps
            a.grad, b.grad = gr.clone(), gr.clone()
        o_ref.step()
        o_ours.step()
    torch.cuda.synchronize()
    for a, b in zip(ref, ours):
        torch.testing.assert_close(b, a, rtol=2e-6, atol=1e-7)
    for a, b in zip(ref[:-1], ours[:-1]):
        sa, sb = o_ref.state[a], o_ours.state[b]
        assert float(sa["step"]) == float(sb["step"]) == 5.0
        for k in ("exp_avg", "exp_avg_sq"):  # a few ulps of the tensor's scale (fma contraction may differ)
            torch.testing.assert_close(sb[k], sa[k], rtol=1e-6, atol=1e-6 * float(sa[k].abs().max()))
    assert len(o_ours.state[ours[-1]]) == 0
    # checkpoint compatibility: torch's state_dict loads into seg_amd.Adam and vice versa
    o2 = Adam(_params(0), lr=lr)
    o2.load_state_dict(o_ref.state_dict())
    o3 = torch.optim.Adam(_params(0), lr=lr)
    o3.load_state_dict(o_ours.state_dict())


def test_adam_rejects_unsupported():
    p = [torch.nn.Parameter(torch.randn(8, device=DEV))]
    p[0].grad = torch.randn(8, device=DEV)
    with pytest.raises(NotImplementedError):
        Adam(p, lr=1e-3, weight_decay=1e-4).step()
    q = [torch.nn.Parameter(torch.randn(8))]
    q[0].grad = torch.randn(8)
    with pytest.raises(NotImplementedError):
        Adam(q, lr=1e-3).step()
