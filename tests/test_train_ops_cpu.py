"""Host-side pieces of the training ops that need no GPU: the kernel-3 tap gather of the task
heads' grouped convs (train_ops.taps3) against the pad + three slices + cat it replaces, values
and gradients in float64."""
import torch
import torch.nn.functional as F


def test_taps3_matches_pad_slices():
    from projects.mmdet3d_plugin.models.utils import train_ops as ops
    g = torch.Generator().manual_seed(0)
    x = torch.randn(6, 2, 37, 64, dtype=torch.float64, generator=g, requires_grad=True)
    dy = torch.randn(6, 2, 37, 192, dtype=torch.float64, generator=g)
    y = ops.taps3(x)
    y.backward(dy)
    got = x.grad.clone()
    x.grad = None
    n = x.shape[-2]
    xp = F.pad(x, (0, 0, 1, 1))
    want = torch.cat([xp[..., 0:n, :], xp[..., 1:n + 1, :], xp[..., 2:n + 2, :]], -1)
    want.backward(dy)
    assert torch.equal(y, want)
    assert (got - x.grad).abs().max().item() < 1e-12
