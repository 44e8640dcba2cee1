"""The fused pose-optimiser loss (torch_renderer_amd.losses.pose_loss, mr_pose_loss_*; SURVEY.md §8f
rank 4) against torch's own nn.L1Loss / HuberLoss(delta=0.05) / MSELoss on CPU, restating
camera_pose_optimizer.py:257-276 calc_loss: the total and its three terms within float32 rounding
of a different summation order (relative 1e-5), and the gradients w.r.t. depth, silhouette and
the RGBA image (through the [..., :3] view the reference passes) within 1e-6 of their scale.
Inputs include exact ties (silhouette == mask: L1's sign(0) = 0) and depth errors at exactly
+-delta (the Huber branch point)."""
import pytest
import torch

from tests.helpers import report
from torch_renderer_amd.losses import pose_loss

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _torch_loss(depth, sil, color, mask, depth_ref, rgb_ref):
    sil_loss = torch.nn.L1Loss()(sil, mask.float())
    color_loss = torch.nn.MSELoss()(color, rgb_ref)
    hloss = torch.nn.HuberLoss(delta=0.05)(torch.masked_select(depth, mask), torch.masked_select(depth_ref, mask))
    return sil_loss + hloss + color_loss * 0.01, (sil_loss, hloss, color_loss)


@pytest.mark.parametrize("shape", [(1, 64, 80), (3, 33, 47)])
@pytest.mark.parametrize("rgba_view", [True, False])
def test_pose_loss_matches_torch(shape, rgba_view):
    g = torch.Generator().manual_seed(7)
    depth = torch.rand(shape, generator=g) * 2
    depth_ref = depth + (torch.rand(shape, generator=g) - 0.5) * 0.2
    flat_d, flat_r = depth.view(-1), depth_ref.view(-1)
    flat_r[:5] = flat_d[:5] + 0.05   # exactly at the Huber branch point (in f32 arithmetic)
    flat_r[5:10] = flat_d[5:10]      # zero error
    mask = torch.rand(shape, generator=g) > 0.4
    sil = torch.rand(shape, generator=g)
    sil.view(-1)[:20] = mask.view(-1)[:20].float()  # exact ties: sign(0) = 0
    rgba = torch.rand(shape + (4,), generator=g)
    rgb_ref = torch.rand(shape + (3,), generator=g)
    # torch reference on CPU
    dr_, sr_, ir_ = (t.clone().requires_grad_(True) for t in (depth, sil, rgba))
    tot_r, terms_r = _torch_loss(dr_, sr_, ir_[..., :3], mask, depth_ref, rgb_ref)
    tot_r.backward()
    # fused on the GPU
    dg, sg, ig = (t.to(DEV).requires_grad_(True) for t in (depth, sil, rgba))
    color = ig[..., :3] if rgba_view else ig[..., :3].contiguous()
    tot, terms = pose_loss(dg, sg, color, mask.to(DEV), depth_ref.to(DEV), rgb_ref.to(DEV), return_terms=True)
    tot.backward()
    for name, a, b in (("total", tot, tot_r), ("sil", terms[0], terms_r[0]), ("huber", terms[1], terms_r[1]),
                       ("mse", terms[2], terms_r[2])):
        a, b = float(a.detach()), float(b.detach())
        print(f"[parity] pose_loss {name}: {a:.9g} vs torch {b:.9g}")
        assert abs(a - b) <= 1e-5 * max(abs(b), 1e-6), name
    report("pose_loss grad depth", dg.grad, dr_.grad, tol=1e-6)
    report("pose_loss grad sil", sg.grad, sr_.grad, tol=1e-6)
    report("pose_loss grad rgba", ig.grad, ir_.grad, tol=1e-6)


def test_pose_loss_deterministic_and_empty_mask():
    g = torch.Generator().manual_seed(3)
    shape = (2, 50, 60)
    args = [torch.rand(shape, generator=g).to(DEV), torch.rand(shape, generator=g).to(DEV),
            torch.rand(shape + (3,), generator=g).to(DEV), (torch.rand(shape, generator=g) > 0.5).to(DEV),
            torch.rand(shape, generator=g).to(DEV), torch.rand(shape + (3,), generator=g).to(DEV)]
    a = pose_loss(*args)
    b = pose_loss(*args)
    assert torch.equal(a, b)
    args[3] = torch.zeros(shape, dtype=torch.bool, device=DEV)
    assert torch.isnan(pose_loss(*args))  # torch: mean over an empty selection


@pytest.mark.parametrize("shape", [(2, 64, 80), (3, 33, 47)])
def test_pose_loss_upstream_scale_and_second_backward(shape):
    """The forward writes the gradients for dL/dtotal = 1 (mr_pose_loss_forward_grad, one pass; the
    (2, 64, 80) case is the vectorised kernel, (3, 33, 47) the two-pass fallback); a backward with
    another upstream rescales them (mr_pose_loss_scale), and a second backward over a retained graph
    recomputes them from the saved inputs: both against torch."""
    g = torch.Generator().manual_seed(11)
    depth = torch.rand(shape, generator=g) * 2
    depth_ref = depth + (torch.rand(shape, generator=g) - 0.5) * 0.2
    mask = torch.rand(shape, generator=g) > 0.4
    sil = torch.rand(shape + (4,), generator=g)
    rgba = torch.rand(shape + (4,), generator=g)
    rgb_ref = torch.rand(shape + (3,), generator=g)
    dr_, sr_, ir_ = (t.clone().requires_grad_(True) for t in (depth, sil, rgba))
    tot_r, _ = _torch_loss(dr_, sr_[..., 3], ir_[..., :3], mask, depth_ref, rgb_ref)
    (2.5 * tot_r).backward()
    dg, sg, ig = (t.to(DEV).requires_grad_(True) for t in (depth, sil, rgba))
    tot = pose_loss(dg, sg[..., 3], ig[..., :3], mask.to(DEV), depth_ref.to(DEV), rgb_ref.to(DEV))
    (2.5 * tot).backward(retain_graph=True)
    report("pose_loss x2.5 grad depth", dg.grad, dr_.grad, tol=1e-6)
    report("pose_loss x2.5 grad sil image", sg.grad, sr_.grad, tol=1e-6)
    report("pose_loss x2.5 grad rgba", ig.grad, ir_.grad, tol=1e-6)
    g1 = [t.grad.clone() for t in (dg, sg, ig)]
    tot.backward()  # second backward, upstream 1: the slow path from the saved inputs
    for a, b, name in zip((dg.grad, sg.grad, ig.grad), g1, ("depth", "sil", "rgba")):
        report(f"pose_loss second backward {name}", a - b, b / 2.5, tol=1e-6)
