"""The N-rank path with ranks that actually render: two processes on the one GPU of the
test box, each rendering its shard of the views with DepthColorRender fwd + bwd (what bench.py's ranks
run), the shared vertex gradient all-reduced and the depth images gathered to rank 0 over gloo (the
measured multi-GPU runs use RCCL; the host logic is the same). Rank 0 checks the gathered images
bitwise and the all-reduced vertex gradient against one process rendering every view."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup(n_total, H, W):
    from tests.helpers import canonical_views, mesh_arrays
    from torch_renderer_amd.structures import Meshes, TexturesVertex

    verts, faces, _ = mesh_arrays("cow")
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, n_total, H, W, dist=0.5)
    g = torch.Generator().manual_seed(4)
    grads = [torch.rand(n_total, H, W, generator=g) * 2 - 1, torch.rand(n_total, H, W, generator=g) * 2 - 1,
             torch.rand(n_total, H, W, 3, generator=g) * 2 - 1]
    return verts, faces, R_cv, t_cv, K, grads, Meshes, TexturesVertex


def _render(verts, faces, R_cv, t_cv, K, grads, H, W, Meshes, TexturesVertex, dev):
    from torch_renderer_amd.torch_renderer import DepthColorRender

    v = verts.to(dev).requires_grad_(True)
    n = R_cv.shape[0]
    m = Meshes([v], [faces.to(dev)], TexturesVertex([torch.ones_like(v).detach()])).extend(n)
    depth, sil, rgb = DepthColorRender(K.to(dev), (H, W), device=dev).render(m, R_cv.to(dev).contiguous(),
                                                                             t_cv.to(dev).contiguous())
    torch.autograd.backward([depth, sil, rgb], [x.to(dev) for x in grads])
    return depth.detach(), v


def _worker(rank, world, port, n_total, H, W, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        from torch_renderer_amd import distributed as D

        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        verts, faces, R_cv, t_cv, K, grads, Meshes, TexturesVertex = _setup(n_total, H, W)
        s, e = D.shard_range(n_total, rank, world)
        depth, v = _render(verts, faces, R_cv[s:e], t_cv[s:e], K, [x[s:e] for x in grads], H, W, Meshes,
                           TexturesVertex, dev)
        D.allreduce_grads([v])
        full_depth = D.gather_to_root(depth, n_total)
        res = None
        if rank == 0:
            ref_depth, vr = _render(verts, faces, R_cv, t_cv, K, grads, H, W, Meshes, TexturesVertex, dev)
            err = (v.grad - vr.grad).abs().max().item()
            scale = max(1.0, vr.grad.abs().max().item())
            res = {"depth_equal": bool(torch.equal(full_depth, ref_depth)), "grad_err": err, "scale": scale,
                   "covered": int((ref_depth > 0).sum())}
        dist.barrier()
        q.put((rank, res))
        dist.destroy_process_group()
    except Exception as exc:  # surfaced by the parent
        q.put((rank, {"error": repr(exc)}))


def test_two_ranks_render_allreduce_gather_equals_single_process():
    world, n_total, H, W = 2, 6, 96, 96
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, H, W, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert res[r] is None or "error" not in res[r], res[r]
    r0 = res[0]
    print(f"[multirank] gathered depth bitwise {r0['depth_equal']}, covered {r0['covered']}, all-reduced vertex "
          f"grad max |diff| {r0['grad_err']:.3e} (scale {r0['scale']:.3e})")
    assert r0["covered"] > 0 and r0["depth_equal"]
    # the per-face sums are grouped by rank (views 0-2 + views 3-5) instead of all six in order
    assert r0["grad_err"] <= 1e-5 * r0["scale"]
