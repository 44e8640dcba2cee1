#!/usr/bin/env python3
"""Headline benchmark: frames/s of fwd+bwd at 512x512, cow mesh (F=5856), 64 views per GPU.

One step = DepthColorRender.render over the rank's 64 views (depth + silhouette +
Phong RGB from one raster pass, TexturesUV cow texture, PointLights (0,0,-3))
followed by the backward of sum(gD*depth + gS*sil + gC*rgb) (fixed U(-1,1)
upstream grads) to the shared vertex positions and every view's OpenCV R, t.
With N > 1 ranks (one process per GPU, torch.distributed over RCCL) each rank
renders its own 64 views (weak scaling) and the shared vertex gradient (V x 3
f32) is all-reduced every step — the only data exchange the path has.

    python bench.py [--gpus N --steps K --warmup W]
Prints ONE JSON line on rank 0 (contract in the task statement / DESIGN.md §Measurement).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec fwd+bwd, 512×512, ~6k-face mesh, batch=64; 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0


def view_distance(mesh, verts):
    """0.5 m for the cow; other meshes at the same distance relative to their extent
    (the cow's 0.172 m), so the framing matches (dolphin 0.71 m -> 2.1 m)."""
    if mesh == "cow":
        return 0.5
    ext = float((verts.max(0).values - verts.min(0).values).max())
    return 0.5 * ext / 0.172


def canonical_views(verts, n_total, H, W, dist_m=0.5, fov_deg=60.0, seed=0):
    """OpenCV look-at from 0.5 m to the centroid, azimuth 360*i/n,
    elevation ~U[-20, 60] deg (seeded), fx = fy for a 60 deg FoV, centred principal point."""
    from torch_renderer_amd.transforms import opencv_look_at

    g = torch.Generator().manual_seed(seed)
    c = verts.mean(0).double()
    az = torch.arange(n_total, dtype=torch.float64) * (2 * math.pi / n_total)
    el = torch.empty(n_total, dtype=torch.float64).uniform_(math.radians(-20.0), math.radians(60.0), generator=g)
    C = torch.stack([dist_m * torch.cos(el) * torch.sin(az), dist_m * torch.sin(el),
                     dist_m * torch.cos(el) * torch.cos(az)], dim=1) + c
    R_cv, t_cv = opencv_look_at(C, c)
    f = (W / 2.0) / math.tan(math.radians(fov_deg) / 2.0)
    K = torch.tensor([[f, 0.0, W / 2.0], [0.0, f, H / 2.0], [0.0, 0.0, 1.0]])
    return R_cv, t_cv, K


def cpu_baseline(verts, faces, d, R_cv, t_cv, K, H, W, n_views=2, reps=3, mesh="cow"):
    """Reference CPU path restated (oracle: C naive rasterizer + torch-CPU shading/autograd) on a
    bounded sample of the same workload: `n_views` frames, 1 warm-up + `reps` timed fwd+bwd passes
    on all host cores, then one view, one timed pass on 1 core."""
    import numpy as np

    from oracle import oracle as O
    from torch_renderer_amd.transforms import opencv_to_pytorch3d

    tex = None  # untextured meshes (dolphin, teapot): white, as the GPU path
    if "texture_u8" in d:
        img = torch.from_numpy(d["texture_u8"].astype(np.float32) / 255.0)
        tex = ("uv", torch.from_numpy(d["verts_uvs"]).float(), torch.from_numpy(d["faces_uvs"]).long(), img)
    s = min(H, W) / 2.0
    intr1 = torch.tensor([[K[0, 0] / s, (W / 2.0 - K[0, 2]) / s, K[1, 1] / s, (H / 2.0 - K[1, 2]) / s]]).float()
    gen = torch.Generator().manual_seed(1)
    gD = torch.rand(n_views, H, W, generator=gen) * 2 - 1
    gS = torch.rand(n_views, H, W, generator=gen) * 2 - 1
    gC = torch.rand(n_views, H, W, 3, generator=gen) * 2 - 1

    def one_pass(nv):
        v = verts.clone().requires_grad_(True)
        Rc = R_cv[:nv].clone().requires_grad_(True)
        tc = t_cv[:nv].clone().requires_grad_(True)
        Rp, Tp = opencv_to_pytorch3d(Rc, tc)
        out = O.render_ref(v, faces, Rp, Tp, intr1.expand(nv, 4).contiguous(), H, W, texture=tex)
        torch.autograd.backward([out["depth"], out["sil"], out["rgba"][..., :3]], [gD[:nv], gS[:nv], gC[:nv]])

    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or cores
    threads = min(omp, cores)
    tt = torch.get_num_threads()
    O.set_threads(threads)
    times = []
    for it in range(reps + 1):
        t0 = time.perf_counter()
        one_pass(n_views)
        if it > 0:
            times.append(time.perf_counter() - t0)
    sec = sum(times) / len(times)
    # 1 core: C rasterizer and torch both single-threaded, one view, one timed pass
    O.set_threads(1)
    torch.set_num_threads(1)
    t0 = time.perf_counter()
    one_pass(1)
    sec1 = time.perf_counter() - t0
    torch.set_num_threads(tt)
    O.set_threads(threads)
    return {"value": n_views / sec, "unit": "frames/s", "cores": threads, "kind": "port",
            "value_1core": round(1.0 / sec1, 4),
            "sample": f"{n_views} views of the same workload ({mesh}, {H}x{W}, fwd+bwd), 1 warm-up + {reps} timed "
                      f"passes, {sec:.2f} s/pass: C naive rasterizer (OpenMP {threads} threads) + torch-CPU "
                      f"shading/autograd ({tt} threads); 1 core: 1 view, 1 timed pass, {sec1:.2f} s"}


# Algorithmic bytes per launch: what each kernel must move at minimum for the
# launch's batch, from the forward's own work counters (kernels.render_stats: list entries,
# covered pixels). Device-side caches may serve part of it; rocprof FETCH/WRITE is reported
# beside it as roofline.traffic.
def algorithmic_bytes(kernel, H, W, F, views, st, bgpix=0):
    """bgpix: pixels whose background k_bin_view's spare workgroups write (mr_binning_background_pixels);
    k_tile_raster writes the background of the others."""
    HW, cov, ent, slots, units = H * W, st["covered"], st["entries"], st["tiles"], st.get("units", 0)
    table = {
        # background (depth + silhouette + rgb(3)) of the pixels k_bin_view did not take, list ids,
        # each face record once, 64 winners per non-empty tile
        "k_tile_raster": 20 * (HW * views - bgpix) + 4 * ent + 64 * F * views + 256 * slots,
        "k_shade<1>": 256 * slots + 20 * cov,              # winners in, 20 B of outputs per covered pixel
        "k_bwd_shade": 256 * slots + (20 + 80) * cov,      # winners + upstream grads, 80-B gradient record out
        "k_bwd_geom": 256 * slots + 80 * cov + 72 * F,     # winners + gradient record in, per-face rows out
        # fused backward: winners + R/T partial per tile, upstream grads per covered pixel, each
        # face's packed record + ShadeRec read once and its 72-B gradient row written once (the
        # per-pixel record gathers are cache traffic, reported by PMC as roofline.traffic)
        "k_bwd_fused": (256 + 48) * slots + 20 * cov + (64 + 144 + 72) * F,
        "k_bin_count": 64 * F * views + 24 * F,            # face records out, mesh in
        "k_bin_fill": 64 * F * views + 4 * ent,            # face records in, list ids out
        "k_bin_rect": (64 + 4) * F * views + 24 * F,       # face records + tile rectangles out, mesh in
        # rectangles in, list ids + work units out, the background of bgpix pixels
        "k_bin_view": 4 * F * views + 4 * ent + 16 * units + 20 * bgpix,
    }
    return table.get(kernel)


# Forward fragment pass (everything from projected geometry to the three images): API-minimum
# bytes per frame = 20 B/px of outputs + 36 B/face of geometry (without p2f).
FORWARD_KERNELS = ("k_setup_zero", "k_vertex_normals", "k_shade_rec", "k_bin_count", "k_bin_scan", "k_bin_fill",
                   "k_bin_rect", "k_bin_view", "k_unit_order",
                   "k_tile_raster", "k_shade<1>")


# Minimum HBM traffic of the fused fwd+bwd step per frame: the three images written once (20 B/px:
# depth, silhouette, rgb), the upstream gradients of the covered pixels read once (20 B each; the
# backward never touches an uncovered pixel's gradient, its contribution is zero), the mesh in and
# its vertex gradients out (108 B/face) and the texture read once (12 B/texel), amortised over the
# views. (SURVEY §8d's 96 B/px also charged the modular path's fragment tensors, which the fused
# path never materialises, and the gradients of every pixel.)
def path_bytes_per_frame(H, W, F, tex_texels, views, covered):
    return 20 * H * W + 20 * covered / views + 108 * F + 12 * tex_texels / views


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--views", type=int, default=64, help="views per GPU")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--mesh", default="cow")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fragment-pass", action="store_true",
                    help="render mode: skip the fragment-pass measurement that follows the headline step")
    ap.add_argument("--cpu-views", type=int, default=2)
    ap.add_argument("--no-secondary", action="store_true",
                    help="render mode: skip the C3 / C5 / soft steps that follow the headline (A/B runs)")
    ap.add_argument("--eager", action="store_true",
                    help="enqueue every step from Python instead of replaying one captured HIP graph")
    ap.add_argument("--texture", choices=("uv", "white"), default="uv",
                    help="experiments only: 'white' drops the UV texture (not the benchmark workload)")
    ap.add_argument("--mode", choices=("render", "fragments", "soft", "gather", "pose", "c5"), default="render",
                    help="render: the headline fwd+bwd step; fragments: the rasterizer alone "
                         "(MeshRasterizer -> PyTorch3D Fragments, K=1; the north-star fragment-pass roofline); "
                         "soft: K=50 soft silhouette fwd+bwd (deform_mesh_with_color.py); gather: C4, depth "
                         "render of --views views IN TOTAL sharded over the ranks + RCCL gather to rank 0 "
                         "(batch_rendering_test.py, strong scaling); pose: C3, camera_pose_optimizer.py's step "
                         "(three renders, calc_loss, backward, Adam) for --views poses per GPU; c5: "
                         "mesh_deformer.py color_train's step (F=81,920 sphere, 1024x1024, --views single-view "
                         "renders per step, default 5)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
    # one GPU per rank; MR_BENCH_REHEARSE=1 (tests only) lets several ranks share the visible GPUs
    # over gloo to rehearse the N-rank path on a 1-GPU box; the measured runs use RCCL
    rehearse = os.environ.get("MR_BENCH_REHEARSE") == "1"
    local = local % torch.cuda.device_count() if rehearse else local
    torch.cuda.set_device(local)  # before the process group: RCCL binds its communicator to this device
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo" if rehearse else "nccl")

    if args.mode == "fragments":
        return bench_fragments(args, dev, world, rank)
    if args.mode == "soft":
        return bench_soft(args, dev, world, rank)
    if args.mode == "gather":
        return bench_gather(args, dev, world, rank)
    if args.mode == "pose":
        return bench_pose(args, dev, world, rank)
    if args.mode == "c5":
        return bench_c5(args, dev, world, rank)
    from torch_renderer_amd import _lib
    from torch_renderer_amd import distributed as D
    from torch_renderer_amd.assets import load_asset, load_asset_arrays
    from torch_renderer_amd.structures import Meshes
    from torch_renderer_amd.torch_renderer import DepthColorRender

    H = W = args.size
    d = load_asset_arrays(args.mesh)
    meshes = load_asset(args.mesh, device=dev)
    verts0 = meshes.shared_verts().detach().cpu()
    faces = meshes.shared_faces()
    Fn = faces.shape[0]
    nv = args.views
    R_all, t_all, K = canonical_views(verts0, nv * world, H, W, dist_m=view_distance(args.mesh, verts0))
    R_cv, t_cv = D.shard_views(R_all, t_all, rank=rank, world_size=world)
    R_cv = R_cv.to(dev).contiguous().requires_grad_(True)
    t_cv = t_cv.to(dev).contiguous().requires_grad_(True)
    verts = meshes.shared_verts().clone().requires_grad_(True)
    tex = meshes.textures
    if args.texture == "white" or tex is None:  # untextured meshes render white (drop-in default)
        from torch_renderer_amd.structures import TexturesVertex
        tex = TexturesVertex([torch.ones_like(verts).detach()])
    bmesh = Meshes([verts], [faces], tex).extend(nv)
    renderer = DepthColorRender(K.to(dev), (H, W), device=dev)
    gen = torch.Generator().manual_seed(1 + rank)
    gD = (torch.rand(nv, H, W, generator=gen) * 2 - 1).to(dev)
    gS = (torch.rand(nv, H, W, generator=gen) * 2 - 1).to(dev)
    gC = (torch.rand(nv, H, W, 3, generator=gen) * 2 - 1).to(dev)

    def fwd_bwd():
        depth, sil, rgb = renderer.render(bmesh, R_cv, t_cv)
        torch.autograd.backward([depth, sil, rgb], [gD, gS, gC])

    def eager_step():
        verts.grad = None
        R_cv.grad = None
        t_cv.grad = None
        fwd_bwd()

    for _ in range(args.warmup):
        eager_step()
        if world > 1:
            D.allreduce_grads([verts])
    from torch_renderer_amd.kernels import render_stats
    _keep = renderer.render(bmesh, R_cv, t_cv)  # autograd keeps the forward workspace alive
    wstats = render_stats()  # work counters of this rank's batch (bytes of data-dependent kernels)
    del _keep
    torch.cuda.synchronize()

    # One step = fwd+bwd of the rank's views (+ the shared-vertex-gradient all-reduce when N > 1).
    # Default: the step is captured into HIP graphs and replayed (every kernel of the step runs each
    # replay; only the Python/launch enqueue work is removed): one graph at N = 1; with N > 1 the forward
    # and the backward are two graphs (one memory pool), and the all-reduce of step k's vertex gradient
    # runs on a side stream while step k+1's forward replays (the forward never reads verts.grad); the backward of step k+1, which
    # rewrites it, waits for the collective — so RCCL's latency hides behind the forward.
    if args.eager:
        fwd_only = bwd_only = None
    else:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                eager_step()
        torch.cuda.current_stream().wait_stream(side)
        verts.grad = None
        R_cv.grad = None
        t_cv.grad = None
        pool = torch.cuda.graph_pool_handle()
        if world == 1:
            # one rank: nothing to overlap between the forward and the backward, so one graph holds the
            # whole step (no graph-boundary gap between the two halves)
            g_fwd = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_fwd, pool=pool):
                outs_static = renderer.render(bmesh, R_cv, t_cv)
                torch.autograd.backward(list(outs_static), [gD, gS, gC])
            # keep the static outputs' memory but not their autograd graph: alive, it would keep the leaves'
            # AccumulateGrad nodes (created on the capture stream) for the eager steps below, whose backward
            # then accumulates across streams (torch's "AccumulateGrad node's stream does not match" warning,
            # which preceded the round-5 capture crash; DESIGN §6, tests/test_gpu_round6.py)
            outs_static = tuple(o.detach() for o in outs_static)
            g_bwd = None
            fwd_only, bwd_only = g_fwd.replay, (lambda: None)
        else:
            g_fwd, g_bwd = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_fwd, pool=pool):
                outs_static = renderer.render(bmesh, R_cv, t_cv)
            with torch.cuda.graph(g_bwd, pool=pool):
                torch.autograd.backward(list(outs_static), [gD, gS, gC], retain_graph=True)
            outs_static = tuple(o.detach() for o in outs_static)  # (as above: no autograd graph kept alive)
            fwd_only, bwd_only = g_fwd.replay, g_bwd.replay

    comm = torch.cuda.Stream() if world > 1 else None
    ar_events = []  # (start, end) HIP events around each timed step's all_reduce (on the comm stream)
    pending = [False]

    def step(timed=False):
        if fwd_only is None:  # eager launches (--eager)
            eager_step()
            if world > 1:
                D.allreduce_grads([verts])
            return
        fwd_only()
        if pending[0]:  # step k's all-reduce must finish before step k+1's backward rewrites verts.grad
            torch.cuda.current_stream().wait_stream(comm)
        bwd_only()
        if world > 1:
            comm.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(comm):
                if timed:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                D.allreduce_grads([verts])  # the step's only exchange: shared vertex grads
                if timed:
                    e1.record()
                    ar_events.append((e0, e1))
            pending[0] = True

    for _ in range(2):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the collective's duration on its side stream (overlapped with the next step's forward): mean over
    # the timed steps, max over ranks
    allreduce_us = None
    if ar_events:
        allreduce_us = sum(a.elapsed_time(b) for a, b in ar_events) / len(ar_events) * 1e3
        t_ar = torch.tensor([allreduce_us], device=dev, dtype=torch.float64)
        dist.all_reduce(t_ar, op=dist.ReduceOp.MAX)
        allreduce_us = t_ar.item()
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = e.item()
    # the replayed graph's gradients against an eager step's: bitwise (the step is deterministic), so
    # the graph runs exactly the step's work
    graph_check = None
    if fwd_only is not None and world == 1:
        torch.cuda.synchronize()
        g_graph = (verts.grad.clone(), R_cv.grad.clone(), t_cv.grad.clone())
        eager_step()
        torch.cuda.synchronize()
        graph_check = all(torch.equal(a, b) for a, b in zip(g_graph, (verts.grad, R_cv.grad, t_cv.grad)))
    # per-kernel device times: HIP events around every launch of a few eager steps (same kernels)
    torch.cuda.synchronize()
    _lib.timing_enable(True)
    for _ in range(min(args.steps, 20)):
        eager_step()
    torch.cuda.synchronize()
    kt = _lib.timing_read()
    _lib.timing_enable(False)
    # rehearsal check (MR_BENCH_REHEARSE, N ranks sharing one GPU over gloo): the all-reduced vertex
    # gradient equals rank 0's single-process fwd+bwd of ALL the ranks' views (tolerance: the per-face sums
    # are grouped by rank there)
    ar_check = None
    if world > 1 and rehearse:
        step()
        torch.cuda.synchronize()
        g_ar = verts.grad.detach().clone()
        if rank == 0:
            Rf, tf = R_all.to(dev).contiguous(), t_all.to(dev).contiguous()
            vf = meshes.shared_verts().clone().requires_grad_(True)
            genf = torch.Generator().manual_seed(1)
            parts = []
            for r in range(world):  # each rank's upstream grads (seeded 1 + r), in rank order
                gr = torch.Generator().manual_seed(1 + r)
                parts.append(((torch.rand(nv, H, W, generator=gr) * 2 - 1), (torch.rand(nv, H, W, generator=gr) * 2 - 1),
                              (torch.rand(nv, H, W, 3, generator=gr) * 2 - 1)))
            del genf
            full = DepthColorRender(K.to(dev), (H, W), device=dev)
            fm = Meshes([vf], [faces], tex).extend(nv * world)
            outs_f = full.render(fm, Rf, tf)
            torch.autograd.backward(list(outs_f), [torch.cat([p[i] for p in parts]).to(dev) for i in range(3)])
            err = (vf.grad - g_ar).abs().max().item()
            scale = max(1.0, vf.grad.abs().max().item())
            ar_check = {"vertex_grad_max_abs_diff": err, "scale": scale, "ok": bool(err <= 1e-4 * scale)}
    # the north-star fragment pass (MeshRasterizer -> Fragments, K = 1) on the same mesh, size and views,
    # timed in the same run so that the driver's record carries it
    if not args.eager:
        del g_fwd, g_bwd, outs_static
    torch.cuda.synchronize()
    frag = None
    if not args.no_fragment_pass:
        f_el, f_kt, f_cov, _ = measure_fragments(args, dev, world, rank)
        frag = fragment_pass_summary(args, f_el, f_kt, f_cov, Fn, world)
    # (one GPU only: the multi-GPU lines report the headline's scaling; a secondary workload's collective
    # must never be able to stall a scaling run)
    secondary = {} if args.no_secondary or world > 1 else secondary_steps(args, dev, world, rank)

    if rank != 0:
        dist.destroy_process_group()
        return

    frames = nv * world * args.steps
    value = frames / elapsed
    # dominant kernel (by summed device time) and its roofline point
    dom = max(kt.items(), key=lambda kv: kv[1][1]) if kt else None
    roof = None
    pmc = {}
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as fh:
            pmc = json.load(fh)
    if dom is not None:
        name, (launches, total_ms) = dom
        avg_s = total_ms / launches / 1e3
        bgpix = int(_lib.load().mr_binning_background_pixels(nv, Fn, H, W, 1))
        b = algorithmic_bytes(name, H, W, Fn, nv, wstats, bgpix)
        ent = pmc.get(name)
        traffic = ent.get("hbm_bytes_per_launch") if ent and ent.get("config") == f"{args.mesh}-{H}x{W}-{nv}" else None
        if b is not None:
            gbs = b / avg_s / 1e9
            roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": name,
                    "avg_launch_us": round(avg_s * 1e6, 2), "algorithmic_bytes_per_launch": b}
            # the second-longest kernel's point as well (the raster and the backward take about the same time)
            ranked = sorted(kt.items(), key=lambda kv: -kv[1][1])
            if len(ranked) > 1:
                name2, (l2, t2) = ranked[1]
                b2 = algorithmic_bytes(name2, H, W, Fn, nv, wstats, bgpix)
                if b2 is not None:
                    s2 = t2 / l2 / 1e3
                    e2 = pmc.get(name2)
                    roof["runner_up"] = {
                        "kernel": name2, "avg_launch_us": round(s2 * 1e6, 2), "algorithmic_bytes_per_launch": b2,
                        "achieved": round(b2 / s2 / 1e9, 1), "frac": round(b2 / s2 / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": e2.get("hbm_bytes_per_launch") if e2 and e2.get("config") == f"{args.mesh}-{H}x{W}-{nv}"
                        else None}
    fwd_us = sum(kt[k][1] / kt[k][0] * 1e3 for k in FORWARD_KERNELS if k in kt)
    fwd_bytes = (20 * H * W + 36 * Fn) * nv
    fwd_roof = {"kernels": [k for k in FORWARD_KERNELS if k in kt], "us_per_launch": round(fwd_us, 2),
                "algorithmic_bytes": fwd_bytes, "achieved": round(fwd_bytes / (fwd_us * 1e-6) / 1e9, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(fwd_bytes / (fwd_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)} if fwd_us > 0 else None
    kernels = {k: {"launches": v[0], "avg_us": round(v[1] / max(v[0], 1) * 1e3, 2),
                   "share": round(v[1] / sum(x[1] for x in kt.values()), 3)} for k, v in kt.items()}
    texels = d["texture_u8"].shape[0] * d["texture_u8"].shape[1] if "texture_u8" in d else 0
    pb = path_bytes_per_frame(H, W, Fn, texels, nv, wstats["covered"])
    path_roof = {"bytes_per_frame": int(pb), "achieved": round(value * pb / 1e9, 1), "peak": HBM_PEAK_GBS,
                 "unit": "GB/s", "frac": round(value * pb / 1e9 / HBM_PEAK_GBS, 4)}
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(verts0, faces.cpu(), d, R_all, t_all, K, H, W, n_views=args.cpu_views, mesh=args.mesh)
    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "launch": "eager" if args.eager else "hipgraph",
        "graph_grads_equal_eager": graph_check,
        "data": (f"synthetic camera poses on the reference's {args.mesh} mesh"
                 + (" + texture (assets/cow.npz from data/cow_mesh)" if "texture_u8" in d and args.texture == "uv"
                    else " (white: no texture map)")),
        "config": {"workload": f"{args.mesh} (F={Fn}, V={verts0.shape[0]}), {H}x{W}, {nv} views/GPU, fwd+bwd: "
                               "depth+silhouette+Phong RGB from one raster pass, grads to verts and per-view R,t",
                   "mesh": args.mesh, "H": H, "W": W, "views_per_gpu": nv, "global_views": nv * world,
                   "parallelism": f"view-sharded x{world}"},
        "roofline": roof, "fragment_pass": frag, **secondary,
        "forward_roofline": fwd_roof, "path_roofline": path_roof,
        "cpu_baseline": cpu,
        "work": wstats, "kernels": kernels,
        "allreduce_us": None if allreduce_us is None else round(allreduce_us, 2),
        "allreduce_overlapped_with_forward": world > 1 and not args.eager,
        "allreduce_check": ar_check,
        "allreduce_bytes": 4 * 3 * int(verts0.shape[0]) if world > 1 else 0,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


FRAG_KERNELS = ("k_project_faces", "k_bin_count", "k_bin_scan", "k_bin_fill", "k_bin_rect", "k_bin_view", "k_tile_raster",
                "k_shade<0>")


def measure_fragments(args, dev, world, rank):
    """Time the fragment pass (see bench_fragments) for args.steps steps after args.warmup, max over
    ranks; returns (elapsed_s, per-kernel HIP-event times, covered pixels, F)."""
    from torch_renderer_amd import _lib
    from torch_renderer_amd import distributed as D
    from torch_renderer_amd.assets import load_asset
    from torch_renderer_amd.kernels import RasterizeMeshesWorld, mesh_topology
    from torch_renderer_amd.cameras import PerspectiveCameras, view_batch
    from torch_renderer_amd.transforms import opencv_to_pytorch3d

    H = W = args.size
    meshes = load_asset(args.mesh, device=dev, textures=False)
    verts = meshes.shared_verts()
    faces = meshes.shared_faces()
    Fn = faces.shape[0]
    nv = args.views
    R_all, t_all, K = canonical_views(verts.cpu(), nv * world, H, W, dist_m=view_distance(args.mesh, verts.cpu()))
    R_cv, t_cv = D.shard_views(R_all, t_all, rank=rank, world_size=world)
    Rp, Tp = opencv_to_pytorch3d(R_cv.to(dev), t_cv.to(dev))
    cams = PerspectiveCameras(focal_length=((float(K[0, 0]), float(K[1, 1])),),
                              principal_point=((float(K[0, 2]), float(K[1, 2])),), in_ndc=False,
                              image_size=torch.tensor([[H, W]]), device=dev)
    Rb, Tb, intr = view_batch(cams, (H, W), Rp, Tp, n_views=nv)
    # the poses as a caller holds them (row-major (N,3,3) / (N,3)): opencv_to_pytorch3d returns a
    # transposed view, whose per-call contiguous copy is input preparation, not the fragment pass
    Rb, Tb, intr = Rb.contiguous(), Tb.contiguous(), intr.contiguous()
    mesh_topology(faces, verts.shape[0])

    def step():  # MeshRasterizer.forward's native call for one mesh shared by the views
        return RasterizeMeshesWorld.apply(verts, Rb, Tb, faces, intr, nv, H, W, 1, 0.0, True, False, False, None)

    with torch.no_grad():
        for _ in range(args.warmup):
            out = step()
        del out
        _host_profile(step, dev)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        covered = int((out[0] >= 0).sum())
        del out
        if world > 1:
            e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            elapsed = e.item()
        _lib.timing_enable(True)
        for _ in range(min(args.steps, 20)):
            out = step()
        torch.cuda.synchronize()
        kt = _lib.timing_read()
        _lib.timing_enable(False)
        del out
        # the pass's device time: one HIP event pair around each whole pass on the launch stream (the
        # per-kernel pairs above add an event between every two kernels of the pass)
        evs = []
        for _ in range(min(args.steps, 20)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = step()
            e1.record()
            evs.append((e0, e1))
            del out
        torch.cuda.synchronize()
        pass_us = sum(a.elapsed_time(b) for a, b in evs) / len(evs) * 1e3
        # host cost of one call: the time step() takes to return (no synchronisation inside the loop; the
        # device queue absorbs the launches as long as it is not full)
        hs = []
        for _ in range(min(args.steps, 20)):
            h0 = time.perf_counter()
            out = step()
            hs.append(time.perf_counter() - h0)
            del out
        torch.cuda.synchronize()
        hs.sort()
        host_us = hs[len(hs) // 2] * 1e6
        # the same call captured once into a HIP graph and replayed (what a caller's captured training step
        # runs): the device work per step without the per-call host launch work, checked bitwise against an
        # eager call's fragments
        graph_us, graph_equal = None, None
        if world == 1:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(2):
                    out = step()
            torch.cuda.current_stream().wait_stream(side)
            del out
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, pool=torch.cuda.graph_pool_handle()):
                gout = step()
            graph.replay()
            eager = step()
            torch.cuda.synchronize()
            graph_equal = all(torch.equal(a, b) for a, b in zip(gout, eager))
            del eager
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                graph.replay()
            torch.cuda.synchronize()
            graph_us = (time.perf_counter() - t0) / args.steps * 1e6
            del graph, gout
            torch.cuda.synchronize()
    kt["__pass_us__"] = (1, pass_us / 1e3)
    kt["__host_us__"] = (1, host_us / 1e3)
    if graph_us is not None:
        kt["__graph_us__"] = (1, graph_us / 1e3)
        kt["__graph_equal__"] = (1, 1.0 if graph_equal else 0.0)
    return elapsed, kt, covered, Fn


def fragment_pass_summary(args, elapsed, kt, covered, Fn, world):
    """The north-star fragment-pass numbers (28 B/px + 36 B/face per frame against 8 TB/s):
    frac by the kernels' summed HIP-event time per step and by the timed step itself."""
    H = W = args.size
    nv = args.views
    value = nv * world * args.steps / elapsed
    per_frame = 28 * H * W + 36 * Fn
    pass_us = kt.pop("__pass_us__")[1] * 1e3
    host_us = kt.pop("__host_us__", (1, float("nan")))[1] * 1e3
    graph_us = kt.pop("__graph_us__", (1, None))[1]
    graph_us = None if graph_us is None else graph_us * 1e3
    graph_equal = kt.pop("__graph_equal__", (1, None))[1]
    us = sum(kt[k][1] / kt[k][0] * 1e3 for k in FRAG_KERNELS if k in kt)
    ach = per_frame * nv / (pass_us * 1e-6) / 1e9
    ach_k = per_frame * nv / (us * 1e-6) / 1e9
    dom = max(kt.items(), key=lambda kv: kv[1][1])
    return {"frames_per_s": round(value, 1), "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "bound": "hbm", "bytes_per_frame": per_frame, "kernels": [k for k in FRAG_KERNELS if k in kt],
            "kernel_us": {k: round(kt[k][1] / kt[k][0] * 1e3, 2) for k in FRAG_KERNELS if k in kt},
            # frac: algorithmic bytes / the pass's device time (one HIP event pair around the pass's launches);
            # kernel_sum_frac: / the sum of its kernels' times with an event pair around each kernel;
            # step_frac: / the timed step's wall time (host launch work included)
            "pass_us": round(pass_us, 2), "host_us_per_call": round(host_us, 1), "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4),
            "us_per_step": round(us, 2), "kernel_sum_frac": round(ach_k / HBM_PEAK_GBS, 4),
            "step_frac": round(value * per_frame / 1e9 / HBM_PEAK_GBS, 4),
            # the call captured in a HIP graph and replayed (no per-call host launch work): us per step and frac
            "graph_us_per_step": None if graph_us is None else round(graph_us, 2),
            "graph_step_frac": None if graph_us is None else round(per_frame * nv / (graph_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "graph_equals_eager": None if graph_equal is None else bool(graph_equal),
            "dominant_kernel": dom[0], "covered_pixels": covered,
            "workload": f"{args.mesh} (F={Fn}), {H}x{W}, {nv} views/GPU, MeshRasterizer(meshes_world, R, T) -> "
                        "Fragments(pix_to_face int64, zbuf, bary_coords, dists), K=1"}


def bench_fragments(args, dev, world, rank):
    """The fragment pass alone: MeshRasterizer(meshes_world, R, T) -> Fragments(pix_to_face int64, zbuf,
    bary_coords, dists), K=1 (camera_pose_optimizer.py:244-246, batch_rendering_test.py:274): projection
    + binning + raster + fragment writes in one native call (mr_rasterize_meshes_world, what
    MeshRasterizer.forward runs for an extended mesh). API-minimum bytes per frame:
    28 B/px of fragments + 36 B/face of face_verts."""
    elapsed, kt, covered, Fn = measure_fragments(args, dev, world, rank)
    if rank != 0:
        dist.destroy_process_group()
        return
    H = W = args.size
    nv = args.views
    frames = nv * world * args.steps
    value = frames / elapsed
    fp = fragment_pass_summary(args, elapsed, kt, covered, Fn, world)  # (takes the pass time out of kt)
    kernels = {k: {"launches": v[0], "avg_us": round(v[1] / max(v[0], 1) * 1e3, 2)} for k, v in kt.items()}
    line = {
        "metric": "frames/sec fragment pass (MeshRasterizer -> Fragments, K=1), 512x512, ~6k-face mesh, batch=64",
        "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "launch": "eager", "data": "synthetic camera poses on the reference mesh",
        "config": {"workload": f"{args.mesh} (F={Fn}), {H}x{W}, {nv} views/GPU, projection + rasterization to "
                               "PyTorch3D Fragments (pix_to_face int64, zbuf, bary_coords, dists)",
                   "mesh": args.mesh, "H": H, "W": W, "views_per_gpu": nv, "parallelism": f"view-sharded x{world}"},
        "fragment_roofline": fp, "work": {"covered": covered}, "kernels": kernels,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_soft(args, dev, world, rank, embed=False):
    """Soft rasterization: the silhouette renderer of deform_mesh_with_color.py:
    153-165 — MeshRenderer(MeshRasterizer(faces_per_pixel=50, blur_radius=ln(1/1e-4 - 1)·1e-4,
    perspective_correct=False), SoftSilhouetteShader) on the normalised cow (:106-111), PerspectiveCameras
    (focal 1, NDC) at look_at_view_transform(2.7, elev, azim) (:118-127), 128x128 (--size), fwd + bwd of a
    silhouette loss to the vertex positions. Not the headline metric: a measured point for the K-deep path."""
    from torch_renderer_amd import _lib
    from torch_renderer_amd import distributed as D
    from torch_renderer_amd.assets import load_asset
    from torch_renderer_amd.cameras import PerspectiveCameras
    from torch_renderer_amd.mesh_renderer import (BlendParams, MeshRasterizer, MeshRenderer, RasterizationSettings,
                                                  SoftSilhouetteShader)
    from torch_renderer_amd.structures import Meshes
    from torch_renderer_amd.transforms import look_at_view_transform

    H = W = args.size
    K = 50
    m = load_asset(args.mesh, device=dev, textures=False)
    v0 = m.shared_verts().detach()
    c = v0.mean(0)
    sc = (v0 - c).abs().max()
    verts = ((v0 - c) / sc).clone().requires_grad_(True)
    faces = m.shared_faces()
    nv = args.views
    n_total = nv * world
    elev = torch.linspace(0, 360, n_total)[rank * nv:(rank + 1) * nv]
    azim = torch.linspace(-180, 180, n_total)[rank * nv:(rank + 1) * nv]
    R, T = look_at_view_transform(dist=2.7, elev=elev, azim=azim)
    R, T = R.to(dev).contiguous(), T.to(dev).contiguous()
    cams = PerspectiveCameras(device=dev, R=R, T=T)
    sigma = 1e-4
    rs = RasterizationSettings(image_size=H, blur_radius=math.log(1.0 / 1e-4 - 1.0) * sigma, faces_per_pixel=K,
                               perspective_correct=False)
    renderer = MeshRenderer(rasterizer=MeshRasterizer(cameras=cams, raster_settings=rs),
                            shader=SoftSilhouetteShader(blend_params=BlendParams(sigma=sigma)))
    gen = torch.Generator().manual_seed(1 + rank)
    target = (torch.rand(nv, H, W, generator=gen) > 0.5).float().to(dev)

    def step():
        verts.grad = None
        img = renderer(Meshes([verts], [faces]).extend(nv), cameras=cams, R=R, T=T)
        ((img[..., 3] - target) ** 2).mean().backward()
        if world > 1:
            D.allreduce_grads([verts])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = e.item()
    kt = _kernel_times(step, min(args.steps, 10))
    if rank != 0 and not embed:
        dist.destroy_process_group()
        return
    value = nv * world * args.steps / elapsed
    kernels = {k: {"launches": v[0], "avg_us": round(v[1] / max(v[0], 1) * 1e3, 2)} for k, v in kt.items()}
    # the forward fragment pass's API-minimum bytes (SURVEY §8d at K = 50: 28 B per fragment slot + 36 B
    # per face) against its kernels' summed time; the whole step's kernels beside it
    Fn = faces.shape[0]
    per_frame = 28 * K * H * W + 36 * Fn
    frag_k = [k for k in ("k_bin_rect", "k_bin_view", "k_fill<0>", "k_raster_k") if k in kt]
    us = sum(kt[k][1] / kt[k][0] * 1e3 for k in frag_k)
    ach = per_frame * nv / max(us, 1e-9) * 1e-3
    roof = {"bound": "hbm", "kernel": "fragment kernels (sum): " + ", ".join(frag_k), "bytes_per_frame": per_frame,
            "us_per_step": round(us, 2), "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4),
            "step_kernels_us": round(sum(v[1] / max(v[0], 1) * 1e3 for v in kt.values()), 2)}
    if embed:
        return _embedded(value, elapsed, args, kt, min(args.steps, 10), roof,
                         f"{args.mesh} (F={Fn}) normalised, {H}x{W}, {nv} views/GPU, K={K}, soft silhouette fwd+bwd "
                         "(deform_mesh_with_color.py:153-165)")
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = soft_cpu_baseline(verts, faces, R, T, H, W, K, rs.blur_radius, sigma, target,
                                n_views=min(args.cpu_views, nv))
    line = {
        "metric": f"frames/sec fwd+bwd, soft silhouette K={K}, {H}x{W} (deform_mesh_with_color.py)",
        "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "launch": "eager", "data": "synthetic views of the reference mesh",
        "config": {"workload": f"{args.mesh} (F={faces.shape[0]}) normalised, {H}x{W}, {nv} views/GPU, K={K}, "
                               "blur=ln(1/1e-4-1)*1e-4, perspective_correct=False, SoftSilhouetteShader, "
                               "L2 silhouette loss -> vertex grads",
                   "mesh": args.mesh, "H": H, "W": W, "views_per_gpu": nv, "K": K, "parallelism": f"view-sharded x{world}"},
        "roofline": roof, "cpu_baseline": cpu, "kernels": kernels,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _time_steps(step, args, dev, world):
    """warmup, then K timed steps between barrier + synchronize on both sides; max over ranks (s)."""
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = e.item()
    return elapsed


def _embedded(value, elapsed, args, kt, kt_steps, roof, workload):
    """The compact object a secondary workload contributes to the default bench line: whole-job
    frames/s and ms per step over its own timed steps, the library kernels' device time per step (HIP
    events around every launch of kt_steps eager steps; the caller's torch kernels are not in it)."""
    dev_us = sum(v[1] for v in kt.values()) / max(kt_steps, 1) * 1e3
    return {"frames_per_s": round(value, 1), "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "steps": args.steps, "warmup": args.warmup, "library_kernel_us_per_step": round(dev_us, 1),
            "roofline": roof, "workload": workload,
            "kernels_us": {k: round(v[1] / max(v[0], 1) * 1e3, 2) for k, v in kt.items()}}


def secondary_steps(args, dev, world, rank):
    """C3 (pose), C5 and the K = 50 soft silhouette, each at its own workload, timed in the default run
    so that the driver's record carries them (bench.py --mode pose / c5 / soft print their full lines)."""
    out = {}
    plans = (("pose_step", bench_pose, dict(size=512, views=64, steps=30, warmup=10)),
             ("c5_step", bench_c5, dict(size=1024, views=5, steps=60, warmup=10)),
             ("soft_step", bench_soft, dict(size=128, views=64, steps=10, warmup=3, mesh="cow")))
    import gc

    for name, fn, over in plans:
        torch.cuda.empty_cache()  # (the headline's graph pool and fragment buffers are gone: start each clean)
        gc.collect()  # the previous workload's garbage collected here, not by a gen-2 pass inside this one's timed
        # steps (r6n_c5_embed_probe.txt: one such pass in C5's window after C3 cost 8 %)
        sub = argparse.Namespace(**{**vars(args), **over, "no_cpu_baseline": True})
        try:
            out[name] = fn(sub, dev, world, rank, embed=True)
        except Exception as e:  # a secondary workload never sinks the headline line; the error is reported
            out[name] = {"error": f"{type(e).__name__}: {e}"}
        torch.cuda.synchronize()
    return out


def _kernel_times(step, n):
    from torch_renderer_amd import _lib

    torch.cuda.synchronize()
    _lib.timing_enable(True)
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    kt = _lib.timing_read()
    _lib.timing_enable(False)
    return kt


def bench_gather(args, dev, world, rank):
    """C4 (batch_rendering_test.py:263-280, 320-328): the depth of a batch of --views views IN TOTAL
    (dolphin at 1024x1024 for C4: --mesh dolphin --size 1024), rendered view-sharded across the ranks
    (DepthRender's fused forward: relu(zbuf), background 0, as render_depth's `-1 -> 0`), then the
    slices gathered to rank 0 over RCCL point-to-point (distributed.gather_to_root) inside the timed
    step (the reference copies the batch to the host at :277). Strong scaling: the batch is fixed.
    After timing, rank 0 renders the whole batch alone and checks the gathered depth bitwise."""
    from torch_renderer_amd import distributed as D
    from torch_renderer_amd.assets import load_asset
    from torch_renderer_amd.torch_renderer import DepthRender

    H = W = args.size
    meshes = load_asset(args.mesh, device=dev, textures=False)
    verts0 = meshes.shared_verts().detach().cpu()
    Fn = meshes.shared_faces().shape[0]
    n_total = args.views
    R_all, t_all, K = canonical_views(verts0, n_total, H, W, dist_m=view_distance(args.mesh, verts0))
    R_cv, t_cv = D.shard_views(R_all, t_all, rank=rank, world_size=world)
    R_cv, t_cv = R_cv.to(dev).contiguous(), t_cv.to(dev).contiguous()
    nv = R_cv.shape[0]
    bmesh = meshes.extend(max(nv, 1))
    renderer = DepthRender(K.to(dev), (H, W), device=dev)
    g_events = []

    def render():
        with torch.no_grad():
            return renderer.render(bmesh, R_cv, t_cv)

    def step(timed=False):
        depth = render()
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        out = D.gather_to_root(depth, n_total)
        if timed:
            e1.record()
            g_events.append((e0, e1))
        return out

    elapsed = _time_steps(lambda: step(True), args, dev, world)
    g_events[:] = g_events[args.warmup:]
    gather_us = sum(a.elapsed_time(b) for a, b in g_events) / max(len(g_events), 1) * 1e3
    if world > 1:
        t = torch.tensor([gather_us], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        gather_us = t.item()
    kt = _kernel_times(render, min(args.steps, 10))
    gathered = step()
    equal = None
    if rank == 0:
        full = DepthRender(K.to(dev), (H, W), device=dev)
        with torch.no_grad():
            ref = full.render(meshes.extend(n_total), R_all.to(dev).contiguous(), t_all.to(dev).contiguous())
        equal = bool(torch.equal(gathered, ref))
    if world > 1:
        dist.barrier()
    if rank != 0:
        dist.destroy_process_group()
        return
    value = n_total * args.steps / elapsed
    kernels = {k: {"launches": v[0], "avg_us": round(v[1] / max(v[0], 1) * 1e3, 2)} for k, v in kt.items()}
    per_frame = 4 * H * W + 36 * Fn  # depth out + face geometry (the fused depth-only forward)
    us = sum(v[1] / max(v[0], 1) * 1e3 for v in kt.values())
    line = {
        "metric": f"frames/sec C4 depth render + RCCL gather to rank 0, {args.mesh} {H}x{W}, {n_total} views total",
        "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32", "launch": "eager", "data": "synthetic camera poses on the reference mesh",
        "config": {"workload": f"{args.mesh} (F={Fn}), {H}x{W}, {n_total} views in total split over {world} rank(s), "
                               "DepthRender forward (relu(zbuf)), depth slices gathered to rank 0",
                   "mesh": args.mesh, "H": H, "W": W, "global_views": n_total, "parallelism": f"view-sharded x{world}"},
        "gather_us": round(gather_us, 2), "gather_bytes": 4 * H * W * n_total,
        "gather_equals_single_gpu_render": equal,
        "roofline": {"bound": "hbm", "kernel": "forward kernels (sum)", "bytes_per_frame": per_frame,
                     "us_per_step": round(us, 2),
                     "achieved": round(per_frame * nv / max(us, 1e-9) * 1e-3, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(per_frame * nv / max(us, 1e-9) * 1e-3 / HBM_PEAK_GBS, 4)},
        "kernels": kernels,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _host_profile(step, dev, n=20):
    """Experiments only (MR_BENCH_CPROFILE=<file>): cProfile of n eager steps — where an eager caller
    loop spends its host time (Python glue, launches) — written as text to <file>."""
    path = os.environ.get("MR_BENCH_CPROFILE")
    if not path:
        return
    import cProfile
    import io
    import pstats

    # autograd runs the Python backward functions on its device thread, which cProfile does not see: time
    # every autograd.Function's forward / backward of the package with wrappers instead
    from torch_renderer_amd import kernels as Kn, losses as Ls, transforms as Tf
    acc = {}
    patched = []
    for mod in (Kn, Ls, Tf):
        for name in dir(mod):
            cls = getattr(mod, name)
            if isinstance(cls, type) and issubclass(cls, torch.autograd.Function) and cls is not torch.autograd.Function:
                for meth in ("forward", "backward"):
                    if meth not in cls.__dict__:
                        continue
                    orig = cls.__dict__[meth]
                    fn = orig.__func__ if isinstance(orig, staticmethod) else orig
                    key = f"{name}.{meth}"

                    def wrap(*a, _fn=fn, _k=key):
                        t = time.perf_counter()
                        try:
                            return _fn(*a)
                        finally:
                            e = acc.setdefault(_k, [0, 0.0])
                            e[0] += 1
                            e[1] += time.perf_counter() - t
                    setattr(cls, meth, staticmethod(wrap))
                    patched.append((cls, meth, orig))
    pr = cProfile.Profile()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(n):
        step()
    pr.disable()
    torch.cuda.synchronize(dev)
    for cls, meth, orig in patched:
        setattr(cls, meth, orig)
    s = io.StringIO()
    s.write(f"{n} steps, {(time.perf_counter() - t0) / n * 1e3:.3f} ms/step under the profiler\n")
    s.write("autograd.Function host time per step (forward: main thread, backward: autograd's device thread):\n")
    for k, (c, t) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
        s.write(f"  {k:40s} {c / n:5.1f} calls/step  {t / n * 1e6:8.1f} us/step  {t / max(c, 1) * 1e6:7.1f} us/call\n")
    ps = pstats.Stats(pr, stream=s)
    ps.sort_stats("tottime").print_stats(45)
    ps.sort_stats("cumulative").print_stats(45)
    with open(path, "w") as f:
        f.write(s.getvalue())


def _pose_refs(meshes, renderers, R, T):
    """camera_pose_optimizer.py:173-191: the reference silhouette mask, depth (-1 -> 0) and colour."""
    rast, sil_r, phong = renderers
    with torch.no_grad():
        depth = rast(meshes_world=meshes, R=R, T=T).zbuf[..., 0]
        rgb = phong(meshes_world=meshes, R=R, T=T)[..., :3]
    depth = torch.where(depth == -1.0, torch.zeros_like(depth), depth)
    mask = depth != 0.0
    rgb = torch.where(mask[..., None], rgb, torch.zeros_like(rgb))
    return mask, depth, rgb


def pose_cpu_baseline(verts, faces, d, q0, refs, H, W, n_views=2, reps=2):
    """The same step on the oracle (C naive rasterizer + torch-CPU shading, FoV camera, near-plane
    clipping, calc_loss with torch, backward, Adam) for `n_views` poses."""
    import numpy as np

    from oracle import oracle as O
    from torch_renderer_amd.transforms import quaternion_to_matrix

    img = torch.from_numpy(d["texture_u8"].astype(np.float32) / 255.0)
    tex = ("uv", torch.from_numpy(d["verts_uvs"]).float(), torch.from_numpy(d["faces_uvs"]).long(), img)
    t = 1.0 / math.tan(math.radians(30.0))
    intr = torch.tensor([[t, 0.0, t, 0.0]]).expand(n_views, 4).contiguous()
    mask, dref, rref = (x[:n_views].cpu() for x in refs)
    q = torch.nn.Parameter(q0[:n_views].cpu().clone())
    opt = torch.optim.Adam([q], lr=1e-3)
    F_ = torch.nn.functional

    def one():
        opt.zero_grad()
        ref = O.render_ref(verts, faces, quaternion_to_matrix(q[:, 3:]), q[:, :3], intr, H, W, texture=tex,
                           bg=(0.0, 0.0, 0.0), z_clip=0.5)
        depth = torch.relu(ref["zbuf"][..., 0])
        loss = (F_.l1_loss(ref["sil"], mask.float()) + F_.huber_loss(depth[mask], dref[mask], delta=0.05)
                + 0.01 * F_.mse_loss(ref["rgba"][..., :3], rref))
        loss.backward()
        opt.step()

    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or cores, cores)
    O.set_threads(threads)
    one()
    t0 = time.perf_counter()
    for _ in range(reps):
        one()
    sec = (time.perf_counter() - t0) / reps
    return {"value": n_views / sec, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n_views} poses of the same step (cow {H}x{W}, FoV camera, clipping, calc_loss, backward, "
                      f"Adam), 1 warm-up + {reps} timed steps, {sec:.2f} s/step, C naive rasterizer (OpenMP "
                      f"{threads} threads) + torch-CPU shading/autograd ({torch.get_num_threads()} threads)"}


def bench_pose(args, dev, world, rank, embed=False):
    """C3 as the caller runs it (camera_pose_optimizer.py:237-305), batched: --views independent pose
    problems per GPU (the cow from look_at_view_transform(0.7, elev, azim) + N(0, 0.03) noise on the
    7-vector pose), each step the caller's three calls — rasterizer(meshes_world=, R=, T=) for the
    depth, the silhouette MeshRenderer, the Phong MeshRenderer — FoVPerspectiveCameras (znear 1: the
    near plane clips at 0.5), calc_loss (fused pose_loss), backward through quaternion_to_matrix and
    one Adam step. Eager launches, as the caller's Python loop."""
    from torch_renderer_amd import distributed as D
    from torch_renderer_amd.assets import load_asset, load_asset_arrays
    from torch_renderer_amd.cameras import FoVPerspectiveCameras
    from torch_renderer_amd.losses import pose_loss
    from torch_renderer_amd.mesh_renderer import (BlendParams, MeshRasterizer, MeshRenderer, PointLights,
                                                  RasterizationSettings, SoftPhongShader, SoftSilhouetteShader)
    from torch_renderer_amd.transforms import look_at_view_transform, matrix_to_quaternion, quaternion_to_matrix

    H = W = args.size
    nv = args.views
    n_total = nv * world
    d = load_asset_arrays("cow")
    base = load_asset("cow", device=dev)
    meshes = base.extend(nv)
    cams = FoVPerspectiveCameras(device=dev)
    blend = BlendParams(sigma=1e-4, gamma=1e-4, background_color=(0, 0, 0))
    rs = RasterizationSettings(image_size=H, blur_radius=0.0, faces_per_pixel=1)
    sil_r = MeshRenderer(MeshRasterizer(cameras=cams, raster_settings=rs), SoftSilhouetteShader(blend_params=blend))
    rast = MeshRasterizer(cameras=cams, raster_settings=rs)
    lights = PointLights(device=dev, location=[[0.0, 0.0, -3.0]])
    phong = MeshRenderer(MeshRasterizer(cameras=cams, raster_settings=rs),
                         SoftPhongShader(device=dev, cameras=cams, lights=lights, blend_params=blend))
    elev = torch.linspace(10.0, 50.0, n_total)[rank * nv:(rank + 1) * nv]
    azim = torch.linspace(0.0, 360.0, n_total + 1)[:-1][rank * nv:(rank + 1) * nv]
    R, T = look_at_view_transform(0.7, elev, azim, device=dev)
    refs = _pose_refs(meshes, (rast, sil_r, phong), R, T)
    mask, depth_ref, rgb_ref = refs
    g = torch.Generator().manual_seed(rank)
    q_ref = torch.cat((T, matrix_to_quaternion(R)), -1)
    q0 = q_ref + (torch.randn(q_ref.shape, generator=g) * 0.03).to(dev)
    q = torch.nn.Parameter(q0.clone())
    opt = torch.optim.Adam([q], lr=1e-3)

    def step():
        opt.zero_grad()
        Rq = quaternion_to_matrix(q[:, 3:])
        Tq = q[:, :3]
        frags = rast(meshes_world=meshes, R=Rq, T=Tq)
        depth = torch.relu(frags.zbuf[..., 0])
        sil = sil_r(meshes, R=Rq, T=Tq)[..., 3]
        color = phong(meshes, R=Rq, T=Tq)[..., :3]
        loss = pose_loss(depth, sil, color, mask, depth_ref, rgb_ref)
        loss.backward()
        opt.step()

    elapsed = _time_steps(step, args, dev, world)
    kt = _kernel_times(step, min(args.steps, 10))
    _host_profile(step, dev)
    # roofline of the step's largest library kernel, calc_loss fused with its gradients (k_pose_loss_fused):
    # per pixel it reads depth 4 + silhouette RGBA 16 + colour RGBA 16 + mask 1 + depth_ref 4 + rgb_ref 12 B
    # and writes the three gradient images 4 + 16 + 16 B (89 B)
    roof = None
    if "k_pose_loss_fused" in kt:
        n_, ms_ = kt["k_pose_loss_fused"]
        b = 89 * nv * H * W
        us_ = ms_ / n_ * 1e3
        roof = {"bound": "hbm", "kernel": "k_pose_loss_fused", "avg_launch_us": round(us_, 2),
                "algorithmic_bytes_per_launch": b, "achieved": round(b / (us_ * 1e-6) / 1e9, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(b / (us_ * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": None}
    if embed:
        return _embedded(n_total * args.steps / elapsed, elapsed, args, kt, min(args.steps, 10), roof,
                         f"cow (F={base.shared_faces().shape[0]}), {H}x{W}, {nv} pose problems/GPU, "
                         "camera_pose_optimizer.py:237-305 step (3 renders, calc_loss, backward, Adam)")
    if rank != 0:
        dist.destroy_process_group()
        return
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        verts0 = base.shared_verts().detach().cpu()
        cpu = pose_cpu_baseline(verts0, base.shared_faces().cpu(), d, q0.detach(), refs, H, W,
                                n_views=min(args.cpu_views, nv))
    value = n_total * args.steps / elapsed
    kernels = {k: {"launches": v[0], "avg_us": round(v[1] / max(v[0], 1) * 1e3, 2)} for k, v in kt.items()}
    line = {
        "metric": f"frames/sec C3 pose-optimiser step (3 renders + calc_loss + backward + Adam), cow {H}x{W}",
        "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "launch": "eager", "data": "synthetic poses around the reference mesh",
        "config": {"workload": f"cow (F={base.shared_faces().shape[0]}), {H}x{W}, {nv} pose problems/GPU, "
                               "camera_pose_optimizer.py step: rasterizer + silhouette + Phong renders (FoV camera, "
                               "near-plane clip), calc_loss, backward, Adam",
                   "mesh": "cow", "H": H, "W": W, "views_per_gpu": nv, "parallelism": f"view-sharded x{world}"},
        "roofline": roof, "cpu_baseline": cpu, "kernels": kernels,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_c5(args, dev, world, rank, embed=False):
    """C5 (BASELINE.json configs[4]; mesh_deformer.py:130-222 color_train) as the caller runs it: the
    F=81,920 subdivided sphere (data/sphere.obj subdivided twice), 1024x1024 (--size), PerspectiveCameras
    (NDC, focal 1) at look_at_view_transform(2, elev, azim) over 10 target views, AmbientLights,
    perspective_correct=False, TexturesVertex(hardtanh(verts_rgb)) with grad; one step = --views
    (default 5: num_views_per_iteration) single-view renderer(mesh, cameras=target_cameras[j], lights=)
    calls (:196-204), the MSE losses + the colour penalty (:207), backward to the per-vertex colours AND
    positions (the mesh is src_mesh.offset_verts(deform_verts)), one SGD(lr=1, momentum=0.9) step."""
    from torch_renderer_amd import _lib
    from torch_renderer_amd.cameras import PerspectiveCameras
    from torch_renderer_amd.kernels import render_stats
    from torch_renderer_amd.mesh_renderer import (AmbientLights, MeshRasterizer, MeshRenderer, RasterizationSettings,
                                                  SoftPhongShader)
    from torch_renderer_amd.structures import Meshes, TexturesVertex
    from torch_renderer_amd.transforms import look_at_view_transform
    from torch_renderer_amd.utils import subdivided_sphere

    H = W = args.size if args.size != 512 else 1024
    nper = args.views if args.views != 64 else 5
    n_targets = 10
    sph = subdivided_sphere(2)
    verts0, faces = sph.verts_list()[0].to(dev), sph.faces_list()[0].to(dev)
    Fn, Vn = faces.shape[0], verts0.shape[0]
    elev = torch.linspace(0, 360, n_targets)
    azim = torch.linspace(-180, 180, n_targets)
    R, T = look_at_view_transform(dist=2.0, elev=elev, azim=azim)
    R, T = R.to(dev), T.to(dev)
    lights = AmbientLights(device=dev)
    rs = RasterizationSettings(image_size=H, blur_radius=0.0, faces_per_pixel=1, perspective_correct=False)
    cams = PerspectiveCameras(device=dev, R=R, T=T)
    renderer = MeshRenderer(MeshRasterizer(cameras=cams, raster_settings=rs),
                            SoftPhongShader(device=dev, cameras=cams, lights=lights))
    target_cameras = [PerspectiveCameras(device=dev, R=R[None, i], T=T[None, i]) for i in range(n_targets)]
    gen = torch.Generator().manual_seed(7 + rank)
    with torch.no_grad():  # targets: the sphere coloured by a smooth function of position
        tcol = (0.5 + 0.5 * torch.sin(3.0 * verts0.cpu() + torch.rand(3, generator=gen))).to(dev)
        tmesh = Meshes([verts0], [faces], TexturesVertex([tcol])).extend(n_targets)
        target_rgb = renderer(tmesh, cameras=cams, lights=lights)[..., :3]
    deform = torch.zeros_like(verts0, requires_grad=True)  # geometry_train's offsets (grads reach them)
    verts_rgb = torch.full((1, Vn, 3), 0.5, device=dev, requires_grad=True)
    opt = torch.optim.SGD([verts_rgb], lr=1.0, momentum=0.9)
    perms = [torch.randperm(n_targets, generator=gen)[:nper].tolist() for _ in range(64)]
    it = [0]

    def step():
        opt.zero_grad()
        deform.grad = None
        norm = torch.nn.functional.hardtanh(verts_rgb, min_val=0.0, max_val=1.0)
        mesh = Meshes([verts0 + deform], [faces], TexturesVertex(verts_features=norm))
        loss = 0
        for j in perms[it[0] % len(perms)]:
            img = renderer(mesh, cameras=target_cameras[j], lights=lights)
            loss = loss + ((img[..., :3].squeeze() - target_rgb[j]) ** 2).mean()
        loss = loss + ((norm - verts_rgb) ** 2).sum()
        loss.backward()
        opt.step()
        it[0] += 1

    windows = None
    if embed:
        # the default line's C5: the eager caller loop is host-bound on a loaded box, and one host hiccup inside a
        # single window moved the recorded value by up to 40 % between boxes (r6n-r6r): three windows of
        # args.steps / 3 steps after the warm-up, the median one reported (all three listed in the line)
        sub = argparse.Namespace(**{**vars(args), "steps": max(1, args.steps // 3)})
        again = argparse.Namespace(**{**vars(sub), "warmup": 0})
        ws = [_time_steps(step, sub if k == 0 else again, dev, world) for k in range(3)]
        windows = [round(w / sub.steps * 1e3, 4) for w in ws]
        elapsed = sorted(ws)[1] * args.steps / sub.steps
    else:
        elapsed = _time_steps(step, args, dev, world)
    kt = _kernel_times(step, min(args.steps, 10))
    _host_profile(step, dev)
    # host cost of one single-view renderer(...) call as the caller makes it (:197), no synchronisation inside
    # the timed calls (the device queue absorbs the launches): median of 20
    hs = []
    with torch.no_grad():
        mesh_h = Meshes([verts0], [faces], TexturesVertex(verts_features=verts_rgb.detach()))
        for i in range(25):
            h0 = time.perf_counter()
            img = renderer(mesh_h, cameras=target_cameras[i % n_targets], lights=lights)
            hs.append(time.perf_counter() - h0)
            del img
    torch.cuda.synchronize()
    host_us = sorted(hs[5:])[len(hs[5:]) // 2] * 1e6
    # work counters of one view's forward (render_stats reads the live workspace)
    # (colours requiring grad: the autograd node holds the workspace, which an inference render would free)
    norm = torch.nn.functional.hardtanh(verts_rgb, 0.0, 1.0).detach().requires_grad_(True)
    keep = renderer(Meshes([verts0], [faces], TexturesVertex(verts_features=norm)), cameras=target_cameras[0],
                    lights=lights)
    wstats = render_stats()
    del keep
    if rank != 0 and not embed:
        dist.destroy_process_group()
        return
    value = nper * world * args.steps / elapsed
    kernels = {k: {"launches": v[0], "avg_us": round(v[1] / max(v[0], 1) * 1e3, 2)} for k, v in kt.items()}
    # roofline of the render's forward (per call = one view): the kernels that move the API's bytes (the
    # RGBA image, 16 B per pixel, and the projected records, 100 B per face) summed — with one view the
    # longest single kernel is the binning, whose algorithmic bytes (4 B per face) say nothing of the path
    fk = [k for k in ("k_bin_rect", "k_band_bucket", "k_bin_view", "k_tile_raster", "k_shade<1>") if k in kt]
    f_us = sum(kt[k][1] / kt[k][0] * 1e3 for k in fk)
    b = 16 * H * W + 100 * Fn
    roof = None
    if f_us > 0:
        roof = {"bound": "hbm", "kernel": "forward kernels (sum): " + ", ".join(fk), "us_per_launch": round(f_us, 2),
                "algorithmic_bytes_per_launch": b, "achieved": round(b / (f_us * 1e-6) / 1e9, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(b / (f_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": None}
    if embed:
        e = _embedded(value, elapsed, args, kt, min(args.steps, 10), roof,
                      f"ico-sphere (F={Fn}, V={Vn}), {H}x{W}, {nper} single-view renders per step, "
                      "mesh_deformer.py:196-215 colour step (backward to colours and positions, SGD)")
        e["host_us_per_render_call"] = round(host_us, 1)
        e["windows_ms_per_step"] = windows
        return e
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = c5_cpu_baseline(verts0.cpu(), faces.cpu(), R.cpu(), T.cpu(), H, W)
    line = {
        "metric": f"frames/sec C5 colour-fitting step (mesh_deformer.py color_train), subdivided sphere F={Fn}, {H}x{W}",
        "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "launch": "eager", "data": "synthetic target colours on the subdivided "
                                                                        "reference sphere",
        "config": {"workload": f"ico-sphere (F={Fn}, V={Vn}), {H}x{W}, {nper} single-view renders per step "
                               "(PerspectiveCameras, AmbientLights, TexturesVertex, perspective_correct=False), "
                               "MSE + colour penalty, backward to vertex colours and positions, SGD",
                   "mesh": "subdivided sphere", "H": H, "W": W, "views_per_step": nper,
                   "parallelism": f"replicas x{world}"},
        "roofline": roof, "cpu_baseline": cpu, "work": wstats, "kernels": kernels,
        "host_us_per_render_call": round(host_us, 1),
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def c5_cpu_baseline(verts, faces, R, T, H, W, win=128, reps=1):
    """The reference CPU path (oracle: C naive rasterizer + torch-CPU ambient shading / blend / autograd) on a
    bounded sample: a win x win window of one C5 view, fwd + bwd to colours and positions, scaled to
    frames/s by the window's share of the image (the naive rasterizer's cost is per pixel x face)."""
    from oracle import oracle as O

    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or cores, cores)
    O.set_threads(threads)
    y0, x0 = H // 2 - win // 2, W // 2 - win // 2
    window = (y0, y0 + win, x0, x0 + win)
    intr = torch.tensor([[1.0, 0.0, 1.0, 0.0]])

    def one():
        v = verts.clone().requires_grad_(True)
        vc = torch.full(verts.shape, 0.5).requires_grad_(True)
        ref = O.render_ref(v, faces, R[:1], T[:1], intr, H, W, texture=("vertex", vc),
                           light={"kind": "ambient", "ambient": (1.0, 1.0, 1.0)}, persp=False, window=window)
        ref["rgba"][..., :3].sum().backward()

    t0 = time.perf_counter()
    for _ in range(reps):
        one()
    sec = (time.perf_counter() - t0) / reps
    scale = (H * W) / float(win * win)
    return {"value": 1.0 / (sec * scale), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"a {win}x{win} window of one view (fwd + bwd, {sec:.2f} s), scaled by the image/window pixel "
                      f"ratio {scale:.0f}: C naive rasterizer (OpenMP {threads} threads) + torch-CPU shading/autograd"}


def soft_cpu_baseline(verts, faces, R, T, H, W, K, blur, sigma, target, n_views=2, reps=2):
    """The soft silhouette step on the oracle (C naive K-deep rasterizer, sigmoid_alpha_blend, L2 loss,
    backward) for `n_views` views."""
    from oracle import oracle as O

    intr = torch.tensor([[1.0, 0.0, 1.0, 0.0]]).expand(n_views, 4).contiguous()
    Rc, Tc, tg = R[:n_views].cpu(), T[:n_views].cpu(), target[:n_views].cpu()

    def one():
        v = verts.detach().cpu().clone().requires_grad_(True)
        ref = O.render_ref(v, faces.cpu(), Rc, Tc, intr, H, W, persp=False, K=K, blur=blur, clip=True,
                           sigma_sil=sigma, light={"kind": "ambient", "ambient": (1.0, 1.0, 1.0)})
        ((ref["sil"] - tg) ** 2).mean().backward()

    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or cores, cores)
    O.set_threads(threads)
    one()
    t0 = time.perf_counter()
    for _ in range(reps):
        one()
    sec = (time.perf_counter() - t0) / reps
    return {"value": n_views / sec, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n_views} views of the same workload ({H}x{W}, K={K}, fwd+bwd), 1 warm-up + {reps} timed "
                      f"passes, {sec:.2f} s/pass: C naive K-deep rasterizer (OpenMP {threads} threads) + torch-CPU "
                      f"blend/autograd"}


def _spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N fresh rank processes (one per GPU) with the
    torch.distributed env a launcher would set, before this parent touches the GPU (it never
    initialises HIP, so no process exec follows GPU init). Rank 0 prints the JSON line."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # poll every rank: if one dies (e.g. a failed RCCL init) the others would wait in a collective
    # forever, so the rest are terminated and the parent exits with the failure
    rc = 0
    while procs:
        time.sleep(0.2)
        for p in list(procs):
            r = p.poll()
            if r is None:
                continue
            procs.remove(p)
            if r != 0:
                rc = r
                for q in procs:
                    q.terminate()
                for q in procs:
                    try:
                        q.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        q.kill()
                return rc
    return rc


if __name__ == "__main__":
    _a = argparse.ArgumentParser(add_help=False)
    _a.add_argument("--gpus", type=int, default=1)
    _known, _ = _a.parse_known_args()
    if _known.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_ranks(_known.gpus))
    main()
