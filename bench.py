"""Benchmark: rendered Mpix/s, fwd+bwd, 1M Gaussians at 1920x1080 (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (driver, N > 1)

One step on each rank = one training step of one view: zero_grad ->
GaussianRenderer.render -> backward of a fixed random cotangent on
(image, alpha, depth) -> [N>1] RCCL all-reduce (mean) of the Gaussian
gradients -> Adam step.  Adam reads the parameters and writes the updated
ones to shadow tensors (gs_adam_tensor.param_out: the in-place step's reads
and writes, with the result kept out of the rendered model), so that every
timed frame renders the same scene.  Rank r renders view r of the same replicated 1M
Gaussian model (weak scaling: one 1080p view per GPU per step).  Inputs are
resident in HBM before the timed region.  Before the W warm-up steps,
--spinup-steps (default 50 at C3, more for the small presets; reported in the line) untimed steps bring the GPU
to its steady clock.  `value` = all ranks' pixels /
max-over-ranks step time.

Also reported: the roofline of the dominant kernel (HIP events on the
kernels' own stream, averaged over the timed steps), priced by SURVEY.md
8(d)'s algorithmic byte and flop models from the frame's work counters
(R, E, C, M), against the 8 TB/s spec and a copy kernel measured on the box;
and a CPU baseline (the oracle, a C restatement of the reference path, on
the host cores and on one core, rank 0, N=1 only) next to the literal
reference's cost model.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "rendered Mpix/s fwd+bwd @1080p, 1M Gaussians; PSNR vs ref; 1/2/4/8-GPU scaling"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_PEAK_TFLOPS = 157.3     # FP32 vector, spec (FMA = 2)
# literal reference cost model (measured on the survey
# host): forward per evaluated pair (sparse / contributing), binning per
# Gaussian, projection + cull + sort at 1M; backward per contributing pair
# 155 ms at 256^2, O(H W) per pair (autograd CopySlices)
REF_FWD_S_PER_PAIR, REF_FWD_S_PER_CONTRIB = 85e-6, 177e-6
REF_BIN_S_PER_GAUSSIAN, REF_PROJ_SORT_S_PER_1M = 8.7e-6, 0.40
REF_BWD_S_PER_CONTRIB_PX = 155e-3 / (256 * 256)
# workload presets (Gaussians, width, height): BASELINE.json configs[0..2] on the
# SURVEY 8(d) synthetic distribution, and a 4K frame; C3 is the metric's config
CONFIGS = {"C1": (5_000, 256, 256), "C2": (100_000, 800, 800), "C3": (1_000_000, 1920, 1080),
           "4K": (4_000_000, 3840, 2160)}
# Untimed spin-up steps per preset, for the GPU clock's ramp over the first
# ~60 ms of load (profiles/r02/warmup.log): 50 C3 steps are ~60 ms, 50 C1
# steps only ~15 ms.  (C1 is host-bound; its step time varies 0.21-0.39 ms
# between runs on the same box whatever the spin-up, profiles/r05/host/.)
SPINUP_STEPS = {"C1": 1000, "C2": 300, "C3": 50, "4K": 20}
TIMED_STEPS = {"C1": 500, "C2": 200, "C3": 30, "4K": 30}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: 30 at C3; more for the small presets, whose ~0.3 ms steps "
                         "would otherwise time a ~10 ms window that one host preemption skews)")
    ap.add_argument("--warmup", type=int, default=10)  # (clocks and allocator settle: a 3-step warmup once timed 20 % slow)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="C3",
                    help="workload preset (BASELINE.json configs; C3 = the metric's, the default)")
    ap.add_argument("--gaussians", type=int, default=None, help="override the preset's Gaussian count")
    ap.add_argument("--width", type=int, default=None, help="override the preset's image width")
    ap.add_argument("--height", type=int, default=None, help="override the preset's image height")
    ap.add_argument("--no-optimizer", action="store_true", help="time render fwd+bwd only")
    ap.add_argument("--diag-steps", type=int, default=5, help="untimed steps for the per-stage breakdown")
    # MI355X clocks ramp over the first ~60 ms of load: with 5 warm-up steps the
    # timed steps ran 1.25 ms, with 50 or 200 1.19 (same box, profiles/r02/warmup.log).
    # A fixed count (not a time) so that every rank runs the same collectives.
    ap.add_argument("--view", type=int, default=None,
                    help="render rank R's view (diagnostics; default: this rank's own)")
    ap.add_argument("--spinup-steps", type=int, default=None,
                    help="untimed steps before the --warmup steps, for the GPU (and host CPU) clock ramp; "
                         "default ~60 ms or more of steps: 50 at C3, more for the smaller presets")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="an extra oracle thread count for the CPU sweep (16..256 and the CPU limit always run)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI) for the driver; gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--force-dist", action="store_true",
                    help="init the process group and all-reduce even at world size 1 (rehearses the RCCL path)")
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="auto",
                    help="replay the step as one HIP graph over a device-resident frame (graph_step.GraphedStep; "
                         "auto: at world size 1 with the optimizer) or run it eagerly through autograd")
    ap.add_argument("--fused-adam", choices=("auto", "on", "off"), default="auto",
                    help="replayed steps: the optimizer in the backward (gs_project_backward_adam: the "
                         "projection backward applies the Adam update, no gradient tensor materialised; auto: on "
                         "with --graph at world size 1) or the separate gs_adam_step launch")
    a = ap.parse_args()
    n0, w0, h0 = CONFIGS[a.config]
    a.gaussians = n0 if a.gaussians is None else a.gaussians
    a.width = w0 if a.width is None else a.width
    a.height = h0 if a.height is None else a.height
    if a.spinup_steps is None:
        a.spinup_steps = SPINUP_STEPS.get(a.config, 50)
    if a.steps is None:
        a.steps = TIMED_STEPS.get(a.config, 30)
    return a


def workload_name(n: int, w: int, h: int) -> str:
    """The BASELINE.json config these sizes are (C1 / C2 / C3 / 4K), or
    "custom": the bench line names its own workload, whatever flags set it."""
    for k, v in CONFIGS.items():
        if v == (n, w, h):
            return k
    return "custom"


def view_matrix(rank: int) -> torch.Tensor:
    """Rank r's camera: a small yaw/translation of the identity view (all
    views look at the same synthetic volume)."""
    if rank == 0:
        return torch.eye(4)
    ang = 0.02 * rank * (1 if rank % 2 else -1)
    c, s = math.cos(ang), math.sin(ang)
    wv = torch.eye(4)
    wv[:3, :3] = torch.tensor([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])
    wv[:3, 3] = torch.tensor([0.01 * rank, 0.0, 0.0])
    return wv


class BenchCamera:
    def __init__(self, w, h, fovx, fovy, wv):
        self._width, self._height, self._FoVx, self._FoVy, self._wv = w, h, fovx, fovy, wv

    def world_view_transform(self):
        return self._wv


def algorithmic_counts(pix_neval, pair_counts, H, W, tiles_x, tiles_y):
    """SURVEY 8(d) work counters of one frame: R (records consumed per tile:
    list prefix up to the deepest pixel's last evaluated entry), E (evaluated
    pairs) and C (contributing pairs) from the forward's per-pixel
    measurement counters."""
    neval = pix_neval.view(H, W).to(torch.int64)
    E = int(neval.sum())
    pad = torch.zeros(tiles_y * 16, tiles_x * 16, dtype=torch.int64, device=neval.device)
    pad[:H, :W] = neval
    per_tile = pad.view(tiles_y, 16, tiles_x, 16).amax(dim=(1, 3))
    R = int(per_tile.sum())
    C = int(pair_counts.to(torch.int64).sum())
    return R, E, C


def copy_peak_gbs(dev, nbytes=1 << 30, reps=10):
    """HBM bandwidth a plain device copy reaches on this box (read + write
    bytes / time, 1 GiB buffers, HIP events): the achievable peak beside the
    8 TB/s spec (the guide measured ~6.3 TB/s with a float4 copy)."""
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).fill_(1.0)
    dst = torch.empty_like(src)
    dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    e1.synchronize()
    gbs = 2.0 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src, dst
    torch.cuda.empty_cache()
    return gbs


def main():
    a = parse()
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from mini3dgs_amd.rasterizer import StageTimer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))  # % only matters for a 1-GPU gloo rehearsal
    torch.cuda.set_device(dev)
    if world > 1 or a.force_dist:
        import torch.distributed as dist
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(a.dist_backend)

    W, H, n = a.width, a.height, a.gaussians
    scene = pkg.synthetic.make_scene(n, W, H, seed=0)
    model = pkg.synthetic.to_model(scene, pkg.GaussianModel, dev)
    params = model.grad_parameters()
    opt = None if a.no_optimizer else pkg.optim.FusedAdam(
        [{"params": [model._xyz], "lr": 1.6e-4}, {"params": [model._features_dc], "lr": 2.5e-3},
         {"params": [model._opacity], "lr": 0.05}, {"params": [model._scaling], "lr": 5e-3},
         {"params": [model._rotation], "lr": 1e-3}])
    cam = BenchCamera(W, H, scene.fovx, scene.fovy, view_matrix(rank if a.view is None else a.view))
    settings = pkg.RenderSettings(image_height=H, image_width=W, bg_color=torch.zeros(3))
    renderer = pkg.GaussianRenderer()
    g = torch.Generator().manual_seed(1)
    cot = [(torch.rand(s, generator=g) * 2 - 1).to(dev) for s in ((3, H, W), (1, H, W), (1, H, W))]
    # the backward writes the gradients straight into the all-reduce bucket
    reducer = pkg.distributed.GradAllReduce(params, dist).attach(model) if dist is not None else None
    frames = []

    # Every step renders the same scene: Adam writes the updated parameters to
    # shadow tensors instead of the model's (the same bytes read and written
    # as an in-place step; its moments evolve as in training), so the workload
    # does not drift and the frame counters R, E below hold for every timed
    # frame.  (Rounds 1-3 restored the parameters from a snapshot with a
    # multi-tensor copy inside each step instead: 29 us of copying that is not
    # part of a training step.)
    if opt is not None:
        for p in params:
            opt.set_output(p, torch.empty_like(p))

    def eager_step():
        if opt is not None:
            opt.zero_grad(set_to_none=True)
        else:
            for p in params:
                p.grad = None
        out = renderer.render(cam, model, settings)
        torch.autograd.backward([out["image"], out["alpha"], out["depth"]], cot)
        if eager_step.no_collective:  # (collective_share's reference run)
            if opt is not None:
                opt.step()
        elif reducer is not None and opt is not None:
            reducer.reduce_and_step(opt)  # (pipelined per range when the backward handed over ranges)
        elif reducer is not None:
            reducer.all_reduce_mean()
        elif opt is not None:
            opt.step()
        frames.append(out)

    eager_step.no_collective = False
    # The step replayed as one HIP graph: the same kernels
    # on the same buffers, no per-frame host read-back, one launch per step;
    # a frame that fails on the device is skipped by Adam and redone eagerly
    # (gstep.redone).  World size 1: the collective stays eager at N > 1.
    use_graph = a.graph == "on" or (a.graph == "auto" and reducer is None and opt is not None)
    gstep = None
    if use_graph:
        fused = a.fused_adam == "on" or (a.fused_adam == "auto" and world == 1)
        gstep = pkg.GraphedStep(renderer, cam, model, settings, cot, opt, eager_step=eager_step, fused_adam=fused)
        torch.cuda.set_stream(gstep.stream)  # (every step, eager or replayed, on the graph's queue)
        step = gstep.step
    else:
        step = eager_step
    graph_fallback = None
    try:
        for _ in range(a.spinup_steps + a.warmup):
            step()
            frames.clear()
    except RuntimeError as e:
        # --graph auto: a HIP runtime that refuses the capture (or a replay's
        # host check) leaves the eager step, which the line then says; --graph
        # on raises.  (A GPU fault is not recoverable here and fails the run.)
        if gstep is None or a.graph == "on":
            raise
        graph_fallback = f"{type(e).__name__}: {e}"
        print(f"bench: graph replay unavailable ({graph_fallback}); eager steps", file=sys.stderr, flush=True)
        gstep.close()
        gstep = None
        torch.cuda.synchronize()
        torch.cuda.set_stream(torch.cuda.default_stream())
        step = eager_step
        for _ in range(a.spinup_steps + a.warmup):
            step()
            frames.clear()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    # Timed region: HIP events only around the dominant kernel (the blend
    # backward, launched while the forward's blend still runs, so its events
    # cost no GPU idle time); the per-stage breakdown comes from extra
    # diagnostic steps after it, whose events would stall the launch chain.
    StageTimer.enabled, StageTimer.only = True, {"blend_bwd", "project_bwd"}
    StageTimer.reset()
    if gstep is not None:
        gstep.finish()
        gstep.timing, gstep.event_pairs = True, []  # (event record nodes re-pointed per replay)
        redone0 = sum(k for _, k in gstep.redone)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
        frames = frames[-1:]
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    if gstep is not None:
        gstep.finish()  # (checks the last replay; a redo would show in graph_info below)
        gstep.timing = False
        bwd_live = gstep.blend_backward_ms()
        graph_info = {"replayed": True, "nodes": gstep.graph.num_nodes if gstep.graph else None,
                      "steps_redone_in_timed_region": sum(k for _, k in gstep.redone) - redone0,
                      "redone": gstep.redone, "disabled": gstep.disabled,
                      "capacity": gstep._cap, "depth_window_bits": (gstep.window_used or (0, 32))[1],
                      "optimizer": ("FusedAdam in the projection backward (gs_project_backward_adam): the same "
                                    "update, no gradient tensor materialised, no separate Adam launch"
                                    if gstep.fused_adam else "FusedAdam, one gs_adam_step launch"),
                      "note": "render fwd + bwd + FusedAdam captured once (hipStreamBeginCapture) over a "
                              "device-resident frame and replayed with hipGraphLaunch; no host read-back"}
    else:
        bwd_live = StageTimer.durations_ms().get("blend_bwd", [])
        graph_info = {"replayed": False} if graph_fallback is None else {"replayed": False, "fallback": graph_fallback}
    dt = t1 - t0
    if dist is not None:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    StageTimer.only = None
    StageTimer.reset()
    coll = collective_share(a, dist, dev, reducer, model, eager_step, frames, dt) if reducer is not None else None
    # the per-stage breakdown from the stage-by-stage path (the same kernels;
    # the frame entry points would time only the blend backward)
    from mini3dgs_amd import rasterizer as _RZ
    frame_calls, _RZ._FRAME_CALLS = _RZ._FRAME_CALLS, False
    for _ in range(a.diag_steps):
        eager_step()
        frames = frames[-1:]
    _RZ._FRAME_CALLS = frame_calls
    stages = {k: sum(v) / len(v) for k, v in StageTimer.durations_ms().items()}
    StageTimer.enabled = False
    ms_per_step = 1000.0 * dt / a.steps
    mpix = world * H * W * a.steps / dt / 1e6

    if rank == 0:
        # --- roofline of the dominant kernel -------------------------------
        from mini3dgs_amd.rasterizer import forward_pipeline  # noqa: F401
        tiles_x, tiles_y = (W + 15) // 16, (H + 15) // 16
        with torch.no_grad():
            out = renderer.render(cam, model, settings)  # the scene every timed step rendered
        # re-run the forward pipeline to read its frame state (not timed)
        from mini3dgs_amd import rasterizer as RZ
        camp = pkg.camera_params(cam, settings)
        pair_counts = torch.empty((H * W,), dtype=torch.int32, device=dev)
        pix_neval = torch.empty((H * W,), dtype=torch.int32, device=dev)
        with torch.no_grad():
            op = torch.sigmoid(model._opacity).squeeze(1)
            img, al, dp, m2, cn, _, _, fr = RZ.forward_pipeline(
                camp, model._xyz, None, model._scaling, model._rotation, model._features_dc[:, 0, :], op,
                pair_counts=pair_counts, pix_neval=pix_neval, need_grad=True)
            # and its backward, for L: the live (entry, cell) pairs -- the partials
            # the blend backward writes and the gather reads (its slot flags)
            RZ.backward_pipeline(camp, fr, model._xyz, None, model._scaling, model._rotation,
                                 model._features_dc[:, 0, :], op, m2, cn, cot[0], cot[1], cot[2], None, None,
                                 outputs=(img, al, dp))
            live_pairs = int(fr.slot_live.count_nonzero())
        R, E, Cc = algorithmic_counts(pix_neval, pair_counts, H, W, tiles_x, tiles_y)
        M, T = fr.M, fr.T
        num_tiles = tiles_x * tiles_y
        # SURVEY 8(d) algorithmic bytes per launch: the consumed records (44 B:
        # mean 8, conic 12, opacity 4, colour 12, depth 4, gradient slot 4),
        # tile ranges, per-pixel outputs + saved state (20 + 8 B) forward;
        # records, per-pixel state + cotangents (36 B) and 40 B of gradient per
        # visible Gaussian backward
        bytes_fwd = 44 * R + 8 * num_tiles + 28 * H * W
        bytes_bwd = 44 * R + 36 * H * W + 40 * M
        # SURVEY 8(d) flops: forward 26 per evaluated pair; backward 70 per
        # contributing pair + 12 per other visited (evaluated) pair
        flops_fwd, flops_bwd = 26 * E, 70 * Cc + 12 * (E - Cc)
        kern = {"blend_fwd": (bytes_fwd, flops_fwd), "blend_bwd": (bytes_bwd, flops_bwd)}
        dom = max((k for k in kern if k in stages), key=lambda k: stages[k]) if stages else "blend_bwd"
        # the dominant kernel's average launch, measured live in the timed region
        t_ms = sum(bwd_live) / len(bwd_live) if dom == "blend_bwd" and bwd_live else stages[dom]
        ach = kern[dom][0] / (t_ms * 1e-3) / 1e9
        copy_gbs = copy_peak_gbs(dev)
        traffic, tinfo = pmc_traffic(dom)
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_raw": tinfo.get("traffic_raw"), "traffic_source": tinfo,
                "avg_launch_ms": round(t_ms, 4), "algorithmic_bytes_per_launch": int(kern[dom][0]),
                "bytes_model": "44 R + 36 H W + 40 M (SURVEY 8d)" if dom == "blend_bwd"
                else "44 R + 8 tiles + 28 H W (SURVEY 8d)",
                "measured_copy_peak": round(copy_gbs, 1), "frac_of_measured_copy": round(ach / copy_gbs, 4)}
        tf = kern[dom][1] / (t_ms * 1e-3) / 1e12
        roof["valu"] = {"achieved_tflops": round(tf, 2), "peak_tflops": VALU_PEAK_TFLOPS,
                        "frac": round(tf / VALU_PEAK_TFLOPS, 4),
                        "flops_model": "70 C + 12 (E - C) (SURVEY 8d)" if dom == "blend_bwd" else "26 E (SURVEY 8d)"}
        # the other blend kernel, same models (its time from the diagnostic steps)
        other = "blend_fwd" if dom == "blend_bwd" else "blend_bwd"
        if other in stages:
            to = stages[other]
            roof["other_blend"] = {"kernel": other, "avg_ms": round(to, 4),
                                   "hbm_frac": round(kern[other][0] / (to * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                   "valu_frac": round(kern[other][1] / (to * 1e-3) / 1e12 / VALU_PEAK_TFLOPS, 4)}
        # --- CPU baseline ---------------------------------------------------
        cpu = psnr = None
        if world == 1 and not a.no_cpu_baseline:
            cpu, ref_img = cpu_baseline(scene, W, H, cot, a.cpu_threads)
            cpu["reference_cost_model"] = reference_cost_model(H, W, M, E, Cc)
            # the metric's "PSNR vs ref": this frame's image against the oracle's
            # (the reference path's CPU restatement, pinned to its fixtures)
            import numpy as np
            img = out["image"].detach().float().cpu().numpy()
            err = img - ref_img
            mse = float(np.mean(err.astype(np.float64) ** 2))
            psnr = {"db": round(10 * math.log10(1.0 / mse), 2) if mse > 0 else None,
                    "mse": mse, "max_abs_err": float(np.abs(err).max()),
                    "pixels_over_1e-4": int((np.abs(err).max(axis=0) > 1e-4).sum()),
                    "ref": "oracle/gs_oracle.c on the same frame (CPU restatement of renderer.py, "
                           "pinned to the reference's own outputs); db None = bit-identical images"}
        wl = workload_name(n, W, H)
        line = {
            "metric": METRIC, "value": round(mpix, 3), "unit": "Mpix/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "spinup_steps": a.spinup_steps, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{wl}: {n:,} synthetic Gaussians (SURVEY 8d), {W}x{H}, 16x16 tiles, "
                                   "render fwd+bwd" + (" + grad all-reduce" if reducer is not None else "")
                                   + ("" if opt is None else " + Adam step"),
                       "preset": wl,
                       "gaussians": n, "width": W, "height": H, "views_per_step": world,
                       "parallelism": f"dp{world} (one view per GPU)", "visible": M, "tile_touches": T,
                       "records_consumed": R, "evaluated_pairs": E, "contributing_pairs": Cc,
                       "live_entry_cells": live_pairs},
            "graph": graph_info,
            "stages_ms": {k: round(v, 4) for k, v in stages.items()},
            "stages_note": f"HIP-event intervals from {a.diag_steps} diagnostic steps after the timed region, "
                           "run stage by stage (GS_FRAME_CALLS=0 path: the same kernels as the timed steps' frame "
                           "entry points) "
                           "(each interval also holds any host launch gap before its kernels; kernel-only "
                           "times: profiles/*/kernel_stats_*.csv)",
            "roofline": roof,
            "cpu_baseline": cpu,
            "psnr_vs_ref": psnr,
        }
        if reducer is not None:
            # steps that issued collectives: spin-up, warm-up, the timed steps,
            # collective_share's timing run (its no-collective run issues none)
            # and the diagnostic steps
            nsteps = a.spinup_steps + a.warmup + 2 * a.steps + a.diag_steps
            line["allreduce"] = {"ranges_per_step": reducer.overlap_chunks(), "pipelined_adam": opt is not None,
                                 "host_us_per_step": {k: round(1e6 * v / nsteps, 1) for k, v in reducer.host_s.items()},
                                 "avg": reducer._avg, "native": reducer.native_status["native"],
                                 "rccl_nranks": reducer.native_status["rccl_nranks"],
                                 "self_check_err": reducer.native_status["self_check_err"],
                                 "fallback_reason": reducer.native_status["fallback_reason"]}
            line["allreduce"].update(coll)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        pkg.distributed.close_native_comms()
        dist.destroy_process_group()


def timed_steps(dist, dev, k, fn):
    """Wall seconds of k calls of fn, barrier + synchronize on both sides,
    max over ranks (the contract's timing, for the extra measurements)."""
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def collective_share(a, dist, dev, reducer, model, step, frames, dt):
    """The all-reduce's part of the timed step (N > 1, or --force-dist), from
    two extra runs of --steps steps after the timed region:
      * the same steps with an event pair on the collective stream around
        each range's collective: gpu_us_per_step = their summed durations per
        step (max over ranks; native RCCL only -- torch.distributed's
        collectives run on streams or threads this process cannot time);
      * the same steps without the collective (the gradients stay local, the
        Adam step reads them unreduced): exposed_frac = (timed step - that
        step) / timed step, the share of the step the collective adds."""
    k = a.steps
    timed = reducer.set_timing(True)
    dt_coll = timed_steps(dist, dev, k, lambda: (step(), frames.clear()))
    ms = reducer.collective_gpu_ms() if timed else None
    reducer.set_timing(False)
    per_step = sum(ms) / k if ms else (0.0 if timed else -1.0)
    t = torch.tensor([per_step], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    per_step = float(t.item())
    model._gs_grad_sink, sink = None, model._gs_grad_sink  # the backward writes local .grad tensors
    step.no_collective = True
    try:
        dt_nc = timed_steps(dist, dev, k, lambda: (step(), frames.clear()))
    finally:
        step.no_collective = False
        model._gs_grad_sink = sink
    return {"gpu_us_per_step": round(1e3 * per_step, 1) if per_step >= 0 else None,
            "collectives_per_step": (len(ms) / k if ms else None),
            "gpu_us_note": "event pair on the native RCCL stream per collective, max over ranks" if timed
            else "not measurable: the collectives run through torch.distributed (" + reducer.native_status[
                "fallback_reason"] + ")",
            "ms_per_step_timing_run": round(1e3 * dt_coll / k, 4),
            "ms_per_step_no_collective": round(1e3 * dt_nc / k, 4),
            "exposed_frac": round(max(0.0, dt - dt_nc) / dt, 4),
            "exposed_note": "(timed step - the same run's step without the all-reduce) / timed step"}


def pmc_traffic(stage):
    """HBM bytes per launch of the stage's kernel from the committed PMC
    summary (tools/pmc_run.sh -> profiles/pmc_current.txt), as
    MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE doubled (gfx950
    tallies 128-B read requests at 64 B) + WRITE_SIZE, KiB -> bytes; the raw
    sum beside it.  The summary names the library build (source hash) its
    counters came from: a summary of another build is flagged and its bytes
    are not reported as this build's traffic."""
    path = os.path.join(ROOT, "profiles", "pmc_current.txt")
    if not os.path.exists(path):
        return None, {"source": None, "note": "no PMC summary"}
    sys.path.insert(0, os.path.join(ROOT, "mini-3d-gaussian-splatting_amd"))
    import build as _build
    want, cur, vals, pmc_build = "k_" + stage, None, {}, None
    for line in open(path):
        if line.startswith("#"):
            parts = line.split()
            if len(parts) == 3 and parts[1] == "library_source_sha256":
                pmc_build = parts[2]
        elif line and not line[0].isspace():
            cur = line.strip()
        elif cur == want:
            parts = line.split()
            if len(parts) == 2:
                vals[parts[0]] = float(parts[1])
    if "FETCH_SIZE" not in vals or "WRITE_SIZE" not in vals:
        return None, {"source": "profiles/pmc_current.txt", "note": f"no FETCH/WRITE for {want}"}
    bench_build = _build.source_hash()
    valu_issue = None
    if all(k in vals for k in ("SQ_INSTS_VALU", "GRBM_GUI_ACTIVE")):
        # VALU issue cycles (2 per wave64 instruction, MI355X_MICROARCH.md "Wave
        # scheduling") over the 1,024 SIMDs' cycles (GRBM_GUI_ACTIVE sums 8 XCDs)
        valu_issue = round(2.0 * vals["SQ_INSTS_VALU"] / (1024.0 * vals["GRBM_GUI_ACTIVE"] / 8.0), 3)
    fetch, write = vals["FETCH_SIZE"] * 1024, vals["WRITE_SIZE"] * 1024
    info = {"source": "profiles/pmc_current.txt (rocprofv3 --pmc, one counter group per pass)",
            "pmc_build": pmc_build, "bench_build": bench_build, "build_match": pmc_build == bench_build,
            "fetch_raw": int(fetch), "write": int(write), "traffic_raw": int(fetch + write),
            "correction": "traffic = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md: gfx950 counts a 128-B "
                          "read request as 64 B; stated there for coalesced streaming reads, this kernel's "
                          "reads are record gathers, so traffic_raw is the lower bound)",
            "valu_issue_frac": valu_issue}
    if not info["build_match"]:
        info["note"] = "stale: the PMC summary is of another library build; traffic not reported"
        return None, info
    return int(2 * fetch + write), info


def cpu_limit():
    """The CPUs this process may use: sched_getaffinity, and the cgroup v2
    quota (cpu.max "quota period"; "max" = none) of its own cgroup.  Returns
    (usable CPUs, info dict)."""
    avail = len(os.sched_getaffinity(0))
    info = {"nproc": os.cpu_count(), "sched_getaffinity": avail, "cgroup_cpu_max": None,
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}
    limit = avail
    try:
        v2, v1 = "/", "/"
        for ln in open("/proc/self/cgroup"):
            parts = ln.strip().split(":", 2)
            if len(parts) == 3 and parts[0] == "0":  # the v2 unified hierarchy
                v2 = parts[2]
            elif len(parts) == 3 and "cpu" in parts[1].split(","):  # v1 cpu controller
                v1 = parts[2]
        quota = None
        for d in (os.path.join("/sys/fs/cgroup", v2.lstrip("/")), "/sys/fs/cgroup"):
            p = os.path.join(d, "cpu.max")
            if os.path.exists(p):
                raw = open(p).read().strip()
                info["cgroup_cpu_max"] = raw
                q, per = raw.split()[:2]
                quota = None if q == "max" else (int(q), int(per))
                break
        else:
            for d in (os.path.join("/sys/fs/cgroup/cpu", v1.lstrip("/")), "/sys/fs/cgroup/cpu"):
                p = os.path.join(d, "cpu.cfs_quota_us")
                if os.path.exists(p):
                    q, per = int(open(p).read()), int(open(os.path.join(d, "cpu.cfs_period_us")).read())
                    info["cgroup_cpu_max"] = f"v1 cfs_quota_us={q} cfs_period_us={per}"
                    quota = (q, per) if q > 0 else None
                    break
        if quota:
            limit = min(limit, max(1, int(math.ceil(quota[0] / quota[1]))))
    except (OSError, ValueError):
        pass
    info["limit"] = limit
    return limit, info


def cpu_baseline(scene, W, H, cot, threads):
    """Oracle (C restatement of the reference render path) fwd+bwd on the
    host cores for the same frame: one frame per thread count of a sweep
    (16, 32, 64, 128, 256, capped by the CPUs this process may use, cgroup
    quota included; `threads` > 0 adds that count), the fastest reported, then
    one frame on one core.  Bounded: ~1 s per multi-thread frame, ~10 s on one
    core."""
    import numpy as np
    from oracle import oracle as orc  # CPU baseline leg: test infrastructure only
    limit, info = cpu_limit()
    counts = sorted({c for c in (16, 32, 64, 128, 256, threads) if 0 < c <= limit} | {limit})
    cov = orc.covariance(scene.scaling.numpy(), scene.rotation.numpy())
    s = orc.Scene(xyz=scene.xyz.numpy(), cov3d=cov, color_logits=scene.features_dc[:, 0].numpy(),
                  opacity=torch.sigmoid(scene.opacity[:, 0]).numpy(), wv=np.eye(4), width=W, height=H,
                  fovx=scene.fovx, fovy=scene.fovy, bg=np.zeros(3, np.float32))
    gi, ga, gd = (c.cpu().numpy() for c in cot)
    sweep, ref, best = {}, None, None
    for c in counts:
        t0 = time.perf_counter()
        r = orc.render_backward(s, gi, ga, gd, nthreads=c)
        dt = time.perf_counter() - t0
        sweep[str(c)] = round(H * W / dt / 1e6, 4)
        print(f"cpu baseline: {c} threads {dt:.2f} s", file=sys.stderr, flush=True)  # (progress)
        if ref is None:
            ref = r
        if best is None or dt < best[1]:
            best = (c, dt)
    t0 = time.perf_counter()
    orc.render_backward(s, gi, ga, gd, nthreads=1)
    dt1 = time.perf_counter() - t0
    threads, dt = best
    return {"value": round(H * W / dt / 1e6, 4), "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": f"one full {workload_name(scene.xyz.shape[0], W, H)} frame ({W}x{H}, {scene.xyz.shape[0]} Gaussians) fwd+bwd per thread count, "
                      f"oracle/gs_oracle.c with OpenMP; fastest x{threads} ({dt:.2f} s), 1 core ({dt1:.2f} s)",
            "thread_sweep_mpix_s": sweep, "cpu_limit": info,
            "one_core": {"value": round(H * W / dt1 / 1e6, 4), "unit": "Mpix/s", "cores": 1},
            "host_cpus_schedulable": info["sched_getaffinity"]}, ref["image"]


def reference_cost_model(H, W, M, E, C):
    """The literal reference (Python per-pixel loop + autograd) priced by
    BASELINE.md section 2's measured coefficients and this frame's counters
    (M visible, E evaluated, C contributing pairs)."""
    fwd = (REF_FWD_S_PER_PAIR * (E - C) + REF_FWD_S_PER_CONTRIB * C + REF_BIN_S_PER_GAUSSIAN * M
           + REF_PROJ_SORT_S_PER_1M * M / 1e6)
    bwd = REF_BWD_S_PER_CONTRIB_PX * H * W * C
    return {"fwd_hours": round(fwd / 3600, 1), "bwd_hours": round(bwd / 3600, 1),
            "value": H * W / (fwd + bwd) / 1e6, "unit": "Mpix/s", "cores": 1,
            "note": "BASELINE.md section 2 coefficients x this frame's E, C, M (not run: the reference "
                    "cannot travel to the GPU box)"}


if __name__ == "__main__":
    main()
