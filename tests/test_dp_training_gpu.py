"""Data-parallel GaussianTrainer step (reference
trainer.py:11-15): two ranks, two views per iteration, three iterations
including one densification.  The replicas must stay bit-identical, and equal
a single-process step on the mean of the two views' gradients.  The ranks
share the one GPU of the box and reduce through gloo (RCCL cannot put two
ranks on one device); the collective is the only difference from the node
run, where GradAllReduce issues the same all_reduce over RCCL."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from scene_util import dp_config, load_scene, write_scene_files

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _mean_of_views_reference(pkg, ds, cfg, world):
    """One process: per iteration, the gradients of the views rank r would
    render (trainer._camera_for with world ranks), averaged, then the same
    learning-rate update, FusedAdam step and densification."""
    tr = pkg.GaussianTrainer(cfg, ds)
    tr.setup()
    cams = ds.get_train_cameras()
    g = tr.gaussians
    for it in range(1, cfg.iterations + 1):
        tr.iteration = it
        grads = []
        for r in range(world):
            cam = cams[int(tr._perm[(it * world + r) % len(cams)])]
            tr.optimizer.zero_grad()
            out = tr.renderer.render(cam, g, tr._settings(cam))
            pkg.loss.photometric_loss(out["image"], cam._image, cfg.lambda_dssim)[0].backward()
            grads.append([p.grad.clone() for p in g.grad_parameters()])
        for i, p in enumerate(g.grad_parameters()):
            s = grads[0][i].clone()
            for k in range(1, world):
                s += grads[k][i]
            p.grad = s / world
        tr.optimizer.update_learning_rate(it)
        tr.optimizer.step()
        tr.optimizer.densify_and_prune(it, tr.scene_extent)
    return tr


@pytest.mark.parametrize("chunks", [1, 2, 4])
def test_dp_trainer_two_ranks_match_mean_of_views(pkg, cuda, tmp_path, chunks):
    """chunks > 1: the render backward hands its gradient rows to the
    all-reduce in that many ranges (GradAllReduce.rows_ready), range k
    reduced while range k+1 is computed, and FusedAdam updates range k as
    soon as its reduction is done (GradAllReduce.reduce_and_step ->
    FusedAdam.step_ranges); chunks = 1: one reduction after the backward,
    then one Adam launch.  Every setting must equal the single-process
    mean-of-views step bit for bit, densification included."""
    write_scene_files(tmp_path)
    port = _free_port()
    outs = [tmp_path / f"rank{r}.npz" for r in range(2)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", GS_ALLREDUCE_CHUNKS=str(chunks),
               GS_ALLREDUCE_MIN_ROWS="256")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"), str(r), "2", str(port),
                               str(tmp_path), str(outs[r])], env=env) for r in range(2)]
    try:
        rcs = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0], rcs
    a, b = (np.load(o) for o in outs)
    assert int(a["iteration"]) == 3 and int(a["n"]) == int(b["n"])
    # iteration 3's reducer (rebuilt after the densification): ranges it reduced
    assert int(a["ranges"]) == chunks
    for i in range(6):
        assert np.array_equal(a[f"p{i}"], b[f"p{i}"]), f"replicas diverged in parameter {i}"
    ds = load_scene(pkg, tmp_path, cuda, split=False)
    ref = _mean_of_views_reference(pkg, ds, dp_config(pkg, tmp_path / "ref"), 2)
    n0 = dp_config(pkg, tmp_path).num_random_points
    print(f"DP: {n0} -> {int(a['n'])} Gaussians after the densification at iteration 2")
    assert int(a["n"]) != n0, "the densification must change the model"
    assert ref.gaussians.get_num_points() == int(a["n"])
    for i, p in enumerate(ref.gaussians.parameter_list()):
        assert np.array_equal(p.detach().cpu().numpy(), a[f"p{i}"]), f"DP step != mean-of-views step (parameter {i})"
