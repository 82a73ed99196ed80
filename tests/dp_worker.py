"""One rank of the data-parallel training test (tests/test_dp_training_gpu.py):
    python tests/dp_worker.py <rank> <world> <port> <scene_dir> <out.npz> [backend]
Renders its own view per iteration with a full model replica; the gradient
mean goes through GradAllReduce (gloo on one GPU here; RCCL = "nccl" on a
node), then FusedAdam and densification, exactly as GaussianTrainer runs."""
import os
import sys
from pathlib import Path

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    scene_dir, out = Path(sys.argv[4]), sys.argv[5]
    backend = sys.argv[6] if len(sys.argv) > 6 else "gloo"
    import numpy as np
    import torch
    import torch.distributed as dist
    import __graft_entry__ as ge
    from scene_util import dp_config, load_scene
    pkg = ge.load_package()
    dev = torch.device("cuda", 0 if backend == "gloo" else rank)
    torch.cuda.set_device(dev)
    dist.init_process_group(backend, rank=rank, world_size=world, init_method=f"tcp://127.0.0.1:{port}")
    ds = load_scene(pkg, scene_dir, dev, split=False)
    tr = pkg.GaussianTrainer(dp_config(pkg, scene_dir / f"out{rank}"), ds)
    tr.setup()
    assert tr._dist is not None
    tr.train(3)
    torch.cuda.synchronize()
    np.savez(out, **{f"p{i}": p.detach().cpu().numpy() for i, p in enumerate(tr.gaussians.parameter_list())},
             iteration=tr.iteration, n=tr.gaussians.get_num_points(),
             ranges=tr._reducer.ranges_reduced if tr._reducer is not None else -1)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
