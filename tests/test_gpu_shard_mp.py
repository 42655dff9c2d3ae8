"""Two processes (gloo, host-staged exchange) sharding one scene on GPU 0
through the real HIP ShardedWorld: bit-identical to a single world."""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, P, port, steps, out):
    for pth in (ROOT, PKG):
        sys.path.insert(0, pth)
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=P)
    from rbhip import scenes
    from rbhip.shard import ShardedWorld
    sc = scenes.tiled(scenes.flat_spheres, P, 16, 16, seed=2)
    sw = ShardedWorld(sc, device=0)
    assert sw.transport == "host"
    sw.step(steps)
    sw.sync()
    q, v = sw.gather_state()
    if rank == 0:
        np.save(out, np.concatenate([q, v], axis=1))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("P", [2])
def test_two_process_shards_match_single_world(tmp_path, P):
    import torch.multiprocessing as mp
    import rbhip
    from rbhip import scenes
    steps = 80
    sc = scenes.tiled(scenes.flat_spheres, P, 16, 16, seed=2)
    with rbhip.World(sc) as w:
        w.step(steps)
        q1, v1 = w.get_state()
    out = str(tmp_path / "state.npy")
    mp.start_processes(_worker, args=(P, _free_port(), steps, out), nprocs=P, start_method="spawn")
    got = np.load(out)
    assert np.array_equal(got[:, :7], q1) and np.array_equal(got[:, 7:], v1)
