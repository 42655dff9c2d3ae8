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


def _scene(P, patch):
    """(scene, World keywords, steps).  patch == "c4": BASELINE configs[3]
    split by body-id range (strong scaling); "boxpile": tilted cube columns
    with sphere caps (ids column by column, so the shards meet along a row of
    columns: box-box, sphere-box and edge contacts across the seam)."""
    from rbhip import scenes
    if patch == "c4":
        return scenes.make("c4"), {}, 80
    if patch == "boxpile":
        return scenes.box_pile(6, 6, 3, seed=0), {"max_partners": 32}, 300
    return scenes.tiled(scenes.flat_spheres, P, patch, patch, seed=2), {}, 80


def _worker(rank, P, port, out, transport="host", halo=False, patch=16):
    for pth in (ROOT, PKG):
        sys.path.insert(0, pth)
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=P)
    from rbhip.shard import ShardedWorld
    sc, kw, steps = _scene(P, patch)
    sw = ShardedWorld(sc, device=0, transport=transport, halo=halo, **kw)
    assert sw.transport == transport and sw.halo == halo
    sw.step(steps)
    sw.sync()
    q, v = sw.gather_state()
    if rank == 0:
        np.save(out, np.concatenate([q, v], axis=1))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("P,transport,halo,patch", [(2, "host", False, 16), (2, "p2p", False, 16),
                                                    (3, "p2p", False, 16), (2, "p2p", True, 16),
                                                    (3, "p2p", True, 16), (2, "p2p", True, 96),
                                                    (2, "p2p", True, "c4"), (2, "p2p", False, "c4"),
                                                    (2, "host", False, "boxpile"), (2, "p2p", False, "boxpile"),
                                                    (2, "p2p", True, "boxpile"), (3, "p2p", True, "boxpile")])
def test_two_process_shards_match_single_world(tmp_path, P, transport, halo, patch):
    """Several processes on one GPU; "p2p" maps the other processes' buffers
    through IPC and synchronises on device flags, as across GPUs; halo=True
    pushes only the bodies within a cell of each peer's bounds (96x96
    patches: 36 push blocks per rank, a wave-aggregated inbox per peer).
    The box piles exchange the boxes' orientations with their positions
    (full reads, halo pushes, host all-gather)."""
    import torch.multiprocessing as mp
    import rbhip
    sc, kw, steps = _scene(P, patch)
    with rbhip.World(sc, **kw) as w:
        w.step(steps)
        q1, v1 = w.get_state()
    out = str(tmp_path / "state.npy")
    mp.start_processes(_worker, args=(P, _free_port(), out, transport, halo, patch), nprocs=P,
                       start_method="spawn")
    got = np.load(out)
    assert np.array_equal(got[:, :7], q1) and np.array_equal(got[:, 7:], v1)


# ---------------------------------------------------------------- in-library RCCL exchange
# One GPU on the test box: RCCL refuses two ranks on one device, so the
# in-library exchange is exercised with a one-rank communicator (the
# all-gather is then a no-op, the graph capture of step + collective +
# remote insert is real).  The multi-rank data path is the same three
# operations as the host-staged test above.

@pytest.mark.parametrize("scene", ["flat", "boxpile"])
def test_inlibrary_exchange_one_rank_matches_world(scene):
    import rbhip
    from rbhip import scenes
    sc, kw = ((scenes.flat_spheres(24, 24, seed=5), {}) if scene == "flat" else
              (scenes.box_pile(4, 4, 3, seed=1), {"max_partners": 32}))   # box pile: orientations gathered too
    with rbhip.World(sc, **kw) as ref:
        ref.step(613)
        q1, v1 = ref.get_state()
    with rbhip.World(sc, **kw) as w:
        w.shard_comm_init(rbhip.World.comm_unique_id())
        for n in (1, 12, 600):              # eager, one graph, a 512 + 88 chunked replay
            w.shard_run(n)
        w.sync()
        q2, v2 = w.get_state()
    assert np.array_equal(q1, q2) and np.array_equal(v1, v2)


@pytest.mark.parametrize("halo", [False, True])
def test_p2p_one_rank_matches_world(halo):
    """The peer-to-peer exchange with one rank (the graph of step kernel and
    exchange kernels, the halo mode's prime, push tail and insert kernel,
    with no peer data): the same state as rb_step, eager, one graph and a
    chunked replay."""
    import rbhip
    from rbhip import scenes
    sc = scenes.flat_spheres(24, 24, seed=5)
    with rbhip.World(sc) as ref:
        ref.step(613)
        q1, v1 = ref.get_state()
    with rbhip.World(sc) as w:
        w.p2p_connect(w.p2p_handles())
        w.p2p_halo(halo)
        for n in (1, 12, 600):
            w.shard_run(n)
        w.sync()
        q2, v2 = w.get_state()
    assert np.array_equal(q1, q2) and np.array_equal(v1, v2)


def test_inlibrary_exchange_requires_comm():
    import rbhip
    from rbhip import scenes
    with rbhip.World(scenes.flat_spheres(4, 4)) as w:
        with pytest.raises(rbhip.RbError):
            w.shard_run(3)


def _nccl_group_worker(rank, P, port, steps, out, transport, expect):
    for pth in (ROOT, PKG):
        sys.path.insert(0, pth)
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=P, device_id=torch.device("cuda:0"))
    from rbhip import scenes
    from rbhip.shard import ShardedWorld
    sc = scenes.tiled(scenes.flat_spheres, P, 16, 16, seed=2)
    sw = ShardedWorld(sc, device=0, transport=transport)
    assert sw.transport == expect
    sw.step(steps)
    sw.sync()
    q, v = sw.gather_state()
    if rank == 0:
        np.save(out, np.concatenate([q, v], axis=1))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("transport,expect", [(None, "p2p"), ("rccl", "rccl")])
def test_sharded_world_on_nccl_group_one_rank(tmp_path, transport, expect):
    """ShardedWorld on an nccl process group: the peer-to-peer exchange by
    default, or the in-library RCCL exchange (communicator id broadcast
    through torch.distributed)."""
    import torch.multiprocessing as mp
    import rbhip
    from rbhip import scenes
    steps = 80
    sc = scenes.tiled(scenes.flat_spheres, 1, 16, 16, seed=2)
    with rbhip.World(sc) as w:
        w.step(steps)
        q1, v1 = w.get_state()
    out = str(tmp_path / "state.npy")
    mp.start_processes(_nccl_group_worker, args=(1, _free_port(), steps, out, transport, expect), nprocs=1,
                       start_method="spawn")
    got = np.load(out)
    assert np.array_equal(got[:, :7], q1) and np.array_equal(got[:, 7:], v1)


def _timeout_worker(rank, P, port, out, halo=False):
    for pth in (ROOT, PKG):
        sys.path.insert(0, pth)
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=P)
    import rbhip
    from rbhip import scenes
    from rbhip.shard import ShardedWorld
    sw = ShardedWorld(scenes.tiled(scenes.flat_spheres, P, 8, 8, seed=1), device=0, transport="p2p", halo=halo)
    msg = "no error"
    if rank == 0:                      # rank 1 never steps: rank 0's exchange must give up, not hang
        sw.step(4)
        try:
            sw.sync()
        except rbhip.RbError as e:
            msg = str(e)
        with open(out, "w") as f:
            f.write(msg)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("halo", [False, True])
def test_p2p_exchange_times_out_instead_of_hanging(tmp_path, halo):
    import time
    import torch.multiprocessing as mp
    out = str(tmp_path / "msg.txt")
    t0 = time.time()
    mp.start_processes(_timeout_worker, args=(2, _free_port(), out, halo), nprocs=2, start_method="spawn")
    msg = open(out).read()
    assert "exchange timed out" in msg, msg
    assert time.time() - t0 < 60


def _halo_move_worker(rank, P, port, out):
    for pth in (ROOT, PKG):
        sys.path.insert(0, pth)
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=P)
    import rbhip
    from rbhip import scenes
    from rbhip.shard import ShardedWorld
    sc = scenes.tiled(scenes.flat_spheres, P, 8, 8, seed=1)
    v0 = sc.qvel0.copy()
    v0[3, 0] = 200.0                   # rank 0's body 3: 2 m per step, five cells
    sw = ShardedWorld(sc.with_(qvel0=v0), device=0, transport="p2p", halo=True)
    msg = "no error"
    try:
        sw.step(3)
        sw.sync()
    except rbhip.RbError as e:
        msg = str(e)
    if rank == 0:
        with open(out, "w") as f:
            f.write(msg)
    dist.barrier()
    dist.destroy_process_group()


def test_halo_push_raises_when_a_body_moves_more_than_a_cell(tmp_path):
    """The halo push (rb_halo.hpp) is exact only while no body moves more
    than one broadphase cell per step: a body that does raises an error on
    its rank (RB_EDOM), not a silent pass."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "msg.txt")
    mp.start_processes(_halo_move_worker, args=(2, _free_port(), out), nprocs=2, start_method="spawn")
    msg = open(out).read()
    assert "more than one broadphase cell" in msg, msg
