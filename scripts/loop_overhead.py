"""Diagnostic: per-step cost of the sharded stepping loop's pieces on one
GPU (host launch overhead vs device time), C2 scene (CFG=..., or NX, NY for
a flat NX x NY scene; LIB=path loads another build of the library, for
A/Bs).  Not part of the product; results go to stdout."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rigidbody-simulation_amd"))
import torch
torch.cuda.init()
from rbhip import _lib
if os.environ.get("LIB"):
    _lib.load(os.environ["LIB"])
import rbhip
from rbhip import scenes
from rbhip.shard import wrap_gpos

K = 400
sc = (scenes.flat_spheres(int(os.environ["NX"]), int(os.environ["NY"])) if os.environ.get("NX")
      else scenes.make(os.environ.get("CFG", "c2")))


def timed(fn):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter(); e0.record()
    fn()
    e1.record(); torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e6, e0.elapsed_time(e1) / K * 1e3


with rbhip.World(sc) as w:
    w.set_stream(torch.cuda.current_stream().cuda_stream)
    w.step(50); w.step(K); torch.cuda.synchronize()
    print("graph replay          host %.2f us/step  device %.2f us/step" % timed(lambda: w.step_async(K)))

    def eager():
        for _ in range(K):
            w.step_async(1)
    eager()
    print("eager step_async(1)   host %.2f us/step  device %.2f us/step" % timed(eager))

    def shard_loop():
        for _ in range(K):
            w.shard_step()
            w.shard_exchange_done()
    shard_loop()
    print("shard_step+exch_done  host %.2f us/step  device %.2f us/step" % timed(shard_loop))

    views = {}
    def shard_loop_torch():
        for _ in range(K):
            w.shard_step()
            ptr = w.gpos_buffer()[0]
            if ptr not in views:
                views[ptr] = wrap_gpos(w, torch)
            buf, n = views[ptr]
            buf[0:n].add_(0.0)          # stand-in for the collective's launch
            w.shard_exchange_done()
    shard_loop_torch()
    print("... + torch op        host %.2f us/step  device %.2f us/step" % timed(shard_loop_torch))

    # the in-library exchange: step kernel + RCCL all-gather (one rank: the
    # collective's launch and its kernel, no peers) + remote insert, K steps
    # replayed from one captured graph
    w.shard_comm_init(rbhip.World.comm_unique_id())
    w.shard_run(K); torch.cuda.synchronize()
    print("shard_run (RCCL, 1 rk) host %.2f us/step  device %.2f us/step" % timed(lambda: w.shard_run(K)))

# the peer-to-peer exchange with one rank: the exchange kernel's flag
# handshake and launch, no peer data
with rbhip.World(sc) as w:
    w.set_stream(torch.cuda.current_stream().cuda_stream)
    w.p2p_connect(w.p2p_handles())
    w.shard_run(K); torch.cuda.synchronize()
    print("shard_run (p2p, 1 rk)  host %.2f us/step  device %.2f us/step" % timed(lambda: w.shard_run(K)))

# the peer-to-peer halo exchange with one rank: step kernel (with the push) +
# insert kernel, no peers (the fixed cost a halo step adds)
with rbhip.World(sc) as w:
    w.set_stream(torch.cuda.current_stream().cuda_stream)
    w.p2p_connect(w.p2p_handles())
    w.p2p_halo(True)
    w.shard_run(K); torch.cuda.synchronize()
    print("shard_run (halo, 1 rk) host %.2f us/step  device %.2f us/step" % timed(lambda: w.shard_run(K)))
