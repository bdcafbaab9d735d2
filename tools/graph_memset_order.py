"""Diagnostic: the order of a captured hipMemsetAsync node against
the kernel nodes around it, on replay, under load.

1. The real thing: a rollout-style graph of T steps of bb_step on the serial route
   with the hand-over count reset by hipMemsetAsync (BB_COUNT_MEMSET=1), captured
   with torch's graph debug mode; the graph is written as DOT
   (hipGraphDebugDotPrint) to gpurun_out/rollout_memset_graph.dot for its node
   types and edges.
2. The ordering test: a graph of R rounds of [memset(c, 0) -> c += 1 -> bad += (c != 1)]
   (a 4-byte hipMemsetAsync node between two torch kernel nodes on one stream),
   replayed while GEMMs load the GPU from a second stream.  A memset that runs
   before the previous round's check or after the next increment shows up in bad.
   The same graph with a kernel node (c.zero_()) in place of the memset is the control.
"""
import ctypes as C
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "openballbot-rl_amd"))
OUT = ROOT / "gpurun_out"
OUT.mkdir(exist_ok=True)
hip = C.CDLL("libamdhip64.so.7")
hip.hipMemsetAsync.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
hip.hipMemsetAsync.restype = C.c_int


def rollout_dot(T=3, n=256):
    """Capture T serial-route steps with the memset reset (raw hipStreamBeginCapture on a
    side stream) and print the graph as DOT with hipGraphDebugDotPrint (verbose)."""
    os.environ["BB_COUNT_MEMSET"] = "1"
    os.environ["BB_ROUTE"] = "1"
    from ballbot_gym import _native as N
    from ballbot_gym.envs import BallbotVecEnv

    hip.hipStreamBeginCapture.argtypes = [C.c_void_p, C.c_int]
    hip.hipStreamEndCapture.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
    hip.hipGraphDebugDotPrint.argtypes = [C.c_void_p, C.c_char_p, C.c_uint]
    hip.hipGraphDestroy.argtypes = [C.c_void_p]
    env = BallbotVecEnv(n, device="cuda:0", max_ep_steps=10, seed=3)
    acts = torch.zeros(n, 3, device="cuda:0")
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    sp = C.c_void_p(side.cuda_stream)
    assert hip.hipStreamBeginCapture(sp, 2) == 0  # hipStreamCaptureModeRelaxed
    for _ in range(T):
        N.check(N.lib().bb_step(env._h, C.c_void_p(acts.data_ptr()), C.c_void_p(env.obs.data_ptr()),
                                C.c_void_p(env.reward.data_ptr()), C.c_void_p(env.done.data_ptr()), None, None,
                                1, sp), "bb_step")
    graph = C.c_void_p()
    assert hip.hipStreamEndCapture(sp, C.byref(graph)) == 0
    path = OUT / "rollout_memset_graph.dot"
    rc = hip.hipGraphDebugDotPrint(graph, str(path).encode(), 0xFFFF)
    txt = path.read_text() if path.exists() else ""
    print(f"hipGraphDebugDotPrint rc={rc}: {path} ({len(txt)} bytes)", flush=True)
    print(txt[:6000], flush=True)
    hip.hipGraphDestroy(graph)
    env.close()
    del os.environ["BB_COUNT_MEMSET"], os.environ["BB_ROUTE"]


def order_test(use_memset, rounds=200, replays=50):
    c = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        for _ in range(rounds):
            if use_memset:
                assert hip.hipMemsetAsync(C.c_void_p(c.data_ptr()), 0, 4, s) == 0
            else:
                c.zero_()
            c.add_(1)
            bad.add_((c != 1).to(torch.int32))
    load = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device="cuda:0")
    for _ in range(replays):
        with torch.cuda.stream(load):
            for _ in range(4):
                a = torch.tanh(a @ a.T * 1e-3)
        g.replay()
    torch.cuda.synchronize()
    return int(bad.item())


if __name__ == "__main__":
    rollout_dot()
    for m in (False, True):
        print(f"order test, {'memset node' if m else 'kernel node (control)'}: "
              f"rounds with c != 1 after the increment: {order_test(m)}", flush=True)
    print("GRAPH_MEMSET_ORDER_DONE", flush=True)
