"""Diagnostic: does a 4-byte hipMemsetAsync captured into a HIP graph write only its 4 bytes?

bb_step's serial route (flat banks) resets its hand-over counter with
hipMemsetAsync(count + 2, 0, 4) -- the only memset node a captured rollout
holds.  This captures such memsets at several offsets of a sentinel-filled
buffer (torch-allocated and hipMalloc'd), replays the graph, and reports any
byte outside the 4 targeted ones that changed.
"""
import ctypes as C

import torch

hip = C.CDLL("libamdhip64.so.7")
hip.hipMemsetAsync.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
hip.hipMemsetAsync.restype = C.c_int
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
hip.hipFree.argtypes = [C.c_void_p]


def check(base_ptr, nbytes, read, write, label):
    bad = 0
    for off in (0, 4, 8, 12, 60, 64, 124):
        write(0x5A)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
            assert hip.hipMemsetAsync(C.c_void_p(base_ptr + off), 0, 4, s) == 0
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        b = read()
        changed = [i for i in range(nbytes) if (b[i] != 0x5A) != (off <= i < off + 4)]
        print(f"{label} offset {off}: bytes changed outside the target: {changed[:16]}", flush=True)
        bad += len(changed)
    return bad


t = torch.empty(256, dtype=torch.uint8, device="cuda:0")
bad = check(t.data_ptr(), 256, lambda: t.cpu().tolist(), lambda v: t.fill_(v), "torch buffer")

p = C.c_void_p()
assert hip.hipMalloc(C.byref(p), 16) == 0   # as bb_create allocates slow_count (4 ints)
q = C.c_void_p()
assert hip.hipMalloc(C.byref(q), 4096) == 0  # a neighbour
host = (C.c_uint8 * 16)()


def w16(v):
    for i in range(16):
        host[i] = v
    hip.hipMemcpy(p, host, 16, 1)


def r16():
    out = (C.c_uint8 * 16)()
    hip.hipMemcpy(out, p, 16, 2)
    return list(out)


nb = (C.c_uint8 * 4096)(*([0x33] * 4096))
hip.hipMemcpy(q, nb, 4096, 1)
for off in (8,):
    w16(0x5A)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        assert hip.hipMemsetAsync(C.c_void_p(p.value + off), 0, 4, s) == 0
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    b = r16()
    changed = [i for i in range(16) if (b[i] != 0x5A) != (off <= i < off + 4)]
    nbr = (C.c_uint8 * 4096)()
    hip.hipMemcpy(nbr, q, 4096, 2)
    print(f"hipMalloc(16) offset {off}: changed {changed}; neighbour intact: {all(x == 0x33 for x in nbr)}; "
          f"p={p.value:#x} q={q.value:#x}", flush=True)
    bad += len(changed)
print("MEMSET_GRAPH_OK" if bad == 0 else f"MEMSET_GRAPH_BAD {bad}", flush=True)
