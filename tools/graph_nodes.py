"""Node census of the captured training-step graph, plain or with the one-rank RCCL GradSync (where the DP graph's
extra time comes from): node types, kernel nodes by name family, nodes with >1 parent (joins) / >1 child (forks),
and the replay wall time of the same graph.   python tools/graph_nodes.py {plain|dp} [dot_path]"""
import collections
import ctypes
import socket
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, ".")
import bench  # noqa: E402
import textmae_amd  # noqa: E402
from textmae_amd import engine  # noqa: E402
from textmae_amd.optim import configure_optimizers  # noqa: E402
from textmae_amd.parallel import enable_data_parallel  # noqa: E402
from textmae_amd.rd_loss import RateDistortionLoss  # noqa: E402

TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "wait_event", 7: "event_record",
         10: "mem_alloc", 11: "mem_free", 12: "memcpy_from_symbol", 13: "memcpy_to_symbol"}

mode = sys.argv[1] if len(sys.argv) > 1 else "dp"
dot = sys.argv[2] if len(sys.argv) > 2 else None
hip = ctypes.CDLL("libamdhip64.so")
_Orig = torch.cuda.CUDAGraph
kept = []


def _keep():
    g = _Orig(keep_graph=True)
    kept.append(g)
    return g


torch.cuda.CUDAGraph = _keep  # engine.GraphedTrainStep captures through torch.cuda.CUDAGraph()
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().train()
m.compute_dtype = torch.bfloat16
m.distortion = "ssim+l1"
if mode == "dp":
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    enable_data_parallel(m, always_collective=True)
opt, aux = configure_optimizers(m, lr=1e-4, aux_lr=1e-4, fused=True)
crit = RateDistortionLoss(lmbda=1e-2)
imgs, scores = bench.synthetic_inputs(64, 256, 256, 2000, "cuda")
step = engine.GraphedTrainStep(m, crit, opt, aux, imgs, scores, clip_max_norm=1.0, warmup=1)
g = kept[-1]
raw = ctypes.c_void_p(g.raw_cuda_graph())
n = ctypes.c_size_t(0)
assert hip.hipGraphGetNodes(raw, None, ctypes.byref(n)) == 0
nodes = (ctypes.c_void_p * n.value)()
assert hip.hipGraphGetNodes(raw, nodes, ctypes.byref(n)) == 0
types = collections.Counter()
forks = joins = 0
for nd in nodes:
    t = ctypes.c_int(0)
    hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
    types[TYPES.get(t.value, str(t.value))] += 1
    c = ctypes.c_size_t(0)
    hip.hipGraphNodeGetDependencies(ctypes.c_void_p(nd), None, ctypes.byref(c))
    joins += c.value > 1
    c = ctypes.c_size_t(0)
    hip.hipGraphNodeGetDependentNodes(ctypes.c_void_p(nd), None, ctypes.byref(c))
    forks += c.value > 1
print(f"{mode}: {n.value} nodes {dict(types)}; forks {forks} joins {joins}", flush=True)
if dot:
    hip.hipGraphDebugDotPrint(raw, dot.encode(), ctypes.c_uint(0))
for _ in range(3):
    step(imgs, scores)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    step(imgs, scores)
torch.cuda.synchronize()
print(f"{mode}: replay {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms per step", flush=True)
if mode == "dp":
    dist.destroy_process_group()
